#ifndef NETC_WS_ROUTE_H
#define NETC_WS_ROUTE_H

/*
 * Per-connection receive routes for ws_parse_frame (libnetc.so).
 *
 * netc's web layer receives a WebSocket message with one call,
 * ws_parse_frame(client, &client->ws_parsing_state, limit) (reference
 * src/web/server.c:86, src/web/client.c:25).  That signature and struct
 * ws_frame_parsing_state are ABI (include/ws/common.h), so a connection cannot
 * carry a pointer to another receiver in its parser state.  Instead libnetc.so
 * keeps a side table keyed by the socket: while a route is attached to a
 * socket, ws_parse_frame on that socket returns route(ctx, sockfd, state,
 * limit) -- same contract: 0 with state->message filled (buffer owned by the
 * caller, freed with free()), 1 for "call again when more data is readable",
 * or a negative WS_FRAME_PARSE_ERROR_* / NETC_GPU_E* code.  Sockets without a
 * route keep the CPU parser.  netc_ws_gpu_attach (include/ws/ingest.h) attaches
 * the GPU ingest ring this way.
 *
 * Threading: attach / detach / parse of ONE socket from one thread at a time
 * (as netc drives a connection); different sockets from any threads.  A route
 * must stay valid until it is detached.
 */

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct ws_frame_parsing_state;

typedef int (*netc_ws_route_fn)(void *ctx, int sockfd, struct ws_frame_parsing_state *state,
                                size_t max_payload_length);

/** Route ws_parse_frame on sockfd to fn(ctx, ...).  0, or -1 (bad fd / null fn; errno = EINVAL / ENOMEM). */
int netc_ws_route_attach(int sockfd, netc_ws_route_fn fn, void *ctx);

/** Back to the CPU parser on sockfd.  0 (also when nothing was attached), -1 on a bad fd. */
int netc_ws_route_detach(int sockfd);

/** The route attached to sockfd, or NULL (*ctx filled when one is). */
netc_ws_route_fn netc_ws_route_get(int sockfd, void **ctx);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_ROUTE_H */
