#ifndef NETC_WS_ROUTE_H
#define NETC_WS_ROUTE_H

/*
 * Per-connection receive routes for ws_parse_frame and send routes for
 * ws_send_message (libnetc.so).
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
 * Send routes work the same way for ws_send_message(client, message, key,
 * num_frames) (reference src/ws/common.c:36-130): while a send route is attached
 * to a socket, ws_send_message on it returns send_route(ctx, sockfd, message,
 * key, num_frames) with ws_send_message's contract (1 once sent, else the failing
 * send() result).  netc_ws_gpu_attach_send (include/ws/egress.h) attaches the GPU
 * egress ring this way.  A socket's receive and send routes are independent.
 *
 * A route belongs to the connection it was attached to, not to the descriptor number:
 * the table records the socket's identity (device, inode) at attach, and a lookup on a
 * descriptor that now names another socket (the connection was closed without a detach
 * and the number reused by accept()) finds no route -- the new connection gets the CPU
 * path.  Attaching a different route to a socket that still has a live one fails with
 * EBUSY (detach first); re-attaching the same (fn, ctx) is a no-op.
 *
 * Threading: attach / detach / parse of ONE socket from one thread at a time
 * (as netc drives a connection); different sockets from any threads.  A route
 * must stay valid until it is detached.
 */

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct ws_frame_parsing_state;
struct ws_message;

typedef int (*netc_ws_route_fn)(void *ctx, int sockfd, struct ws_frame_parsing_state *state,
                                size_t max_payload_length);

/** Route ws_parse_frame on sockfd to fn(ctx, ...).  0, or -1 (errno = EINVAL: bad or closed fd,
 *  null fn; ENOMEM; EBUSY: another route serves this connection). */
int netc_ws_route_attach(int sockfd, netc_ws_route_fn fn, void *ctx);

/** Back to the CPU parser on sockfd.  0 (also when nothing was attached), -1 on a bad fd. */
int netc_ws_route_detach(int sockfd);

/** The route attached to sockfd's connection, or NULL (*ctx filled when one is). */
netc_ws_route_fn netc_ws_route_get(int sockfd, void **ctx);

/** The route recorded under the descriptor number, live or left by a closed connection (for detach). */
netc_ws_route_fn netc_ws_route_get_raw(int sockfd, void **ctx);

typedef int (*netc_ws_send_route_fn)(void *ctx, int sockfd, struct ws_message *message, uint8_t masking_key[4],
                                     size_t num_frames);

/** Route ws_send_message on sockfd to fn(ctx, ...).  0, or -1 (errno as netc_ws_route_attach). */
int netc_ws_send_route_attach(int sockfd, netc_ws_send_route_fn fn, void *ctx);

/** Back to the CPU path on sockfd.  0 (also when nothing was attached), -1 on a bad fd. */
int netc_ws_send_route_detach(int sockfd);

/** The send route attached to sockfd's connection, or NULL (*ctx filled when one is). */
netc_ws_send_route_fn netc_ws_send_route_get(int sockfd, void **ctx);

/** The send route recorded under the descriptor number, live or stale (for detach). */
netc_ws_send_route_fn netc_ws_send_route_get_raw(int sockfd, void **ctx);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_ROUTE_H */
