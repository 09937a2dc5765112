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
 * A route belongs to the connection it was attached to, not to the descriptor number.
 * libnetc.so defines close(): where the process's close() binds to it (netc linked against
 * libnetc.so, which comes before libc), closing a socket first runs the close hooks its
 * routes registered (netc_ws_route_on_close: a hub sends what it queued for the socket, a
 * ring lets go of it), then drops its routes and its send backlog, then closes it -- so a
 * server-initiated close (reference src/ws/server.c:123-124, src/tcp/server.c:67-70) sends
 * the close frame and everything queued before it, as the reference's direct send() does.
 * Where close() does not reach libnetc.so (loaded RTLD_LOCAL; NETC_WS_ROUTE_VERIFY=1), the
 * table records the socket's identity (device, inode) at attach, and a lookup on a
 * descriptor that now names another socket (closed without a detach, number reused by
 * accept()) finds no route -- the new connection gets the CPU path; that costs one fstat
 * per routed call, which close tracking removes (netc_ws_route_close_tracked).
 * Attaching a different route to a socket that still has a live one fails with EBUSY
 * (detach first); re-attaching the same (fn, ctx) is a no-op.
 *
 * Sends never wait for a peer (round 6).  ws_send_message on a non-blocking socket, and
 * every hub and ring flush (which send with MSG_DONTWAIT), write what the socket takes; the
 * rest goes to the connection's send backlog, kept here, and is written ahead of any later
 * byte of that connection, without waiting, by the next ws_send_message, ws_parse_frame or
 * netc_ws_send_flush on the socket (and by the next flush of a hub it is attached to).  A
 * server whose loop also waits for EPOLLOUT calls netc_ws_send_flush while
 * netc_ws_send_pending(fd) > 0.  The backlog is bounded (netc_ws_send_backlog_limit): past
 * the bound the connection fails alone -- its bytes are dropped, errno ENOBUFS,
 * netc_errno_reason BADSEND -- and its later sends return -1 until it is closed.  The
 * reference sends once and returns send()'s result (src/tcp/server.c:219-225): -1 with
 * EAGAIN on a full socket, a short count taken as success (its defect B5).
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

/** Called with the route's (ctx, sockfd) when close() is called on its socket, before the descriptor is
 *  closed (close tracking only; see above).  The route is detached right after. */
typedef void (*netc_ws_route_close_fn)(void *ctx, int sockfd);

/** Registers the close hook of the receive route attached to sockfd.  0, or -1 (EINVAL: none attached). */
int netc_ws_route_on_close(int sockfd, netc_ws_route_close_fn hook);

/** Registers the close hook of the send route attached to sockfd.  0, or -1 (EINVAL: none attached). */
int netc_ws_send_route_on_close(int sockfd, netc_ws_route_close_fn hook);

/** 1 when this process's close() reaches libnetc.so (lookups need no identity check), else 0. */
int netc_ws_route_close_tracked(void);

struct iovec;

/** Writes the iovecs' bytes on sockfd behind whatever its backlog holds, never waiting when dontwait
 *  (else the socket's own blocking mode decides): what the socket does not take joins the backlog.
 *  1 (all written or queued), or -1 (errno; netc_errno_reason BADSEND): a send error, or the bound. */
int netc_ws_send_nb(int sockfd, const struct iovec *iov, int iovcnt, int dontwait);

/** Writes what sockfd's backlog holds without waiting.  Bytes still held (0: empty), or -1 when the
 *  connection's sends failed (errno; BADSEND). */
long netc_ws_send_flush(int sockfd);

/** Bytes sockfd's backlog holds, or -1 when its sends failed. */
long netc_ws_send_pending(int sockfd);

/** Sets the per-connection backlog bound in bytes (0 = unbounded; default 64 MiB); returns the old one. */
size_t netc_ws_send_backlog_limit(size_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_ROUTE_H */
