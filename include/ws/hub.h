#ifndef NETC_WS_HUB_H
#define NETC_WS_HUB_H

/*
 * One GPU receive ring shared by many connections -- SURVEY.md §8(f) row 4 widened to the
 * shape of netc's server, MI355X (gfx950) edition.
 *
 * netc's server multiplexes every client on one event loop (reference src/tcp/server.c:30-75,
 * epoll over client_count + 1 descriptors) and calls ws_parse_frame for whichever client is
 * readable (src/web/server.c:69-98, the client looked up with map_get at :72).  An ingest ring
 * (include/ws/ingest.h) serves one connection; a hub serves all of them.  Every attached
 * connection's complete frames go into the same page-locked slots, back to back, so one H2D
 * copy and one unmask launch cover frames from many sockets -- the C2 shape of independent
 * frames with their own keys, produced by real sockets.
 *
 * Per connection the hub keeps only what a connection owns: the bytes of its incomplete frame
 * (a carry, host memory, grown to the frame's size), its partly reassembled message, and the
 * ranges of its frames in the shared slots.  The slots, their device buffers and streams are
 * shared: memory is bounded by the slots, not by the number of connections.
 *
 *   netc_ws_hub_create()         slots + device buffers on one GPU
 *   netc_ws_gpu_attach_hub()     serve netc's own ws_parse_frame on a socket from the hub
 *   netc_ws_gpu_detach_hub()
 *   netc_ws_hub_stats()          launches, frames, and how many connections each launch spanned
 *   netc_ws_hub_destroy()
 *
 * The route (include/ws/route.h) keeps ws_parse_frame's contract for netc's once-per-EPOLLIN
 * caller, as the single-connection route does: bytes are read ahead with MSG_PEEK and taken out
 * of the socket all but one, the hostage, which stays there while the hub holds bytes of that
 * connection it has not delivered -- so the level-triggered event fires again for each message
 * read ahead.  A call that has just read a connection's frames into the filling slot returns 1
 * with the hostage in place instead of launching at once: netc's loop goes on to the other
 * readable sockets, whose frames join the same slot, and the next call for the connection
 * submits the slot and delivers.  A slot that fills is submitted at once.
 *
 * Back-pressure: frames a connection has not yet been handed hold their slot.  When every slot
 * holds undelivered frames, a call for a connection with nothing pending reads nothing and
 * returns 1 (its socket stays readable) until the others drain -- a connection whose messages are
 * never asked for should be detached (its frames are then dropped) rather than left attached.
 * Reads never block: the route peeks with MSG_DONTWAIT, on blocking sockets too.
 *
 * Threading: a hub is driven by one thread -- the event loop's, as netc's server runs one loop
 * for all of its clients.  Errors as in include/ws/mask.h.
 */

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct netc_ws_hub;

/**
 * *out = a hub on `device`: nslots (2..64, 0 = 8) shared slots of slot_bytes each (0 = 16 MiB;
 * at least max_frame_bytes + 14), frames of at most max_frame_bytes payload bytes (0 = 65536,
 * the reference server's default limit, src/web/server.c:86).  flags: 0, or
 * NETC_WS_INGEST_STRICT (include/ws/ingest.h) to reject what RFC 6455 forbids a client.
 * Allocates the slots' page-locked host and device memory up front.  0 or a negative code.
 */
int netc_ws_hub_create(struct netc_ws_hub **out, int device, size_t slot_bytes, int nslots, size_t max_frame_bytes,
                       int flags);

/** Waits for the GPU work of every slot and frees everything; detach every socket first. */
void netc_ws_hub_destroy(struct netc_ws_hub *hub);

/**
 * While attached, libnetc's ws_parse_frame(client, &state, limit) on sockfd returns that
 * connection's next message from the hub, with the reference's contract (src/ws/common.c:134-348):
 * 0 and state->message filled (buffer owned by the caller, src/web/server.c:139), 1 when there is
 * nothing more now, WS_FRAME_PARSE_ERROR_* (PAYLOAD_TOO_BIG against `limit` or the hub's frame
 * limit; INVALID_FRAME_LENGTH for a header strict mode rejects; RECV once the peer closed and
 * every message was returned), or a NETC_GPU_E* code (-101..-105) for a device failure.  A socket
 * already served by a route is refused; re-attaching a socket to the same hub is a no-op.
 * 0 or NETC_GPU_EINVAL.
 */
int netc_ws_gpu_attach_hub(int sockfd, struct netc_ws_hub *hub);

/** Drops the connection from the hub (frames of it still in the slots are discarded).  0 or a code. */
int netc_ws_gpu_detach_hub(int sockfd);

/** Counters since creation. */
struct netc_ws_hub_stats
{
    uint64_t launches;          /* slots submitted to the GPU (one H2D + one unmask launch each) */
    uint64_t frames;            /* frames those slots held */
    uint64_t bytes;             /* bytes those slots held */
    uint64_t max_connections;   /* the most connections one launch held frames of */
    uint64_t connection_slots;  /* the sum over launches of the connections each held frames of */
    uint64_t connections;       /* connections attached now */
};
int netc_ws_hub_stats(const struct netc_ws_hub *hub, struct netc_ws_hub_stats *out);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_HUB_H */
