#ifndef NETC_WS_EGRESS_HUB_H
#define NETC_WS_EGRESS_HUB_H

/*
 * One GPU send ring shared by many connections -- the send side of include/ws/hub.h,
 * SURVEY.md §8(f) row 2 (frame assembly) in the shape of netc's server, MI355X (gfx950) edition.
 *
 * netc's server sends from its one event loop to whichever clients its callbacks answer: each
 * ws_send_message (reference src/ws/common.c:36-131) builds and masks one message and send()s
 * it, frame by frame (src/web/server.c:112, :381; src/ws/server.c:101, :123).  An egress ring
 * (include/ws/egress.h) serves one connection; an egress hub serves all of them: every attached
 * socket's messages go into the same page-locked slots, back to back, so ONE frame-assembly
 * launch (netc_gpu_encode_frames' kernels; one launch when the slot's frames are in one length
 * class) builds the wire bytes of many connections' messages, and each connection's bytes then
 * leave with one sendmsg() per slot (an iovec per run of its messages in the slot's wire).
 *
 *   netc_ws_egress_hub_create()      slots + device buffers on one GPU
 *   netc_ws_gpu_attach_send_hub()    serve netc's own ws_send_message on a socket from the hub
 *   netc_ws_egress_hub_flush()       frame every queued message on the GPU and send it
 *   netc_ws_gpu_detach_send_hub()
 *   netc_ws_egress_hub_stats()       launches, messages, and how many connections each launch spanned
 *   netc_ws_egress_hub_destroy()
 *
 * Contract.  While attached, ws_send_message(client, message, key, num_frames) on the socket
 * queues the message and returns 1 -- as an egress ring created with NETC_WS_EGRESS_DEFER does:
 * its bytes go out at the next netc_ws_egress_hub_flush (a server calls it once per loop
 * iteration, after its callbacks), or earlier when the slots run out (a full slot goes to the
 * GPU at once; with no slot free the oldest is sent first).  Per connection the bytes are
 * exactly libnetc's ws_send_message's for the same messages, keys and frame counts, in the
 * order they were queued (include/ws/egress.h lists the rules: the reference's split, header
 * forms, one key per message, each frame masked from its own first byte).
 *
 * Sends never wait (round 6): each connection's bytes leave with sendmsg(MSG_DONTWAIT), and what
 * its socket does not take moves to the connection's send backlog (include/ws/route.h), so the
 * slot is free at once and a client that stops reading delays nobody else.  The backlog goes
 * out ahead of the connection's later bytes at the next flush (or ws_send_message /
 * ws_parse_frame / netc_ws_send_flush on it); netc_ws_egress_hub_pending says how much is
 * held.  A backlog past its bound (netc_ws_send_backlog_limit) fails that connection alone.  A
 * connection whose send() fails (the peer went away) drops its remaining bytes; its next
 * ws_send_message returns -1 (netc_errno_reason BADSEND) and the failure is counted in the
 * stats.  A close frame (WS_OPCODE_CLOSE) is flushed as soon as it is queued, with everything
 * before it: netc closes the socket right after sending one (src/ws/server.c:123-124); with
 * close tracking (include/ws/route.h) a close() on an attached socket flushes and detaches it
 * first, so nothing queued for it is lost.  A message larger than slot_bytes, or in more frames than
 * a slot's table holds, is refused (-1, NETC_WS_EGRESS_TOO_BIG in netc_gpu_strerror).
 *
 * Threading: a hub is driven by one thread, the event loop's.  Errors as in include/ws/mask.h.
 */

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct netc_ws_egress_hub;

/**
 * *out = an egress hub on `device`: nslots (2..16, 0 = 4) shared slots of slot_bytes payload
 * bytes each (0 = 16 MiB, at least 4096), max_frames frames per slot (0 = slot_bytes / 64 + 64).
 * Allocates the slots' page-locked host and device memory up front.  0 or a negative code.
 */
int netc_ws_egress_hub_create(struct netc_ws_egress_hub **out, int device, size_t slot_bytes, int nslots,
                              size_t max_frames);

/** Sends what is queued (netc_ws_egress_hub_flush), then frees everything; detaches every socket. */
void netc_ws_egress_hub_destroy(struct netc_ws_egress_hub *hub);

/**
 * ws_send_message on sockfd now queues into the hub (see above).  A socket already served by
 * another send route is refused; re-attaching a socket to the same hub is a no-op.
 * 0 or NETC_GPU_EINVAL.
 */
int netc_ws_gpu_attach_send_hub(int sockfd, struct netc_ws_egress_hub *hub);

/**
 * Sends every message the hub holds for the socket (ws_send_message returned 1 for them; what its
 * socket does not take now stays in its backlog, ahead of its later CPU-path bytes), then drops
 * the socket's route.  0, or the flush's negative code (the route is dropped either way).
 */
int netc_ws_gpu_detach_send_hub(int sockfd);

/**
 * Every queued message framed on the GPU and sent: the filling slot is submitted, then each
 * slot in queue order is waited for and its connections' bytes are sent, never waiting for a
 * socket (what one does not take is held in its backlog), then the backlogs are written as far
 * as their sockets take them.  Bytes handed to the sockets or their backlogs (>= 0), or
 * a negative code for a device failure.  Per-connection send failures do not fail the flush.
 * A slot whose wire the device does not vouch for (its wire length is not the host's) fails
 * each of its connections as a failed send does, and the flush returns NETC_GPU_ERUNTIME after
 * sending the later slots; the hub goes on serving the other connections.
 */
long netc_ws_egress_hub_flush(struct netc_ws_egress_hub *hub);

/** Bytes the hub's connections hold in their send backlogs (0: everything is on the sockets). */
long netc_ws_egress_hub_pending(const struct netc_ws_egress_hub *hub);

/** Counters since creation. */
struct netc_ws_egress_hub_stats
{
    uint64_t launches;          /* slots framed on the GPU (one assembly per slot) */
    uint64_t messages;          /* messages those slots held */
    uint64_t frames;
    uint64_t wire_bytes;        /* bytes of wire they produced */
    uint64_t max_connections;   /* the most connections one launch held messages of */
    uint64_t connection_slots;  /* the sum over launches of the connections each held messages of */
    uint64_t sendmsg_calls;     /* sendmsg() calls that put those bytes on the sockets */
    uint64_t send_errors;       /* connections whose send() failed */
    uint64_t connections;       /* connections attached now */
    uint64_t deferred_sends;    /* times a connection's socket left bytes for its send backlog */
    uint64_t pending_bytes;     /* bytes its connections' backlogs hold now */
};
int netc_ws_egress_hub_stats(const struct netc_ws_egress_hub *hub, struct netc_ws_egress_hub_stats *out);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_EGRESS_HUB_H */
