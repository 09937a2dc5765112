#ifndef NETC_WS_EGRESS_H
#define NETC_WS_EGRESS_H

/*
 * Host-resident messages framed and masked on the GPU into a pinned ring, and
 * sent on a socket -- the send-side counterpart of include/ws/ingest.h
 * (SURVEY.md §8(f) row 2 from host buffers), MI355X (gfx950) edition.
 *
 * The reference sends a message frame by frame (ws_send_message,
 * src/ws/common.c:36-130): per frame a payload copy (:96-101), a byte-by-byte
 * mask (:104-107), a copy of header + key + payload into one stack buffer
 * (:112-119) and one send() (:121).  Here messages are appended to a
 * page-locked payload slot (the only host copy) with their frame table; a
 * submitted slot goes to the device, where netc_gpu_encode_frames writes every
 * frame's header, key and masked payload back to back, and the wire comes back
 * into a page-locked wire slot, ready for large send() calls.  Slots are
 * pipelined: while the GPU assembles one, the caller fills the next and sends
 * a finished one.
 *
 *   netc_ws_egress_create()    slots + device buffers on one GPU
 *   netc_ws_egress_queue()     append one message (split into frames as ws_send_message)
 *   netc_ws_egress_submit()    send the current slot to the GPU now (done
 *                              automatically when the next message does not fit)
 *   netc_ws_egress_next()      the oldest finished slot's wire bytes
 *   netc_ws_egress_release()   hand a wire batch's slot back to the ring
 *   netc_ws_egress_send()      send finished slots' wire bytes on a socket
 *   netc_ws_egress_flush()     submit, then send everything queued
 *   netc_ws_egress_destroy()
 *   netc_ws_gpu_attach_send()  serve netc's own ws_send_message on a socket from a ring
 *
 * Wire bytes are identical to libnetc's ws_send_message (host/ws_common.c) for
 * the same message, key and frame count: the reference's frame split (equal
 * parts, the remainder on the last frame, :42-49), its header forms (:55-82),
 * the same key on every frame, each frame's slice masked from key phase 0
 * (DESIGN.md B2), payload_length rather than strlen (B1, B3), and a masked empty
 * frame still carrying its key (RFC 6455 §5.2).
 *
 * Threading: an egress object serves one connection from one thread at a time,
 * as netc sends on a connection; objects are independent.  Errors as in
 * include/ws/mask.h: negative codes, netc_errno_reason, netc_gpu_strerror().
 */

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct netc_ws_egress;
struct ws_message;   /* include/ws/common.h */

/** netc_ws_egress_create flag for netc_ws_gpu_attach_send: ws_send_message returns once the message
 *  is queued; its bytes go out when its slot fills, or on netc_ws_egress_flush / _send.  Without it
 *  (the default) every ws_send_message is submitted and sent before it returns, as the CPU path. */
#define NETC_WS_EGRESS_DEFER 1

/* return codes of the egress entries, besides 0 and the NETC_GPU_E* codes of mask.h */
#define NETC_WS_EGRESS_FULL    -30   /* no free slot: take (next / send) and release finished slots first; nothing queued */
#define NETC_WS_EGRESS_TOO_BIG -31   /* the message's payload exceeds slot_bytes, or its frames max_frames */
#define NETC_WS_EGRESS_ESEND   -32   /* send() failed (errno kept, netc_errno_reason = BADSEND) or sent nothing */

/** A finished slot: the wire bytes of its messages, in queue order, in pinned host memory. */
struct netc_ws_wire
{
    const uint8_t *wire;   /* len bytes: every frame's header, key and masked payload */
    uint64_t len;
    uint64_t nframes;
    uint64_t nmessages;
    int32_t slot;          /* ring slot holding it (for netc_ws_egress_release) */
};

/**
 * *out = a new egress ring on `device`: nslots (2..16, 0 = 4) slots of slot_bytes
 * payload bytes each (>= 4096, 0 = 16 MiB) and max_frames frames each (0 =
 * slot_bytes / 64 + 64).  Allocates page-locked host and device memory up front.
 * flags: 0 or NETC_WS_EGRESS_DEFER.  Returns 0 or a negative code.
 */
int netc_ws_egress_create(struct netc_ws_egress **out, int device, size_t slot_bytes, int nslots, size_t max_frames,
                          int flags);

/** Waits for the GPU work of every slot and frees everything (wire batches taken are invalid afterwards). */
void netc_ws_egress_destroy(struct netc_ws_egress *eg);

/**
 * Appends one message: len payload bytes (copied now; the caller's buffer is free on
 * return), opcode on the first frame, num_frames frames (0 = 1) split as
 * ws_send_message splits them, masked with masking_key (4 bytes, the same on every
 * frame) or unmasked when masking_key is NULL.  A slot holds masked or unmasked frames,
 * not both: a change submits the current slot first, as does a message that does not
 * fit.  Returns 0, NETC_WS_EGRESS_FULL (no slot to put it in; nothing was queued),
 * NETC_WS_EGRESS_TOO_BIG, or a code.
 */
int netc_ws_egress_queue(struct netc_ws_egress *eg, const void *payload, size_t len, uint8_t opcode,
                         const uint8_t *masking_key, size_t num_frames);

/** Sends the current slot's messages to the GPU now.  0 or a code. */
int netc_ws_egress_submit(struct netc_ws_egress *eg);

/** The oldest submitted slot: 1 with *out filled, 0 when none is finished (wait == 0) or none is in flight, or a code. */
int netc_ws_egress_next(struct netc_ws_egress *eg, struct netc_ws_wire *out, int wait);

/** Returns a wire batch's slot to the ring.  0 or NETC_GPU_EINVAL. */
int netc_ws_egress_release(struct netc_ws_egress *eg, const struct netc_ws_wire *wire);

/**
 * Sends finished slots on fd, oldest first, each completely (a send that would block
 * waits for POLLOUT, as ws_send_message does), then releases them.  wait != 0 also
 * waits for slots still on the GPU.  Returns the bytes sent (>= 0) or a code
 * (NETC_WS_EGRESS_ESEND: the slot being sent is lost mid-way, as a failed
 * ws_send_message leaves its frames).
 */
long netc_ws_egress_send(struct netc_ws_egress *eg, int fd, int wait);

/** netc_ws_egress_submit, then netc_ws_egress_send(eg, fd, 1): everything queued is on the socket.  Bytes or a code. */
long netc_ws_egress_flush(struct netc_ws_egress *eg, int fd);

/**
 * Serve netc's own ws_send_message (libnetc.so) on `sockfd` from `ring`
 * (include/ws/route.h): while attached, ws_send_message(client, message, key,
 * num_frames) on that socket queues the message in the ring and -- unless the ring
 * was created with NETC_WS_EGRESS_DEFER -- submits it and sends it before
 * returning, with ws_send_message's contract: 1 once sent, else the failing send()
 * result (-1; netc_errno_reason BADSEND, or the ring's code in netc_gpu_strerror).
 * A message larger than the ring's slot_bytes (or in more frames than a slot
 * holds) is refused with -1 and NETC_WS_EGRESS_TOO_BIG in netc_gpu_strerror:
 * size the ring's slots for the connection's largest message.
 * Other sockets keep the CPU path.  One ring serves one connection: attaching a ring
 * that already serves another open socket, or one holding queued messages, fails
 * with NETC_GPU_EINVAL, and the route refuses a call for any other socket.  Detach
 * before destroying the ring: netc_ws_gpu_detach_send first sends every message a
 * DEFER ring still holds (ws_send_message returned 1 for them) and returns 0, or
 * the flush's negative code when they could not all be sent (the route is detached
 * either way).  0 or a negative code.
 */
int netc_ws_gpu_attach_send(int sockfd, struct netc_ws_egress *ring);
int netc_ws_gpu_detach_send(int sockfd);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_EGRESS_H */
