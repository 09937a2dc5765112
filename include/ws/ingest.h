#ifndef NETC_WS_INGEST_H
#define NETC_WS_INGEST_H

/*
 * Socket ingest into a pinned ring, framed and unmasked on the GPU — the C-ABI
 * of SURVEY.md §8(f) row 4, MI355X (gfx950) edition.
 *
 * The reference receives a client frame field by field: one recv() for byte 0
 * (src/ws/common.c:149), one for byte 1 (:172), one for the extended length
 * (:237), one for the key (:283), then the payload into the reassembly vector
 * (:303-306), which it unmasks byte by byte (:317-323).  Here a connection's
 * bytes go with large recv() calls straight into page-locked host slots.  A
 * filled slot is copied to the device, where the frame-boundary scan of
 * include/ws/frame.h finds its frames and the batch kernel unmasks every
 * payload in place; the unmasked stream comes back into the same page-locked
 * slot, the frame descriptors into page-locked arrays.  A frame cut by a slot
 * edge is carried to the front of the next slot, so every delivered frame is
 * whole, and batches come out in stream order.
 *
 *   netc_ws_ingest_create()    slots + device buffers on one GPU
 *   netc_ws_ingest_recv()      one recv() from a socket into the current slot
 *   netc_ws_ingest_write()     the same from memory (bytes that arrived elsewhere)
 *   netc_ws_ingest_submit()    send the current slot to the GPU now (done
 *                              automatically when a slot fills)
 *   netc_ws_ingest_next()      the oldest finished batch
 *   netc_ws_ingest_release()   hand a batch's slot back to the ring
 *   netc_ws_ingest_next_message()  the next reassembled message, in ws_parse_frame's
 *                              form (struct ws_message, 0 / 1 / WS_FRAME_PARSE_ERROR_*)
 *   netc_ws_ingest_destroy()
 *   netc_ws_ingest_scan_counts()  which scan found the frames of the slots so far
 *   netc_ws_batch_payload()    where frame k's payload lies in a batch
 *
 * Threading: an ingest object serves one connection from one thread at a time,
 * as the reference's per-connection parser state does (src/web/server.c:86);
 * objects are independent of each other.  Errors as in include/ws/mask.h:
 * negative codes, the thread-local netc_errno_reason (NETC_REASON_GPU, or
 * BADRECV = 10 for a failing recv), and netc_gpu_strerror().
 */

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct netc_ws_ingest;

/** netc_ws_ingest_create flag: reject what RFC 6455 forbids from a client (as NETC_WS_SCAN_STRICT).
 *  Without it (the default, 0) every header is accepted, as the reference's parser does. */
#define NETC_WS_INGEST_STRICT 1

/** Where a slot's frames are found (netc_ws_ingest_create flags).  Neither flag (the default):
 *  per slot, from the previous slot -- the host header walk over the pinned slot
 *  (netc_ws_scan_frames_host, O(frames)), whose descriptors go to the GPU with the bytes for
 *  the unmask only, when its frames averaged >= 16 KiB or (without NETC_WS_INGEST_STRICT) it
 *  held headers with RSV2 / RSV3 bits, reserved opcodes or fragmented control frames (the
 *  GPU scan's parallel pass stops at those; RSV1, which permessage-deflate sets, it accepts),
 *  or, when it was GPU-scanned, any part of it was walked serially for another reason (a
 *  capacity of the parallel pass overflowed: netc_gpu_scan_diag's nonzero reasons, which the
 *  host walk handles at its O(frames) cost); otherwise the GPU frame scan
 *  (netc_gpu_scan_frames, O(bytes), no host work).  The results are the same either way. */
#define NETC_WS_INGEST_SCAN_GPU  2   /* always the GPU frame scan */
#define NETC_WS_INGEST_SCAN_HOST 4   /* always the host header walk */

/* return codes of the ingest entries, besides 0 and the NETC_GPU_E* codes of mask.h */
#define NETC_WS_INGEST_CLOSED   -20   /* recv: the peer closed the connection (what it sent is submitted) */
#define NETC_WS_INGEST_FULL     -21   /* no free slot: take (next) and release batches first; nothing was read */
#define NETC_WS_INGEST_TOO_BIG  -22   /* a frame longer than max_frame_bytes (the reference's PAYLOAD_TOO_BIG) */
#define NETC_WS_INGEST_PROTOCOL -23   /* strict mode: a header RFC 6455 forbids; the stream ends before it */
#define NETC_WS_INGEST_ERECV    -24   /* recv() failed (errno kept, netc_errno_reason = BADRECV) */

/** A delivered batch: whole frames of the stream, payloads unmasked, in pinned host memory. */
struct netc_ws_batch
{
    const uint8_t *wire;      /* len stream bytes: headers as received, payloads unmasked */
    uint64_t len;             /* bytes of the batch's complete frames */
    const uint64_t *hdr;      /* nframes + 1 header offsets into wire; hdr[nframes] == len */
    const uint32_t *keys;     /* packed key32 of each frame (k0 | k1 << 8 | k2 << 16 | k3 << 24; 0 if unmasked) */
    const uint8_t *b0;        /* header byte 0 of each frame (FIN | RSV | opcode) */
    uint64_t nframes;
    uint64_t stream_offset;   /* position of wire[0] in the connection's byte stream */
    int32_t slot;             /* ring slot holding the batch (for netc_ws_ingest_release) */
};

/**
 * *out = a new ingest ring on `device`: nslots (2..16, 0 = 4) slots of
 * slot_bytes received bytes each (>= 4096, 0 = 16 MiB), frames of at most
 * max_frame_bytes payload bytes (0 = 65536, the reference server's default
 * limit, src/web/server.c:86).  Allocates page-locked host and device memory
 * up front; nothing is allocated later.  Returns 0 or a negative code.
 */
int netc_ws_ingest_create(struct netc_ws_ingest **out, int device, size_t slot_bytes, int nslots,
                          size_t max_frame_bytes, int flags);

/** Waits for the GPU work of every slot and frees everything (batches taken are invalid afterwards). */
void netc_ws_ingest_destroy(struct netc_ws_ingest *ing);

/**
 * One recv() from fd into the current slot (submitted when it fills).  Returns
 * the bytes read (> 0), 0 if the socket has nothing now (EAGAIN), or a negative
 * code: NETC_WS_INGEST_CLOSED, NETC_WS_INGEST_FULL, NETC_WS_INGEST_ERECV, or a
 * sticky stream error (TOO_BIG, PROTOCOL) once one was found.
 */
long netc_ws_ingest_recv(struct netc_ws_ingest *ing, int fd);

/** Appends len bytes of the stream from memory; returns the bytes taken (< len when the ring is full) or a code. */
long netc_ws_ingest_write(struct netc_ws_ingest *ing, const void *data, size_t len);

/** Sends the current slot's bytes to the GPU now (e.g. when the socket went idle).  0 or a code. */
int netc_ws_ingest_submit(struct netc_ws_ingest *ing);

/**
 * The oldest submitted batch, in stream order: 1 with *out filled, 0 when
 * none is finished (wait == 0) or none is in flight, or a negative code (a
 * sticky stream error is reported after the batch holding the frames before it).
 */
int netc_ws_ingest_next(struct netc_ws_ingest *ing, struct netc_ws_batch *out, int wait);

/** Returns a batch's slot to the ring.  0 or NETC_GPU_EINVAL. */
int netc_ws_ingest_release(struct netc_ws_ingest *ing, const struct netc_ws_batch *batch);

struct ws_message;   /* include/ws/common.h */

/**
 * The next complete message of the stream, with the reference's receive contract
 * (ws_parse_frame, include/ws/common.h; src/ws/common.c:146-347), read from the
 * delivered batches (payloads already unmasked on the GPU):
 *   0   *message is filled: opcode = the last non-continuation frame's opcode (:163-164),
 *       buffer = every frame's payload up to and including the one with FIN, back to
 *       back, in one malloc'd buffer the caller now owns and frees with free(); a TEXT
 *       message gets a NUL appended, counted in payload_length (:340-344)
 *   1   no complete message yet: receive more (netc_ws_ingest_recv / _write) and call
 *       again; with wait != 0 the call waits for batches already on the GPU
 *   WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG (-3)  the message's accumulated payload would
 *       exceed max_payload_length (:210-211, :261-262), or a frame exceeded the ring's
 *       max_frame_bytes
 *   WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH (-2)  strict mode rejected a header
 *   WS_FRAME_PARSE_ERROR_RECV (-1)  the peer closed (or recv failed) and every complete
 *       message before that point has been returned
 *   NETC_GPU_E*  a device / runtime failure
 * Errors are sticky: the connection is over, as with the reference (its caller closes
 * with 1002, src/web/server.c:88-95).  As in the reference, a control frame that arrives
 * between the fragments of a message is appended to that message and sets its opcode
 * (the reference's reassembly does not set control frames aside); a control frame
 * between messages is its own message.  A message the call has started stays in the
 * ring object (freed by netc_ws_ingest_destroy if never completed).  Batches are taken
 * and released by this call: do not mix it with netc_ws_ingest_next on one object.
 */
int netc_ws_ingest_next_message(struct netc_ws_ingest *ing, struct ws_message *message, size_t max_payload_length,
                                int wait);

/**
 * Serve netc's own ws_parse_frame (libnetc.so) on `sockfd` from `ring` (include/ws/route.h):
 * while attached, ws_parse_frame(client, &state, limit) on that socket takes the next message
 * from the ring -- frames found and unmasked on the GPU -- with the reference's contract
 * (src/ws/common.c:134-348): 0 and state->message filled (the caller frees message.buffer,
 * src/web/server.c:139), 1 when the socket has nothing more now, or WS_FRAME_PARSE_ERROR_*
 * (PAYLOAD_TOO_BIG against `limit`, RECV once the peer closed and every message was
 * returned); a device / runtime failure returns its NETC_GPU_E* code (-101..-105), never one of
 * those.  netc's caller calls ws_parse_frame ONCE per EPOLLIN (src/tcp/server.c:72-75 ->
 * src/web/server.c:86-98), and that is enough: the ring reads ahead with MSG_PEEK and takes the
 * peeked bytes out of the socket all but one, which it leaves there while it holds bytes it has
 * not delivered, so the level-triggered event fires again for every message already in the
 * ring (a caller may also call again after a 0 until it gets 1).  While the caller works on a
 * message, bytes that arrived since are sent to the GPU.  Other sockets keep the CPU parser.
 * One ring serves one connection: attaching a ring that already serves another open socket,
 * or one that has carried a stream, fails (NETC_GPU_EINVAL); so does a second ring on one
 * socket.  netc_ws_ingest_recv / _write on an attached ring are refused.  A route left behind
 * by a socket closed without a detach does not serve the next socket given its number.  One
 * thread per connection, as netc runs it; detach before destroying the ring.  0 or
 * NETC_GPU_EINVAL.
 */
int netc_ws_gpu_attach(int sockfd, struct netc_ws_ingest *ring);
int netc_ws_gpu_detach(int sockfd);

/** Slots submitted so far whose frames the GPU scan found (*gpu) / the host walk found (*host).  0 or EINVAL. */
int netc_ws_ingest_scan_counts(const struct netc_ws_ingest *ing, uint64_t *gpu, uint64_t *host);

/** Frame k's payload inside batch->wire: *offset, *length.  0 or NETC_GPU_EINVAL.  Host only. */
int netc_ws_batch_payload(const struct netc_ws_batch *batch, uint64_t k, uint64_t *offset, uint64_t *length);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_INGEST_H */
