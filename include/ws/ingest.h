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
 *   netc_ws_ingest_destroy()
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

/** netc_ws_ingest_create flag: reject what RFC 6455 forbids from a client (as NETC_WS_SCAN_STRICT). */
#define NETC_WS_INGEST_STRICT 1

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

/** Frame k's payload inside batch->wire: *offset, *length.  0 or NETC_GPU_EINVAL.  Host only. */
int netc_ws_batch_payload(const struct netc_ws_batch *batch, uint64_t k, uint64_t *offset, uint64_t *length);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_INGEST_H */
