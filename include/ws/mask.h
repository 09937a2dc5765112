#ifndef NETC_WS_MASK_H
#define NETC_WS_MASK_H

/*
 * RFC 6455 §5.3 payload masking — the drop-in C-ABI for netc's WebSocket
 * masking path, MI355X (gfx950) edition.
 *
 * The reference (Altanis/netc @ 2024-08-07) masks in two scalar per-byte loops:
 *   - receive / unmask  src/ws/common.c:317-323
 *       buffer_ptr[i] ^= frame.masking_key[(received_length + i) % 4];
 *   - send / mask       src/ws/common.c:104-107
 *       payload_data_encoded[i] ^= payload_masking_key[i % 4];
 * Both are out[i] = in[i] ^ key[(phase + i) mod 4] with the phase reset at
 * every frame start.  This header replaces those loops with:
 *
 *   netc_ws_mask()                 host CPU entry, one (partial) frame
 *                                  (libnetc.so; called by ws_parse_frame and
 *                                  ws_send_message of this repo)
 *   netc_gpu_mask_batch()          device-resident batch of frames on one GPU
 *                                  (libnetc_ws_gpu.so, HIP / gfx950)
 *   netc_gpu_mask_batch_multi()    the same, sharded across several GPUs of
 *                                  one node, no collective
 *   netc_gpu_mask_stream_host()    host→device→host pipeline through pinned
 *                                  staging slots on overlapped HIP streams
 *   netc_shard_frames()            byte-balanced frame partition (host)
 *
 * No HIP / torch types appear here: device buffers are plain pointers and a
 * stream is an opaque `void *` (a hipStream_t, NULL = the default stream).
 *
 * Key packing.  A frame's 4 wire key bytes k0 k1 k2 k3 (the order they appear
 * on the wire, struct ws_frame.masking_key in include/ws/common.h) travel as
 * one little-endian word: key32 = k0 | k1 << 8 | k2 << 16 | k3 << 24.
 *
 * Frame layout.  Frame k covers payload bytes [offsets[k], offsets[k+1]) of
 * the batch; offsets has nframes + 1 entries, is non-decreasing and
 * offsets[nframes] <= total_bytes.  Bytes of [0, total_bytes) that lie in no
 * frame are passed through unmasked (copied when dst != src).  Frames may be
 * of any length, including 0, and start at any byte offset (frames are packed
 * back to back, unpadded).  Each frame's phase starts at 0 (RFC 6455; the
 * reference's receive path, src/ws/common.c:301,337).
 *
 * Errors.  Every int-returning entry returns 0 on success or a negative
 * NETC_GPU_E* code; the failing call also sets the thread-local
 * netc_errno_reason (include/utils/error.h) to NETC_REASON_GPU and records
 * a message readable with netc_gpu_strerror().  Nothing here aborts, and the
 * caller owns every buffer.  Entry points are reentrant and thread-safe;
 * the first GPU call on a thread initialises the HIP runtime (call
 * netc_gpu_init() up front to keep that off an event loop).
 */

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* -------------------------------------------------------------- errors -- */
/* Numbered apart from ws_parse_frame's WS_FRAME_PARSE_ERROR_* (-1..-3, include/ws/common.h:42-50),
   which a GPU route returns through the kept API: a device failure must never read as
   "payload too big" to netc's web layer (src/web/server.c:88-95). */
#define NETC_GPU_OK          0
#define NETC_GPU_EINVAL   -101   /* bad argument (null buffer, bad sizes, partial overlap) */
#define NETC_GPU_ENODEV   -102   /* no such device / HIP runtime has no GPU                */
#define NETC_GPU_ELAUNCH  -103   /* kernel launch failed                                   */
#define NETC_GPU_ERUNTIME -104   /* a HIP runtime call failed (memcpy, stream, event …)    */
#define NETC_GPU_ENOMEM   -105   /* device or pinned host allocation failed                */

/** netc_errno_reason value set by a failing GPU entry (extends include/utils/error.h:28-45). */
#define NETC_REASON_GPU   18

/* ---------------------------------------------------------------- host -- */

/**
 * dst[i] = src[i] ^ key[(phase + i) & 3] for i < len.  dst == src is allowed
 * (in place, as the reference's receive path); other overlaps are not.
 * Replaces src/ws/common.c:319-322 (phase = received_length) and
 * src/ws/common.c:104-107 (phase = 0).  Host memory only; never touches a GPU.
 */
void netc_ws_mask(uint8_t *dst, const uint8_t *src, size_t len, const uint8_t key[4], size_t phase);

/**
 * Partition frames 0..nframes-1 (host offsets, nframes + 1 entries) into
 * nshards contiguous ranges balanced by payload bytes, cutting only at frame
 * boundaries.  Writes nshards + 1 frame indices to cuts (cuts[0] = 0,
 * cuts[nshards] = nframes).  Returns 0 or NETC_GPU_EINVAL.
 */
int netc_shard_frames(const uint64_t *offsets, size_t nframes, size_t nshards, size_t *cuts);

/* ----------------------------------------------------------------- gpu -- */

/** Number of visible GPUs (0 when the runtime has none); never negative. */
int netc_gpu_device_count(void);

/** Eagerly initialise the HIP runtime on `device`.  Optional. */
int netc_gpu_init(int device);

/**
 * Process-wide launch shape of the batch kernel (defaults: 1, 0, AUTO).
 * unroll: KiB of payload a wavefront loads at once (1, 2, 4 or 8); flags:
 * NETC_GPU_TUNE_AUTO (non-temporal payload stream; a grid covering the batch, one
 * window of two steps of `unroll` KiB per wavefront) or a mix of the bits below
 * (0 = plain loads / stores, one step per window).  NETC_GPU_TUNE_PERSISTENT
 * selects round 1's walk — one resident round of workgroups striding over the
 * chunks — where max_blocks caps the workgroups (0 = exactly the workgroups the
 * device holds at once); max_blocks is ignored otherwise.  The frame assembly of
 * include/ws/frame.h reads the same knob: 2 or 4 select 2 KiB chunks there, any
 * other value 4 KiB (the default; pipelined above 256 MiB, knob ENC_PF), and it
 * always walks persistently.  Diagnostic knob.  The
 * shape is one atomic word: a launch on another thread sees the old shape or the
 * new one, never a mix.
 */
#define NETC_GPU_TUNE_AUTO       -1
#define NETC_GPU_TUNE_NT_LOADS    1   /* non-temporal payload loads                        */
#define NETC_GPU_TUNE_NT_STORES   2   /* non-temporal payload stores                       */
#define NETC_GPU_TUNE_PERSISTENT  4   /* round 1's persistent grid-stride walk             */
#define NETC_GPU_TUNE_TWO_STEPS   8   /* a wavefront's window is two steps of unroll KiB   */
#define NETC_GPU_TUNE_XCD_ORDER  16   /* each XCD takes a contiguous share of the windows  */
#define NETC_GPU_TUNE_XCD_GROUPS 32   /* each XCD takes 8 consecutive blocks of every 64    */
int netc_gpu_tune(int unroll, int max_blocks, int flags);

/**
 * Measurement / test knobs of the §8(f) kernels (defaults in brackets).  Each is one
 * atomic word, seeded once per process from the environment variable named beside
 * it; value < 0 restores the default.  Returns 0 or NETC_GPU_EINVAL.
 *   ENC_DENSE_BYTES    mean payload bytes per frame under which netc_gpu_encode_frames
 *                      composes every span per lane [80]          (NETC_ENC_DENSE_BYTES)
 *   ENC_SCAN_PER       frames per thread of the wire-offsets scan, 1/2/4/8/16
 *                      [4 up to 256 Ki frames, else 16]            (NETC_ENC_SCAN_PER)
 *   SCAN_FAST_RANK     0 sends the frame scan's list ranking through the generic
 *                      loop [1]                                     (NETC_SCAN_FAST_RANK)
 *   SCAN_ANCHOR_SLOTS  cap on the frame scan's anchor slots [all]  (NETC_SCAN_ANCHOR_SLOTS)
 *   VAL_STEPS          netc_gpu_unmask_validate's 4 KiB window as 1, 2 or 4 steps
 *                      [2 up to 256 MiB, 1 above]                  (NETC_VAL_STEPS)
 *   SCAN_FUSE          the frame scan's links / tiles / resolve phases: 0 three launches;
 *                      1 one launch up to 512 MiB (arrival counters; sc1 hand-offs);
 *                      2 links, then tiles + resolve as one launch up to 256 MiB
 *                      [one launch on the one-pass path (SCAN_ONEPASS) up to 128 MiB,
 *                      else as 2]
 *                                                                  (NETC_SCAN_FUSE)
 *   ENC_SRC            1 selects the source-driven frame assembly (one pass over the payload
 *                      buffer, headers written in it; measured slower than the default
 *                      wire-driven kernels + header fixups) [0]      (NETC_ENC_SRC)
 *   MASK_TAPER         bytes at the end of a netc_gpu_mask_batch batch walked in one-step
 *                      windows instead of two-step ones, so the launch's last waves are
 *                      short and finish together [0]               (NETC_MASK_TAPER)
 *   ENC_FIX            where netc_gpu_encode_frames composes the 16-B vectors holding header
 *                      bytes: 0 trailing blocks of the assembly launch; 1 the wire-offsets
 *                      scan (measured slower); 2 the assembly's own wavefronts after their
 *                      windows [0]                                  (NETC_ENC_FIX)
 *   ENC_PROBE          entries of the frame assembly's first table probe per chunk, when dense:
 *                      0 always 64 (round 4's table), > 0 that many more than the default
 *                      (expected frames + 10) [default]             (NETC_ENC_PROBE)
 *   ENC_PF             the frame assembly's walk software-pipelined -- a chunk's payload loads
 *                      issued before the previous chunk is stored: 0 never; 1 2 KiB chunks at
 *                      5 wavefronts per SIMD; 2 4 KiB chunks at 4 [2 above 256 MiB of wire,
 *                      else 0]                                      (NETC_ENC_PF)
 *   SCAN_BLOCK_CHUNKS  chunks per block of the frame scan's link and emit phases: 32 or 64
 *                      [32 up to 128 MiB of stream, 64 above]       (NETC_SCAN_BLOCK_CHUNKS)
 *   SCAN_ONEPASS       the frame scan's one-pass path (K1 publishes each chunk's exit
 *                      prediction; one launch speculates every chunk's entry from them, walks
 *                      and checks it and writes the frames; the graph kernels then only check
 *                      a flag): 0 never, 1 forced up to 256 MiB of stream, 2 forced up to
 *                      128 MiB [up to 128 MiB when max_frames allows 1-12 frames per 4 KiB
 *                      chunk; DESIGN.md §16.4]                      (NETC_SCAN_ONEPASS)
 *   INJECT_FAULT       fault injection for tests: the ingest / egress ring submission this
 *                      countdown reaches (0 = the next one) fails as NETC_GPU_ELAUNCH
 *                      without launching, then the knob disarms itself [off]
 *                                                                  (NETC_INJECT_FAULT)
 */
#define NETC_GPU_KNOB_ENC_DENSE_BYTES   1
#define NETC_GPU_KNOB_ENC_SCAN_PER      2
#define NETC_GPU_KNOB_SCAN_FAST_RANK    3
#define NETC_GPU_KNOB_SCAN_ANCHOR_SLOTS 4
#define NETC_GPU_KNOB_VAL_STEPS         5
#define NETC_GPU_KNOB_SCAN_FUSE         6
#define NETC_GPU_KNOB_MASK_TAPER        7
#define NETC_GPU_KNOB_ENC_SRC           8
#define NETC_GPU_KNOB_ENC_FIX           9
#define NETC_GPU_KNOB_INJECT_FAULT     10
#define NETC_GPU_KNOB_ENC_PROBE        11
#define NETC_GPU_KNOB_ENC_PF           12
#define NETC_GPU_KNOB_SCAN_BLOCK_CHUNKS 13
#define NETC_GPU_KNOB_SCAN_ONEPASS     14
int netc_gpu_knob(int knob, int64_t value);

/**
 * Free every piece of scratch this library keeps for (device, stream): the frame
 * scan's (netc_gpu_scan_frames, include/ws/frame.h), the frame assembly's
 * (netc_gpu_encode_frames) and the UTF-8 flags of netc_gpu_unmask_validate.  It
 * synchronises the stream first.  Call it before destroying a stream those entries
 * ran on; a later call on the stream allocates afresh.  netc_gpu_scan_release is
 * the same call under its round-1 name.
 */
int netc_gpu_stream_release(int device, void *stream);

/** Message for the last failing netc_gpu_* call on this thread ("" if none). */
const char *netc_gpu_strerror(void);

/**
 * Mask (or unmask — the operation is an involution) a device-resident batch of
 * frames on `device`, asynchronously on `stream`.
 *   d_dst, d_src      device buffers of total_bytes; d_dst == d_src is in place
 *   d_frame_offsets   device, nframes + 1 uint64 (see "Frame layout")
 *   d_keys            device, nframes packed key32 words
 * Returns once the kernel is queued; synchronise `stream` before reading d_dst.
 * The batch is processed by one kernel launch whose only device traffic is the
 * payload read + write plus 12 B per frame of descriptors.
 */
int netc_gpu_mask_batch(int device, void *d_dst, const void *d_src, size_t total_bytes,
                        const uint64_t *d_frame_offsets, const uint32_t *d_keys, size_t nframes,
                        void *stream);

/**
 * netc_gpu_mask_batch plus, in the same pass over the bytes, the UTF-8 check RFC
 * 6455 §8.1 requires of TEXT messages (RFC 3629: shortest form, no surrogates,
 * nothing above U+10FFFF) — SURVEY.md §8(f) row 3; the reference never checks
 * (src/ws/common.c:342 only appends a NUL).
 *   d_header0   device, nframes bytes: header byte 0 of each frame (FIN | RSV | opcode)
 *   d_valid     device output, nframes bytes
 * A TEXT message is a frame with opcode 1 and the continuation frames (opcode 0)
 * after it up to the first with FIN; control frames between them (opcode >= 8)
 * are not part of it.  d_valid[k] = 0 on the FIN frame of a TEXT message whose
 * unmasked payload, concatenated over its frames, is not valid UTF-8 (a code point
 * may be split between frames); 1 everywhere else — other messages, and a message
 * the batch does not finish.  d_dst receives the unmasked payload as with
 * netc_gpu_mask_batch.  Scratch of nframes bytes is kept per (device, stream).
 */
int netc_gpu_unmask_validate(int device, void *d_dst, const void *d_src, size_t total_bytes,
                             const uint64_t *d_frame_offsets, const uint32_t *d_keys, const uint8_t *d_header0,
                             size_t nframes, uint8_t *d_valid, void *stream);

/**
 * One shard per device, already resident: shard i lives on devices[i] and is
 * described exactly as for netc_gpu_mask_batch (offsets rebased to the shard's
 * own payload start).  All shards are launched before any is waited for; with
 * `synchronize` != 0 the call returns after every shard has completed.
 * streams may be NULL (each device's default stream).  No collective is used:
 * frames are independent.  On failure no work of the call is left in flight: the
 * shards before the failing one have completed (they are synchronised before the
 * call returns), the failing shard and the ones after it were not launched, and
 * netc_gpu_strerror() names the failing shard ("shard i ...").
 */
int netc_gpu_mask_batch_multi(int nshards, const int *devices, void *const *d_dst, const void *const *d_src,
                              const size_t *total_bytes, const uint64_t *const *d_frame_offsets,
                              const uint32_t *const *d_keys, const size_t *nframes, void *const *streams,
                              int synchronize);

/**
 * Host-resident batch: h_src → device → mask → h_dst, through `nslots`
 * device slots of `slot_bytes` payload bytes each, cut at frame boundaries, with
 * H2D copy, kernel and D2H copy of consecutive slots overlapped on separate HIP
 * streams (BASELINE config 5).  h_offsets / h_keys are host arrays laid out as for
 * netc_gpu_mask_batch.  h_dst == h_src is allowed.  A frame longer than
 * slot_bytes is split across slots (its phase is carried).  Synchronous: returns
 * when h_dst is complete.  Page-locked h_src / h_dst (netc_gpu_host_alloc, or
 * hipHostMalloc / hipHostRegister) run at the PCIe rate; pageable memory works
 * but is slower (the runtime stages it).  Two slots of 512 MiB are the fastest
 * shape measured on MI355X (one copy in each direction in flight).
 *
 * netc_gpu_stream_create / _mask / _destroy: the same pipeline with the slots,
 * streams, events and descriptor staging kept in a handle across calls (a call
 * allocates only when one of its slots holds more frames than any earlier call's
 * did).  slot_bytes 0 = 512 MiB, nslots 0 = 2.  A handle serves one thread at a
 * time.  netc_gpu_mask_stream_host is create + mask + destroy.
 */
int netc_gpu_mask_stream_host(int device, void *h_dst, const void *h_src, size_t total_bytes,
                              const uint64_t *h_frame_offsets, const uint32_t *h_keys, size_t nframes,
                              size_t slot_bytes, int nslots);

struct netc_gpu_stream;
int netc_gpu_stream_create(struct netc_gpu_stream **out, int device, size_t slot_bytes, int nslots);
int netc_gpu_stream_mask(struct netc_gpu_stream *stream, void *h_dst, const void *h_src, size_t total_bytes,
                         const uint64_t *h_frame_offsets, const uint32_t *h_keys, size_t nframes);
void netc_gpu_stream_destroy(struct netc_gpu_stream *stream);

/**
 * Page-locked host memory for the host side of the pipeline (the pinned receive
 * ring of a netc server): NULL on failure (error set as above).  Free with
 * netc_gpu_host_free.
 */
void *netc_gpu_host_alloc(size_t bytes);
void netc_gpu_host_free(void *ptr);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_MASK_H */
