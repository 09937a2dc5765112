#ifndef NETC_WS_FRAME_H
#define NETC_WS_FRAME_H

/*
 * Send-side frame assembly for a batch of frames — the C-ABI of SURVEY.md §8(f)
 * row 2, MI355X (gfx950) edition.
 *
 * The reference frames one message at a time (ws_send_message,
 * src/ws/common.c:36-130): per frame it builds the 2-byte header (FIN | opcode,
 * MASK | 7-bit length code, :55-67), the 16- or 64-bit big-endian extended
 * length (:69-82), copies the payload and masks it (:96-107), and copies header,
 * key and payload into one frame buffer (:112-119) before send().  This header
 * turns that into ONE out-of-place device pass over a batch:
 *
 *   netc_ws_wire_size()       exact wire bytes of a batch (host)
 *   netc_gpu_encode_frames()  headers + keys + masked payloads of every frame,
 *                             back to back, into a device wire buffer
 *
 * Frames use the layout of include/ws/mask.h ("Frame layout", "Key packing"):
 * frame k's payload is [offsets[k], offsets[k+1]) of the payload buffer.  Each
 * frame also has its first header byte, header0[k] = FIN << 7 | RSV << 4 |
 * opcode (e.g. 0x82 = final BINARY, 0x01 = first TEXT fragment, 0x80 = final
 * continuation).  Header lengths follow the reference (:63): payloads of up to
 * 125 bytes use the 7-bit code, up to 65535 the 16-bit form, longer the 64-bit
 * form.  With masked != 0 every frame carries MASK and its 4 key bytes — also a
 * frame with an empty payload (RFC 6455 §5.2; the reference omits the key
 * there, defect B9 in DESIGN.md).  Errors as in include/ws/mask.h.
 */

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/** Largest header (+ key) of one frame: 2 + 8 extended length + 4 key bytes. */
#define NETC_WS_MAX_HEADER(masked) ((uint64_t)((masked) ? 14 : 10))

/** Upper bound of the wire bytes of nframes frames holding total_bytes of payload. */
#define NETC_WS_WIRE_BOUND(total_bytes, nframes, masked) \
    ((uint64_t)(total_bytes) + (uint64_t)(nframes) * NETC_WS_MAX_HEADER(masked))

/**
 * Exact wire bytes of frames 0..nframes-1 (host offsets, nframes + 1 entries):
 * the sum of header lengths and payload lengths.  Host only.
 */
uint64_t netc_ws_wire_size(const uint64_t *offsets, size_t nframes, int masked);

/**
 * Assemble the wire bytes of a device-resident batch of frames on `device`,
 * asynchronously on `stream`.
 *   d_wire            device output, wire_capacity bytes; must be at least
 *                     NETC_WS_WIRE_BOUND(total_bytes, nframes, masked) and must
 *                     not overlap the payload (out of place)
 *   d_wire_offsets    device output, nframes + 1 uint64: frame k's header starts
 *                     at wire byte d_wire_offsets[k]; d_wire_offsets[nframes] is
 *                     the wire length
 *   d_payload         device, total_bytes readable; frames as in mask.h
 *   d_frame_offsets   device, nframes + 1 uint64
 *   d_keys            device, nframes packed key32 words (ignored unless masked)
 *   d_header0         device, nframes header bytes, or NULL for 0x82 (final BINARY)
 * Wire bytes past d_wire_offsets[nframes] are not written.  Returns once the
 * kernels are queued.
 */
int netc_gpu_encode_frames(int device, void *d_wire, size_t wire_capacity, uint64_t *d_wire_offsets,
                           const void *d_payload, size_t total_bytes, const uint64_t *d_frame_offsets,
                           const uint32_t *d_keys, const uint8_t *d_header0, size_t nframes, int masked,
                           void *stream);

/** Length classes for netc_gpu_encode_frames_class: the extended-length bytes of every frame. */
#define NETC_WS_CLASS_7BIT  0   /* every payload 0..125 bytes     (header 2 B + key)  */
#define NETC_WS_CLASS_16BIT 2   /* every payload 126..65535 bytes (header 4 B + key)  */
#define NETC_WS_CLASS_64BIT 8   /* every payload 65536 bytes or more (10 B + key)     */

/** d_wire_offsets[nframes] after netc_gpu_encode_frames_class when a frame broke the class. */
#define NETC_WS_WIRE_INVALID UINT64_MAX

/**
 * netc_gpu_encode_frames for a batch whose frames all lie in one length class, as the caller
 * promises (length_class: NETC_WS_CLASS_*) -- e.g. a broadcast of equal-sized messages, or a
 * batch a host packer saw every length of.  The wire offsets are then affine in the payload
 * offsets, d_wire_offsets[k] = (offsets[k] - offsets[0]) + k * (2 + length_class + (masked ? 4 :
 * 0)), so the assembly computes them itself and writes them: one launch, where
 * netc_gpu_encode_frames runs a prefix scan over the frames before it.
 *
 * The promise is checked for every frame.  If a frame breaks it, d_wire_offsets[nframes] reads
 * NETC_WS_WIRE_INVALID once the call's work is done and the wire bytes are unspecified; no byte
 * outside the wire bound is written.  A batch that takes the general path -- one averaging under
 * 80 payload bytes per frame, one whose wire bound exceeds 256 MiB (there the scan costs less
 * than the one-launch form saves), or one the measurement knobs send to another path -- runs the
 * scan and is exact whatever its frames are.  Other arguments and errors as
 * netc_gpu_encode_frames.
 */
int netc_gpu_encode_frames_class(int device, void *d_wire, size_t wire_capacity, uint64_t *d_wire_offsets,
                                 const void *d_payload, size_t total_bytes, const uint64_t *d_frame_offsets,
                                 const uint32_t *d_keys, const uint8_t *d_header0, size_t nframes, int masked,
                                 int length_class, void *stream);

/* ---------------------------------------------------------- receive side -- */

/** netc_gpu_scan_frames flag: reject what RFC 6455 forbids from a client (see below). */
#define NETC_WS_SCAN_STRICT 1

/** d_result layout of netc_gpu_scan_frames. */
#define NETC_WS_SCAN_FRAMES   0   /* complete frames found (may exceed max_frames)        */
#define NETC_WS_SCAN_CONSUMED 1   /* offset of the first incomplete frame, or len        */
#define NETC_WS_SCAN_ERROR    2   /* offset of the first rejected header, or UINT64_MAX  */

/**
 * The frame boundaries of a received byte stream, found on `device` —
 * the header state machine of ws_parse_frame
 * (src/ws/common.c:146-296) over a whole buffer, in parallel.
 *   d_wire, len       device, the stream; the first header is at `start`
 *   flags             0: accept every header, as the reference does;
 *                     NETC_WS_SCAN_STRICT: stop at the first header with MASK
 *                     clear, an RSV bit set, a reserved opcode, a control frame
 *                     that is fragmented or longer than 125 bytes, or a 64-bit
 *                     length with its top bit set (RFC 6455 §5.1, §5.2, §5.5)
 *   d_hdr             device output, max_frames + 1 uint64: header offset of
 *                     frame k; d_hdr[n] = the consumed offset (when n <= max_frames)
 *   d_keys, d_b0      device outputs, max_frames each: packed key32 (0 when the
 *                     frame is unmasked) and header byte 0 (FIN | RSV | opcode)
 *   d_result          device output, 3 uint64 (NETC_WS_SCAN_*)
 * A frame counts when its header and whole payload lie inside [start, len); the
 * scan stops at the first frame that does not (its offset is CONSUMED — keep the
 * bytes from there for the next call) or, in strict mode, at a rejected header
 * (ERROR = CONSUMED = its offset).  Frames past max_frames are counted but not
 * recorded.  max_frames is also a density hint: when it allows 1 to 12 frames per 4 KiB of
 * stream (up to 128 MiB), the scan first tries its one-pass path for dense streams, with the
 * same results either way (NETC_GPU_KNOB_SCAN_ONEPASS, include/ws/mask.h).
 * Asynchronous on `stream`; read d_result after synchronising.
 * Scratch memory is allocated on first use per (device, stream) and reused until
 * netc_gpu_stream_release(device, stream) (include/ws/mask.h) frees it: call that
 * before destroying a stream the scan ran on.
 */
int netc_gpu_scan_frames(int device, const void *d_wire, size_t len, uint64_t start, int flags, uint64_t *d_hdr,
                         uint32_t *d_keys, uint8_t *d_b0, size_t max_frames, uint64_t *d_result, void *stream);

/** Same as netc_gpu_stream_release (include/ws/mask.h): frees ALL scratch kept for
 *  (device, stream) -- scan, assembly, UTF-8 flags; waits for that stream first.  0 or a code. */
int netc_gpu_scan_release(int device, void *stream);

/**
 * Diagnostics: waits for `stream`, then returns why the last netc_gpu_scan_frames
 * call on it finished with the serial walk instead of the parallel scan (0: it
 * did not; bits 0-7: a capacity overflowed — a chunk's candidate bucket, a
 * chunk's exit set, an exit onto no candidate, a tile's external list; 256+: the
 * tile resolution; 65536: a scan without NETC_WS_SCAN_STRICT -- which runs its
 * parallel pass with the strict checks except MASK, speculatively -- met a header
 * those checks reject and walked on serially from it), -1 when no scan ran on that
 * stream, or a negative code.  The results are the same either way; only the
 * speed differs.  Bit 32 is set when the call finished on its one-pass path (the
 * chunks resolved their entries and frame indexes inside the first launch; knob
 * SCAN_ONEPASS), clear when the graph kernels resolved it.
 */
int64_t netc_gpu_scan_diag(int device, void *stream);

/**
 * The same scan over a stream in host memory, on the calling thread (libnetc.so): the
 * header walk of ws_parse_frame (src/ws/common.c:146-296) hopping from header to header,
 * O(frames) instead of O(bytes).  Arguments, outputs (hdr[n] = the consumed offset when
 * n <= max_frames) and strict checks as netc_gpu_scan_frames, all pointers host memory.
 * Returns 0 or NETC_GPU_EINVAL.  The ingest ring uses it for slots of large frames.
 */
int netc_ws_scan_frames_host(const void *wire, size_t len, uint64_t start, int flags, uint64_t *hdr, uint32_t *keys,
                             uint8_t *b0, size_t max_frames, uint64_t *result);

/**
 * Unmask, in place, the payloads of the frames a netc_gpu_scan_frames call found
 * in d_wire (the reference's unmask loop, src/ws/common.c:317-323, for every
 * frame of the stream at once); header bytes and bytes past the last recorded
 * frame are left as they are.  d_hdr / d_keys / max_frames / d_result are that
 * call's outputs, read on the device: queue this on the same stream right after
 * the scan, no synchronisation needed.  Frames beyond max_frames are not unmasked.
 */
int netc_gpu_unmask_frames(int device, void *d_wire, size_t len, const uint64_t *d_hdr, const uint32_t *d_keys,
                           size_t max_frames, const uint64_t *d_result, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NETC_WS_FRAME_H */
