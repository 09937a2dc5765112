// Socket ingest into a pinned ring, framed and unmasked on the GPU:
// include/ws/ingest.h.
//
// The reference reads a frame field by field with one recv() per header field and
// the payload last (src/ws/common.c:149,172,237,283,306), then unmasks it byte by
// byte (:317-323).  Here the bytes of a connection land, with recv() calls as large
// as a slot, in page-locked host memory; per slot, on the slot's own HIP stream:
//
//   H2D     the slot's stream bytes: the carry of the previous slot + the new bytes
//   scan    netc_gpu_scan_frames' kernels -> header offsets, keys, byte 0s, result
//   D2H     the 3-word result (frames, consumed, error), then event "scanned"
//           (or, for a slot of large frames: the host header walk over the pinned
//           slot before the H2D, O(frames), and its descriptors H2D -- see kHostWalkMean)
//   unmask  every frame the scan found, in place (the batch kernel reads the frame
//           count on the device: no host round trip between scan and unmask)
//   D2H     the stream back into the same pinned slot, then event "done"
//
// The host needs one number per slot before the NEXT slot can go: where the last
// complete frame ends (the carry point).  It waits for the previous slot's
// "scanned" event only when the next slot is submitted -- by then the scan has
// long finished, a slot takes far longer to arrive on a socket than to scan.  The
// carried bytes (the incomplete frame at the slot's end) are still raw in the
// previous slot's pinned buffer: the unmask leaves bytes past the last complete
// frame as they are, so the copy back writes them unchanged.  They are copied in
// front of the next slot's received bytes (each slot keeps max-frame headroom in
// front for that), so every H2D is one contiguous range and every frame is whole.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/ioctl.h>
#include <sys/stat.h>
#include <sys/uio.h>

#include <new>

#include "ws_mask_gpu.h"

extern "C" {
#include "../../include/ws/mask.h"
#include "../../include/ws/frame.h"
#include "../../include/ws/ingest.h"
#include "../../include/ws/common.h"
#include "../../include/ws/route.h"
extern __thread int netc_errno_reason;   // include/utils/error.h
}

using netc_gpu::api_fail;
using netc_gpu::api_fail_hip;

namespace {

constexpr int kBadRecv = 10;   // netc's BADRECV reason (include/utils/error.h)
constexpr size_t kScratch = 1u << 20;   // discard buffer of the route on non-TCP sockets

// Default scan choice per slot: the host header walk when the previous slot's frames
// averaged at least this many bytes.  The walk costs the submitting thread one header
// parse per frame (<= 1,024 per 16 MiB slot at this size); the GPU scan reads every byte
// but costs the host nothing, so small frames stay on the GPU.
constexpr uint64_t kHostWalkMean = 16384;
// ... and for a slot of fewer bytes than this, whatever its frames: the GPU scan's fixed cost
// (its launches, ~20 us) is more than the walk of the few frames such a slot can hold, and a
// small slot is a latency case (one message submitted as it arrives)
constexpr uint64_t kHostWalkBytes = 64 * 1024;

enum SlotState : int { kFree = 0, kFilling, kInflight, kTaken };

struct IngestSlot {
    uint8_t* h_buf = nullptr;    // pinned: [0, carry_cap) carry room, then slot_bytes received; D2H target too
    uint8_t* d_buf = nullptr;    // device copy of the slot's stream
    uint64_t* d_hdr = nullptr;   // scan outputs (max_frames + 1 / max_frames / max_frames / 3)
    uint32_t* d_keys = nullptr;
    uint8_t* d_b0 = nullptr;
    uint64_t* d_res = nullptr;
    uint64_t* h_hdr = nullptr;   // pinned descriptor copies
    uint32_t* h_keys = nullptr;
    uint8_t* h_b0 = nullptr;
    uint64_t* h_res = nullptr;   // pinned: frames, consumed, error, then the scan's diag word (GPU scan)
    hipStream_t stream = nullptr;
    hipEvent_t scanned = nullptr, done = nullptr;
    netc_gpu::ScanScratch* scratch = nullptr;   // the frame scan's device scratch, sized for the slot
    int state = kFree;
    uint64_t fill = 0;           // received bytes, at h_buf + carry_cap
    uint64_t carry = 0;          // carried bytes in front of them, at h_buf + carry_cap - carry
    uint64_t pos = 0;            // stream position of the slot's first byte
    bool resolved = false;       // scan result read: frames and carry point known, descriptors queued
    uint64_t frames = 0;
    uint64_t cut = 0;            // end of the last complete frame (slot coordinates)
    uint64_t err = ~0ull;        // offset of a rejected header (strict), or ~0
    bool host_walk = false;      // frames found by the host header walk (descriptors already in h_*)
    bool slow_scan = false;      // the GPU scan walked part of the slot serially (diag != 0, e.g. RSV headers)
};

struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int device) {
        err = hipGetDevice(&prev);
        if (err != hipSuccess || prev == device) return;
        err = hipSetDevice(device);
        switched = err == hipSuccess;
    }
    ~DeviceGuard() {
        if (switched) (void)hipSetDevice(prev);
    }
};

// the message-level reader (netc_ws_ingest_next_message): the reference's reassembly
// state, src/ws/common.c:163-164,210-216,303-309,333-347
struct MessageState {
    bool have = false;           // a batch is taken and being read
    netc_ws_batch batch{};
    uint64_t k = 0;              // next frame of the batch
    uint8_t* buf = nullptr;      // the message so far (malloc; the caller's once delivered)
    size_t size = 0, cap = 0;
    uint8_t opcode = 0;          // the last non-continuation frame's opcode, as the reference
    int err = 0;                 // sticky message-level error (WS_FRAME_PARSE_ERROR_*)
    uint64_t end_pos = 0;        // stream position just past the last delivered message
};

// the socket a ring serves through ws_parse_frame (netc_ws_gpu_attach), and how far the
// route has taken bytes out of it: the route reads ahead with MSG_PEEK and removes bytes
// from the socket only up to the end of the message it returns (see gpu_route)
struct RouteState {
    int fd = -1;                 // attached socket, -1 = none
    uint64_t dev = 0, ino = 0;   // its identity at attach time (fstat), against fd reuse
    int tcp = 0;                 // TCP: discard with MSG_TRUNC (no copy); else recv into scratch
    uint64_t sock_pos = 0;       // stream bytes removed from the socket
    uint8_t* scratch = nullptr;  // discard buffer for non-TCP sockets
};

}  // namespace

struct netc_ws_ingest {
    int device = 0;
    int strict = 0;
    int scan_mode = 0;     // 0: per slot by frame size, NETC_WS_INGEST_SCAN_GPU / _HOST: always that
    uint64_t n_gpu = 0, n_host = 0;   // slots scanned each way
    int nslots = 0;
    uint64_t slot_bytes = 0, carry_cap = 0, cap = 0, max_frames = 0;
    IngestSlot* slots = nullptr;
    int cur = -1;          // slot being filled, -1 = none
    int next_fill = 0;     // the slot to fill next (ring order)
    int prev = -1;         // the last submitted slot: its carry goes in front of the next
    int fifo[16] = {0};    // submitted slots not yet handed out, in stream order
    int head = 0, count = 0;
    int sticky = 0;        // a stream error (TOO_BIG / PROTOCOL): reported from then on
    int sticky_after = -1; // ... once the batch of this slot has been handed out (-1: now)
    uint64_t max_frame = 0;   // max_frame_bytes (payload bytes per frame)
    bool closed = false;   // recv saw the peer close
    uint64_t in_pos = 0;   // stream bytes taken into the ring (recv / peek / write)
    MessageState msg;
    RouteState route;
};

namespace {

void free_slot(IngestSlot& s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    netc_gpu::scan_scratch_free(s.scratch);
    if (s.h_buf) (void)hipHostFree(s.h_buf);
    if (s.h_hdr) (void)hipHostFree(s.h_hdr);
    if (s.h_keys) (void)hipHostFree(s.h_keys);
    if (s.h_b0) (void)hipHostFree(s.h_b0);
    if (s.h_res) (void)hipHostFree(s.h_res);
    if (s.d_buf) (void)hipFree(s.d_buf);
    if (s.d_hdr) (void)hipFree(s.d_hdr);
    if (s.d_keys) (void)hipFree(s.d_keys);
    if (s.d_b0) (void)hipFree(s.d_b0);
    if (s.d_res) (void)hipFree(s.d_res);
    if (s.scanned) (void)hipEventDestroy(s.scanned);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = IngestSlot();
}

int alloc_slot(const netc_ws_ingest* g, IngestSlot& s) {
    hipError_t e;
    const uint64_t mf = g->max_frames;
    if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&s.scanned, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: stream / event create", e);
    if ((e = hipHostMalloc((void**)&s.h_buf, g->cap, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_hdr, (mf + 1) * sizeof(uint64_t), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_keys, mf * sizeof(uint32_t), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_b0, mf, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&s.h_res, 4 * sizeof(uint64_t), hipHostMallocDefault)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "ingest: pinned host allocation", e);
    if ((e = hipMalloc((void**)&s.d_buf, g->cap)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_hdr, (mf + 1) * sizeof(uint64_t))) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_keys, mf * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_b0, mf)) != hipSuccess ||
        (e = hipMalloc((void**)&s.d_res, 3 * sizeof(uint64_t))) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "ingest: device allocation", e);
    // the scan's scratch belongs to the slot (freed with it), sized for a full slot now
    if (!(s.scratch = netc_gpu::scan_scratch_new())) return api_fail(NETC_GPU_ENOMEM, "ingest: host allocation");
    if ((e = netc_gpu::scan_scratch_reserve(s.scratch, g->cap, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ENOMEM, "ingest: frame scan scratch", e);
    return 0;
}

// Wait for a submitted slot's scan result; fix its frames and carry point and
// queue the copy of its descriptors behind the unmask (the "done" event is
// recorded again after them).  Idempotent.
int resolve(netc_ws_ingest* g, IngestSlot& s) {
    if (s.resolved) return 0;
    hipError_t e = hipEventSynchronize(s.scanned);
    if (e != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: scan wait", e);
    const uint64_t n = s.h_res[0], consumed = s.h_res[1], len = s.carry + s.fill;
    // max_frames is sized so that every frame of a slot is recorded (>= 2 or 6 bytes each)
    if (n + 1 > g->max_frames || consumed > len)
        return api_fail(NETC_GPU_ERUNTIME, "ingest: scan result out of range (%llu frames, consumed %llu of %llu)",
                        (unsigned long long)n, (unsigned long long)consumed, (unsigned long long)len);
    s.frames = n;
    s.cut = consumed;
    s.err = s.h_res[2];
    s.slow_scan = (uint32_t)s.h_res[3] != 0;   // copied behind the result, before "scanned"
    if ((e = hipMemcpyAsync(s.h_hdr, s.d_hdr, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream)) !=
            hipSuccess ||
        (n && (e = hipMemcpyAsync(s.h_keys, s.d_keys, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream)) !=
                  hipSuccess) ||
        (n && (e = hipMemcpyAsync(s.h_b0, s.d_b0, n, hipMemcpyDeviceToHost, s.stream)) != hipSuccess) ||
        (e = hipEventRecord(s.done, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: descriptor copy", e);
    s.resolved = true;
    return 0;
}

// A non-strict stream whose previous slot held headers a client must not send (RSV2 / RSV3
// set; a reserved opcode; a fragmented control frame): the GPU scan's parallel pass filters
// like strict mode except for MASK and RSV1 (permessage-deflate) and would stop at the
// first of them and walk on serially, so such streams go to the host walk.
//   * GPU-scanned slot: the scan says so itself -- its diag word (nonzero when any part
//     of the slot was walked serially: a speculative stop at such a header, or a capacity
//     of the parallel pass overflowed -- adversarial payloads, for which the host walk is
//     the cheaper route too) is copied to h_res[3] before "scanned", so resolve() reads it
//     with the result.  The slot's descriptors (h_b0) are NOT read
//     here: their copy back is queued behind the unmask and may still be running.
//   * host-walked slot: h_b0 was written by the walk itself, before the submission.
bool unchecked_headers(const IngestSlot& p) {
    if (!p.host_walk) return p.slow_scan;
    uint32_t bad = 0;
    for (uint64_t k = 0; k < p.frames; ++k) {
        const uint32_t b = p.h_b0[k], op = b & 0x0F;
        bad |= (b & 0x30) | (op - 3 <= 4) | (op >= 11) | ((op >= 8) & !(b & 0x80));
    }
    return bad != 0;
}

int set_sticky(netc_ws_ingest* g, int code, int after_slot) {
    if (!g->sticky) {
        g->sticky = code;
        g->sticky_after = after_slot;
    }
    if (code == NETC_WS_INGEST_TOO_BIG)
        return api_fail(code, "ingest: a frame is longer than the %llu-byte limit",
                        (unsigned long long)(g->carry_cap - 14));
    return api_fail(code, "ingest: strict mode rejected a frame header (RFC 6455 §5.1-5.5)");
}

// the sticky error, once it is due (after the batch holding the frames before it)
int sticky_now(const netc_ws_ingest* g) {
    if (!g->sticky) return 0;
    if (g->sticky_after >= 0) {
        for (int i = 0; i < g->count; ++i)
            if (g->fifo[(g->head + i) % 16] == g->sticky_after) return 0;
    }
    return g->sticky;
}

// Queue the filling slot on the GPU (see the file comment).
int submit_cur(netc_ws_ingest* g) {
    if (g->cur < 0) return 0;
    IngestSlot& s = g->slots[g->cur];
    if (s.fill == 0) return 0;   // nothing new: the carry alone cannot complete a frame
    if (netc_gpu::inject_fault())
        return api_fail(NETC_GPU_ELAUNCH, "ingest: injected fault (NETC_GPU_KNOB_INJECT_FAULT)");
    uint64_t carry = 0, pos = 0;
    const uint8_t* carry_src = nullptr;
    bool host_walk = g->scan_mode == NETC_WS_INGEST_SCAN_HOST;
    if (g->prev >= 0) {
        IngestSlot& p = g->slots[g->prev];
        if (int r = resolve(g, p)) return r;
        if (p.err != ~0ull) return set_sticky(g, NETC_WS_INGEST_PROTOCOL, g->prev);
        carry = p.carry + p.fill - p.cut;
        carry_src = p.h_buf + (g->carry_cap - p.carry) + p.cut;
        pos = p.pos + p.cut;
        // no complete frame in a whole slot: the frames are larger than a slot
        if (g->scan_mode == 0)
            host_walk = p.frames == 0 || p.cut / p.frames >= kHostWalkMean || (!g->strict && unchecked_headers(p));
    }
    if (g->scan_mode == 0 && carry + s.fill < kHostWalkBytes) host_walk = true;
    if (carry > g->carry_cap) return set_sticky(g, NETC_WS_INGEST_TOO_BIG, g->prev);
    // the carried bytes are raw in the previous slot (the unmask stops at its last
    // complete frame, its copy back rewrites them unchanged)
    uint8_t* h = s.h_buf + (g->carry_cap - carry);
    if (carry) memmove(h, carry_src, carry);
    s.carry = carry;
    s.pos = pos;
    s.resolved = false;
    s.frames = s.cut = 0;
    s.err = ~0ull;
    s.host_walk = host_walk;
    s.slow_scan = false;
    const uint64_t len = carry + s.fill;
    hipError_t e;
    if (host_walk) {
        // the header walk over the pinned slot, then its descriptors go to the device
        // behind the bytes (the unmask reads them there, as it reads the GPU scan's)
        if (netc_ws_scan_frames_host(h, len, 0, g->strict ? NETC_WS_SCAN_STRICT : 0, s.h_hdr, s.h_keys, s.h_b0,
                                     g->max_frames, s.h_res) != 0)
            return api_fail(NETC_GPU_ERUNTIME, "ingest: host header walk");
        const uint64_t n = s.h_res[0];
        if (n + 1 > g->max_frames || s.h_res[1] > len)
            return api_fail(NETC_GPU_ERUNTIME, "ingest: host walk result out of range");
        s.frames = n;
        s.cut = s.h_res[1];
        s.err = s.h_res[2];
        s.resolved = true;
        if ((e = hipMemcpyAsync(s.d_buf, h, len, hipMemcpyHostToDevice, s.stream)) != hipSuccess ||
            (e = hipMemcpyAsync(s.d_hdr, s.h_hdr, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream)) !=
                hipSuccess ||
            (n && (e = hipMemcpyAsync(s.d_keys, s.h_keys, n * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream)) !=
                      hipSuccess) ||
            (e = hipMemcpyAsync(s.d_res, s.h_res, 3 * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream)) !=
                hipSuccess)
            return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: H2D copy", e);
        ++g->n_host;
    } else {
        if ((e = hipMemcpyAsync(s.d_buf, h, len, hipMemcpyHostToDevice, s.stream)) != hipSuccess)
            return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: H2D copy", e);
        if ((e = netc_gpu::launch_scan_frames(s.d_buf, len, 0, g->strict != 0, s.d_hdr, s.d_keys, s.d_b0,
                                              g->max_frames, s.d_res, s.stream, s.scratch)) != hipSuccess)
            return api_fail_hip(e == hipErrorOutOfMemory ? NETC_GPU_ENOMEM : NETC_GPU_ELAUNCH, "ingest: frame scan",
                                e);
        s.h_res[3] = 0;
        if ((e = hipMemcpyAsync(s.h_res, s.d_res, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream)) !=
                hipSuccess ||
            (e = hipMemcpyAsync(s.h_res + 3, netc_gpu::scan_scratch_diag_word(s.scratch), sizeof(uint32_t),
                                hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
            (e = hipEventRecord(s.scanned, s.stream)) != hipSuccess)
            return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: result copy", e);
        ++g->n_gpu;
    }
    if ((e = netc_gpu::launch_unmask_scanned(s.d_buf, len, s.d_hdr, s.d_keys, g->max_frames, s.d_res, s.stream,
                                             netc_gpu::api_cfg())) != hipSuccess)
        return api_fail_hip(e == hipErrorOutOfMemory ? NETC_GPU_ENOMEM : NETC_GPU_ELAUNCH, "ingest: unmask", e);
    if ((e = hipMemcpyAsync(h, s.d_buf, len, hipMemcpyDeviceToHost, s.stream)) != hipSuccess ||
        (e = hipEventRecord(s.done, s.stream)) != hipSuccess)
        return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: D2H copy", e);
    s.state = kInflight;
    g->fifo[(g->head + g->count) % 16] = g->cur;
    ++g->count;
    g->prev = g->cur;
    g->cur = -1;
    return 0;
}

// make a slot the filling one (ring order); NETC_WS_INGEST_FULL if it is still in use
int acquire(netc_ws_ingest* g) {
    if (g->cur >= 0) return 0;
    IngestSlot& s = g->slots[g->next_fill];
    if (s.state != kFree) return api_fail(NETC_WS_INGEST_FULL, "ingest: no free slot (take and release batches)");
    s.state = kFilling;
    s.fill = 0;
    g->cur = g->next_fill;
    g->next_fill = (g->next_fill + 1) % g->nslots;
    return 0;
}

}  // namespace

extern "C" {

int netc_ws_ingest_create(struct netc_ws_ingest** out, int device, size_t slot_bytes, int nslots,
                          size_t max_frame_bytes, int flags) {
    if (!out) return api_fail(NETC_GPU_EINVAL, "ingest: null output pointer");
    *out = nullptr;
    if (int r = netc_gpu::api_check_device(device)) return r;
    if (flags & ~(NETC_WS_INGEST_STRICT | NETC_WS_INGEST_SCAN_GPU | NETC_WS_INGEST_SCAN_HOST) ||
        (flags & NETC_WS_INGEST_SCAN_GPU && flags & NETC_WS_INGEST_SCAN_HOST))
        return api_fail(NETC_GPU_EINVAL, "ingest: unknown or conflicting flags 0x%x", flags);
    if (!slot_bytes) slot_bytes = 16u << 20;
    if (!nslots) nslots = 4;
    if (!max_frame_bytes) max_frame_bytes = 65536;
    if (slot_bytes < 4096 || slot_bytes > (1ull << 40) || nslots < 2 || nslots > 16 || max_frame_bytes > (1ull << 40))
        return api_fail(NETC_GPU_EINVAL, "ingest: need 4096 <= slot_bytes <= 2^40, 2 <= nslots <= 16, "
                                         "max_frame_bytes <= 2^40");
    DeviceGuard dg(device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    netc_ws_ingest* g = new (std::nothrow) netc_ws_ingest();
    if (!g) return api_fail(NETC_GPU_ENOMEM, "ingest: host allocation");
    g->device = device;
    g->strict = (flags & NETC_WS_INGEST_STRICT) ? 1 : 0;
    g->scan_mode = flags & (NETC_WS_INGEST_SCAN_GPU | NETC_WS_INGEST_SCAN_HOST);
    g->nslots = nslots;
    g->slot_bytes = slot_bytes;
    g->max_frame = max_frame_bytes;
    g->carry_cap = max_frame_bytes + 14;   // one whole frame: payload + the longest masked header
    g->cap = g->carry_cap + slot_bytes;
    // every frame is >= 6 bytes under the strict checks (masked), >= 2 otherwise
    g->max_frames = g->cap / (g->strict ? 6 : 2) + 2;
    g->slots = new (std::nothrow) IngestSlot[nslots];
    if (!g->slots) {
        delete g;
        return api_fail(NETC_GPU_ENOMEM, "ingest: host allocation");
    }
    for (int i = 0; i < nslots; ++i) {
        if (int r = alloc_slot(g, g->slots[i])) {
            for (int j = 0; j <= i; ++j) free_slot(g->slots[j]);
            delete[] g->slots;
            delete g;
            return r;
        }
    }
    *out = g;
    return 0;
}

void netc_ws_ingest_destroy(struct netc_ws_ingest* g) {
    if (!g) return;
    free(g->msg.buf);   // a message not completed yet (delivered ones are the caller's)
    free(g->route.scratch);
    DeviceGuard dg(g->device);
    for (int i = 0; i < g->nslots; ++i) free_slot(g->slots[i]);
    delete[] g->slots;
    delete g;
}

// One recv() into the current slot; the bytes read (> 0), 0 when the socket has none now, or a
// code.  skip >= 0 (the ws_parse_frame route): MSG_PEEK, the bytes stay in the socket until the
// route removes them (RouteState), and the first `skip` bytes the socket holds -- already in the
// ring, its hostage byte -- go to a scratch byte instead of the slot.
static long ring_recv(netc_ws_ingest* g, int fd, int skip = -1) {
    if (!g) return api_fail(NETC_GPU_EINVAL, "ingest: null ingest");
    if (g->sticky) return sticky_now(g) ? g->sticky : api_fail(g->sticky, "ingest: the stream has ended (error)");
    DeviceGuard dg(g->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    if (int r = acquire(g)) return r;
    if (g->slots[g->cur].fill == g->slot_bytes) {
        // a full slot whose submission failed earlier: submit it (or report why not) rather
        // than recv() into no room, which would read as the peer closing
        if (int e = submit_cur(g)) return e;
        if (int r = acquire(g)) return r;
    }
    IngestSlot& s = g->slots[g->cur];
    uint8_t* dst = s.h_buf + g->carry_cap + s.fill;
    const size_t room = (size_t)(g->slot_bytes - s.fill);
    ssize_t r;
    if (skip < 0) {
        do r = recv(fd, dst, room, 0);
        while (r < 0 && errno == EINTR);
    } else {
        uint8_t held[1];
        if (skip > (int)sizeof held) return api_fail(NETC_GPU_ERUNTIME, "ingest: %d bytes held in the socket", skip);
        struct iovec iov[2] = {{held, (size_t)skip}, {dst, room}};
        struct msghdr mh;
        memset(&mh, 0, sizeof mh);
        mh.msg_iov = skip ? iov : iov + 1;
        mh.msg_iovlen = skip ? 2 : 1;
        // MSG_DONTWAIT: the route peeks again after releasing its hostage, when the socket may
        // hold nothing -- a blocking socket must not stall the caller's loop there
        do r = recvmsg(fd, &mh, MSG_PEEK | MSG_DONTWAIT);
        while (r < 0 && errno == EINTR);
        if (r > 0 && r <= skip) return 0;   // only what the ring already has
        if (r > 0) r -= skip;
    }
    if (r < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) return 0;
        const int saved = errno;
        api_fail(NETC_WS_INGEST_ERECV, "ingest: recv: %s", strerror(saved));
        netc_errno_reason = kBadRecv;
        errno = saved;
        return NETC_WS_INGEST_ERECV;
    }
    if (r == 0) {   // the peer closed: what it sent goes to the GPU
        g->closed = true;
        if (int e = submit_cur(g)) return e;
        return api_fail(NETC_WS_INGEST_CLOSED, "ingest: the peer closed the connection");
    }
    s.fill += (uint64_t)r;
    g->in_pos += (uint64_t)r;
    if (s.fill == g->slot_bytes) {
        if (int e = submit_cur(g)) return e;
    }
    return (long)r;
}

long netc_ws_ingest_recv(struct netc_ws_ingest* g, int fd) {
    if (g && g->route.fd >= 0)
        return api_fail(NETC_GPU_EINVAL, "ingest: the ring serves socket %d through ws_parse_frame "
                        "(netc_ws_gpu_attach); detach it first", g->route.fd);
    return ring_recv(g, fd);
}

long netc_ws_ingest_write(struct netc_ws_ingest* g, const void* data, size_t len) {
    if (!g || (len && !data)) return api_fail(NETC_GPU_EINVAL, "ingest: null argument");
    if (g->route.fd >= 0)
        return api_fail(NETC_GPU_EINVAL, "ingest: the ring serves socket %d through ws_parse_frame", g->route.fd);
    if (g->sticky) return api_fail(g->sticky, "ingest: the stream has ended (error)");
    DeviceGuard dg(g->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    const uint8_t* p = (const uint8_t*)data;
    size_t taken = 0;
    while (taken < len) {
        if (int r = acquire(g)) return taken ? (long)taken : r;
        IngestSlot& s = g->slots[g->cur];
        const size_t room = (size_t)(g->slot_bytes - s.fill);
        const size_t k = len - taken < room ? len - taken : room;
        memcpy(s.h_buf + g->carry_cap + s.fill, p + taken, k);
        s.fill += k;
        taken += k;
        g->in_pos += k;
        if (s.fill == g->slot_bytes) {
            if (int e = submit_cur(g)) return e;
        }
    }
    return (long)taken;
}

int netc_ws_ingest_submit(struct netc_ws_ingest* g) {
    if (!g) return api_fail(NETC_GPU_EINVAL, "ingest: null ingest");
    if (g->sticky) return 0;
    DeviceGuard dg(g->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    return submit_cur(g);
}

int netc_ws_ingest_next(struct netc_ws_ingest* g, struct netc_ws_batch* out, int wait) {
    if (!g || !out) return api_fail(NETC_GPU_EINVAL, "ingest: null argument");
    if (const int st = sticky_now(g)) return api_fail(st, "ingest: the stream has ended (error)");
    if (g->count == 0) return 0;
    DeviceGuard dg(g->device);
    if (dg.err != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", dg.err);
    const int i = g->fifo[g->head];
    IngestSlot& s = g->slots[i];
    if (!wait) {
        const hipError_t q = hipEventQuery(s.done);
        if (q == hipErrorNotReady) return 0;
        if (q != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: event query", q);
    }
    if (int r = resolve(g, s)) return r;
    hipError_t e = hipEventSynchronize(s.done);
    if (e != hipSuccess) return api_fail_hip(NETC_GPU_ERUNTIME, "ingest: batch wait", e);
    out->wire = s.h_buf + (g->carry_cap - s.carry);
    out->len = s.cut;
    out->hdr = s.h_hdr;
    out->keys = s.h_keys;
    out->b0 = s.h_b0;
    out->nframes = s.frames;
    out->stream_offset = s.pos;
    out->slot = i;
    s.state = kTaken;
    g->head = (g->head + 1) % 16;
    --g->count;
    // the payload limit (the reference's PAYLOAD_TOO_BIG per frame, src/ws/common.c:210,261):
    // a longer frame ends the batch before it, and the stream with NETC_WS_INGEST_TOO_BIG
    // (frames that do not fit a slot's carry room never get here: submit_cur stops them)
    if (g->max_frame < s.carry + s.fill) {
        for (uint64_t k = 0; k < out->nframes; ++k) {
            uint64_t off = 0, len = 0;
            (void)netc_ws_batch_payload(out, k, &off, &len);
            if (len > g->max_frame) {
                out->nframes = k;
                out->len = out->hdr[k];
                set_sticky(g, NETC_WS_INGEST_TOO_BIG, i);   // reported from the next call on
                return 1;
            }
        }
    }
    if (s.err != ~0ull) set_sticky(g, NETC_WS_INGEST_PROTOCOL, i);   // reported from the next call on
    return 1;
}

int netc_ws_ingest_release(struct netc_ws_ingest* g, const struct netc_ws_batch* b) {
    if (!g || !b || b->slot < 0 || b->slot >= g->nslots || g->slots[b->slot].state != kTaken)
        return api_fail(NETC_GPU_EINVAL, "ingest: not a batch handed out by this ingest");
    g->slots[b->slot].state = kFree;
    return 0;
}

// the reference's error code for an ingest stream error (ws_parse_frame's contract)
static int message_code(int r) {
    switch (r) {
        case NETC_WS_INGEST_TOO_BIG: return WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG;
        case NETC_WS_INGEST_PROTOCOL: return WS_FRAME_PARSE_ERROR_INVALID_FRAME_LENGTH;
        case NETC_WS_INGEST_CLOSED:
        case NETC_WS_INGEST_ERECV: return WS_FRAME_PARSE_ERROR_RECV;
        default: return r;   // NETC_GPU_E* (a device / runtime failure)
    }
}

// a new message whose frames up to FIN are all in the batch: its buffer at its exact size
// (the payloads + a NUL), so the appends never reallocate and copy it again
static void msg_reserve_exact(MessageState& m, const netc_ws_batch& b, uint64_t k) {
    uint64_t need = 1;
    for (uint64_t j = k, stop = k + 1024 < b.nframes ? k + 1024 : b.nframes; j < stop; ++j) {
        uint64_t off = 0, len = 0;
        (void)netc_ws_batch_payload(&b, j, &off, &len);
        need += len;
        if (b.b0[j] & 0x80) {
            if ((m.buf = (uint8_t*)malloc(need))) m.cap = need;
            return;
        }
    }
}

static bool msg_append(MessageState& m, const uint8_t* p, size_t n) {
    if (m.size + n > m.cap || !m.buf) {
        size_t cap = m.cap ? m.cap : 64;
        while (cap < m.size + n) cap *= 2;
        uint8_t* nb = (uint8_t*)realloc(m.buf, cap);
        if (!nb) return false;
        m.buf = nb;
        m.cap = cap;
    }
    if (n) memcpy(m.buf + m.size, p, n);
    m.size += n;
    return true;
}

int netc_ws_ingest_next_message(struct netc_ws_ingest* g, struct ws_message* message, size_t max_payload_length,
                                int wait) {
    if (!g || !message) return api_fail(NETC_GPU_EINVAL, "ingest: null argument");
    MessageState& m = g->msg;
    if (m.err) return m.err;
    for (;;) {
        if (!m.have) {
            int r = netc_ws_ingest_next(g, &m.batch, wait);
            if (r == 0 && g->count == 0 && g->cur >= 0 && g->slots[g->cur].fill) {
                // nothing in flight but received bytes waiting: send them to the GPU now
                if (int e = netc_ws_ingest_submit(g)) return m.err = message_code(e);
                r = netc_ws_ingest_next(g, &m.batch, wait);
            }
            if (r < 0) return m.err = message_code(r);
            if (r == 0) {
                if (g->closed && g->count == 0 && (g->cur < 0 || g->slots[g->cur].fill == 0))
                    return m.err = WS_FRAME_PARSE_ERROR_RECV;   // the peer closed (recv() == 0, :151-154)
                return 1;                                      // need more data (:153)
            }
            m.have = true;
            m.k = 0;
        }
        const netc_ws_batch& b = m.batch;
        while (m.k < b.nframes) {
            const uint64_t k = m.k++;
            const uint8_t b0 = b.b0[k];
            const uint8_t op = b0 & 0x0F;
            uint64_t off = 0, len = 0;
            (void)netc_ws_batch_payload(&b, k, &off, &len);
            if (op != WS_OPCODE_CONTINUE) m.opcode = op;                        // :163-164
            if (len + m.size > max_payload_length)                             // :210-211, :261-262
                return m.err = WS_FRAME_PARSE_ERROR_PAYLOAD_TOO_BIG;
            if (!m.buf) msg_reserve_exact(m, b, k);
            if (!msg_append(m, b.wire + off, (size_t)len))
                return m.err = api_fail(NETC_GPU_ENOMEM, "ingest: message buffer");
            if (b0 & 0x80) {                                                    // FIN: the message (:340-346)
                if (m.opcode == WS_OPCODE_TEXT && !msg_append(m, (const uint8_t*)"", 1))
                    return m.err = api_fail(NETC_GPU_ENOMEM, "ingest: message buffer");
                if (!m.buf && !(m.buf = (uint8_t*)malloc(1)))   // an empty message still gets a buffer
                    return m.err = api_fail(NETC_GPU_ENOMEM, "ingest: message buffer");
                message->opcode = m.opcode;
                message->buffer = m.buf;
                message->payload_length = m.size;
                m.end_pos = b.stream_offset + b.hdr[k + 1];
                m.buf = nullptr;
                m.size = m.cap = 0;
                return 0;
            }
        }
        (void)netc_ws_ingest_release(g, &b);
        m.have = false;
    }
}

// Remove the socket's bytes up to stream position `to` (<= in_pos: the ring holds a copy of
// them, read with MSG_PEEK).  TCP discards them without a copy (recv with MSG_TRUNC and no
// buffer); other stream sockets refuse that (EFAULT, nothing taken) and read into scratch.
static int sock_consume(netc_ws_ingest* g, int fd, uint64_t to) {
    RouteState& rs = g->route;
    while (rs.sock_pos < to) {
        const uint64_t want = to - rs.sock_pos;
        ssize_t r;
        if (rs.tcp) {
            r = recv(fd, nullptr, (size_t)want, MSG_TRUNC | MSG_DONTWAIT);
            if (r < 0 && errno == EFAULT) {
                rs.tcp = 0;   // this socket copies: use the scratch from now on
                continue;
            }
        } else {
            if (!rs.scratch && !(rs.scratch = (uint8_t*)malloc(kScratch)))
                return api_fail(NETC_GPU_ENOMEM, "ingest: discard buffer");
            r = recv(fd, rs.scratch, (size_t)(want < kScratch ? want : kScratch), MSG_DONTWAIT);
        }
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {   // the bytes were peeked, so they are there: the socket has failed
            const int saved = r < 0 ? errno : ECONNRESET;
            api_fail(NETC_WS_INGEST_ERECV, "ingest: removing delivered bytes from socket %d: %s", fd,
                     strerror(saved));
            netc_errno_reason = kBadRecv;
            errno = saved;
            return NETC_WS_INGEST_ERECV;
        }
        rs.sock_pos += (uint64_t)r;
    }
    return 0;
}

// ws_parse_frame on a socket attached to a ring (include/ws/route.h): the reference's receive
// contract (src/ws/common.c:134-348) for its once-per-readiness-event caller
// (src/tcp/server.c:72-75 -> src/web/server.c:86-98, which calls ws_parse_frame ONCE per
// EPOLLIN and goes back to epoll_wait).
//
// The ring reads ahead -- MSG_PEEK as large as the slot's room, then the GPU scan and unmask
// over every frame in it -- and then takes the peeked bytes out of the socket (recv with
// MSG_TRUNC: no copy) all but the last one.  That byte, the hostage, stays in the socket as long
// as the ring holds bytes it has not delivered: the level-triggered event keeps firing for them,
// so a complete message never waits in the ring while the peer is quiet, and the socket buffer
// is still drained at once (the peer is not throttled by bytes the ring already has).  The
// hostage is released when the ring has delivered everything it read, or when it holds no
// complete message and the socket nothing new.  The next peek reads the hostage into a scratch
// byte (it is in the ring already).  While the caller works on a message, bytes that have
// arrived since go to the GPU (`pump`), so the next batch is in flight in the meantime.
//   0   state->message filled as ws_parse_frame fills it (opcode, caller-owned malloc'd
//       buffer, payload_length with a TEXT message's NUL); nothing else of the state is used
//   1   the socket has nothing more now and the ring no complete message
//   WS_FRAME_PARSE_ERROR_*   PAYLOAD_TOO_BIG against the caller's limit (or the ring's frame
//       limit); INVALID_FRAME_LENGTH for a header strict mode rejects; RECV once the peer
//       closed and every message before that was returned, or recv failed
//   NETC_GPU_E*   a device / runtime failure (-101..-105: never one of the above)

// peek what the socket has past the ring's bytes into the ring, then take it out of the socket
// but for the hostage; returns new bytes (> 0), 0 when nothing new, or a code (CLOSED, ...)
static long route_take(netc_ws_ingest* g, int fd) {
    RouteState& rs = g->route;
    const int held = (int)(g->in_pos - rs.sock_pos);   // 0 or 1
    long n = ring_recv(g, fd, held);
    if (n > 0) {
        if (int e = sock_consume(g, fd, g->in_pos - 1)) return e;
        return n;
    }
    if (n == 0 && held) {   // only the hostage: release it and look once more
        if (int e = sock_consume(g, fd, g->in_pos)) return e;
        n = ring_recv(g, fd, 0);
        if (n > 0) {
            if (int e = sock_consume(g, fd, g->in_pos - 1)) return e;
        }
    }
    return n;
}

// while the caller works on a delivered message: bytes that arrived since go to the GPU now
static void route_pump(netc_ws_ingest* g, int fd) {
    if (g->count != 0 || g->sticky) return;   // a batch is already on its way, or the stream is over
    int avail = 0;
    if (ioctl(fd, FIONREAD, &avail) != 0 || avail <= (int)(g->in_pos - g->route.sock_pos)) return;
    if (route_take(g, fd) > 0) (void)netc_ws_ingest_submit(g);   // (a failure resurfaces on the next call)
}

static int gpu_route(void* ctx, int sockfd, struct ws_frame_parsing_state* state, size_t max_payload_length) {
    netc_ws_ingest* g = (netc_ws_ingest*)ctx;
    if (sockfd != g->route.fd)
        return api_fail(NETC_GPU_EINVAL, "route: the ring serves socket %d, not %d", g->route.fd, sockfd);
    int full = 0;
    for (;;) {
        struct ws_message m;
        const int r = netc_ws_ingest_next_message(g, &m, max_payload_length, 1);
        if (r == 0) {
            // everything the ring read is delivered: the hostage goes too (a failing socket is
            // reported by the next call, after this message)
            if (g->msg.end_pos == g->in_pos && !g->msg.buf) (void)sock_consume(g, sockfd, g->in_pos);
            else route_pump(g, sockfd);
            state->message = m;
            return 0;
        }
        if (r < 0) return r;
        // no complete message in the ring: read on
        const long n = route_take(g, sockfd);
        if (n == 0) return 1;                              // drained: wait for readiness
        if (n > 0 || n == NETC_WS_INGEST_CLOSED) {         // (closed: what it sent is delivered first)
            full = 0;
            continue;
        }
        // no free slot: next_message releases slots as it consumes them; a ring that stays full
        // with no message completing cannot progress
        if (n == NETC_WS_INGEST_FULL && ++full < 3) continue;
        return g->msg.err = message_code((int)n);
    }
}

// the identity of an open socket (device, inode), to tell a reused descriptor from the attached one
static bool sock_identity(int fd, uint64_t* dev, uint64_t* ino) {
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISSOCK(st.st_mode)) return false;
    *dev = (uint64_t)st.st_dev;
    *ino = (uint64_t)st.st_ino;
    return true;
}

// close() on the attached socket (close tracking, include/ws/route.h): the ring lets go of it
static void ingest_close_hook(void* ctx, int sockfd) { (void)netc_ws_gpu_detach(sockfd); }

int netc_ws_gpu_attach(int sockfd, struct netc_ws_ingest* ring) {
    if (!ring) return api_fail(NETC_GPU_EINVAL, "attach: null ring");
    uint64_t dev = 0, ino = 0;
    if (!sock_identity(sockfd, &dev, &ino)) return api_fail(NETC_GPU_EINVAL, "attach: %d is not an open socket", sockfd);
    RouteState& rs = ring->route;
    if (rs.fd >= 0) {
        uint64_t d2 = 0, i2 = 0;
        const bool same = rs.fd == sockfd && rs.dev == dev && rs.ino == ino;
        if (same) return 0;   // already serving this connection
        if (sock_identity(rs.fd, &d2, &i2) && d2 == rs.dev && i2 == rs.ino)
            return api_fail(NETC_GPU_EINVAL, "attach: the ring already serves socket %d (one ring, one connection)",
                            rs.fd);
        // its connection was closed without a detach: drop the stale route if it is still ours
        void* ctx = nullptr;
        if (netc_ws_route_get_raw(rs.fd, &ctx) && ctx == ring) (void)netc_ws_route_detach(rs.fd);
        rs.fd = -1;
    }
    // a ring carries one connection's stream: a used one would splice two streams together
    if (ring->in_pos != 0 || ring->closed || ring->sticky || ring->msg.err)
        return api_fail(NETC_GPU_EINVAL, "attach: the ring has already carried a stream (create a fresh one)");
    int type = 0, domain = 0;
    socklen_t tl = sizeof type, dl = sizeof domain;
    if (getsockopt(sockfd, SOL_SOCKET, SO_TYPE, &type, &tl) != 0 || type != SOCK_STREAM)
        return api_fail(NETC_GPU_EINVAL, "attach: socket %d is not a stream socket", sockfd);
    (void)getsockopt(sockfd, SOL_SOCKET, SO_DOMAIN, &domain, &dl);
    const int r = netc_ws_route_attach(sockfd, gpu_route, ring);
    if (r != 0)
        return api_fail(NETC_GPU_EINVAL, "attach: socket %d: %s", sockfd,
                        errno == EBUSY ? "another route serves it" : "out of range");
    rs.fd = sockfd;
    rs.dev = dev;
    rs.ino = ino;
    rs.tcp = domain == AF_INET || domain == AF_INET6;
    rs.sock_pos = 0;
    (void)netc_ws_route_on_close(sockfd, ingest_close_hook);
    return 0;
}

int netc_ws_gpu_detach(int sockfd) {
    if (sockfd < 0) return api_fail(NETC_GPU_EINVAL, "detach: socket %d out of range", sockfd);
    void* ctx = nullptr;
    if (netc_ws_route_get_raw(sockfd, &ctx) == gpu_route && ctx) {
        netc_ws_ingest* g = (netc_ws_ingest*)ctx;
        if (g->route.fd == sockfd) g->route.fd = -1;
    }
    if (netc_ws_route_detach(sockfd) != 0) return api_fail(NETC_GPU_EINVAL, "detach: socket %d out of range", sockfd);
    return 0;
}

// diagnostics (tests): the ring's stream accounting
int netc_ws_ingest_debug_state(const struct netc_ws_ingest* g, uint64_t* out8) {
    if (!g || !out8) return NETC_GPU_EINVAL;
    out8[0] = g->in_pos;
    out8[1] = g->route.sock_pos;
    out8[2] = g->msg.end_pos;
    out8[3] = (uint64_t)g->count;
    out8[4] = g->cur >= 0 ? g->slots[g->cur].fill : ~0ull;
    out8[5] = g->msg.size;
    out8[6] = (uint64_t)(int64_t)(g->sticky ? g->sticky : g->msg.err);
    out8[7] = g->prev >= 0 ? g->slots[g->prev].pos + g->slots[g->prev].cut : 0;
    return 0;
}

int netc_ws_ingest_scan_counts(const struct netc_ws_ingest* g, uint64_t* gpu, uint64_t* host) {
    if (!g || !gpu || !host) return NETC_GPU_EINVAL;
    *gpu = g->n_gpu;
    *host = g->n_host;
    return 0;
}

int netc_ws_batch_payload(const struct netc_ws_batch* b, uint64_t k, uint64_t* offset, uint64_t* length) {
    if (!b || !offset || !length || k >= b->nframes) return NETC_GPU_EINVAL;
    // header bytes are as received (the unmask touches payloads only)
    const uint64_t h = b->hdr[k];
    const uint8_t second = b->wire[h + 1];
    const uint64_t code = second & 0x7F;
    const uint64_t hl = 2 + (code == 126 ? 2 : (code == 127 ? 8 : 0)) + ((second & 0x80) ? 4 : 0);
    *offset = h + hl;
    *length = b->hdr[k + 1] - (h + hl);
    return 0;
}

}  // extern "C"
