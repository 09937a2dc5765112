// C-ABI for the gfx950 masking kernels: include/ws/mask.h (GPU half).
// Built into libnetc_ws_gpu.so, which links libnetc.so for netc_errno_reason.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

#include "ws_mask_gpu.h"

extern "C" {
#include "../../include/ws/mask.h"
#include "../../include/ws/frame.h"
// netc's thread-local error side channel (include/utils/error.h:19-23, src/utils/error.c:5)
extern __thread int netc_errno_reason;
}

namespace {

thread_local char g_err[512];

// Process-wide launch shape (netc_gpu_tune) as ONE atomic word, so a launch on another
// thread reads either the old shape or the new one, never a mix: bits 0-7 unroll, 8-39
// max_blocks, 40-63 flags + 1 (flags is -1 for auto).
uint64_t pack_cfg(int unroll, int max_blocks, int flags) {
    return (uint64_t)(uint8_t)unroll | ((uint64_t)(uint32_t)max_blocks << 8) | ((uint64_t)(uint32_t)(flags + 1) << 40);
}
std::atomic<uint64_t> g_cfg_word{pack_cfg(1, 0, -1)};

netc_gpu::LaunchCfg cfg_now() {
    const uint64_t w = g_cfg_word.load(std::memory_order_acquire);
    netc_gpu::LaunchCfg c;
    c.unroll = (int)(w & 0xFF);
    c.max_blocks = (int)((w >> 8) & 0xFFFFFFFFu);
    c.flags = (int)((w >> 40) & 0xFFFFFF) - 1;
    return c;
}

// Measurement / test knobs (netc_gpu_knob).  Seeded once per process from the environment
// (tools/ sweeps set NETC_ENC_SCAN_PER=...), then changed only through netc_gpu_knob; the
// launch paths read one atomic word, never getenv.
constexpr int kKnobs = 15;   // knobs 1 .. 14 (include/ws/mask.h NETC_GPU_KNOB_*)
std::atomic<int64_t> g_knob[kKnobs];
std::once_flag g_knob_once;
void knobs_init() {
    static const char* const env[kKnobs] = {nullptr, "NETC_ENC_DENSE_BYTES", "NETC_ENC_SCAN_PER", "NETC_SCAN_FAST_RANK",
                                            "NETC_SCAN_ANCHOR_SLOTS", "NETC_VAL_STEPS", "NETC_SCAN_FUSE", "NETC_MASK_TAPER",
                                            "NETC_ENC_SRC", "NETC_ENC_FIX", "NETC_INJECT_FAULT",
                                            "NETC_ENC_PROBE", "NETC_ENC_PF", "NETC_SCAN_BLOCK_CHUNKS",
                                            "NETC_SCAN_ONEPASS"};
    for (int k = 0; k < kKnobs; ++k) {
        const char* e = env[k] ? getenv(env[k]) : nullptr;
        g_knob[k].store(e && *e ? (int64_t)strtoll(e, nullptr, 10) : -1, std::memory_order_relaxed);
    }
}

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    netc_errno_reason = NETC_REASON_GPU;
    return code;
}

int fail_hip(int code, const char* what, hipError_t e) {
    return fail(code, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

// Selects `device` for the calling thread for the lifetime of the guard.  The hot
// path (the device is already current) costs one hipGetDevice (a thread-local read
// in the runtime) and nothing on exit.
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

// device count, queried once per process (HIP's device list is fixed at runtime init)
int cached_device_count() {
    static const int n = [] {
        int c = 0;
        return hipGetDeviceCount(&c) == hipSuccess && c > 0 ? c : 0;
    }();
    return n;
}

int check_device(int device) {
    const int n = cached_device_count();
    if (n <= 0) return fail(NETC_GPU_ENODEV, "no HIP device available");
    if (device < 0 || device >= n) return fail(NETC_GPU_ENODEV, "device %d out of range [0, %d)", device, n);
    return 0;
}

bool partial_overlap(const void* a, const void* b, size_t n) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    if (x == y) return false;
    return x < y + n && y < x + n;
}

bool ranges_overlap(const void* a, size_t na, const void* b, size_t nb) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    if (na == 0 || nb == 0) return false;
    return x < y + nb && y < x + na;
}

int mask_batch_on_current(void* d_dst, const void* d_src, size_t total, const uint64_t* d_off,
                          const uint32_t* d_keys, size_t nframes, hipStream_t stream) {
    if (total == 0) return 0;
    if (!d_dst || !d_src) return fail(NETC_GPU_EINVAL, "null payload buffer");
    if (!d_off) return fail(NETC_GPU_EINVAL, "null frame offsets");
    if (nframes && !d_keys) return fail(NETC_GPU_EINVAL, "null keys with %zu frames", nframes);
    if (partial_overlap(d_dst, d_src, total)) return fail(NETC_GPU_EINVAL, "dst and src partially overlap");
    hipError_t e = netc_gpu::launch_mask_frames((uint8_t*)d_dst, (const uint8_t*)d_src, total, d_off, d_keys,
                                                nframes, stream, cfg_now());
    if (e != hipSuccess) return fail_hip(NETC_GPU_ELAUNCH, "mask kernel launch", e);
    return 0;
}

// Per (device, stream) flag scratch of netc_gpu_unmask_validate, grown geometrically.
// A call flags frames with its own tag (1..255), so the flags need clearing only when
// the scratch is new and when the tags wrap.  Outgrown arrays are kept (work queued
// before the growth may still use them) until netc_gpu_stream_release frees them all.
struct FlagScratch {
    int device;
    hipStream_t stream;
    uint8_t* p;
    size_t cap;
    uint8_t tag;
    std::vector<void*> retired;
};
std::mutex g_flag_mu;
std::vector<FlagScratch> g_flags;

int validate_scratch(int device, hipStream_t stream, size_t nframes, uint8_t** verr, uint8_t* tag) {
    std::lock_guard<std::mutex> lk(g_flag_mu);
    auto it = std::find_if(g_flags.begin(), g_flags.end(),
                           [&](const FlagScratch& f) { return f.device == device && f.stream == stream; });
    if (it == g_flags.end()) {
        g_flags.push_back({device, stream, nullptr, 0, 0, {}});
        it = g_flags.end() - 1;
    }
    bool clear = false;
    if (it->cap < nframes) {
        size_t want = it->cap ? 2 * it->cap : 65536;
        while (want < nframes) want *= 2;
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) return fail_hip(NETC_GPU_ENOMEM, "validation scratch", e);
        if (it->p) it->retired.push_back(it->p);
        it->p = (uint8_t*)p;
        it->cap = want;
        it->tag = 0;
    }
    if (it->tag == 0xFF || it->tag == 0) {
        it->tag = 0;
        clear = true;
    }
    *tag = ++it->tag;
    *verr = it->p;
    if (clear) {
        hipError_t e = hipMemsetAsync(it->p, 0, it->cap, stream);
        if (e != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "validation scratch clear", e);
    }
    return 0;
}

int validate_scratch_release(int device, hipStream_t stream) {   // the stream is synchronised
    std::lock_guard<std::mutex> lk(g_flag_mu);
    auto it = std::find_if(g_flags.begin(), g_flags.end(),
                           [&](const FlagScratch& f) { return f.device == device && f.stream == stream; });
    if (it == g_flags.end()) return 0;
    if (it->p) (void)hipFree(it->p);
    for (void* q : it->retired) (void)hipFree(q);
    g_flags.erase(it);
    return 1;
}

}  // namespace

// error / config helpers shared with the other C-ABI files (ws_ingest.hip)
namespace netc_gpu {
int api_fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    netc_errno_reason = NETC_REASON_GPU;
    return code;
}
int api_fail_hip(int code, const char* what, hipError_t e) { return fail_hip(code, what, e); }
int api_check_device(int device) { return check_device(device); }
LaunchCfg api_cfg() { return cfg_now(); }
int64_t knob(int k) {
    std::call_once(g_knob_once, knobs_init);
    return k > 0 && k < kKnobs ? g_knob[k].load(std::memory_order_relaxed) : -1;
}
// NETC_GPU_KNOB_INJECT_FAULT: true for the submission the knob's countdown reaches (then disarmed)
bool inject_fault() {
    std::call_once(g_knob_once, knobs_init);
    std::atomic<int64_t>& k = g_knob[NETC_GPU_KNOB_INJECT_FAULT];
    int64_t v = k.load(std::memory_order_relaxed);
    while (v >= 0) {
        if (k.compare_exchange_weak(v, v == 0 ? -1 : v - 1, std::memory_order_relaxed)) return v == 0;
    }
    return false;
}
}  // namespace netc_gpu

extern "C" {

int netc_gpu_device_count(void) { return cached_device_count(); }

int netc_gpu_init(int device) {
    if (int r = check_device(device)) return r;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    hipError_t e = hipFree(nullptr);   // forces context creation
    if (e != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "context init", e);
    return 0;
}

const char* netc_gpu_strerror(void) { return g_err; }

int netc_gpu_tune(int unroll, int max_blocks, int flags) {
    if (!(unroll == 1 || unroll == 2 || unroll == 4 || unroll == 8))
        return fail(NETC_GPU_EINVAL, "unroll must be 1, 2, 4 or 8 (got %d)", unroll);
    if (max_blocks < 0 || max_blocks > (1 << 24)) return fail(NETC_GPU_EINVAL, "max_blocks out of range");
    if (flags != NETC_GPU_TUNE_AUTO &&
        (flags & ~(NETC_GPU_TUNE_NT_LOADS | NETC_GPU_TUNE_NT_STORES | NETC_GPU_TUNE_PERSISTENT |
                   NETC_GPU_TUNE_TWO_STEPS | NETC_GPU_TUNE_XCD_ORDER | NETC_GPU_TUNE_XCD_GROUPS)))
        return fail(NETC_GPU_EINVAL, "unknown tune flags");
    g_cfg_word.store(pack_cfg(unroll, max_blocks, flags), std::memory_order_release);
    return 0;
}

int netc_gpu_knob(int knob, int64_t value) {
    if (knob < NETC_GPU_KNOB_ENC_DENSE_BYTES || knob >= kKnobs)
        return fail(NETC_GPU_EINVAL, "unknown knob %d", knob);
    std::call_once(g_knob_once, knobs_init);
    g_knob[knob].store(value < 0 ? -1 : value, std::memory_order_relaxed);
    return 0;
}

int netc_gpu_mask_batch(int device, void* d_dst, const void* d_src, size_t total_bytes,
                        const uint64_t* d_frame_offsets, const uint32_t* d_keys, size_t nframes, void* stream) {
    if (int r = check_device(device)) return r;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    return mask_batch_on_current(d_dst, d_src, total_bytes, d_frame_offsets, d_keys, nframes,
                                 (hipStream_t)stream);
}

int netc_gpu_unmask_validate(int device, void* d_dst, const void* d_src, size_t total_bytes,
                             const uint64_t* d_frame_offsets, const uint32_t* d_keys, const uint8_t* d_header0,
                             size_t nframes, uint8_t* d_valid, void* stream) {
    if (int r = check_device(device)) return r;
    if (nframes == 0) return 0;
    if (!d_frame_offsets || !d_keys || !d_header0 || !d_valid) return fail(NETC_GPU_EINVAL, "null frame array");
    if (total_bytes && (!d_dst || !d_src)) return fail(NETC_GPU_EINVAL, "null payload buffer");
    if (partial_overlap(d_dst, d_src, total_bytes)) return fail(NETC_GPU_EINVAL, "dst and src partially overlap");
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    uint8_t* verr = nullptr;
    uint8_t tag = 0;
    if (int r = validate_scratch(device, (hipStream_t)stream, nframes, &verr, &tag)) return r;
    hipError_t e = netc_gpu::launch_mask_validate((uint8_t*)d_dst, (const uint8_t*)d_src, total_bytes,
                                                  d_frame_offsets, d_keys, d_header0, nframes, verr, tag, d_valid,
                                                  (hipStream_t)stream, cfg_now());
    if (e != hipSuccess) return fail_hip(NETC_GPU_ELAUNCH, "unmask + validate launch", e);
    return 0;
}

int netc_gpu_mask_batch_multi(int nshards, const int* devices, void* const* d_dst, const void* const* d_src,
                              const size_t* total_bytes, const uint64_t* const* d_frame_offsets,
                              const uint32_t* const* d_keys, const size_t* nframes, void* const* streams,
                              int synchronize) {
    if (nshards < 0) return fail(NETC_GPU_EINVAL, "negative shard count");
    if (nshards == 0) return 0;
    if (!devices || !d_dst || !d_src || !total_bytes || !d_frame_offsets || !d_keys || !nframes)
        return fail(NETC_GPU_EINVAL, "null shard array");
    // Launch every shard before waiting on any: the shards run concurrently.  A shard that
    // fails (bad arguments, an unknown device, a launch error) ends the call only after the
    // shards launched before it have completed, so on any return no work of this call is in
    // flight: shards 0 .. i-1 are then complete, shard i (named in netc_gpu_strerror) and the
    // ones after it untouched.
    auto drain = [&](int upto) {
        for (int j = 0; j < upto; ++j) {
            DeviceGuard g(devices[j]);
            if (g.err == hipSuccess) (void)hipStreamSynchronize(streams ? (hipStream_t)streams[j] : nullptr);
        }
    };
    for (int i = 0; i < nshards; ++i) {
        int r = check_device(devices[i]);
        if (!r) {
            DeviceGuard g(devices[i]);
            if (g.err != hipSuccess) {
                r = fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
            } else {
                hipStream_t s = streams ? (hipStream_t)streams[i] : nullptr;
                r = mask_batch_on_current(d_dst[i], d_src[i], total_bytes[i], d_frame_offsets[i], d_keys[i],
                                          nframes[i], s);
            }
        }
        if (r) {
            char why[sizeof(g_err)];
            snprintf(why, sizeof(why), "%s", g_err);
            drain(i);
            return fail(r, "shard %d (shards before it completed, none after it launched): %s", i, why);
        }
    }
    if (synchronize) {
        int rc = 0;
        for (int i = 0; i < nshards; ++i) {   // every shard is waited for, even after a failure
            DeviceGuard g(devices[i]);
            if (g.err != hipSuccess) {
                if (!rc) rc = fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
                continue;
            }
            hipError_t e = hipStreamSynchronize(streams ? (hipStream_t)streams[i] : nullptr);
            if (e != hipSuccess && !rc) rc = fail(NETC_GPU_ERUNTIME, "shard %d: hipStreamSynchronize: %s", i,
                                                  hipGetErrorString(e));
        }
        return rc;
    }
    return 0;
}

static int encode_frames(int device, void* d_wire, size_t wire_capacity, uint64_t* d_wire_offsets, const void* d_payload,
                         size_t total_bytes, const uint64_t* d_frame_offsets, const uint32_t* d_keys,
                         const uint8_t* d_header0, size_t nframes, int masked, int ext_class, void* stream) {
    if (int r = check_device(device)) return r;
    if (!d_wire_offsets) return fail(NETC_GPU_EINVAL, "null wire offsets");
    if (nframes && (!d_frame_offsets || !d_wire)) return fail(NETC_GPU_EINVAL, "null frame buffer");
    if (total_bytes && !d_payload) return fail(NETC_GPU_EINVAL, "null payload buffer");
    if (masked && nframes && !d_keys) return fail(NETC_GPU_EINVAL, "masked frames need keys");
    const uint64_t per = NETC_WS_MAX_HEADER(masked);
    if (nframes > (UINT64_MAX - total_bytes) / per)
        return fail(NETC_GPU_EINVAL, "wire size overflows (%zu frames)", nframes);
    const uint64_t bound = NETC_WS_WIRE_BOUND(total_bytes, nframes, masked);
    if (nframes && wire_capacity < bound)
        return fail(NETC_GPU_EINVAL, "wire capacity %zu < bound %llu (payload + %llu B per frame)", wire_capacity,
                    (unsigned long long)bound, (unsigned long long)per);
    const size_t wo_bytes = (nframes + 1) * sizeof(uint64_t);
    if (nframes && ranges_overlap(d_wire, bound, d_payload, total_bytes))
        return fail(NETC_GPU_EINVAL, "wire and payload overlap (the assembly is out of place)");
    if (nframes && (ranges_overlap(d_wire_offsets, wo_bytes, d_frame_offsets, wo_bytes) ||
                    ranges_overlap(d_wire_offsets, wo_bytes, d_wire, bound)))
        return fail(NETC_GPU_EINVAL, "wire offsets overlap the frame offsets or the wire");
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    hipError_t e = netc_gpu::launch_encode_frames((uint8_t*)d_wire, bound, (const uint8_t*)d_payload, total_bytes,
                                                  d_frame_offsets, d_keys, d_header0, nframes, masked != 0,
                                                  d_wire_offsets, (hipStream_t)stream, cfg_now(), ext_class);
    if (e != hipSuccess) return fail_hip(NETC_GPU_ELAUNCH, "frame assembly launch", e);
    return 0;
}

int netc_gpu_encode_frames(int device, void* d_wire, size_t wire_capacity, uint64_t* d_wire_offsets,
                           const void* d_payload, size_t total_bytes, const uint64_t* d_frame_offsets,
                           const uint32_t* d_keys, const uint8_t* d_header0, size_t nframes, int masked,
                           void* stream) {
    return encode_frames(device, d_wire, wire_capacity, d_wire_offsets, d_payload, total_bytes, d_frame_offsets,
                         d_keys, d_header0, nframes, masked, -1, stream);
}

int netc_gpu_encode_frames_class(int device, void* d_wire, size_t wire_capacity, uint64_t* d_wire_offsets,
                                 const void* d_payload, size_t total_bytes, const uint64_t* d_frame_offsets,
                                 const uint32_t* d_keys, const uint8_t* d_header0, size_t nframes, int masked,
                                 int length_class, void* stream) {
    if (length_class != NETC_WS_CLASS_7BIT && length_class != NETC_WS_CLASS_16BIT &&
        length_class != NETC_WS_CLASS_64BIT)
        return fail(NETC_GPU_EINVAL, "unknown length class %d (NETC_WS_CLASS_7BIT, _16BIT or _64BIT)", length_class);
    return encode_frames(device, d_wire, wire_capacity, d_wire_offsets, d_payload, total_bytes, d_frame_offsets,
                         d_keys, d_header0, nframes, masked, length_class, stream);
}

int netc_gpu_scan_frames(int device, const void* d_wire, size_t len, uint64_t start, int flags, uint64_t* d_hdr,
                         uint32_t* d_keys, uint8_t* d_b0, size_t max_frames, uint64_t* d_result, void* stream) {
    if (int r = check_device(device)) return r;
    if (flags & ~NETC_WS_SCAN_STRICT) return fail(NETC_GPU_EINVAL, "unknown scan flags 0x%x", flags);
    if (!d_hdr || !d_result || (max_frames && (!d_keys || !d_b0))) return fail(NETC_GPU_EINVAL, "null output");
    if (len && !d_wire) return fail(NETC_GPU_EINVAL, "null stream");
    if (start > len) return fail(NETC_GPU_EINVAL, "start %llu past the stream end %zu", (unsigned long long)start, len);
    if (len >= (1ull << 60)) return fail(NETC_GPU_EINVAL, "stream too long");
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    hipError_t e = netc_gpu::launch_scan_frames((const uint8_t*)d_wire, len, start, (flags & NETC_WS_SCAN_STRICT) != 0,
                                                d_hdr, d_keys, d_b0, max_frames, d_result, (hipStream_t)stream);
    if (e == hipErrorOutOfMemory) return fail_hip(NETC_GPU_ENOMEM, "frame scan scratch", e);
    if (e != hipSuccess) return fail_hip(NETC_GPU_ELAUNCH, "frame scan launch", e);
    return 0;
}

int netc_gpu_stream_release(int device, void* stream) {
    if (int r = check_device(device)) return r;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    // work queued on that stream may still use the scratch
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipStreamSynchronize", e);
    (void)netc_gpu::release_stream_scratch(device, (hipStream_t)stream);   // frame scan
    (void)netc_gpu::release_enc_scratch(device, (hipStream_t)stream);      // frame assembly
    (void)validate_scratch_release(device, (hipStream_t)stream);           // UTF-8 flags
    return 0;
}

int netc_gpu_scan_release(int device, void* stream) { return netc_gpu_stream_release(device, stream); }

int64_t netc_gpu_scan_diag(int device, void* stream) {
    if (int r = check_device(device)) return r;
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipStreamSynchronize", e);
    return netc_gpu::scan_diag(device, (hipStream_t)stream);
}

int netc_gpu_unmask_frames(int device, void* d_wire, size_t len, const uint64_t* d_hdr, const uint32_t* d_keys,
                           size_t max_frames, const uint64_t* d_result, void* stream) {
    if (int r = check_device(device)) return r;
    if (!d_hdr || !d_result || (max_frames && !d_keys)) return fail(NETC_GPU_EINVAL, "null scan output");
    if (len == 0) return 0;
    if (!d_wire) return fail(NETC_GPU_EINVAL, "null stream");
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    hipError_t e = netc_gpu::launch_unmask_scanned((uint8_t*)d_wire, len, d_hdr, d_keys, max_frames, d_result,
                                                   (hipStream_t)stream, cfg_now());
    if (e != hipSuccess) return fail_hip(NETC_GPU_ELAUNCH, "unmask launch", e);
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Host → device → host pipeline (BASELINE config 5).  Slots are fixed byte
// ranges of the payload; a frame cut by a slot edge continues in the next slot
// with its key pre-rotated by the bytes already consumed (the phase carry of
// the reference's received_length, src/ws/common.c:301,321).  A persistent
// handle (netc_gpu_stream_*) owns the device slots, the pinned descriptor
// staging, the streams and the events, so a run allocates nothing unless a slot
// holds more frames than any earlier run's did.
// ---------------------------------------------------------------------------

namespace {

struct Slot {
    uint8_t* d_buf = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t* d_key = nullptr;
    uint64_t* h_off = nullptr;   // pinned descriptor staging
    uint32_t* h_key = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t desc_free = nullptr;   // descriptor staging may be rewritten
};

size_t upper_frame(const uint64_t* off, size_t n, uint64_t pos) {
    // number of frame starts <= pos among off[0..n-1]
    return (size_t)(std::upper_bound(off, off + n, pos) - off);
}

void free_desc(Slot& s) {
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_key) (void)hipFree(s.d_key);
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_key) (void)hipHostFree(s.h_key);
    s.d_off = nullptr;
    s.d_key = nullptr;
    s.h_off = nullptr;
    s.h_key = nullptr;
}

}  // namespace

struct netc_gpu_stream {
    int device = 0;
    size_t slot_bytes = 0;
    size_t cap = 0;   // descriptor entries each slot holds
    std::vector<Slot> slots;
};

namespace {

void stream_release(netc_gpu_stream* h) {
    for (Slot& s : h->slots) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (s.d_buf) (void)hipFree(s.d_buf);
        free_desc(s);
        if (s.desc_free) (void)hipEventDestroy(s.desc_free);
        if (s.stream) (void)hipStreamDestroy(s.stream);
    }
    delete h;
}

// every slot's descriptor staging holds >= want entries (grown only when a run needs more)
int ensure_desc(netc_gpu_stream* h, size_t want) {
    if (want <= h->cap) return 0;
    size_t cap = h->cap ? h->cap : 4096;
    while (cap < want) cap *= 2;
    hipError_t e;
    for (Slot& s : h->slots) {
        if ((e = hipStreamSynchronize(s.stream)) != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "stream sync", e);
        free_desc(s);
        if ((e = hipMalloc(&s.d_off, (cap + 1) * sizeof(uint64_t))) != hipSuccess ||
            (e = hipMalloc(&s.d_key, cap * sizeof(uint32_t))) != hipSuccess ||
            (e = hipHostMalloc(&s.h_off, (cap + 1) * sizeof(uint64_t), hipHostMallocDefault)) != hipSuccess ||
            (e = hipHostMalloc(&s.h_key, cap * sizeof(uint32_t), hipHostMallocDefault)) != hipSuccess) {
            free_desc(s);
            h->cap = 0;
            return fail_hip(NETC_GPU_ENOMEM, "slot descriptor allocation", e);
        }
    }
    h->cap = cap;
    return 0;
}

}  // namespace

extern "C" {

int netc_gpu_stream_create(struct netc_gpu_stream** out, int device, size_t slot_bytes, int nslots) {
    if (!out) return fail(NETC_GPU_EINVAL, "null output pointer");
    *out = nullptr;
    if (int r = check_device(device)) return r;
    if (!slot_bytes) slot_bytes = (size_t)512 << 20;
    if (!nslots) nslots = 2;
    if (slot_bytes < 4096 || nslots < 2 || nslots > 16)
        return fail(NETC_GPU_EINVAL, "need slot_bytes >= 4096 and 2 <= nslots <= 16");
    DeviceGuard g(device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    netc_gpu_stream* h = new (std::nothrow) netc_gpu_stream();
    if (!h) return fail(NETC_GPU_ENOMEM, "host allocation");
    h->device = device;
    h->slot_bytes = slot_bytes & ~(size_t)15;
    h->slots.resize((size_t)nslots);
    hipError_t e;
    for (Slot& s : h->slots) {
        if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&s.desc_free, hipEventDisableTiming)) != hipSuccess) {
            stream_release(h);
            return fail_hip(NETC_GPU_ERUNTIME, "stream/event create", e);
        }
        if ((e = hipMalloc(&s.d_buf, h->slot_bytes)) != hipSuccess) {
            stream_release(h);
            return fail_hip(NETC_GPU_ENOMEM, "slot allocation", e);
        }
    }
    *out = h;
    return 0;
}

void netc_gpu_stream_destroy(struct netc_gpu_stream* h) {
    if (!h) return;
    DeviceGuard g(h->device);
    stream_release(h);
}

int netc_gpu_stream_mask(struct netc_gpu_stream* h, void* h_dst, const void* h_src, size_t total,
                         const uint64_t* h_off, const uint32_t* h_keys, size_t nframes) {
    if (!h) return fail(NETC_GPU_EINVAL, "null stream handle");
    if (total == 0) return 0;
    if (!h_dst || !h_src || !h_off || (nframes && !h_keys)) return fail(NETC_GPU_EINVAL, "null host buffer");
    if (partial_overlap(h_dst, h_src, total)) return fail(NETC_GPU_EINVAL, "dst and src partially overlap");
    if (h_off[nframes] > total) return fail(NETC_GPU_EINVAL, "offsets[nframes] > total_bytes");
    DeviceGuard g(h->device);
    if (g.err != hipSuccess) return fail_hip(NETC_GPU_ERUNTIME, "hipSetDevice", g.err);
    const size_t slot_bytes = h->slot_bytes, nslots = h->slots.size();
    const size_t nchunks = (total + slot_bytes - 1) / slot_bytes;
    // descriptor capacity: frames overlapping any one slot
    size_t need = 1;
    for (size_t c = 0; c < nchunks; ++c) {
        const uint64_t lo = c * slot_bytes, hi = std::min<uint64_t>(total, lo + slot_bytes);
        const size_t k0 = upper_frame(h_off, nframes, lo), k1 = upper_frame(h_off, nframes, hi - 1);
        const size_t first = k0 ? k0 - 1 : 0;
        need = std::max(need, k1 - first + 1);
    }
    if (int r = ensure_desc(h, need)) return r;
    int rc = 0;
    hipError_t e = hipSuccess;
    for (size_t c = 0; rc == 0 && c < nchunks; ++c) {
        Slot& s = h->slots[c % nslots];
        const uint64_t lo = c * slot_bytes, hi = std::min<uint64_t>(total, lo + slot_bytes);
        const size_t len = (size_t)(hi - lo);
        // the previous chunk of this slot must have consumed its descriptors
        if ((e = hipEventSynchronize(s.desc_free)) != hipSuccess) {
            rc = fail_hip(NETC_GPU_ERUNTIME, "hipEventSynchronize", e);
            break;
        }
        // clip frames to [lo, hi), rebase to the slot, rotate a cut frame's key
        size_t m = 0;
        const size_t k0 = upper_frame(h_off, nframes, lo);
        size_t k = k0 ? k0 - 1 : 0;
        s.h_off[0] = 0;
        for (; k < nframes && h_off[k] < hi; ++k) {
            const uint64_t fs = h_off[k], fe = h_off[k + 1];
            if (fe <= lo) continue;
            const uint64_t cs = std::max<uint64_t>(fs, lo);
            const uint32_t key = h_keys[k];
            const uint32_t r = (uint32_t)((cs - fs) & 3u) * 8u;
            s.h_off[m] = cs - lo;
            s.h_key[m] = r ? (key >> r) | (key << (32u - r)) : key;
            ++m;
            s.h_off[m] = std::min<uint64_t>(fe, hi) - lo;
        }
        const uint8_t* src = (const uint8_t*)h_src + lo;
        uint8_t* dst = (uint8_t*)h_dst + lo;
        if ((e = hipMemcpyAsync(s.d_buf, src, len, hipMemcpyHostToDevice, s.stream)) != hipSuccess ||
            (e = hipMemcpyAsync(s.d_off, s.h_off, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream)) !=
                hipSuccess ||
            (m && (e = hipMemcpyAsync(s.d_key, s.h_key, m * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream)) !=
                      hipSuccess) ||
            (e = hipEventRecord(s.desc_free, s.stream)) != hipSuccess) {
            rc = fail_hip(NETC_GPU_ERUNTIME, "H2D copy", e);
            break;
        }
        if ((rc = mask_batch_on_current(s.d_buf, s.d_buf, len, s.d_off, s.d_key, m, s.stream)) != 0) break;
        if ((e = hipMemcpyAsync(dst, s.d_buf, len, hipMemcpyDeviceToHost, s.stream)) != hipSuccess) {
            rc = fail_hip(NETC_GPU_ERUNTIME, "D2H copy", e);
            break;
        }
    }
    for (Slot& s : h->slots) {
        const hipError_t w = hipStreamSynchronize(s.stream);
        if (rc == 0 && w != hipSuccess) rc = fail_hip(NETC_GPU_ERUNTIME, "hipStreamSynchronize", w);
    }
    return rc;
}

int netc_gpu_mask_stream_host(int device, void* h_dst, const void* h_src, size_t total, const uint64_t* h_off,
                              const uint32_t* h_keys, size_t nframes, size_t slot_bytes, int nslots) {
    if (int r = check_device(device)) return r;
    if (total == 0) return 0;
    if (!h_dst || !h_src || !h_off || (nframes && !h_keys)) return fail(NETC_GPU_EINVAL, "null host buffer");
    if (slot_bytes < 4096 || nslots < 2 || nslots > 16)
        return fail(NETC_GPU_EINVAL, "need slot_bytes >= 4096 and 2 <= nslots <= 16");
    netc_gpu_stream* h = nullptr;
    if (int r = netc_gpu_stream_create(&h, device, slot_bytes, nslots)) return r;
    const int rc = netc_gpu_stream_mask(h, h_dst, h_src, total, h_off, h_keys, nframes);
    netc_gpu_stream_destroy(h);
    return rc;
}

void* netc_gpu_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0) bytes = 1;
    const hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        fail_hip(NETC_GPU_ENOMEM, "hipHostMalloc", e);
        return nullptr;
    }
    return p;
}

void netc_gpu_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

}  // extern "C"
