// MI355X (gfx950 / CDNA4) send-side frame assembly — device kernels.
//
// Replaces the reference's per-frame send path
//   src/ws/common.c:55-82   header byte (FIN | opcode), MASK | 7-bit length code,
//                           16-bit / 64-bit big-endian extended length
//   src/ws/common.c:104-107 payload[i] ^= payload_masking_key[i % 4]
//   src/ws/common.c:112-119 header + key + payload copied into one frame buffer
// for a batch of frames resident in HBM: ONE out-of-place pass writes the wire
// bytes (header, key, masked payload) of every frame back to back.  The masking
// key always follows the MASK bit, also for an empty payload (RFC 6455 §5.2; the
// reference omits it there, defect B9 in DESIGN.md).
//
// Two launches on the caller's stream:
//   1. wire offsets: wo[j] = sum over k < j of (header_len(k) + len(k)), a
//      single-pass chained scan over the frames (decoupled look-back, 64
//      predecessors inspected at once);
//   2. the assembly kernel, output-driven: the wire buffer is walked in 16-byte
//      vectors aligned to the destination, chunk by chunk in grid-stride order as
//      in ws_mask_gpu.hip.  A 64-entry frame table in VGPRs (wire start, payload
//      offset, key, header byte of 64 consecutive frames) places each vector:
//      one unaligned 16-B load, one XOR with the key of the frame holding the
//      vector's first byte, rotated to its phase, one aligned store -- of the
//      vectors that hold no header byte only.  Spans the table does not cover
//      (more than ~60 frames in 1 KiB) and the buffer edges are listed per
//      wavefront and composed byte-exactly by it after its chunks; the launch's
//      trailing blocks compose, one thread per frame, the vectors holding each
//      frame's header bytes (fix_vectors).
//   A batch averaging under 80 B of payload per frame takes a compose launch
//   instead of step 2 (encode_queued_kernel: every span composed per lane).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "gpu_util.h"
#include "ws_mask_gpu.h"

namespace netc_gpu {

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));   // unaligned 16-B access

// extended-length bytes for a payload of len bytes (src/ws/common.c:63,71-82)
__device__ __forceinline__ uint32_t ext_len(uint64_t len) { return len < 126 ? 0u : (len < 65536 ? 2u : 8u); }

// ------------------------------------------------------------ wire offsets --

static constexpr int kScanThreads = 256;

// exclusive prefix sum over the block (kScanThreads threads); returns the block total in *total
__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* total) {
    __shared__ uint64_t wsum[kScanThreads / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint64_t inc = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint64_t o = (uint64_t)__shfl_up((unsigned long long)inc, d, kWave);
        if (lane >= d) inc += o;
    }
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int i = 0; i < kScanThreads / kWave; ++i) {
        before += i < w ? wsum[i] : 0;
        all += wsum[i];
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}

// ---------------------------------------------------------------- assembly --

struct EncArgs {
    uint8_t* wire_base;        // wire rounded down to 16
    const uint8_t* src;        // payload buffer: frame j's payload is src[off[j], off[j+1])
    uint64_t src_total;        // bytes readable at src
    const uint64_t* off;       // n + 1 payload offsets
    const uint64_t* wo;        // n + 1 wire offsets (step 1)
    const uint32_t* keys;      // n packed keys (masked), else unused
    const uint8_t* b0;         // n header bytes (FIN | RSV | opcode), or null: 0x82
    uint64_t n;
    uint64_t wmis;             // wire & 15
    uint32_t masked;
    uint64_t* defer;           // queued span starts (W coordinates), capacity defer_cap
    uint32_t* defer_count;
    uint64_t defer_cap;
    uint32_t all_spans;        // dense batch: the compose launch takes every span (no assembly launch)
    uint32_t main_blocks;      // encode_frames_kernel: blocks 0 .. main_blocks-1 assemble, the rest fix headers
    uint32_t per_wave;         // ... each assembly wavefront lists its unmapped spans at defer[wave * per_wave ..]
    uint32_t fix_blocks;       // 1: the header vectors by trailing blocks of the assembly (0: by the scan, or none needed)
    uint32_t fix_tail;         // 1: ... by the assembly wavefronts themselves, after their windows (ENC_FIX = 2)
    // source-driven assembly (encode_src_kernel)
    const uint8_t* src_base;   // src rounded down to 16 (P coordinates: byte q of src is at P = q + smis)
    uint64_t smis;             // src & 15
    uint64_t nwin;             // windows of the source walk
    double density;            // frames per payload byte (table-base guesses)
    int32_t probe_e;           // entries of a window's first table probe (<= 64)
    int32_t probe_bias;        // wire-driven assembly: frames the probe's base sits before the density guess
    const uint32_t* keys_ld;   // keys, or any readable array when unmasked (loads are never branched around)
    const uint8_t* b0_ld;      // b0, or any readable array when null
    // one length class (netc_gpu_encode_frames_class): the wire offsets are affine in the payload
    // offsets, wo[k] = off[k] - off[0] + hstride * k, so the assembly computes them instead of
    // reading wo[] and no scan launch runs before it; its trailing fixup blocks write wo[] and
    // check every frame's class
    uint32_t affine;
    uint32_t ext;              // ... the class's extended-length bytes (0, 2 or 8)
    uint64_t hstride;          // ... header + key bytes of every frame
    uint64_t off0;             // ... off[0] (loaded by the kernel)
    uint64_t* wo_out;          // ... wo[] as the fixup blocks write it
    uint32_t* fix_done;        // ... fixup blocks retired + 0x10000 per block that met a frame outside
                               //     the class; zero between calls (the last block resets it)
};

// wire offset of frame k (k <= n): from wo[], or affine in off[k] (one length class)
__device__ __forceinline__ uint64_t wire_at(const EncArgs& a, uint64_t k) {
    if (a.affine) return gptr(a.off)[k] - a.off0 + a.hstride * k;
    return gptr(a.wo)[k];
}

// spans per wave trip of the dense compose launch
static constexpr int kDenseGroup = 4;

// Frame table: lane l holds virtual frame kb + l.  W coordinates = wire byte + wmis.
struct EncTable {
    int64_t kb;
    uint64_t start;   // W start of the frame's header (virtual head: 0, past the end: inf)
    uint64_t poff;    // payload offset off[v] (clamped)
    uint32_t key;
    uint32_t b0;
    uint64_t last;    // start of entry e - 1 (uniform)
    bool tail;        // entry for frame n is in the table
    int e;            // entries held: 64, or fewer for a chunk's first probe (uniform); lanes >= e: start inf
};

__device__ __forceinline__ void enc_entry(const EncArgs& a, int64_t v, EncTable& t, bool held = true) {
    if (!held) {   // past the probe's entries: nothing loaded (the loads below are skipped for the lane)
        t.start = kInf;
        t.poff = 0;
        t.key = 0;
        t.b0 = 0x82u;
        return;
    }
    const int64_t n = (int64_t)a.n;
    const int64_t vo = v < 0 ? 0 : (v > n ? n : v);
    const int64_t vk = v < 0 ? 0 : (v >= n ? (n > 0 ? n - 1 : 0) : v);
    t.poff = gptr(a.off)[vo];
    const uint64_t wo = a.affine ? t.poff - a.off0 + a.hstride * (uint64_t)vo : gptr(a.wo)[vo];
    const uint32_t key = a.masked ? gptr(a.keys)[vk] : 0u;
    const uint32_t b0 = a.b0 ? (uint32_t)gptr(a.b0)[vk] : 0x82u;
    t.start = v < 0 ? 0 : (v <= n ? wo + a.wmis : kInf);
    t.key = (v >= 0 && v < n) ? key : 0u;
    t.b0 = b0;
}

__device__ __forceinline__ void enc_table_issue(const EncArgs& a, EncTable& t, int64_t kb, int lane, int e = kWave) {
    t.kb = kb;
    t.e = e;
    enc_entry(a, kb + lane, t, lane < e);
    t.tail = kb + (e - 1) >= (int64_t)a.n;
}

__device__ __forceinline__ void enc_table_finish(EncTable& t) { t.last = readlane64(t.start, t.e - 1); }

__device__ __forceinline__ void enc_table_load(const EncArgs& a, EncTable& t, int64_t kb, int lane) {
    enc_table_issue(a, t, kb, lane);
    enc_table_finish(t);
}

// Largest virtual frame L whose header starts at or before W (wave-uniform):
// 64-ary narrowing over wo[], one coalesced probe + one ballot per step,
// starting from an interpolation guess bracket.
__device__ int64_t enc_locate(const EncArgs& a, uint64_t W, uint64_t wire_total, int lane) {
    if (W < a.wmis) return -1;
    const uint64_t q = W - a.wmis;
    int64_t L = -1, H = (int64_t)a.n + 1;
    if (a.n > (uint64_t)kWave && wire_total > 0) {
        constexpr int64_t kStride = 16;
        int64_t g = (int64_t)((double)q * ((double)a.n / (double)wire_total));
        g = g > (int64_t)a.n ? (int64_t)a.n : g;
        const int64_t base = g - 31 * kStride;
        const int64_t idx = base + (int64_t)lane * kStride;
        const bool valid = idx >= 0 && idx <= (int64_t)a.n;
        const uint64_t val = valid ? wire_at(a, (uint64_t)idx) : 0;
        const uint64_t le = __ballot(valid && val <= q);
        const uint64_t gt = __ballot(valid && val > q);
        if (le) L = base + (int64_t)(63 - __builtin_clzll(le)) * kStride;
        if (gt) H = base + (int64_t)__builtin_ctzll(gt) * kStride;
    }
    while (H - L > kWave) {
        const int64_t lo = L + 1;
        const int64_t step = (H - lo + kWave - 1) / kWave;
        const int64_t idx = lo + (int64_t)lane * step;
        const bool valid = idx < H;
        const uint64_t val = valid ? wire_at(a, (uint64_t)idx) : kInf;
        const uint64_t le = __ballot(valid && val <= q);
        const uint64_t gt = __ballot(valid && val > q);
        if (le) L = lo + (int64_t)(63 - __builtin_clzll(le)) * step;
        if (gt) H = lo + (int64_t)__builtin_ctzll(gt) * step;
    }
    return L;
}

// make t hold the frame containing W (wave-uniform): keep it if it does, else search
__device__ __forceinline__ void enc_resolve(const EncArgs& a, EncTable& t, uint64_t W, uint64_t wire_total,
                                            int lane) {
    const uint64_t m = __ballot(t.start <= W);
    if (!(m != 0 && (t.tail || __popcll(m) < t.e))) enc_table_load(a, t, enc_locate(a, W, wire_total, lane), lane);
}

// The frame header as 16 little-endian bytes (h <= 14 used), wave-uniform:
// b0 | MASK, length code | extended length, big-endian | key bytes.
__device__ __forceinline__ void build_header(uint32_t b0, uint64_t len, bool masked, uint32_t key, uint64_t& lo,
                                             uint64_t& hi) {
    // branch-free selects (a branchy form makes the compiler index {lo, hi} through scratch)
    const bool e2 = len >= 126 && len < 65536, e8 = len >= 65536;
    const uint64_t code = len < 126 ? len : (e2 ? 126 : 127);
    const uint64_t k = masked ? (uint64_t)key : 0;
    const uint64_t be = __builtin_bswap64(len);   // byte i = (len >> 8 (7 - i)) & 0xFF
    // bytes 0..1: b0, MASK | length code; then the extended length (big-endian), then the key
    lo = (uint64_t)(b0 & 0xFF) | ((code | (masked ? 0x80u : 0u)) << 8);
    const uint64_t lo2 = ((len >> 8) & 0xFF) << 16 | (len & 0xFF) << 24 | k << 32;   // 16-bit form, key at 4
    const uint64_t lo8 = be << 16;                                                  // 64-bit form
    lo |= e8 ? lo8 : (e2 ? lo2 : k << 16);                                          // 7-bit form: key at 2
    hi = e8 ? ((be >> 48) | k << 16) : 0;                                           // 64-bit form: key at 10
}

// 16-byte value (lo, hi) moved by sh bytes (sh > 0: toward higher byte positions)
__device__ __forceinline__ u32x4 shift_bytes(uint64_t lo, uint64_t hi, int sh) {
    uint64_t rl, rh;
    if (sh >= 16 || sh <= -16) {
        rl = rh = 0;
    } else if (sh >= 8) {
        rl = 0;
        rh = lo << (8 * (sh - 8));
    } else if (sh > 0) {
        rl = lo << (8 * sh);
        rh = (hi << (8 * sh)) | (lo >> (64 - 8 * sh));
    } else if (sh == 0) {
        rl = lo;
        rh = hi;
    } else if (sh > -8) {
        const int s = -sh;
        rl = (lo >> (8 * s)) | (hi << (64 - 8 * s));
        rh = hi >> (8 * s);
    } else {
        rl = hi >> (8 * (-sh - 8));
        rh = 0;
    }
    u32x4 r = {(uint32_t)rl, (uint32_t)(rl >> 32), (uint32_t)rh, (uint32_t)(rh >> 32)};
    return r;
}

#ifdef NETC_ENC_CHECKS
// diagnostic build only (tools/): range checks that record the first violation
// (site, value, limit, count) instead of making the access
__device__ unsigned long long g_enc_fault[4];
extern "C" int netc_gpu_debug_encode_faults(unsigned long long* out4) {
    return (int)hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_enc_fault), 4 * sizeof(unsigned long long));
}
__device__ __forceinline__ bool enc_ok(int site, uint64_t v, uint64_t limit) {
    if (v <= limit) return true;
    if (atomicAdd(&g_enc_fault[3], 1ull) == 0) {
        g_enc_fault[0] = (unsigned long long)site;
        g_enc_fault[1] = v;
        g_enc_fault[2] = limit;
    }
    return false;
}
#define ENC_OK(site, v, limit) enc_ok(site, (uint64_t)(v), (uint64_t)(limit))
#else
#define ENC_OK(site, v, limit) true
#endif

template <bool NT>
__device__ __forceinline__ u32x4 load_u(const uint8_t* p) {
    const NETC_GLOBAL u32x4u* q = (const NETC_GLOBAL u32x4u*)p;
    if constexpr (NT) return __builtin_nontemporal_load(q);
    return *q;
}

// bytes [lo, hi) of the lane's vector from src + s0 (s0 may be outside [0, src_total):
// only in-range bytes are read, the rest is left 0)
__device__ __forceinline__ u32x4 load_guarded(const EncArgs& a, int64_t s0, int lo, int hi) {
    u32x4 v = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b) {   // unrolled: constant vector indices (no scratch)
        const int64_t s = s0 + b;
        if (b >= lo && b < hi && s >= 0 && (uint64_t)s < a.src_total)
            v[b >> 2] |= (uint32_t)gptr(a.src)[s] << (8 * (b & 3));
    }
    return v;
}

template <bool NT>
__device__ __forceinline__ void store_wire(const EncArgs& a, uint64_t W, u32x4 v, uint64_t wlo, uint64_t whi) {
    if (W >= wlo && W + 16 <= whi) {
        NETC_GLOBAL u32x4* p = gptr(reinterpret_cast<u32x4*>(a.wire_base + W));
        if constexpr (NT) __builtin_nontemporal_store(v, p);
        else *p = v;
    } else {
#pragma unroll
        for (int b = 0; b < 16; ++b)
            if (W + b >= wlo && W + b < whi) gptr(a.wire_base)[W + b] = (uint8_t)(v[b >> 2] >> (8 * (b & 3)));
    }
}

// Wave-uniform description of the frame in table entry l (needs entry l + 1).
struct FrameInfo {
    uint64_t Ws, We, pw, o, len;   // wire start / end, payload start (W coords); payload offset, length
    uint32_t key, b0;
};

__device__ __forceinline__ FrameInfo frame_info(const EncArgs& a, const EncTable& t, int l) {
    FrameInfo f;
    f.Ws = readlane64(t.start, l);
    f.We = readlane64(t.start, l + 1);
    f.o = readlane64(t.poff, l);
    f.len = readlane64(t.poff, l + 1) - f.o;
    f.key = readlane32(t.key, l);
    f.b0 = readlane32(t.b0, l);
    f.pw = f.Ws + 2 + ext_len(f.len) + (a.masked ? 4 : 0);
    return f;
}

// OR the header bytes of frame f that fall into the lane's vector into v
__device__ __forceinline__ u32x4 put_header(const EncArgs& a, const FrameInfo& f, uint64_t W, u32x4 v) {
    const int64_t hs = (int64_t)(f.Ws - W), he = (int64_t)(f.pw - W);
    if (he > 0 && hs < 16) {
        uint64_t hl, hh;
        build_header(f.b0, f.len, a.masked != 0, f.key, hl, hh);
        v |= shift_bytes(hl, hh, (int)hs) & select_range(hs, he);
    }
    return v;
}

// Frame in table entry c (needs entry c + 1), per lane: each lane reads the entry its
// own walk is at (ds_bpermute; every lane of the wave executes it)
__device__ __forceinline__ FrameInfo frame_info_lane(const EncArgs& a, const EncTable& t, int c) {
    FrameInfo f;
    f.Ws = bperm64(t.start, c);
    f.We = bperm64(t.start, c + 1);
    f.o = bperm64(t.poff, c);
    f.len = bperm64(t.poff, c + 1) - f.o;
    f.key = (uint32_t)__builtin_amdgcn_ds_bpermute(c << 2, (int)t.key);
    f.b0 = (uint32_t)__builtin_amdgcn_ds_bpermute(c << 2, (int)t.b0);
    f.pw = f.Ws + 2 + ext_len(f.len) + (a.masked ? 4 : 0);
    return f;
}

// Wire vector of this lane for the span at A0, composed byte-exactly from every frame
// touching it (header bytes, payload bytes, any number of frame edges).  Per lane: a
// binary search of the table (entries 0 .. 62, each needs the next one) finds the
// frame holding the lane's first byte, then the lane walks the frames starting inside
// its 16 bytes -- at most three (a masked frame is 6 wire bytes or more), so the walk
// is a few trips whatever the frame count of the span.  A span with more frames than
// the table holds is walked in 62-entry windows, the next window's load in flight
// while this one is composed; entry 62 is shared by two windows and its bytes are
// ORed twice with the same values.  On entry entry 0 of t starts at or before A0.
__device__ u32x4 compose_vec(const EncArgs& a, EncTable& t, uint64_t A0, uint64_t W, int lane) {
    const uint64_t Aend = A0 + kSpan;
    u32x4 out = {0, 0, 0, 0};
    for (;;) {
        const int kLast = t.e - 2;   // last usable entry (uniform)
        const bool more = !t.tail && t.last < Aend;   // wave-uniform
        EncTable tn;
        if (more) enc_table_issue(a, tn, t.kb + kLast, lane);
        int l = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const int c = l + step;
            const uint64_t sc = bperm64(t.start, c <= kLast ? c : kLast);   // every lane takes part
            if (c <= kLast && sc <= W) l = c;
        }
        if (readlane64(t.start, 0) > W) l = 0;   // no entry at or before W: walk from entry 0
        for (int c = l;; ++c) {
            const int cc = c <= kLast ? c : kLast;
            const FrameInfo f = frame_info_lane(a, t, cc);
            const int64_t j = t.kb + cc;
            const bool active = c <= kLast && j < (int64_t)a.n && f.Ws < W + 16;
            if (active && j >= 0) {
                out = put_header(a, f, W, out);
                // payload bytes [pw, We) of this vector
                const int64_t plo = (int64_t)(f.pw - W), phi = (int64_t)(f.We - W);
                if (phi > 0 && plo < 16 && phi > plo) {
                    const int64_t s0 = (int64_t)f.o - plo;   // src offset of the vector's byte 0
                    u32x4 v;
                    if (s0 >= 0 && (uint64_t)s0 + 16 <= a.src_total) v = load_u<false>(a.src + s0);
                    else v = load_guarded(a, s0, plo < 0 ? 0 : (int)plo, phi > 16 ? 16 : (int)phi);
                    const uint32_t rk = rotr8(f.key, (uint64_t)(-plo));   // phase of byte 0: W - pw
                    const u32x4 kv = {rk, rk, rk, rk};
                    out |= (v ^ kv) & select_range(plo, phi);
                }
            }
            if (!__ballot(active)) break;
        }
        if (!more) break;
        t = tn;
        enc_table_finish(t);
    }
    return out;
}

// ------------------------------------------------------------ fast spans --
// A frame's payload follows the previous frame's payload in the source (frames are
// [off[k], off[k+1])), so the wire is the source with the headers inserted.  For a
// lane's wire vector at W, take the frame l holding W (header start S <= W < next
// header start Sn): one unaligned 16-B load at s = W + (off[l] - pw_l) (pw = wire
// payload start) XOR frame l's key rotated to W gives every byte of the vector that
// is payload of frame l.  A vector holding any header byte (frame l's when W is inside
// its header, or the next frame's) is not stored here: fix_vectors (one thread per frame,
// the launch's trailing blocks) composes each of those whole.  So the vector path has no per-lane header work: the
// previous form inserted the header and shifted the tail in the lane a header
// touched, with a wave-wide branch costing about 200 vector instructions per span at
// 1 KiB frames.  A span takes this path when the 64-entry table covers it and every
// load stays inside the payload buffer; any other span is queued for the compose
// kernel.

// per-lane frame data from the table (ds_bpermute: every lane of the wave executes it)
struct LaneFrames {
    uint64_t S, Sn;   // wire header starts of frames l, l + 1 (W coordinates)
    uint64_t P, Pn;   // payload offsets of frames l, l + 1
    uint32_t K;       // key of frame l
};

__device__ __forceinline__ uint32_t bperm32(uint32_t x, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)x);
}

__device__ __forceinline__ LaneFrames lane_frames(const EncTable& t, int l) {
    LaneFrames f;
    f.S = bperm64(t.start, l);
    f.Sn = bperm64(t.start, l + 1);
    f.P = bperm64(t.poff, l);
    f.Pn = bperm64(t.poff, l + 1);
    f.K = bperm32(t.key, l);
    return f;
}

// The same for a span holding at most one frame start (nb <= 1): entries l0 .. l0 + 2
// read once for the wave (readlane), each lane picks frame l0 or l0 + 1.
__device__ __forceinline__ LaneFrames frames_near(const EncTable& t, int l0, int nb, uint64_t W, int l) {
    if (nb > 1) return lane_frames(t, l);
    const uint64_t S0 = readlane64(t.start, l0), S1 = readlane64(t.start, l0 + 1), S2 = readlane64(t.start, l0 + 2);
    const uint64_t P0 = readlane64(t.poff, l0), P1 = readlane64(t.poff, l0 + 1), P2 = readlane64(t.poff, l0 + 2);
    const uint32_t K0 = readlane32(t.key, l0), K1 = readlane32(t.key, l0 + 1);
    const bool in1 = nb == 1 && W >= S1;
    LaneFrames f;
    f.S = in1 ? S1 : S0;
    f.Sn = in1 ? S2 : S1;
    f.P = in1 ? P1 : P0;
    f.Pn = in1 ? P2 : P1;
    f.K = in1 ? K1 : K0;
    return f;
}

__device__ __forceinline__ uint64_t header_len(uint64_t len, bool masked) {
    return 2 + ext_len(len) + (masked ? 4 : 0);
}

enum : int { kSpanFast = 0, kSpanQueued = 2, kSpanNone = 3 };

// What the store phase needs for one span: the load and the rotated key.
struct SpanPlan {
    int kind, l0, nb;   // kind; the span's first table entry and frame starts inside it (uniform)
    u32x4 d;
    uint32_t rk;
};
template <int U>
struct Plan {
    SpanPlan s[U];
    uint32_t own;       // bit u: span u's vector of this lane holds no header byte, so this kernel
                        // stores it (the others: fix_vectors)
};

// f(integral_constant<int, I>) for I = 0 .. N-1, unrolled at compile time: span
// state stays in registers (a runtime-indexed span array lands in scratch, and
// every load then waits on vmcnt(0) to be stored there)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

template <int U, bool NT>
__device__ __forceinline__ void plan_chunk(const EncArgs& a, const EncTable& t, uint64_t A, uint64_t wlo,
                                           uint64_t whi, int lane, Plan<U>& P) {
    const bool masked = a.masked != 0;
    P.own = 0;
    static_for<0, U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        SpanPlan& sp = P.s[u];
        const uint64_t A0 = A + (uint64_t)u * kSpan, Aend = A0 + kSpan;
        const uint64_t W = A0 + 16ull * (uint64_t)lane;
        // classified first (wave-uniform); the load is then issued unconditionally at
        // the end (one exit path: loads under branches end up staged through scratch
        // with full vmcnt drains)
        int kind = kSpanNone, l0 = 0, nb = 0;
        int64_t ad = 0;
        uint32_t rk = 0;
        bool own = false;
        do {
            if (A0 >= whi) break;
            kind = kSpanQueued;
            l0 = __popcll(__ballot(t.start <= A0)) - 1;
            const uint64_t bm = __ballot(t.start > A0 && t.start < Aend);
            nb = __popcll(bm);
            const bool covered = (t.tail || t.last >= Aend) && l0 >= 0 && l0 + nb + 2 <= t.e - 1;
            if (!covered || A0 < wlo || Aend > whi || t.kb + l0 < 0 || t.kb + l0 + nb >= (int64_t)a.n) break;
            if (nb == 0) {
                // one frame covers the span: everything is wave-uniform
                const uint64_t S0 = readlane64(t.start, l0), P0 = readlane64(t.poff, l0);
                const uint64_t pw = S0 + header_len(readlane64(t.poff, l0 + 1) - P0, masked);
                const int64_t delta = (int64_t)(P0 - pw);   // source offset = W + delta
                if ((int64_t)A0 + delta < 0 || (int64_t)Aend + delta > (int64_t)a.src_total) break;
                kind = kSpanFast;
                ad = (int64_t)W + delta;
                rk = rotr8(readlane32(t.key, l0), A0 - pw);
                const uint64_t Sn = readlane64(t.start, l0 + 1);
                own = W >= pw && (W + 16 <= Sn || Sn >= whi);   // (the last frame: store_wire clips at whi)
                break;
            }
            // this lane's frame: the entries starting at or before W
            int l = l0;
            for (uint64_t b = bm; b; b &= b - 1) l += readlane64(t.start, __builtin_ctzll(b)) <= W ? 1 : 0;
            const LaneFrames f = frames_near(t, l0, nb, W, l);
            const uint64_t pw = f.S + header_len(f.Pn - f.P, masked);
            const int64_t s0 = (int64_t)(W + f.P - pw);   // source offset of the vector's byte 0
            if (__ballot(s0 < 0 || (uint64_t)s0 + 16 > a.src_total)) break;
            kind = kSpanFast;
            ad = s0;
            rk = rotr8(f.K, W - pw);
            own = W >= pw && (W + 16 <= f.Sn || f.Sn >= whi);
        } while (false);
        P.own |= own ? 1u << u : 0u;
        sp.l0 = l0;
        sp.nb = nb;
        sp.kind = kind;
        sp.rk = rk;
        sp.d = u32x4{0, 0, 0, 0};
        // a payload buffer under 16 bytes (possibly NULL when empty) is never read
        // here: every span is queued then, and the compose kernel reads byte-wise
        if (a.src_total >= 16) {   // kernel-uniform
            if (ENC_OK(1, ad, a.src_total - 16)) sp.d = load_u<NT>(a.src + ad);
        }
    });
}

template <int U, bool NT>
__device__ __forceinline__ void finish_chunk(const EncArgs& a, const EncTable& t, uint64_t A, uint64_t wlo,
                                             uint64_t whi, int lane, const Plan<U>& P, uint64_t* list, uint32_t& nl) {
    static_for<0, U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const SpanPlan& sp = P.s[u];
        const uint64_t A0 = A + (uint64_t)u * kSpan;
        const uint64_t W = A0 + 16ull * (uint64_t)lane;
        if (sp.kind == kSpanNone) return;
        if (sp.kind == kSpanQueued) {   // wave-uniform: listed, composed after the wavefront's windows
            // (bounded: the slice is sized from the host's wire bound; device offsets that break
            // the contract -- not monotonic, or not ending at total_bytes -- must not write past it)
            if (nl < a.per_wave) {
                if (lane == 0) list[nl] = A0;
                ++nl;
            }
            return;
        }
        const u32x4 kv = {sp.rk, sp.rk, sp.rk, sp.rk};
        const u32x4 v = sp.d ^ kv;
        if ((P.own >> u) & 1u) store_wire<NT>(a, W, v, wlo, whi);
    });
}

// The wire vector at V (W coordinates, 16-aligned), byte-exact, by one thread: every frame from
// j0 (the frame holding byte V, its header at S, its payload at o) to the last one starting
// inside it -- header bytes from build_header, payload bytes from one 16-B source load each --
// then one store.  The later frames' starts follow from off[] alone (wo[j + 1] = wo[j] +
// header_len + len), so this runs before wo[] is complete (in the wire-offsets scan); the wire
// ends where frame n would start.
__device__ __forceinline__ void compose_from(const EncArgs& a, uint64_t V, uint64_t j0, uint64_t S, uint64_t o, uint64_t wlo) {
    const bool masked = a.masked != 0;
    u32x4 out = {0, 0, 0, 0};
    uint64_t whi = kInf;
    for (uint64_t j = j0; S < V + 16; ++j) {
        if (j >= a.n) {
            whi = S;
            break;
        }
        const uint64_t on = gptr(a.off)[j + 1];
        const uint64_t len = on - o, pw = S + header_len(len, masked), Sn = pw + len;
        const uint32_t key = masked ? gptr(a.keys)[j] : 0u;
        const int64_t hs = (int64_t)(S - V), he = (int64_t)(pw - V), phi = (int64_t)(Sn - V);
        if (he > 0 && hs < 16) {
            uint64_t hl, hh;
            build_header(a.b0 ? (uint32_t)gptr(a.b0)[j] : 0x82u, len, masked, key, hl, hh);
            out |= shift_bytes(hl, hh, (int)hs) & select_range(hs, he);
        }
        if (phi > 0 && he < 16 && phi > he) {
            const int64_t s0 = (int64_t)o - he;   // source offset of the vector's byte 0
            u32x4 v;
            if (s0 >= 0 && (uint64_t)s0 + 16 <= a.src_total) v = load_u<false>(a.src + s0);
            else v = load_guarded(a, s0, he < 0 ? 0 : (int)he, phi > 16 ? 16 : (int)phi);
            const uint32_t rk = rotr8(key, (uint64_t)(-he));   // phase of byte 0: V - pw
            const u32x4 kv = {rk, rk, rk, rk};
            out |= (v ^ kv) & select_range(he, phi);
        }
        S = Sn;
        o = on;
    }
    store_wire<false>(a, V, out, wlo, whi);
}

// The vectors holding frame k's header bytes (one, or two when the header crosses a 16-B
// edge) that frame k owns -- the first is frame k - 1's when k - 1's header reaches into it --
// composed byte-exactly.  The assembly stores only vectors with no header byte (SpanPlan::own),
// so the two write disjoint vectors and need no ordering (round 4: the fixups were a launch of
// their own after the assembly, 7.9 us at config 2; as the assembly launch's trailing blocks the
// step went 39.2-40.0 -> 37.6-37.8 us at config 2 and 414-417 -> 418-421 us at config 4,
// profiles/r04xyz_encode_fused.json.  Tried on the way: a per-wavefront done counter so the
// trailing blocks could take the queued spans -- 5,120 same-address atomics at the end of the
// launch tripled it (79 us) -- and the trailing blocks resident beside the assembly (fewer
// assembly blocks: 39.8-40.2 / 462-463 us).)
// Frame k's header at S (W coordinates); its payload [o, on), frame k - 1's [op, o) (k > 0);
// the keys of both and frame k's header byte.  fix_plan places the (one or two) vectors holding
// frame k's header bytes that frame k owns -- the first is frame k - 1's when k - 1's header
// reaches into it -- and issues their payload loads; fix_store composes and stores them.  The
// split lets a thread issue the loads of several frames before its first store (the compiler
// may not move a load above a store that could alias it: four frames fixed one after the other
// were four round trips).  Every byte written lies in frames k - 1 and k (the simple case), or
// comes from compose_from, so no wire end is needed here.
struct FixGeo {   // frame k's fixup geometry (fix_geo)
    uint64_t pw, Sn, len, v0, v1;
    bool own0, simple;
};

__device__ __forceinline__ FixGeo fix_geo(const EncArgs& a, uint64_t k, uint64_t S, uint64_t op, uint64_t o, uint64_t on) {
    FixGeo g;
    g.len = on - o;
    g.pw = S + header_len(g.len, a.masked != 0);
    g.Sn = g.pw + g.len;
    const uint64_t hpe = S - (o - op);   // frame k - 1's payload start (k > 0)
    g.v0 = S & ~15ull;
    g.v1 = (g.pw - 1) & ~15ull;
    g.own0 = k == 0 || ((hpe - 1) & ~15ull) < g.v0;
    // the usual case: the vectors hold only frame k - 1's payload tail, frame k's header and frame
    // k's payload (frame k ends at or past the last one); the payload bytes by one load per frame
    g.simple = g.Sn >= g.v1 + 16 && (k == 0 || g.v0 >= S || g.v0 >= hpe);
    return g;
}

__device__ __forceinline__ u32x4 fix_load(const EncArgs& a, int64_t s0, int lo, int hi) {
    if (s0 >= 0 && (uint64_t)s0 + 16 <= a.src_total) return load_u<false>(a.src + s0);
    return load_guarded(a, s0, lo, hi);
}

// the payload loads of the simple case: frame k's bytes for v0 (ld[0]) and v1 (ld[2]), frame
// k - 1's tail for v0 (ld[1])
__device__ __forceinline__ void fix_plan(const EncArgs& a, uint64_t k, uint64_t S, uint64_t op, uint64_t o, uint64_t on,
                                         u32x4 (&ld)[3]) {
    const FixGeo g = fix_geo(a, k, S, op, o, on);
    ld[0] = ld[1] = ld[2] = u32x4{0, 0, 0, 0};
    if (!g.simple) return;
    const int64_t phi0 = (int64_t)g.Sn - (int64_t)g.v0, phi1 = (int64_t)g.Sn - (int64_t)g.v1;
    const int64_t plo0 = (int64_t)g.pw - (int64_t)g.v0, plo1 = (int64_t)g.pw - (int64_t)g.v1;
    if (g.own0) {
        if (plo0 < 16 && g.len) ld[0] = fix_load(a, (int64_t)o - plo0, plo0 < 0 ? 0 : (int)plo0, phi0 > 16 ? 16 : (int)phi0);
        if (g.v0 < S && k > 0) ld[1] = fix_load(a, (int64_t)o - ((int64_t)S - (int64_t)g.v0), 0, (int)((int64_t)S - (int64_t)g.v0));
    }
    if (g.v1 != g.v0 && plo1 < 16 && g.len)
        ld[2] = fix_load(a, (int64_t)o - plo1, plo1 < 0 ? 0 : (int)plo1, phi1 > 16 ? 16 : (int)phi1);
}

__device__ __forceinline__ void fix_store(const EncArgs& a, uint64_t k, uint64_t S, uint64_t op, uint64_t o, uint64_t on,
                                          uint32_t keyp, uint32_t key, uint32_t b0, const u32x4 (&ld)[3], uint64_t wlo) {
    const bool masked = a.masked != 0;
    const FixGeo g = fix_geo(a, k, S, op, o, on);
    if (!g.simple) {   // small frames: the general walk
        if (g.own0) {
            if (k > 0 && g.v0 < S) compose_from(a, g.v0, k - 1, S - header_len(o - op, masked) - (o - op), op, wlo);
            else compose_from(a, g.v0, k, S, o, wlo);
        }
        if (g.v1 != g.v0) compose_from(a, g.v1, k, S, o, wlo);
        return;
    }
    uint64_t hlo, hhi;
    build_header(b0, g.len, masked, key, hlo, hhi);
    auto vec = [&](uint64_t V, const u32x4& pa, const u32x4& pb) {
        u32x4 out = shift_bytes(hlo, hhi, (int)((int64_t)S - (int64_t)V)) &
                    select_range((int64_t)S - (int64_t)V, (int64_t)g.pw - (int64_t)V);
        // frame k's payload bytes [pw, V + 16)
        const int64_t plo = (int64_t)g.pw - (int64_t)V;
        if (plo < 16 && g.len) {
            const uint32_t rk = rotr8(key, (uint64_t)(-plo));
            const u32x4 kv = {rk, rk, rk, rk};
            out |= (pa ^ kv) & select_range(plo, (int64_t)g.Sn - (int64_t)V);
        }
        // frame k - 1's payload bytes [V, S): its payload ends at o (= off[k]); the phase of
        // byte 0 is its offset in frame k - 1's payload
        if (V < S && k > 0) {
            const int64_t e = (int64_t)S - (int64_t)V;
            const uint32_t rk = rotr8(keyp, (uint64_t)((int64_t)o - e - (int64_t)op));
            const u32x4 kv = {rk, rk, rk, rk};
            out |= (pb ^ kv) & select_range(0, e);
        }
        store_wire<false>(a, V, out, wlo, kInf);
    };
    if (g.own0) vec(g.v0, ld[0], ld[1]);
    if (g.v1 != g.v0) vec(g.v1, ld[2], ld[2]);
}

__device__ __forceinline__ void fix_vectors(const EncArgs& a, uint64_t k, uint64_t wlo) {
    const bool masked = a.masked != 0;
    // frame k's header start and frames k - 1, k, k + 1's payload offsets in one trip (k - 1
    // clamped: its values are unused for k = 0)
    const uint64_t kp = k > 0 ? k - 1 : 0;
    const uint64_t op = gptr(a.off)[kp], o = gptr(a.off)[k], on = gptr(a.off)[k + 1];
    const uint64_t S = (a.affine ? o - a.off0 + a.hstride * k : gptr(a.wo)[k]) + a.wmis;
    const uint32_t keyp = masked ? gptr(a.keys)[kp] : 0u, key = masked ? gptr(a.keys)[k] : 0u;
    const uint32_t b0 = a.b0 ? (uint32_t)gptr(a.b0)[k] : 0x82u;
    const uint64_t opk = k > 0 ? op : o;
    u32x4 ld[3];
    fix_plan(a, k, S, opk, o, on, ld);
    fix_store(a, k, S, opk, o, on, keyp, key, b0, ld, wlo);
}

// One tile = kScanBlock frames.  The offsets go through LDS both ways so that every
// global access is coalesced (thread t owns frames t*16 .. t*16+15 of the tile: read
// straight from HBM, each load instruction would touch 64 cache lines, and with one
// tile per CU that strided traffic, not the scan, set the kernel's time).
//
// FIX (netc_gpu_encode_frames with NETC_GPU_KNOB_ENC_FIX = 1): the tile's frames then compose the 16-B wire vectors
// holding their header bytes (fix_at), which the assembly launch after this one never stores.
// Each thread owns frames base + t0 .. + kScanPer - 1 and holds their payload offsets, so a
// frame's wire start is known the moment the tile's prefix is: its keys and header bytes are
// loaded before the look-back, its payload vectors after it -- one trip more in this launch in
// place of the assembly's trailing fixup blocks.  Slower on MI355X (see launch_encode_frames).
template <int kScanPer, bool FIX>
__global__ __launch_bounds__(kScanThreads) void wire_offsets_chained(const uint64_t* off, uint64_t n, uint32_t fixed,
                                                                     uint64_t* wo, uint64_t* status, uint32_t epoch,
                                                                     uint32_t* defer_count, EncArgs fa) {
    constexpr uint64_t kScanBlock = (uint64_t)kScanThreads * kScanPer;   // frames per tile
    __shared__ uint64_t tile_prefix;
    __shared__ uint64_t v[kScanBlock + kScanBlock / kScanPer + 1];   // entry j at j + j / kScanPer
    auto pos = [](uint32_t j) { return j + j / kScanPer; };
    const uint64_t tile = blockIdx.x, base = tile * kScanBlock;
    const uint32_t t0 = threadIdx.x * kScanPer;   // this thread's frames: base + t0 ..
    if (tile == 0 && threadIdx.x == 0) *defer_count = 0;   // (a spare word of the scratch; no reader since round 4)
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        const uint32_t j = i * kScanThreads + threadIdx.x;
        v[pos(j)] = gptr(off)[base + j < n ? base + j : n];
    }
    if (threadIdx.x == 0) v[pos(kScanBlock)] = gptr(off)[base + kScanBlock < n ? base + kScanBlock : n];
    const uint64_t off0 = gptr(off)[0];
    // FIX: keys and header bytes of this thread's frames and of the frame before them
    uint32_t key[kScanPer + 1], hb[kScanPer];
    if constexpr (FIX) {
        const uint64_t k0 = base + t0;
#pragma unroll
        for (int i = 0; i <= kScanPer; ++i) {
            const uint64_t k = k0 + i - 1;   // i = 0: frame k0 - 1
            key[i] = fa.masked && k0 + i >= 1 && k < n ? gptr(fa.keys)[k] : 0u;
            if (i > 0) hb[i - 1] = fa.b0 && k < n ? (uint32_t)gptr(fa.b0)[k] : 0x82u;
        }
    }
    __syncthreads();
    uint64_t o[kScanPer + 1];
#pragma unroll
    for (int i = 0; i <= kScanPer; ++i) o[i] = v[pos(t0 + i)];
    uint64_t op0 = 0;   // FIX: off[] of the frame before this thread's first
    if constexpr (FIX) op0 = t0 > 0 ? v[pos(t0 - 1)] : (base > 0 ? gptr(off)[base - 1] : 0);
    uint32_t e[kScanPer];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        e[i] = base + t0 + i < n ? ext_len(o[i + 1] - o[i]) : 0u;
        s += e[i];
    }
    uint64_t agg;
    const uint64_t ex = block_exclusive_scan(s, &agg);   // its barriers also end the LDS reads above
    if (threadIdx.x < kWave) {
        const int lane = threadIdx.x;
        if (lane == 0)
            __hip_atomic_store(&status[tile], status_word(tile == 0 ? 2 : 1, epoch, agg), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t prefix = tile == 0 ? 0 : look_back(status, (int64_t)tile, epoch, lane);
        if (lane == 0) {
            if (tile) __hip_atomic_store(&status[tile], status_word(2, epoch, prefix + agg), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            tile_prefix = prefix;
        }
    }
    __syncthreads();
    uint64_t run = tile_prefix + ex;
    uint64_t S[kScanPer];
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        const uint64_t j = base + t0 + i;
        S[i] = (o[i] - off0) + (uint64_t)fixed * j + run;
        v[pos(t0 + i)] = S[i];
        run += e[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        const uint32_t j = i * kScanThreads + threadIdx.x;
        if (base + j <= n) gptr(wo)[base + j] = v[pos(j)];
    }
    if constexpr (FIX) {   // two frames' loads at a time, then their stores (four: the loads went to scratch)
        constexpr int G = kScanPer < 2 ? kScanPer : 2;
#pragma unroll
        for (int g = 0; g < kScanPer; g += G) {
            u32x4 ld[G][3];
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (base + t0 + g + i < n)
                    fix_plan(fa, base + t0 + g + i, S[g + i] + fa.wmis, g + i == 0 ? op0 : o[g + i - 1], o[g + i], o[g + i + 1], ld[i]);
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (base + t0 + g + i < n)
                    fix_store(fa, base + t0 + g + i, S[g + i] + fa.wmis, g + i == 0 ? op0 : o[g + i - 1], o[g + i], o[g + i + 1],
                              key[g + i], key[g + i + 1], hb[g + i], ld[i], fa.wmis);
        }
    }
}

// Chunk = U spans.  Wavefront w of W takes chunks w, w+W, ...  Per trip: the table
// of chunk c+W (issued a trip ago) is resolved and chunk c+W's loads are issued,
// chunk c+2W's table is issued, then chunk c (loaded a trip ago) is stored.
// W: wavefronts per SIMD the register budget must allow (launch_enc_u picks it per batch)
// Blocks main_blocks .. gridDim.x - 1 (dispatched as the assembly blocks retire: its tail)
// compose the vectors holding header bytes (fix_vectors, one thread per frame).  They share
// no vector with the assembly's stores, so nothing orders the two.
// One length class (a.affine): the same threads write wo[k] and check frame k's class; a frame
// outside it gets no header vectors (the wire is then unspecified, and no byte is written outside
// [wire, wire + the bound)).  The last fixup block to retire writes wo[n]: the wire length, or
// UINT64_MAX when any block met such a frame -- one atomic word carries both the count and the
// verdict, so no fence orders them.
__device__ void fixup_block(const EncArgs& a) {
    const uint64_t wlo = a.wmis;
    const uint64_t fb = blockIdx.x - a.main_blocks, nfb = gridDim.x - a.main_blocks;
    int broken = 0;
    for (uint64_t k = fb * blockDim.x + threadIdx.x; k < a.n; k += nfb * blockDim.x) {
        bool fix = true;
        uint64_t o = 0;
        if (a.affine) {
            o = gptr(a.off)[k];
            const uint64_t on = gptr(a.off)[k + 1];
            fix = on >= o && ext_len(on - o) == a.ext;
            broken |= fix ? 0 : 1;
        }
        if (fix) fix_vectors(a, k, wlo);   // (one call site: a second inlined copy spills the kernel)
        // (wo[k] stored last: a store before fix_vectors would make it reload off[])
        if (a.affine) gptr(a.wo_out)[k] = o - a.off0 + a.hstride * k;
    }
    if (!a.affine) return;
    broken = __syncthreads_or(broken);
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(a.fix_done, 1u + (broken ? 0x10000u : 0u), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if ((old & 0xFFFFu) == (uint32_t)nfb - 1) {
            gptr(a.wo_out)[a.n] = (old >> 16) || broken ? ~0ull : wire_at(a, a.n);
            __hip_atomic_store(a.fix_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// PF (knob ENC_PF): the walk software-pipelined -- chunk c + W's table is resolved and its loads
// issued before chunk c is stored, so a wavefront keeps two chunks of loads in flight (one plan
// more in registers).
template <int U, bool NT, int W, bool PF = false>
__global__ __launch_bounds__(256, W) void encode_frames_kernel(EncArgs a) {
    if (a.affine) a.off0 = gptr(a.off)[0];
    const uint64_t wire_total = wire_at(a, a.n);
    if (blockIdx.x >= a.main_blocks) {   // block-uniform
        fixup_block(a);
        return;
    }
    constexpr uint64_t kWin = kSpan * U;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wpb = blockDim.x / kWave;
    const uint64_t nwaves = (uint64_t)a.main_blocks * wpb;
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // uniform: scalar branches, exact vmcnt waits
    const uint64_t wlo = a.wmis, whi = a.wmis + wire_total;
    const uint64_t nwin = (whi + kWin - 1) / kWin;
    const double density = wire_total ? (double)a.n / (double)wire_total : 0.0;   // frames per wire byte
    // spans the assembly cannot map (kSpanQueued: the first and last, spans the frame table does not
    // cover, loads that would leave the payload): listed by lane 0 in the wavefront's own slice of
    // the defer array (plain stores, read back by the same lane), composed after its windows
    uint64_t* list = a.defer + wave * a.per_wave;
    uint32_t nl = 0;   // wave-uniform
    auto done = [&]() {
        for (uint32_t i = 0; i < nl; ++i) {
            uint64_t A0 = 0;
            if (lane == 0) A0 = list[i];
            A0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(A0 >> 32)) << 32) |
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)A0);
            EncTable t;
            enc_table_load(a, t, enc_locate(a, A0, wire_total, lane), lane);
            const uint64_t Wq = A0 + 16ull * (uint64_t)lane;
            const u32x4 v = compose_vec(a, t, A0, Wq, lane);
            if (Wq < whi) store_wire<false>(a, Wq, v, wlo, whi);
        }
    };

    // ENC_FIX = 2: the header vectors by the assembly's own wavefronts once their windows are
    // stored (64 frames a wavefront, one per lane: fix_vectors), instead of trailing blocks
    auto tail_fix = [&]() {
        if (!a.fix_tail) return;
        for (uint64_t k = wave * kWave + (uint64_t)lane; k < a.n; k += nwaves * kWave) fix_vectors(a, k, wlo);
    };
    uint64_t c = wave;
    if (c >= nwin) {
        tail_fix();
        return;
    }
    // table base for the chunk at A from a frame f_known starting at s_known,
    // biased 24 frames back (the spread of independent random sizes)
    auto guess = [&](int64_t f_known, uint64_t s_known, uint64_t A) -> int64_t {
        if (A < a.wmis) return -1;
        int64_t g = f_known + (int64_t)((double)(A - s_known) * density) - a.probe_bias;
        g = g < -1 ? -1 : g;
        return g > (int64_t)a.n ? (int64_t)a.n : g;
    };
    auto known = [&](const EncTable& t, uint64_t A, int64_t& f, uint64_t& s) {
        const int j = __popcll(__ballot(t.start <= A)) - 1;
        f = t.kb + j;
        s = readlane64(t.start, j);
    };
    // Per trip: the table of this chunk (issued a trip ago) is resolved, the chunk's
    // loads are issued, the next chunk's table is issued, then this chunk is stored.
    // No payload prefetch across trips: the state stays small (one plan, two tables)
    // so that 4+ wavefronts per SIMD keep the loads in flight instead.
    EncTable tc;
    uint64_t A = c * kWin;
    enc_table_issue(a, tc, guess(0, a.wmis, A), lane, a.probe_e);
    if constexpr (PF) {
        enc_table_finish(tc);
        enc_resolve(a, tc, A, wire_total, lane);
        Plan<U> pc;
        plan_chunk<U, NT>(a, tc, A, wlo, whi, lane, pc);
        int64_t f;
        uint64_t s;
        known(tc, A, f, s);
        uint64_t cn = c + nwaves;
        if (cn < nwin) enc_table_issue(a, tc, guess(f, s, cn * kWin), lane, a.probe_e);   // tc: chunk cn's table
        for (;;) {
            const bool more = cn < nwin;   // wave-uniform
            const uint64_t An = cn * kWin;
            Plan<U> pn;
            if (more) {
                enc_table_finish(tc);
                enc_resolve(a, tc, An, wire_total, lane);
                plan_chunk<U, NT>(a, tc, An, wlo, whi, lane, pn);
                known(tc, An, f, s);
                if (cn + nwaves < nwin) enc_table_issue(a, tc, guess(f, s, (cn + nwaves) * kWin), lane, a.probe_e);
            }
            finish_chunk<U, NT>(a, tc, A, wlo, whi, lane, pc, list, nl);   // (finish_chunk reads no table)
            if (!more) break;
            pc = pn;
            A = An;
            cn += nwaves;
        }
        done();
        tail_fix();
        return;
    }
    for (;;) {
        enc_table_finish(tc);
        enc_resolve(a, tc, A, wire_total, lane);
        Plan<U> pc;
        plan_chunk<U, NT>(a, tc, A, wlo, whi, lane, pc);
        int64_t f;
        uint64_t s;
        known(tc, A, f, s);
        const uint64_t cn = c + nwaves;
        EncTable tn;
        if (cn < nwin) enc_table_issue(a, tn, guess(f, s, cn * kWin), lane, a.probe_e);
        finish_chunk<U, NT>(a, tc, A, wlo, whi, lane, pc, list, nl);
        if (cn >= nwin) break;
        c = cn;
        A = cn * kWin;
        tc = tn;
    }
    done();
    tail_fix();
}

typedef unsigned __int128 u128;

// the low `left` (<= 16) bytes of v at w, with the widest naturally aligned stores
__device__ __forceinline__ void put_bytes(NETC_GLOBAL uint8_t* w, u128 v, uint64_t left) {
    uint64_t addr = (uint64_t)(uintptr_t)w;
    while (left) {
        const uint64_t sz = (addr & 1) || left < 2 ? 1 : (addr & 2) || left < 4 ? 2 : (addr & 4) || left < 8 ? 4 : 8;
        NETC_GLOBAL uint8_t* q = (NETC_GLOBAL uint8_t*)addr;
        if (sz == 8) *(NETC_GLOBAL uint64_t*)q = (uint64_t)v;
        else if (sz == 4) *(NETC_GLOBAL uint32_t*)q = (uint32_t)v;
        else if (sz == 2) *(NETC_GLOBAL uint16_t*)q = (uint16_t)v;
        else *q = (uint8_t)v;
        v >>= 8 * sz;
        addr += sz;
        left -= sz;
    }
}

// Dense batches (all_spans): every span composed per lane, no assembly launch before this one.
__global__ __launch_bounds__(256) void encode_queued_kernel(EncArgs a) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / kWave);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / kWave) + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t wire_total = gptr(a.wo)[a.n];
    const uint64_t wlo = a.wmis, whi = a.wmis + wire_total;
    {
        // dense batch: no assembly launch before this one -- every span is composed
        // here, so no header fixups either.  A wave takes kDenseGroup consecutive
        // spans per trip: one search for the first, then each next span's table is
        // re-based at the frame holding its start (one load, no search).
        const uint64_t nspans = (whi + kSpan - 1) / kSpan;
        const uint64_t ngroups = (nspans + kDenseGroup - 1) / kDenseGroup;
        for (uint64_t g = wave; g < ngroups; g += nwaves) {
            uint64_t A0 = g * kDenseGroup * kSpan;
            EncTable t;
            enc_table_load(a, t, enc_locate(a, A0, wire_total, lane), lane);
            for (int s = 0; s < kDenseGroup && A0 < whi; ++s, A0 += kSpan) {
                const int j = __popcll(__ballot(t.start <= A0)) - 1;   // >= 0: entry 0 is at or before A0
                if (j > 0 && !t.tail) enc_table_load(a, t, t.kb + j, lane);
                const uint64_t W = A0 + 16ull * (uint64_t)lane;
                const u32x4 v = compose_vec(a, t, A0, W, lane);
                if (W < whi) store_wire<false>(a, W, v, wlo, whi);
            }
        }
    }
}

// ------------------------------------------------------------ source-driven --
// Round 4 (an A/B path, NETC_GPU_KNOB_ENC_SRC = 1 -- measured slower than the
// wire-driven default, see launch_encode_frames): the assembly walks the SOURCE.  The wire is the payload buffer with
// a header inserted before each frame's payload, so a wavefront takes a window of the payload
// buffer and issues its 16-B loads at once -- their addresses need no frame table, where the
// wire-driven kernel above could not issue a window's loads before its table resolved -- and
// looks up the window's frames while they are in flight.  Each lane's 16 bytes then go to
// their wire position:
//   * inside one frame's payload (all lanes but about one per frame): one unaligned 16-B store
//     of the bytes XOR the frame's key at its phase;
//   * holding one frame start, at byte j (that frame's first payload byte): the lane's wire
//     region is its 16 bytes with the frame's header (hl bytes) inserted at j -- 16 + hl
//     contiguous bytes -- written as two overlapping 16-B stores (the bytes before j, the
//     bytes from j on shifted by hl) and then the header's narrow stores; one lane's stores to
//     one address land in program order, so the header overwrites what the 16-B stores left
//     in its place;
//   * anything else (frame starts closer than 16 bytes, empty frames, the batch's ends, a
//     partial vector): byte-exact per lane from the frame table (src_general).
// The lanes' regions tile the wire, so no byte is written by two lanes and the headers need
// no launch of their own (encode_queued_kernel, one thread per frame: 8 us at config 2).
static constexpr int64_t kPastEnd = INT64_MAX;

struct SrcTable {
    int64_t kb;        // frame index of lane 0's entry (-1: the virtual head)
    int64_t start;     // P coordinates of the entry's payload start; -1 for the head, kPastEnd past frame n
    uint64_t wo;       // its wire offset (header start)
    uint32_t key, b0;
    int64_t last;      // start of entry e - 1 (uniform)
    bool tail;         // the entry for frame n is in the table
    int e;             // entries held: 64, or fewer for a window's first probe (uniform)
};

// issue the table loads of frames kb .. kb + e - 1 (lanes past e - 1 re-load entry e - 1: the
// same lines, no lane branches around a load); the values are selected in src_finish
__device__ __forceinline__ void src_issue(const EncArgs& a, SrcTable& t, int64_t kb, int lane, int e = kWave) {
    const int64_t n = (int64_t)a.n, v = kb + (lane < e ? lane : e - 1);
    const int64_t vo = v < 0 ? 0 : (v > n ? n : v);
    const int64_t vk = v < 0 ? 0 : (v >= n ? (n > 0 ? n - 1 : 0) : v);
    const uint64_t off = gptr(a.off)[vo];
    t.wo = gptr(a.wo)[vo];
    t.key = gptr(a.keys_ld)[vk];   // (selected in src_finish: a branch here would drain the payload loads)
    t.b0 = (uint32_t)gptr(a.b0_ld)[vk];
    t.kb = kb;
    t.e = e;
    t.start = v < 0 ? -1 : (v <= n ? (int64_t)(off + a.smis) : kPastEnd);
    t.tail = kb + (e - 1) >= n;
}

__device__ __forceinline__ void src_finish(const EncArgs& a, SrcTable& t) {
    t.key = a.masked ? t.key : 0u;
    t.b0 = a.b0 ? t.b0 : 0x82u;
    if (t.e < kWave && (int)__lane_id() >= t.e) t.start = kPastEnd;
    t.last = (int64_t)readlane64((uint64_t)t.start, t.e - 1);
}

__device__ __forceinline__ void src_load(const EncArgs& a, SrcTable& t, int64_t kb, int lane) {
    src_issue(a, t, kb, lane);
    src_finish(a, t);
}

// Largest virtual frame L whose payload starts strictly before P (-1: the head), wave-uniform:
// a comb probe around the density's guess, then 64-ary narrowing over off[] (as ws_mask_gpu's
// locate, with a strict bound: the frames starting AT P belong to the span from P on)
__device__ int64_t src_locate(const EncArgs& a, uint64_t P, int lane) {
    if (P <= a.smis) return -1;
    const uint64_t q = P - a.smis;
    int64_t L = -1, H = (int64_t)a.n + 1;
    if (a.n > (uint64_t)kWave && a.src_total > 0) {
        constexpr int64_t kStride = 16;
        int64_t g = (int64_t)((double)q * a.density);
        g = g > (int64_t)a.n ? (int64_t)a.n : g;
        const int64_t base = g - 31 * kStride;
        const int64_t idx = base + (int64_t)lane * kStride;
        const bool valid = idx >= 0 && idx <= (int64_t)a.n;
        const uint64_t val = valid ? gptr(a.off)[idx] : 0;
        const uint64_t lt = __ballot(valid && val < q);
        const uint64_t ge = __ballot(valid && val >= q);
        if (lt) L = base + (int64_t)(63 - __builtin_clzll(lt)) * kStride;
        if (ge) H = base + (int64_t)__builtin_ctzll(ge) * kStride;
    }
    while (H - L > kWave) {
        const int64_t lo = L + 1;
        const int64_t step = (H - lo + kWave - 1) / kWave;
        const int64_t idx = lo + (int64_t)lane * step;
        const bool valid = idx < H;
        const uint64_t val = valid ? gptr(a.off)[idx] : kInf;
        const uint64_t lt = __ballot(valid && val < q);
        const uint64_t ge = __ballot(valid && val >= q);
        if (lt) L = lo + (int64_t)(63 - __builtin_clzll(lt)) * step;
        if (ge) H = lo + (int64_t)__builtin_ctzll(ge) * step;
    }
    return L;
}

__device__ __forceinline__ int64_t src_clamp(const EncArgs& a, int64_t g) {
    g = g < -1 ? -1 : g;
    return g > (int64_t)a.n ? (int64_t)a.n : g;
}

// the table base the density predicts for the window at A: the frame holding byte A - 1
__device__ __forceinline__ int64_t src_guess(const EncArgs& a, uint64_t A) {
    if (A <= a.smis) return -1;
    return src_clamp(a, (int64_t)((double)(A - a.smis - 1) * a.density));
}

// make t (issued at a guessed base) bracket A: entry 0 starts before A, a later entry at or after it
__device__ __forceinline__ void src_resolve(const EncArgs& a, SrcTable& t, uint64_t A, int lane) {
    src_finish(a, t);
#pragma unroll 1
    for (int step = 0; step < 2; ++step) {
        const uint64_t m = __ballot(t.start < (int64_t)A);
        if (m != 0 && (t.tail || __popcll(m) < t.e)) return;
        int64_t g;
        if (m == 0) {   // every entry starts at or after A: step back by the distance from entry 0
            const int64_t s0 = (int64_t)readlane64((uint64_t)t.start, 0);
            g = t.kb - (int64_t)((double)(s0 - (int64_t)A) * a.density) - 40;
        } else {        // every entry starts before A: step on from the last
            g = t.kb + (t.e - 1) + (int64_t)((double)((int64_t)A - t.last) * a.density) - 24;
        }
        src_load(a, t, src_clamp(a, g), lane);
    }
    const uint64_t m = __ballot(t.start < (int64_t)A);
    if (!(m != 0 && (t.tail || __popcll(m) < t.e))) src_load(a, t, src_locate(a, A, lane), lane);
}

__device__ __forceinline__ uint8_t vbyte(const u32x4& d, int64_t i) {
    const uint32_t w = i < 4 ? d[0] : (i < 8 ? d[1] : (i < 12 ? d[2] : d[3]));
    return (uint8_t)(w >> (8 * (i & 3)));
}

// The byte-exact path: every payload byte of the lane's vector [P, P + 16) (d) to its wire
// position, and the header of every frame whose payload starts in it (empty frames too).
// Per lane a binary search of the table (ds_bpermute) finds the last frame starting before
// P, then the lane walks the frames starting in its 16 bytes; spans with more frames than
// one table holds are walked in 62-entry windows (entry 62 is shared by two windows: its
// bytes are written twice, with the same values).  act: the lane takes part.
__device__ void src_general(const EncArgs& a, SrcTable t, uint64_t A0, int64_t P, u32x4 d, bool act, int lane) {
    constexpr int kLast = kWave - 2;
    const int64_t Aend = (int64_t)(A0 + kSpan);
    const bool masked = a.masked != 0;
    NETC_GLOBAL uint8_t* wire = gptr(a.wire_base) + a.wmis;
    if (t.e < kWave) src_load(a, t, t.kb, lane);   // a window's first probe: the full table
    for (;;) {
        const bool more = !t.tail && t.last < Aend;   // wave-uniform
        SrcTable tn;
        if (more) src_issue(a, tn, t.kb + kLast, lane);
        int l = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const int c = l + step;
            const int64_t sc = (int64_t)bperm64((uint64_t)t.start, c <= kLast ? c : kLast);   // every lane takes part
            if (c <= kLast && sc < P) l = c;
        }
        for (int c = l;; ++c) {
            const int cc = c <= kLast ? c : kLast;
            const int64_t S = (int64_t)bperm64((uint64_t)t.start, cc), Sn = (int64_t)bperm64((uint64_t)t.start, cc + 1);
            const uint64_t wo = bperm64(t.wo, cc);
            const uint32_t key = (uint32_t)__builtin_amdgcn_ds_bpermute(cc << 2, (int)t.key);
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_ds_bpermute(cc << 2, (int)t.b0);
            const int64_t j = t.kb + cc;
            const bool cont = act && c <= kLast && j < (int64_t)a.n && S < P + 16;
            if (cont && j >= 0) {
                const uint64_t len = (uint64_t)(Sn - S), hl = header_len(len, masked);
                if (S >= P) {   // the frame's header: this lane holds its first payload byte (or its place)
                    uint64_t lo, hi;
                    build_header(b0, len, masked, key, lo, hi);
                    put_bytes(wire + wo, (u128)hi << 64 | lo, hl);
                }
                const int64_t blo = S > P ? S : P, bhi = Sn < P + 16 ? Sn : P + 16;
                for (int64_t p = blo; p < bhi; ++p)
                    wire[wo + hl + (uint64_t)(p - S)] = vbyte(d, p - P) ^ (uint8_t)(key >> (8 * ((p - S) & 3)));
            }
            if (!__ballot(cont)) break;
        }
        if (!more) break;
        t = tn;
        src_finish(a, t);
    }
}

typedef uint32_t u32x4s __attribute__((ext_vector_type(4), aligned(1)));   // unaligned 16-B store

template <bool NT>
__device__ __forceinline__ void store_u(NETC_GLOBAL uint8_t* p, u32x4 v) {
    NETC_GLOBAL u32x4s* q = (NETC_GLOBAL u32x4s*)p;
    if constexpr (NT) __builtin_nontemporal_store(v, q);
    else *q = v;
}

__device__ __forceinline__ u128 as128(u32x4 v) {
    return (u128)v[0] | (u128)v[1] << 32 | (u128)v[2] << 64 | (u128)v[3] << 96;
}
__device__ __forceinline__ u32x4 from128(u128 x) {
    return u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)};
}
__device__ __forceinline__ u128 low_bytes(int64_t k) {   // bytes [0, k) set, k clamped to [0, 16]
    return k <= 0 ? (u128)0 : (k >= 16 ? ~(u128)0 : (((u128)1 << (8 * k)) - 1));
}

// One span of the window (1 KiB of source at A0; d = the lane's 16 bytes at P).  interior:
// d was loaded whole (every byte inside the buffer).
template <bool NT>
__device__ __forceinline__ void src_span(const EncArgs& a, SrcTable& t, uint64_t A0, u32x4 d, bool interior, int lane) {
    const int64_t Aend = (int64_t)(A0 + kSpan);
    const int64_t P = (int64_t)(A0 + 16ull * (uint64_t)lane);
    const bool masked = a.masked != 0;
    int lbase = __popcll(__ballot(t.start < (int64_t)A0)) - 1;
    if (!(t.tail || t.last >= Aend) && (lbase > 0 || t.e < kWave)) {   // a full table from the span's first frame on
        src_load(a, t, t.kb + lbase, lane);
        lbase = __popcll(__ballot(t.start < (int64_t)A0)) - 1;
    }
    const uint64_t bm = __ballot(t.start >= (int64_t)A0 && t.start < Aend);
    const int nb = __popcll(bm);
    const bool covered = interior && lbase >= 0 && lbase + nb + 2 <= t.e - 1 && (t.tail || t.last >= Aend);
    bool fast = false;
    if (covered) {   // wave-uniform
        NETC_GLOBAL uint8_t* wire = gptr(a.wire_base) + a.wmis;
        int lp = lbase, cnt = 0;
        for (uint64_t b = bm; b; b &= b - 1) {   // the span's frame starts (wave-uniform loop)
            const int64_t sb = (int64_t)readlane64((uint64_t)t.start, __builtin_ctzll(b));
            lp += sb < P ? 1 : 0;
            cnt += (sb >= P && sb < P + 16) ? 1 : 0;
        }
        const int64_t f = t.kb + lp;
        fast = cnt <= 1 && f >= 0 && f + cnt < (int64_t)a.n;
        // the lane's frames: lp (its first byte's, or the one ending at P) and lp + 1 (the start)
        int64_t S0, S1, S2;
        uint64_t w0, w1;
        uint32_t k0, k1, h1;
        if (nb == 0) {   // one frame covers the span: read once for the wave
            S0 = (int64_t)readlane64((uint64_t)t.start, lbase);
            S1 = (int64_t)readlane64((uint64_t)t.start, lbase + 1);
            S2 = S1;
            w0 = readlane64(t.wo, lbase);
            w1 = w0;
            k0 = readlane32(t.key, lbase);
            k1 = k0;
            h1 = 0;
        } else {
            S0 = (int64_t)bperm64((uint64_t)t.start, lp);
            S1 = (int64_t)bperm64((uint64_t)t.start, lp + 1);
            S2 = (int64_t)bperm64((uint64_t)t.start, lp + 2);
            w0 = bperm64(t.wo, lp);
            w1 = bperm64(t.wo, lp + 1);
            k0 = (uint32_t)__builtin_amdgcn_ds_bpermute(lp << 2, (int)t.key);
            k1 = (uint32_t)__builtin_amdgcn_ds_bpermute((lp + 1) << 2, (int)t.key);
            h1 = (uint32_t)__builtin_amdgcn_ds_bpermute((lp + 1) << 2, (int)t.b0);
        }
        if (fast) {
            const uint64_t len0 = (uint64_t)(S1 - S0);
            const uint32_t rk0 = rotr8(k0, (uint64_t)(P - S0));
            u32x4 m = {rk0, rk0, rk0, rk0};
            if (cnt == 0) {   // inside frame lp's payload
                store_u<NT>(wire + w0 + header_len(len0, masked) + (uint64_t)(P - S0), d ^ m);
            } else {          // frame lp + 1 starts at byte j
                const int64_t j = S1 - P;
                const uint64_t len1 = (uint64_t)(S2 - S1), hl = header_len(len1, masked);
                const uint32_t rk1 = rotr8(k1, (uint64_t)(P - S1));
                const u32x4 sel = select_from(j);
                m = (m & ~sel) | (u32x4{rk1, rk1, rk1, rk1} & sel);
                const u32x4 out = d ^ m;
                NETC_GLOBAL uint8_t* R = wire + w1 - (uint64_t)j;   // the lane's wire region: 16 + hl bytes
                // (plain stores: the header's narrow stores overwrite part of them, and a lane's
                // stores to one address are kept in order under one cache policy)
                if (j > 0) store_u<false>(R, out);                   // bytes before j (the rest overwritten below)
                const u128 o = as128(out);
                store_u<false>(R + hl, from128(((o >> (8 * hl)) & low_bytes(j - (int64_t)hl)) | (o & ~low_bytes(j))));
                uint64_t lo, hi;
                build_header(h1, len1, masked, k1, lo, hi);
                put_bytes(wire + w1, (u128)hi << 64 | lo, hl);        // last: over what the stores left there
            }
        }
    }
    if (__ballot(!fast)) src_general(a, t, A0, P, d, !fast, lane);
}

// guarded load of the lane's 16 bytes at P (partial vectors at the buffer's ends): bytes
// outside [smis, smis + src_total) read as 0 and never written
__device__ __forceinline__ u32x4 src_guarded(const EncArgs& a, int64_t P) {
    u32x4 v = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        const int64_t p = P + b;
        if (p >= (int64_t)a.smis && p < (int64_t)(a.smis + a.src_total))
            v[b >> 2] |= (uint32_t)gptr(a.src_base)[p] << (8 * (b & 3));
    }
    return v;
}

// One window of K KiB of the payload buffer per wavefront, a grid covering the buffer (as the
// mask kernel's default walk): the window's loads first, the table lookup under them.
template <int K, bool NT>
__global__ __launch_bounds__(256) void encode_src_kernel(EncArgs a) {
    constexpr uint64_t kWin = kSpan * K;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / kWave) +
                          (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // uniform
    if (wave >= a.nwin) return;
    const uint64_t A = wave * kWin;
    const uint64_t full_lo = a.smis ? 16 : 0, full_hi = (a.smis + a.src_total) & ~15ull;
    const bool interior = A >= full_lo && A + kWin <= full_hi;   // wave-uniform
    u32x4 d[K];
    if (interior) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const NETC_GLOBAL u32x4* p = gptr(reinterpret_cast<const u32x4*>(a.src_base + A + (uint64_t)k * kSpan + 16ull * lane));
            if constexpr (NT) d[k] = __builtin_nontemporal_load(p);
            else d[k] = *p;
        }
    }
    SrcTable t;
    src_issue(a, t, src_guess(a, A), lane, a.probe_e);
    src_resolve(a, t, A, lane);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t A0 = A + (uint64_t)k * kSpan;
        const u32x4 v = interior ? d[k] : src_guarded(a, (int64_t)(A0 + 16ull * lane));
        src_span<NT>(a, t, A0, v, interior, lane);
    }
}

template <int U, bool NT, int W, bool PF>
static int enc_resident_blocks() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
    if (cache[dev] > 0) return cache[dev];
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, encode_frames_kernel<U, NT, W, PF>, 256, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu <= 0 || cus <= 0)
        return 1024;
    cache[dev] = per_cu * cus;
    return cache[dev];
}

// Per (device, stream) scratch: the scan's status words (one per tile) and the
// span queue.  Work queued on one stream runs in order, so it can share them (the
// epoch tells scans apart); streams may run concurrently and get their own.
// Arrays grow geometrically; an outgrown one may still be read by work queued
// before the growth, so it is kept (retired) until netc_gpu_stream_release frees
// the stream's scratch, after synchronising it.
struct EncScratch {
    uint64_t* status = nullptr;
    uint64_t tiles = 0;
    uint32_t epoch = 0;
    uint64_t* defer = nullptr;   // defer[0 .. cap), then the counter word
    uint64_t defer_cap = 0;
    std::vector<void*> retired;
};

static std::map<std::pair<int, hipStream_t>, EncScratch> g_scratch;
static std::mutex g_scratch_mu;

static hipError_t scratch_for(hipStream_t stream, uint64_t tiles, uint64_t spans, EncScratch& out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(g_scratch_mu);
    EncScratch& sc = g_scratch[{dev, stream}];
    if (sc.tiles < tiles) {
        uint64_t* p = nullptr;
        uint64_t want = sc.tiles ? 2 * sc.tiles : 1024;
        while (want < tiles) want *= 2;
        if ((e = hipMalloc(&p, want * sizeof(uint64_t))) != hipSuccess) return e;
        if ((e = hipMemsetAsync(p, 0, want * sizeof(uint64_t), stream)) != hipSuccess) {
            (void)hipFree(p);
            return e;
        }
        if (sc.status) sc.retired.push_back(sc.status);
        sc.status = p;
        sc.tiles = want;
        sc.epoch = 0;
    }
    if (sc.defer_cap < spans) {
        uint64_t* p = nullptr;
        uint64_t want = sc.defer_cap ? 2 * sc.defer_cap : 4096;
        while (want < spans) want *= 2;
        if ((e = hipMalloc(&p, (want + 1) * sizeof(uint64_t))) != hipSuccess) return e;
        // the word past the spans: the scan's spare word, then the fixup blocks' counter (fix_done)
        if ((e = hipMemsetAsync(p + want, 0, sizeof(uint64_t), stream)) != hipSuccess) {
            (void)hipFree(p);
            return e;
        }
        if (sc.defer) sc.retired.push_back(sc.defer);
        sc.defer = p;
        sc.defer_cap = want;
    }
    sc.epoch = (sc.epoch + 1) & 0xFFFF;
    if (sc.epoch == 0) {   // epochs wrapped: clear the words so no stale epoch can match
        if ((e = hipMemsetAsync(sc.status, 0, sc.tiles * sizeof(uint64_t), stream)) != hipSuccess) return e;
        sc.epoch = 1;
    }
    out.status = sc.status;
    out.tiles = sc.tiles;
    out.epoch = sc.epoch;
    out.defer = sc.defer;
    out.defer_cap = sc.defer_cap;
    return hipSuccess;
}

int release_enc_scratch(int device, hipStream_t stream) {   // the stream is synchronised
    EncScratch sc;
    {
        std::lock_guard<std::mutex> g(g_scratch_mu);
        auto it = g_scratch.find({device, stream});
        if (it == g_scratch.end()) return 0;
        sc = std::move(it->second);
        g_scratch.erase(it);
    }
    if (sc.status) (void)hipFree(sc.status);
    if (sc.defer) (void)hipFree(sc.defer);
    for (void* p : sc.retired) (void)hipFree(p);
    return 1;
}

// frames per thread of the wire-offsets scan: tiles of 1,024 frames up to 256 Ki frames
// (C2 shape, one box: 1 / 2 / 4 / 8 / 16 frames per thread gave 43.9 / 43.2 / 42.3 /
// 42.8 / 44.2 us per call), tiles of 4,096 frames above (1-8 Mi frames of 8-64 B: the
// look-back over 4x the tiles cost more than the shorter tiles saved).
// NETC_GPU_KNOB_ENC_SCAN_PER (env NETC_ENC_SCAN_PER) overrides: measurement.
static int scan_per(uint64_t n) {
    const int64_t k = knob(NETC_GPU_KNOB_ENC_SCAN_PER);
    const int dflt = n <= (256u << 10) ? 4 : 16;
    const int v = k >= 0 ? (int)k : dflt;
    return (v == 1 || v == 2 || v == 4 || v == 8 || v == 16) ? v : dflt;
}

static uint64_t scan_tiles_for(uint64_t n, int per) { return n / ((uint64_t)kScanThreads * per) + 1; }   // frames 0 .. n

// fa: the assembly's arguments when the scan also composes the header vectors (FIX), else null
template <int PER>
static hipError_t launch_scan_per(const uint64_t* off, uint64_t n, bool masked, uint64_t* wo, hipStream_t stream,
                                  const EncScratch& sc, const EncArgs* fa) {
    const uint64_t tiles = scan_tiles_for(n, PER);
    const uint32_t fixed = 2 + (masked ? 4 : 0);
    uint32_t* spare = (uint32_t*)(sc.defer + sc.defer_cap);
    if (fa)
        hipLaunchKernelGGL((wire_offsets_chained<PER, true>), dim3((unsigned)tiles), dim3(kScanThreads), 0, stream, off,
                           n, fixed, wo, sc.status, sc.epoch, spare, *fa);
    else
        hipLaunchKernelGGL((wire_offsets_chained<PER, false>), dim3((unsigned)tiles), dim3(kScanThreads), 0, stream, off,
                           n, fixed, wo, sc.status, sc.epoch, spare, EncArgs{});
    return hipGetLastError();
}

static hipError_t launch_scan(const uint64_t* off, uint64_t n, bool masked, uint64_t* wo, hipStream_t stream,
                              const EncScratch& sc, int per, const EncArgs* fa) {
    switch (per) {
        case 1: return launch_scan_per<1>(off, n, masked, wo, stream, sc, fa);
        case 2: return launch_scan_per<2>(off, n, masked, wo, stream, sc, fa);
        case 4: return launch_scan_per<4>(off, n, masked, wo, stream, sc, fa);
        case 8: return launch_scan_per<8>(off, n, masked, wo, stream, sc, fa);
        default: return launch_scan_per<16>(off, n, masked, wo, stream, sc, fa);
    }
}

hipError_t launch_wire_offsets(const uint64_t* off, uint64_t n, bool masked, uint64_t* wo, hipStream_t stream) {
    if (n == 0) return hipMemsetAsync(wo, 0, sizeof(uint64_t), stream);
    const int per = scan_per(n);
    const uint64_t tiles = scan_tiles_for(n, per);
    if (tiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
    EncScratch sc;
    hipError_t e = scratch_for(stream, tiles, 1, sc);
    if (e != hipSuccess) return e;
    return launch_scan(off, n, masked, wo, stream, sc, per, nullptr);
}

// mean payload bytes per frame under which a batch takes the dense compose path
// (NETC_GPU_KNOB_ENC_DENSE_BYTES overrides: measurement, and the parity tests run both
// paths over the same batches; 0 = never dense)
static uint64_t dense_bytes() {
    const int64_t k = knob(NETC_GPU_KNOB_ENC_DENSE_BYTES);
    return k >= 0 ? (uint64_t)k : (uint64_t)80;
}

template <int U, int W, bool PF = false>
static hipError_t launch_enc_u(EncArgs a, uint64_t wire_bound, bool nt, int max_blocks, hipStream_t stream) {
    const uint64_t nwin = (a.wmis + wire_bound + kSpan * U - 1) / (kSpan * U);
    const uint64_t cap = (uint64_t)(max_blocks > 0 ? max_blocks
                                                  : (nt ? enc_resident_blocks<U, true, W, PF>() : enc_resident_blocks<U, false, W, PF>()));
    const uint64_t want = (nwin + 3) / 4;
    const int blocks = (int)(want < cap ? want : cap);
    if (blocks <= 0) return hipSuccess;
    if (a.all_spans) {
        const uint64_t groups = (nwin * U + kDenseGroup - 1) / kDenseGroup;
        const uint64_t gb = (groups + 3) / 4;   // one group per wavefront, 4 per block
        hipLaunchKernelGGL(encode_queued_kernel, dim3((unsigned)(gb < 8192 ? gb : 8192)), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    // the header fixups as trailing blocks of the same launch (fixup_block), one thread per frame
    // up to 1,024 blocks, unless the wire-offsets scan has composed them (ENC_FIX = 1)
    const uint64_t fix = (a.n + 255) / 256;
    const uint64_t fix_blocks = !a.fix_blocks ? 0 : (fix < 64 ? 64 : (fix > 1024 ? 1024 : fix));
    // each chunk's first table probe: as many entries as the frames a chunk is expected to touch
    // (+ the bias and a margin) when that is a few -- dense batches (config 2: 10 of 64 entries,
    // the rest of the 64-entry table loads were the launch's excess counter traffic) -- else 64
    // entries from 24 frames before the density guess (random sizes).  A probe that misses is
    // replaced by a full table from the binary search (enc_resolve).
    const double reach = (double)(kSpan * U) * ((double)a.n / (double)(wire_bound ? wire_bound : 1));
    const int64_t pk = knob(NETC_GPU_KNOB_ENC_PROBE);
    if (pk == 0 || reach < 1.0 || reach > (double)(kWave - 16)) {
        a.probe_e = kWave;
        a.probe_bias = 24;
    } else {
        a.probe_bias = 2;
        a.probe_e = (int)reach + 10 + (pk > 0 ? (int)pk : 0);
        if (a.probe_e > kWave) a.probe_e = kWave;
    }
    a.main_blocks = (uint32_t)blocks;
    a.per_wave = (uint32_t)(((nwin + 4 * (uint64_t)blocks - 1) / (4 * (uint64_t)blocks)) * U);   // windows per wave x U
    if ((uint64_t)a.per_wave * 4 * (uint64_t)blocks > a.defer_cap) return hipErrorInvalidValue;   // (sized with slack below)
    const unsigned grid = (unsigned)(blocks + fix_blocks);
    if (nt) hipLaunchKernelGGL((encode_frames_kernel<U, true, W, PF>), dim3(grid), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((encode_frames_kernel<U, false, W, PF>), dim3(grid), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_encode_frames(uint8_t* wire, uint64_t wire_bound, const uint8_t* src, uint64_t src_total,
                                const uint64_t* off, const uint32_t* keys, const uint8_t* b0, uint64_t n, bool masked,
                                uint64_t* wo, hipStream_t stream, const LaunchCfg& cfg, int ext_class) {
    if (n == 0) return hipMemsetAsync(wo, 0, sizeof(uint64_t), stream);
    // frames averaging under dense_bytes() of payload: every span is composed per lane
    // (the vector path would queue most spans and leave a header fixup per frame)
    const bool all_spans = src_total < dense_bytes() * n;
    const bool src_walk = !all_spans && knob(NETC_GPU_KNOB_ENC_SRC) == 1;
    // the header vectors: composed by trailing blocks of the assembly launch (default), by the
    // wire-offsets scan (NETC_GPU_KNOB_ENC_FIX = 1), or not at all (dense batches and the
    // source-driven walk write every byte themselves).  The scan variant measured slower: config
    // 2 40.5-47 us per step (1-4 frames per scan thread) against 37.3 with the trailing blocks,
    // config 4 421-430 against 417-424 -- on the scan's critical path the fixups cost more than
    // in the assembly's tail, where they fill the CUs its last waves leave (r04kk)
    const bool fix_in_scan = !all_spans && !src_walk && knob(NETC_GPU_KNOB_ENC_FIX) == 1;
    const bool fix_tail = !all_spans && !src_walk && knob(NETC_GPU_KNOB_ENC_FIX) == 2;
#ifdef NETC_ENC_DIAG_NOFIX   // diagnostic build only (tools/pmc_encode.sh): no header fixups -- wrong
    const bool fix_blocks = false;   // wire bytes, for attributing the assembly's counter traffic
#else
    const bool fix_blocks = !all_spans && !src_walk && !fix_in_scan && !fix_tail;
#endif
    // (the scan with the fixups holds 8 frames per thread at most: 16 spilled)
    const int per0 = scan_per(n), per = fix_in_scan && per0 > 8 ? 8 : per0;
    const uint64_t tiles = scan_tiles_for(n, per);
    if (tiles > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const uint64_t wmis = (uint64_t)(uintptr_t)wire & 15u;
    // every span could be listed, in per-wavefront slices of the same length (+ slack: a wavefront's
    // share of windows rounds up)
    const uint64_t spans = (wmis + wire_bound + kSpan - 1) / kSpan + 8 + 4 * 4 * 8192;
    EncScratch sc;
    hipError_t e = scratch_for(stream, tiles, spans, sc);
    if (e != hipSuccess) return e;
    EncArgs a;
    a.wmis = wmis;
    a.wire_base = wire - a.wmis;
    a.src = src;
    a.src_total = src_total;
    a.off = off;
    a.wo = wo;
    a.keys = masked ? keys : nullptr;
    a.b0 = b0;
    a.n = n;
    a.masked = masked ? 1u : 0u;
    a.defer = sc.defer;
    a.defer_count = (uint32_t*)(sc.defer + sc.defer_cap);
    a.defer_cap = sc.defer_cap;
    a.all_spans = all_spans ? 1u : 0u;
    a.fix_blocks = fix_blocks ? 1u : 0u;
    a.fix_tail = fix_tail ? 1u : 0u;
    // One length class (ext_class 0, 2 or 8: netc_gpu_encode_frames_class): on the default path
    // the wire offsets are affine and the trailing fixup blocks write them -- no scan launch, whose
    // ~5 us at config 2 the assembly waited for.  Up to 256 MiB of wire: the affine form costs the
    // assembly itself a little per chunk (config 2 kernel 35.3 against 33.7 us, the step 35.3
    // against 38.4), and at config 4's 1 GiB more than the scan it saves (424.4-427.7 against
    // 419.2-419.6 us a step; profiles/r05_kernels/encode_class.json).  The other paths run the scan,
    // which needs no class and is exact whatever the frames are.
    const bool one_launch_ok = wire_bound <= (256ull << 20);
    a.affine = ext_class >= 0 && fix_blocks && one_launch_ok ? 1u : 0u;
    a.ext = ext_class >= 0 ? (uint32_t)ext_class : 0u;
    a.hstride = 2u + (masked ? 4u : 0u) + a.ext;
    a.off0 = 0;
    a.fix_done = a.defer_count + 1;
    a.wo_out = wo;
    if (!a.affine &&
        (e = launch_scan(off, n, masked, wo, stream, sc, per, fix_in_scan ? &a : nullptr)) != hipSuccess)
        return e;
    const bool nt = cfg.flags < 0 || (cfg.flags & (kNtLoads | kNtStores));
    // Chunk size: 4 KiB chunks, 5 wavefronts per SIMD by default; netc_gpu_tune's unroll 2 or 4
    // select 2 KiB chunks at 6 wavefronts (A/B only).  Round 3 took 2 KiB above 256 MiB of wire
    // (C4 416-417 against 422-423 us then); the kernel has grown since, and at 6 wavefronts the
    // 2 KiB form spills 18 VGPRs to scratch: C4 435-437 us against 421-423 for 4 KiB (round 5,
    // three interleaved rounds, profiles/r05_kernels/encode_c4_chunk.json).  C2 39.0-39.3 against
    // 39.8-39.9 us (profiles/r03r_enc_chunk.json).
    // NETC_GPU_KNOB_ENC_SRC = 1: the source-driven walk (round 4 experiment, kept for A/B: parity
    // green, but slower than the wire-driven kernels at both shapes measured -- config 2 35.3 us
    // against 26.6 + 7.9 for the wire-driven kernel and the header fixups, config 4 428-438 us
    // against 404 + 8; its unaligned 16-B stores cost ~5 % at config 4 and the per-span frame
    // logic more than the fixup launch at config 2; profiles/r04c_encode_src_ab.json)
    if (src_walk) {
        constexpr int K = 2;
        constexpr uint64_t kWin = kSpan * K;
        a.smis = (uint64_t)(uintptr_t)src & 15u;
        a.src_base = src - a.smis;
        a.density = (double)n / (double)src_total;
        // + 1: the window holding P = smis + src_total writes the headers of empty frames at the end
        a.nwin = (a.smis + src_total) / kWin + 1;
        const double reach = (double)kWin * a.density;
        a.probe_e = reach < (double)(kWave - 6) ? (int)reach + 6 : kWave;
        a.keys_ld = masked ? keys : reinterpret_cast<const uint32_t*>(off);   // off[0 .. n] is readable
        a.b0_ld = b0 ? b0 : reinterpret_cast<const uint8_t*>(off);
        const uint64_t blocks = (a.nwin + 3) / 4;
        if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
        if (nt) hipLaunchKernelGGL((encode_src_kernel<K, true>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
        else hipLaunchKernelGGL((encode_src_kernel<K, false>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    // The software-pipelined walk (4 KiB chunks, 4 wavefronts per SIMD) above 256 MiB of wire: C4
    // 416.2-416.8 us against 422.8-424.2, while at C2 it loses (41.1-41.3 against 38.0-38.5 us:
    // ~4 chunks per wavefront, the deeper prologue is not repaid).  2 KiB chunks pipelined at 5
    // wavefronts lose at both (C2 40.9-41.1, C4 425.3-426.7 us).  Three interleaved rounds, one
    // box, profiles/r05_kernels/encode_pf_ab.json.  NETC_GPU_KNOB_ENC_PF: 0 never, 1 / 2 always.
    const int64_t pf = knob(NETC_GPU_KNOB_ENC_PF);
    if (pf == 1) return launch_enc_u<2, 5, true>(a, wire_bound, nt, cfg.max_blocks, stream);
    if (pf == 2 || (pf < 0 && cfg.unroll <= 1 && wire_bound > (256ull << 20)))
        return launch_enc_u<4, 4, true>(a, wire_bound, nt, cfg.max_blocks, stream);
    if (cfg.unroll == 2 || cfg.unroll == 4) return launch_enc_u<2, 6>(a, wire_bound, nt, cfg.max_blocks, stream);
    return launch_enc_u<4, 5>(a, wire_bound, nt, cfg.max_blocks, stream);
}

}  // namespace netc_gpu
