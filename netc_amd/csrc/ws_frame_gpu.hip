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
// Two steps on the caller's stream:
//   1. wire offsets: wo[j] = sum over k < j of (header_len(k) + len(k)), a scan
//      over the frames (three small kernels, no scratch memory: the block sums
//      live in wo[] itself until the last kernel overwrites them);
//   2. the assembly kernel, output-driven: the wire buffer is walked in 16-byte
//      vectors aligned to the destination, chunk by chunk in grid-stride order
//      as in ws_mask_gpu.hip; a 64-entry frame table in VGPRs (wire start,
//      payload offset, key, header byte of 64 consecutive frames) places each
//      vector.  A vector inside one frame's payload is one unaligned 16-B load
//      of the payload, one XOR with the key rotated to its phase, one aligned
//      store; vectors holding a header or a frame edge are composed from the
//      header (built once per frame, wave-uniform) and the masked payload of
//      every frame they touch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpu_util.h"
#include "ws_mask_gpu.h"

namespace netc_gpu {

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));   // unaligned 16-B access

// extended-length bytes for a payload of len bytes (src/ws/common.c:63,71-82)
__device__ __forceinline__ uint32_t ext_len(uint64_t len) { return len < 126 ? 0u : (len < 65536 ? 2u : 8u); }

// ------------------------------------------------------------ wire offsets --

static constexpr int kScanThreads = 256;
static constexpr int kScanPer = 16;
static constexpr uint64_t kScanBlock = (uint64_t)kScanThreads * kScanPer;   // frames per block

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

// 1. per block: sum of extended-length bytes of its frames -> wo[block * kScanBlock]
__global__ __launch_bounds__(kScanThreads) void wire_block_sums(const uint64_t* off, uint64_t n, uint64_t* wo) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanBlock;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        const uint64_t j = base + (uint64_t)i * kScanThreads + threadIdx.x;
        if (j < n) s += ext_len(gptr(off)[j + 1] - gptr(off)[j]);
    }
    uint64_t total;
    (void)block_exclusive_scan(s, &total);
    if (threadIdx.x == 0) gptr(wo)[base] = total;
}

// 2. one block: exclusive scan of the nb block sums in place (stride kScanBlock)
__global__ __launch_bounds__(kScanThreads) void wire_scan_sums(uint64_t nb, uint64_t* wo) {
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nb; b0 += kScanThreads) {
        const uint64_t b = b0 + threadIdx.x;
        const uint64_t v = b < nb ? gptr(wo)[b * kScanBlock] : 0;
        uint64_t total;
        const uint64_t ex = block_exclusive_scan(v, &total);
        if (b < nb) gptr(wo)[b * kScanBlock] = carry + ex;
        carry += total;
    }
}

// 3. per block: wo[j] = (off[j] - off[0]) + (2 + 4 masked) j + (extended-length
//    bytes of frames < j); the block's last thread with frames also writes wo[n].
__global__ __launch_bounds__(kScanThreads) void wire_offsets(const uint64_t* off, uint64_t n, uint32_t fixed,
                                                             uint64_t* wo) {
    __shared__ uint64_t block_prefix;
    const uint64_t base = (uint64_t)blockIdx.x * kScanBlock;
    if (threadIdx.x == 0) block_prefix = gptr(wo)[base];
    __syncthreads();
    const uint64_t first = base + (uint64_t)threadIdx.x * kScanPer;   // this thread's kScanPer frames
    uint32_t e[kScanPer];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        const uint64_t j = first + i;
        e[i] = j < n ? ext_len(gptr(off)[j + 1] - gptr(off)[j]) : 0u;
        s += e[i];
    }
    uint64_t total;
    uint64_t run = block_prefix + block_exclusive_scan(s, &total);
    const uint64_t off0 = gptr(off)[0];
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        const uint64_t j = first + i;
        if (j <= n) gptr(wo)[j] = (gptr(off)[j] - off0) + (uint64_t)fixed * j + run;
        run += e[i];
    }
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
    uint64_t nwin;             // chunks covering the wire upper bound
    uint32_t masked;
};

// Frame table: lane l holds virtual frame kb + l.  W coordinates = wire byte + wmis.
struct EncTable {
    int64_t kb;
    uint64_t start;   // W start of the frame's header (virtual head: 0, past the end: inf)
    uint64_t poff;    // payload offset off[v] (clamped)
    uint32_t key;
    uint32_t b0;
    uint64_t last;    // start of entry 63 (uniform)
    bool tail;        // entry for frame n is in the table
};

__device__ __forceinline__ void enc_entry(const EncArgs& a, int64_t v, EncTable& t) {
    const int64_t n = (int64_t)a.n;
    const int64_t vo = v < 0 ? 0 : (v > n ? n : v);
    const int64_t vk = v < 0 ? 0 : (v >= n ? (n > 0 ? n - 1 : 0) : v);
    const uint64_t wo = gptr(a.wo)[vo];
    t.poff = gptr(a.off)[vo];
    const uint32_t key = a.masked ? gptr(a.keys)[vk] : 0u;
    const uint32_t b0 = a.b0 ? (uint32_t)gptr(a.b0)[vk] : 0x82u;
    t.start = v < 0 ? 0 : (v <= n ? wo + a.wmis : kInf);
    t.key = (v >= 0 && v < n) ? key : 0u;
    t.b0 = b0;
}

__device__ __forceinline__ void enc_table_load(const EncArgs& a, EncTable& t, int64_t kb, int lane) {
    t.kb = kb;
    enc_entry(a, kb + lane, t);
    t.tail = kb + (kWave - 1) >= (int64_t)a.n;
    t.last = readlane64(t.start, kWave - 1);
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
        const uint64_t val = valid ? gptr(a.wo)[idx] : 0;
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
        const uint64_t val = valid ? gptr(a.wo)[idx] : kInf;
        const uint64_t le = __ballot(valid && val <= q);
        const uint64_t gt = __ballot(valid && val > q);
        if (le) L = lo + (int64_t)(63 - __builtin_clzll(le)) * step;
        if (gt) H = lo + (int64_t)__builtin_ctzll(gt) * step;
    }
    return L;
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

// Wire vector of this lane for the span at A0 (general path: header bytes and any
// number of frame edges).  Frames are taken from the table from entry l0 on.
template <bool NT>
__device__ u32x4 compose_vec(const EncArgs& a, EncTable& t, int l0, uint64_t A0, uint64_t W, int lane) {
    const uint64_t Aend = A0 + kSpan;
    u32x4 out = {0, 0, 0, 0};
    int l = l0;
    for (;;) {
        if (l >= kWave - 1) {   // entry l needs entry l + 1: slide the table
            enc_table_load(a, t, t.kb + l, lane);
            l = 0;
        }
        const int64_t j = t.kb + l;
        if (j >= (int64_t)a.n) break;
        const uint64_t Ws = readlane64(t.start, l);
        if (Ws >= Aend) break;
        if (j < 0) {
            ++l;
            continue;
        }
        const uint64_t We = readlane64(t.start, l + 1);
        const uint64_t o0 = readlane64(t.poff, l), o1 = readlane64(t.poff, l + 1);
        const uint32_t key = readlane32(t.key, l), b0 = readlane32(t.b0, l);
        const uint64_t len = o1 - o0;
        const uint64_t pw = Ws + 2 + ext_len(len) + (a.masked ? 4 : 0);   // payload start (W)
        // header bytes [Ws, pw) of this vector
        const int64_t hlo = (int64_t)(Ws - W), hhi = (int64_t)(pw - W);
        if (hhi > 0 && hlo < 16) {
            uint64_t hl, hh;
            build_header(b0, len, a.masked != 0, key, hl, hh);
            const u32x4 sel = select_range(hlo, hhi);
            out = (out & ~sel) | (shift_bytes(hl, hh, (int)hlo) & sel);
        }
        // payload bytes [pw, We) of this vector
        const int64_t plo = (int64_t)(pw - W), phi = (int64_t)(We - W);
        if (phi > 0 && plo < 16 && phi > plo) {
            const int64_t s0 = (int64_t)o0 - plo;   // src offset of the vector's byte 0
            u32x4 v;
            if (s0 >= 0 && (uint64_t)s0 + 16 <= a.src_total) v = load_u<false>(a.src + s0);
            else v = load_guarded(a, s0, plo < 0 ? 0 : (int)plo, phi > 16 ? 16 : (int)phi);
            const uint32_t rk = rotr8(key, (uint64_t)(-plo));   // phase of byte 0: W - pw
            const u32x4 kv = {rk, rk, rk, rk};
            const u32x4 sel = select_range(plo, phi);
            out = (out & ~sel) | ((v ^ kv) & sel);
        }
        ++l;
    }
    return out;
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

template <int U, bool NT>
__global__ __launch_bounds__(256) void encode_frames_kernel(EncArgs a) {
    constexpr uint64_t kWin = kSpan * U;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wpb = blockDim.x / kWave;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + (threadIdx.x / kWave);
    const uint64_t wire_total = gptr(a.wo)[a.n];
    const uint64_t wlo = a.wmis, whi = a.wmis + wire_total;
    const uint64_t nwin = (whi + kWin - 1) / kWin;

    EncTable t;
    t.kb = -2;   // no table yet
    for (uint64_t c = wave; c < nwin; c += nwaves) {
        const uint64_t A = c * kWin;
        // table holding the frame that contains A
        bool ok = false;
        if (t.kb != -2) {
            const uint64_t m = __ballot(t.start <= A);
            ok = m != 0 && (t.tail || m != ~0ull);
        }
        if (!ok) enc_table_load(a, t, enc_locate(a, A, wire_total, lane), lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t A0 = A + (uint64_t)u * kSpan;
            if (A0 >= whi) break;
            const uint64_t Aend = A0 + kSpan;
            int l0 = __popcll(__ballot(t.start <= A0)) - 1;
            if (l0 >= kWave - 1 || (l0 > 0 && !t.tail && t.last < Aend)) {
                enc_table_load(a, t, t.kb + l0, lane);
                l0 = 0;
            }
            const uint64_t W = A0 + 16ull * (uint64_t)lane;
            const int64_t j0 = t.kb + l0;
            bool fast = false;
            uint64_t Ws = 0, We = 0, o0 = 0, pw = 0;
            uint32_t key = 0;
            if (j0 >= 0 && j0 < (int64_t)a.n && A0 >= wlo && Aend <= whi) {
                Ws = readlane64(t.start, l0);
                We = readlane64(t.start, l0 + 1);
                o0 = readlane64(t.poff, l0);
                const uint64_t o1 = readlane64(t.poff, l0 + 1);
                key = readlane32(t.key, l0);
                pw = Ws + 2 + ext_len(o1 - o0) + (a.masked ? 4 : 0);
                fast = pw <= A0 && Aend <= We;
            }
            u32x4 v;
            if (fast) {   // the whole span is payload of frame j0 (wave-uniform)
                const uint64_t s = o0 + (W - pw);
                const uint32_t rk = rotr8(key, A0 - pw);
                const u32x4 kv = {rk, rk, rk, rk};
                v = load_u<NT>(a.src + s) ^ kv;
            } else {
                v = compose_vec<NT>(a, t, l0, A0, W, lane);
            }
            store_wire<NT>(a, W, v, wlo, whi);
        }
    }
}

template <int U, bool NT>
static int enc_resident_blocks() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
    if (cache[dev] > 0) return cache[dev];
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, encode_frames_kernel<U, NT>, 256, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu <= 0 || cus <= 0)
        return 1024;
    cache[dev] = per_cu * cus;
    return cache[dev];
}

hipError_t launch_wire_offsets(const uint64_t* off, uint64_t n, bool masked, uint64_t* wo, hipStream_t stream) {
    if (n == 0) return hipMemsetAsync(wo, 0, sizeof(uint64_t), stream);
    // blocks cover frames 0 .. n inclusive: every block base is <= n, so wo[base]
    // can hold that block's sum, and some block writes wo[n]
    const uint64_t nb = n / kScanBlock + 1;
    if (nb > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wire_block_sums, dim3((unsigned)nb), dim3(kScanThreads), 0, stream, off, n, wo);
    hipLaunchKernelGGL(wire_scan_sums, dim3(1), dim3(kScanThreads), 0, stream, nb, wo);
    hipLaunchKernelGGL(wire_offsets, dim3((unsigned)nb), dim3(kScanThreads), 0, stream, off, n,
                       (uint32_t)(2 + (masked ? 4 : 0)), wo);
    return hipGetLastError();
}

hipError_t launch_encode_frames(uint8_t* wire, uint64_t wire_bound, const uint8_t* src, uint64_t src_total,
                                const uint64_t* off, const uint32_t* keys, const uint8_t* b0, uint64_t n, bool masked,
                                uint64_t* wo, hipStream_t stream, const LaunchCfg& cfg) {
    hipError_t e = launch_wire_offsets(off, n, masked, wo, stream);
    if (e != hipSuccess || n == 0) return e;
    constexpr int U = 4;
    EncArgs a;
    a.wmis = (uint64_t)(uintptr_t)wire & 15u;
    a.wire_base = wire - a.wmis;
    a.src = src;
    a.src_total = src_total;
    a.off = off;
    a.wo = wo;
    a.keys = masked ? keys : nullptr;
    a.b0 = b0;
    a.n = n;
    a.masked = masked ? 1u : 0u;
    a.nwin = (a.wmis + wire_bound + kSpan * U - 1) / (kSpan * U);
    const bool nt = cfg.flags < 0 || (cfg.flags & (kNtLoads | kNtStores));
    const uint64_t cap = (uint64_t)(cfg.max_blocks > 0 ? cfg.max_blocks
                                                       : (nt ? enc_resident_blocks<U, true>() : enc_resident_blocks<U, false>()));
    const uint64_t want = (a.nwin + 3) / 4;
    const int blocks = (int)(want < cap ? want : cap);
    if (blocks <= 0) return hipSuccess;
    if (nt) hipLaunchKernelGGL((encode_frames_kernel<U, true>), dim3(blocks), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((encode_frames_kernel<U, false>), dim3(blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace netc_gpu
