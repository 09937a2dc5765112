// MI355X (gfx950 / CDNA4) WebSocket payload masking — device kernels.
//
// Replaces the reference's scalar per-byte loops
//   src/ws/common.c:317-323  buffer_ptr[i] ^= masking_key[(received_length + i) % 4]   (unmask)
//   src/ws/common.c:104-107  payload[i]    ^= payload_masking_key[i % 4]              (mask)
// for a batch of independent frames resident in HBM.  Pure stream: 16 B read +
// 16 B written per 16 B of payload, no arithmetic worth a matrix core.
//
// Data layout (see DESIGN.md "Kernel"):
//   * the payload is walked in 16-byte vectors aligned to the *destination*
//     address; "P" below is a byte position measured from dst rounded down to
//     16, so vector v covers P in [16v, 16v+16).  mis = dst & 15.
//   * frames are [off[k], off[k+1]) in payload coordinates, i.e.
//     [off[k]+mis, off[k+1]+mis) in P coordinates.  Two virtual frames with a
//     zero key close the range: -1 = [0, off[0]+mis) and n = [off[n]+mis, inf).
//   * the batch is cut into chunks of U spans (a span = 64 vectors = 1 KiB, one
//     wave-instruction); wavefront w of W takes chunks w, w+W, w+2W, ... so the
//     resident wavefronts always stream one compact region of HBM.
//   * per chunk a wavefront holds a 64-entry "frame table" in registers: lane j
//     holds the start and key of virtual frame kb + j.  A span's frame is found
//     with one ballot; the (rare) frame boundaries inside a span are applied with
//     a wave-uniform loop; the table slides forward with one coalesced 768-byte
//     reload if a chunk runs past it.  The table for the NEXT chunk is loaded at a
//     guessed base while the current chunk is processed (exact for evenly sized
//     frames, within a few frames otherwise); a miss falls back to locate().
//   * the key stays in registers and is rotated per vector with v_alignbit
//     (rotr by 8*((P - frame_start) & 3)); it is the same for the 4 dwords of a
//     16-B vector, and the same for every lane of a span.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "gpu_util.h"
#include "ws_mask_gpu.h"

namespace netc_gpu {

// waves per SIMD the register budget is sized for, by U (KiB per chunk): two
// chunks of payload are live per wavefront (current + prefetched), 8 U VGPRs
__device__ constexpr int kMinWaves[9] = {8, 8, 4, 4, 4, 4, 4, 4, 2};


#ifdef NETC_MASK_STAMPS
__device__ uint64_t* g_stamps;   // diagnostic build only: 2 x u64 per wavefront
extern "C" int netc_gpu_debug_stamps(void* d_buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_buf, sizeof(d_buf));
}
// per-wave start / end wall clock (100 MHz), written by lane 0 when the wave leaves
// (tools/mask_timeline.py sizes the buffer for every window of the launch)
struct StampOnExit {
    uint64_t w, s0;
    __device__ ~StampOnExit() {
        if ((threadIdx.x & 63) == 0 && g_stamps) {
            g_stamps[2 * w] = s0;
            g_stamps[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
};
#define MASK_STAMP_SCOPE(w) StampOnExit stamp_guard{(w), __builtin_amdgcn_s_memrealtime()}
#else
#define MASK_STAMP_SCOPE(w) ((void)0)
#endif

struct Table {
    int64_t kb;       // virtual frame index held by lane 0
    uint64_t start;   // this lane's entry: start of frame kb + lane (P coords); kInf past entry e - 1
    uint32_t key;     // this lane's entry: packed key of frame kb + lane
    uint64_t last;    // start of frame kb + e - 1, the last entry held (uniform)
    bool tail;        // frame n (the open-ended pass-through frame) is in the table
    int e;            // entries held: 64, or fewer for a window's first probe (uniform)
};

// Frame k's offset / key.  Args: the caller's arrays.  ArgsScan (frames a
// netc_gpu_scan_frames call found, unmasked in place): virtual frame 2k is frame k's
// header (key 0: passed through), 2k + 1 its payload, read from the scan's header
// offsets, keys and the header bytes in the buffer itself -- no view array is built.
__device__ __forceinline__ uint64_t off_at(const Args& a, int64_t i) { return gptr(a.off)[i]; }
__device__ __forceinline__ uint32_t key_at(const Args& a, int64_t i) { return gptr(a.keys)[i]; }

struct ArgsScan : Args {
    const uint64_t* hdr;       // scan output: header offset of frame k
    const uint32_t* fkeys;     // scan output: packed key of frame k
    const uint64_t* result;    // scan result (frames found: result[0])
    uint64_t max_frames;       // frames the scan recorded at most
};

// header length of the frame whose header starts at p (the wire bytes are in the buffer)
__device__ __forceinline__ uint64_t header_len(const ArgsScan& a, uint64_t p) {
    const uint32_t second = gptr(a.src_base + a.mis)[p + 1];
    const uint32_t code = second & 0x7F;
    return 2 + (code == 126 ? 2 : (code == 127 ? 8 : 0)) + ((second & 0x80) ? 4 : 0);
}

__device__ __forceinline__ uint64_t off_at(const ArgsScan& a, int64_t i) {
    const int64_t nf = (int64_t)(a.n >> 1), k = i >> 1;
    if (k < nf) {
        const uint64_t p = gptr(a.hdr)[k];
        return (i & 1) ? p + header_len(a, p) : p;
    }
    if (nf == 0) return 0;
    // i == 2 nf: the end of the last frame's payload (its extended length read from the header)
    const uint64_t p = gptr(a.hdr)[nf - 1];
    const NETC_GLOBAL uint8_t* w = gptr(a.src_base + a.mis) + p;
    const uint32_t code = w[1] & 0x7F;
    uint64_t len = code;
    if (code >= 126) {
        len = 0;
        for (int j = 0; j < (code == 126 ? 2 : 8); ++j) len = len << 8 | w[2 + j];
    }
    return p + header_len(a, p) + len;
}

__device__ __forceinline__ uint32_t key_at(const ArgsScan& a, int64_t i) {
    return (i & 1) ? gptr(a.fkeys)[i >> 1] : 0u;
}

// start / key of virtual frame v in P coordinates.  Branch-free: both loads are
// always issued at clamped (valid) indices and the virtual-frame values are
// selected afterwards, so the loads stay straight-line code and the compiler can
// count them in vmcnt instead of draining every outstanding load (a load under a
// per-lane branch forces s_waitcnt vmcnt(0) at the next use).  With n == 0 the
// host points keys at the offsets array, so keys[0] is always readable.
template <class A>
__device__ __forceinline__ void frame_entry(const A& a, int64_t v, uint64_t& s, uint32_t& k) {
    const int64_t n = (int64_t)a.n;
    const int64_t vo = v < 0 ? 0 : (v > n ? n : v);
    const int64_t vk = v < 0 ? 0 : (v >= n ? (n > 0 ? n - 1 : 0) : v);
    const uint64_t off = off_at(a, vo);
    const uint32_t key = key_at(a, vk);
    s = v < 0 ? 0 : (v <= n ? off + a.mis : kInf);
    k = (v >= 0 && v < n) ? key : 0u;
}

// issue the table loads (frames kb .. kb+e-1, one per lane) without waiting for them.
// e < 64 (a window's first probe, sized to the frames the window can reach): lanes past
// e - 1 load entry e - 1 again -- the same cache lines, so the probe touches only the
// lines of its e entries, and no lane branches around a load (which would draw a
// vmcnt(0) wait behind the window's payload loads) -- and then hold kInf.
template <class A>
__device__ __forceinline__ void table_issue(const A& a, Table& t, int64_t kb, int lane, int e = kWave) {
    t.kb = kb;
    t.e = e;
    frame_entry(a, kb + (lane < e ? lane : e - 1), t.start, t.key);
    t.tail = kb + (e - 1) >= (int64_t)a.n;
}

// the table's loads have landed: entries past e - 1 become kInf (here, at the first use,
// not at the issue -- a select on a loaded value there would wait for the load)
__device__ __forceinline__ void table_finish(Table& t) {
    if (t.e < kWave && (int)__lane_id() >= t.e) t.start = kInf;
    t.last = readlane64(t.start, t.e - 1);
}

template <class A>
__device__ __forceinline__ void table_load(const A& a, Table& t, int64_t kb, int lane) {
    table_issue(a, t, kb, lane);
    table_finish(t);
}

// Does the table hold the frame containing P (entry 0 starts at or before P and a
// later entry starts after it, or the open-ended tail frame is in the table)?
__device__ __forceinline__ bool table_brackets(const Table& t, uint64_t P) {
    const uint64_t m = __ballot(t.start <= P);
    if (m == 0) return false;
    return t.tail || __popcll(m) < t.e;
}

// Table base for the chunk at P guessed from a frame known to start at s_known
// (index f_known) and the batch's mean frame density: frames are independent
// draws, so the guess error grows only with the square root of the frames in
// between; the window is biased forward so the chunk's later frames fit too.
template <class A>
__device__ __forceinline__ int64_t guess_base(const A& a, int64_t f_known, uint64_t s_known, uint64_t P,
                                              int64_t bias = 24) {
    if (P < a.mis) return -1;
    const double ahead = (double)(P - s_known) * a.density;
    int64_t g = f_known + (int64_t)ahead - bias;
    g = g < -1 ? -1 : g;
    return g > (int64_t)a.n ? (int64_t)a.n : g;
}

// Virtual frame index L whose start is <= P and such that the frame containing
// P is among L .. L+63, i.e. a valid base for the frame table (wave-uniform).
// Invariant of the search: off'[L] <= q (L = -1: the virtual head frame) and
// H > n or off[H] > q, so the containing frame is in [L, H - 1].
//   1. interpolation probe: frames are usually spread evenly over the batch, so
//      64 lanes probe a +-512-frame comb (stride 16) around q * n / total; when
//      it brackets q (always, for uniform frames) H - L <= 16 after ONE load;
//   2. otherwise 64-ary narrowing, one coalesced probe + one ballot per step.
// The caller's table load is the final (second) dependent load.
template <class A>
__device__ int64_t locate(const A& a, uint64_t P, int lane) {
    if (P < a.mis) return -1;
    const uint64_t q = P - a.mis;
    int64_t L = -1, H = (int64_t)a.n + 1;
    if (a.n > (uint64_t)kWave && a.total > 0) {
        constexpr int64_t kStride = 16;
        const double fg = (double)q * ((double)a.n / (double)a.total);
        int64_t g = (int64_t)fg;
        g = g > (int64_t)a.n ? (int64_t)a.n : g;
        const int64_t base = g - 31 * kStride;
        const int64_t idx = base + (int64_t)lane * kStride;
        const bool valid = idx >= 0 && idx <= (int64_t)a.n;
        const uint64_t val = valid ? off_at(a, idx) : 0;
        const uint64_t le = __ballot(valid && val <= q);   // probes at or before q
        const uint64_t gt = __ballot(valid && val > q);    // probes after q
        if (le) {
            const int j = 63 - __builtin_clzll(le);
            L = base + (int64_t)j * kStride;
        }
        if (gt) {
            const int j = __builtin_ctzll(gt);
            H = base + (int64_t)j * kStride;
        }
        // probes are sorted, so [L, H) is a valid bracket whenever both sides
        // were seen; an unseen side keeps its global bound (-1 / n + 1)
    }
    while (H - L > kWave) {
        const int64_t lo = L + 1;
        const int64_t step = (H - lo + kWave - 1) / kWave;   // probes lo, lo + step, ... cover [lo, H)
        const int64_t idx = lo + (int64_t)lane * step;
        const bool valid = idx < H;
        const uint64_t val = valid ? off_at(a, idx) : kInf;
        const uint64_t le = __ballot(valid && val <= q);
        const uint64_t gt = __ballot(valid && val > q);
        if (le) L = lo + (int64_t)(63 - __builtin_clzll(le)) * step;
        if (gt) H = lo + (int64_t)__builtin_ctzll(gt) * step;
    }
    return L;
}

// Mask for this lane's vector in the span starting at A0 (P coords, 16-aligned,
// lane's vector = A0 + 16 * lane).  Slides the table forward when needed.
template <class A>
__device__ __forceinline__ u32x4 span_mask(const A& a, Table& t, uint64_t A0, int lane) {
    const uint64_t Aend = A0 + kSpan;
    // invariant: entry 0 starts at or before A0.  Make the table cover the span.
    if (!t.tail && t.last < Aend) {   // a full table from the span's first frame on
        const uint64_t m = __ballot(t.start <= A0);
        const int j0 = __popcll(m) - 1;
        if (j0 > 0 || t.e < kWave) table_load(a, t, t.kb + j0, lane);
    }
    const uint64_t m0 = __ballot(t.start <= A0);
    const int j0 = __popcll(m0) - 1;
    const uint64_t s0 = readlane64(t.start, j0);
    const uint32_t rk0 = rotr8(readlane32(t.key, j0), A0 - s0);
    u32x4 mask = {rk0, rk0, rk0, rk0};
    // frame boundaries strictly inside (A0, Aend)
    uint64_t b = __ballot(t.start > A0 && t.start < Aend);
    const bool covered = t.tail || t.last >= Aend;
    if (b == 0 && covered) return mask;   // common case: one frame

    const uint64_t a_lane = A0 + 16ull * (uint64_t)lane;
    if (__popcll(b) > 2) {
        // Dense span (frames under ~340 B): per lane instead of per boundary.  The
        // frame holding the lane's first byte by a binary search of the table
        // (ds_bpermute), then the frames starting inside the lane's 16 bytes in turn
        // -- one for frames of 16 B or more; the loop runs as long as any lane has
        // another.  Every lane takes part in each ds_bpermute (the loop is uniform).
        // More than 63 frame starts in the span (frames under ~16 B): the table is
        // walked in 63-entry windows, the next window's load in flight while this
        // one is applied; a lane whose first byte lies before a window's entry 0
        // keeps what the earlier windows gave it (re-applying the shared entry is
        // idempotent), so the last window holding entries at or before the lane's
        // bytes decides, as one table covering the whole span would.
        u32x4 m = mask;   // the frame holding A0 (same rotation for every lane)
        for (;;) {
            const bool more = !(t.tail || t.last >= Aend);   // wave-uniform
            Table tn;
            if (more) table_issue(a, tn, t.kb + (t.e - 1), lane);
            int l = 0;
#pragma unroll
            for (int step = 32; step > 0; step >>= 1)
                if (bperm64(t.start, l + step) <= a_lane) l += step;
            const uint64_t sl = bperm64(t.start, l);
            const uint32_t rl = rotr8((uint32_t)__builtin_amdgcn_ds_bpermute(l << 2, (int)t.key), a_lane - sl);
            const bool has = sl <= a_lane;   // false: entry 0 starts after the lane's first byte
            if (has) m = u32x4{rl, rl, rl, rl};
            for (int j = has ? l + 1 : 0;; ++j) {
                const int c = j < kWave ? j : kWave - 1;
                const uint64_t sj = bperm64(t.start, c);
                const uint32_t kj = (uint32_t)__builtin_amdgcn_ds_bpermute(c << 2, (int)t.key);
                const bool in = j < kWave && sj < a_lane + 16;
                if (in) {
                    const uint32_t rj = rotr8(kj, a_lane - sj);
                    const u32x4 sel = select_from((int64_t)(sj - a_lane));
                    const u32x4 kv = {rj, rj, rj, rj};
                    m = (m & ~sel) | (kv & sel);
                }
                if (!__ballot(in)) break;
            }
            if (!more) break;
            t = tn;
            table_finish(t);
        }
        return m;
    }
    for (;;) {
        while (b) {
            const int j = __builtin_ctzll(b);
            b &= b - 1;
            const uint64_t sj = readlane64(t.start, j);
            const uint32_t rkj = rotr8(readlane32(t.key, j), A0 - sj);
            const u32x4 sel = select_from((int64_t)(sj - a_lane));
            const u32x4 kv = {rkj, rkj, rkj, rkj};
            mask = (mask & ~sel) | (kv & sel);
        }
        if (t.tail || t.last >= Aend) break;
        // more than 63 boundaries in one span: advance the table past the last
        // applied entry (re-applying entry 0 again is idempotent) and continue
        table_load(a, t, t.kb + (t.e - 1), lane);
        b = __ballot(t.start > A0 && t.start < Aend);
    }
    return mask;
}

template <bool SRC_ALIGNED, bool NT, class A>
__device__ __forceinline__ u32x4 load_vec(const A& a, uint64_t P) {
    if constexpr (SRC_ALIGNED) {
        const NETC_GLOBAL u32x4* p = gptr(reinterpret_cast<const u32x4*>(a.src_base + P));
        if constexpr (NT) return __builtin_nontemporal_load(p);
        return *p;
    } else {
        // src and dst differ mod 16: one unaligned 16-B load (global_load_dwordx4 takes
        // any byte address on gfx950; it was 16 global_load_ubyte per lane in round 1)
        typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
        const NETC_GLOBAL u32x4u* p = (const NETC_GLOBAL u32x4u*)gptr(a.src_base + P);
        if constexpr (NT) return __builtin_nontemporal_load(p);
        return *p;
    }
}

// src misaligned against dst by sh = src_base & 15 (uniform over the batch): a lane loads
// the ALIGNED 16 bytes holding the start of its source vector (P - sh from src_base), and
// its vector is bytes [sh, sh + 16) of that block and the next lane's (lane 63: the block
// after the span, one broadcast load).  Every aligned block read holds at least one byte
// of the vector, so no access leaves the buffer's pages.  (16 global_load_ubyte per lane
// in round 1; an unaligned global_load_dwordx4 since: 85 % of the aligned rate at C2.)
template <bool NT, class A>
__device__ __forceinline__ u32x4 load_block(const A& a, uint64_t off) {   // a.src_base + off is 16-aligned
    const NETC_GLOBAL u32x4* p = gptr(reinterpret_cast<const u32x4*>(a.src_base + off));
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// bytes [sh, sh + 16) of (b, the next lane's block; lane 63: n63) -- every lane executes it.
// Only the next block's dwords the shift reaches are fetched across lanes (1 + sh / 4).
__device__ __forceinline__ u32x4 shift_in(u32x4 b, u32x4 n63, uint32_t sh, int lane) {
    auto nb = [&](int k) {
        const uint32_t x = (uint32_t)__shfl_down((int)b[k], 1, kWave);
        return lane == kWave - 1 ? n63[k] : x;
    };
    const uint32_t r = sh & 3;
    u32x4 o;
    switch (sh >> 2) {   // uniform: constant register indices in each case
        case 0: {
            const uint32_t n0 = nb(0);
            o = u32x4{__builtin_amdgcn_alignbyte(b[1], b[0], r), __builtin_amdgcn_alignbyte(b[2], b[1], r),
                      __builtin_amdgcn_alignbyte(b[3], b[2], r), __builtin_amdgcn_alignbyte(n0, b[3], r)};
            break;
        }
        case 1: {
            const uint32_t n0 = nb(0), n1 = nb(1);
            o = u32x4{__builtin_amdgcn_alignbyte(b[2], b[1], r), __builtin_amdgcn_alignbyte(b[3], b[2], r),
                      __builtin_amdgcn_alignbyte(n0, b[3], r), __builtin_amdgcn_alignbyte(n1, n0, r)};
            break;
        }
        case 2: {
            const uint32_t n0 = nb(0), n1 = nb(1), n2 = nb(2);
            o = u32x4{__builtin_amdgcn_alignbyte(b[3], b[2], r), __builtin_amdgcn_alignbyte(n0, b[3], r),
                      __builtin_amdgcn_alignbyte(n1, n0, r), __builtin_amdgcn_alignbyte(n2, n1, r)};
            break;
        }
        default: {
            const uint32_t n0 = nb(0), n1 = nb(1), n2 = nb(2), n3 = nb(3);
            o = u32x4{__builtin_amdgcn_alignbyte(n0, b[3], r), __builtin_amdgcn_alignbyte(n1, n0, r),
                      __builtin_amdgcn_alignbyte(n2, n1, r), __builtin_amdgcn_alignbyte(n3, n2, r)};
            break;
        }
    }
    return o;
}

// ---------------------------------------------------------------------------
// Line-aligned source (one-window-per-wave walk, src misaligned against dst).
// A wave's 1 KiB span read at a 16-B but not 128-B aligned address touches 9 lines,
// not 8; a plain float4 copy from such a source runs 3.5 % slower
// (profiles/r02j_probe_lineoff.jsonl), and round 2's form -- aligned 16-B blocks at
// P - sh plus a one-lane load of the block after each span -- touched 10 lines per
// span.  Here a window of M spans loads its source as M whole-line spans from the
// line holding its first byte (c[0..M-1], 8 lines each) plus the <= 8 blocks of the
// line after them (c[M], one line), and each output vector is assembled across lanes:
// span m's lane i takes bytes [o + 16 i, o + 16 i + 16) of c[m]:c[m+1], o = the source
// line offset, i.e. blocks j = i + o/16 and j + 1 (from c[m+1] once j >= 64), shifted
// by o & 15 bytes.  The permutes (ds_bpermute) of each c[m] are shared by spans m - 1
// and m.  Every line read holds a byte of the window's source, so no access leaves the
// source's pages.
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t lane_pick(int idx4, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(idx4, (int)v);
}

// bytes [4 D + r, 4 D + r + 16) of the 32 bytes X:Y
template <int D>
__device__ __forceinline__ u32x4 join_shift(u32x4 X, u32x4 Y, uint32_t r) {
    uint32_t w[8] = {X[0], X[1], X[2], X[3], Y[0], Y[1], Y[2], Y[3]};
    return u32x4{__builtin_amdgcn_alignbyte(w[D + 1], w[D], r), __builtin_amdgcn_alignbyte(w[D + 2], w[D + 1], r),
                 __builtin_amdgcn_alignbyte(w[D + 3], w[D + 2], r), __builtin_amdgcn_alignbyte(w[D + 4], w[D + 3], r)};
}

// the source vectors of the window's M spans, from c[0..M] (see above); o = line offset
template <int M, int D>
__device__ __forceinline__ void shift_window(const u32x4 (&c)[M + 1], u32x4 (&v)[M], uint32_t o, int lane) {
    const uint32_t q = o >> 4, r = o & 3;
    const int j0 = (int)(((uint32_t)lane + q) & 63u) * 4, j1 = (int)(((uint32_t)lane + q + 1) & 63u) * 4;
    const bool lo0 = (uint32_t)lane + q < 64u, lo1 = (uint32_t)lane + q + 1 < 64u;
    u32x4 px[M + 1], py[M + 1];
#pragma unroll
    for (int m = 0; m <= M; ++m) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // X needs dwords D..3, Y dwords 0..D
            px[m][k] = k >= D ? lane_pick(j0, c[m][k]) : 0u;
            py[m][k] = k <= D ? lane_pick(j1, c[m][k]) : 0u;
        }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const u32x4 X = lo0 ? px[m] : px[m + 1];
        const u32x4 Y = lo1 ? py[m] : py[m + 1];
        v[m] = join_shift<D>(X, Y, r);
    }
}

template <bool NT>
__device__ __forceinline__ u32x4 load_line_block(const uint8_t* p) {   // p 16-aligned
    const NETC_GLOBAL u32x4* g = gptr(reinterpret_cast<const u32x4*>(p));
    if constexpr (NT) return __builtin_nontemporal_load(g);
    return *g;
}

template <bool NT, class A>
__device__ __forceinline__ void store_vec(const A& a, uint64_t P, u32x4 v) {
    NETC_GLOBAL u32x4* p = gptr(reinterpret_cast<u32x4*>(a.dst_base + P));
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Partial vector at either end of the buffer: byte-granular, only bytes in
// P in [mis, mis + total) are read or written.
template <class A>
__device__ __forceinline__ void edge_vec(const A& a, uint64_t P, u32x4 mask) {
    const uint64_t lo = a.mis, hi = a.mis + a.total;
#pragma unroll
    for (int bi = 0; bi < 16; ++bi) {
        const uint64_t p = P + bi;
        if (p >= lo && p < hi) {
            const uint8_t mb = (uint8_t)(mask[bi >> 2] >> (8 * (bi & 3)));
            gptr(a.dst_base)[p] = gptr(a.src_base)[p] ^ mb;
        }
    }
}

// A chunk that holds one of the two partial 16-B vectors at the ends of an
// unaligned buffer (at most three chunks per batch): per-vector range checks,
// a fresh frame search, no prefetch.
// ------------------------------------------------------ UTF-8 validation --
// RFC 3629 by the three-lookup rule (Keiser & Lemire, "Validating UTF-8 in less than one
// instruction per byte", 2021): for each byte, the AND of three 16-entry lookups -- the
// previous byte's high nibble, its low nibble, the byte's own high nibble -- flags every
// error a two-byte window shows (too short, too long, overlong, surrogate, > U+10FFFF, two
// continuations); that bit (TWO_CONTS, bit 7) is XORed with "a lead two or three bytes back
// asks for a continuation here".  A message is valid exactly when no byte is flagged and it
// does not end inside a sequence.  Four bytes at a time in a dword (SWAR): a lookup is one
// v_perm_b32 over an 8-entry byte table (the high-nibble tables are constant below 0x80, so
// 8 entries and a select on bit 7 do; the low-nibble table takes two), the previous bytes
// come by v_alignbyte_b32 from the previous dword, whose own lookups are carried: about 25
// VALU operations per dword (the round-2 rule took about 45).  tools/utf8_swar_check.py:
// this formula == the scalar rule (utf8_rule, phase B) at every position over every 4-byte
// context of 31 boundary bytes, and rule + end check == CPython's strict decoder over every
// string of up to 4 bytes from 27 of them.
constexpr uint32_t kB1H_HI = 0x49150121u, kB1H_LO = 0x80808080u;   // prev byte, high nibble 8..F
constexpr uint32_t kB2H_HI = 0x01010101u, kB2H_LO = 0xBABAAEE6u;   // this byte, high nibble 8..F
constexpr uint32_t kCLS_HI = 0xC0800000u;                          // high nibble E: 0x80, F: 0xC0
constexpr uint32_t kB1L_0H = 0xCBCBCB8Bu, kB1L_0L = 0x8383A3E7u;   // prev byte, low nibble 0..7
constexpr uint32_t kB1L_1H = 0xCBCBDBCBu, kB1L_1L = 0xCBCBCBCBu;   // prev byte, low nibble 8..F
constexpr uint32_t kSignSel = 0x090B080Au;   // v_perm_b32: byte i <- bit 7 of byte i of S1 (S0 = S1 << 8)

// 0xFF in each byte of v whose bit 7 is set (v_perm_b32's sign selectors: bits 15 / 31 of
// its two sources, here v << 8 and v)
__device__ __forceinline__ uint32_t sign_bytes(uint32_t v) { return __builtin_amdgcn_perm(v << 8, v, kSignSel); }

struct Utf8Carry {
    uint32_t x, b1h, cls;   // the previous dword, its byte_1_high lookup, its lead class (>= E0 / >= F0)
};

__device__ __forceinline__ Utf8Carry utf8_carry(uint32_t prev) {
    const uint32_t m = sign_bytes(prev), h = (prev >> 4) & 0x07070707u;
    return {prev, (m & __builtin_amdgcn_perm(kB1H_HI, kB1H_LO, h)) | (~m & 0x02020202u),
            m & __builtin_amdgcn_perm(kCLS_HI, 0u, h)};
}

// nonzero in each byte of x the rule flags; c: the dword before x (updated to x)
__device__ __forceinline__ uint32_t utf8_err_word(uint32_t x, Utf8Carry& c) {
    const uint32_t mx = sign_bytes(x);                    // x >= 0x80
    const uint32_t hx = (x >> 4) & 0x07070707u;           // high nibble & 7 (a perm index)
    const uint32_t b1hx = (mx & __builtin_amdgcn_perm(kB1H_HI, kB1H_LO, hx)) | (~mx & 0x02020202u);
    const uint32_t b2h = (mx & __builtin_amdgcn_perm(kB2H_HI, kB2H_LO, hx)) | (~mx & 0x01010101u);
    const uint32_t cls = mx & __builtin_amdgcn_perm(kCLS_HI, 0u, hx);
    const uint32_t p1 = __builtin_amdgcn_alignbyte(x, c.x, 3);          // the byte before each byte
    const uint32_t b1h = __builtin_amdgcn_alignbyte(b1hx, c.b1h, 3);
    const uint32_t l1 = p1 & 0x07070707u;
    const uint32_t m3 = __builtin_amdgcn_perm(p1 << 12, p1 << 4, kSignSel);   // bit 3 of each p1 byte
    const uint32_t b1l = (m3 & __builtin_amdgcn_perm(kB1L_1H, kB1L_1L, l1)) |
                         (~m3 & __builtin_amdgcn_perm(kB1L_0H, kB1L_0L, l1));
    // a lead >= E0 two bytes back, or >= F0 three bytes back: this byte must continue it
    const uint32_t must =
        (__builtin_amdgcn_alignbyte(cls, c.cls, 2) | (__builtin_amdgcn_alignbyte(cls, c.cls, 1) << 1)) & 0x80808080u;
    c = {x, b1hx, cls};
    return (b1h & b1l & b2h) ^ must;
}

// bit 7 of each byte of e set where the byte is nonzero (the rare error path)
__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t e) {
    return (((e & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | e) & 0x80808080u;
}

// The frame holding position P (P coordinates), or -1: a binary search over the
// offsets array (the UTF-8 check's rare path).
__device__ int64_t frame_of(const Args& a, uint64_t P) {
    if (P < a.mis || a.n == 0) return -1;
    const uint64_t q = P - a.mis;
    const NETC_GLOBAL uint64_t* off = gptr(a.off);
    if (off[0] > q) return -1;
    uint64_t lo = 0, hi = a.n;   // off[lo] <= q
    while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (off[mid] <= q) lo = mid;
        else hi = mid;
    }
    return q < off[lo + 1] ? (int64_t)lo : -1;
}

// Phase A of the TEXT check, per span: flag the frames holding a byte that breaks
// the local rules.  out = this lane's unmasked 16 bytes, prevd = the 4 bytes before
// them (from the neighbouring lane / the previous span of the chunk).  Skipped here:
// the first 3 bytes of every frame (their rule reaches into the previous frame of
// the message; utf8_messages() checks them), bytes in no frame, and, with seam set
// (a chunk's first span), the chunk's first 3 bytes: the bytes before them belong to
// another wavefront's chunk, which in place may already hold unmasked or still
// masked bytes -- utf8_messages() checks them once the whole batch is unmasked.
// Errors are rare: their frame lookup is a slow path.
__device__ __forceinline__ void validate_span(const Args& a, const Table& t, uint64_t A0, u32x4 out, uint32_t& sc,
                                              bool seam, int lane) {
    const uint64_t W = A0 + 16ull * (uint64_t)lane;
    // the 4 bytes before the lane's (lane 0: the previous span's last 4, or 0 at a window start):
    // one DPP move, wave_shr:1 -- lane 0 keeps sc (an LDS permute here put a ds_bpermute round
    // trip on every span's dependency chain)
    const uint32_t prevd = (uint32_t)__builtin_amdgcn_update_dpp((int)sc, (int)out[3], 0x138, 0xF, 0xF, false);
    sc = (uint32_t)__builtin_amdgcn_readlane((int)out[3], kWave - 1);
    u32x4 e;
    // all ASCII across the wave, the 4 bytes before each lane's included (the common case
    // for text): nothing to check
    if (!__ballot(((out[0] | out[1] | out[2] | out[3] | prevd) & 0x80808080u) != 0)) return;
    Utf8Carry c = utf8_carry(prevd);
    e[0] = utf8_err_word(out[0], c);
    e[1] = utf8_err_word(out[1], c);
    e[2] = utf8_err_word(out[2], c);
    e[3] = utf8_err_word(out[3], c);
    if (seam && lane == 0) e[0] &= ~0x00FFFFFFu;
    if (!__ballot((e[0] | e[1] | e[2] | e[3]) != 0)) return;
    // one bit per broken byte of the lane's vector
    uint32_t bits = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t m = (nonzero_bytes(e[w]) >> 7) & 0x01010101u;
        bits |= ((m | m >> 7 | m >> 14 | m >> 21) & 0xFu) << (4 * w);
    }
    if (readlane64(t.start, 0) > A0) {
        // more than 63 frames start inside this span, so the table holds only its last
        // ones (span_mask slid it): each broken byte's frame from the offsets array
        while (bits) {
            const int k = __builtin_ctz(bits);
            bits &= bits - 1;
            const int64_t f = frame_of(a, W + (uint64_t)k);
            if (f >= 0 && W + (uint64_t)k >= gptr(a.off)[f] + a.mis + 3) a.verr[f] = a.vtag;
        }
        return;
    }
    // drop bytes within 3 of a frame start: the span's first frame (if it starts
    // less than 3 bytes before A0) and every frame starting inside the span
    const uint64_t Aend = A0 + kSpan;
    const int l0 = __popcll(__ballot(t.start <= A0)) - 1;
    const uint64_t s0 = readlane64(t.start, l0);
    u32x4 drop = {0, 0, 0, 0};
    if (s0 + 3 > A0) drop = select_from((int64_t)(s0 - W)) & ~select_from((int64_t)(s0 + 3 - W));
    uint64_t b = __ballot(t.start > A0 && t.start < Aend);
    while (b) {
        const int j = __builtin_ctzll(b);
        b &= b - 1;
        const uint64_t sj = readlane64(t.start, j);
        drop |= select_from((int64_t)(sj - W)) & ~select_from((int64_t)(sj + 3 - W));
    }
    uint32_t dbits = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t m = (drop[w] >> 7) & 0x01010101u;
        dbits |= ((m | m >> 7 | m >> 14 | m >> 21) & 0xFu) << (4 * w);
    }
    bits &= ~dbits;
    // The frame of a broken byte p: the last table entry starting at or before it,
    // by a binary search over the 64 entries (ds_bpermute: each lane reads the entry
    // its own search is at; every lane takes part, so the loop is wave-uniform).
    // The lane's bytes before the next frame start are then done: one search per
    // frame touched.  Entry 0 starts at or before A0 <= p (checked above).
    while (__ballot(bits != 0)) {
        const uint64_t p = W + (uint64_t)(bits ? __builtin_ctz(bits) : 0);
        int idx = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
            if (bperm64(t.start, idx + step) <= p) idx += step;
        const uint64_t next = bperm64(t.start, idx < kWave - 1 ? idx + 1 : idx);
        if (bits) {
            const int64_t f = t.kb + idx;
            if (f >= 0 && f < (int64_t)a.n) a.verr[f] = a.vtag;
            // entry 63 is the last: the table covers the span (span_mask), so no later frame starts here
            const int64_t keep = idx < kWave - 1 ? (int64_t)(next - W) : 16;
            bits &= keep >= 16 ? 0u : (keep <= 0 ? ~0u : (~0u << keep));
        }
    }
}

// VAL, out of place (seam_src): the 4 bytes before window start A (P coordinates, A a multiple
// of 4 KiB, so the dword is aligned when src is) unmasked from src, which no wavefront writes,
// with the key of the frame holding A at its phase there.  When that frame starts less than 4
// bytes before A, the bytes before its start come out wrong -- they only feed the rule for the
// frame's first 3 bytes, which validate_span drops (utf8_messages checks them).  The caller's
// table holds the frame containing A (entry 0 starts at or before A).
template <bool SRC_ALIGNED>
__device__ __forceinline__ uint32_t seam_raw(const Args& a, uint64_t A) {   // issued with the window's loads
    if constexpr (SRC_ALIGNED) {
        return *(const NETC_GLOBAL uint32_t*)(a.src_base + A - 4);
    } else {
        typedef uint32_t u32u __attribute__((aligned(1)));
        return *(const NETC_GLOBAL u32u*)(a.src_base + A - 4);
    }
}
__device__ __forceinline__ uint32_t seam_unmask(const Table& t, uint64_t A, uint32_t raw) {   // once t is resolved
    const int j0 = __popcll(__ballot(t.start <= A)) - 1;
    const uint64_t s0 = readlane64(t.start, j0);
    return raw ^ rotr8(readlane32(t.key, j0), A - 4 - s0);
}
template <bool SRC_ALIGNED>
__device__ __forceinline__ uint32_t seam_carry(const Args& a, const Table& t, uint64_t A) {
    return seam_unmask(t, A, seam_raw<SRC_ALIGNED>(a, A));
}
__device__ __forceinline__ bool own_seam(const Args& a, uint64_t A) { return a.seam_src && A >= a.mis + 4; }

template <class A>
__device__ __forceinline__ int64_t clamp_base(const A& a, int64_t g) {
    g = g < -1 ? -1 : g;
    return g > (int64_t)a.n ? (int64_t)a.n : g;
}

// make t (issued at a guessed base) hold the frame containing A
template <class AT>
__device__ __forceinline__ void np_resolve(const AT& a, Table& t, uint64_t A, int lane) {
    table_finish(t);
#pragma unroll 1
    for (int step = 0; step < 2; ++step) {
        const uint64_t m = __ballot(t.start <= A);
        if (m != 0 && (t.tail || __popcll(m) < t.e)) return;   // brackets A
        int64_t g;
        if (m == 0) {   // every entry starts after A: step back by the distance from entry 0
            const uint64_t s0 = readlane64(t.start, 0);
            g = t.kb - (int64_t)((double)(s0 - A) * a.density) - 40;
        } else {        // every entry starts at or before A: step on from entry 63
            g = t.kb + (t.e - 1) + (int64_t)((double)(A - t.last) * a.density) - 24;
        }
        table_load(a, t, clamp_base(a, g), lane);
    }
    if (!table_brackets(t, A)) table_load(a, t, locate(a, A, lane), lane);
}

template <int U, bool SRC_ALIGNED, bool NT, bool VAL, class AT>
__device__ __forceinline__ void edge_chunk(const AT& a, uint64_t A, int lane, uint32_t& carry, bool first) {
    const uint64_t full_lo = a.mis ? 16 : 0;
    const uint64_t full_hi = (a.mis + a.total) & ~15ull;
    const uint64_t vec_end = (a.mis + a.total + 15) & ~15ull;
    u32x4 d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t P = A + (uint64_t)u * kSpan + 16ull * lane;
        if (P >= full_lo && P < full_hi) d[u] = load_vec<SRC_ALIGNED, NT>(a, P);
    }
    Table t;
    table_load(a, t, locate(a, A, lane), lane);
    // VAL: carry = the previous span's last 4 unmasked bytes, across the steps of a window
    // (first: this is the window's first step; its first 3 bytes are left to utf8_messages
    // unless the window checks its own seam)
    bool seam = first;
    if constexpr (VAL) {
        if constexpr (std::is_same<AT, Args>::value) {
            if (first && own_seam(a, A)) {   // wave-uniform
                carry = seam_carry<SRC_ALIGNED>(a, t, A);
                seam = false;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t A0 = A + (uint64_t)u * kSpan;
        if (A0 >= vec_end) break;                                   // wave-uniform
        const u32x4 m = span_mask(a, t, A0, lane);
        const uint64_t P = A0 + 16ull * lane;
        u32x4 out = {0, 0, 0, 0};   // VAL: the unmasked vector, bytes outside the buffer 0
        if constexpr (VAL) {
            // read before the store below: in place, the store overwrites these bytes
            if (P >= full_lo && P < full_hi) {
                out = d[u] ^ m;
            } else {
                const uint64_t lo = a.mis, hi = a.mis + a.total;
#pragma unroll
                for (int bi = 0; bi < 16; ++bi)
                    if (P + bi >= lo && P + bi < hi)
                        out[bi >> 2] |= (uint32_t)(gptr(a.src_base)[P + bi] ^ (uint8_t)(m[bi >> 2] >> (8 * (bi & 3))))
                                        << (8 * (bi & 3));
            }
        }
        if (P >= full_lo && P < full_hi) store_vec<NT>(a, P, d[u] ^ m);
        else if (P < vec_end) edge_vec(a, P, m);
        if constexpr (VAL) {
            validate_span(a, t, A0, out, carry, seam && u == 0, lane);
        }
    }
}

// Chunk = U spans (U KiB).  Wavefront w of W takes chunks w, w+W, w+2W, ...: at
// any moment the resident wavefronts stream one compact region of HBM (the
// order a grid-stride copy has), 10-14 % faster than each wavefront walking its
// own contiguous share (tools/order_probe.py).  Giving each XCD (blocks
// b % 8 == x) its own contiguous eighth of the chunks -- so its L2 would fetch
// only an eighth of the frame descriptors -- measured 7 % slower.
//
// Software pipeline per wavefront: the NEXT chunk's payload loads and its frame
// table load are in flight while the current chunk is masked and stored.  The
// interior chunks (every vector full) run a straight-line body: unconditional
// loads / stores, the prefetch issued every trip (the last chunk is peeled), so
// the compiler waits with counted vmcnt(N) and the prefetch stays in flight.  The
// table base of the next chunk is guessed from the frame known to hold this one
// (exact for evenly sized frames); a miss falls back to locate().  The <= 3
// partial chunks at the buffer ends go through edge_chunk().
template <int U, bool SRC_ALIGNED, bool NT, bool VAL = false>
__global__ __launch_bounds__(256, kMinWaves[U]) void mask_frames_kernel(Args a) {
    constexpr uint64_t kWin = kSpan * U;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wpb = blockDim.x / kWave;                     // wavefronts per block
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    if (a.n_dev) {   // frame count produced on the device by an earlier kernel (scan -> unmask)
        a.n = *gptr(a.n_dev);
        a.density = a.total ? (double)a.n / (double)a.total : 0.0;
    }
    MASK_STAMP_SCOPE(wave);   // diagnostic build only (tools/)

    // interior chunks [ci_lo, ci_hi): every 16-B vector inside the buffer
    const uint64_t full_hi = (a.mis + a.total) & ~15ull;
    const uint64_t ci_lo = a.mis ? 1 : 0;
    uint64_t ci_hi = full_hi / kWin;
    if (ci_hi < ci_lo) ci_hi = ci_lo;
    // edge chunks: chunk 0 when the buffer start is unaligned, and [ci_hi, nwin)
    uint32_t ec = 0;
    if (a.mis && wave == 0) edge_chunk<U, SRC_ALIGNED, NT, VAL>(a, 0, lane, ec, true);
    for (uint64_t e = ci_hi; e < a.nwin; ++e)
        if (e % nwaves == (wave + 1) % nwaves) edge_chunk<U, SRC_ALIGNED, NT, VAL>(a, e * kWin, lane, ec, true);

    uint64_t c = ci_lo + wave;
    if (c >= ci_hi) return;

    auto load_window = [&](u32x4 (&dst)[U], uint64_t base) {
#pragma unroll
        for (int u = 0; u < U; ++u) dst[u] = load_vec<SRC_ALIGNED, NT>(a, base + (uint64_t)u * kSpan + 16ull * lane);
    };
    auto process = [&](const u32x4 (&src)[U], Table& t, uint64_t base) {
        uint32_t carry = 0;   // the previous span's last 4 unmasked bytes (VAL)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t A0 = base + (uint64_t)u * kSpan;
            const u32x4 m = span_mask(a, t, A0, lane);
            const u32x4 out = src[u] ^ m;
            store_vec<NT>(a, A0 + 16ull * lane, out);
            if constexpr (VAL) {
                validate_span(a, t, A0, out, carry, u == 0, lane);
            }
        }
    };
    // make t hold the frame containing A (its probe was issued a chunk ago)
    auto resolve = [&](Table& t, uint64_t A, int64_t& f0, uint64_t& s0) {
        table_finish(t);
        if (!table_brackets(t, A)) table_load(a, t, locate(a, A, lane), lane);
        const int j0 = __popcll(__ballot(t.start <= A)) - 1;
        f0 = t.kb + j0;
        s0 = readlane64(t.start, j0);
    };

    u32x4 d[U];
    uint64_t A = c * kWin;
    load_window(d, A);
    Table t;
    table_issue(a, t, guess_base(a, 0, a.mis, A), lane);   // global guess: frame 0 starts near P = mis

    for (uint64_t cn = c + nwaves; cn < ci_hi; cn += nwaves) {
        int64_t f0;
        uint64_t s0;
        resolve(t, A, f0, s0);
        const uint64_t An = cn * kWin;
        u32x4 dn[U];
        load_window(dn, An);
        Table tn;
        table_issue(a, tn, guess_base(a, f0, s0, An), lane);
        process(d, t, A);
        A = An;
        t = tn;
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = dn[u];
    }
    int64_t f0;
    uint64_t s0;
    resolve(t, A, f0, s0);
    process(d, t, A);
}

// ---------------------------------------------------------------------------
// The default walk: one window of U x K KiB per wavefront, a grid covering the
// batch (no persistent loop).  The dispatcher hands the next workgroup to a CU as
// soon as one retires, and that sustains more of the HBM rate than any persistent
// grid-stride walk measured on MI355X: a frame-free XOR stream over 1 GiB ran at
// 6.45-6.58 TB/s this way and at <= 5.95 TB/s as one resident round striding over
// the chunks (tools/ceiling_sweep.py).
//
// Per wavefront: the window's payload loads are issued first (U vectors per lane);
// the frame-table lookup runs while they are in flight.  Its loads hit L2 / MALL
// almost always (neighbouring wavefronts read the same descriptor lines), so the
// lookup hides under the payload's HBM latency:
//   1. a 64-entry table at the base the batch's mean density predicts (exact for
//      evenly sized frames: configs 2, 3, 5);
//   2. on a miss, at most two interpolation steps from the window's own edge
//      entries (the distance left, times the density: for independent random
//      sizes the error shrinks from ~sqrt(frames before) to ~sqrt(frames skipped));
//   3. then locate() (comb + 64-ary narrowing), which always converges.
// K > 1: the window's K steps of U KiB run one after another (load, mask, store),
// the table carried across them.
// ---------------------------------------------------------------------------

// the frame count when it is produced on the device by an earlier kernel (scan -> unmask)
__device__ __forceinline__ void init_frames(Args& a) {
    if (a.n_dev) {
        a.n = *gptr(a.n_dev);
        a.density = a.total ? (double)a.n / (double)a.total : 0.0;
    }
}
__device__ __forceinline__ void init_frames(ArgsScan& a) {
    const uint64_t f = *gptr(a.result);
    a.n = 2 * (f < a.max_frames ? f : a.max_frames);   // header + payload per frame
    a.density = a.total ? (double)a.n / (double)a.total : 0.0;
}

// A window's first table probe: its base from the batch's mean density, biased back by
// a.probe_bias frames, holding a.probe_e entries.  Both come from the host (make_args),
// so the probe is straight-line code with kernel-argument (scalar) parameters -- a
// branch here on the density made the compiler wait (vmcnt(0)) for the window's payload
// loads before issuing the table's: +7 % at config 2, +2.5 % at config 4.
template <class AT>
__device__ __forceinline__ void first_probe(const AT& a, Table& t, uint64_t A, int lane) {
    table_issue(a, t, guess_base(a, 0, a.mis, A, a.probe_bias), lane, a.probe_e);
}

template <int U, int K, bool SRC_ALIGNED, bool NT, bool VAL = false, class AT = Args>
__global__ __launch_bounds__(256, (VAL && K == 1) ? 8 : 1) void mask_np_kernel(AT a) {
    constexpr uint64_t kStep = kSpan * U;
    constexpr uint64_t kWin = kStep * K;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wpb = blockDim.x / kWave;
    uint64_t block = blockIdx.x;
    if (a.xcd_remap == 1) {
        // blocks b and b + 8 share an XCD (round-robin dispatch): give each XCD one
        // contiguous share of the batch, so its L2 fetches only that share's descriptors
        const uint64_t nb = gridDim.x, per = nb / 8;
        if (block < per * 8) block = (block % 8) * per + block / 8;
    } else if (a.xcd_remap == 2) {
        // groups of 64 blocks: the 8 blocks of a group that share an XCD take 8 consecutive
        // blocks' windows (64 KiB), so a descriptor line (16 frame offsets) is fetched by one
        // XCD, while the grid as a whole still streams one compact front
        const uint64_t nb = gridDim.x;
        if (block < nb / 64 * 64) block = (block / 64) * 64 + (block % 8) * 8 + (block / 8) % 8;
    }
    const uint64_t wave = block * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // uniform: scalar branches
    if (wave >= a.nwin) return;
    MASK_STAMP_SCOPE(wave);   // diagnostic build only (tools/mask_timeline.py)
    extern __shared__ uint32_t lds_occupancy_pad[];   // dynamic LDS only limits workgroups per CU
    (void)lds_occupancy_pad;
    init_frames(a);
    // tapered end (aligned mask walk only): the windows from a.full_win on are one step each, so
    // the last waves of the launch are short (wave-uniform, scalar)
    constexpr bool kTaper = SRC_ALIGNED && !VAL && K > 1;
    const bool short_win = kTaper && wave >= a.full_win;
    const uint64_t A = short_win ? a.full_win * kWin + (wave - a.full_win) * kStep : wave * kWin;
    const int ksteps = short_win ? 1 : K;
    const uint64_t full_lo = a.mis ? 16 : 0;
    const uint64_t full_hi = (a.mis + a.total) & ~15ull;
    if (A < full_lo || A + (uint64_t)ksteps * kStep > full_hi) {   // a window holding a partial vector (<= 2 per batch)
        uint32_t ec = 0;   // VAL: the carry runs across the window's steps (a step start is no seam)
#pragma unroll 1
        for (int k = 0; k < ksteps; ++k)
            edge_chunk<U, SRC_ALIGNED, NT, VAL>(a, A + (uint64_t)k * kStep, lane, ec, k == 0);
        return;
    }
    uint32_t carry = 0;   // the previous span's last 4 unmasked bytes (VAL)
    // VAL, out of place: the window checks its own first bytes (seam_raw / seam_unmask); the
    // src dword before it is loaded with the window's payload, unmasked once the table is in
    constexpr bool kOwn = VAL && K == 1;      // (launch_mask_validate sets seam_src for one-step windows only)
    const bool own = kOwn && own_seam(a, A);  // wave-uniform
    uint32_t seam_w = 0;
    Table t;
    auto emit = [&](uint64_t A0, u32x4 src, bool first) {
        const u32x4 m = span_mask(a, t, A0, lane);
        const u32x4 out = src ^ m;
        store_vec<NT>(a, A0 + 16ull * lane, out);
        if constexpr (VAL) {
            validate_span(a, t, A0, out, carry, first, lane);
        }
    };
    if constexpr (!SRC_ALIGNED) {
        // src misaligned against dst: whole source lines + a shift across lanes (shift_window)
        constexpr int M = U * K;
        const uint8_t* S = a.src_base + A;                       // the window's first source byte
        const uint32_t o = (uint32_t)((uintptr_t)S & 127u);      // uniform over the batch
        const uint8_t* L = S - o + 16 * lane;
        u32x4 c[M + 1], v[M];
#pragma unroll
        for (int m = 0; m < M; ++m) c[m] = load_line_block<NT>(L + (uint64_t)m * kSpan);
        // the line after: lanes 0 .. o/16 hold its blocks; the others re-read lane o/16's
        // block (same line) instead of branching -- a load under a lane branch is followed
        // by vmcnt(0), which held the table's trip behind the payload's
        const uint32_t lm = min((uint32_t)lane, o >> 4);
        c[M] = load_line_block<NT>(S - o + 16 * lm + (uint64_t)M * kSpan);
        if constexpr (kOwn) seam_w = seam_raw<SRC_ALIGNED>(a, own ? A : A + 4);   // (not own: a dword of the window, unused)
        first_probe(a, t, A, lane);
        np_resolve(a, t, A, lane);
        if constexpr (kOwn) {
            if (own) carry = seam_unmask(t, A, seam_w);
        }
        switch ((o >> 2) & 3) {   // uniform: constant register indices in each case
            case 0: shift_window<M, 0>(c, v, o, lane); break;
            case 1: shift_window<M, 1>(c, v, o, lane); break;
            case 2: shift_window<M, 2>(c, v, o, lane); break;
            default: shift_window<M, 3>(c, v, o, lane); break;
        }
#pragma unroll
        for (int m = 0; m < M; ++m) emit(A + (uint64_t)m * kSpan, v[m], m == 0 && !own);
        return;
    }
    u32x4 d[U];
    auto load_step = [&](uint64_t base) {
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = load_vec<true, NT>(a, base + (uint64_t)u * kSpan + 16ull * lane);
    };
    load_step(A);
    if constexpr (kOwn) seam_w = seam_raw<true>(a, own ? A : A + 4);   // (not own: a dword of the window, unused)
    first_probe(a, t, A, lane);
    np_resolve(a, t, A, lane);
    if constexpr (kOwn) {
        if (own) carry = seam_unmask(t, A, seam_w);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t base = A + (uint64_t)k * kStep;
        if (kTaper && k >= ksteps) break;   // wave-uniform: a tapered window's single step is done
        if (k > 0) load_step(base);
#pragma unroll
        for (int u = 0; u < U; ++u) emit(base + (uint64_t)u * kSpan, d[u], k == 0 && u == 0 && !own);
    }
}

}  // namespace netc_gpu

// ------------------------------------------------------------------ launch --

namespace netc_gpu {

// Workgroups that fit on the device at once for one kernel instantiation
// (occupancy x CUs), cached per device: the grid is exactly one resident round
// and every wavefront strides over the chunks.
template <int U, bool AL, bool NT>
static int resident_blocks() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
    if (cache[dev] > 0) return cache[dev];
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, mask_frames_kernel<U, AL, NT>, 256, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu <= 0 || cus <= 0)
        return 1024;
    cache[dev] = per_cu * cus;
    return cache[dev];
}

template <int U, bool AL, bool NT>
static hipError_t launch_u(const Args& a, int max_blocks, hipStream_t s) {
    const uint64_t cap = (uint64_t)(max_blocks > 0 ? max_blocks : resident_blocks<U, AL, NT>());
    const uint64_t want = (a.nwin + 3) / 4;                   // one chunk per wavefront at most
    const int blocks = (int)(want < cap ? want : cap);
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL((mask_frames_kernel<U, AL, NT>), dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int U>
static hipError_t launch_nt(const Args& a, bool nt, int max_blocks, hipStream_t s) {
    return nt ? launch_u<U, true, true>(a, max_blocks, s) : launch_u<U, true, false>(a, max_blocks, s);
}

// dynamic LDS per workgroup of the one-window-per-wave walk (0 = none); only limits
// workgroups per CU.  NETC_MASK_LDS overrides (measurement sweeps, tools/).
static int np_lds_bytes() {
    static const int v = [] {
        const char* e = getenv("NETC_MASK_LDS");
        const long x = e ? strtol(e, nullptr, 10) : 0;
        return (int)(x < 0 ? 0 : (x > 65536 ? 65536 : x));
    }();
    return v;
}

template <int U, int K, bool AL, bool NT, bool VAL = false>
static hipError_t launch_np(const Args& a, hipStream_t s) {
    const uint64_t blocks = (a.nwin + 3) / 4;   // 4 wavefronts per 256-thread workgroup
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL((mask_np_kernel<U, K, AL, NT, VAL>), dim3((unsigned)blocks), dim3(256), np_lds_bytes(), s, a);
    return hipGetLastError();
}

template <int U, bool AL, bool NT>
static hipError_t launch_np_k(const Args& a, bool two, hipStream_t s) {
    return two ? launch_np<U, 2, AL, NT>(a, s) : launch_np<U, 1, AL, NT>(a, s);
}

template <int U, bool AL>
static hipError_t launch_np_nt(const Args& a, bool nt, bool two, hipStream_t s) {
    return nt ? launch_np_k<U, AL, true>(a, two, s) : launch_np_k<U, AL, false>(a, two, s);
}

template <bool AL>
static hipError_t launch_np_u(const Args& a, int U, bool nt, bool two, hipStream_t s) {
    switch (U) {
        case 1: return launch_np_nt<1, AL>(a, nt, two, s);
        case 4: return launch_np_nt<4, AL>(a, nt, two, s);
        case 8: return launch_np_nt<8, AL>(a, nt, two, s);
        default: return launch_np_nt<2, AL>(a, nt, two, s);
    }
}

static Args make_args(uint8_t* dst, const uint8_t* src, uint64_t total, const uint64_t* off, const uint32_t* keys,
                      uint64_t n, const uint64_t* n_dev) {
    Args a;
    a.n_dev = n_dev;
    a.verr = nullptr;
    a.vtag = 0;
    a.xcd_remap = 0;
    a.seam_src = 0;
    a.mis = (uint64_t)(uintptr_t)dst & 15u;
    a.dst_base = dst - a.mis;
    a.src_base = src - a.mis;
    a.total = total;
    a.off = off;
    a.keys = (n || n_dev) ? keys : reinterpret_cast<const uint32_t*>(off);   // frame_entry always reads keys[0]
    a.n = n;
    a.density = total ? (double)n / (double)total : 0.0;
    a.nwin = 0;
    a.probe_e = kWave;
    a.probe_bias = 24;
    a.full_win = ~0ull;
    return a;
}

// The default walk's first table probe (first_probe), from the window size: windows that
// hold a frame start or more on average (frames up to ~2 KiB: config 2, small frames) take
// the base the mean density predicts minus one frame and only the entries the window can
// reach, ceil(window x density) + 3 -- exact for evenly sized frames.  A full 64-entry
// probe read 768 B of descriptors per 2 KiB window at config 2 for the 3 entries used,
// and every XCD's L2 fetched every descriptor line (PMC: 1.048x the algorithmic bytes).
// Sparser windows (config 4's 256 B - 64 KiB frames) keep 64 entries biased 24 frames
// back, whose reach absorbs the guess error of random sizes.
static void set_probe(Args& a, uint64_t win) {
    const double reach = (double)win * a.density;
    if (reach >= 1.0 && reach < (double)(kWave - 4)) {
        a.probe_e = (int)reach + 4;
        a.probe_bias = 1;
    }
}

// In-place unmask of the frames a scan found (ws_scan_gpu.hip): the default walk,
// frames read from the scan's outputs on the device (ArgsScan; nothing is allocated).
hipError_t launch_mask_scanned(uint8_t* wire, uint64_t len, const uint64_t* hdr, const uint32_t* keys,
                               uint64_t max_frames, const uint64_t* result, hipStream_t stream) {
    ArgsScan a;
    static_cast<Args&>(a) = make_args(wire, wire, len, hdr, keys, 0, result);
    a.hdr = hdr;
    a.fkeys = keys;
    a.result = result;
    a.max_frames = max_frames;
    const uint64_t nvec = (a.mis + len + 15) / 16;
    a.nwin = (nvec + 127) / 128;   // windows of 2 x 1 KiB
    const uint64_t blocks = (a.nwin + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL((mask_np_kernel<1, 2, true, true, false, ArgsScan>), dim3((unsigned)blocks), dim3(256), 0,
                       stream, a);
    return hipGetLastError();
}

hipError_t launch_mask_frames(uint8_t* dst, const uint8_t* src, uint64_t total, const uint64_t* off,
                              const uint32_t* keys, uint64_t n, hipStream_t stream, const LaunchCfg& cfg,
                              const uint64_t* n_dev) {
    // n_dev: n is only an upper bound here (keys must then always be readable)
    Args a = make_args(dst, src, total, off, keys, n, n_dev);
    const bool aligned = (((uintptr_t)src ^ (uintptr_t)dst) & 15u) == 0;
    const uint64_t nvec = (a.mis + total + 15) / 16;
    if (nvec == 0) return hipSuccess;
    const int flags = cfg.flags;
    // payload loads / stores non-temporal unless asked otherwise: every byte is touched once
    const bool nt = flags < 0 || (flags & (kNtLoads | kNtStores));
    if (flags >= 0 && (flags & kPersistent)) {   // round 1's walk: one resident round striding over the chunks
        const int U = aligned ? cfg.unroll : 4;
        const uint64_t win_vec = 64ull * (uint64_t)U;
        a.nwin = (nvec + win_vec - 1) / win_vec;
        const int mb = cfg.max_blocks;
        if (!aligned) return nt ? launch_u<4, false, true>(a, mb, stream) : launch_u<4, false, false>(a, mb, stream);
        switch (U) {
            case 1: return launch_nt<1>(a, nt, mb, stream);
            case 2: return launch_nt<2>(a, nt, mb, stream);
            case 8: return launch_nt<8>(a, nt, mb, stream);
            default: return launch_nt<4>(a, nt, mb, stream);
        }
    }
    // auto: two steps of `unroll` KiB per wavefront (1 KiB x 2: the fastest walk measured,
    // frame-free and with frames, at 64 MiB and at 1 GiB)
    const bool two = flags < 0 || (flags & kTwoSteps);
    a.xcd_remap = (flags >= 0 && (flags & kXcdRemap)) ? 1 : ((flags >= 0 && (flags & kXcdGroups)) ? 2 : 0);
    // src misaligned against dst, auto, >= 256 MiB: windows of 4 x 1 KiB (33 source lines per
    // 4 spans, not 17 per 2): 1 GiB mixed frames 0.88 -> 0.97 of the aligned rate; at 64 MiB
    // 2 x 1 KiB stays ahead (profiles/r02j_misaligned_sweep.jsonl)
    const int U = (!aligned && flags < 0 && total >= (256ull << 20)) ? 2 : cfg.unroll;
    const uint64_t win_vec = 64ull * (uint64_t)U * (two ? 2 : 1);
    a.nwin = (nvec + win_vec - 1) / win_vec;
    set_probe(a, 16 * win_vec);
    // NETC_GPU_KNOB_MASK_TAPER (A/B, tools/): the batch's last `taper` bytes in one-step windows
    const int64_t taper = knob(NETC_GPU_KNOB_MASK_TAPER);
    if (two && aligned && taper > 0) {
        const uint64_t step = 1024ull * (uint64_t)U, span = nvec * 16;
        uint64_t t = ((uint64_t)taper + step - 1) / step * step;
        t = t < span ? t : span;
        a.full_win = (span - t) / (2 * step);
        a.nwin = a.full_win + (span - a.full_win * 2 * step + step - 1) / step;
    }
    return aligned ? launch_np_u<true>(a, U, nt, two, stream) : launch_np_u<false>(a, U, nt, two, stream);
}


// Phase B of the TEXT check: one thread per frame; the thread of a data frame with
// FIN walks back to its message's first frame and, for a TEXT message, forward
// again over its data frames (control frames skipped): any frame flagged by
// phase A fails it; the first 3 bytes of every frame are checked here with the 3
// bytes before them in the message; the message must not end inside a sequence.
__device__ __forceinline__ bool utf8_rule(uint32_t b3, uint32_t b2, uint32_t b1, uint32_t b0) {
    // utf8_err_word's rule for one byte b0 and the 3 before it (0 before a message's start)
    auto lut8 = [](uint32_t hi, uint32_t lo, uint32_t i) { return ((i < 4 ? lo >> (8 * i) : hi >> (8 * (i - 4)))) & 0xFFu; };
    const uint32_t b1h = b1 < 0x80 ? 0x02u : lut8(kB1H_HI, kB1H_LO, (b1 >> 4) & 7);
    const uint32_t b1l = (b1 & 8) ? lut8(kB1L_1H, kB1L_1L, b1 & 7) : lut8(kB1L_0H, kB1L_0L, b1 & 7);
    const uint32_t b2h = b0 < 0x80 ? 0x01u : lut8(kB2H_HI, kB2H_LO, (b0 >> 4) & 7);
    const uint32_t must = (b2 >= 0xE0 || b3 >= 0xF0) ? 0x80u : 0u;
    return ((b1h & b1l & b2h) ^ must) != 0;
}

// the first 3 and last 3 bytes of [lo, hi) (clamped into it; bytes past a short frame's end are
// never used) in one trip -- a load in a loop of data-dependent length was a trip per byte
__device__ __forceinline__ void frame_edges(const uint8_t* dst, uint64_t lo, uint64_t hi, uint32_t (&fb)[3],
                                            uint32_t (&lb)[3]) {
    if (hi > lo) {
        const uint64_t last = hi - 1;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            fb[d] = dst[lo + d < last ? lo + d : last];
            lb[d] = dst[hi - lo > 3 ? hi - 3 + d : lo];   // (used only when hi - lo > 3)
        }
    }
}

// the first 3 bytes of every window start strictly inside [lo + 3, hi) (the bytes phase A left:
// in place another wavefront's window held the bytes before them); the 4 bytes before and
// after each start (aligned dwords: dst - mis is 16-aligned, window starts are multiples of
// win >= 4096) are read for 8 windows at a time, unconditionally (a start past the frame
// re-reads the first one; a load under a per-lane branch made the compiler wait for each one
// in turn: 29.7 us at config 4, r03k).  win 0: no seams to check.
__device__ __forceinline__ bool seams_bad(const uint8_t* dst, uint64_t lo, uint64_t hi, uint64_t mis, uint64_t win) {
    bool bad = false;
    const uint64_t cb0 = win ? (lo + 3 + mis + win - 1) / win * win : ~0ull;
    for (uint64_t cb = cb0; win && cb < hi + mis && !bad; cb += 8 * win) {
        uint32_t wb[8], wa[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t c = cb + (uint64_t)i * win;
            const uint64_t q = (c < hi + mis ? c : cb) - mis;   // q: the window's first byte
            wb[i] = *(const NETC_GLOBAL uint32_t*)(dst + q - 4);
            wa[i] = *(const NETC_GLOBAL uint32_t*)(dst + q);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t c = cb + (uint64_t)i * win, q = c - mis;
            const uint64_t w = (uint64_t)wa[i] << 32 | wb[i];   // bytes q - 4 .. q + 3
            auto B = [&](int j) { return (uint32_t)(w >> (8 * j)) & 0xFFu; };
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (c < hi + mis && q + d >= lo + 3 && q + d < hi) bad |= utf8_rule(B(1 + d), B(2 + d), B(3 + d), B(4 + d));
        }
    }
    return bad;
}

// Phase B of the TEXT check: one thread per frame.  Everything a single-frame TEXT message (FIN
// and opcode 1: config 2's frames) needs -- its header byte, flag, offsets -- comes in one trip,
// its first and last 3 bytes in a second (round 4: the message walk took four dependent trips
// for it, 6.6 us at config 2); the thread of a FIN continuation frame walks back to its
// message's first frame and, for a TEXT message, forward again over its data frames (control
// frames skipped).  Any frame flagged by phase A fails the message; the first 3 bytes of every
// frame are checked here with the 3 bytes before them in the message; the message must not end
// inside a sequence.
__global__ void utf8_messages(const uint8_t* dst, const uint64_t* off, const uint8_t* h0, uint64_t n,
                              const uint8_t* verr, uint8_t tag, uint64_t mis, uint64_t win, uint8_t* valid) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t hk = h0[k];
    const uint8_t fk = verr[k];
    const uint64_t lk = off[k], hk_end = off[k + 1];
    uint8_t verdict = 1;
    const uint32_t opk = hk & 0x0F;
    if ((hk & 0x80) && opk == 1) {
        // a single-frame TEXT message
        bool bad = fk == tag;
        uint32_t fb[3] = {0, 0, 0}, lb[3] = {0, 0, 0};
        frame_edges(dst, lk, hk_end, fb, lb);
        uint32_t h1 = 0, h2 = 0, h3 = 0;   // the last 3 bytes of the message so far (h1 = last)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (lk + d < hk_end) {
                bad |= utf8_rule(h3, h2, h1, fb[d]);
                h3 = h2;
                h2 = h1;
                h1 = fb[d];
            }
        }
        if (hk_end - lk > 3) {
            h3 = lb[0];
            h2 = lb[1];
            h1 = lb[2];
        }
        if (h1 >= 0xC0 || h2 >= 0xE0 || h3 >= 0xF0) bad = true;   // ends inside a sequence
        if (!bad) bad = seams_bad(dst, lk, hk_end, mis, win);
        verdict = bad ? 0 : 1;
    } else if ((hk & 0x80) && opk == 0) {
        // the last frame of a fragmented message: its first frame
        int64_t first = -1;
        for (int64_t j = (int64_t)k - 1; j >= 0; --j) {
            const uint32_t op = h0[j] & 0x0F;
            if (op >= 8) continue;                              // control frame inside the message
            if (op != 0) {
                first = j;
                break;
            }
            if (h0[j] & 0x80) break;                            // a finished message: orphan continuation
        }
        if (first >= 0 && (h0[first] & 0x0F) == 1) {
            uint32_t h1 = 0, h2 = 0, h3 = 0;   // the last 3 bytes of the message so far (h1 = last)
            bool bad = false;
            for (uint64_t j = (uint64_t)first; j <= k && !bad; ++j) {
                if ((h0[j] & 0x0F) >= 8) continue;
                if (verr[j] == tag) bad = true;
                const uint64_t lo = off[j], hi = off[j + 1];
                uint32_t fb[3] = {0, 0, 0}, lb[3] = {0, 0, 0};
                frame_edges(dst, lo, hi, fb, lb);
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    if (lo + d < hi) {
                        bad |= utf8_rule(h3, h2, h1, fb[d]);
                        h3 = h2;
                        h2 = h1;
                        h1 = fb[d];
                    }
                }
                bad |= seams_bad(dst, lo, hi, mis, win);
                if (hi - lo > 3) {   // the frame's own last 3 bytes become the history
                    h3 = lb[0];
                    h2 = lb[1];
                    h1 = lb[2];
                }
            }
            if (h1 >= 0xC0 || h2 >= 0xE0 || h3 >= 0xF0) bad = true;   // ends inside a sequence
            verdict = bad ? 0 : 1;
        }
    }
    valid[k] = verdict;
}

// the VAL kernels: 4 KiB windows (the seams utf8_messages re-checks are at multiples of it)
// a 4 KiB window per wavefront as U KiB x K steps (NETC_GPU_KNOB_VAL_STEPS = K: 1, 2 or 4).
// Default by batch size: two 2 KiB steps up to 256 MiB (config 2: 32.3 against 33.2 us), one
// 4 KiB step above (config 4: 454-461 against 468-475 us; r03l)
static int val_steps(uint64_t total) {
    const int64_t k = knob(NETC_GPU_KNOB_VAL_STEPS);
    return k == 2 || k == 4 ? (int)k : (k == 1 ? 1 : (total <= (256ull << 20) ? 2 : 1));
}

template <bool AL>
static hipError_t launch_val(const Args& a, bool persistent, int k, hipStream_t s) {
    if (!persistent) {
        switch (k) {
            // two steps (up to 256 MiB by default): plain payload loads and stores, so phase B
            // reads the unmasked bytes from cache (config 2 31.7 against 32.4 us); one step
            // (above 256 MiB): non-temporal (config 4 458-463 against 474-480 with plain; r03w)
            case 2: return launch_np<2, 2, AL, false, true>(a, s);
            case 4: return launch_np<1, 4, AL, true, true>(a, s);
            default: return launch_np<4, 1, AL, true, true>(a, s);
        }
    }
    const uint64_t cap = (uint64_t)resident_blocks<4, AL, true>();
    const uint64_t want = (a.nwin + 3) / 4;
    const int blocks = (int)(want < cap ? want : cap);
    if (blocks > 0) hipLaunchKernelGGL((mask_frames_kernel<4, AL, true, true>), dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_mask_validate(uint8_t* dst, const uint8_t* src, uint64_t total, const uint64_t* off,
                                const uint32_t* keys, const uint8_t* header0, uint64_t n, uint8_t* verr, uint8_t tag,
                                uint8_t* valid, hipStream_t stream, const LaunchCfg& cfg) {
    if (n == 0) return hipSuccess;
    Args a = make_args(dst, src, total, off, keys, n, nullptr);
    a.verr = verr;
    a.vtag = tag;
    const uint64_t nvec = (a.mis + total + 15) / 16;
    a.nwin = (nvec + 255) / 256;   // windows of 4 KiB (64 vectors x 4)
    set_probe(a, 4096);
    const bool persistent = cfg.flags >= 0 && (cfg.flags & kPersistent);
    // out of place, one-window walk: each window checks the bytes after its own start (the 4
    // before it unmasked from src, which nobody writes), so utf8_messages skips the seams (win
    // 0).  In place the bytes before a window may or may not be unmasked yet when it reads them.
    // Only with one-step windows: with two steps the kernel measured 2 us slower at config 2
    // (27.9 against 26.0 us) than the seams cost phase B there; at config 4 (one step) it saves
    // 3 us (442.5 against 445.5; phase B 27.7 -> 8.1 us) (r03n)
    const int k = val_steps(total);
    a.seam_src = dst != src && !persistent && k == 1;
    hipError_t e;
    if (a.nwin) {
        const bool aligned = (((uintptr_t)src ^ (uintptr_t)dst) & 15u) == 0;
        e = aligned ? launch_val<true>(a, persistent, k, stream) : launch_val<false>(a, persistent, k, stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(utf8_messages, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, dst, off, header0, n,
                       verr, tag, a.mis, a.seam_src ? 0 : kSpan * 4, valid);
    return hipGetLastError();
}

}  // namespace netc_gpu
