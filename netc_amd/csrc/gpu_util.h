// Device helpers shared by the gfx950 kernels (ws_mask_gpu.hip, ws_frame_gpu.hip).
// Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace netc_gpu {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Every device buffer here is global memory.  Accesses go through explicit
// address-space-1 pointers so the compiler emits global_* instructions: a flat_*
// access (what a generic pointer becomes once its provenance is lost) completes
// out of order and forces s_waitcnt vmcnt(0) lgkmcnt(0) at every use, which
// drains prefetched loads and kills a software pipeline.
#define NETC_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const NETC_GLOBAL T* gptr(const T* p) {
    return (const NETC_GLOBAL T*)p;
}
template <typename T>
__device__ __forceinline__ NETC_GLOBAL T* gptr(T* p) {
    return (NETC_GLOBAL T*)p;
}

static constexpr int kWave = 64;
static constexpr uint64_t kSpan = 64ull * 16ull;          // bytes one wave-instruction moves
static constexpr uint64_t kInf = ~0ull;

__device__ __forceinline__ uint32_t rotr8(uint32_t key, uint64_t r) {
    // rotate right by 8 * (r & 3) bits: v_alignbit_b32 key, key, sh
    return __builtin_amdgcn_alignbit(key, key, (uint32_t)((r & 3u) << 3));
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t readlane32(uint32_t x, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, lane);
}

// x of lane `src` (per-lane source; every lane of the wave must execute it)
__device__ __forceinline__ uint64_t bperm64(uint64_t x, int src) {
    const int addr = src << 2;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Bytes [t, 16) of a vector selected, as 4 dword masks; t is clamped to [0, 16].
__device__ __forceinline__ u32x4 select_from(int64_t t) {
    t = t < 0 ? 0 : (t > 16 ? 16 : t);
    u32x4 s;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        int64_t b = t - 4 * w;
        b = b < 0 ? 0 : (b > 4 ? 4 : b);
        s[w] = (uint32_t)(0xFFFFFFFFull << (8 * b));
    }
    return s;
}

// Bytes [lo, hi) of a vector selected (both clamped to [0, 16]).
__device__ __forceinline__ u32x4 select_range(int64_t lo, int64_t hi) { return select_from(lo) & ~select_from(hi); }

// ---------------------------------------------------- chained scans (shared) --
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int d = kWave / 2; d > 0; d >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, d, kWave);
    return v;
}

// Single-pass chained scans (decoupled look-back) over tiles: each tile publishes
// one 64-bit status word
//   [63:62] flag (1 = tile aggregate, 2 = inclusive prefix) | [61:46] epoch | [45:0] value
// The epoch (one per call and stream) makes words left from earlier calls read as
// "not yet published", so a status array is never cleared between calls.  The
// look-back (one wavefront) reads 64 predecessors at once and sums their
// aggregates back to the nearest inclusive prefix, so tiles do not wait on each
// other one by one.  A tile only waits on lower-numbered tiles, which are
// dispatched first.
static constexpr uint64_t kValBits = 46;
static constexpr uint64_t kValMask = (1ull << kValBits) - 1;

__device__ __forceinline__ uint64_t status_word(uint64_t flag, uint32_t epoch, uint64_t v) {
    return flag << 62 | (uint64_t)(epoch & 0xFFFF) << kValBits | (v & kValMask);
}

// exclusive prefix of tile `tile` (every lane of the calling wavefront takes part)
__device__ inline uint64_t look_back(uint64_t* status, int64_t tile, uint32_t epoch, int lane) {
    uint64_t prefix = 0;
    for (int64_t top = tile - 1; top >= 0;) {
        const int64_t idx = top - lane;
        uint64_t v = 0;
        bool ok = true, incl = idx < 0;   // before tile 0: an inclusive prefix of 0
        if (idx >= 0) {
            const uint64_t w = __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (w >> 62) != 0 && ((w >> kValBits) & 0xFFFF) == (epoch & 0xFFFF);
            incl = ok && (w >> 62) == 2;
            v = w & kValMask;
        }
        const uint64_t im = __ballot(incl);
        const int stop = im ? __builtin_ctzll(im) : kWave;   // nearest inclusive prefix
        const uint64_t need = stop >= kWave - 1 ? ~0ull : ((2ull << stop) - 1);
        if ((__ballot(ok) & need) != need) {
            __builtin_amdgcn_s_sleep(1);   // a predecessor has not published yet
            continue;
        }
        prefix += wave_sum(lane <= stop ? v : 0);
        if (stop < kWave) break;
        top -= kWave;
    }
    return prefix;
}

}  // namespace netc_gpu
