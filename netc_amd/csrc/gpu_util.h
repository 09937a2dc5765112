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

}  // namespace netc_gpu
