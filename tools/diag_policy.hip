// DIAGNOSTIC ONLY: cache-policy bits of the payload stream on gfx950.  In-place XOR
// (or out-of-place) over 4 KiB chunks in the masking kernel's walk order (wavefront w takes chunks
// w, w+W, ...), buffer_load/store_dwordx4 with explicit aux bits:
//   aux bit 0 = sc0, bit 1 = nt, bit 4 = sc1   (cdna_hip_programming.md T8 / G16)
// Each chunk gets its own 4 KiB buffer descriptor (wave-uniform base), so any
// batch size works with 32-bit offsets.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int LAUX, int SAUX>
__global__ __launch_bounds__(256) void policy_kernel(uint8_t* dst, const uint8_t* src, uint64_t nchunks, uint32_t key) {
    const int lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const u32x4 k = {key, key, key, key};
    for (uint64_t c = w; c < nchunks; c += W) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(src + c * 4096), 0, 4096, 0x00020000);
        const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc(dst + c * 4096, 0, 4096, 0x00020000);
        u32x4 d[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            d[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, u * 1024 + lane * 16, 0, LAUX));
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(d[u] ^ k, w, u * 1024 + lane * 16, 0, SAUX);
    }
}

#define CASE(L, S)                                                                                        \
    if (laux == L && saux == S) {                                                                         \
        hipLaunchKernelGGL((policy_kernel<L, S>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,         \
                           (uint8_t*)dst, (const uint8_t*)src, nbytes / 4096, key);                                            \
        return (int)hipGetLastError();                                                                    \
    }

extern "C" int diag_policy(int laux, int saux, void* dst, const void* src, uint64_t nbytes, uint32_t key, int blocks, void* stream) {
    CASE(0, 0) CASE(2, 2) CASE(2, 0) CASE(0, 2) CASE(2, 16) CASE(2, 17) CASE(2, 18) CASE(0, 16) CASE(1, 2) CASE(2, 1)
    CASE(16, 2) CASE(3, 3)
    return -1;
}

// Unaligned-source stream: dst (16-B aligned) <- src + shift (any byte shift), 16-B
// loads at byte granularity (global_load_dwordx4 on an unaligned address), NT.
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
__global__ __launch_bounds__(256) void shift_kernel(uint8_t* dst, const uint8_t* src, uint64_t nchunks, uint32_t key) {
    const int lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const u32x4 k = {key, key, key, key};
    for (uint64_t c = w; c < nchunks; c += W) {
        u32x4 d[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            d[u] = __builtin_nontemporal_load(
                (const __attribute__((address_space(1))) u32x4u*)(src + c * 4096 + u * 1024 + lane * 16));
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_nontemporal_store(d[u] ^ k, (__attribute__((address_space(1))) u32x4*)(dst + c * 4096 + u * 1024 + lane * 16));
    }
}

extern "C" int diag_shift(void* dst, const void* src, uint64_t nbytes, int shift, uint32_t key, int blocks,
                          void* stream) {
    hipLaunchKernelGGL(shift_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (uint8_t*)dst,
                       (const uint8_t*)src + shift, nbytes / 4096 - 1, key);
    return (int)hipGetLastError();
}
