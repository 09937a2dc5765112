// DIAGNOSTIC ONLY (not part of the product): the simplest possible 16-B-per-lane
// streaming XOR with one constant key word, grid-stride, U vectors in flight per
// lane.  Its rate on a buffer is the practical HBM ceiling for the masking
// kernel's access pattern (read 16 B + write 16 B per lane-vector).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void xor_const(u32x4* dst, const u32x4* src, uint64_t nvec, uint32_t key) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const u32x4 k = {key, key, key, key};
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(d[u] ^ k, dst + i + u * stride);
            else dst[i + u * stride] = d[u] ^ k;
        }
    }
    for (; i < nvec; i += stride) dst[i] = src[i] ^ k;
}

extern "C" int diag_xor_const(void* dst, const void* src, uint64_t nbytes, uint32_t key, int blocks, int nt,
                              void* stream) {
    const uint64_t nvec = nbytes / 16;
    if (nt) hipLaunchKernelGGL((xor_const<4, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, (u32x4*)dst,
                               (const u32x4*)src, nvec, key);
    else hipLaunchKernelGGL((xor_const<4, false>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, (u32x4*)dst,
                            (const u32x4*)src, nvec, key);
    return (int)hipGetLastError();
}
