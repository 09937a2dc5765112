// DIAGNOSTIC ONLY: does the ORDER in which wavefronts walk an in-place XOR stream
// matter on MI355X HBM?  All variants: 16 B per lane, U = 4 wave-instructions
// (4 KiB) per chunk, non-temporal loads + stores, next chunk's loads issued before
// the current chunk is stored (prefetch depth 1).
//   order 1  wave-contiguous: wave w owns chunks [w*C/W, (w+1)*C/W)
//   order 2  static interleave: wave w owns chunks w, w+W, w+2W, ...
//   order 3  dynamic, in address order: chunks handed out by one atomic ticket
//            counter (zeroed by the caller before the launch), fetched one ahead
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int U = 4;
constexpr uint64_t kChunkVec = 64 * U;   // vectors per chunk (4 KiB)

template <int ORDER>
__global__ __launch_bounds__(256, 4) void order_kernel(u32x4* buf, uint64_t nchunks, uint32_t key,
                                                      unsigned long long* ticket) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const u32x4 k = {key, key, key, key};
    uint64_t c, c_end = 0, stride = 1;
    if (ORDER == 1) {
        c = wave * nchunks / W;
        c_end = (wave + 1) * nchunks / W;
    } else if (ORDER == 2) {
        c = wave;
        c_end = nchunks;
        stride = W;
    } else {
        uint64_t t = 0;
        if (lane == 0) t = atomicAdd(ticket, 1ull);
        c = __builtin_amdgcn_readfirstlane((uint32_t)t);   // < 2^32 chunks
        c_end = nchunks;
    }
    if (c >= c_end) return;
    u32x4 d[U], dn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(buf + c * kChunkVec + 64 * u + lane);
    uint64_t nxt_t = 0;
    if (ORDER == 3 && lane == 0) nxt_t = atomicAdd(ticket, 1ull);
    for (;;) {
        uint64_t cn;
        if (ORDER == 3) cn = __builtin_amdgcn_readfirstlane((uint32_t)nxt_t);
        else cn = c + stride;
        const bool more = cn < c_end;
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) dn[u] = __builtin_nontemporal_load(buf + cn * kChunkVec + 64 * u + lane);
            if (ORDER == 3 && lane == 0) nxt_t = atomicAdd(ticket, 1ull);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(d[u] ^ k, buf + c * kChunkVec + 64 * u + lane);
        if (!more) break;
        c = cn;
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = dn[u];
    }
}

extern "C" int diag_order(int order, void* buf, uint64_t nbytes, uint32_t key, int blocks, void* ticket,
                          void* stream) {
    const uint64_t nchunks = nbytes / (kChunkVec * 16);
    hipStream_t s = (hipStream_t)stream;
    if (order == 3) (void)hipMemsetAsync(ticket, 0, 16, s);   // 16-B multiple: cheaper memset node
    switch (order) {
        case 1: hipLaunchKernelGGL((order_kernel<1>), dim3(blocks), dim3(256), 0, s, (u32x4*)buf, nchunks, key,
                                   (unsigned long long*)ticket); break;
        case 2: hipLaunchKernelGGL((order_kernel<2>), dim3(blocks), dim3(256), 0, s, (u32x4*)buf, nchunks, key,
                                   (unsigned long long*)ticket); break;
        default: hipLaunchKernelGGL((order_kernel<3>), dim3(blocks), dim3(256), 0, s, (u32x4*)buf, nchunks, key,
                                    (unsigned long long*)ticket); break;
    }
    return (int)hipGetLastError();
}
