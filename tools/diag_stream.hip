// DIAGNOSTIC ONLY (not part of the product): HBM stream ceilings on gfx950 for
// the masking kernel's access pattern.  Every variant moves 16 B per lane per
// vector with dwordx4 loads / stores; `contig` = each wavefront walks one
// contiguous 1/nwaves share (as the masking kernel does), otherwise grid-stride.
//   mode 0  in-place XOR with a constant key   (read N + write N)
//   mode 1  read only: XOR-reduce, one dword per wave out   (read N)
//   mode 2  write only: constant fill          (write N)
//   mode 3  out-of-place copy-XOR src -> dst   (read N + write N)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, bool NT, int U>
__global__ __launch_bounds__(256) void stream_kernel(u32x4* dst, const u32x4* src, uint64_t nvec, uint32_t key,
                                                     int contig, uint32_t* sink) {
    const u32x4 k = {key, key, key, key};
    u32x4 acc = {0, 0, 0, 0};
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4;
    uint64_t begin, end, step, first;
    if (contig) {
        // wave-contiguous: [begin, end) in units of 64*U vectors
        const uint64_t nwin = nvec / (64 * U);
        begin = wave * nwin / nwaves * 64 * U;
        end = (wave + 1) * nwin / nwaves * 64 * U;
        step = 64 * U;
        first = begin + lane;
    } else {
        begin = 0;
        end = nvec / (64 * U * nwaves) * (64 * U * nwaves);
        step = 64 * U * nwaves;
        first = wave * 64 * U + lane;
    }
    for (uint64_t base = first; base < end; base += step) {
        u32x4 d[U];
        if constexpr (MODE != 2) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32x4* p = src + base + 64 * u;
                d[u] = NT ? __builtin_nontemporal_load(p) : *p;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4* q = dst + base + 64 * u;
            if constexpr (MODE == 1) {
                acc ^= d[u];
            } else {
                const u32x4 v = (MODE == 2) ? k : (d[u] ^ k);
                if (NT) __builtin_nontemporal_store(v, q);
                else *q = v;
            }
        }
    }
    if constexpr (MODE == 1) {
        const uint32_t r = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
        if (r == 0x12345678u) sink[wave] = r;   // keeps the loads alive
    }
    (void)begin;
}

template <int MODE, bool NT>
static int launch(void* dst, const void* src, uint64_t nvec, uint32_t key, int blocks, int contig, void* sink,
                  hipStream_t s) {
    hipLaunchKernelGGL((stream_kernel<MODE, NT, 4>), dim3(blocks), dim3(256), 0, s, (u32x4*)dst, (const u32x4*)src,
                       nvec, key, contig, (uint32_t*)sink);
    return (int)hipGetLastError();
}

extern "C" int diag_stream(int mode, int nt, int contig, void* dst, const void* src, uint64_t nbytes, uint32_t key,
                           int blocks, void* sink, void* stream) {
    const uint64_t nvec = nbytes / 16;
    hipStream_t s = (hipStream_t)stream;
    switch (mode * 2 + (nt ? 1 : 0)) {
        case 0: return launch<0, false>(dst, src, nvec, key, blocks, contig, sink, s);
        case 1: return launch<0, true>(dst, src, nvec, key, blocks, contig, sink, s);
        case 2: return launch<1, false>(dst, src, nvec, key, blocks, contig, sink, s);
        case 3: return launch<1, true>(dst, src, nvec, key, blocks, contig, sink, s);
        case 4: return launch<2, false>(dst, src, nvec, key, blocks, contig, sink, s);
        case 5: return launch<2, true>(dst, src, nvec, key, blocks, contig, sink, s);
        case 6: return launch<3, false>(dst, src, nvec, key, blocks, contig, sink, s);
        default: return launch<3, true>(dst, src, nvec, key, blocks, contig, sink, s);
    }
}
