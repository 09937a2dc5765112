// MEASUREMENT ONLY (not on the product path): the HBM stream ceilings bench.py
// reports next to the masking kernel, measured in the same process on the same
// buffer rotation.  Hand-written gfx950 kernels, every one a
// plain 16-byte-per-lane stream with no frame logic:
//
//   mode 0  out-of-place copy  dst[i] = src[i]              (read N + write N)  the guide's "float4 copy"
//   mode 1  in-place XOR       buf[i] ^= key                (read N + write N)  the mask kernel minus frames
//   mode 2  out-of-place XOR   dst[i] = src[i] ^ key        (read N + write N)
//   mode 3  read only          XOR-reduce, one word per wave (read N)
//   mode 4  write only         dst[i] = key                 (write N)
//
// Walk: chunks of U x 1 KiB (one 16-B vector per lane per KiB).  blocks > 0: a
// persistent grid of that many workgroups, wavefront w taking chunks w, w + W, ...
// (the mask kernel's order), the next chunk's loads in flight while this one is
// stored; blocks == 0: the same with one resident round (occupancy x CUs);
// blocks < 0: one chunk per wavefront, a grid covering the buffer (the classic
// copy kernel: the dispatcher refills CUs as workgroups retire).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define G1 __attribute__((address_space(1)))

template <bool NT>
__device__ __forceinline__ u32x4 ld(const G1 u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(G1 u32x4* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int MODE, bool NT, int U>
__global__ __launch_bounds__(1024) void stream_kernel(u32x4* dst_, const u32x4* src_, uint64_t nchunks, uint32_t key,
                                                      int persistent, uint32_t* sink) {
    G1 u32x4* dst = (G1 u32x4*)dst_;
    const G1 u32x4* src = (const G1 u32x4*)src_;
    const u32x4 k = {key, key, key, key};
    const int lane = threadIdx.x & 63;
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    u32x4 acc = {0, 0, 0, 0};
    auto loadc = [&](u32x4(&d)[U], uint64_t c) {
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = ld<NT>(src + c * (64 * U) + 64 * u + lane);
    };
    auto storec = [&](const u32x4(&d)[U], uint64_t c) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            G1 u32x4* q = dst + c * (64 * U) + 64 * u + lane;
            if constexpr (MODE == 0) st<NT>(q, d[u]);
            else if constexpr (MODE == 1 || MODE == 2) st<NT>(q, d[u] ^ k);
            else if constexpr (MODE == 3) acc ^= d[u];
            else st<NT>(q, k);
        }
    };
    uint64_t c = wave;
    if (c >= nchunks) return;
    u32x4 d[U];
    if constexpr (MODE != 4) loadc(d, c);
    if (persistent) {
        for (uint64_t cn = c + nwaves; cn < nchunks; cn += nwaves) {
            u32x4 dn[U];
            if constexpr (MODE != 4) loadc(dn, cn);
            storec(d, c);
            c = cn;
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = dn[u];
        }
    }
    storec(d, c);
    if constexpr (MODE == 3) {
        const uint32_t r = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
        if (r == 0x9E3779B9u) sink[wave & 1023] = r;   // keeps the loads alive
    }
}

template <int MODE, bool NT, int U>
int launch(void* dst, const void* src, uint64_t nbytes, uint32_t key, int threads, int blocks, void* sink,
           hipStream_t s) {
    const uint64_t nchunks = nbytes / (1024ull * U);
    if (nchunks == 0) return 0;
    const int wpb = threads / 64;
    if (blocks == 0) {
        int per_cu = 0, cus = 0, dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, stream_kernel<MODE, NT, U>, threads, 0) !=
                hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -2;
        blocks = per_cu * cus;
    }
    const int persistent = blocks > 0;
    uint64_t grid = persistent ? (uint64_t)blocks : (nchunks + wpb - 1) / wpb;
    const uint64_t need = (nchunks + wpb - 1) / wpb;
    if (grid > need) grid = need;
    hipLaunchKernelGGL((stream_kernel<MODE, NT, U>), dim3((unsigned)grid), dim3(threads), 0, s, (u32x4*)dst,
                       (const u32x4*)src, nchunks, key, persistent, (uint32_t*)sink);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int MODE, bool NT>
int by_u(int u, void* dst, const void* src, uint64_t nbytes, uint32_t key, int threads, int blocks, void* sink,
         hipStream_t s) {
    switch (u) {
        case 1: return launch<MODE, NT, 1>(dst, src, nbytes, key, threads, blocks, sink, s);
        case 2: return launch<MODE, NT, 2>(dst, src, nbytes, key, threads, blocks, sink, s);
        case 4: return launch<MODE, NT, 4>(dst, src, nbytes, key, threads, blocks, sink, s);
        case 8: return launch<MODE, NT, 8>(dst, src, nbytes, key, threads, blocks, sink, s);
        default: return -1;
    }
}

template <int MODE>
int by_nt(int nt, int u, void* dst, const void* src, uint64_t nbytes, uint32_t key, int threads, int blocks,
          void* sink, hipStream_t s) {
    return nt ? by_u<MODE, true>(u, dst, src, nbytes, key, threads, blocks, sink, s)
              : by_u<MODE, false>(u, dst, src, nbytes, key, threads, blocks, sink, s);
}

// Walk variants (diagnostic sweep, tools/ceiling_sweep.py --walk): every wavefront
// takes k consecutive chunks of U KiB (persistent == 0) or chunks w, w + W, ...
// (persistent != 0); PIPE issues chunk i + 1's loads before chunk i's stores.
// Dynamic LDS (lds_bytes) only limits how many workgroups a CU holds.
template <int MODE, bool NT, int U, bool PIPE>
__global__ __launch_bounds__(1024) void walk_kernel(u32x4* dst_, const u32x4* src_, uint64_t nchunks, uint32_t key,
                                                    uint32_t k, int persistent, uint32_t* sink) {
    extern __shared__ uint32_t lds_pad[];
    G1 u32x4* dst = (G1 u32x4*)dst_;
    const G1 u32x4* src = (const G1 u32x4*)src_;
    const u32x4 kk = {key, key, key, key};
    const int lane = threadIdx.x & 63;
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    u32x4 acc = {0, 0, 0, 0};
    uint64_t c, stride, end;
    if (persistent) {
        c = wave;
        stride = nwaves;
        end = nchunks;
    } else {
        c = wave * k;
        stride = 1;
        end = c + k < nchunks ? c + k : nchunks;
    }
    if (c >= end) return;
    auto loadc = [&](u32x4(&d)[U], uint64_t cc) {
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = ld<NT>(src + cc * (64 * U) + 64 * u + lane);
    };
    auto storec = [&](const u32x4(&d)[U], uint64_t cc) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            G1 u32x4* q = dst + cc * (64 * U) + 64 * u + lane;
            if constexpr (MODE == 0) st<NT>(q, d[u]);
            else if constexpr (MODE == 1 || MODE == 2) st<NT>(q, d[u] ^ kk);
            else if constexpr (MODE == 3) acc ^= d[u];
            else st<NT>(q, kk);
        }
    };
    u32x4 d[U];
    if constexpr (PIPE) {
        if constexpr (MODE != 4) loadc(d, c);
        for (uint64_t cn = c + stride; cn < end; cn += stride) {
            u32x4 dn[U];
            if constexpr (MODE != 4) loadc(dn, cn);
            storec(d, c);
            c = cn;
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = dn[u];
        }
        storec(d, c);
    } else {
        for (; c < end; c += stride) {
            if constexpr (MODE != 4) loadc(d, c);
            storec(d, c);
        }
    }
    if constexpr (MODE == 3) {
        const uint32_t r = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
        if (r == 0x9E3779B9u) sink[wave & 1023] = r;
    }
    if (lds_pad[0] == 0x9E3779B9u && lane == 64) sink[0] = 1;   // never true; keeps the LDS allocation
}

template <int MODE, bool NT, int U, bool PIPE>
int launch_walk(void* dst, const void* src, uint64_t nbytes, uint32_t key, int threads, int blocks, int k,
                int lds_bytes, void* sink, hipStream_t s) {
    const uint64_t nchunks = nbytes / (1024ull * U);
    if (nchunks == 0) return 0;
    const int wpb = threads / 64;
    if (k < 1) k = 1;
    int persistent = 0;
    uint64_t grid;
    if (blocks >= 0) {
        persistent = 1;
        if (blocks == 0) {
            int per_cu = 0, cus = 0, dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, walk_kernel<MODE, NT, U, PIPE>, threads,
                                                             lds_bytes) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                return -2;
            blocks = per_cu * cus;
        }
        grid = (uint64_t)blocks;
        const uint64_t need = (nchunks + wpb - 1) / wpb;
        if (grid > need) grid = need;
    } else {
        const uint64_t waves = (nchunks + k - 1) / k;
        grid = (waves + wpb - 1) / wpb;
    }
    hipLaunchKernelGGL((walk_kernel<MODE, NT, U, PIPE>), dim3((unsigned)grid), dim3(threads), lds_bytes, s,
                       (u32x4*)dst, (const u32x4*)src, nchunks, key, (uint32_t)k, persistent, (uint32_t*)sink);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int MODE, bool NT, bool PIPE>
int walk_by_u(int u, void* dst, const void* src, uint64_t nbytes, uint32_t key, int threads, int blocks, int k,
              int lds, void* sink, hipStream_t s) {
    switch (u) {
        case 1: return launch_walk<MODE, NT, 1, PIPE>(dst, src, nbytes, key, threads, blocks, k, lds, sink, s);
        case 2: return launch_walk<MODE, NT, 2, PIPE>(dst, src, nbytes, key, threads, blocks, k, lds, sink, s);
        case 4: return launch_walk<MODE, NT, 4, PIPE>(dst, src, nbytes, key, threads, blocks, k, lds, sink, s);
        default: return -1;
    }
}

template <int MODE>
int walk_by_flags(int nt, int pipe, int u, void* dst, const void* src, uint64_t nbytes, uint32_t key, int threads,
                  int blocks, int k, int lds, void* sink, hipStream_t s) {
    if (nt) {
        return pipe ? walk_by_u<MODE, true, true>(u, dst, src, nbytes, key, threads, blocks, k, lds, sink, s)
                    : walk_by_u<MODE, true, false>(u, dst, src, nbytes, key, threads, blocks, k, lds, sink, s);
    }
    return pipe ? walk_by_u<MODE, false, true>(u, dst, src, nbytes, key, threads, blocks, k, lds, sink, s)
                : walk_by_u<MODE, false, false>(u, dst, src, nbytes, key, threads, blocks, k, lds, sink, s);
}

}  // namespace

// Diagnostic walk sweep: blocks < 0 = each wavefront k consecutive chunks (grid covers the
// buffer), blocks >= 0 = persistent grid-stride (0 = one resident round).
extern "C" int netc_ceiling_walk(int mode, int nt, int u, int pipe, int k, int threads, int blocks, int lds_bytes,
                                 void* dst, const void* src, uint64_t nbytes, uint32_t key, void* sink, void* stream) {
    if (threads < 64 || threads > 1024 || threads % 64 || lds_bytes < 4 || lds_bytes > 65536) return -1;
    hipStream_t s = (hipStream_t)stream;
    switch (mode) {
        case 0: return walk_by_flags<0>(nt, pipe, u, dst, src, nbytes, key, threads, blocks, k, lds_bytes, sink, s);
        case 1: return walk_by_flags<1>(nt, pipe, u, dst, dst, nbytes, key, threads, blocks, k, lds_bytes, sink, s);
        case 2: return walk_by_flags<2>(nt, pipe, u, dst, src, nbytes, key, threads, blocks, k, lds_bytes, sink, s);
        default: return -1;
    }
}

// Returns 0, or -1 (bad argument), -2 (occupancy query failed), -3 (launch failed).
// nbytes is rounded down to whole chunks of u KiB; threads is 64..1024, a multiple of 64.
extern "C" int netc_ceiling_stream(int mode, int nt, int u, int threads, int blocks, void* dst, const void* src,
                                   uint64_t nbytes, uint32_t key, void* sink, void* stream) {
    if (threads < 64 || threads > 1024 || threads % 64) return -1;
    hipStream_t s = (hipStream_t)stream;
    switch (mode) {
        case 0: return by_nt<0>(nt, u, dst, src, nbytes, key, threads, blocks, sink, s);
        case 1: return by_nt<1>(nt, u, dst, dst, nbytes, key, threads, blocks, sink, s);
        case 2: return by_nt<2>(nt, u, dst, src, nbytes, key, threads, blocks, sink, s);
        case 3: return by_nt<3>(nt, u, dst, src, nbytes, key, threads, blocks, sink, s);
        case 4: return by_nt<4>(nt, u, dst, src, nbytes, key, threads, blocks, sink, s);
        default: return -1;
    }
}
