// Diagnostic: the cost of back-to-back dependent launches on one stream, by grid
// size, for kernels that do (almost) nothing -- the floor under every extra launch
// of the multi-kernel rows (frame scan, frame assembly).  Prints one JSON line per
// grid size: microseconds per launch from HIP events over 2000 launches.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void flag_exit(const unsigned* flag, unsigned* out) {
    if (*flag) out[blockIdx.x * blockDim.x + threadIdx.x] = 1;   // never taken
}

int main() {
    unsigned *flag, *out;
    if (hipMalloc(&flag, 4) != hipSuccess || hipMalloc(&out, 64u << 20) != hipSuccess) return 1;
    hipMemset(flag, 0, 4);
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grids[] = {1, 8, 64, 256, 1024, 4096, 16384};
    const int reps = 2000;
    for (int g : grids) {
        for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(flag_exit, dim3(g), dim3(256), 0, s, flag, out);
        hipEventRecord(e0, s);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(flag_exit, dim3(g), dim3(256), 0, s, flag, out);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"blocks\": %d, \"threads_per_block\": 256, \"us_per_launch\": %.3f}\n", g, ms * 1000.0 / reps);
    }
    return 0;
}
