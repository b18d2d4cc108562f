// microbench_sha.hip -- SHA-256 compression throughput / latency on gfx950.
//
// Registers only (no memory in the loop): each lane runs `iters` dependent
// compressions on ILP independent states.  Varying the workgroups per CU
// (waves per SIMD) and ILP tells how many waves the round function needs to
// keep the VALU busy, and the single-wave latency of one compression (which
// bounds the serial top levels of a tree).  Build & run on the box:
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_sha.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../immustore_amd/csrc/sha256_cdna.hpp"

using namespace mh;

template <int ILP>
__global__ __launch_bounds__(256) void k_bench(uint32_t *out, int iters, uint32_t seed) {
    State s[ILP];
    uint32_t w[16];
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = seed * (j + 1) + t;
#pragma unroll
    for (int k = 0; k < ILP; k++) {
        s[k].init();
        s[k].h[0] ^= k;
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < ILP; k++) compress(s[k], w);
        w[0] ^= s[0].h[1];
        w[5] += s[ILP - 1].h[2];
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < ILP; k++)
#pragma unroll
        for (int j = 0; j < 8; j++) x ^= s[k].h[j];
    out[t] = x;
}

template <int ILP>
static double run(int blocks, int threads, int iters, uint32_t *d) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k_bench<ILP>, dim3(blocks), dim3(threads), 0, 0, d, 2, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_bench<ILP>, dim3(blocks), dim3(threads), 0, 0, d, iters, 1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 256 * 1024 * 64 * sizeof(uint32_t));
    const int iters = 2000;
    printf("# lanes x ILP x iters compressions; Gcomp/s = compressions / time\n");
    // latency: one wave on the whole chip
    {
        double ms = run<1>(1, 64, iters, d);
        printf("latency 1 wave ILP1: %.1f ns per compression\n", ms * 1e6 / iters);
        ms = run<2>(1, 64, iters, d);
        printf("latency 1 wave ILP2: %.1f ns per compression pair\n", ms * 1e6 / iters);
    }
    for (int wps : {1, 2, 3, 4, 5, 6, 8}) {  // waves per SIMD
        const int blocks = 256 * wps;     // 256-thread blocks: one wave per SIMD each
        double ms1 = run<1>(blocks, 256, iters, d);
        double ms2 = run<2>(blocks, 256, iters, d);
        const double comps = (double)blocks * 256 * iters;
        printf("waves/SIMD %d: ILP1 %.1f Gcomp/s   ILP2 %.1f Gcomp/s\n", wps, comps / ms1 / 1e6,
               2 * comps / ms2 / 1e6);
    }
    hipFree(d);
    return 0;
}
