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
__global__ __launch_bounds__(256) void k_bench(uint32_t *out, int iters, uint32_t seed,
                                               unsigned long long *clk) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
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
    if (t == 0 && clk) {  // shader cycles and 100 MHz wall clock over block 0's life
        clk[0] = __builtin_amdgcn_s_memtime() - c0;
        clk[1] = wall_clock64() - w0;
    }
}

static unsigned long long *g_clk;
static double g_mhz;

// best of `reps` timed launches (after one short launch); the shader clock of
// block 0 during the best one
template <int ILP>
static double run(int blocks, int threads, int iters, uint32_t *d, int reps = 5) {
    double best = 1e30;
    for (int r = 0; r < reps; r++) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipLaunchKernelGGL(k_bench<ILP>, dim3(blocks), dim3(threads), 0, 0, d, 2, 1u, nullptr);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_bench<ILP>, dim3(blocks), dim3(threads), 0, 0, d, iters, 1u, g_clk);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        hipEventDestroy(a);
        hipEventDestroy(b);
        if (ms < best) {
            unsigned long long c[2];
            hipMemcpy(c, g_clk, sizeof c, hipMemcpyDeviceToHost);
            best = ms;
            g_mhz = c[1] ? 100.0 * (double)c[0] / (double)c[1] : 0;
        }
    }
    return best;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 256 * 1024 * 64 * sizeof(uint32_t));
    hipMalloc(&g_clk, 2 * sizeof(unsigned long long));
    const int iters = 2000;
    printf("# lanes x ILP x iters compressions; Gcomp/s = compressions / time\n");
    // warm the clock: ~1 s of the full-chip loop before anything is timed (a
    // cold GPU runs ~2.1 GHz, a warm one ~2.37: the ceiling must be the warm one)
    {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        float total = 0;
        while (total < 1000.f) {
            float ms = 0;
            hipEventRecord(a);
            hipLaunchKernelGGL(k_bench<1>, dim3(2048), dim3(256), 0, 0, d, iters, 1u, nullptr);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
            total += ms;
        }
        printf("# pre-warm: %.0f ms of the 8 waves/SIMD loop\n", total);
    }
    // latency: one wave on the whole chip
    {
        double ms = run<1>(1, 64, iters, d);
        printf("latency 1 wave ILP1: %.1f ns per compression (shader clock %.0f MHz)\n",
               ms * 1e6 / iters, g_mhz);
    }
    for (int wps : {1, 2, 3, 4, 5, 6, 8}) {  // waves per SIMD
        const int blocks = 256 * wps;     // 256-thread blocks: one wave per SIMD each
        double ms1 = run<1>(blocks, 256, iters, d);
        const double mhz1 = g_mhz;
        const double comps = (double)blocks * 256 * iters;
        printf("waves/SIMD %d: ILP1 %.2f Gcomp/s (shader clock %.0f MHz)\n", wps,
               comps / ms1 / 1e6, mhz1);
    }
    hipFree(d);
    hipFree(g_clk);
    return 0;
}
