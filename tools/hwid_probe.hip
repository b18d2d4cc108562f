// hwid_probe.hip -- where do the waves of a k_entries_fixed-shaped launch land?
//
// Launches the same geometry as the C2 leaf kernel (1024 workgroups x 256
// threads, 33 KB of dynamic LDS each, so 4 workgroups per CU) and records, for
// every wave, its workgroup, its wave index and the hardware ids
// (HW_REG_HW_ID: wave slot, SIMD, CU, SH, SE; HW_REG_XCC_ID).  Each wave does
// a fixed amount of busy work so the workgroups are co-resident.  Output:
// one line per wave "blk wave hw_id xcc_id" on stdout.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

__global__ __launch_bounds__(256) void k_probe(uint32_t *out, uint32_t iters) {
    extern __shared__ uint32_t lds[];
    const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)); // XCC_ID
    uint32_t x = threadIdx.x;
    for (uint32_t i = 0; i < iters; i++) x = __builtin_amdgcn_alignbit(x, x, 7) + i;
    lds[threadIdx.x] = x;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = threadIdx.x >> 6;
        uint32_t *o = out + ((size_t)blockIdx.x * 4 + w) * 4;
        o[0] = blockIdx.x;
        o[1] = w;
        o[2] = hw;
        o[3] = xcc + (lds[(threadIdx.x + 64) & 255] == 12345u ? 1u : 0u) * 0;
    }
}

int main(int argc, char **argv) {
    const unsigned grid = argc > 1 ? atoi(argv[1]) : 1024;
    const size_t lds = argc > 2 ? atoi(argv[2]) : 4 * 8192 + 256;
    uint32_t *d;
    const size_t n = (size_t)grid * 4 * 4;
    if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), lds, 0, d, 200000u);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<uint32_t> h(n);
    hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < n; i += 4) printf("%u %u %u %u\n", h[i], h[i + 1], h[i + 2], h[i + 3]);
    hipFree(d);
    return 0;
}
