// microbench_valu.hip -- issue throughput of the integer VALU instructions the
// SHA-256 round uses, on gfx950 (8 independent dependency chains per lane,
// 4 waves per SIMD, inline asm so the exact opcode is measured).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu.hip -o mbv && ./mbv
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHAINS8(OP)                                                                               \
    asm volatile(OP : "+v"(a0) : "v"(b), "v"(c));                                                \
    asm volatile(OP : "+v"(a1) : "v"(b), "v"(c));                                                \
    asm volatile(OP : "+v"(a2) : "v"(b), "v"(c));                                                \
    asm volatile(OP : "+v"(a3) : "v"(b), "v"(c));                                                \
    asm volatile(OP : "+v"(a4) : "v"(b), "v"(c));                                                \
    asm volatile(OP : "+v"(a5) : "v"(b), "v"(c));                                                \
    asm volatile(OP : "+v"(a6) : "v"(b), "v"(c));                                                \
    asm volatile(OP : "+v"(a7) : "v"(b), "v"(c));

#define KERNEL(NAME, OP)                                                                          \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, int iters) {                       \
        uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;                                       \
        uint32_t a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, \
                 a7 = t + 7, b = t * 3, c = t * 5;                                                \
        for (int i = 0; i < iters; i++) {                                                         \
            CHAINS8(OP) CHAINS8(OP) CHAINS8(OP) CHAINS8(OP)                                       \
        }                                                                                         \
        out[t] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                           \
    }

KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_alignbit_same, "v_alignbit_b32 %0, %0, %0, 7")
KERNEL(k_alignbit_diff, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 3, %0")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")

typedef void (*kfn)(uint32_t *, int);

static void run(const char *name, kfn k, uint32_t *d) {
    const int iters = 4000, blocks = 256 * 4;  // 4 waves per SIMD
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 10);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double wave_instr = (double)blocks * 4 * iters * 32;  // waves x instr per wave
    const double per_simd = wave_instr / 1024.0;
    printf("%-16s %.3f ms  %.2f G wave-instr/s per SIMD  (%.2f ns each)\n", name, ms,
           per_simd / (ms * 1e6), ms * 1e6 / per_simd);
}

int main() {
    uint32_t *d;
    (void)hipMalloc(&d, 1 << 24);
    run("v_add_u32", k_add, d);
    run("v_xor_b32", k_xor, d);
    run("v_add3_u32", k_add3, d);
    run("v_bitop3_b32", k_bitop3, d);
    run("v_alignbit same", k_alignbit_same, d);
    run("v_alignbit diff", k_alignbit_diff, d);
    run("v_lshrrev_b32", k_lshr, d);
    run("v_perm_b32", k_perm, d);
    (void)hipFree(d);
    return 0;
}
