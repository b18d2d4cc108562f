// wg_trace.hip -- workgroup timeline of one isolated k_entries_fixed launch
// (BASELINE configs[1]: 2^20 x 1 KiB entries, 8-byte keys, v1): for every
// workgroup its XCC, CU, and wall-clock (100 MHz) start, end of the leaf
// phase and end, through the MH_WG_PROBE hook of htree_kernels.hip.  Shows
// where an isolated launch loses time against three builds in flight
// (dispatch ramp, per-XCC speed, the workgroup subtree, the last stragglers).
// Prints one JSON object.  Build: tools/Makefile (wg_trace).
#include <cstdio>
#include <vector>

// per workgroup: wall clock at probe points 0..2, XCC << 32 | CU, shader-clock
// cycles at points 0 and 2 (s_memtime) -> the clock the workgroup ran at
__device__ unsigned long long g_probe[8 * 4096];
__device__ const uint8_t *g_traced_levels;  // only the launch writing these levels records

#define MH_WG_PROBE(point)                                                                     \
    do {                                                                                       \
        if (threadIdx.x == 0 && levels == g_traced_levels) {                                   \
            g_probe[8 * blockIdx.x + ((point) == 3 ? 6 : (point))] = wall_clock64();           \
            if ((point) == 0) {                                                                \
                const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));   \
                g_probe[8 * blockIdx.x + 3] = ((unsigned long long)xcc << 32) | __smid();      \
                g_probe[8 * blockIdx.x + 4] = clock64();                                       \
            }                                                                                  \
            if ((point) == 2) g_probe[8 * blockIdx.x + 5] = clock64();                         \
        }                                                                                      \
    } while (0)

#include "../immustore_amd/csrc/htree_kernels.hip"

int main(int argc, char **argv) {
    // argv[1]: warm-up builds with 3 in flight before the traced launch (heats
    // the GPU to its steady clock); argv[2]: 1 = trace a launch with two more
    // builds in flight on other streams, 0 = an isolated launch
    const uint64_t n = 1ull << 20, vlen = 1024, klen = 8;
    const int warm = argc > 1 ? atoi(argv[1]) : 0;
    const int contended = argc > 2 ? atoi(argv[2]) : 0;
    uint8_t *vals, *keys, *levels[3];
    mh::LevelGeom g;
    g.init(n);
    if (hipMalloc(&vals, n * vlen + 64) || hipMalloc(&keys, n * klen + 64)) return 1;
    for (int k = 0; k < 3; k++)
        if (hipMalloc(&levels[k], g.total * 32 + 64)) return 1;
    hipStream_t st[3];
    for (int k = 0; k < 3; k++) hipStreamCreate(&st[k]);
    mh::launch_fill_random(st[0], vals, n * vlen, 2);
    mh::launch_fill_keys_be64(st[0], keys, n, 0);
    const uint8_t *tl = levels[0];
    hipMemcpyToSymbol(HIP_SYMBOL(g_traced_levels), &tl, sizeof(tl));
    hipDeviceSynchronize();
    int done = 0;
    for (int r = 0; r < warm; r++)
        for (int k = 1; k < 3; k++)
            if (mh::launch_entries_fixed(st[k], nullptr, 1, n, keys, (uint32_t)klen, vals,
                                         (uint32_t)vlen, nullptr, levels[k], g, &done) != hipSuccess)
                return 2;
    hipDeviceSynchronize();
    // the traced launch on stream 0 (levels[0]); with `contended`, the other
    // two streams get two builds each around it
    if (contended)
        for (int k = 1; k < 3; k++)
            mh::launch_entries_fixed(st[k], nullptr, 1, n, keys, (uint32_t)klen, vals,
                                     (uint32_t)vlen, nullptr, levels[k], g, &done);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, st[0]);
    if (mh::launch_entries_fixed(st[0], nullptr, 1, n, keys, (uint32_t)klen, vals, (uint32_t)vlen,
                                 nullptr, levels[0], g, &done) != hipSuccess)
        return 2;
    hipEventRecord(b, st[0]);
    if (contended)
        for (int k = 1; k < 3; k++)
            mh::launch_entries_fixed(st[k], nullptr, 1, n, keys, (uint32_t)klen, vals,
                                     (uint32_t)vlen, nullptr, levels[k], g, &done);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> p(8 * 4096);
    hipMemcpyFromSymbol(p.data(), HIP_SYMBOL(g_probe), p.size() * 8);
    // entries per lane as choose_lpl picks them (MH_LPL, else 2 from 2^19 up)
    const char *le = getenv("MH_LPL");
    const uint64_t lpl = le ? (uint64_t)atoi(le) : (n >= (1ull << 19) ? 2 : 1);
    const unsigned nwg = (unsigned)((n / lpl + 255) / 256);
    printf("{\"warm\": %d, \"contended\": %d, \"kernel_ms\": %.4f, \"workgroups\": %u, "
           "\"lpl\": %llu, \"clock_mhz\": 100, \"wg\": [", warm, contended, ms, nwg,
           (unsigned long long)lpl);
    for (unsigned w = 0; w < nwg; w++)
        printf("%s[%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu]", w ? "," : "", p[8 * w + 3] >> 32,
               p[8 * w + 3] & 0xffffffffull, p[8 * w], p[8 * w + 1], p[8 * w + 2], p[8 * w + 4],
               p[8 * w + 5], p[8 * w + 6]);
    printf("]}\n");
    return 0;
}
