// proof_kernels.hip -- device-side proof generation:
// gathers of proof terms over the device-resident htree levels / ahtree dLog,
// one proof per lane, no hashing.  The index walks (htree.go:121-164,
// ahtree.go:547-661) are in proof_walk.hpp.  Each kernel walks twice: once
// to count, once to copy each term to position count-1-q (no per-lane
// arrays, no scratch).
#include "digest_io.hpp"
#include "mh_internal.hpp"
#include "proof_walk.hpp"

namespace mh {

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

__device__ __forceinline__ void copy32(uint8_t *__restrict__ d, const uint8_t *__restrict__ s) {
    const uint4 *a = reinterpret_cast<const uint4 *>(s);
    uint4 *b = reinterpret_cast<uint4 *>(d);
    b[0] = a[0];
    b[1] = a[1];
}

// htree.go:121-164 for leaf[p] of one tree of width w.
__global__ __launch_bounds__(256) void k_htree_proof(const uint8_t *__restrict__ levels, uint64_t w,
                                                     uint64_t n, const uint64_t *__restrict__ leaf,
                                                     uint8_t *__restrict__ terms,
                                                     uint32_t max_terms,
                                                     uint32_t *__restrict__ nterms,
                                                     int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t i = leaf[p];
    if (i >= w) {
        status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
        nterms[p] = 0;
        return;
    }
    const uint32_t cnt = htree_walk(i, w, [](uint32_t, uint64_t) {});
    nterms[p] = cnt;
    if (cnt > max_terms) {
        status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
        return;
    }
    uint8_t *out = terms + (uint64_t)p * max_terms * 32;
    htree_walk(i, w, [&](uint32_t q, uint64_t idx) {
        copy32(out + (uint64_t)(cnt - 1 - q) * 32, levels + idx * 32);
    });
    status[p] = MH_OK;
}

// ahtree.go:547-577 (kind 0) and :599-651 (kind 1) over the device dLog.
__global__ __launch_bounds__(256) void k_ahtree_proof(int kind, const uint8_t *__restrict__ dlog,
                                                      uint64_t size, uint64_t n,
                                                      const uint64_t *__restrict__ vi,
                                                      const uint64_t *__restrict__ vj,
                                                      uint8_t *__restrict__ terms,
                                                      uint32_t max_terms,
                                                      uint32_t *__restrict__ nterms,
                                                      int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t i = vi[p], j0 = vj[p];
    // ahtree.go:535-541 / :589-595; j == 0 has no nodes to read (Go fails the read)
    if (i > j0 || j0 > size || j0 == 0) {
        status[p] = i > j0 ? MH_ERR_ILLEGAL_ARGUMENTS : MH_ERR_UNEXISTENT_DATA;
        nterms[p] = 0;
        return;
    }
    const bool cons = kind == 1;
    const uint32_t cnt = ahtree_walk(cons, i, j0, [](uint32_t, uint64_t) {});
    nterms[p] = cnt;
    if (cnt > max_terms) {
        status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
        return;
    }
    uint8_t *out = terms + (uint64_t)p * max_terms * 32;
    ahtree_walk(cons, i, j0, [&](uint32_t q, uint64_t idx) {
        copy32(out + (uint64_t)(cnt - 1 - q) * 32, dlog + idx * 32);
    });
    status[p] = MH_OK;
}

hipError_t launch_htree_proof(hipStream_t st, Timer *tm, const uint8_t *levels, uint64_t w,
                              uint64_t n, const uint64_t *leaf, uint8_t *terms, uint32_t max_terms,
                              uint32_t *nterms, int32_t *status) {
    if (!n) return hipSuccess;
    TimerScope ts(tm, "htree_proof", st);
    hipLaunchKernelGGL(k_htree_proof, dim3(grid_for(n, 256)), dim3(256), 0, st, levels, w, n, leaf,
                       terms, max_terms, nterms, status);
    return hipGetLastError();
}

hipError_t launch_ahtree_proof(hipStream_t st, Timer *tm, int kind, const uint8_t *dlog,
                               uint64_t size, uint64_t n, const uint64_t *i, const uint64_t *j,
                               uint8_t *terms, uint32_t max_terms, uint32_t *nterms,
                               int32_t *status) {
    if (!n) return hipSuccess;
    TimerScope ts(tm, "ahtree_proof", st);
    hipLaunchKernelGGL(k_ahtree_proof, dim3(grid_for(n, 256)), dim3(256), 0, st, kind, dlog, size,
                       n, i, j, terms, max_terms, nterms, status);
    return hipGetLastError();
}

}  // namespace mh
