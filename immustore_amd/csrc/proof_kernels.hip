// proof_kernels.hip -- device-side proof generation:
// gathers of proof terms over the device-resident htree levels / ahtree dLog,
// one proof per lane, no hashing.
//
//   htree  (*HTree).InclusionProof            embedded/htree/htree.go:121-164
//   ahtree inclusionProof / consistencyProof  embedded/ahtree/ahtree.go:547-651
//          highestNode                        ahtree.go:653-661
//
// Go builds every proof by PREPENDING terms; both ahtree recursions are tail
// calls, so a proof is the reverse of the sequence in which the loops below
// meet its terms.  Each kernel walks twice: once to count, once to copy each
// term to position count-1-q (no per-lane arrays, no scratch).
#include "digest_io.hpp"
#include "mh_internal.hpp"

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

__device__ __forceinline__ int bits_len(uint64_t x) { return x ? 64 - __clzll(x) : 0; }

// offset (in nodes) of level `layer` in the flat level-major layout of width w
__device__ __forceinline__ uint64_t level_off(uint64_t w, int layer) {
    uint64_t o = 0;
    for (int j = 0; j < layer; j++) o += (w + (1ull << j) - 1) >> j;
    return o;
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
    uint32_t cnt = 0;
    for (int pass = 0; pass < 2; pass++) {
        uint64_t m = i, nn = w, offset = 0;
        uint32_t q = 0;
        if (w > 1) {
            for (;;) {
                const int d = bits_len(nn - 1);
                const uint64_t k = 1ull << (d - 1);
                uint64_t l, r;
                if (m < k) {
                    l = offset + k;
                    r = offset + nn - 1;
                    nn = k;
                } else {
                    l = offset;
                    r = offset + k - 1;
                    m -= k;
                    nn -= k;
                    offset += k;
                }
                if (pass == 1) {
                    const int layer = bits_len(r - l);
                    const uint64_t idx = level_off(w, layer) + (l >> layer);
                    copy32(terms + ((uint64_t)p * max_terms + (cnt - 1 - q)) * 32, levels + idx * 32);
                }
                q++;
                if (nn < 1 || (nn == 1 && m == 0)) break;
            }
        }
        if (pass == 0) {
            cnt = q;
            if (cnt > max_terms) {
                status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
                nterms[p] = cnt;
                return;
            }
        }
    }
    nterms[p] = cnt;
    status[p] = MH_OK;
}

__device__ __forceinline__ uint64_t aht_node_index(uint64_t n, int l) {
    return (n <= 1 ? 0 : ahtree_nodes_upto_dev(n - 1)) + (uint64_t)l;
}

// highestNode(i, d): node(i, popcount((i-1) & (2^d - 1)))  (ahtree.go:653-661)
__device__ __forceinline__ uint64_t aht_highest(uint64_t i, int d) {
    const uint64_t mask = d >= 64 ? ~0ull : ((1ull << d) - 1);
    return aht_node_index(i, __popcll((i - 1) & mask));
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
    uint32_t cnt = 0;
    for (int pass = 0; pass < 2; pass++) {
        uint32_t q = 0;
        auto emit = [&](uint64_t idx) {
            if (pass == 1) copy32(terms + ((uint64_t)p * max_terms + (cnt - 1 - q)) * 32, dlog + idx * 32);
            q++;
        };
        uint64_t j = j0;
        int height = bits_len(j0 - 1);
        bool done = false;
        while (!done) {
            bool restarted = false;
            for (int h = height - 1; h >= 0 && !restarted && !done; h--) {
                if (!((j - 1) & (1ull << h))) continue;
                const uint64_t k = (j - 1) >> h << h;
                if (i <= k) {
                    emit(aht_highest(j, h));
                    if (kind == 0 || i < k) {  // tail call on (i, k, h)
                        j = k;
                        height = h;
                        restarted = true;
                    } else {                    // consistency, i == k
                        emit(aht_highest(i, h));
                        done = true;
                    }
                } else {
                    emit(aht_node_index(k, h));
                    if (kind == 1 && i == j) {
                        emit(aht_highest(i, h));
                        done = true;
                    }
                }
            }
            if (!restarted) done = true;
        }
        if (pass == 0) {
            cnt = q;
            if (cnt > max_terms) {
                status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
                nterms[p] = cnt;
                return;
            }
        }
    }
    nterms[p] = cnt;
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
