// verify_kernels.hip -- batch proof re-hash on CDNA4, one proof per lane.
//
//   htree.VerifyInclusion          embedded/htree/htree.go:166-195
//   ahtree.VerifyInclusion / EvalInclusion           ahtree/verification.go:21-56
//   ahtree.VerifyConsistency / EvalConsistency       ahtree/verification.go:58-109
//   ahtree.VerifyLastInclusion / EvalLastInclusion   ahtree/verification.go:111-137
// The left/right choice of every step is a per-lane select of the operands
// of ONE node_hash call, so lanes of a wave never diverge on it.
#include "digest_io.hpp"
#include "mh_internal.hpp"

namespace mh {

__device__ __forceinline__ bool eq8(const uint32_t a[8], const uint32_t b[8]) {
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) x |= a[j] ^ b[j];
    return x == 0;
}

__global__ __launch_bounds__(256) void k_htree_verify(uint64_t np, const uint64_t *__restrict__ leaf,
                                                      const uint64_t *__restrict__ width,
                                                      const uint64_t *__restrict__ term_off,
                                                      const uint8_t *__restrict__ terms,
                                                      const uint8_t *__restrict__ digests,
                                                      const uint8_t *__restrict__ roots,
                                                      uint8_t *__restrict__ ok) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    uint32_t d[8], calc[8], root[8];
    load_digest(digests + p * 32, d);
    leaf_hash(d, calc);
    uint64_t i = leaf[p], r = width[p] - 1;
    const uint64_t t0 = term_off[p], t1 = term_off[p + 1];
    for (uint64_t t = t0; t < t1; t++) {
        uint32_t term[8], l[8], rr[8];
        load_digest(terms + t * 32, term);
        const bool calc_left = (i % 2 == 0) && (i != r);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            l[j] = calc_left ? calc[j] : term[j];
            rr[j] = calc_left ? term[j] : calc[j];
        }
        node_hash(l, rr, calc);
        i >>= 1;
        r >>= 1;
    }
    load_digest(roots + p * 32, root);
    ok[p] = (i == r) && eq8(calc, root);
}

__global__ __launch_bounds__(256) void k_ahtree_verify(int kind, uint64_t np,
                                                       const uint64_t *__restrict__ vi,
                                                       const uint64_t *__restrict__ vj,
                                                       const uint64_t *__restrict__ term_off,
                                                       const uint8_t *__restrict__ terms,
                                                       const uint8_t *__restrict__ va,
                                                       const uint8_t *__restrict__ vb,
                                                       uint8_t *__restrict__ ok,
                                                       uint8_t *__restrict__ eval_out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    const uint64_t i = vi[p], j = vj[p];
    const uint64_t t0 = term_off[p], t1 = term_off[p + 1], len = t1 - t0;
    uint32_t a[8], b[8];
    load_digest(va + p * 32, a);
    load_digest(vb + p * 32, b);
    bool res = false;
    if (kind == MH_AHT_INCLUSION) {
        // verification.go:21-56
        uint32_t c[8];
        copy8(c, a);
        if (!(i > j || i == 0 || (i < j && len == 0))) {
            uint64_t i1 = i - 1, j1 = j - 1;
            for (uint64_t t = t0; t < t1; t++) {
                uint32_t h[8], l[8], r[8];
                load_digest(terms + t * 32, h);
                const bool c_left = (i1 % 2 == 0) && (i1 != j1);
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    l[k] = c_left ? c[k] : h[k];
                    r[k] = c_left ? h[k] : c[k];
                }
                node_hash(l, r, c);
                i1 >>= 1;
                j1 >>= 1;
            }
            res = eq8(c, b);
        }
        if (eval_out) store_digest(eval_out + p * 32, c);
    } else if (kind == MH_AHT_LAST_INCLUSION) {
        // verification.go:111-137 (every term is a left sibling)
        uint32_t c[8];
        copy8(c, a);
        for (uint64_t t = t0; t < t1; t++) {
            uint32_t h[8];
            load_digest(terms + t * 32, h);
            node_hash(h, c, c);
        }
        res = (i != 0) && eq8(c, b);
        if (eval_out) store_digest(eval_out + p * 32, c);
    } else {
        // verification.go:58-109
        uint32_t ci[8] = {0, 0, 0, 0, 0, 0, 0, 0}, cj[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i > j || i == 0 || (i < j && len == 0)) {
            res = false;
        } else if (i == j && len == 0) {
            res = eq8(a, b);
        } else {
            uint64_t fn = i - 1, sn = j - 1;
            while (fn % 2 == 1) {
                fn >>= 1;
                sn >>= 1;
            }
            load_digest(terms + t0 * 32, ci);
            copy8(cj, ci);
            for (uint64_t t = t0 + 1; t < t1; t++) {
                uint32_t h[8], l[8], r[8];
                load_digest(terms + t * 32, h);
                const bool both = (fn % 2 == 1) || (fn == sn);
                if (both) node_hash(h, ci, ci);
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    l[k] = both ? h[k] : cj[k];
                    r[k] = both ? cj[k] : h[k];
                }
                node_hash(l, r, cj);
                if (both) {
                    while (fn % 2 == 0 && fn != 0) {
                        fn >>= 1;
                        sn >>= 1;
                    }
                }
                fn >>= 1;
                sn >>= 1;
            }
            res = eq8(a, ci) && eq8(b, cj);
        }
        if (eval_out) {
            store_digest(eval_out + p * 64, ci);
            store_digest(eval_out + p * 64 + 32, cj);
        }
    }
    ok[p] = res ? 1 : 0;
}

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

hipError_t launch_htree_verify(hipStream_t st, Timer *tm, uint64_t np, const uint64_t *leaf,
                               const uint64_t *width, const uint64_t *term_off,
                               const uint8_t *terms, const uint8_t *digests, const uint8_t *roots,
                               uint8_t *ok) {
    if (tm) tm->begin("htree_verify", st);
    hipLaunchKernelGGL(k_htree_verify, dim3(grid_for(np, 256)), dim3(256), 0, st, np, leaf, width,
                       term_off, terms, digests, roots, ok);
    if (tm) tm->end(st);
    return hipGetLastError();
}

hipError_t launch_ahtree_verify(hipStream_t st, Timer *tm, int kind, uint64_t np,
                                const uint64_t *i, const uint64_t *j, const uint64_t *term_off,
                                const uint8_t *terms, const uint8_t *a, const uint8_t *b,
                                uint8_t *ok, uint8_t *eval_out) {
    if (tm) tm->begin("ahtree_verify", st);
    hipLaunchKernelGGL(k_ahtree_verify, dim3(grid_for(np, 256)), dim3(256), 0, st, kind, np, i, j,
                       term_off, terms, a, b, ok, eval_out);
    if (tm) tm->end(st);
    return hipGetLastError();
}

}  // namespace mh
