// verify_kernels.hip -- batch proof re-hash on CDNA4, one proof per lane.
//
//   htree.VerifyInclusion          embedded/htree/htree.go:166-195
//   ahtree.VerifyInclusion / EvalInclusion           ahtree/verification.go:21-56
//   ahtree.VerifyConsistency / EvalConsistency       ahtree/verification.go:58-109
//   ahtree.VerifyLastInclusion / EvalLastInclusion   ahtree/verification.go:111-137
// The left/right choice of every step is a per-lane select of the operands
// of ONE node_hash call, so lanes of a wave never diverge on it.
#include <algorithm>

#include "digest_io.hpp"
#include "mh_internal.hpp"

namespace mh {

__device__ __forceinline__ bool eq8(const uint32_t a[8], const uint32_t b[8]) {
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) x |= a[j] ^ b[j];
    return x == 0;
}

// Both kernels run grid-stride over the proofs with 512-thread workgroups that
// first build the node-tail schedule table in LDS (sha256_cdna.hpp).
__global__ __launch_bounds__(512) void k_htree_verify(uint64_t np, const uint64_t *__restrict__ leaf,
                                                      const uint64_t *__restrict__ width,
                                                      const uint64_t *__restrict__ term_off,
                                                      const uint8_t *__restrict__ terms,
                                                      const uint8_t *__restrict__ digests,
                                                      const uint8_t *__restrict__ roots,
                                                      uint8_t *__restrict__ ok) {
    extern __shared__ uint32_t tab[];
    node_tab_init(tab);
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < np;
         p += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t d[8], calc[8], root[8];
    load_digest(digests + p * 32, d);
    leaf_hash(d, calc);
    // Go's int arithmetic (htree.go:175-190): leaf / width are the bits of
    // a Go int; a negative one (a proof decoded from the wire) takes the
    // signed % and / (truncating), as Go does
    int64_t i = (int64_t)leaf[p], r = (int64_t)(width[p] - 1);
    // offsets running backwards (device CSR, unchecked by the host): no terms
    const uint64_t t0 = term_off[p], t1 = max(term_off[p + 1], t0);
    // the next term's load is issued before this step's node hash, so the
    // wave does not wait on HBM between two steps of its chain
    // (profiles/ab_c5_prefetch_r03.txt: +2.7 %)
    uint4 na = make_uint4(0, 0, 0, 0), nb = na;
    if (t0 < t1) {
        na = reinterpret_cast<const uint4 *>(terms + t0 * 32)[0];
        nb = reinterpret_cast<const uint4 *>(terms + t0 * 32)[1];
    }
    for (uint64_t t = t0; t < t1; t++) {
        uint32_t term[8], l[8], rr[8];
        term[0] = bswap(na.x); term[1] = bswap(na.y); term[2] = bswap(na.z); term[3] = bswap(na.w);
        term[4] = bswap(nb.x); term[5] = bswap(nb.y); term[6] = bswap(nb.z); term[7] = bswap(nb.w);
        if (t + 1 < t1) {
            na = reinterpret_cast<const uint4 *>(terms + (t + 1) * 32)[0];
            nb = reinterpret_cast<const uint4 *>(terms + (t + 1) * 32)[1];
        }
        const bool calc_left = (i % 2 == 0) && (i != r);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            l[j] = calc_left ? calc[j] : term[j];
            rr[j] = calc_left ? term[j] : calc[j];
        }
        node_hash_tab(l, rr, calc, tab);
        i /= 2;
        r /= 2;
    }
    load_digest(roots + p * 32, root);
    ok[p] = (i == r) && eq8(calc, root);
    }
}

// One node hash per loop iteration for all three kinds (a single inlined
// compression site keeps the kernel at full occupancy).  A consistency step
// over term h is up to two hashes: "A" (ci = H(h, ci), only when the first
// tree's path turns here) and "B" (cj = H(h, cj) or H(cj, h)); `phase`
// walks them in order.
// KIND is a template argument so that each kind is compiled on its own: the
// two inclusion kinds (one hash per term, no consistency state) then have the
// registers to load the next term under the current step's hash.
template <int KIND>
__global__ __launch_bounds__(512) void k_ahtree_verify(uint64_t np,
                                                       const uint64_t *__restrict__ vi,
                                                       const uint64_t *__restrict__ vj,
                                                       const uint64_t *__restrict__ term_off,
                                                       const uint8_t *__restrict__ terms,
                                                       const uint8_t *__restrict__ va,
                                                       const uint8_t *__restrict__ vb,
                                                       uint8_t *__restrict__ ok,
                                                       uint8_t *__restrict__ eval_out) {
    extern __shared__ uint32_t tab[];
    node_tab_init(tab);
    constexpr int kind = KIND;
    constexpr bool cons = kind == MH_AHT_CONSISTENCY;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < np;
         p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = vi[p], j = vj[p];
        // offsets running backwards (device CSR, unchecked by the host): no terms
        const uint64_t t0 = term_off[p], t1 = max(term_off[p + 1], t0), len = t1 - t0;
        uint32_t c[8], cj[8];
        // verification.go:22-24 / :59-61: argument checks shared by inclusion
        // and consistency; last inclusion only needs i != 0 (:112-114)
        const bool bad = i > j || i == 0 || (i < j && len == 0);
        uint64_t x = i - 1, y = j - 1;  // i1/j1 (inclusion) or fn/sn (consistency)
        uint64_t t = t0;
        bool run;
        if (kind == MH_AHT_INCLUSION) {
            load_digest(va + p * 32, c);
            run = !bad;
        } else if (kind == MH_AHT_LAST_INCLUSION) {
            load_digest(va + p * 32, c);
            run = true;
        } else {
#pragma unroll
            for (int k = 0; k < 8; k++) c[k] = cj[k] = 0;
            run = !bad && !(i == j && len == 0);
            if (run) {
                while (x % 2 == 1) {  // verification.go:71-74
                    x >>= 1;
                    y >>= 1;
                }
                load_digest(terms + t0 * 32, c);  // ci = cj = proof[0]
                copy8(cj, c);
                t = t0 + 1;
            }
        }
        int phase = 0;
        uint4 na = make_uint4(0, 0, 0, 0), nb = na;  // inclusion: term t, loaded one step ahead
        if (!cons && run && t < t1) {
            na = reinterpret_cast<const uint4 *>(terms + t * 32)[0];
            nb = reinterpret_cast<const uint4 *>(terms + t * 32)[1];
        }
        while (run && t < t1) {
            uint32_t h[8], L[8], R[8], o[8];
            if (cons) {
                load_digest(terms + t * 32, h);
            } else {
                h[0] = bswap(na.x); h[1] = bswap(na.y); h[2] = bswap(na.z); h[3] = bswap(na.w);
                h[4] = bswap(nb.x); h[5] = bswap(nb.y); h[6] = bswap(nb.z); h[7] = bswap(nb.w);
                if (t + 1 < t1) {
                    na = reinterpret_cast<const uint4 *>(terms + (t + 1) * 32)[0];
                    nb = reinterpret_cast<const uint4 *>(terms + (t + 1) * 32)[1];
                }
            }
            bool h_left, to_c;
            const bool both = (x % 2 == 1) || (x == y);
            if (!cons) {
                // inclusion: calc is the left operand iff i1 even and i1 != j1
                // (verification.go:37-45); last inclusion: always H(h, calc)
                h_left = kind == MH_AHT_LAST_INCLUSION || !((x % 2 == 0) && (x != y));
                to_c = true;
            } else {
                if (phase == 0 && !both) phase = 1;
                to_c = phase == 0;  // A: ci = H(h, ci)
                h_left = to_c || both;  // B: H(h, cj) if both else H(cj, h)
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t cur = to_c ? c[k] : cj[k];
                L[k] = h_left ? h[k] : cur;
                R[k] = h_left ? cur : h[k];
            }
            node_hash_tab(L, R, o, tab);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                c[k] = to_c ? o[k] : c[k];
                cj[k] = to_c ? cj[k] : o[k];
            }
            if (cons && phase == 0) {
                phase = 1;  // same term, hash B next
                continue;
            }
            if (cons && both) {  // verification.go:95-100
                while (x % 2 == 0 && x != 0) {
                    x >>= 1;
                    y >>= 1;
                }
            }
            x >>= 1;
            y >>= 1;
            t++;
            phase = 0;
        }
        uint32_t a[8], b[8];
        load_digest(va + p * 32, a);
        load_digest(vb + p * 32, b);
        bool res;
        if (kind == MH_AHT_INCLUSION)
            res = !bad && eq8(c, b);
        else if (kind == MH_AHT_LAST_INCLUSION)
            res = i != 0 && eq8(c, b);
        else if (bad)
            res = false;
        else if (i == j && len == 0)
            res = eq8(a, b);  // verification.go:63-65
        else
            res = eq8(a, c) && eq8(b, cj);
        if (eval_out) {
            if (cons) {
                store_digest(eval_out + p * 64, c);
                store_digest(eval_out + p * 64 + 32, cj);
            } else {
                store_digest(eval_out + p * 32, c);
            }
        }
        ok[p] = res ? 1 : 0;
    }
}

static unsigned resident_grid(const void *kern, int block, uint64_t work_items) {
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, kNodeTabBytes) !=
            hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const uint64_t need = (work_items + block - 1) / block;
    // a few resident waves of workgroups: the table build is amortised, the
    // tail of uneven proof lengths still balances
    const uint64_t cap = (uint64_t)cus * (uint64_t)per_cu * 4;
    return (unsigned)std::max<uint64_t>(1, std::min(need, cap));
}

hipError_t launch_htree_verify(hipStream_t st, Timer *tm, uint64_t np, const uint64_t *leaf,
                               const uint64_t *width, const uint64_t *term_off,
                               const uint8_t *terms, const uint8_t *digests, const uint8_t *roots,
                               uint8_t *ok) {
    if (!np) return hipSuccess;
    if (tm) tm->begin("htree_verify", st);
    hipLaunchKernelGGL(k_htree_verify, dim3(resident_grid((const void *)k_htree_verify, 512, np)),
                       dim3(512), kNodeTabBytes, st, np, leaf, width,
                       term_off, terms, digests, roots, ok);
    if (tm) tm->end(st);
    return hipGetLastError();
}

hipError_t launch_ahtree_verify(hipStream_t st, Timer *tm, int kind, uint64_t np,
                                const uint64_t *i, const uint64_t *j, const uint64_t *term_off,
                                const uint8_t *terms, const uint8_t *a, const uint8_t *b,
                                uint8_t *ok, uint8_t *eval_out) {
    if (!np) return hipSuccess;
    if (tm) tm->begin("ahtree_verify", st);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(resident_grid((const void *)kern, 512, np)), dim3(512),
                           kNodeTabBytes, st, np, i, j, term_off, terms, a, b, ok, eval_out);
    };
    if (kind == MH_AHT_INCLUSION) go(k_ahtree_verify<MH_AHT_INCLUSION>);
    else if (kind == MH_AHT_CONSISTENCY) go(k_ahtree_verify<MH_AHT_CONSISTENCY>);
    else go(k_ahtree_verify<MH_AHT_LAST_INCLUSION>);
    if (tm) tm->end(st);
    return hipGetLastError();
}

}  // namespace mh
