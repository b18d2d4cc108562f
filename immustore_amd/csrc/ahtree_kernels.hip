// ahtree_kernels.hip -- batch append for embedded/ahtree on CDNA4.
//
// Reference: embedded/ahtree/ahtree.go:246-373 (Append), :460-523 (node /
// nodesUntil / nodesUpto / levelsAt).  Appending n (1-based) writes
// 1 + popcount(n-1) digests at dLog[nodesUntil(n)]:
//   d_0 = SHA256(0x00 || payload_n)
//   for every set bit l of n-1, low to high:  d_{t+1} = SHA256(0x01 || node(k,l) || d_t)
//   with k = (n-1) with the bits below l cleared and node(k,l) = dLog[nodesUntil(k)+l].
// The first tz(n) of those steps combine a node with its own right sibling,
// i.e. they are the perfect subtree roots ending at n.  A batch of m appends
// is therefore computed in three data-parallel phases over the device dLog:
//   1. leaves        d_0 for every new n                       (m x 1 compression)
//   2. perfect nodes level by level, P(l, e) = H(P(l-1, e-2^(l-1)), P(l-1, e))
//                    stored at node(e, l)                        (~m node hashes)
//   3. spine         for every new n, the chain over the set bits of n-1 above
//                    tz(n), reading the (old or new) perfect nodes to its left
// which reproduces the reference's dLog byte stream exactly (tests compare it
// with Go's tree/00000000.sha fixtures and with the oracle).
#include <algorithm>

#include "digest_io.hpp"
#include "mh_internal.hpp"

namespace mh {

// S(x) = sum_{i<x} popcount(i): process the set bits of x from the top; the
// j-th set bit b (j = 1 for the highest) contributes b*2^(b-1) + (j-1)*2^b.
__host__ __device__ inline uint64_t popsum_below(uint64_t x) {
    uint64_t s = 0, j = 0;
    while (x) {
        const int b = 63 - __builtin_clzll(x);
        s += (b ? ((uint64_t)b << (b - 1)) : 0) + (j << b);
        j++;
        x &= ~(1ull << b);
    }
    return s;
}

// nodesUpto(n) = n + S(n)           (ahtree.go:492-511)
// nodesUntil(n) = nodesUpto(n - 1)  (ahtree.go:485-490)
__host__ __device__ inline uint64_t until_from_s(uint64_t n, uint64_t s_n) {
    return (n - 1) + s_n - (uint64_t)__builtin_popcountll(n - 1);
}

uint64_t ahtree_nodes_upto(uint64_t n) { return n + popsum_below(n); }
uint64_t ahtree_nodes_until(uint64_t n) { return n <= 1 ? 0 : ahtree_nodes_upto(n - 1); }

__device__ __forceinline__ uint64_t dev_nodes_until(uint64_t n) {
    return until_from_s(n, popsum_below(n));
}

// phase 1: d_0 = leaf of payload (plen == 32: one block, the store's Alh)
__global__ __launch_bounds__(256) void k_aht_leaves(uint8_t *__restrict__ dlog, uint64_t n0,
                                                    const uint8_t *__restrict__ payloads,
                                                    uint64_t m, uint32_t plen) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t n = n0 + 1 + i;
    uint32_t h[8];
    if (plen == 32) {
        uint32_t d[8];
        load_digest(payloads + i * 32, d);
        leaf_hash(d, h);
    } else {
        sha256_bytes(payloads + i * (uint64_t)plen, plen, 0x00, h);
    }
    store_digest(dlog + dev_nodes_until(n) * 32, h);
}

// phase 2: perfect nodes of level l ending at e = (j+1)*2^l, j in [j0, j0+cnt)
__global__ __launch_bounds__(256) void k_aht_perfect(uint8_t *__restrict__ dlog, int l,
                                                     uint64_t j0, uint64_t cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint64_t e = (j0 + t + 1) << l;
    const uint64_t half = 1ull << (l - 1);
    uint32_t a[8], b[8], o[8];
    load_digest(dlog + (dev_nodes_until(e - half) + (uint64_t)(l - 1)) * 32, a);
    const uint64_t ue = dev_nodes_until(e);
    load_digest(dlog + (ue + (uint64_t)(l - 1)) * 32, b);
    node_hash(a, b, o);
    store_digest(dlog + (ue + (uint64_t)l) * 32, o);
}

// phase 3: spine chains (ahtree.go:296-322 above the trailing-ones run)
__global__ __launch_bounds__(256) void k_aht_spine(uint8_t *__restrict__ dlog, uint64_t n0,
                                                   uint64_t m, uint8_t *__restrict__ roots_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t n = n0 + 1 + i;
    const uint64_t n1 = n - 1;
    const int t0 = __builtin_ctzll(n);
    const uint64_t un = dev_nodes_until(n);
    uint32_t h[8];
    load_digest(dlog + (un + (uint64_t)t0) * 32, h);  // node(n, tz(n)) = perfect root ending at n
    uint64_t rest = t0 + 1 < 64 ? (n1 >> (t0 + 1)) << (t0 + 1) : 0;
    uint64_t sk = popsum_below(rest);  // S(k) for k = rest (incrementally updated)
    int t = t0;
    while (rest) {
        const int l = __builtin_ctzll(rest);
        const uint64_t uk = until_from_s(rest, sk);  // nodesUntil(k), k = rest
        uint32_t left[8];
        load_digest(dlog + (uk + (uint64_t)l) * 32, left);
        node_hash(left, h, h);
        t++;
        store_digest(dlog + (un + (uint64_t)t) * 32, h);
        // drop bit l (the lowest set bit, rank popcount(rest) from the top)
        sk -= (l ? ((uint64_t)l << (l - 1)) : 0) +
              ((uint64_t)(__builtin_popcountll(rest) - 1) << l);
        rest &= rest - 1;
    }
    if (roots_out) store_digest(roots_out + i * 32, h);
}

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

hipError_t launch_ahtree_append(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0,
                                const uint8_t *payloads, uint64_t m, uint32_t plen,
                                uint8_t *roots_out) {
    if (!m) return hipSuccess;
    if (tm) tm->begin("aht_leaves", st);
    hipLaunchKernelGGL(k_aht_leaves, dim3(grid_for(m, 256)), dim3(256), 0, st, dlog, n0, payloads,
                       m, plen);
    if (tm) tm->end(st);
    const uint64_t n_end = n0 + m;
    if (tm) tm->begin("aht_perfect", st);
    for (int l = 1; l < 64 && (n_end >> l) != 0; l++) {
        const uint64_t j0 = n0 >> l;             // first j with (j+1)*2^l > n0
        const uint64_t j1 = n_end >> l;          // one past the last j with (j+1)*2^l <= n_end
        if (j1 <= j0) continue;
        hipLaunchKernelGGL(k_aht_perfect, dim3(grid_for(j1 - j0, 256)), dim3(256), 0, st, dlog, l,
                           j0, j1 - j0);
    }
    if (tm) tm->end(st);
    if (tm) tm->begin("aht_spine", st);
    hipLaunchKernelGGL(k_aht_spine, dim3(grid_for(m, 256)), dim3(256), 0, st, dlog, n0, m, roots_out);
    if (tm) tm->end(st);
    return hipGetLastError();
}

}  // namespace mh
