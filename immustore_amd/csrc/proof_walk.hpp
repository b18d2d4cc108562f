// proof_walk.hpp -- the index walks of proof generation, shared by the
// term-gather kernels (proof_kernels.hip) and the protobuf writers
// (wire_kernels.hip).  No memory is read: a walk only names the nodes.
//
//   htree  (*HTree).InclusionProof            embedded/htree/htree.go:121-164
//   ahtree inclusionProof / consistencyProof  embedded/ahtree/ahtree.go:547-651
//          highestNode                        ahtree.go:653-661
//
// Go builds every proof by PREPENDING terms; both ahtree recursions are tail
// calls, so a proof is the reverse of the sequence in which a walk meets its
// terms: emit(q, node) is called with q = 0, 1, ... and the term at proof
// position cnt-1-q is `node`.  Each walk returns cnt.
#pragma once
#include "mh_internal.hpp"

namespace mh {

__device__ __forceinline__ int bits_len(uint64_t x) { return x ? 64 - __clzll(x) : 0; }

// offset (in nodes) of level `layer` in the flat level-major layout of width w
__device__ __forceinline__ uint64_t level_off(uint64_t w, int layer) {
    uint64_t o = 0;
    for (int j = 0; j < layer; j++) o += (w + (1ull << j) - 1) >> j;
    return o;
}

// htree.go:121-164: proof of leaf i (< w) in a tree of width w; emit gets the
// node index in the flat level layout.
template <class F>
__device__ __forceinline__ uint32_t htree_walk(uint64_t i, uint64_t w, F &&emit) {
    uint32_t q = 0;
    if (w <= 1) return 0;
    uint64_t m = i, nn = w, offset = 0;
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
        const int layer = bits_len(r - l);
        emit(q, level_off(w, layer) + (l >> layer));
        q++;
        if (nn < 1 || (nn == 1 && m == 0)) break;
    }
    return q;
}

__device__ __forceinline__ uint64_t aht_node_index(uint64_t n, int l) {
    return (n <= 1 ? 0 : ahtree_nodes_upto_dev(n - 1)) + (uint64_t)l;
}

// highestNode(i, d): node(i, popcount((i-1) & (2^d - 1)))  (ahtree.go:653-661)
__device__ __forceinline__ uint64_t aht_highest(uint64_t i, int d) {
    const uint64_t mask = d >= 64 ? ~0ull : ((1ull << d) - 1);
    return aht_node_index(i, __popcll((i - 1) & mask));
}

// ahtree.go:547-577 (consistency = false) and :599-651 (consistency = true)
// for 0 < j, i <= j; emit gets dLog node indices.
template <class F>
__device__ __forceinline__ uint32_t ahtree_walk(bool consistency, uint64_t i, uint64_t j0,
                                                F &&emit) {
    uint32_t q = 0;
    uint64_t j = j0;
    int height = bits_len(j0 - 1);
    bool done = false;
    while (!done) {
        bool restarted = false;
        for (int h = height - 1; h >= 0 && !restarted && !done; h--) {
            if (!((j - 1) & (1ull << h))) continue;
            const uint64_t k = (j - 1) >> h << h;
            if (i <= k) {
                emit(q++, aht_highest(j, h));
                if (!consistency || i < k) {  // tail call on (i, k, h)
                    j = k;
                    height = h;
                    restarted = true;
                } else {                      // consistency, i == k
                    emit(q++, aht_highest(i, h));
                    done = true;
                }
            } else {
                emit(q++, aht_node_index(k, h));
                if (consistency && i == j) {
                    emit(q++, aht_highest(i, h));
                    done = true;
                }
            }
        }
        if (!restarted) done = true;
    }
    return q;
}

}  // namespace mh
