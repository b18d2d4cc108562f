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
// position cnt-1-q is `node`.  Each walk returns cnt.  HtreeWalk / AhtreeWalk
// are the same walks as resumable generators (the staged protobuf writers
// take a few terms per round).
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

// htree.go:121-164: proof of leaf i (< w) in a tree of width w, as a
// generator: next() gives the node index (flat level layout) of each term in
// the order the walk meets them, ~0 after the last.
struct HtreeWalk {
    uint64_t w, m, nn, offset;
    bool done;
    __device__ __forceinline__ HtreeWalk(uint64_t i, uint64_t w_)
        : w(w_), m(i), nn(w_), offset(0), done(w_ <= 1) {}
    __device__ __forceinline__ uint64_t next() {
        if (done) return ~0ull;
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
        if (nn < 1 || (nn == 1 && m == 0)) done = true;
        const int layer = bits_len(r - l);
        return level_off(w, layer) + (l >> layer);
    }
};

// The same walk as a loop calling emit(q, node): with an empty emit (term
// counting) the compiler drops the index math entirely.  lo(layer) gives
// level_off(w, layer) (a table when many proofs share one width).
template <class LO, class F>
__device__ __forceinline__ uint32_t htree_walk_lo(uint64_t i, uint64_t w, LO &&lo, F &&emit) {
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
        emit(q, lo(layer) + (l >> layer));
        q++;
        if (nn < 1 || (nn == 1 && m == 0)) break;
    }
    return q;
}

template <class F>
__device__ __forceinline__ uint32_t htree_walk(uint64_t i, uint64_t w, F &&emit) {
    return htree_walk_lo(i, w, [&](int layer) { return level_off(w, layer); }, emit);
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
// for 0 < j, i <= j, as a generator of dLog node indices.  Both Go
// recursions are tail calls that restart the descent one level lower with
// j = k, so the walk is a single pass over the bits h of j-1, high to low;
// the consistency base cases emit two terms in one step (`pend`).
struct AhtreeWalk {
    uint64_t i, j, pend;
    int h;
    bool cons, done, pending;
    __device__ __forceinline__ AhtreeWalk(bool consistency, uint64_t i_, uint64_t j0)
        : i(i_), j(j0), pend(0), h(bits_len(j0 - 1) - 1), cons(consistency), done(false),
          pending(false) {}
    __device__ __forceinline__ uint64_t next() {
        if (pending) {
            pending = false;
            return pend;
        }
        while (h >= 0 && !done) {
            const int hh = h--;
            if (!((j - 1) & (1ull << hh))) continue;
            const uint64_t k = (j - 1) >> hh << hh;
            if (i <= k) {
                const uint64_t r = aht_highest(j, hh);
                if (!cons || i < k) {  // tail call on (i, k, hh)
                    j = k;
                } else {               // consistency, i == k
                    pend = aht_highest(i, hh);
                    pending = true;
                    done = true;
                }
                return r;
            }
            const uint64_t r = aht_node_index(k, hh);
            if (cons && i == j) {
                pend = aht_highest(i, hh);
                pending = true;
                done = true;
            }
            return r;
        }
        done = true;
        return ~0ull;
    }
};

// The same walk as a loop calling emit(q, node) (index math dropped when the
// emit ignores it, as in the size passes).
template <class F>
__device__ __forceinline__ uint32_t ahtree_walk(bool consistency, uint64_t i, uint64_t j0,
                                                F &&emit) {
    uint32_t q = 0;
    uint64_t j = j0;
    for (int h = bits_len(j0 - 1) - 1; h >= 0; h--) {
        if (!((j - 1) & (1ull << h))) continue;
        const uint64_t k = (j - 1) >> h << h;
        if (i <= k) {
            emit(q++, aht_highest(j, h));
            if (!consistency || i < k) {  // tail call on (i, k, h)
                j = k;
                continue;
            }
            emit(q++, aht_highest(i, h));  // consistency, i == k
            break;
        }
        emit(q++, aht_node_index(k, h));
        if (consistency && i == j) {
            emit(q++, aht_highest(i, h));
            break;
        }
    }
    return q;
}

}  // namespace mh
