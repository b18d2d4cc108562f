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
#include <cstdlib>

#include "digest_io.hpp"
#include "mh_internal.hpp"

namespace mh {

uint64_t ahtree_nodes_upto(uint64_t n) { return n + popsum_below(n); }
uint64_t ahtree_nodes_until(uint64_t n) { return n <= 1 ? 0 : ahtree_nodes_upto(n - 1); }

__device__ __forceinline__ uint64_t dev_nodes_until(uint64_t n) {
    return until_from_s(n, popsum_below(n));
}

// node(k, l) of an append range that starts after edge.lo: a node ending at
// or before edge.lo is a peak of edge.lo (the perfect subtree of its set bit
// l), kept in the frontier edge.fr[l] instead of the dLog.  With no edge
// (lo = 0) every node comes from the dLog.
__device__ __forceinline__ const uint8_t *edge_node(const uint8_t *dlog, const AhtEdge &edge,
                                                    uint64_t k, int l) {
    return k <= edge.lo ? edge.fr + l * 32 : dlog + (dev_nodes_until(k) + (uint64_t)l) * 32;
}

// phase 1: d_0 = leaf of payload (plen == 32: one block, the store's Alh),
// plus, when asked, the appendable records of the same appends (SURVEY.md
// 8(f) row 4): pLog BE32 len || payload (ahtree.go:266-282) and cLog
// BE64 poff || BE32 len (ahtree.go:341-351), written while the payload is in
// registers.  dlog == nullptr writes only the records.  For 32-byte payloads
// the workgroup stages its 256 records in LDS and stores them as contiguous
// dwords (36-byte / 12-byte records would otherwise be strided per lane).
__global__ __launch_bounds__(256) void k_aht_leaves(uint8_t *__restrict__ dlog, uint64_t n0,
                                                    const uint8_t *__restrict__ payloads,
                                                    uint64_t m, uint32_t plen, AhtLogs lg) {
    const uint64_t base = (uint64_t)blockIdx.x * blockDim.x;
    const uint64_t i = base + threadIdx.x;
    const bool live = i < m;
    const bool logs = lg.plog || lg.clog;
    const bool staged = logs && plen == 32 && !((uintptr_t)lg.plog & 3) && !((uintptr_t)lg.clog & 3);
    if (!live && !staged) return;
    const uint64_t n = n0 + 1 + i;
    uint32_t raw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (live && plen == 32) {
        const uint4 a = *reinterpret_cast<const uint4 *>(payloads + i * 32);
        const uint4 b = *reinterpret_cast<const uint4 *>(payloads + i * 32 + 16);
        raw[0] = a.x; raw[1] = a.y; raw[2] = a.z; raw[3] = a.w;
        raw[4] = b.x; raw[5] = b.y; raw[6] = b.z; raw[7] = b.w;
        if (dlog) {
            uint32_t d[8], h[8];
#pragma unroll
            for (int j = 0; j < 8; j++) d[j] = bswap(raw[j]);
            leaf_hash(d, h);
            store_digest(dlog + dev_nodes_until(n) * 32, h);
        }
    } else if (live && dlog) {
        uint32_t h[8];
        sha256_bytes(payloads + i * (uint64_t)plen, plen, 0x00, h);
        store_digest(dlog + dev_nodes_until(n) * 32, h);
    }
    if (!logs) return;
    const uint64_t rec = 4 + (uint64_t)plen;
    const uint64_t poff = lg.p_off0 + i * rec;
    if (staged) {
        __shared__ uint32_t sp[256 * 9];
        __shared__ uint32_t sc[256 * 3];
        const int t = threadIdx.x;
        sp[t * 9] = bswap(32u);
#pragma unroll
        for (int j = 0; j < 8; j++) sp[t * 9 + 1 + j] = raw[j];
        sc[t * 3 + 0] = bswap((uint32_t)(poff >> 32));
        sc[t * 3 + 1] = bswap((uint32_t)poff);
        sc[t * 3 + 2] = bswap(32u);
        __syncthreads();
        const uint64_t cnt = m - base < 256 ? m - base : 256;
        if (lg.plog) {
            uint32_t *dp = reinterpret_cast<uint32_t *>(lg.plog) + base * 9;
            for (uint32_t k = t; k < cnt * 9; k += 256) dp[k] = sp[k];
        }
        if (lg.clog) {
            uint32_t *dc = reinterpret_cast<uint32_t *>(lg.clog) + base * 3;
            for (uint32_t k = t; k < cnt * 3; k += 256) dc[k] = sc[k];
        }
        return;
    }
    if (lg.plog) {
        uint8_t *r = lg.plog + i * rec;
        for (int k = 0; k < 4; k++) r[k] = (uint8_t)(plen >> (24 - 8 * k));
        const uint8_t *src = payloads + i * (uint64_t)plen;
        for (uint32_t k = 0; k < plen; k++) r[4 + k] = src[k];
    }
    if (lg.clog) {
        uint8_t *c = lg.clog + i * 12;
        for (int k = 0; k < 8; k++) c[k] = (uint8_t)(poff >> (56 - 8 * k));
        for (int k = 0; k < 4; k++) c[8 + k] = (uint8_t)(plen >> (24 - 8 * k));
    }
}

// phase 2: perfect nodes of level l ending at e = (j+1)*2^l, j in [j0, j0+cnt)
__global__ __launch_bounds__(256) void k_aht_perfect(uint8_t *__restrict__ dlog, int l,
                                                     uint64_t j0, uint64_t cnt, AhtEdge edge) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint64_t e = (j0 + t + 1) << l;
    const uint64_t half = 1ull << (l - 1);
    uint32_t a[8], b[8], o[8];
    load_digest(edge_node(dlog, edge, e - half, l - 1), a);
    const uint64_t ue = dev_nodes_until(e);
    load_digest(dlog + (ue + (uint64_t)(l - 1)) * 32, b);
    node_hash(a, b, o);
    store_digest(dlog + (ue + (uint64_t)l) * 32, o);
}

// phase 3: spine chains (ahtree.go:296-322 above the trailing-ones run)
__global__ __launch_bounds__(256) void k_aht_spine(uint8_t *__restrict__ dlog, uint64_t n0,
                                                   uint64_t m, uint8_t *__restrict__ roots_out,
                                                   AhtEdge edge) {
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
        load_digest(rest <= edge.lo ? edge.fr + l * 32 : dlog + (uk + (uint64_t)l) * 32, left);
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

// ---------------------------------------------------------------------------
// Table-driven variants (sha256_cdna.hpp node_hash_tab): every workgroup
// builds the 256 node-tail schedules in LDS once and then runs a grid-stride
// loop, so the table cost is amortised over many node hashes.

__global__ __launch_bounds__(512) void k_aht_perfect_t(uint8_t *__restrict__ dlog, int l,
                                                       uint64_t j0, uint64_t cnt, AhtEdge edge) {
    extern __shared__ uint32_t tab[];
    node_tab_init(tab);
    const uint64_t half = 1ull << (l - 1);
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cnt;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = (j0 + t + 1) << l;
        uint32_t a[8], b[8], o[8];
        load_digest(edge_node(dlog, edge, e - half, l - 1), a);
        const uint64_t ue = dev_nodes_until(e);
        load_digest(dlog + (ue + (uint64_t)(l - 1)) * 32, b);
        node_hash_tab(a, b, o, tab);
        store_digest(dlog + (ue + (uint64_t)l) * 32, o);
    }
}

// Spine with balanced lanes.  The chain of n has popcount(n-1) - tz(n) steps:
// the low 7 bits of n-1 (r) contribute len(r) = popcount(r) - trailing_ones(r)
// steps (0..6, 321 in total over r = 0..127), the higher bits B = (n-1) >> 7
// are shared by the 128 n of an aligned block and give popcount(B) steps each.
// One wave takes one aligned block; lane L runs the chains of TWO n of it,
// r = pr.ra[L] then r = pr.rb[L], paired so that len(ra) + len(rb) <= 6
// (longest with shortest).  All lanes of a wave then do 5..6 + 2 popcount(B)
// hash steps, against up to 6 + popcount(B) with 1 chain per lane, where the
// low-bit part idles most of the wave (~40 % of the lanes' time at 10^7).
// The B-part reads (node(k, l), l >= 7) are wave-uniform broadcast loads.
struct SpinePairs {
    uint8_t ra[64], rb[64];
};

// Blocks are handed out through a work queue (one atomic per wave and block):
// a block's work varies with popcount(B), and a static grid-stride split left
// the longest wave ~15 % behind the average.  amdgpu_waves_per_eu(6) caps the
// kernel at 80 VGPRs so three 512-thread workgroups (the LDS limit with the
// 53 KB table) fit per CU, 6 waves per SIMD.
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(6))) void k_aht_spine_pairs(uint8_t *__restrict__ dlog,
                                                            uint64_t n0, uint64_t m,
                                                            uint8_t *__restrict__ roots_out,
                                                            SpinePairs pr, uint64_t blk0,
                                                            uint64_t nblk,
                                                            uint32_t *__restrict__ work_ctr,
                                                            AhtEdge edge) {
    extern __shared__ uint32_t tab[];
    node_tab_init(tab);
    const int lane = threadIdx.x & 63;
    const uint64_t nlast = n0 + m;
    const uint32_t ra = pr.ra[lane], rb = pr.rb[lane];
    for (;;) {
        uint32_t got = 0;
        if (lane == 0) got = atomicAdd(work_ctr, 1u);
        const uint64_t bi = __builtin_amdgcn_readfirstlane(got);
        if (bi >= nblk) break;
        const uint64_t base = (blk0 + bi) << 7;  // n - 1 of r = 0 (wave-uniform)
        // S(base + x) = S(base) + x * popcount(B) + S(x) for x <= 128: the
        // per-lane index math only walks the 7 low bits
        const uint64_t sb = popsum_below(base);
        const uint32_t pcb = (uint32_t)__builtin_popcountll(base);
        const uint64_t nA = base + ra + 1, nB = base + rb + 1;
        const bool vA = nA > n0 && nA <= nlast, vB = nB > n0 && nB <= nlast;
        bool second = !vA, done = !(vA || vB);
        uint32_t r = vA ? ra : rb;
        uint64_t n = 0, un = 0, rest = 0, sk = 0;
        int t = 0;
        uint32_t h[8], left[8];
#define MH_SPINE_SETUP()                                                                          \
    do {                                                                                          \
        n = base + r + 1;                                                                         \
        const int t0_ = __builtin_ctzll(n);                                                       \
        un = (n - 1) + sb + (uint64_t)(r + 1) * pcb + popsum_below(r + 1) -                       \
             (pcb + (uint32_t)__builtin_popcount(r));                                             \
        load_digest(dlog + (un + (uint64_t)t0_) * 32, h);                                         \
        if (r != 127) {                                                                           \
            const uint32_t rr_ = (r >> (t0_ + 1)) << (t0_ + 1);                                   \
            rest = base + rr_;                                                                    \
            sk = sb + (uint64_t)rr_ * pcb + popsum_below(rr_);                                    \
        } else {                                                                                  \
            rest = t0_ + 1 < 64 ? ((n - 1) >> (t0_ + 1)) << (t0_ + 1) : 0;                        \
            sk = popsum_below(rest);                                                              \
        }                                                                                         \
        t = t0_;                                                                                  \
    } while (0)
        if (!done) MH_SPINE_SETUP();
        for (;;) {
            while (!done && rest == 0) {
                if (roots_out) store_digest(roots_out + (n - n0 - 1) * 32, h);
                if (!second && vB) {
                    second = true;
                    r = rb;
                    MH_SPINE_SETUP();
                } else {
                    done = true;
                }
            }
            if (done) break;
            // drop the lowest set bit l of rest (rank popcount(rest) from the
            // top) and prefetch the next step's left node before hashing
            const int l = __builtin_ctzll(rest);
            load_digest(rest <= edge.lo ? edge.fr + l * 32
                                        : dlog + (until_from_s(rest, sk) + (uint64_t)l) * 32,
                        left);
            sk -= (l ? ((uint64_t)l << (l - 1)) : 0) +
                  ((uint64_t)(__builtin_popcountll(rest) - 1) << l);
            rest &= rest - 1;
            node_hash_tab(left, h, h, tab);
            t++;
            store_digest(dlog + (un + (uint64_t)t) * 32, h);
        }
#undef MH_SPINE_SETUP
    }
}

static SpinePairs make_spine_pairs() {
    int len[128], ord[128];
    for (int r = 0; r < 128; r++) {
        int to = 0;
        while ((r >> to) & 1) to++;
        len[r] = __builtin_popcount(r) - to;
        ord[r] = r;
    }
    std::stable_sort(ord, ord + 128, [&](int x, int y) { return len[x] < len[y]; });
    SpinePairs p;
    for (int i = 0; i < 64; i++) {
        p.ra[i] = (uint8_t)ord[127 - i];  // long chain first, short one second
        p.rb[i] = (uint8_t)ord[i];
    }
    return p;
}

// Resident workgroups for a grid-stride kernel with the node table in LDS.
static unsigned resident_grid(const void *kern, int block, uint64_t work_items) {
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, kNodeTabBytes) !=
            hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const uint64_t need = (work_items + block - 1) / block;
    const uint64_t cap = (uint64_t)cus * (uint64_t)per_cu;
    return (unsigned)std::max<uint64_t>(1, std::min(need, cap));
}

// the node hashes' second block from the LDS schedule table (C5 509 -> 576 M
// proofs/s, C3 spine pairs; the plain kernels remain for small launches)
static constexpr bool use_node_table() { return true; }

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

// Phase 1: leaves of (n0, n0 + m].
hipError_t launch_ahtree_leaves(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0,
                                const uint8_t *payloads, uint64_t m, uint32_t plen,
                                const AhtLogs &lg) {
    if (!m) return hipSuccess;
    TimerScope ts(tm, dlog ? "aht_leaves" : "aht_records", st);
    hipLaunchKernelGGL(k_aht_leaves, dim3(grid_for(m, 256)), dim3(256), 0, st, dlog, n0, payloads,
                       m, plen, lg);
    return hipGetLastError();
}

// Phase 2: perfect nodes of levels [lmin, lmax] whose end lies in (n0, n_end].
hipError_t launch_ahtree_perfect(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0,
                                 uint64_t n_end, int lmin, int lmax, const AhtEdge &edge) {
    const bool tab = use_node_table();
    TimerScope ts(tm, "aht_perfect", st);
    for (int l = std::max(lmin, 1); l <= std::min(lmax, 63) && (n_end >> l) != 0; l++) {
        const uint64_t j0 = n0 >> l;             // first j with (j+1)*2^l > n0
        const uint64_t j1 = n_end >> l;          // one past the last j with (j+1)*2^l <= n_end
        if (j1 <= j0) continue;
        // small levels are launch/latency bound: skip the per-workgroup table copy
        if (tab && j1 - j0 >= (1ull << 18))
            hipLaunchKernelGGL(k_aht_perfect_t,
                               dim3(resident_grid((const void *)k_aht_perfect_t, 512, j1 - j0)),
                               dim3(512), kNodeTabBytes, st, dlog, l, j0, j1 - j0, edge);
        else
            hipLaunchKernelGGL(k_aht_perfect, dim3(grid_for(j1 - j0, 256)), dim3(256), 0, st, dlog,
                               l, j0, j1 - j0, edge);
    }
    return hipGetLastError();
}

// Phase 3: spine chains of (n0, n0 + m] (every perfect node they read must be
// in the dLog already, or a peak of edge.lo in the frontier).
hipError_t launch_ahtree_spine(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0, uint64_t m,
                               uint8_t *roots_out, uint32_t *work_ctr, const AhtEdge &edge) {
    if (!m) return hipSuccess;
    TimerScope ts(tm, "aht_spine", st);
    const uint64_t n_end = n0 + m;
    if (use_node_table()) {
        static const SpinePairs pairs = make_spine_pairs();
        if (hipError_t e = hipMemsetAsync(work_ctr, 0, sizeof(uint32_t), st)) return e;
        const uint64_t blk0 = n0 >> 7, nblk = ((n_end - 1) >> 7) - blk0 + 1;
        hipLaunchKernelGGL(k_aht_spine_pairs,
                           dim3(resident_grid((const void *)k_aht_spine_pairs, 512, nblk * 64)),
                           dim3(512), kNodeTabBytes, st, dlog, n0, m, roots_out, pairs, blk0, nblk,
                           work_ctr, edge);
    } else {
        hipLaunchKernelGGL(k_aht_spine, dim3(grid_for(m, 256)), dim3(256), 0, st, dlog, n0, m,
                           roots_out, edge);
    }
    return hipGetLastError();
}

hipError_t launch_ahtree_append(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0,
                                const uint8_t *payloads, uint64_t m, uint32_t plen,
                                uint8_t *roots_out, uint32_t *work_ctr, const AhtLogs &lg,
                                const AhtEdge &edge) {
    if (!m) return hipSuccess;
    if (hipError_t e = launch_ahtree_leaves(st, tm, dlog, n0, payloads, m, plen, lg)) return e;
    if (hipError_t e = launch_ahtree_perfect(st, tm, dlog, n0, n0 + m, 1, 63, edge)) return e;
    return launch_ahtree_spine(st, tm, dlog, n0, m, roots_out, work_ctr, edge);
}

// Sharded appends: write the all-gathered shard roots
// node((r+1) 2^level, level), r < count, into a rank's dLog.
__global__ void k_aht_put_roots(uint8_t *__restrict__ dlog, int level, uint64_t count,
                                const uint8_t *__restrict__ roots) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= count) return;
    const uint64_t e = (r + 1) << level;
    const uint4 *s = reinterpret_cast<const uint4 *>(roots + r * 32);
    uint4 *d = reinterpret_cast<uint4 *>(dlog + (dev_nodes_until(e) + (uint64_t)level) * 32);
    d[0] = s[0];
    d[1] = s[1];
}

hipError_t launch_ahtree_put_shard_roots(hipStream_t st, Timer *tm, uint8_t *dlog, int level,
                                         uint64_t count, const uint8_t *roots) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_aht_put_roots, dim3(grid_for(count, 256)), dim3(256), 0, st, dlog, level,
                       count, roots);
    if (hipError_t e = hipGetLastError()) return e;
    // the cross-shard perfect nodes above them, for every end <= count * 2^level
    return launch_ahtree_perfect(st, tm, dlog, 0, count << level, level + 1, 63);
}

// ---------------------------------------------------------------------------
// Ranged multi-device append (capi_multi.hip): pieces, the piece tree, frontiers.

__device__ __forceinline__ void copy32(uint8_t *dst, const uint8_t *src) {
    reinterpret_cast<uint4 *>(dst)[0] = reinterpret_cast<const uint4 *>(src)[0];
    reinterpret_cast<uint4 *>(dst)[1] = reinterpret_cast<const uint4 *>(src)[1];
}

__global__ void k_aht_gather_pieces(const uint8_t *__restrict__ dlog, int k, uint64_t e0,
                                    uint64_t count, uint8_t *__restrict__ send) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint64_t e = (e0 + i) << k;
    copy32(send + i * 32, dlog + (dev_nodes_until(e) + (uint64_t)k) * 32);
}

// One workgroup.  Piece level l' (global level k + l') holds slots
// j in [N0 >> l', Pend >> l'] (node ending at (j << l') * S); slot N0 >> l' is
// the old peak of n0 at level k + l' when that bit of n0 is set (a left child
// ending at or before n0 is always one), every other slot is new:
// level 0 = the all-gathered piece roots, level l' = H(slot 2j-1, slot 2j) of
// level l'-1 (ahtree.go:296-322 restricted to perfect nodes).  The tree is
// tiny (tens of pieces per device); it runs replicated on every device.
__global__ __launch_bounds__(256) void k_aht_top(AhtTopArgs a, const uint8_t *__restrict__ recv,
                                                 const uint8_t *__restrict__ peaks_n0,
                                                 uint8_t *__restrict__ top,
                                                 uint8_t *__restrict__ dlog,
                                                 uint8_t *__restrict__ fr) {
    const int t = threadIdx.x;
    for (uint64_t j = a.N0 + t; j <= a.Pend; j += 256) {
        uint8_t *dst = top + (a.lev_off[0] + j - a.N0) * 32;
        if (j == a.N0) {
            if ((a.n0 >> a.k) & 1) copy32(dst, peaks_n0 + a.k * 32);
            continue;
        }
        int d = 0;
        while (d + 1 < a.G && j > a.pe0[d + 1]) d++;
        copy32(dst, recv + ((uint64_t)d * a.Pmax + (j - a.pe0[d] - 1)) * 32);
    }
    __syncthreads();
    for (int l = 1; l < a.nlev; l++) {
        const uint64_t b = a.N0 >> l, bp = a.N0 >> (l - 1), jend = a.Pend >> l;
        const int gl = a.k + l;
        for (uint64_t j = b + t; j <= jend; j += 256) {
            uint8_t *dst = top + (a.lev_off[l] + j - b) * 32;
            if (j == b) {
                if ((a.n0 >> gl) & 1) copy32(dst, peaks_n0 + gl * 32);
                continue;
            }
            uint32_t x[8], y[8], o[8];
            load_digest(top + (a.lev_off[l - 1] + 2 * j - 1 - bp) * 32, x);
            load_digest(top + (a.lev_off[l - 1] + 2 * j - bp) * 32, y);
            node_hash(x, y, o);
            store_digest(dst, o);
            const uint64_t e = j << gl;
            if (e > a.lo && e <= a.hi) store_digest(dlog + (dev_nodes_until(e) + (uint64_t)gl) * 32, o);
        }
        __syncthreads();
    }
    // the peaks of lo (a multiple of S, so every set bit is >= k)
    if (a.lo > a.n0 && t < 64 && t >= a.k && ((a.lo >> t) & 1)) {
        const int lp = t - a.k;
        const uint64_t j = (a.lo >> a.k) >> lp;
        copy32(fr + t * 32, top + (a.lev_off[lp] + j - (a.N0 >> lp)) * 32);
    }
}

__global__ void k_aht_peaks(const uint8_t *__restrict__ dlog, uint64_t n, uint8_t *__restrict__ fr) {
    const int l = threadIdx.x;
    if (l >= 64 || !((n >> l) & 1)) return;
    const uint64_t kk = l ? (n >> l) << l : n;
    copy32(fr + l * 32, dlog + (dev_nodes_until(kk) + (uint64_t)l) * 32);
}

hipError_t launch_ahtree_gather_pieces(hipStream_t st, const uint8_t *dlog, int k, uint64_t e0,
                                       uint64_t count, uint8_t *send) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_aht_gather_pieces, dim3(grid_for(count, 256)), dim3(256), 0, st, dlog, k,
                       e0, count, send);
    return hipGetLastError();
}

hipError_t launch_ahtree_top(hipStream_t st, const AhtTopArgs &a, const uint8_t *recv,
                             const uint8_t *peaks_n0, uint8_t *top, uint8_t *dlog, uint8_t *fr) {
    hipLaunchKernelGGL(k_aht_top, dim3(1), dim3(256), 0, st, a, recv, peaks_n0, top, dlog, fr);
    return hipGetLastError();
}

__global__ void k_aht_put_slots(AhtSlots s, uint8_t *__restrict__ dst) {
    const int t = threadIdx.x;  // 128 threads x 16 B
    reinterpret_cast<uint4 *>(dst)[t] = reinterpret_cast<const uint4 *>(s.b)[t];
}

hipError_t launch_ahtree_put_slots(hipStream_t st, const AhtSlots &s, uint8_t *dst) {
    hipLaunchKernelGGL(k_aht_put_slots, dim3(1), dim3(128), 0, st, s, dst);
    return hipGetLastError();
}

hipError_t launch_ahtree_peaks(hipStream_t st, const uint8_t *dlog, uint64_t n, uint8_t *fr) {
    hipLaunchKernelGGL(k_aht_peaks, dim3(1), dim3(64), 0, st, dlog, n, fr);
    return hipGetLastError();
}

}  // namespace mh
