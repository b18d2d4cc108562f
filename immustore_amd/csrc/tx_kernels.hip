// tx_kernels.hip -- the transaction layer around the Merkle path on CDNA4.
//
//   TxHeader.innerHash / Alh             embedded/store/tx.go:249-319        (a7)
//   advanceLinearHash / VerifyLinearProof embedded/store/verification.go:32-64 (a13)
//   leafFor                              embedded/store/verification.go:237-242
//   many small htrees at once            htree.BuildWith (htree.go:68-113) per tx,
//                                        for the read path (tx.go:605-630, a14)
//                                        and for concurrent BuildHashTree calls
//                                        (tx.go:332-355, immustore.go:1632)
//   entry-digest messages from raw tx-log records (tx.go:520-588 + 690-731)
//
// Everything is one message (or one chain) per lane; the per-tx work is a few
// compressions, so these kernels are latency/occupancy shaped rather than
// roofline shaped, and they exist so that no hashing of this layer runs on
// the host.
#include <algorithm>
#include <mutex>
#include <vector>

#include "digest_io.hpp"
#include "mh_internal.hpp"

namespace mh {

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

__device__ __forceinline__ uint32_t ld_be32_aligned(const uint8_t *p) {
    return bswap(*reinterpret_cast<const uint32_t *>(p));
}

// SHA256(BE64 id || prev[8 words] || inner[8 words]): 72 bytes, two blocks
// (tx.go:307-319, verification.go:32-38).
__device__ __forceinline__ void alh_hash(uint64_t id, const uint32_t prev[8],
                                         const uint32_t inner[8], uint32_t out[8]) {
    uint32_t w[16];
    w[0] = (uint32_t)(id >> 32);
    w[1] = (uint32_t)id;
#pragma unroll
    for (int j = 0; j < 8; j++) w[2 + j] = prev[j];
#pragma unroll
    for (int j = 0; j < 6; j++) w[10 + j] = inner[j];
    State s;
    s.init();
    compress(s, w);
    w[0] = inner[6];
    w[1] = inner[7];
    w[2] = 0x80000000u;
#pragma unroll
    for (int j = 3; j < 15; j++) w[j] = 0;
    w[15] = 72u * 8u;
    compress(s, w);
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = s.h[j];
}

__device__ __forceinline__ void put_be(uint8_t *&o, uint64_t v, int n) {
    for (int k = n - 1; k >= 0; k--) *o++ = (uint8_t)(v >> (8 * k));
}

// One header per lane: innerHash (message assembled in the lane's scratch
// slot, <= 356 bytes) then Alh.  eh_src (nullable) replaces hdrs[p].eh;
// expect (nullable) turns the Alh into a pass / MH_ERR_CORRUPTED_DATA status.
// e: the stored Alh to compare against (nullable).
__device__ __forceinline__ void tx_alh_one(uint64_t p, const MhTxHeader &h,
                                           const uint8_t *__restrict__ md_blob,
                                           const uint8_t *__restrict__ eh, uint8_t *__restrict__ msg,
                                           const uint8_t *__restrict__ e,
                                           uint8_t *__restrict__ inner_out,
                                           uint8_t *__restrict__ alh_out,
                                           int32_t *__restrict__ status) {
    uint8_t *o = msg;
    put_be(o, (uint64_t)h.ts, 8);
    put_be(o, h.version, 2);
    if (h.version == 0) {
        put_be(o, h.nentries, 2);
    } else {
        put_be(o, h.md_len, 2);
        const uint8_t *md = md_blob + h.md_off;
        for (uint32_t k = 0; k < h.md_len; k++) *o++ = md[k];
        put_be(o, h.nentries, 4);
    }
    for (int k = 0; k < 32; k++) *o++ = eh[k];
    put_be(o, h.bl_tx_id, 8);
    for (int k = 0; k < 32; k++) *o++ = h.bl_root[k];
    uint32_t inner[8], prev[8], a[8];
    sha256_bytes(msg, (uint64_t)(o - msg), -1, inner);
#pragma unroll
    for (int j = 0; j < 8; j++) prev[j] = ld_be32_aligned(h.prev_alh + 4 * j);
    alh_hash(h.id, prev, inner, a);
    if (inner_out) store_digest(inner_out + p * 32, inner);
    if (alh_out) store_digest(alh_out + p * 32, a);
    if (status) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t v = ((uint32_t)e[4 * j] << 24) | ((uint32_t)e[4 * j + 1] << 16) |
                               ((uint32_t)e[4 * j + 2] << 8) | e[4 * j + 3];
            x |= v ^ a[j];
        }
        status[p] = x ? MH_ERR_CORRUPTED_DATA : MH_OK;
    }
}

__global__ __launch_bounds__(256) void k_tx_alh(uint64_t n, const MhTxHeader *__restrict__ hdrs,
                                                const uint8_t *__restrict__ md_blob,
                                                const uint8_t *__restrict__ eh_src,
                                                uint8_t *__restrict__ scratch,
                                                const uint8_t *__restrict__ expect,
                                                const uint64_t *__restrict__ expect_off,
                                                uint8_t *__restrict__ inner_out,
                                                uint8_t *__restrict__ alh_out,
                                                int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const MhTxHeader &h = hdrs[p];
    tx_alh_one(p, h, md_blob, eh_src ? eh_src + p * 32 : h.eh, scratch + p * kTxInnerStride,
               status ? expect + (expect_off ? expect_off[p] : p * 32) : nullptr, inner_out,
               alh_out, status);
}

// leafFor(d) = SHA256(0x00 || d)  (verification.go:237-242, ahtree.go:288-292)
__global__ __launch_bounds__(256) void k_leaf_for(uint64_t n, const uint8_t *__restrict__ in,
                                                  uint8_t *__restrict__ out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint32_t d[8], h[8];
    load_digest(in + p * 32, d);
    leaf_hash(d, h);
    store_digest(out + p * 32, h);
}

__global__ __launch_bounds__(256) void k_select32(uint64_t n, const uint8_t *__restrict__ sel,
                                                  const uint8_t *__restrict__ x,
                                                  const uint8_t *__restrict__ y,
                                                  uint8_t *__restrict__ out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint4 *s = reinterpret_cast<const uint4 *>((sel[p] ? x : y) + p * 32);
    uint4 *d = reinterpret_cast<uint4 *>(out + p * 32);
    d[0] = s[0];
    d[1] = s[1];
}

// VerifyLinearProof (verification.go:40-64), one proof per lane.
__global__ __launch_bounds__(256) void k_linear_verify(
    uint64_t n, const uint64_t *__restrict__ psrc, const uint64_t *__restrict__ ptgt,
    const uint64_t *__restrict__ src, const uint64_t *__restrict__ tgt,
    const uint64_t *__restrict__ term_off, const uint8_t *__restrict__ terms,
    const uint8_t *__restrict__ src_alh, const uint8_t *__restrict__ tgt_alh,
    uint8_t *__restrict__ ok) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t s = psrc[p], t = ptgt[p], t0 = term_off[p], t1 = term_off[p + 1];
    bool res = s == src[p] && t == tgt[p] && s != 0 && s <= t && t1 > t0 && (t1 - t0) == t - s + 1;
    uint32_t c[8], x[8];
    if (res) {
        load_digest(terms + t0 * 32, c);
        load_digest(src_alh + p * 32, x);
        uint32_t d = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) d |= c[j] ^ x[j];
        res = d == 0;
    }
    if (res) {
        for (uint64_t i = 1; i < t1 - t0; i++) {
            uint32_t term[8];
            load_digest(terms + (t0 + i) * 32, term);
            alh_hash(s + i, c, term, c);
        }
        load_digest(tgt_alh + p * 32, x);
        uint32_t d = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) d |= c[j] ^ x[j];
        res = d == 0;
    }
    ok[p] = res ? 1 : 0;
}

// VerifyLinearAdvanceProof chain (verification.go:106-121) for proofs that
// passed the host-side length checks: calc starts at terms[0] (Alh of
// start+1); before every advance the current calc is written to
// leaves_src[first + k] (its leafFor must be included in the target tree at
// index start+1+k), then calc = advanceLinearHash(calc, start+2+k, terms[k+1]).
// ok[p] = (final calc == end_alh[p]).
__global__ __launch_bounds__(256) void k_advance_chain(
    uint64_t n, const uint64_t *__restrict__ start, const uint64_t *__restrict__ cnt,
    const uint64_t *__restrict__ term_off, const uint8_t *__restrict__ terms,
    const uint64_t *__restrict__ first, const uint8_t *__restrict__ end_alh,
    uint8_t *__restrict__ leaves_src, uint8_t *__restrict__ ok) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t t0 = term_off[p], c0 = cnt[p], s = start[p], f = first[p];
    uint32_t c[8], x[8];
    load_digest(terms + t0 * 32, c);
    for (uint64_t k = 0; k < c0; k++) {
        store_digest(leaves_src + (f + k) * 32, c);
        uint32_t term[8];
        load_digest(terms + (t0 + k + 1) * 32, term);
        alh_hash(s + 2 + k, c, term, c);
    }
    load_digest(end_alh + p * 32, x);
    uint32_t d = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) d |= c[j] ^ x[j];
    ok[p] = d == 0;
}

// Entry digest (tx.go:690-731) -- and, with leaf != 0, its htree leaf
// SHA256(0x00 || digest) (htree.go:79-83) -- hashed in place from the raw
// tx-log entry record (sha256_skip12): no message buffer, no offsets scan.
__device__ __forceinline__ void txe_digest_one(const uint8_t *__restrict__ r, uint8_t ver,
                                               uint32_t d[8]) {
    const uint32_t ml = ((uint32_t)r[0] << 8) | r[1];
    const uint32_t kl = ((uint32_t)r[2 + ml] << 8) | r[3 + ml];
    if (ver == 1)
        sha256_skip12(r, 4 + ml + kl, d);
    else
        sha256_skip12(r + 4 + ml, kl, d);
}

__global__ __launch_bounds__(256) void k_txe_leaf(uint64_t n, const uint8_t *__restrict__ buf,
                                                  const uint64_t *__restrict__ rec_off,
                                                  const uint8_t *__restrict__ ver, int leaf,
                                                  uint8_t *__restrict__ out) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    uint32_t d[8];
    txe_digest_one(buf + rec_off[e], ver[e], d);
    if (leaf) {
        uint32_t h[8];
        leaf_hash(d, h);
        store_digest(out + e * 32, h);
    } else {
        store_digest(out + e * 32, d);
    }
}

// TxHeader of each record from the raw tx-log bytes (the fields readHeader
// reads, tx.go:419-518; the host hop already validated the structure), plus
// the offset of its first entry.  md_off is relative to the log buffer.
// returns the offset of the record's first entry
__device__ __forceinline__ uint64_t tx_hdr_one(const uint8_t *__restrict__ buf, uint64_t p,
                                               MhTxHeader &h) {
    const uint8_t *r = buf + p;
    auto be = [&](int o, int n) {
        uint64_t v = 0;
        for (int k = 0; k < n; k++) v = v << 8 | r[o + k];
        return v;
    };
    h.id = be(0, 8);
    h.ts = (int64_t)be(8, 8);
    h.bl_tx_id = be(16, 8);
    for (int k = 0; k < 32; k++) {
        h.bl_root[k] = r[24 + k];
        h.prev_alh[k] = r[56 + k];
        h.eh[k] = 0;
    }
    h.version = (uint32_t)be(88, 2);
    uint64_t q = 90;
    if (h.version == 0) {
        h.nentries = (uint32_t)be(90, 2);
        h.md_len = 0;
        h.md_off = 0;
        q = 92;
    } else {
        h.md_len = (uint32_t)be(90, 2);
        h.md_off = (uint32_t)(p + 92);
        h.nentries = (uint32_t)be(92 + h.md_len, 4);
        q = 96 + h.md_len;
    }
    return p + q;
}

__global__ __launch_bounds__(256) void k_tx_hdr_from_raw(uint64_t ntx, const uint8_t *__restrict__ buf,
                                                         const uint64_t *__restrict__ rec_off,
                                                         MhTxHeader *__restrict__ hdrs,
                                                         uint64_t *__restrict__ ent_start) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    MhTxHeader h;
    ent_start[t] = tx_hdr_one(buf, rec_off[t], h);
    hdrs[t] = h;
}

__global__ __launch_bounds__(256) void k_put_eh(uint64_t n, const uint8_t *__restrict__ eh,
                                                MhTxHeader *__restrict__ hdrs) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    for (int k = 0; k < 32; k++) hdrs[t].eh[k] = eh[t * 32 + k];
}

hipError_t launch_tx_hdr_from_raw(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                                  const uint64_t *rec_off, MhTxHeader *hdrs, uint64_t *ent_start) {
    if (!ntx) return hipSuccess;
    TimerScope ts(tm, "tx_hdr_from_raw", st);
    hipLaunchKernelGGL(k_tx_hdr_from_raw, dim3(grid_for(ntx, 256)), dim3(256), 0, st, ntx, buf,
                       rec_off, hdrs, ent_start);
    return hipGetLastError();
}

// Up to three runs of 64-bit words from pinned host memory into HBM, read by
// the kernel over PCIe: a small upload that does not queue behind the large
// host-to-device copies the DMA engine is busy with (the tx-log chunks).
__global__ __launch_bounds__(256) void k_fetch_host(HostRuns r) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (int k = 0; k < 3; k++)
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.n[k]; i += stride)
            r.dst[k][i] = r.src[k][i];
}

hipError_t launch_fetch_host(hipStream_t st, const HostRuns &r) {
    const uint64_t m = std::max(r.n[0], std::max(r.n[1], r.n[2]));
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_fetch_host, dim3((unsigned)std::min<uint64_t>(grid_for(m, 256), 1024)),
                       dim3(256), 0, st, r);
    return hipGetLastError();
}

// Up to three runs of 32-bit words from HBM into pinned host memory by
// kernel stores over PCIe: results that do not wait for the DMA engine.  A
// run whose ends are 16-byte aligned goes in 16-byte stores (4-byte stores
// reach only ~25 GB/s over the link).
__global__ __launch_bounds__(256) void k_store_host(HostWordRuns r) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < 3; k++) {
        const uint64_t n = r.n[k];
        if ((((uintptr_t)r.src[k] | (uintptr_t)r.dst[k]) & 15) == 0) {
            const uint4 *s = reinterpret_cast<const uint4 *>(r.src[k]);
            uint4 *d = reinterpret_cast<uint4 *>(r.dst[k]);
            for (uint64_t i = tid; i < n / 4; i += stride) d[i] = s[i];
            for (uint64_t i = (n & ~3ull) + tid; i < n; i += stride) r.dst[k][i] = r.src[k][i];
        } else {
            for (uint64_t i = tid; i < n; i += stride) r.dst[k][i] = r.src[k][i];
        }
    }
    __threadfence_system();
}

hipError_t launch_store_host(hipStream_t st, const HostWordRuns &r) {
    const uint64_t m = std::max(r.n[0], std::max(r.n[1], r.n[2]));
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_store_host, dim3((unsigned)std::min<uint64_t>(grid_for(m / 4 + 1, 256), 1024)),
                       dim3(256), 0, st, r);
    return hipGetLastError();
}

hipError_t launch_put_eh(hipStream_t st, uint64_t n, const uint8_t *eh, MhTxHeader *hdrs) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_put_eh, dim3(grid_for(n, 256)), dim3(256), 0, st, n, eh, hdrs);
    return hipGetLastError();
}

// Entry index of a run of tx records (tx.go:520-588 readEntry, structure
// only), one lane per tx: the host hop already validated every length, so
// the lane walks its entries from ent_start[t] and records each entry's
// record offset and header version for k_txe_leaf.
__global__ __launch_bounds__(256) void k_txe_index(uint64_t ntx, const uint8_t *__restrict__ buf,
                                                   const MhTxHeader *__restrict__ hdrs,
                                                   const uint64_t *__restrict__ ent_start,
                                                   const uint64_t *__restrict__ leaf_off,
                                                   uint64_t *__restrict__ rec_off,
                                                   uint8_t *__restrict__ ver) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    const uint8_t v = (uint8_t)hdrs[t].version;
    uint64_t q = ent_start[t];
    for (uint64_t e = leaf_off[t]; e < leaf_off[t + 1]; e++) {
        const uint32_t ml = ((uint32_t)buf[q] << 8) | buf[q + 1];
        const uint32_t kl = ((uint32_t)buf[q + 2 + ml] << 8) | buf[q + 3 + ml];
        rec_off[e] = q;
        ver[e] = v;
        q += 4 + ml + kl + 12 + 32;
    }
}

hipError_t launch_txe_index(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                            const MhTxHeader *hdrs, const uint64_t *ent_start,
                            const uint64_t *leaf_off, uint64_t *rec_off, uint8_t *ver) {
    if (!ntx) return hipSuccess;
    TimerScope ts(tm, "txe_index", st);
    hipLaunchKernelGGL(k_txe_index, dim3(grid_for(ntx, 256)), dim3(256), 0, st, ntx, buf, hdrs,
                       ent_start, leaf_off, rec_off, ver);
    return hipGetLastError();
}

__global__ void k_txlog_patch(uint64_t ne, const uint64_t *__restrict__ e_idx,
                              const uint64_t *__restrict__ e_off, uint64_t *__restrict__ rec_off,
                              uint64_t nh, const uint64_t *__restrict__ h_idx,
                              const uint64_t *__restrict__ h_val, MhTxHeader *__restrict__ hdrs) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ne) rec_off[e_idx[t]] = e_off[t];
    if (t < nh) {
        hdrs[h_idx[t]].md_off = (uint32_t)h_val[t];
        hdrs[h_idx[t]].md_len = (uint32_t)(h_val[t] >> 32);
    }
}

hipError_t launch_txlog_patch(hipStream_t st, uint64_t ne, const uint64_t *e_idx,
                              const uint64_t *e_off, uint64_t *rec_off, uint64_t nh,
                              const uint64_t *h_idx, const uint64_t *h_val, MhTxHeader *hdrs) {
    const uint64_t n = std::max(ne, nh);
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_txlog_patch, dim3(grid_for(n, 256)), dim3(256), 0, st, ne, e_idx, e_off,
                       rec_off, nh, h_idx, h_val, hdrs);
    return hipGetLastError();
}

__device__ __constant__ static const uint8_t kEmptyRootDev[32] = {
    0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4, 0xc8, 0x99, 0x6f, 0xb9, 0x24,
    0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

// Roots of many small htrees, one lane per tree, level by level in place
// over the tree's own leaf range (exactly htree.go:85-110: node k of the next
// level = H(node 2k, node 2k+1) written to slot k -- slots 2k, 2k+1 >= k are
// read first -- and an odd last node promoted to slot (w-1)/2).  nodes holds
// the leaf hashes of all trees back to back and is consumed.  Width 0 gives
// SHA256(nil) (htree.go:73-77).  For batches whose widest tree is small
// (immudb txs: a handful of entries) this replaces the host tree plan.
__global__ __launch_bounds__(256) void k_small_roots(uint64_t ntrees,
                                                     const uint64_t *__restrict__ leaf_off,
                                                     uint8_t *__restrict__ nodes,
                                                     uint8_t *__restrict__ roots) {
    extern __shared__ uint32_t tab[];
    node_tab_init(tab);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntrees) return;
    uint8_t *lv = nodes + (leaf_off[t] - leaf_off[0]) * 32;
    uint64_t w = leaf_off[t + 1] - leaf_off[t];
    const uint4 *src;
    if (w == 0) {
        src = reinterpret_cast<const uint4 *>(kEmptyRootDev);
    } else {
        while (w > 1) {
            const uint64_t half = w / 2;
            for (uint64_t k = 0; k < half; k++) {
                uint32_t a[8], b[8], h[8];
                load_digest(lv + 64 * k, a);
                load_digest(lv + 64 * k + 32, b);
                node_hash_tab(a, b, h, tab);
                store_digest(lv + 32 * k, h);
            }
            if (w & 1) {  // promote the odd last node
                const uint4 *q = reinterpret_cast<const uint4 *>(lv + 32 * (w - 1));
                uint4 *d = reinterpret_cast<uint4 *>(lv + 32 * half);
                const uint4 x = q[0], y = q[1];
                d[0] = x;
                d[1] = y;
            }
            w = (w + 1) / 2;
        }
        src = reinterpret_cast<const uint4 *>(lv);
    }
    uint4 *d = reinterpret_cast<uint4 *>(roots + t * 32);
    d[0] = src[0];
    d[1] = src[1];
}

// The same roots with one WAVE per tree (width <= 64): lane k holds node k of
// the current level in LDS, every level's nodes are hashed at once, so a tree
// costs ceil(log2 w) node-hash latencies instead of w - 1 -- for the small
// batches of a group commit, where the lane-per-tree kernel is one lone
// wave walking each tree serially.
__global__ __launch_bounds__(256) void k_small_roots_wave(uint64_t ntrees,
                                                          const uint64_t *__restrict__ leaf_off,
                                                          const uint8_t *__restrict__ nodes,
                                                          uint8_t *__restrict__ roots) {
    __shared__ uint32_t lvl[4][64][9];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
    if (t >= ntrees) return;  // wave-uniform
    const uint8_t *lv = nodes + (leaf_off[t] - leaf_off[0]) * 32;
    uint64_t w = leaf_off[t + 1] - leaf_off[t];
    if (w == 0) {
        if (lane < 2)
            reinterpret_cast<uint4 *>(roots + t * 32)[lane] =
                reinterpret_cast<const uint4 *>(kEmptyRootDev)[lane];
        return;
    }
    uint32_t(*L)[9] = lvl[wv];
    if ((uint64_t)lane < w) {
        uint32_t d[8];
        load_digest(lv + 32 * lane, d);
#pragma unroll
        for (int j = 0; j < 8; j++) L[lane][j] = d[j];
    }
    while (w > 1) {  // htree.go:85-110, level by level
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint64_t half = w / 2;
        uint32_t a[8], b[8], h[8];
        const bool hash = (uint64_t)lane < half, promote = (w & 1) && (uint64_t)lane == half;
        if (hash || promote) {
#pragma unroll
            for (int j = 0; j < 8; j++) a[j] = L[promote ? w - 1 : 2 * lane][j];
        }
        if (hash) {
#pragma unroll
            for (int j = 0; j < 8; j++) b[j] = L[2 * lane + 1][j];
            node_hash_g(a, b, h);
        } else {
            copy8(h, a);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (hash || promote) {
#pragma unroll
            for (int j = 0; j < 8; j++) L[lane][j] = h[j];
        }
        w = (w + 1) / 2;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) {
        uint32_t r[8];
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] = L[0][j];
        store_digest(roots + t * 32, r);
    }
}

// The same roots for MANY small trees, level-parallel: a 256-thread
// workgroup takes TPW = 512 / P consecutive trees (P = the widest tree rounded
// up to a power of two, <= 64), their leaves in LDS at stride P, and hashes
// every node of a level at once -- node j of tree k at level l on thread
// k * (P >> l) + j, so level 1 keeps all 256 threads busy (for trees of the
// widest width), each further level half as many -- double-buffered in LDS
// (htree.go:85-110: pairs hashed, an odd last node promoted).  Against one
// lane per tree (k_small_roots: w - 1 dependent node hashes on a lone wave
// per SIMD) the work is the same but spread over 8x the waves.
__global__ __launch_bounds__(256) void k_small_roots_pack(uint64_t ntrees,
                                                          const uint64_t *__restrict__ leaf_off,
                                                          const uint8_t *__restrict__ nodes,
                                                          uint8_t *__restrict__ roots, int lgp) {
    __shared__ uint32_t buf[2][512][9];  // +1 word pad: 2j / 2j+1 reads spread over the banks
    const int P = 1 << lgp, TPW = 512 >> lgp;
    const int tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * TPW;
    const uint64_t o0 = leaf_off[0];
    for (int i = tid; i < TPW * P; i += 256) {
        const int k = i >> lgp, j = i & (P - 1);
        const uint64_t t = t0 + k;
        if (t >= ntrees) continue;
        const uint64_t lo = leaf_off[t], w = leaf_off[t + 1] - lo;
        if ((uint64_t)j < w) {
            uint32_t d[8];
            load_digest(nodes + (lo - o0 + j) * 32, d);
#pragma unroll
            for (int q = 0; q < 8; q++) buf[0][i][q] = d[q];
        }
    }
    int cur = 0;
    for (int l = 1; l <= lgp; l++) {
        __syncthreads();
        const int S = P >> l;  // node slots per tree at level l
        if (tid < TPW * S) {
            const int k = tid / S, j = tid - k * S;
            const uint64_t t = t0 + k;
            if (t < ntrees) {
                const uint64_t w = leaf_off[t + 1] - leaf_off[t];
                const uint64_t wp = (w + (1ull << (l - 1)) - 1) >> (l - 1);  // width at level l-1
                const int a = k * P + 2 * j;
                if ((uint64_t)(2 * j + 1) < wp) {
                    uint32_t x[8], y[8], h[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        x[q] = buf[cur][a][q];
                        y[q] = buf[cur][a + 1][q];
                    }
                    node_hash_g(x, y, h);
#pragma unroll
                    for (int q = 0; q < 8; q++) buf[cur ^ 1][k * P + j][q] = h[q];
                } else if ((uint64_t)(2 * j) < wp) {  // odd last node: promoted
#pragma unroll
                    for (int q = 0; q < 8; q++) buf[cur ^ 1][k * P + j][q] = buf[cur][a][q];
                }
            }
        }
        cur ^= 1;
    }
    __syncthreads();
    if (tid < TPW) {
        const uint64_t t = t0 + tid;
        if (t < ntrees) {
            if (leaf_off[t + 1] == leaf_off[t]) {  // width 0: SHA256(nil), htree.go:73-77
                reinterpret_cast<uint4 *>(roots + t * 32)[0] = reinterpret_cast<const uint4 *>(kEmptyRootDev)[0];
                reinterpret_cast<uint4 *>(roots + t * 32)[1] = reinterpret_cast<const uint4 *>(kEmptyRootDev)[1];
            } else {
                uint32_t r[8];
#pragma unroll
                for (int q = 0; q < 8; q++) r[q] = buf[cur][tid * P][q];
                store_digest(roots + t * 32, r);
            }
        }
    }
}

hipError_t launch_small_roots(hipStream_t st, Timer *tm, uint64_t ntrees, const uint64_t *leaf_off,
                              uint8_t *nodes, uint8_t *roots, uint64_t wmax) {
    if (!ntrees) return hipSuccess;
    TimerScope ts(tm, "small_roots", st);
    if (ntrees <= 2048) {
        // few trees: latency-bound, a wave per tree
        hipLaunchKernelGGL(k_small_roots_wave, dim3(grid_for(ntrees, 4)), dim3(256), 0, st, ntrees,
                           leaf_off, nodes, roots);
    } else if (wmax <= 64 && !getenv("MH_SMALL_ROOTS_LANE")) {
        int lgp = 0;
        while ((1ull << lgp) < wmax) lgp++;
        lgp = std::max(lgp, 1);
        const uint64_t tpw = 512 >> lgp;
        hipLaunchKernelGGL(k_small_roots_pack, dim3(grid_for(ntrees, (unsigned)tpw)), dim3(256), 0,
                           st, ntrees, leaf_off, nodes, roots, lgp);
    } else {
        hipLaunchKernelGGL(k_small_roots, dim3(grid_for(ntrees, 256)), dim3(256), kNodeTabBytes, st,
                           ntrees, leaf_off, nodes, roots);
    }
    return hipGetLastError();
}

// The levels above a row of w <= 64 inner nodes in ONE launch
// (mh_dev_htree_reduce_nodes for the all-gathered shard roots of a multi-GPU
// build, w = ranks): one wave, node k of the current level on lane k in LDS,
// every level's nodes hashed at once (htree.go:85-110: pairs, an odd last
// node promoted) and written to levels in the flat level-major layout
// (level 0 = the input row), the root to root.  Replaces a copy kernel, the
// level launches and a device-to-device copy per build.
__global__ __launch_bounds__(64) void k_reduce_small(const uint8_t *__restrict__ nodes, uint32_t w,
                                                     uint8_t *__restrict__ levels,
                                                     uint8_t *__restrict__ root) {
    __shared__ uint32_t L[64][9];
    const uint32_t lane = threadIdx.x;
    if (lane < w) {
        uint32_t d[8];
        load_digest(nodes + 32 * lane, d);
#pragma unroll
        for (int j = 0; j < 8; j++) L[lane][j] = d[j];
        store_digest(levels + 32 * lane, d);
    }
    uint64_t off = w;
    while (w > 1) {
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t half = w / 2;
        uint32_t a[8], b[8], h[8];
        const bool hash = lane < half, promote = (w & 1) && lane == half;
        if (hash || promote) {
#pragma unroll
            for (int j = 0; j < 8; j++) a[j] = L[promote ? w - 1 : 2 * lane][j];
        }
        if (hash) {
#pragma unroll
            for (int j = 0; j < 8; j++) b[j] = L[2 * lane + 1][j];
            node_hash_g(a, b, h);
        } else {
            copy8(h, a);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (hash || promote) {
#pragma unroll
            for (int j = 0; j < 8; j++) L[lane][j] = h[j];
            store_digest(levels + 32 * (off + lane), h);
        }
        w = (w + 1) / 2;
        off += w;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0 && root) {
        uint32_t r[8];
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] = L[0][j];
        store_digest(root, r);
    }
}

hipError_t launch_reduce_small(hipStream_t st, const uint8_t *nodes, uint64_t w, uint8_t *levels,
                               uint8_t *root) {
    if (w == 0 || w > kSmallTreeMax) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_reduce_small, dim3(1), dim3(64), 0, st, nodes, (uint32_t)w, levels, root);
    return hipGetLastError();
}

// The whole a14 check of a group of tx-log records whose trees are small, in
// ONE launch (tx.go:533-630 per record: header, entry walk, entry digests and
// leaves, the tx's htree, innerHash + Alh against the stored Alh).  A
// 256-thread workgroup takes TPW = 512 >> lgp consecutive records (every tx
// <= P = 1 << lgp entries, P <= 64): lane k < TPW parses record k's header
// and walks its entries into LDS; every thread then hashes entry digests and
// leaves (two entry slots per thread), the trees are reduced level-parallel in
// LDS exactly as k_small_roots_pack does (htree.go:85-110), and lane k ends
// with innerHash + Alh (tx.go:249-319).  Replaces the six dependent launches
// of a group (header, entry index, leaves, small roots, Alh, Eh copy), whose
// latencies added up after the last chunk of the log had landed.  Groups with
// metadata patches (a header or entry whose metadata the host re-encoded)
// keep the multi-launch path.
static_assert(sizeof(MhTxHeader) == 17 * 8, "headers are staged as 17 words");

__global__ __launch_bounds__(256) void k_txlog_group(
    uint64_t ntx, const uint8_t *__restrict__ buf, const uint64_t *__restrict__ rec_off,
    const uint64_t *__restrict__ alh_off, const uint64_t *__restrict__ leaf_off,
    MhTxHeader *__restrict__ hdrs, uint8_t *__restrict__ scratch, uint8_t *__restrict__ eh_out,
    uint8_t *__restrict__ alh_out, int32_t *__restrict__ status, TxlogHostOut ho, int lgp,
    int warm) {
    __shared__ uint32_t nb[2][512][9];  // +1 word pad, as k_small_roots_pack; headers staged here last
    __shared__ uint64_t erec[1024];     // entry record offsets (tree k at k * P); Alh staged here last
    __shared__ uint8_t tver[256];
    const int P = 1 << lgp, TPW = 512 >> lgp;
    const int tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * TPW;
    const uint64_t nmine = min((uint64_t)TPW, ntx - t0);  // records of this workgroup
    const bool mine = (uint64_t)tid < nmine;            // this lane owns record t0 + tid
    if (warm) {
        // The workgroup's records are contiguous in the log (record t ends
        // with its stored Alh at alh_off[t]): every thread touches 16-byte
        // pieces of that range at once, so the serial header / entry walks
        // below hit L2 instead of paying an HBM round trip per dependent load.
        const uint64_t lo = rec_off[t0] & ~15ull, hi = alh_off[t0 + nmine - 1] + 32;
        uint32_t acc = 0;
        for (uint64_t p = lo + 16 * (uint64_t)tid; p < hi; p += 16 * 256)
            acc ^= reinterpret_cast<const uint4 *>(buf + p)->x;
        asm volatile("" ::"v"(acc));
    }
    if (mine) {
        const uint64_t t = t0 + tid;
        MhTxHeader h;
        uint64_t q = tx_hdr_one(buf, rec_off[t], h);  // tx.go:419-518
        hdrs[t] = h;
        tver[tid] = (uint8_t)h.version;
        const uint64_t w = leaf_off[t + 1] - leaf_off[t];
        for (uint64_t j = 0; j < w; j++) {  // tx.go:578-585 (lengths validated by the hop)
            const uint32_t ml = ((uint32_t)buf[q] << 8) | buf[q + 1];
            const uint32_t kl = ((uint32_t)buf[q + 2 + ml] << 8) | buf[q + 3 + ml];
            erec[tid * P + j] = q;
            q += 4 + ml + kl + 12 + 32;
        }
    }
    __syncthreads();
    for (int i = tid; i < TPW * P; i += 256) {  // entry digest + leaf (tx.go:690-731, htree.go:79-83)
        const int k = i >> lgp, j = i & (P - 1);
        const uint64_t t = t0 + k;
        if (t < ntx && (uint64_t)j < leaf_off[t + 1] - leaf_off[t]) {
            uint32_t d[8], h[8];
            txe_digest_one(buf + erec[i], tver[k], d);
            leaf_hash(d, h);
#pragma unroll
            for (int q = 0; q < 8; q++) nb[0][i][q] = h[q];
        }
    }
    int cur = 0;
    for (int l = 1; l <= lgp; l++) {  // htree.go:85-110, every tree of the workgroup at once
        __syncthreads();
        const int S = P >> l;
        if (tid < TPW * S) {
            const int k = tid / S, j = tid - k * S;
            const uint64_t t = t0 + k;
            if (t < ntx) {
                const uint64_t w = leaf_off[t + 1] - leaf_off[t];
                const uint64_t wp = (w + (1ull << (l - 1)) - 1) >> (l - 1);
                const int a = k * P + 2 * j;
                if ((uint64_t)(2 * j + 1) < wp) {
                    uint32_t x[8], y[8], h[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        x[q] = nb[cur][a][q];
                        y[q] = nb[cur][a + 1][q];
                    }
                    node_hash_g(x, y, h);
#pragma unroll
                    for (int q = 0; q < 8; q++) nb[cur ^ 1][k * P + j][q] = h[q];
                } else if ((uint64_t)(2 * j) < wp) {
#pragma unroll
                    for (int q = 0; q < 8; q++) nb[cur ^ 1][k * P + j][q] = nb[cur][a][q];
                }
            }
        }
        cur ^= 1;
    }
    __syncthreads();
    const uint64_t t = t0 + tid;
    uint32_t eh[8];
    if (mine) {
        if (leaf_off[t + 1] == leaf_off[t]) {  // no entries: SHA256(nil), htree.go:73-77
            load_digest(kEmptyRootDev, eh);
        } else {
#pragma unroll
            for (int q = 0; q < 8; q++) eh[q] = nb[cur][tid * P][q];
        }
    }
    __syncthreads();  // nb and erec are free: results are staged there
    uint64_t *hst = reinterpret_cast<uint64_t *>(&nb[0][0][0]);  // nmine headers, 17 words each
    uint32_t *ast = reinterpret_cast<uint32_t *>(erec);          // nmine Alh, 8 words each
    if (mine) {
        store_digest(eh_out + t * 32, eh);
        uint32_t *he = reinterpret_cast<uint32_t *>(hdrs[t].eh);  // 8-byte aligned field
#pragma unroll
        for (int q = 0; q < 8; q++) he[q] = bswap(eh[q]);
        tx_alh_one(t, hdrs[t], buf, eh_out + t * 32, scratch + t * kTxInnerStride,
                   buf + alh_off[t], nullptr, alh_out, status);
        // results straight into the caller's pinned arrays (no store kernel
        // after the group): the lane's own status, the workgroup's Alh and
        // headers staged in LDS and written below as contiguous runs
        if (ho.status) ho.status[t] = (uint32_t)status[t];
        if (ho.alh) {
            const uint32_t *a = reinterpret_cast<const uint32_t *>(alh_out + t * 32);
#pragma unroll
            for (int q = 0; q < 8; q++) ast[tid * 8 + q] = a[q];
        }
        if (ho.hdrs) {
            const uint64_t *hw = reinterpret_cast<const uint64_t *>(hdrs + t);
#pragma unroll
            for (int q = 0; q < 17; q++) hst[tid * 17 + q] = hw[q];
        }
    }
    if (ho.alh || ho.hdrs) {  // kernel arguments: uniform
        __syncthreads();
        if (ho.alh)
            for (uint64_t i = tid; i < nmine * 8; i += 256) ho.alh[t0 * 8 + i] = ast[i];
        if (ho.hdrs)
            for (uint64_t i = tid; i < nmine * 17; i += 256) ho.hdrs[t0 * 17 + i] = hst[i];
    }
    if (ho.status || ho.alh || ho.hdrs) __threadfence_system();
}

hipError_t launch_txlog_group(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                              const uint64_t *rec_off, const uint64_t *alh_off,
                              const uint64_t *leaf_off, MhTxHeader *hdrs, uint8_t *scratch,
                              uint8_t *eh_out, uint8_t *alh_out, int32_t *status,
                              const TxlogHostOut &ho, uint64_t wmax) {
    if (!ntx) return hipSuccess;
    if (wmax > 64 || ((uintptr_t)ho.hdrs & 7) || ((uintptr_t)ho.alh & 3) || ((uintptr_t)ho.status & 3))
        return hipErrorInvalidValue;
    int lgp = 1;
    while ((1ull << lgp) < wmax) lgp++;
    const uint64_t tpw = 512 >> lgp;
    static const int warm = [] {
        const char *e = getenv("MH_TXLOG_WARM");
        return e ? atoi(e) : 1;
    }();
    TimerScope ts(tm, "txlog_group", st);
    hipLaunchKernelGGL(k_txlog_group, dim3(grid_for(ntx, (unsigned)tpw)), dim3(256), 0, st, ntx,
                       buf, rec_off, alh_off, leaf_off, hdrs, scratch, eh_out, alh_out, status, ho,
                       lgp, warm);
    return hipGetLastError();
}

// ---------------------------------------------------------------- a14, wave per records
// The same a14 check of a group (tx.go:533-630 per record) with ONE WAVE per
// R = 64 / L consecutive records and L lanes per record, so that nothing of a
// record waits on another wave and a record's tree is reduced by shuffles
// (four independent waves per workgroup: the dispatcher spreads workgroups
// over the CUs and a workgroup's waves over the CU's four SIMDs, so a small
// launch -- the last chunk's group -- runs one wave per SIMD):
//   1. the wave's records (contiguous in the log, each ending with its stored
//      Alh) are copied into LDS with 16-byte loads, one HBM round trip; the
//      header parse, the entry walk and the entry digests then read LDS (a
//      wave whose records do not fit reads the log in HBM instead);
//   2. the record's first lane walks its entries (tx.go:578-585, lengths
//      validated by the host hop) into an LDS offset table;
//   3. lane i of a record hashes entries E*i .. E*i+E-1 (entry digest
//      tx.go:690-731 + leaf htree.go:79-83, in place from the raw records)
//      and reduces them to its level-log2(E) node; the L lanes then reduce
//      those level by level with cross-lane shuffles (htree.go:85-110:
//      node (k, l) hashes its two children when the right one covers any leaf,
//      else it is its left child promoted);
//   4. the record's lanes assemble the innerHash message ts || version ||
//      (mdLen || md)? || nentries || Eh || blTxID || blRoot (tx.go:249-302;
//      every part but Eh is a byte range of the record head) as SHA words in
//      LDS, the first lane hashes it and the Alh (tx.go:307-319) and compares
//      it with the stored one;
//   5. the results are staged in LDS and the whole workgroup stores its
//      records' header words, Alh words and statuses as contiguous runs
//      (device arrays, and the caller's pinned arrays when given).
// Against k_txlog_group (one lane per record walks, parses and hashes the
// Alh while the other lanes wait at workgroup barriers) a record's serial
// chain is ~16 compressions of one wave with no workgroup barrier until the
// final store.
__device__ __forceinline__ uint32_t rd_le32(const uint8_t *p) {  // 4 bytes of any alignment
    const uint32_t al = (uint32_t)((uintptr_t)p & 3);
    const uint32_t *b = reinterpret_cast<const uint32_t *>(p - al);
    return __builtin_amdgcn_alignbyte(b[1], b[0], al);
}
__device__ __forceinline__ uint32_t rd_be16(const uint8_t *p) {
    return ((uint32_t)p[0] << 8) | p[1];
}
__device__ __forceinline__ uint64_t rd_be64(const uint8_t *p) {
    return ((uint64_t)bswap(rd_le32(p)) << 32) | bswap(rd_le32(p + 4));
}
__device__ __forceinline__ uint64_t rd_raw64(const uint8_t *p) {
    return (uint64_t)rd_le32(p) | ((uint64_t)rd_le32(p + 4) << 32);
}

constexpr int kTxMsgWords = 96;  // innerHash message <= 356 B: 6 blocks
typedef __attribute__((address_space(3))) void tx_lds_void_t;
typedef __attribute__((address_space(1))) void tx_glb_void_t;

// ---- the same record pipeline with ONE compression site (txlog_wave_loop).
// Every hash of a record -- entry digests, leaves, the tree's nodes, the
// innerHash and the Alh -- is a sequence of message blocks; each lane walks
// its own sequence through one loop whose body builds the lane's next block
// and runs the one inlined compress.  The kernel's code is then ~one
// compression long instead of ~20 straight-line copies (173 KB, more than the
// CU pair's instruction cache: waves at different points of it stall on
// instruction fetch).

// first min(max(n, 0), 4) bytes of a big-endian word: (~0 << 32) >> 8c
__device__ __forceinline__ uint32_t head_mask(int n) {
    const int c = min(max(n, 0), 4);
    return (uint32_t)(0xffffffff00000000ull >> (8 * c));
}

// block b of nb of SHA256(p[0:la] || p[la+12 : la+44]) (sha256_skip12's
// words), padding included.  GUARD: loads confined to [p, p + la + 44) (the
// log in HBM); staged records have >= 96 readable bytes past every message
// the 20 dwords block b of skip12_block reads (unguarded)
__device__ __forceinline__ void skip12_load(const uint8_t *p, uint32_t b, uint32_t d[20]) {
    const uint32_t *qq = reinterpret_cast<const uint32_t *>(p - ((uintptr_t)p & 3)) + b * 16;
#pragma unroll
    for (int j = 0; j < 20; j++) d[j] = qq[j];
}
// Message words j = 0..15 of block b from the 20 dwords d[] read at the
// block's aligned start (al = p & 3, hv0 = la - 64 b): the head bytes, then
// the hVal 12 bytes further on, cut at the message end (la + 32 - 64 b) with
// the 0x80 marker after it.  Each word's bytes come out of one v_perm (the
// byte-aligned window and the big-endian swap in one selector); the end mask
// of word j is the head mask of word j - 8 (the message ends 32 bytes after
// the head), and the marker is the one byte by which the end mask of a
// message one byte longer, (em_j >> 8) | (em_{j-1} << 24), exceeds em_j --
// 25 masks for the 48 masks and markers of the direct form.
__device__ __forceinline__ void skip12_assemble(const uint32_t d[20], uint32_t al, int hv0,
                                                uint32_t w[16]) {
    const uint32_t sel = be_sel(al);
    uint32_t hm[25];  // hm[k] = head_mask(hv0 - 4 (k - 9)): words -9..15
#pragma unroll
    for (int k = 0; k < 25; k++) hm[k] = head_mask(hv0 - 4 * (k - 9));
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t w1 = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
        const uint32_t w2 = __builtin_amdgcn_perm(d[j + 4], d[j + 3], sel);
        const uint32_t x = __builtin_amdgcn_bitop3_b32(hm[j + 9], w1, w2, 0xCA);  // head ? w1 : w2
        const uint32_t em = hm[j + 1], nm = __builtin_amdgcn_alignbit(hm[j], em, 8);
        w[j] = __builtin_amdgcn_bitop3_b32(em, x, nm & 0x80808080u, 0xCA);  // message ? x : marker
    }
}
// the block's message words from those dwords (al = p & 3)
__device__ __forceinline__ void skip12_words(const uint32_t d[20], uint32_t al, uint32_t la,
                                             uint32_t b, uint32_t nb, uint32_t w[16]) {
    const uint32_t L = la + 32;
    skip12_assemble(d, al, (int)la - (int)(b * 64), w);
    if (b + 1 == nb) {
        w[14] = 0;
        w[15] = L * 8;
    }
}

template <bool GUARD>
__device__ __forceinline__ void skip12_block(const uint8_t *p, uint32_t la, uint32_t b,
                                             uint32_t nb, uint32_t w[16]) {
    const uint32_t L = la + 32;
    const uint32_t al = (uint32_t)((uintptr_t)p & 3);
    const uint32_t *qq = reinterpret_cast<const uint32_t *>(p - al) + b * 16;
    uint32_t d[20];
    if (GUARD) {
        const uint8_t *end = p + la + 44;
#pragma unroll
        for (int j = 0; j < 20; j++) d[j] = ld_guard(qq + j, p, end);
    } else {
#pragma unroll
        for (int j = 0; j < 20; j++) d[j] = qq[j];
    }
    skip12_assemble(d, al, (int)la - (int)(b * 64), w);
    if (b + 1 == nb) {
        w[14] = 0;
        w[15] = L * 8;
    }
}

// MH_TXLOG_PROBE=1: s_memtime stamps of each wave's phases (diagnosis only;
// the pointer is null otherwise), reported by txlog_probe_report(); pw is
// the wave's slot
#define TXW_PROBE(k)                                                                              \
    do {                                                                                          \
        if (probe && (threadIdx.x & 63) == 0) probe[pw * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// a wave's LDS writes complete and visible to its other lanes (each wave
// works in its own LDS slices: no workgroup barrier)
#define TXW_SYNC()                                                                                \
    do {                                                                                          \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                       \
        __builtin_amdgcn_wave_barrier();                                                          \
    } while (0)

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, m, 64));
    return x;
}

template <int E, bool GUARD>
__device__ __forceinline__ void txlog_wave_body_loop(
    const uint8_t *rp, const uint8_t *ap, uint64_t t, uint64_t rec_g, uint64_t w, bool act,
    int lgl, int r, int i, uint32_t *__restrict__ eoff, uint32_t *__restrict__ msg,
    uint32_t *__restrict__ ehb, uint8_t *__restrict__ eh_out, uint8_t *__restrict__ alh_out,
    int32_t *__restrict__ status, uint64_t *probe, uint64_t pw) {
    const int L = 1 << lgl, P = L * E, R = 64 >> lgl;
    uint32_t ver = 0, ml = 0, nent = 0, q0 = 92;
    if (act) {  // tx.go:419-518
        ver = rd_be16(rp + 88);
        if (ver == 0) {
            nent = rd_be16(rp + 90);
        } else {
            ml = rd_be16(rp + 90);
            nent = bswap(rd_le32(rp + 92 + ml));
            q0 = 96 + ml;
        }
    }
    if (act && i == 0) {  // the entry walk, tx.go:578-585
        uint32_t q = q0;
        for (uint64_t j = 0; j < w; j++) {
            eoff[r * P + j] = q;
            const uint32_t m = rd_be16(rp + q);
            const uint32_t k = rd_be16(rp + q + 2 + m);
            q += 48 + m + k;
        }
    }
    TXW_SYNC();
    TXW_PROBE(2);
    // this lane's entries: digest message start / head length / blocks
    const uint8_t *mp0 = rp, *mp1 = rp;
    uint32_t la0 = 0, la1 = 0, nb0 = 0, nb1 = 0, steps0 = 0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint64_t j = (uint64_t)i * E + e;
        if (act && j < w) {
            const uint8_t *er = rp + eoff[r * P + j];
            const uint32_t m = rd_be16(er), k = rd_be16(er + 2 + m);
            const uint8_t *pp = ver == 1 ? er : er + 4 + m;  // tx.go:690-731
            const uint32_t la = ver == 1 ? 4 + m + k : k;
            const uint32_t nb = (la + 32 + 8) / 64 + 1;
            if (e == 0) { mp0 = pp; la0 = la; nb0 = nb; } else { mp1 = pp; la1 = la; nb1 = nb; }
            steps0 += nb + 1;
        }
    }
    const uint32_t blen = ver ? 8 + ml : 4;  // version || (mdLen || md || nentries) | nentries16
    const uint32_t mlen = 80 + blen;
    const uint32_t nw = ((mlen + 8) / 64 + 1) * 16, nbi = nw / 16;
    const uint32_t n0 = wave_max_u32(steps0);
    const uint32_t n1 = 2 * ((E == 2 ? 1 : 0) + lgl);
    const uint32_t n2 = wave_max_u32(act && i == 0 ? nbi + 2 : 0);
    uint32_t *M = msg + r * kTxMsgWords;
    uint32_t *EB = ehb + r * 8;
    State s;
    s.init();
    uint32_t nd[8], lf1[8], rt[8], inner[8];
#pragma unroll
    for (int q = 0; q < 8; q++) nd[q] = lf1[q] = rt[q] = inner[q] = 0;
    uint32_t e = 0, b = 0;
#pragma unroll 1
    for (uint32_t g = 0; g < n0 + n1 + n2; g++) {
        uint32_t wv[16];
        bool on = false, lev = false;
        uint32_t half = 0;
        if (g == n0) TXW_PROBE(3);
        if (g == n0 + n1) TXW_PROBE(4);
        if (g < n0) {  // entry digest blocks, then its leaf (htree.go:79-83)
            const bool e1 = E == 2 && e == 1;
            const uint32_t nbe = e1 ? nb1 : nb0;
            if (e < (uint32_t)E && nbe > 0) {
                on = true;
                if (b < nbe) {
                    if (b == 0) s.init();
                    skip12_block<GUARD>(e1 ? mp1 : mp0, e1 ? la1 : la0, b, nbe, wv);
                } else {
                    wv[0] = s.h[0] >> 8;
#pragma unroll
                    for (int j = 1; j < 8; j++) wv[j] = __builtin_amdgcn_alignbit(s.h[j - 1], s.h[j], 8);
                    wv[8] = (s.h[7] << 24) | 0x00800000u;
#pragma unroll
                    for (int j = 9; j < 15; j++) wv[j] = 0;
                    wv[15] = 33u * 8u;
                    s.init();
                }
            }
        } else if (g < n0 + n1) {  // one tree level per two blocks (htree.go:85-110)
            const uint32_t k = g - n0, lv = k >> 1;
            half = k & 1;
            const bool local = E == 2 && lv == 0;  // the lane's own two leaves
            const uint32_t sft = local ? 0 : 1u << (lv - (E == 2 ? 1 : 0));
            if (half == 0) {
                if (local) {
                    copy8(rt, lf1);
                } else {
#pragma unroll
                    for (int q = 0; q < 8; q++) rt[q] = (uint32_t)__shfl_down((int)nd[q], sft, 64);
                }
            }
            const bool h = local ? act && (uint64_t)i * 2 + 1 < w
                                 : act && (i & (2 * sft - 1)) == 0 && (uint64_t)(i + sft) * E < w;
            if (h) {
                on = lev = true;
                if (half == 0) {
                    s.init();
                    wv[0] = 0x01000000u | (nd[0] >> 8);
#pragma unroll
                    for (int j = 1; j < 8; j++) wv[j] = __builtin_amdgcn_alignbit(nd[j - 1], nd[j], 8);
                    wv[8] = __builtin_amdgcn_alignbit(nd[7], rt[0], 8);
#pragma unroll
                    for (int j = 1; j < 8; j++) wv[8 + j] = __builtin_amdgcn_alignbit(rt[j - 1], rt[j], 8);
                }  // half 1: the padding block, from the K+W table below
            }
        } else {  // innerHash (tx.go:249-302) then Alh (tx.go:307-319)
            const uint32_t k = g - n0 - n1;
            if (k == 0) {
                if (act && i == 0) {
                    if (w == 0) load_digest(kEmptyRootDev, nd);  // SHA256(nil), htree.go:73-77
#pragma unroll
                    for (int q = 0; q < 8; q++) EB[q] = bswap(nd[q]);
                }
                TXW_SYNC();
                if (act) {
                    const uint8_t *eb = reinterpret_cast<const uint8_t *>(EB);
                    for (uint32_t jw = i; jw < nw; jw += L) {
                        uint32_t x = 0;
                        if (jw == nw - 1) {
                            x = mlen * 8;
                        } else {
#pragma unroll
                            for (int bb = 0; bb < 4; bb++) {
                                const uint32_t kk = 4 * jw + bb;
                                uint32_t v;
                                if (kk < 8) v = rp[8 + kk];
                                else if (kk < 8 + blen) v = rp[80 + kk];
                                else if (kk < 40 + blen) v = eb[kk - 8 - blen];
                                else if (kk < mlen) v = rp[kk - 24 - blen];
                                else v = kk == mlen ? 0x80u : 0u;
                                x = x << 8 | v;
                            }
                        }
                        M[jw] = x;
                    }
                }
                TXW_SYNC();
                TXW_PROBE(5);
            }
            if (act && i == 0 && k < nbi + 2) {
                on = true;
                if (k < nbi) {
                    if (k == 0) s.init();
                    const uint4 *m4 = reinterpret_cast<const uint4 *>(M + 16 * k);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint4 y = m4[q];
                        wv[4 * q] = y.x;
                        wv[4 * q + 1] = y.y;
                        wv[4 * q + 2] = y.z;
                        wv[4 * q + 3] = y.w;
                    }
                } else if (k == nbi) {  // BE64 id || prevAlh || innerHash[0:24]
                    copy8(inner, s.h);
                    s.init();
                    const uint64_t id = rd_be64(rp);
                    wv[0] = (uint32_t)(id >> 32);
                    wv[1] = (uint32_t)id;
#pragma unroll
                    for (int q = 0; q < 8; q++) wv[2 + q] = bswap(rd_le32(rp + 56 + 4 * q));
#pragma unroll
                    for (int q = 0; q < 6; q++) wv[10 + q] = inner[q];
                } else {
                    wv[0] = inner[6];
                    wv[1] = inner[7];
                    wv[2] = 0x80000000u;
#pragma unroll
                    for (int q = 3; q < 15; q++) wv[q] = 0;
                    wv[15] = 72u * 8u;
                }
            }
        }
        if (on) {
            if (lev && half == 1)
                compress_node_tail_g(s, rt[7]);
            else
                compress(s, wv);
        }
        if (g < n0) {
            if (on) {
                const bool e1 = E == 2 && e == 1;
                if (b == (e1 ? nb1 : nb0)) {
                    if (e1) copy8(lf1, s.h);
                    else copy8(nd, s.h);
                    e++;
                    b = 0;
                } else {
                    b++;
                }
            }
        } else if (lev && half == 1) {
            copy8(nd, s.h);
        }
    }
    TXW_PROBE(6);
    uint32_t a[8];
    copy8(a, s.h);
    int32_t stv = MH_OK;
    if (act && i == 0) {
        uint32_t x = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) x |= bswap(rd_le32(ap + 4 * q)) ^ a[q];
        stv = x ? MH_ERR_CORRUPTED_DATA : MH_OK;
        status[t] = stv;
        store_digest(eh_out + t * 32, nd);
        store_digest(alh_out + t * 32, a);
    }
    TXW_SYNC();  // msg is free: results staged there
    uint64_t *hst = reinterpret_cast<uint64_t *>(msg);  // R x 17 header words
    uint32_t *ast = msg + R * 34;                        // R x 8 Alh words (bytes as stored)
    uint32_t *sst = msg + R * 42;                        // R statuses
    if (act) {
        if (i == 0) {
#pragma unroll
            for (int q = 0; q < 8; q++) ast[r * 8 + q] = bswap(a[q]);
            sst[r] = (uint32_t)stv;
        }
        for (int q = i; q < 17; q += L) {
            uint64_t v;
            if (q < 3) v = rd_be64(rp + 8 * q);
            else if (q < 11) v = rd_raw64(rp + 24 + 8 * (q - 3));
            else if (q < 15) v = (uint64_t)EB[2 * (q - 11)] | ((uint64_t)EB[2 * (q - 11) + 1] << 32);
            else if (q == 15) v = (uint64_t)ver | ((uint64_t)nent << 32);
            else v = ver ? (uint64_t)ml | ((uint64_t)(uint32_t)(rec_g + 92) << 32) : 0;
            hst[r * 17 + q] = v;
        }
    }
    TXW_SYNC();
    TXW_PROBE(7);
}

constexpr int kTxWaves = 4;  // independent waves per workgroup

// per-wave LDS: [records sbytes][innerHash messages / results R x 384 B]
// [entry offsets 64 E words][Eh R x 32 B]
__host__ __device__ constexpr uint32_t txw_wave_bytes(uint32_t sbytes, int R, int E) {
    return sbytes + R * kTxMsgWords * 4 + 64 * E * 4 + R * 32;
}

template <int E, bool STAGED>
__global__ __launch_bounds__(256) void k_txlog_wave(
    uint64_t ntx, const uint8_t *__restrict__ buf, const uint64_t *__restrict__ rec_off,
    const uint64_t *__restrict__ alh_off, const uint64_t *__restrict__ leaf_off,
    MhTxHeader *__restrict__ hdrs, uint8_t *__restrict__ eh_out, uint8_t *__restrict__ alh_out,
    int32_t *__restrict__ status, TxlogHostOut ho, int lgl, uint32_t sbytes, uint64_t *probe,
    int fence) {
    extern __shared__ uint4 lds[];
    const int R = 64 >> lgl;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane >> lgl, i = lane & ((1 << lgl) - 1);
    const uint32_t wbytes = txw_wave_bytes(sbytes, R, E);
    uint8_t *wl = reinterpret_cast<uint8_t *>(lds) + wv * wbytes;
    uint32_t *msg = reinterpret_cast<uint32_t *>(wl + sbytes);
    uint32_t *eoff = msg + R * kTxMsgWords, *ehb = eoff + 64 * E;
    const uint64_t T0 = (uint64_t)blockIdx.x * kTxWaves * R;  // the workgroup's first record
    const uint64_t t0 = T0 + (uint64_t)wv * R;                 // the wave's
    const uint64_t pw = (uint64_t)blockIdx.x * kTxWaves + wv;
    if (t0 < ntx) {  // wave-uniform
        const uint64_t nmine = min((uint64_t)R, ntx - t0);
        const bool act = (uint64_t)r < nmine;
        const uint64_t t = act ? t0 + r : t0;
        const uint64_t w = act ? leaf_off[t + 1] - leaf_off[t] : 0;
        const uint64_t rec_g = rec_off[t];
        TXW_PROBE(0);
        if (probe && lane == 0) probe[pw * 16 + 10] = __builtin_amdgcn_s_memrealtime();
        if (STAGED) {
            // 1. the wave's records into LDS by LDS-DMA, every piece in flight
            // at once (+96 bytes: rd_le32 reads a dword ahead, skip12_block a
            // block's 80 bytes from its start unguarded)
            const uint64_t lo = rec_off[t0] & ~15ull, hi = alh_off[t0 + nmine - 1] + 32 + 96;
            const uint8_t *g = buf + lo;
            const uint32_t n16 = (uint32_t)((hi - lo + 15) >> 4);
            for (uint32_t k = 0; k < n16; k += 64) {
                const uint32_t c = min(k + lane, n16 - 1);  // the last lanes repeat the last piece
                __builtin_amdgcn_global_load_lds((tx_glb_void_t *)(g + 16 * (uint64_t)c),
                                                 (tx_lds_void_t *)(wl + 16 * k), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            TXW_PROBE(1);
            txlog_wave_body_loop<E, false>(wl + (rec_g - lo), wl + (alh_off[t] - lo), t, rec_g, w,
                                           act, lgl, r, i, eoff, msg, ehb, eh_out, alh_out, status,
                                           probe, pw);
        } else {
            txlog_wave_body_loop<E, true>(buf + rec_g, buf + alh_off[t], t, rec_g, w, act, lgl, r, i,
                                          eoff, msg, ehb, eh_out, alh_out, status, probe, pw);
        }
    }
    __syncthreads();  // every wave's results are staged in its msg slice
    // 5. the workgroup's records [T0, T0 + nb) out as contiguous runs
    const uint64_t nb = T0 < ntx ? min((uint64_t)kTxWaves * R, ntx - T0) : 0;
    const uint32_t *m0 = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(lds) + sbytes);
    const uint32_t wwords = wbytes / 4;
    const int lgr = 6 - lgl;
    // the device headers only when the caller's are not written here (they
    // are what a D2H copy takes to pageable outputs)
    uint64_t *hd = ho.hdrs ? ho.hdrs + T0 * 17 : reinterpret_cast<uint64_t *>(hdrs) + T0 * 17;
    if (ho.hdrs && ho.eh_only) {  // words 11-14 of each record's header (Eh); the host fills the rest
        for (uint32_t k = threadIdx.x; k < nb * 4; k += 256) {
            const uint32_t rec = k >> 2, j = 11 + (k & 3);
            hd[rec * 17 + j] = reinterpret_cast<const uint64_t *>(m0 + (rec >> lgr) * wwords)[(rec & (R - 1)) * 17 + j];
        }
    } else {
        for (uint32_t k = threadIdx.x; k < nb * 17; k += 256) {
            const uint32_t rec = k / 17, j = k - rec * 17;
            hd[k] = reinterpret_cast<const uint64_t *>(m0 + (rec >> lgr) * wwords)[(rec & (R - 1)) * 17 + j];
        }
    }
    if (ho.alh)
        for (uint32_t k = threadIdx.x; k < nb * 8; k += 256) {
            const uint32_t rec = k >> 3;
            ho.alh[T0 * 8 + k] = m0[(rec >> lgr) * wwords + R * 34 + (rec & (R - 1)) * 8 + (k & 7)];
        }
    if (ho.status)
        for (uint32_t k = threadIdx.x; k < nb; k += 256)
            ho.status[T0 + k] = m0[(k >> lgr) * wwords + R * 42 + (k & (R - 1))];
    if (t0 < ntx) TXW_PROBE(8);
    // (no system fence per wave: the caller reads the pinned results only
    // after synchronizing the stream, whose end-of-kernel release is
    // system-scope; a fence here held every wave until its PCIe writes
    // completed -- MH_TXLOG_FENCE=1 restores it for A/B)
    if (fence && (ho.status || ho.alh || ho.hdrs)) __threadfence_system();
    if (t0 < ntx) {
        TXW_PROBE(9);
        if (probe && lane == 0) probe[pw * 16 + 11] = __builtin_amdgcn_s_memrealtime();
    }
}

// ---- MH_TXLOG_PROBE=1 (diagnosis): one stamp buffer per launch of a call,
// reported after the call's final sync
namespace {
struct TxwProbe {
    std::vector<std::pair<uint64_t *, unsigned>> bufs;  // (device stamps, waves)
    size_t used = 0;
    std::mutex mu;  // contexts validating concurrently share the slots
};
TxwProbe &txw_probe() {
    static TxwProbe p;
    return p;
}
bool txw_probe_on() {
    static const bool on = getenv("MH_TXLOG_PROBE") != nullptr;
    return on;
}
}  // namespace

static uint64_t *txlog_probe_slot(unsigned waves) {
    if (!txw_probe_on()) return nullptr;
    TxwProbe &p = txw_probe();
    std::lock_guard<std::mutex> lk(p.mu);
    if (p.used == p.bufs.size()) p.bufs.push_back({nullptr, 0});
    auto &b = p.bufs[p.used++];
    if (b.second < waves) {
        if (b.first) (void)hipFree(b.first);
        b.first = nullptr;
        b.second = 0;
        if (hipMalloc(&b.first, (size_t)waves * 16 * 8) != hipSuccess) return nullptr;
        b.second = waves;
    }
    (void)hipMemset(b.first, 0, (size_t)b.second * 16 * 8);  // stale stamps past this launch too
    return b.first;
}

// per launch of the last call: waves, and the median / max over waves of each
// phase's shader cycles (stamp k+1 - stamp k), plus the spread of wave starts
// and ends from the launch's first start
void txlog_probe_report() {
    if (!txw_probe_on()) return;
    TxwProbe &p = txw_probe();
    std::lock_guard<std::mutex> lk(p.mu);
    for (size_t l = 0; l < p.used; l++) {
        const unsigned n = p.bufs[l].second;
        std::vector<uint64_t> h((size_t)n * 16);
        if (hipMemcpy(h.data(), p.bufs[l].first, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) break;
        unsigned nw = 0;
        while (nw < n && h[(size_t)nw * 16]) nw++;
        if (!nw) continue;
        (void)nw;
        uint64_t t0 = ~0ull;
        for (unsigned w = 0; w < nw; w++) t0 = std::min(t0, h[(size_t)w * 16]);
        fprintf(stderr, "txlog_probe launch %zu waves %u:", l, nw);
        for (int k = 0; k < 9; k++) {
            std::vector<uint64_t> d;
            for (unsigned w = 0; w < nw; w++) {
                const uint64_t a = h[(size_t)w * 16 + k], b = h[(size_t)w * 16 + k + 1];
                if (a && b >= a) d.push_back(b - a);
            }
            if (d.empty()) continue;
            std::sort(d.begin(), d.end());
            fprintf(stderr, " p%d-%d=%llu/%llu", k, k + 1, (unsigned long long)d[d.size() / 2],
                    (unsigned long long)d.back());
        }
        std::vector<uint64_t> st, en;
        for (unsigned w = 0; w < nw; w++) {
            st.push_back(h[(size_t)w * 16] - t0);
            en.push_back(h[(size_t)w * 16 + 9] - t0);
        }
        std::sort(st.begin(), st.end());
        std::sort(en.begin(), en.end());
        // shader clock of the waves: s_memtime cycles / s_memrealtime (100 MHz) ticks
        std::vector<double> ghz, life;
        uint64_t r0 = ~0ull, r1 = 0;
        for (unsigned w = 0; w < nw; w++) {
            const uint64_t c0 = h[(size_t)w * 16], c1 = h[(size_t)w * 16 + 9];
            const uint64_t q0 = h[(size_t)w * 16 + 10], q1 = h[(size_t)w * 16 + 11];
            if (q1 > q0 && c1 > c0) {
                ghz.push_back((double)(c1 - c0) / (double)(q1 - q0) / 10.0);
                life.push_back((double)(q1 - q0) / 100.0);
            }
            if (q0) r0 = std::min(r0, q0);
            r1 = std::max(r1, q1);
        }
        std::sort(ghz.begin(), ghz.end());
        std::sort(life.begin(), life.end());
        for (int k = 12; k < 16; k++) {  // k_txlog_lanes: loop cycles by iteration kind (+1)
            std::vector<uint64_t> d;
            for (unsigned w = 0; w < nw; w++)
                if (h[(size_t)w * 16 + k]) d.push_back(h[(size_t)w * 16 + k] - 1);
            if (d.empty()) continue;
            std::sort(d.begin(), d.end());
            fprintf(stderr, " it%d=%llu/%llu", k - 12, (unsigned long long)d[d.size() / 2],
                    (unsigned long long)d.back());
        }
        fprintf(stderr, " clock_ghz med %.2f wave_life_us med/max %.1f/%.1f launch_span_us %.1f\n",
                ghz.empty() ? 0.0 : ghz[ghz.size() / 2], life.empty() ? 0.0 : life[life.size() / 2],
                life.empty() ? 0.0 : life.back(), r1 > r0 ? (double)(r1 - r0) / 100.0 : 0.0);
        (void)st;
    }
    p.used = 0;
}

hipError_t launch_txlog_wave(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                             const uint64_t *rec_off, const uint64_t *alh_off,
                             const uint64_t *leaf_off, MhTxHeader *hdrs, uint8_t *eh_out,
                             uint8_t *alh_out, int32_t *status, const TxlogHostOut &ho,
                             uint64_t wmax, const uint64_t *h_rec_off, const uint64_t *h_alh_off) {
    if (!ntx) return hipSuccess;
    if (wmax > 64 || ((uintptr_t)ho.hdrs & 7) || ((uintptr_t)ho.alh & 3) || ((uintptr_t)ho.status & 3))
        return hipErrorInvalidValue;
    static const int e2 = [] {
        const char *e = getenv("MH_TXLOG_E");
        return e && atoi(e) == 1 ? 0 : 1;
    }();
    const int E = e2 ? 2 : 1;
    int lgp = 0;
    while ((1ull << lgp) < wmax) lgp++;
    const int lgl = std::max(2, lgp - (E == 2 ? 1 : 0));  // >= 4 lanes per record: <= 16 records a wave
    const int R = 64 >> lgl;
    // the widest wave's records (+ alignment and over-read pad) decide whether
    // the waves stage their records in LDS
    uint64_t span = 0;
    for (uint64_t t0 = 0; t0 < ntx; t0 += R) {
        const uint64_t tl = std::min<uint64_t>(ntx, t0 + R) - 1;
        span = std::max<uint64_t>(span, h_alh_off[tl] + 32 + 96 - (h_rec_off[t0] & ~15ull));
    }
    // whole 1 KiB pieces: the LDS-DMA's last pass writes all 64 lanes' slots
    const uint64_t sb = (span + 1023) & ~1023ull;
    // MH_TXLOG_STAGE_MAX (bytes, read per call: tests force the HBM path with 0);
    // four waves' slices must fit the CU's 160 KB
    const char *sm = getenv("MH_TXLOG_STAGE_MAX");
    const uint64_t smax = sm ? strtoull(sm, nullptr, 10) : (32u << 10);
    const bool staged = sb <= std::min<uint64_t>(smax, 32u << 10);
    const uint32_t sbytes = staged ? (uint32_t)sb : 0;
    const size_t sh = (size_t)kTxWaves * txw_wave_bytes(sbytes, R, E);
    TimerScope ts(tm, "txlog_wave", st);
    const dim3 grid((unsigned)((ntx + (uint64_t)kTxWaves * R - 1) / ((uint64_t)kTxWaves * R))), blk(256);
    uint64_t *probe = txlog_probe_slot(grid.x * kTxWaves);
    static const int fence = [] {
        const char *e = getenv("MH_TXLOG_FENCE");
        return e && atoi(e) ? 1 : 0;
    }();
    // up to 160 KB of dynamic LDS (once per instantiation)
    static const bool attr = [] {
        const int mx = 160 << 10;
        hipFuncSetAttribute((const void *)k_txlog_wave<2, true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        hipFuncSetAttribute((const void *)k_txlog_wave<2, false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        hipFuncSetAttribute((const void *)k_txlog_wave<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        hipFuncSetAttribute((const void *)k_txlog_wave<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
#define MH_TXW(e_, s_)                                                                             \
    hipLaunchKernelGGL((k_txlog_wave<e_, s_>), grid, blk, sh, st, ntx, buf, rec_off, alh_off,    \
                       leaf_off, hdrs, eh_out, alh_out, status, ho, lgl, sbytes, probe, fence)
    if (E == 2) {
        if (staged) MH_TXW(2, true); else MH_TXW(2, false);
    } else {
        if (staged) MH_TXW(1, true); else MH_TXW(1, false);
    }
#undef MH_TXW
    return hipGetLastError();
}

// ---------------------------------------------------------------- a14, workgroup phases
// The same a14 check of a group (tx.go:533-630 per record) with the work of
// every phase spread over the WHOLE workgroup, so that a compression slot
// never idles lanes of a busy wave (k_txlog_wave: R = 64 / L records per wave,
// its tree levels and the innerHash + Alh of lane 0 per record leave half of
// the wave's lanes idle -- VALU active 0.51, profiles/pmc_txlog_wave_r04.txt).
// A 256-thread workgroup takes RPW = min(128, 512 / P) consecutive records
// (P = the widest tx rounded up to a power of two >= 2):
//   0. the records are copied into LDS by LDS-DMA (every wave a quarter of the
//      16-byte pieces, one round trip); record r's thread parses its header
//      (tx.go:419-518) and walks its entries (tx.go:578-585) into an offset
//      table;
//   1. thread k hashes entry slots 2k and 2k+1 (record 2k / P: the entry
//      digest tx.go:690-731 in place from the staged record, then the leaf
//      htree.go:79-83) and their level-1 node (or promotes the lone left leaf),
//      so every thread is busy and level 1 needs no barrier;
//   2. levels 2 .. log2 P: node j of record r on thread r * (P >> l) + j, both
//      children from LDS (htree.go:85-110), a barrier per level -- the idle
//      threads of a level are whole waves, which issue nothing while the
//      other workgroups' waves on the SIMD run;
//   3. thread r hashes record r's innerHash (tx.go:249-302, its message built
//      from the staged header bytes and Eh) and Alh (tx.go:307-319) and
//      compares it with the stored one (tx.go:623-627);
//   4. the results are staged in LDS and stored by the whole workgroup as
//      contiguous runs (as k_txlog_wave).
// Every hash goes through the one compression site of one loop over the
// workgroup-uniform slot sequence (entries | levels 2.. | innerHash + Alh);
// the phase boundaries are the barriers.
__host__ __device__ constexpr uint32_t txb_res_bytes(int rpw) { return (uint32_t)rpw * 172; }
struct TxbLds {
    uint32_t stage, a, b, eoff, info, red, total;
};
__host__ __device__ inline TxbLds txb_lds(uint32_t sbytes, int lgp, int rpw) {
    TxbLds o{};
    const uint32_t P = 1u << lgp;
    o.stage = 0;
    uint32_t x = sbytes > txb_res_bytes(rpw) ? sbytes : txb_res_bytes(rpw);  // results alias the stage
    o.a = x;
    x += (uint32_t)rpw * (P / 2) * 36;
    o.b = x;
    x += (uint32_t)rpw * (P / 4 ? P / 4 : 1) * 36;
    o.eoff = x;
    x += (uint32_t)rpw * P * 4;
    o.info = x;
    x += (uint32_t)rpw * 16;
    o.red = x;
    x += 16;
    o.total = (x + 15) & ~15u;
    return o;
}

// workgroup max of a per-thread value (red: 4 LDS words; includes barriers)
__device__ __forceinline__ uint32_t txb_wg_max(uint32_t v, uint32_t *red) {
    v = wave_max_u32(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const uint32_t m = max(max(red[0], red[1]), max(red[2], red[3]));
    __syncthreads();
    return m;
}

template <bool STAGED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_txlog_blk(
    uint64_t ntx, const uint8_t *__restrict__ buf, const uint64_t *__restrict__ rec_off,
    const uint64_t *__restrict__ alh_off, const uint64_t *__restrict__ leaf_off,
    MhTxHeader *__restrict__ hdrs, uint8_t *__restrict__ eh_out, uint8_t *__restrict__ alh_out,
    int32_t *__restrict__ status, TxlogHostOut ho, int lgp, int rpw, uint32_t sbytes, int fence,
    uint64_t *probe) {
    extern __shared__ uint4 lds[];
    uint8_t *sm = reinterpret_cast<uint8_t *>(lds);
    const TxbLds Lo = txb_lds(sbytes, lgp, rpw);
    uint32_t(*NA)[9] = reinterpret_cast<uint32_t(*)[9]>(sm + Lo.a);
    uint32_t(*NB)[9] = reinterpret_cast<uint32_t(*)[9]>(sm + Lo.b);
    uint32_t *eoff = reinterpret_cast<uint32_t *>(sm + Lo.eoff);
    uint32_t *info = reinterpret_cast<uint32_t *>(sm + Lo.info);
    uint32_t *red = reinterpret_cast<uint32_t *>(sm + Lo.red);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int P = 1 << lgp;
    const uint64_t T0 = (uint64_t)blockIdx.x * rpw;
    const uint64_t nrec = min((uint64_t)rpw, ntx - T0);  // the grid covers ntx: >= 1
    const uint64_t lo = STAGED ? rec_off[T0] & ~15ull : 0;
    // MH_TXLOG_PROBE=1: s_memtime stamps of the workgroup's phases (thread 0)
#define TXB_PROBE(k_)                                                                             \
    do {                                                                                          \
        if (probe && tid == 0) probe[(uint64_t)blockIdx.x * 16 + (k_)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
    TXB_PROBE(0);
    if (probe && tid == 0) probe[(uint64_t)blockIdx.x * 16 + 10] = __builtin_amdgcn_s_memrealtime();
    // record r's bytes (LDS when staged, else the log in HBM)
    auto rec_ptr = [&](uint64_t r) -> const uint8_t * {
        return STAGED ? sm + (rec_off[T0 + r] - lo) : buf + rec_off[T0 + r];
    };
    if (STAGED) {
        // 0. the workgroup's records (contiguous in the log, each ending with
        // its stored Alh) into LDS by LDS-DMA: wave wv moves pieces 64 wv +
        // 256 k; +96 bytes past the last Alh (rd_le32 reads a dword ahead,
        // skip12_block a block's 80 bytes unguarded), inside the device buffer
        const uint64_t hi = alh_off[T0 + nrec - 1] + 32 + 96;
        const uint8_t *g = buf + lo;
        const uint32_t n16 = (uint32_t)((hi - lo + 15) >> 4);
        for (uint32_t k = 64 * wv; k < n16; k += 256) {
            const uint32_t c = min(k + lane, n16 - 1);  // the last lanes repeat the last piece
            __builtin_amdgcn_global_load_lds((tx_glb_void_t *)(g + 16 * (uint64_t)c),
                                             (tx_lds_void_t *)(sm + 16 * k), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    TXB_PROBE(1);
    // header + entry walk of record tid (tx.go:419-518, 578-585; lengths
    // validated by the host hop)
    uint32_t nbi = 0;
    if ((uint64_t)tid < nrec) {
        const uint8_t *rp = rec_ptr(tid);
        const uint32_t ver = rd_be16(rp + 88);
        uint32_t ml = 0, nent, q = 92;
        if (ver == 0) {
            nent = rd_be16(rp + 90);
        } else {
            ml = rd_be16(rp + 90);
            nent = bswap(rd_le32(rp + 92 + ml));
            q = 96 + ml;
        }
        info[tid * 4 + 0] = ver;
        info[tid * 4 + 1] = ml;
        info[tid * 4 + 2] = nent;
        const uint64_t w = leaf_off[T0 + tid + 1] - leaf_off[T0 + tid];
        info[tid * 4 + 3] = (uint32_t)w;
        for (uint64_t j = 0; j < w; j++) {
            eoff[tid * P + j] = q;
            const uint32_t m = rd_be16(rp + q);
            const uint32_t k = rd_be16(rp + q + 2 + m);
            q += 48 + m + k;
        }
        const uint32_t mlen = 80 + (ver ? 8 + ml : 4);  // innerHash message bytes
        nbi = (mlen + 8) / 64 + 1;
    }
    __syncthreads();
    TXB_PROBE(2);
    // 1. this thread's two entry slots and their level-1 node
    const uint32_t s0 = 2u * tid;
    const uint64_t r1 = s0 >> lgp;
    const bool act1 = r1 < nrec && s0 < (uint32_t)rpw * P;
    const uint32_t j0 = s0 & (P - 1);
    uint32_t w1 = 0, ver1 = 0;
    const uint8_t *rp1 = nullptr;
    if (act1) {
        w1 = info[r1 * 4 + 3];
        ver1 = info[r1 * 4 + 0];
        rp1 = rec_ptr(r1);
    }
    const uint32_t ne = act1 ? (uint32_t)min(2u, w1 > j0 ? w1 - j0 : 0u) : 0u;  // entries of this thread
    const uint8_t *mp[2] = {rp1, rp1};
    uint32_t la[2] = {0, 0}, nb[2] = {0, 0};
#pragma unroll
    for (int e = 0; e < 2; e++) {
        if ((uint32_t)e < ne) {
            const uint8_t *er = rp1 + eoff[r1 * P + j0 + e];
            const uint32_t m = rd_be16(er), k = rd_be16(er + 2 + m);
            mp[e] = ver1 == 1 ? er : er + 4 + m;  // tx.go:690-731
            la[e] = ver1 == 1 ? 4 + m + k : k;
            nb[e] = (la[e] + 32 + 8) / 64 + 1;
        }
    }
    const uint32_t steps = (ne > 0 ? nb[0] + 1 : 0) + (ne > 1 ? nb[1] + 1 + 2 : 0);
    const uint32_t nE = txb_wg_max(steps, red);
    const uint32_t nH = txb_wg_max(nbi ? nbi + 2 : 0, red);
    const uint32_t nT = 2u * (uint32_t)(lgp - 1);
    TXB_PROBE(3);
    // 2./3. the slot loop
    State s;
    s.init();
    // lf0 / lf1: the leaves, then a node's children; lf0 the innerHash in H
    uint32_t lf0[8], lf1[8];
#pragma unroll
    for (int q = 0; q < 8; q++) lf0[q] = lf1[q] = 0;
    uint32_t e = 0, b = 0;
    bool tnode = false, tprom = false;  // this thread's node at the current level: hash / promote
    uint32_t tdst = 0;
    const uint32_t rH = tid;            // record of the H phase
    const bool actH = (uint64_t)tid < nrec;
    const uint8_t *rpH = actH ? rec_ptr(rH) : nullptr;
    uint32_t blenH = 0, mlenH = 0, nbiH = nbi;
    // record rH's root (Eh) stays in LDS: the final level's buffer, slot rH
    uint32_t(*fin)[9] = (lgp & 1) ? NA : NB;
#pragma unroll 1
    for (uint32_t g = 0; g < nE + nT + nH; g++) {
        uint32_t wv16[16];
        bool on = false, tail = false;
        uint32_t tail_r7 = 0;
        if (g == nE) TXB_PROBE(4);
        if (g == nE + nT) TXB_PROBE(5);
        if (g < nE) {
            // entry e's digest blocks, its leaf, then (two entries) the node
            if (e < ne) {
                on = true;
                if (b < nb[e]) {
                    if (b == 0) s.init();
                    skip12_block<!STAGED>(mp[e], la[e], b, nb[e], wv16);
                } else {
                    wv16[0] = s.h[0] >> 8;
#pragma unroll
                    for (int j = 1; j < 8; j++) wv16[j] = __builtin_amdgcn_alignbit(s.h[j - 1], s.h[j], 8);
                    wv16[8] = (s.h[7] << 24) | 0x00800000u;
#pragma unroll
                    for (int j = 9; j < 15; j++) wv16[j] = 0;
                    wv16[15] = 33u * 8u;
                    s.init();
                }
            } else if (ne == 2 && e == 2) {
                on = true;
                if (b == 0) {  // SHA256(0x01 || leaf0 || leaf1), first block
                    s.init();
                    wv16[0] = 0x01000000u | (lf0[0] >> 8);
#pragma unroll
                    for (int j = 1; j < 8; j++) wv16[j] = __builtin_amdgcn_alignbit(lf0[j - 1], lf0[j], 8);
                    wv16[8] = __builtin_amdgcn_alignbit(lf0[7], lf1[0], 8);
#pragma unroll
                    for (int j = 1; j < 8; j++) wv16[8 + j] = __builtin_amdgcn_alignbit(lf1[j - 1], lf1[j], 8);
                } else {
                    tail = true;
                    tail_r7 = lf1[7];
                }
            }
        } else if (g < nE + nT) {
            const uint32_t k = g - nE, l = 2 + (k >> 1), half = k & 1;
            if (half == 0) {
                __syncthreads();  // level l - 1 is written
                const uint32_t S = (uint32_t)P >> l;  // node slots per record at level l
                const uint64_t r = tid / S;           // (S >= 1: l <= lgp)
                const uint32_t j = tid - (uint32_t)r * S;
                tnode = tprom = false;
                if (tid < rpw * S && r < nrec) {
                    const uint32_t w = info[r * 4 + 3];
                    const uint32_t wp = (w + (1u << (l - 1)) - 1) >> (l - 1);  // width at level l-1
                    const uint32_t a = (uint32_t)r * 2 * S + 2 * j;
                    uint32_t(*src)[9] = (l & 1) ? NB : NA;  // level l-1: odd levels in A
                    if (2 * j + 1 < wp) {
                        tnode = true;
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            lf0[q] = src[a][q];
                            lf1[q] = src[a + 1][q];
                        }
                    } else if (2 * j < wp) {
                        tprom = true;
#pragma unroll
                        for (int q = 0; q < 8; q++) lf0[q] = src[a][q];
                    }
                    tdst = tid;
                }
                if (tnode) {
                    on = true;
                    s.init();
                    wv16[0] = 0x01000000u | (lf0[0] >> 8);
#pragma unroll
                    for (int j2 = 1; j2 < 8; j2++) wv16[j2] = __builtin_amdgcn_alignbit(lf0[j2 - 1], lf0[j2], 8);
                    wv16[8] = __builtin_amdgcn_alignbit(lf0[7], lf1[0], 8);
#pragma unroll
                    for (int j2 = 1; j2 < 8; j2++) wv16[8 + j2] = __builtin_amdgcn_alignbit(lf1[j2 - 1], lf1[j2], 8);
                }
            } else if (tnode) {
                on = true;
                tail = true;
                tail_r7 = lf1[7];
            }
        } else {
            const uint32_t k = g - nE - nT;
            if (k == 0) {
                __syncthreads();  // every tree is reduced
                if (actH) {
                    if (info[rH * 4 + 3] == 0) {  // no entries: SHA256(nil), htree.go:73-77
                        uint32_t d[8];  // (slot rH of no other record: no reader but this thread)
                        load_digest(kEmptyRootDev, d);
#pragma unroll
                        for (int q = 0; q < 8; q++) fin[rH][q] = d[q];
                    }
                    const uint32_t ver = info[rH * 4 + 0];
                    blenH = ver ? 8 + info[rH * 4 + 1] : 4;
                    mlenH = 80 + blenH;
                }
            }
            if (actH && k < nbiH + 2) {
                on = true;
                if (k < nbiH) {  // innerHash block k: ts || version || md part || Eh || blTxID || blRoot
                    if (k == 0) s.init();
#pragma unroll 4
                    for (int jw = 0; jw < 16; jw++) {
                        const uint32_t kk0 = 64 * k + 4 * jw;
                        uint32_t v32 = 0;
                        if (jw == 15 && k + 1 == nbiH) {  // the bit length (< 2^32)
                            v32 = mlenH * 8;
                        } else {
#pragma unroll
                            for (int bb = 0; bb < 4; bb++) {
                                const uint32_t kk = kk0 + bb;
                                uint32_t v;
                                if (kk < 8) v = rpH[8 + kk];
                                else if (kk < 8 + blenH) v = rpH[80 + kk];
                                else if (kk < 40 + blenH) {
                                    const uint32_t o = kk - 8 - blenH;
                                    v = (fin[rH][o >> 2] >> (24 - 8 * (o & 3))) & 0xffu;
                                } else if (kk < mlenH) v = rpH[kk - 24 - blenH];
                                else v = kk == mlenH ? 0x80u : 0u;
                                v32 = v32 << 8 | v;
                            }
                        }
                        wv16[jw] = v32;
                    }
                } else if (k == nbiH) {  // BE64 id || prevAlh || innerHash[0:24]
                    copy8(lf0, s.h);  // the innerHash
                    s.init();
                    const uint64_t id = rd_be64(rpH);
                    wv16[0] = (uint32_t)(id >> 32);
                    wv16[1] = (uint32_t)id;
#pragma unroll
                    for (int q = 0; q < 8; q++) wv16[2 + q] = bswap(rd_le32(rpH + 56 + 4 * q));
#pragma unroll
                    for (int q = 0; q < 6; q++) wv16[10 + q] = lf0[q];
                } else {
                    wv16[0] = lf0[6];
                    wv16[1] = lf0[7];
                    wv16[2] = 0x80000000u;
#pragma unroll
                    for (int q = 3; q < 15; q++) wv16[q] = 0;
                    wv16[15] = 72u * 8u;
                }
            }
        }
        if (on) {
            if (tail)
                compress_node_tail_g(s, tail_r7);
            else
                compress(s, wv16);
        }
        // bookkeeping after the block
        if (g < nE) {
            if (on) {
                if (e < ne) {
                    if (b == nb[e]) {  // the leaf is done
                        if (e == 0) copy8(lf0, s.h);
                        else copy8(lf1, s.h);
                        e++;
                        b = 0;
                        if (e == ne && ne == 1 && act1) {  // a lone left leaf: promoted to level 1
#pragma unroll
                            for (int q = 0; q < 8; q++) NA[tid][q] = lf0[q];
                        }
                    } else {
                        b++;
                    }
                } else {  // the level-1 node
                    if (b == 1) {
#pragma unroll
                        for (int q = 0; q < 8; q++) NA[tid][q] = s.h[q];
                        e++;
                    }
                    b++;
                }
            }
        } else if (g < nE + nT) {
            const uint32_t k = g - nE, l = 2 + (k >> 1), half = k & 1;
            if (half == 1 && (tnode || tprom)) {
                uint32_t(*dst)[9] = (l & 1) ? NA : NB;  // level l: odd levels in A
#pragma unroll
                for (int q = 0; q < 8; q++) dst[tdst][q] = tnode ? s.h[q] : lf0[q];
            }
        }
    }
    TXB_PROBE(6);
    // compare + results (tx.go:623-627)
    int32_t stv = MH_OK;
    uint32_t a[8];
    copy8(a, s.h);
    const uint64_t t = T0 + tid;
    uint32_t eh[8];
    if (actH) {
#pragma unroll
        for (int q = 0; q < 8; q++) eh[q] = fin[rH][q];
        const uint8_t *ap = STAGED ? sm + (alh_off[t] - lo) : buf + alh_off[t];
        uint32_t xx = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) xx |= bswap(rd_le32(ap + 4 * q)) ^ a[q];
        stv = xx ? MH_ERR_CORRUPTED_DATA : MH_OK;
        status[t] = stv;
        store_digest(eh_out + t * 32, eh);
        store_digest(alh_out + t * 32, a);
    }
    // header words of record tid (before the stage is overwritten)
    uint64_t hw[17];
    if (actH) {
        const uint32_t ver = info[rH * 4 + 0], ml = info[rH * 4 + 1], nent = info[rH * 4 + 2];
#pragma unroll
        for (int q = 0; q < 3; q++) hw[q] = rd_be64(rpH + 8 * q);
#pragma unroll
        for (int q = 0; q < 8; q++) hw[3 + q] = rd_raw64(rpH + 24 + 8 * q);
#pragma unroll
        for (int q = 0; q < 4; q++)
            hw[11 + q] = (uint64_t)bswap(eh[2 * q]) | ((uint64_t)bswap(eh[2 * q + 1]) << 32);
        hw[15] = (uint64_t)ver | ((uint64_t)nent << 32);
        hw[16] = ver ? (uint64_t)ml | ((uint64_t)(uint32_t)(rec_off[t] + 92) << 32) : 0;
    }
    __syncthreads();  // the stage is free: results staged there
    uint64_t *hst = reinterpret_cast<uint64_t *>(sm);     // rpw x 17 header words
    uint32_t *ast = reinterpret_cast<uint32_t *>(sm + (uint32_t)rpw * 136);  // rpw x 8 Alh words
    uint32_t *sst = ast + rpw * 8;                         // rpw statuses
    if (actH) {
#pragma unroll
        for (int q = 0; q < 17; q++) hst[tid * 17 + q] = hw[q];
#pragma unroll
        for (int q = 0; q < 8; q++) ast[tid * 8 + q] = bswap(a[q]);
        sst[tid] = (uint32_t)stv;
    }
    __syncthreads();
    TXB_PROBE(7);
    uint64_t *hd = ho.hdrs ? ho.hdrs + T0 * 17 : reinterpret_cast<uint64_t *>(hdrs) + T0 * 17;
    if (ho.hdrs && ho.eh_only) {
        for (uint32_t k = tid; k < nrec * 4; k += 256) {
            const uint32_t rec = k >> 2, j = 11 + (k & 3);
            hd[rec * 17 + j] = hst[rec * 17 + j];
        }
    } else {
        for (uint32_t k = tid; k < nrec * 17; k += 256) hd[k] = hst[k];
    }
    if (ho.alh)
        for (uint32_t k = tid; k < nrec * 8; k += 256) ho.alh[T0 * 8 + k] = ast[k];
    if (ho.status)
        for (uint32_t k = tid; k < nrec; k += 256) ho.status[T0 + k] = sst[k];
    if (fence && (ho.status || ho.alh || ho.hdrs)) __threadfence_system();
    TXB_PROBE(8);
    TXB_PROBE(9);
    if (probe && tid == 0) probe[(uint64_t)blockIdx.x * 16 + 11] = __builtin_amdgcn_s_memrealtime();
#undef TXB_PROBE
}

hipError_t launch_txlog_blk(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                            const uint64_t *rec_off, const uint64_t *alh_off,
                            const uint64_t *leaf_off, MhTxHeader *hdrs, uint8_t *eh_out,
                            uint8_t *alh_out, int32_t *status, const TxlogHostOut &ho,
                            uint64_t wmax, const uint64_t *h_rec_off, const uint64_t *h_alh_off) {
    if (!ntx) return hipSuccess;
    if (wmax > 64 || ((uintptr_t)ho.hdrs & 7) || ((uintptr_t)ho.alh & 3) || ((uintptr_t)ho.status & 3))
        return hipErrorInvalidValue;
    int lgp = 1;
    while ((1ull << lgp) < wmax) lgp++;
    const int rpw = std::min(128, 512 >> lgp);
    // the widest workgroup's records (+ alignment and over-read pad), in the
    // LDS-DMA's whole passes of 64 pieces
    uint64_t span = 0;
    for (uint64_t t0 = 0; t0 < ntx; t0 += rpw) {
        const uint64_t tl = std::min<uint64_t>(ntx, t0 + rpw) - 1;
        span = std::max<uint64_t>(span, h_alh_off[tl] + 32 + 96 - (h_rec_off[t0] & ~15ull));
    }
    const uint64_t sb = (span + 1023) & ~1023ull;
    // staged when the workgroup's LDS leaves room for two per CU (MH_TXLOG_STAGE_MAX
    // bytes, read per call: tests force the HBM path with 0)
    const char *sm = getenv("MH_TXLOG_STAGE_MAX");
    const uint64_t smax = sm ? strtoull(sm, nullptr, 10) : (64u << 10);
    const bool staged = sb <= smax && txb_lds((uint32_t)std::min<uint64_t>(sb, 1u << 20), lgp, rpw).total <= (80u << 10);
    const uint32_t sbytes = staged ? (uint32_t)sb : 0;
    const size_t sh = txb_lds(sbytes, lgp, rpw).total;
    static const int fence = [] {
        const char *e = getenv("MH_TXLOG_FENCE");
        return e && atoi(e) ? 1 : 0;
    }();
    static const bool attr = [] {
        const int mx = 160 << 10;
        hipFuncSetAttribute((const void *)k_txlog_blk<true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        hipFuncSetAttribute((const void *)k_txlog_blk<false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    TimerScope ts(tm, "txlog_blk", st);
    const dim3 grid((unsigned)((ntx + rpw - 1) / rpw)), blk(256);
    uint64_t *probe = txlog_probe_slot(grid.x);
    if (staged)
        hipLaunchKernelGGL(k_txlog_blk<true>, grid, blk, sh, st, ntx, buf, rec_off, alh_off, leaf_off,
                           hdrs, eh_out, alh_out, status, ho, lgp, rpw, sbytes, fence, probe);
    else
        hipLaunchKernelGGL(k_txlog_blk<false>, grid, blk, sh, st, ntx, buf, rec_off, alh_off, leaf_off,
                           hdrs, eh_out, alh_out, status, ho, lgp, rpw, sbytes, fence, probe);
    return hipGetLastError();
}

// ---------------------------------------------------------------- a14, lanes per record
// The same a14 check with every record on L = 1, 2, 4, 8 or 16 lanes (k_txlog_lanes<LGL>):
// lane i of a record takes its entries [i EP, (i+1) EP) (EP = P / L, P = the
// widest tx rounded up to a power of two) and builds their subtree itself --
// entry digest (tx.go:690-731) and leaf (htree.go:79-83) per entry, pushed on
// a per-lane stack in LDS; after the c-th leaf, tz(c) merges
// SHA256(0x01 || left || right), and at the end the stack folded from the
// right, which is htree's pairing with the odd last node promoted
// (htree.go:85-110): an aligned block of 2^k leaves of a tree is the htree of
// its leaves (SURVEY.md finding 3).  The L lane roots of a record are then
// paired log2 L more levels, and the record's first lane hashes innerHash
// (tx.go:249-302) and Alh (tx.go:307-319) and compares.  No staging, no
// workgroup barrier before the final stores: a lane is busy on its own record
// for all but the log2 L combine levels and the four innerHash + Alh
// compressions, so with L = 1 every lane of a wave works in every compression
// slot (uniform records).  Against k_txlog_wave (one wave per 64 / L' records,
// L' = P / 2 lanes per record: its tree levels and the innerHash + Alh leave
// half of the wave's lanes idle, VALU active 0.51) the lanes stay busy; the
// price is latency: a record is ~66 dependent compressions on L = 1 lane, so
// the launch picks L from the record count (few records: more lanes).
constexpr int kTxlStackPad = 9;  // words per stack slot (8 + 1: bank spread)

__device__ __forceinline__ void txl_node_first(const uint32_t l[8], const uint32_t r[8], uint32_t w[16]) {
    w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(l[j - 1], l[j], 8);
    w[8] = __builtin_amdgcn_alignbit(l[7], r[0], 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[8 + j] = __builtin_amdgcn_alignbit(r[j - 1], r[j], 8);
}

__device__ unsigned g_txl_viol = 0;  // MH_TXLOG_LANES_CHECK: reported violations

template <int LGL, bool CHK>
__global__ __launch_bounds__(256) void k_txlog_lanes(
    uint64_t ntx, const uint8_t *__restrict__ buf, const uint64_t *__restrict__ rec_off,
    const uint64_t *__restrict__ alh_off, const uint64_t *__restrict__ leaf_off,
    MhTxHeader *__restrict__ hdrs, uint8_t *__restrict__ eh_out, uint8_t *__restrict__ alh_out,
    int32_t *__restrict__ status, TxlogHostOut ho, int lgp, int dep, int fence, uint64_t blen_,
    uint64_t *__restrict__ probe) {
    extern __shared__ uint4 lds[];
    constexpr int L = 1 << LGL, R = 64 >> LGL;
    uint32_t *stk = reinterpret_cast<uint32_t *>(lds);  // [dep][256][9]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r = lane >> LGL, i = lane & (L - 1);
    const int EP = (1 << lgp) >> LGL;  // entries per lane (>= 1)
    const uint64_t TW = ((uint64_t)blockIdx.x * 4 + wv) * R;  // the wave's first record
    const uint64_t T0 = (uint64_t)blockIdx.x * 4 * R;        // the workgroup's
    const uint64_t t = TW + r;
    const bool act = t < ntx;
    auto slot = [&](int d) -> uint32_t * { return stk + ((uint32_t)d * 256 + tid) * kTxlStackPad; };
    // MH_TXLOG_PROBE=1: s_memtime stamps of the wave's phases (lane 0; 0 start,
    // 1 loop start, 2 loop end, 3 lanes combined, 4 innerHash message built, 5
    // Alh done, 6 results staged, 9 end; 10 / 11 s_memrealtime) and the cycles
    // of the loop's iterations by kind (12 digest blocks, 13 leaves, 14 node
    // first blocks, 15 node tails)
    const uint64_t pw = (uint64_t)blockIdx.x * 4 + wv;
    auto stamp = [&](int k) {
        if (probe && lane == 0) probe[pw * 16 + k] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);
    if (probe && lane == 0) probe[pw * 16 + 10] = __builtin_amdgcn_s_memrealtime();
    uint64_t acc[4] = {0, 0, 0, 0};
    // CHK (MH_TXLOG_LANES_CHECK=1, diagnosis): every read range of the log
    // checked against [buf, buf + len + 256); a range outside is reported and
    // read from buf instead
    auto ok_ = [&](const uint8_t *p, uint32_t n, int tag) -> const uint8_t * {
        if (!CHK) return p;
        const int64_t o = (int64_t)(p - buf);
        if (o >= 0 && (uint64_t)o + n <= blen_ + 256) return p;
        if (atomicAdd(&g_txl_viol, 1u) < 16)
            printf("txlog_lanes OOB tag=%d blk=%u tid=%d t=%llu off=%lld n=%u len=%llu\n", tag,
                   blockIdx.x, tid, (unsigned long long)t, (long long)o, n, (unsigned long long)blen_);
        return buf;
    };
    // ---- header (tx.go:419-518) and this lane's first entry (tx.go:578-585)
    const uint8_t *rp = act ? buf + rec_off[t] : buf;
    uint32_t ver = 0, ml = 0, nent = 0, w = 0, q = 0;
    if (act) {
        ver = rd_be16(ok_(rp + 88, 4, 1));
        if (ver == 0) {
            nent = rd_be16(ok_(rp + 90, 2, 2));
            q = 92;
        } else {
            ml = rd_be16(ok_(rp + 90, 2, 2));
            nent = bswap(rd_le32(ok_(rp + 92 + ml, 8, 3)));
            q = 96 + ml;
        }
        w = (uint32_t)(leaf_off[t + 1] - leaf_off[t]);
    }
    const uint32_t j0 = (uint32_t)i * EP;
    const uint32_t ne = act && w > j0 ? min((uint32_t)EP, w - j0) : 0;  // this lane's entries
    // skip the j0 entries of the lanes to the left (lengths validated by the
    // host hop). Only a lane with entries walks: written as `j < j0 && j < w`
    // for every lane, the compiler dropped the `j < w` bound (q is dead when
    // ne == 0) and lanes past the record's last entry walked off the log.
    // Each step reads the entry's first 24 bytes at once (mdLen and, for
    // mdLen <= 16, kLen in them): one load round trip per entry, not two.
    if (ne) {
        for (uint32_t j = 0; j < j0; j++) {
            const uint8_t *e = rp + q;
            const uint32_t o = (uint32_t)((uintptr_t)e & 3);
            const uint32_t *ea = reinterpret_cast<const uint32_t *>(ok_(e - o, 24, 4));
            uint32_t x[6];
#pragma unroll
            for (int u = 0; u < 6; u++) x[u] = ea[u];
            auto be16x = [&](uint32_t y) -> uint32_t {  // bytes y, y+1 of x (y <= 22)
                uint32_t lo = x[0], hi = x[1];
#pragma unroll
                for (int u = 1; u < 5; u++)
                    if ((y >> 2) == (uint32_t)u) {
                        lo = x[u];
                        hi = x[u + 1];
                    }
                const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, y & 3);
                return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu);
            };
            const uint32_t m = be16x(o);
            const uint32_t k = o + 4 + m <= 24 ? be16x(o + 2 + m) : rd_be16(ok_(e + 2 + m, 2, 5));
            q += 48 + m + k;
        }
    }
    // ---- 1. this lane's subtree: entries, leaves, merges, the final fold
    State s;
    s.init();
    uint32_t mode = ne ? 0u : 5u;  // 0 digest blocks, 1 leaf, 2 merge / fold (first block), 3 its tail, 5 done
    uint32_t ej = 0, b = 0, nb = 0, la = 0, c = 0, sp = 0, rt7 = 0;
    bool fold = false;
    const uint8_t *mp = rp;
    auto entry_setup = [&]() {  // entry ej of this lane at offset q
        const uint8_t *er = rp + q;
        const uint32_t m = rd_be16(ok_(er, 2, 6)), k = rd_be16(ok_(er + 2 + m, 2, 7));
        mp = ver == 1 ? er : er + 4 + m;  // tx.go:690-731
        la = ver == 1 ? 4 + m + k : k;
        nb = (la + 32 + 8) / 64 + 1;
        q += 48 + m + k;
        b = 0;
    };
    if (ne) entry_setup();
    // the next entry prefetched while this one hashes (a lane's loads are
    // otherwise ~3 dependent round trips per entry with no other wave on the
    // SIMD to cover them at L = 1): its first 24 bytes (mdLen, kLen) issued
    // before one compression, its first message block before the next, each
    // consumed after the compression it was issued before
    uint32_t pst = ne > 1 ? 0u : 3u;  // 0 issue head, 1 parse head + issue block, 2 block loaded, 3 none
    uint32_t nq = q, n_la = 0, n_nb = 0, n_adv = 0;
    const uint8_t *n_mp = rp;
    uint32_t nx[6], pf[20];
    bool pfok = false;
    stamp(1);
#pragma unroll 1
    while (__builtin_amdgcn_ballot_w64(mode != 5)) {
        uint32_t wv16[16];
        bool on = true, tail = false;
        const uint64_t it0 = probe ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t mode0 = mode;
        if (mode == 0) {
            if (b == 0) s.init();
            uint32_t d[20];
            if (b == 0 && pfok) {
#pragma unroll
                for (int j = 0; j < 20; j++) d[j] = pf[j];
                pfok = false;
            } else {
                const uint8_t *p0 = mp - ((uintptr_t)mp & 3) + 64 * b;
                skip12_load(ok_(p0, 80, 8) == p0 ? mp : buf + 4, b, d);
            }
            skip12_words(d, (uint32_t)((uintptr_t)mp & 3), la, b, nb, wv16);
        } else if (mode == 1) {
            wv16[0] = s.h[0] >> 8;
#pragma unroll
            for (int j = 1; j < 8; j++) wv16[j] = __builtin_amdgcn_alignbit(s.h[j - 1], s.h[j], 8);
            wv16[8] = (s.h[7] << 24) | 0x00800000u;
#pragma unroll
            for (int j = 9; j < 15; j++) wv16[j] = 0;
            wv16[15] = 33u * 8u;
            s.init();
        } else if (mode == 2) {  // pop right and left, SHA256(0x01 || left || right)
            uint32_t lf[8], rg[8];
            const uint32_t *pl = slot(sp - 2), *pr = slot(sp - 1);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) {
                lf[q2] = pl[q2];
                rg[q2] = pr[q2];
            }
            rt7 = rg[7];
            s.init();
            txl_node_first(lf, rg, wv16);
        } else if (mode == 3) {
            tail = true;
        } else {
            on = false;
        }
        // the prefetch stage of this iteration (loads land during the compression)
        if (pst == 0) {
            const uint8_t *e = rp + nq;
            const uint32_t *ea = reinterpret_cast<const uint32_t *>(ok_(e - ((uintptr_t)e & 3), 24, 17));
#pragma unroll
            for (int j = 0; j < 6; j++) nx[j] = ea[j];
            pst = 1;
        } else if (pst == 1) {
            const uint32_t o = (uint32_t)((uintptr_t)(rp + nq) & 3);
            auto be16_at = [&](uint32_t x) -> uint32_t {  // bytes x, x+1 of nx (x <= 22)
                uint32_t lo = nx[0], hi = nx[1];
#pragma unroll
                for (int j = 1; j < 5; j++)
                    if ((x >> 2) == (uint32_t)j) {
                        lo = nx[j];
                        hi = nx[j + 1];
                    }
                const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, x & 3);
                return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu);
            };
            const uint32_t m = be16_at(o);
            const uint32_t k = o + 4 + m <= 24 ? be16_at(o + 2 + m) : rd_be16(ok_(rp + nq + 2 + m, 2, 18));
            const uint8_t *er = rp + nq;
            n_mp = ver == 1 ? er : er + 4 + m;  // as entry_setup
            n_la = ver == 1 ? 4 + m + k : k;
            n_nb = (n_la + 32 + 8) / 64 + 1;
            n_adv = 48 + m + k;
            const uint8_t *p0 = n_mp - ((uintptr_t)n_mp & 3);
            skip12_load(ok_(p0, 80, 19) == p0 ? n_mp : buf + 4, 0, pf);
            pst = 2;
        }
        if (on) {
            if (tail)
                compress_node_tail_g(s, rt7);
            else
                compress(s, wv16);
        }
        // bookkeeping after the block
        if (mode == 0) {
            if (++b == nb) mode = 1;
        } else if (mode == 1 || mode == 3) {
            uint32_t *d = slot(mode == 1 ? sp : sp - 2);  // a leaf is pushed; a node replaces its children
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) d[q2] = s.h[q2];
            if (mode == 1) {
                sp++;
                c++;
                ej++;
            } else {
                sp--;
            }
            // next: the merges the c-th leaf owes (tz(c): the stack holds one
            // perfect subtree per set bit of c once they are done), the next
            // entry, or the fold
            if (!fold && sp > (uint32_t)__builtin_popcount(c)) {
                mode = 2;  // two perfect subtrees of one size on top: merge
            } else if (ej < ne) {
                if (pst == 2) {  // the prefetched entry (q is at its start)
                    mp = n_mp;
                    la = n_la;
                    nb = n_nb;
                    q += n_adv;
                    b = 0;
                    pfok = true;
                } else {
                    entry_setup();
                }
                nq = q;
                pst = ej + 1 < ne ? 0u : 3u;
                mode = 0;
            } else if (sp >= 2) {
                fold = true;  // right edge: fold the stack from the right
                mode = 2;
            } else {
                mode = 5;
            }
        } else if (mode == 2) {
            mode = 3;
        }
        if (probe && mode0 < 4) acc[mode0] += __builtin_amdgcn_s_memtime() - it0;
    }
    stamp(2);
    if (probe && lane == 0)
        for (int k = 0; k < 4; k++) probe[pw * 16 + 12 + k] = acc[k] + 1;
    // ---- 2. the record's L lane roots paired (htree.go:85-110), via LDS
    // (slot 0 of each lane; a lane without entries holds nothing)
#pragma unroll 1
    for (int l = 0; l < LGL; l++) {
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t sft = 1u << l;
        const bool me = act && (i & (2 * sft - 1)) == 0 && (uint32_t)(i + sft) * EP < w;
        uint32_t wv16[16];
        if (me) {
            uint32_t lf[8], rg[8];
            const uint32_t *pl = slot(0), *pr = stk + (((uint32_t)0 * 256 + tid + sft) * kTxlStackPad);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) {
                lf[q2] = pl[q2];
                rg[q2] = pr[q2];
            }
            rt7 = rg[7];
            s.init();
            txl_node_first(lf, rg, wv16);
            compress(s, wv16);
            compress_node_tail_g(s, rt7);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (me) {
            uint32_t *d = slot(0);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) d[q2] = s.h[q2];
        }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(3);
    // ---- 3. innerHash + Alh on the record's first lane
    const bool head = act && i == 0;
    uint32_t eh[8], a[8];
    const uint32_t blen = ver ? 8 + ml : 4, mlen = 80 + blen;
    // fast path (every v0 record, v1 with mdLen <= 16): the record head
    // [rp, rp + 116) and the stored Alh in ONE batch of aligned dword loads,
    // the innerHash message assembled in this record's LDS row (33 words: no
    // bank conflicts between the wave's rows) with two aligned runs -- ts ||
    // (version ...nentries) and Eh || blTxID || blRoot shifted by blen & 3 --
    // and read back word by word; otherwise message bytes straight from the log
    const bool fast = !ver || ml <= 16;
    const uint32_t al = (uint32_t)((uintptr_t)rp & 3);
    uint32_t hrw[30], av[9];
    if (head && fast) {  // (a record is >= 124 bytes: header + Alh)
        const uint32_t *hb = reinterpret_cast<const uint32_t *>(ok_(rp - al, 120, 20));
#pragma unroll
        for (int j = 0; j < 30; j++) hrw[j] = hb[j];
        const uint8_t *ap = buf + alh_off[t];
        const uint32_t *ab = reinterpret_cast<const uint32_t *>(ok_(ap - ((uintptr_t)ap & 3), 36, 21));
#pragma unroll
        for (int j = 0; j < 9; j++) av[j] = ab[j];
    }
    auto le = [&](int o) -> uint32_t {  // the LE dword at rp + o (o: a constant multiple of 4, <= 112)
        return __builtin_amdgcn_alignbyte(hrw[o / 4 + 1], hrw[o / 4], al);
    };
    uint32_t *msg = stk + (uint32_t)dep * 256 * kTxlStackPad + ((uint32_t)wv * R + r) * 33;
    if (head) {
        if (w == 0) {
            load_digest(kEmptyRootDev, eh);  // SHA256(nil), htree.go:73-77
        } else {
            const uint32_t *p0 = slot(0);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) eh[q2] = p0[q2];
        }
        if (fast) {  // message bytes in order: [0,8) ts, [8, 8 + blen) rp[88..), then Eh, rp[16..56)
            msg[0] = le(8);
            msg[1] = le(12);
            const uint32_t nY = blen >> 2, sh = blen & 3;
#pragma unroll
            for (int u = 0; u < 7; u++)
                if ((uint32_t)u <= nY) msg[2 + u] = le(88 + 4 * u);  // u == nY: the partial word
            uint32_t S[18];
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) S[q2] = bswap(eh[q2]);
#pragma unroll
            for (int u = 0; u < 10; u++) S[8 + u] = le(16 + 4 * u);
            uint32_t *dst = msg + 2 + nY;
            const uint32_t prev = sh ? dst[0] << (8 * (4 - sh)) : 0u;  // Y's last sh bytes, on top
#pragma unroll
            for (int t2 = 0; t2 < 19; t2++) {
                const uint32_t lo = t2 ? S[t2 - 1] : prev, hi = t2 < 18 ? S[t2] : 0u;
                dst[t2] = sh ? __builtin_amdgcn_alignbyte(hi, lo, 4 - sh) : hi;
            }
        }
    }
    const uint32_t nbi = head ? (mlen + 8) / 64 + 1 : 0;
    const uint32_t nH = wave_max_u32(head ? nbi + 2 : 0);
    stamp(4);
#pragma unroll 1
    for (uint32_t k = 0; k < nH; k++) {
        uint32_t wv16[16];
        const bool on = head && k < nbi + 2;
        if (on) {
            if (k < nbi) {  // ts || version || md part || Eh || blTxID || blRoot
                if (k == 0) s.init();
                if (fast) {
#pragma unroll
                    for (int jw = 0; jw < 16; jw++) {
                        const int v = (int)mlen - (int)(64 * k + 4 * jw);  // message bytes left at this word
                        const uint32_t pad = (uint32_t)(0x80000000ull >> (8 * (v < 0 ? 5 : min(v, 4))));
                        wv16[jw] = __builtin_amdgcn_bitop3_b32(bswap(msg[16 * k + jw]), head_mask(v), pad, 0xEA);
                    }
                    if (k + 1 == nbi) {
                        wv16[14] = 0;
                        wv16[15] = mlen * 8;  // the bit length
                    }
                } else {
#pragma unroll 4
                    for (int jw = 0; jw < 16; jw++) {
                        uint32_t v32 = 0;
                        if (jw == 15 && k + 1 == nbi) {
                            v32 = mlen * 8;  // the bit length
                        } else {
#pragma unroll
                            for (int bb = 0; bb < 4; bb++) {
                                const uint32_t kk = 64 * k + 4 * jw + bb;
                                uint32_t v;
                                if (kk < 8) v = *ok_(rp + 8 + kk, 1, 9);
                                else if (kk < 8 + blen) v = *ok_(rp + 80 + kk, 1, 10);
                                else if (kk < 40 + blen) {
                                    const uint32_t o = kk - 8 - blen;
                                    v = (eh[o >> 2] >> (24 - 8 * (o & 3))) & 0xffu;
                                } else if (kk < mlen) v = *ok_(rp + kk - 24 - blen, 1, 11);
                                else v = kk == mlen ? 0x80u : 0u;
                                v32 = v32 << 8 | v;
                            }
                        }
                        wv16[jw] = v32;
                    }
                }
            } else if (k == nbi) {  // BE64 id || prevAlh || innerHash[0:24]
                copy8(a, s.h);      // (a: the innerHash until the Alh is done)
                s.init();
                if (fast) {
                    wv16[0] = bswap(le(0));
                    wv16[1] = bswap(le(4));
#pragma unroll
                    for (int q2 = 0; q2 < 8; q2++) wv16[2 + q2] = bswap(le(56 + 4 * q2));
                } else {
                    const uint64_t id = rd_be64(ok_(rp, 16, 12));
                    wv16[0] = (uint32_t)(id >> 32);
                    wv16[1] = (uint32_t)id;
#pragma unroll
                    for (int q2 = 0; q2 < 8; q2++) wv16[2 + q2] = bswap(rd_le32(ok_(rp + 56 + 4 * q2, 8, 13)));
                }
#pragma unroll
                for (int q2 = 0; q2 < 6; q2++) wv16[10 + q2] = a[q2];
            } else {
                wv16[0] = a[6];
                wv16[1] = a[7];
                wv16[2] = 0x80000000u;
#pragma unroll
                for (int q2 = 3; q2 < 15; q2++) wv16[q2] = 0;
                wv16[15] = 72u * 8u;
            }
            compress(s, wv16);
        }
    }
    copy8(a, s.h);
    stamp(5);
    int32_t stv = MH_OK;
    uint64_t hw[17];
    if (head) {  // tx.go:623-627
        uint32_t xx = 0;
        if (fast) {
            const uint32_t aal = (uint32_t)((uintptr_t)(buf + alh_off[t]) & 3);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++)
                xx |= bswap(__builtin_amdgcn_alignbyte(av[q2 + 1], av[q2], aal)) ^ a[q2];
        } else {
            const uint8_t *ap = ok_(buf + alh_off[t], 40, 14);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) xx |= bswap(rd_le32(ap + 4 * q2)) ^ a[q2];
        }
        stv = xx ? MH_ERR_CORRUPTED_DATA : MH_OK;
        status[t] = stv;
        store_digest(eh_out + t * 32, eh);
        store_digest(alh_out + t * 32, a);
        if (fast) {
#pragma unroll
            for (int q2 = 0; q2 < 3; q2++)
                hw[q2] = ((uint64_t)bswap(le(8 * q2)) << 32) | bswap(le(8 * q2 + 4));
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++)
                hw[3 + q2] = (uint64_t)le(24 + 8 * q2) | ((uint64_t)le(28 + 8 * q2) << 32);
        } else {
#pragma unroll
            for (int q2 = 0; q2 < 3; q2++) hw[q2] = rd_be64(ok_(rp + 8 * q2, 16, 15));
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) hw[3 + q2] = rd_raw64(ok_(rp + 24 + 8 * q2, 16, 16));
        }
#pragma unroll
        for (int q2 = 0; q2 < 4; q2++)
            hw[11 + q2] = (uint64_t)bswap(eh[2 * q2]) | ((uint64_t)bswap(eh[2 * q2 + 1]) << 32);
        hw[15] = (uint64_t)ver | ((uint64_t)nent << 32);
        hw[16] = ver ? (uint64_t)ml | ((uint64_t)(uint32_t)(rec_off[t] + 92) << 32) : 0;
    }
    // ---- 4. the workgroup's records out as contiguous runs (the stack is free)
    __syncthreads();
    const uint32_t RW = 4 * R;  // records per workgroup
    uint64_t *hst = reinterpret_cast<uint64_t *>(lds);
    uint32_t *ast = reinterpret_cast<uint32_t *>(hst + RW * 17);
    uint32_t *sst = ast + RW * 8;
    const uint32_t rw = (uint32_t)wv * R + r;  // this record in the workgroup
    if (head) {
#pragma unroll
        for (int q2 = 0; q2 < 17; q2++) hst[rw * 17 + q2] = hw[q2];
#pragma unroll
        for (int q2 = 0; q2 < 8; q2++) ast[rw * 8 + q2] = bswap(a[q2]);
        sst[rw] = (uint32_t)stv;
    }
    __syncthreads();
    stamp(6);
    const uint64_t nb_ = T0 < ntx ? min((uint64_t)RW, ntx - T0) : 0;
    uint64_t *hd = ho.hdrs ? ho.hdrs + T0 * 17 : reinterpret_cast<uint64_t *>(hdrs) + T0 * 17;
    if (ho.hdrs && ho.eh_only) {
        for (uint32_t k = tid; k < nb_ * 4; k += 256) {
            const uint32_t rec = k >> 2, j = 11 + (k & 3);
            hd[rec * 17 + j] = hst[rec * 17 + j];
        }
    } else {
        for (uint32_t k = tid; k < nb_ * 17; k += 256) hd[k] = hst[k];
    }
    if (ho.alh)
        for (uint32_t k = tid; k < nb_ * 8; k += 256) ho.alh[T0 * 8 + k] = ast[k];
    if (ho.status)
        for (uint32_t k = tid; k < nb_; k += 256) ho.status[T0 + k] = sst[k];
    if (fence && (ho.status || ho.alh || ho.hdrs)) __threadfence_system();
    stamp(7);
    stamp(8);
    stamp(9);
    if (probe && lane == 0) probe[pw * 16 + 11] = __builtin_amdgcn_s_memrealtime();
}

hipError_t launch_txlog_lanes(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                              const uint64_t *rec_off, const uint64_t *alh_off,
                              const uint64_t *leaf_off, MhTxHeader *hdrs, uint8_t *eh_out,
                              uint8_t *alh_out, int32_t *status, const TxlogHostOut &ho,
                              uint64_t wmax, uint64_t log_len) {
    if (!ntx) return hipSuccess;
    if (wmax > 64 || ((uintptr_t)ho.hdrs & 7) || ((uintptr_t)ho.alh & 3) || ((uintptr_t)ho.status & 3))
        return hipErrorInvalidValue;
    int lgp = 0;
    while ((1ull << lgp) < wmax) lgp++;
    // lanes per record: the fewest that give every SIMD two waves (2048 waves
    // of 64 lanes: one wave per SIMD issues VALU 0.76 of its cycles, two 0.9,
    // for ~10 % more instructions at L = 2, profiles/txlog_lanes_r05.txt; a
    // record's chain is 2 EP + 2 (EP - 1) + 2 log2 L + 4 compressions, EP = P /
    // L, so fewer records take more lanes: latency), at most 16;
    // MH_TXLOG_LANES=1|2|4|8|16 forces it (read per call)
    int lgl = 0;
    while (lgl < 4 && (ntx << lgl) < 2048ull * 64) lgl++;  // two waves per SIMD (176 VGPRs: at most 2)
    if (const char *e = getenv("MH_TXLOG_LANES")) {
        const int v = atoi(e);
        lgl = v >= 16 ? 4 : v >= 8 ? 3 : v >= 4 ? 2 : v >= 2 ? 1 : 0;
    }
    lgl = std::min(lgl, lgp);  // never more lanes than entries
    const int R = 64 >> lgl;
    const int dep = std::max(1, lgp - lgl + 1);  // stack depth: log2(EP) + 1
    const size_t stack = (size_t)dep * 256 * kTxlStackPad * 4 + (size_t)4 * R * 33 * 4;  // + innerHash rows
    const size_t res = (size_t)4 * R * (17 * 8 + 8 * 4 + 4);
    const size_t sh = std::max(stack, res);
    static const int fence = [] {
        const char *e = getenv("MH_TXLOG_FENCE");
        return e && atoi(e) ? 1 : 0;
    }();
    static const bool attr = [] {
        const int mx = 160 << 10;
        const void *fs[] = {(const void *)k_txlog_lanes<0, false>, (const void *)k_txlog_lanes<1, false>,
                            (const void *)k_txlog_lanes<2, false>, (const void *)k_txlog_lanes<3, false>,
                            (const void *)k_txlog_lanes<4, false>, (const void *)k_txlog_lanes<0, true>,
                            (const void *)k_txlog_lanes<1, true>,  (const void *)k_txlog_lanes<2, true>,
                            (const void *)k_txlog_lanes<3, true>,  (const void *)k_txlog_lanes<4, true>};
        for (const void *f : fs) hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    TimerScope ts(tm, "txlog_lanes", st);
    const dim3 grid((unsigned)((ntx + 4ull * R - 1) / (4ull * R))), blk(256);
    static const bool chk = [] {
        const char *e = getenv("MH_TXLOG_LANES_CHECK");
        return e && atoi(e) != 0;
    }();
    uint64_t *probe = txlog_probe_slot(grid.x * 4);
#define MH_TXL(l_, c_)                                                                             \
    hipLaunchKernelGGL((k_txlog_lanes<l_, c_>), grid, blk, sh, st, ntx, buf, rec_off, alh_off,   \
                       leaf_off, hdrs, eh_out, alh_out, status, ho, lgp, dep, fence, log_len, probe)
    if (chk) {  // diagnosis: the launch is synchronous and fails on any out-of-range read
        unsigned zero = 0, viol = 0;
        hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_txl_viol), &zero, sizeof zero, 0,
                                              hipMemcpyHostToDevice, st);
        if (e != hipSuccess) return e;
        if (lgl == 0) MH_TXL(0, true);
        else if (lgl == 1) MH_TXL(1, true);
        else if (lgl == 2) MH_TXL(2, true);
        else if (lgl == 3) MH_TXL(3, true);
        else MH_TXL(4, true);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        e = hipMemcpyFromSymbolAsync(&viol, HIP_SYMBOL(g_txl_viol), sizeof viol, 0,
                                     hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        if (viol) {
            fprintf(stderr, "txlog_lanes: %u out-of-range reads\n", viol);
            return hipErrorIllegalAddress;
        }
    } else {
        if (lgl == 0) MH_TXL(0, false);
        else if (lgl == 1) MH_TXL(1, false);
        else if (lgl == 2) MH_TXL(2, false);
        else if (lgl == 3) MH_TXL(3, false);
        else MH_TXL(4, false);
    }
#undef MH_TXL
    return hipGetLastError();
}

// ---------------------------------------------------------------- many trees
// Level l of a batch of independent htrees.  Item k describes one tree that
// still has > 1 node at level l-1: its nodes at level l are written at
// cur_base[k] .. cur_base[k] + ceil(prev_w[k] / 2), its level-(l-1) nodes
// live at prev_base[k].  Thread i finds its item by binary search over
// cur_base (sorted) and pairs (or promotes) exactly as htree.go:85-110.
__global__ __launch_bounds__(256) void k_seg_level(uint64_t nnodes, uint64_t level_base,
                                                   uint32_t nitems,
                                                   const uint64_t *__restrict__ cur_base,
                                                   const uint64_t *__restrict__ prev_base,
                                                   const uint64_t *__restrict__ prev_w,
                                                   uint8_t *__restrict__ nodes) {
    extern __shared__ uint32_t tab[];
    node_tab_init(tab);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnodes;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = level_base + i;
        uint32_t lo = 0, hi = nitems - 1;
        while (lo < hi) {  // last k with cur_base[k] <= g
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (cur_base[mid] <= g)
                lo = mid;
            else
                hi = mid - 1;
        }
        const uint64_t j = g - cur_base[lo];
        const uint64_t lpos = prev_base[lo] + 2 * j;
        uint32_t a[8], o[8];
        load_digest(nodes + lpos * 32, a);
        if (2 * j + 1 < prev_w[lo]) {
            uint32_t b[8];
            load_digest(nodes + (lpos + 1) * 32, b);
            node_hash_tab(a, b, o, tab);
        } else {
            copy8(o, a);
        }
        store_digest(nodes + g * 32, o);
    }
}

__global__ __launch_bounds__(256) void k_gather32(uint64_t n, const uint8_t *__restrict__ src,
                                                  const uint64_t *__restrict__ idx,
                                                  uint8_t *__restrict__ out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = idx[p];
    const uint4 *s = reinterpret_cast<const uint4 *>(k == ~0ull ? kEmptyRootDev : src + k * 32);
    uint4 *d = reinterpret_cast<uint4 *>(out + p * 32);
    d[0] = s[0];
    d[1] = s[1];
}

// ---------------------------------------------------------------- launchers
hipError_t launch_tx_alh(hipStream_t st, Timer *tm, uint64_t n, const MhTxHeader *hdrs,
                         const uint8_t *md_blob, const uint8_t *eh_src, uint8_t *scratch,
                         const uint8_t *expect, const uint64_t *expect_off, uint8_t *inner_out,
                         uint8_t *alh_out, int32_t *status) {
    if (!n) return hipSuccess;
    TimerScope ts(tm, "tx_alh", st);
    hipLaunchKernelGGL(k_tx_alh, dim3(grid_for(n, 256)), dim3(256), 0, st, n, hdrs, md_blob,
                       eh_src, scratch, expect, expect_off, inner_out, alh_out, status);
    return hipGetLastError();
}

hipError_t launch_leaf_for(hipStream_t st, Timer *tm, uint64_t n, const uint8_t *in, uint8_t *out) {
    if (!n) return hipSuccess;
    TimerScope ts(tm, "leaf_for", st);
    hipLaunchKernelGGL(k_leaf_for, dim3(grid_for(n, 256)), dim3(256), 0, st, n, in, out);
    return hipGetLastError();
}

hipError_t launch_select32(hipStream_t st, uint64_t n, const uint8_t *sel, const uint8_t *x,
                           const uint8_t *y, uint8_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_select32, dim3(grid_for(n, 256)), dim3(256), 0, st, n, sel, x, y, out);
    return hipGetLastError();
}

hipError_t launch_linear_verify(hipStream_t st, Timer *tm, uint64_t n, const uint64_t *psrc,
                                const uint64_t *ptgt, const uint64_t *src, const uint64_t *tgt,
                                const uint64_t *term_off, const uint8_t *terms,
                                const uint8_t *src_alh, const uint8_t *tgt_alh, uint8_t *ok) {
    if (!n) return hipSuccess;
    TimerScope ts(tm, "linear_verify", st);
    hipLaunchKernelGGL(k_linear_verify, dim3(grid_for(n, 256)), dim3(256), 0, st, n, psrc, ptgt,
                       src, tgt, term_off, terms, src_alh, tgt_alh, ok);
    return hipGetLastError();
}

hipError_t launch_advance_chain(hipStream_t st, Timer *tm, uint64_t n, const uint64_t *start,
                                const uint64_t *cnt, const uint64_t *term_off,
                                const uint8_t *terms, const uint64_t *first,
                                const uint8_t *end_alh, uint8_t *leaves_src, uint8_t *ok) {
    if (!n) return hipSuccess;
    TimerScope ts(tm, "advance_chain", st);
    hipLaunchKernelGGL(k_advance_chain, dim3(grid_for(n, 256)), dim3(256), 0, st, n, start, cnt,
                       term_off, terms, first, end_alh, leaves_src, ok);
    return hipGetLastError();
}

hipError_t launch_txe_leaf(hipStream_t st, Timer *tm, uint64_t n, const uint8_t *buf,
                           const uint64_t *rec_off, const uint8_t *ver, bool leaf, uint8_t *out) {
    if (!n) return hipSuccess;
    TimerScope ts(tm, "txe_leaf", st);
    hipLaunchKernelGGL(k_txe_leaf, dim3(grid_for(n, 256)), dim3(256), 0, st, n, buf, rec_off, ver,
                       leaf ? 1 : 0, out);
    return hipGetLastError();
}

hipError_t launch_seg_level(hipStream_t st, Timer *tm, uint64_t nnodes, uint64_t level_base,
                            uint32_t nitems, const uint64_t *cur_base, const uint64_t *prev_base,
                            const uint64_t *prev_w, uint8_t *nodes) {
    if (!nnodes || !nitems) return hipSuccess;
    TimerScope ts(tm, "seg_level", st);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const unsigned grid = (unsigned)std::min<uint64_t>(grid_for(nnodes, 256), (uint64_t)cus * 8);
    hipLaunchKernelGGL(k_seg_level, dim3(grid), dim3(256), kNodeTabBytes, st, nnodes, level_base,
                       nitems, cur_base, prev_base, prev_w, nodes);
    return hipGetLastError();
}

hipError_t launch_gather32(hipStream_t st, uint64_t n, const uint8_t *src, const uint64_t *idx,
                           uint8_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather32, dim3(grid_for(n, 256)), dim3(256), 0, st, n, src, idx, out);
    return hipGetLastError();
}

}  // namespace mh
