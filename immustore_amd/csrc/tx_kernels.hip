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
    } else if (wmax <= 64) {
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
