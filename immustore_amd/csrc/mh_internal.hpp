// mh_internal.hpp -- shared declarations between the kernel translation units
// and the C-ABI implementation (capi.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/immustore_merkle.h"

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

// nodesUpto(n) for device code (proof_kernels.hip)
__host__ __device__ inline uint64_t ahtree_nodes_upto_dev(uint64_t n) { return n + popsum_below(n); }


constexpr int kMaxLevels = 66;

// Level-major flat layout of an htree of width n (embedded/htree/htree.go:
// levels[l] holds ceil(n/2^l) used nodes; promoted odd nodes are copied up).
struct LevelGeom {
    uint64_t n = 0;
    int nlevels = 0;                // number of levels incl. root level
    uint64_t off[kMaxLevels] = {};  // offset (in 32-byte nodes) of level l
    uint64_t width[kMaxLevels] = {};
    uint64_t total = 0;             // total nodes
    void init(uint64_t n_);
};

// Kernel arguments passed by value (fits in the 4 KB kernarg segment).
struct LevelArgs {
    uint64_t off[kMaxLevels];
    uint64_t width[kMaxLevels];
};

struct KWTable {
    uint32_t kw[64];
};

// Compute K[t]+W[t] of the padding block of a message of `len` bytes whose
// length is a multiple of 64 (constant schedule: 0x80, zeros, bit length).
void pad_block_kw(uint64_t len, KWTable *out);

// ---------------------------------------------------------------- launchers
// All return hipError_t (hipSuccess == 0) and enqueue on `st`.
// Per-kernel timing hook (ctx-level); may be null.
struct Timer {
    virtual void begin(const char *name, hipStream_t st) = 0;
    virtual void end(hipStream_t st) = 0;
    virtual ~Timer() {}
};

struct TimerScope {
    Timer *tm;
    hipStream_t st;
    TimerScope(Timer *t, const char *name, hipStream_t s) : tm(t), st(s) {
        if (tm) tm->begin(name, st);
    }
    ~TimerScope() {
        if (tm) tm->end(st);
    }
};

hipError_t launch_entries_fixed(hipStream_t st, Timer *tm, int version, uint64_t n,
                                const uint8_t *keys, uint32_t key_len, const uint8_t *vals,
                                uint32_t val_len, uint8_t *hvals_out, uint8_t *levels,
                                const LevelGeom &g, int *lanes_levels_done);
bool entries_fixed_supported(int version, const uint8_t *keys, uint32_t key_len,
                             const uint8_t *vals, uint32_t val_len);

// SHA-256 of n ragged byte ranges buf[off[i] .. off[i+1]) (varlen_kernels.hip);
// override32[i] replaces message i where use_override[i] != 0.  scratch
// (sha_varlen_scratch_bytes(n), device, stream-ordered on st) lets the
// messages be bucketed by block count first; null hashes them in input order.
size_t sha_varlen_scratch_bytes(uint64_t n);
hipError_t launch_sha256_csr(hipStream_t st, Timer *tm, const uint8_t *buf, const uint64_t *off,
                             uint64_t n, const uint8_t *override32, const uint8_t *use_override,
                             uint8_t *out32, uint8_t *scratch);
// readValueAt's integrity check (immustore.go:3235) over a batch: status[i] =
// MH_OK iff off[i+1] - off[i] == exp_len[i] (exp_len may be null) and
// SHA256(buf[off[i] .. off[i+1])) == expect[i], else MH_ERR_CORRUPTED_DATA.
hipError_t launch_verify_values(hipStream_t st, Timer *tm, const uint8_t *buf, const uint64_t *off,
                                uint64_t n, const uint64_t *exp_len, const uint8_t *expect,
                                int32_t *status, uint8_t *scratch);
// Fused ragged entries (varlen_kernels.hip): hVal (or override) -> hvals_out
// (may be null), entry digest (tx.go:690-731) -> out32, or its htree leaf when
// leaf is set (level 0 of the tree).  scratch as for launch_sha256_csr.
// ver_e (device, n bytes, may be null): per-entry digest version instead of
// `version` (a v0 entry's metadata is then not hashed).  override32 with a
// null use_override overrides every entry (val_off / vals may be null).
hipError_t launch_entries_varlen(hipStream_t st, Timer *tm, int version, uint64_t n,
                                 const uint8_t *keys, const uint64_t *key_off, const uint8_t *md,
                                 const uint64_t *md_off, const uint8_t *vals,
                                 const uint64_t *val_off, const uint8_t *override32,
                                 const uint8_t *use_override, uint8_t *hvals_out, uint8_t *out32,
                                 bool leaf, uint8_t *scratch, const uint8_t *ver_e = nullptr);
// Leaves from digests (htree.go:79-83) + in-lane levels up to log2(LPL).
hipError_t launch_leaves_from_digests(hipStream_t st, Timer *tm, const uint8_t *digests,
                                      uint64_t n, uint8_t *levels, const LevelGeom &g,
                                      int *levels_done);
// Copy nodes into level 0 (no leaf hashing): used for reducing subtree roots.
// Reduce levels [from, top] in place (htree.go:85-110).
hipError_t launch_reduce(hipStream_t st, Timer *tm, uint8_t *levels, const LevelGeom &g,
                         int from_level, uint8_t *root = nullptr);

// Generic helpers
hipError_t launch_fill_random(hipStream_t st, uint8_t *dst, uint64_t nbytes, uint64_t seed);
hipError_t launch_fill_keys_be64(hipStream_t st, uint8_t *dst, uint64_t n, uint64_t first);
hipError_t launch_iota_offsets(hipStream_t st, uint64_t *off, uint64_t n, uint64_t stride);
hipError_t launch_gather_nodes(hipStream_t st, const uint8_t *src, const uint64_t *idx, uint64_t n,
                               uint8_t *dst);

// ---- verification (embedded/htree/htree.go:166-195, ahtree/verification.go)
hipError_t launch_htree_verify(hipStream_t st, Timer *tm, uint64_t np, const uint64_t *leaf,
                               const uint64_t *width, const uint64_t *term_off,
                               const uint8_t *terms, const uint8_t *digests, const uint8_t *roots,
                               uint8_t *ok);
hipError_t launch_ahtree_verify(hipStream_t st, Timer *tm, int kind, uint64_t np,
                                const uint64_t *i, const uint64_t *j, const uint64_t *term_off,
                                const uint8_t *terms, const uint8_t *a, const uint8_t *b,
                                uint8_t *ok, uint8_t *eval_out);

// ---- ahtree batch append (embedded/ahtree/ahtree.go:246-373)
// work_ctr: 4 bytes of device memory private to this launch's stream order
// (the spine kernel's work queue; reset on `st` before the launch).
// Optional appendable record streams of the appended payloads (SURVEY.md
// 8(f) row 4): pLog records BE32 len || payload at plog + i*(4+plen), cLog
// entries BE64 (p_off0 + i*(4+plen)) || BE32 len at clog + i*12.
struct AhtLogs {
    uint8_t *plog = nullptr;
    uint8_t *clog = nullptr;
    uint64_t p_off0 = 0;
};
// The left edge of an append range (n0, ...] whose dLog buffer does not hold
// the nodes before it: every node such a range reads that ends at or before
// lo is a peak of lo (node(lo with the bits below l cleared, l) for a set bit
// l of lo, ahtree.go:296-322), so the 64-slot frontier fr[l] (device, 32 B
// per level, only set bits of lo meaningful) replaces the old dLog.  lo = 0:
// no edge, every node from the dLog.
struct AhtEdge {
    const uint8_t *fr = nullptr;
    uint64_t lo = 0;
};
hipError_t launch_ahtree_append(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0,
                                const uint8_t *payloads, uint64_t m, uint32_t plen,
                                uint8_t *roots_out, uint32_t *work_ctr,
                                const AhtLogs &lg = AhtLogs(), const AhtEdge &edge = AhtEdge());
// The three phases of launch_ahtree_append, for sharded appends.
// dlog == nullptr: records only.
hipError_t launch_ahtree_leaves(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0,
                                const uint8_t *payloads, uint64_t m, uint32_t plen,
                                const AhtLogs &lg = AhtLogs());
hipError_t launch_ahtree_perfect(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0,
                                 uint64_t n_end, int lmin, int lmax,
                                 const AhtEdge &edge = AhtEdge());
hipError_t launch_ahtree_spine(hipStream_t st, Timer *tm, uint8_t *dlog, uint64_t n0, uint64_t m,
                               uint8_t *roots_out, uint32_t *work_ctr,
                               const AhtEdge &edge = AhtEdge());
hipError_t launch_ahtree_put_shard_roots(hipStream_t st, Timer *tm, uint8_t *dlog, int level,
                                         uint64_t count, const uint8_t *roots);

// Ranged multi-device append (capi_multi.hip): the batch (n0, n0 + total] is
// cut at multiples of S = 2^k into G <= 64 device ranges (b[d], b[d+1]]; a
// device keeps only its own dLog range.  Pieces are the aligned blocks of S
// appends; piece E ends at E*S and its level-k root is node(E*S, k).
constexpr int kAhtMaxRanges = 64;
struct AhtTopArgs {
    int k = 0;                           // shard bits: S = 2^k
    int nlev = 0;                        // levels of the piece tree (l' = 0 .. nlev-1)
    int G = 0;                           // device ranges
    uint64_t n0 = 0;                     // old size
    uint64_t lo = 0, hi = 0;             // this device's range (lo, hi]
    uint64_t N0 = 0, Pend = 0, Pmax = 0; // floor(n0/S), floor((n0+total)/S), pieces per send slot
    uint64_t lev_off[64] = {};           // slot offset of piece level l' in the top buffer
    uint64_t pe0[kAhtMaxRanges + 1] = {};  // floor(b[d]/S), d = 0..G
};
// the level-k roots of this device's pieces E in (pe0[d], pe0[d+1]] into send
hipError_t launch_ahtree_gather_pieces(hipStream_t st, const uint8_t *dlog, int k, uint64_t e0,
                                       uint64_t count, uint8_t *send);
// piece tree over the all-gathered piece roots and the old peaks of n0 (levels
// >= k), the nodes above level k that end in (lo, hi] into dlog, and this
// device's frontier (peaks of lo) into fr (lo > n0 only)
hipError_t launch_ahtree_top(hipStream_t st, const AhtTopArgs &a, const uint8_t *recv,
                             const uint8_t *peaks_n0, uint8_t *top, uint8_t *dlog, uint8_t *fr);
// the 64-slot frontier (32 B per level) by value, written to dst on st
struct AhtSlots {
    uint8_t b[64 * 32];
};
hipError_t launch_ahtree_put_slots(hipStream_t st, const AhtSlots &s, uint8_t *dst);
// the peaks of n from a device dLog into the 64-slot frontier layout
hipError_t launch_ahtree_peaks(hipStream_t st, const uint8_t *dlog, uint64_t n, uint8_t *fr);

// host-side index math shared with the C API
uint64_t ahtree_nodes_upto(uint64_t n);
uint64_t ahtree_nodes_until(uint64_t n);


// ---------------------------------------------------------------- tx layer
typedef mh_tx_header MhTxHeader;
constexpr uint64_t kTxInnerStride = 384;  // >= 8+2+2+268+4+32+8+32 (tx.go:249-302)

hipError_t launch_tx_alh(hipStream_t st, Timer *tm, uint64_t n, const MhTxHeader *hdrs,
                         const uint8_t *md_blob, const uint8_t *eh_src, uint8_t *scratch,
                         const uint8_t *expect, const uint64_t *expect_off, uint8_t *inner_out,
                         uint8_t *alh_out, int32_t *status);
hipError_t launch_leaf_for(hipStream_t st, Timer *tm, uint64_t n, const uint8_t *in, uint8_t *out);
hipError_t launch_select32(hipStream_t st, uint64_t n, const uint8_t *sel, const uint8_t *x,
                           const uint8_t *y, uint8_t *out);
hipError_t launch_linear_verify(hipStream_t st, Timer *tm, uint64_t n, const uint64_t *psrc,
                                const uint64_t *ptgt, const uint64_t *src, const uint64_t *tgt,
                                const uint64_t *term_off, const uint8_t *terms,
                                const uint8_t *src_alh, const uint8_t *tgt_alh, uint8_t *ok);
hipError_t launch_advance_chain(hipStream_t st, Timer *tm, uint64_t n, const uint64_t *start,
                                const uint64_t *cnt, const uint64_t *term_off,
                                const uint8_t *terms, const uint64_t *first,
                                const uint8_t *end_alh, uint8_t *leaves_src, uint8_t *ok);
// roots of many htrees (widths leaf_off[t+1]-leaf_off[t], small), one lane
// each, in place over nodes = their leaf hashes back to back
constexpr uint64_t kSmallTreeMax = 64;
// launch_small_roots covers every batch whose widest tree has <= 64 leaves
// without a host tree plan: a wave per tree for <= 2048 trees (latency), the
// level-parallel packed kernel for more (every node of a level at once,
// 512 / P trees per workgroup); wider trees go through the host tree plan
// (k_seg_level).
inline bool small_roots_fit(uint64_t ntrees, uint64_t wmax) {
    (void)ntrees;
    return wmax <= kSmallTreeMax;
}
// wmax: the widest tree (<= kSmallTreeMax picks the level-parallel kernel
// for many trees)
hipError_t launch_small_roots(hipStream_t st, Timer *tm, uint64_t ntrees, const uint64_t *leaf_off,
                              uint8_t *nodes, uint8_t *roots, uint64_t wmax);
// the levels above a row of 1 <= w <= 64 nodes (flat level-major, level 0 =
// the row) and their root, one single-wave launch
hipError_t launch_reduce_small(hipStream_t st, const uint8_t *nodes, uint64_t w, uint8_t *levels,
                               uint8_t *root);
// headers + first-entry offsets of tx records from the raw log (md_off relative to buf)
hipError_t launch_tx_hdr_from_raw(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                                  const uint64_t *rec_off, MhTxHeader *hdrs, uint64_t *ent_start);
// non-canonical metadata of a tx log: rec_off[e_idx[k]] = e_off[k];
// hdrs[h_idx[k]].md_off / md_len = low / high 32 bits of h_val[k]
hipError_t launch_txlog_patch(hipStream_t st, uint64_t ne, const uint64_t *e_idx,
                              const uint64_t *e_off, uint64_t *rec_off, uint64_t nh,
                              const uint64_t *h_idx, const uint64_t *h_val, MhTxHeader *hdrs);
hipError_t launch_put_eh(hipStream_t st, uint64_t n, const uint8_t *eh, MhTxHeader *hdrs);
// The fused a14 kernels (tx.go:533-630 per record, one launch for a group of
// records): headers, entry walk, entry digests + leaves, each tx's htree, Eh,
// innerHash + Alh against the stored Alh (statuses).  Arrays are indexed from
// the group's first record; leaf_off has ntx + 1 entries (nullable for
// k_txlog_lanes: the entry count is then the header's, checked by the
// structure pre-pass).  pre (nullable): the pre-pass statuses -- a record with
// pre[t] != 0 is not walked, its status is pre[t] and its Alh / Eh / header 0.
// ho (device addresses of pinned host arrays, or device arrays, each member
// nullable, indexed like the device arrays): results written there by the
// kernel too.  hdrs 8-byte aligned, alh / status 4-byte.
struct TxlogHostOut {
    uint32_t *status = nullptr;
    uint32_t *alh = nullptr;
    uint64_t *hdrs = nullptr;
    int eh_only = 0;  // of hdrs, only the Eh words (the host writes the rest)
};
// one wave per 64 / L records (k_txlog_wave, txlog_wave.hip), wmax <= 64;
// h_rec_off / h_alh_off: host-readable copies of rec_off / alh_off (the
// wave's LDS staging is sized from them)
hipError_t launch_txlog_wave(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                             const uint64_t *rec_off, const uint64_t *alh_off,
                             const uint64_t *leaf_off, const int32_t *pre, MhTxHeader *hdrs,
                             uint8_t *eh_out, uint8_t *alh_out, int32_t *status,
                             const TxlogHostOut &ho, uint64_t wmax, const uint64_t *h_rec_off,
                             const uint64_t *h_alh_off);
// every record on 1-16 lanes, each lane's subtree serial (k_txlog_lanes,
// txlog_lanes.hip), wmax <= kTxlLanesMaxEntries; log_len: the log's length
// (the checking build's range).  wmax_dev (nullable): the widest record as the
// structure pass found it on the device; wmax is then the launch shape (an
// upper bound of it, or a guess), the kernel takes the entries per lane from
// wmax_dev -- and if that is wider than the shape, does nothing but set
// *redo (device, required with wmax_dev) for the caller to launch again.
constexpr uint64_t kTxlLanesMaxEntries = 1024;
hipError_t launch_txlog_lanes(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                              const uint64_t *rec_off, const uint64_t *alh_off,
                              const uint64_t *leaf_off, const int32_t *pre, MhTxHeader *hdrs,
                              uint8_t *eh_out, uint8_t *alh_out, int32_t *status,
                              const TxlogHostOut &ho, uint64_t wmax, uint64_t log_len,
                              const uint64_t *wmax_dev = nullptr, uint64_t *redo = nullptr);
// The device structure pass over tx-log records (txlog_struct.hip), one lane
// per record, every check of the host hop (tx.go:419-588) on the device bytes:
//  * clog != null (mh_txlog_validate_clog): record t at the offset of cLog
//    entry t (BE64 offset || BE32 size [|| Alh], clog_es = 12 or 44 bytes,
//    immustore.go:122-123, 2569-2597); writes rec_off / alh_off / leaf_off
//    (leaf_off[t] = t's entry count, not a prefix);
//  * clog == null (mh_txlog_validate_resident): rec_off / alh_off / leaf_off
//    (prefix) from the host hop; the device bytes must parse to the same
//    structure, else the record is MH_ERR_CORRUPTED_DATA.
// pre[t]: the record's status (0, or the reader's error), kTxlNeedsHost for a
// record whose metadata is valid but not canonical or that is wider than the
// lanes kernel takes (the host re-validates those).  stats (device, zeroed by
// the caller): [0] widest accepted record, [1] records needing the host.
// lim (cLog mode, <= len): the bytes landed so far -- a record whose read runs
// past lim while lim < len needs the whole log and is left to the host
// (kTxlNeedsHost).
// Check mode: a record the device bytes give otherwise is MH_ERR_CORRUPTED_DATA.
constexpr int32_t kTxlNeedsHost = 0x40000000;
hipError_t launch_txlog_struct(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                               uint64_t len, uint64_t lim, const uint8_t *clog, uint32_t clog_es,
                               uint64_t *rec_off, uint64_t *alh_off, uint64_t *leaf_off,
                               uint32_t max_entries, uint32_t max_key_len, int32_t *pre,
                               uint64_t *stats);
// pre[t] = MH_ERR_CORRUPTED_DATA where a and b differ over record t's bytes
// [rec_off[t], alh_off[t] + 32), else MH_OK
hipError_t launch_txlog_bytes_cmp(hipStream_t st, uint64_t ntx, const uint8_t *a, const uint8_t *b,
                                  const uint64_t *rec_off, const uint64_t *alh_off, int32_t *pre);
// status[t] = pre[t] and the Alh zeroed where pre[t] != 0
hipError_t launch_txlog_apply_pre(hipStream_t st, uint64_t ntx, const int32_t *pre, int32_t *status,
                                  uint8_t *alh);
// stats[2] += the number of non-OK statuses, stats[3] = min(stats[3], the
// first non-OK record)
hipError_t launch_txlog_status_summary(hipStream_t st, uint64_t ntx, const int32_t *status,
                                       uint64_t *stats);
// up to three runs of words pinned host memory -> HBM by a kernel (k_fetch_host)
struct HostRuns {
    const uint64_t *src[3];
    uint64_t *dst[3];
    uint64_t n[3];
};
hipError_t launch_fetch_host(hipStream_t st, const HostRuns &r);
// up to three runs of 32-bit words HBM -> pinned host memory by a kernel (k_store_host)
struct HostWordRuns {
    const uint32_t *src[3];
    uint32_t *dst[3];
    uint64_t n[3];
};
hipError_t launch_store_host(hipStream_t st, const HostWordRuns &r);
hipError_t launch_txe_index(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                            const MhTxHeader *hdrs, const uint64_t *ent_start,
                            const uint64_t *leaf_off, uint64_t *rec_off, uint8_t *ver);
// entry digests (leaf = false) or their htree leaves, hashed in place from
// the raw tx-log entry records (k_txe_leaf)
hipError_t launch_txe_leaf(hipStream_t st, Timer *tm, uint64_t n, const uint8_t *buf,
                           const uint64_t *rec_off, const uint8_t *ver, bool leaf, uint8_t *out);
hipError_t launch_seg_level(hipStream_t st, Timer *tm, uint64_t nnodes, uint64_t level_base,
                            uint32_t nitems, const uint64_t *cur_base, const uint64_t *prev_base,
                            const uint64_t *prev_w, uint8_t *nodes);
// idx[p] == ~0 writes SHA256(nil) (the empty tree's root, htree.go:73-77)
hipError_t launch_gather32(hipStream_t st, uint64_t n, const uint8_t *src, const uint64_t *idx,
                           uint8_t *out);

// ---------------------------------------------------------------- proofs on the device
hipError_t launch_htree_proof(hipStream_t st, Timer *tm, const uint8_t *levels, uint64_t w,
                              uint64_t n, const uint64_t *leaf, uint8_t *terms, uint32_t max_terms,
                              uint32_t *nterms, int32_t *status);
hipError_t launch_ahtree_proof(hipStream_t st, Timer *tm, int kind, const uint8_t *dlog,
                               uint64_t size, uint64_t n, const uint64_t *i, const uint64_t *j,
                               uint8_t *terms, uint32_t max_terms, uint32_t *nterms,
                               int32_t *status);

// ---------------------------------------------------------------- wire formats (wire_kernels.hip)
// phase bit 1: sizes + status + off[0..n]; bit 2: write messages
uint64_t pb_scratch_bytes(uint64_t n);
// exclusive-offset scan: out[0] = 0, out[k+1] = sum in[0..k]; temp: pb_scan_temp_bytes(n)
size_t pb_scan_temp_bytes(uint64_t n);
hipError_t scan_offsets_u64(hipStream_t st, uint64_t n, const uint64_t *in, uint64_t *out,
                            uint8_t *temp);
hipError_t launch_pb_dual_v2(hipStream_t st, Timer *tm, int phase, const uint8_t *dlog,
                             uint64_t size, uint64_t n, const MhTxHeader *src,
                             const MhTxHeader *tgt, const uint8_t *md_blob, uint8_t *out,
                             uint64_t out_cap, uint64_t *off, int32_t *status, uint8_t *scratch);
hipError_t launch_pb_inclusion(hipStream_t st, Timer *tm, int phase, const uint8_t *levels,
                               uint64_t w, uint64_t n, const uint64_t *leaf, uint8_t *out,
                               uint64_t out_cap, uint64_t *off, int32_t *status, uint8_t *scratch);
}  // namespace mh
