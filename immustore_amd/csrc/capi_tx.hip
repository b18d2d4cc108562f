// capi_tx.hip -- C ABI of the transaction layer (include/immustore_merkle.h,
// "tx layer" section): header Alh (a7), linear and dual proofs (a13), tx-log
// read-path validation (a14) and many-tree htree builds (a3 over many txs).
//
// Host code here parses records, lays out device buffers and combines
// per-proof verdicts; every SHA-256 runs in tx_kernels.hip / verify_kernels.hip
// / htree_kernels.hip.
#include <cstring>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>

#include <atomic>
#include <chrono>
#include <cstdio>

#include "capi_internal.hpp"

namespace {

uint64_t be_at(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | p[i];
    return v;
}

}  // namespace

// Leaves + levels + roots of a planned batch on `st`.  d_digests: E x 32 on
// the device; d_roots: ntrees x 32.  run_tree_plan uses the ctx's s_tree
// scratch, run_tree_plan_on the caller's.
int run_tree_plan(mh_ctx *c, hipStream_t st, const TreePlan &P, uint64_t ntrees, uint64_t nleaves,
                  const uint8_t *d_digests, uint8_t *d_roots) {
    return run_tree_plan_on(c->s_tree, st, c->tm(), P, ntrees, nleaves, d_digests, d_roots, nullptr);
}

int run_tree_plan_on(DevBuf &scratch, hipStream_t st, Timer *tm, const TreePlan &P, uint64_t ntrees,
                     uint64_t nleaves, const uint8_t *d_digests, uint8_t *d_roots, uint8_t *pinned) {
    Layout L;
    const uint64_t nitems = P.cur.size();
    const uint64_t b_nodes = L.add(std::max<uint64_t>(P.total_nodes, 1) * 32);
    const uint64_t b_cur = L.add(nitems * 8), b_prev = L.add(nitems * 8),
                   b_prevw = L.add(nitems * 8), b_root = L.add(ntrees * 8);
    MH_HIP(scratch.ensure(L.total));
    uint8_t *base = scratch.as<uint8_t>();
    uint8_t *nodes = base + b_nodes;
    // index arrays: straight from the plan's vectors, or through `pinned`
    // (plan_index_bytes(P, ntrees) bytes the caller keeps alive until `st`
    // has passed this point) so the copies stay asynchronous
    const uint64_t *src_cur = P.cur.data(), *src_prev = P.prev.data(),
                   *src_prevw = P.prevw.data(), *src_root = P.root_idx.data();
    if (pinned) {
        uint64_t *q = reinterpret_cast<uint64_t *>(pinned);
        memcpy(q, src_cur, nitems * 8);
        memcpy(q + nitems, src_prev, nitems * 8);
        memcpy(q + 2 * nitems, src_prevw, nitems * 8);
        memcpy(q + 3 * nitems, src_root, ntrees * 8);
        src_cur = q;
        src_prev = q + nitems;
        src_prevw = q + 2 * nitems;
        src_root = q + 3 * nitems;
    }
    if (nitems) {
        MH_HIP(hipMemcpyAsync(base + b_cur, src_cur, nitems * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_prev, src_prev, nitems * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_prevw, src_prevw, nitems * 8, hipMemcpyHostToDevice, st));
    }
    MH_HIP(hipMemcpyAsync(base + b_root, src_root, ntrees * 8, hipMemcpyHostToDevice, st));
    MH_HIP(launch_leaf_for(st, tm, nleaves, d_digests, nodes));  // htree.go:79-83
    for (const auto &lv : P.levels)
        MH_HIP(launch_seg_level(st, tm, lv.nodes, lv.base, (uint32_t)lv.nitems,
                                (const uint64_t *)(base + b_cur) + lv.item0,
                                (const uint64_t *)(base + b_prev) + lv.item0,
                                (const uint64_t *)(base + b_prevw) + lv.item0, nodes));
    MH_HIP(launch_gather32(st, ntrees, nodes, (const uint64_t *)(base + b_root), d_roots));
    return MH_OK;
}


// ------------------------------------------------------------------ a7
// innerHash / Alh of n checked headers (tx.go:249-319); c->mu held by the
// caller.  From pinned host memory the header copy is one DMA.
int tx_alh_core(mh_ctx *c, uint64_t n, const mh_tx_header *hdrs, const uint8_t *md_blob,
                uint64_t md_blob_len, uint8_t *inner_out, uint8_t *alh_out) {
    MH_HIP(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    Layout L;
    const uint64_t b_h = L.add(n * sizeof(mh_tx_header)), b_md = L.add(md_blob_len),
                   b_s = L.add(n * kTxInnerStride), b_in = L.add(n * 32), b_a = L.add(n * 32);
    MH_HIP(c->s_tx.ensure(L.total));
    uint8_t *base = c->s_tx.as<uint8_t>();
    MH_HIP(hipMemcpyAsync(base + b_h, hdrs, n * sizeof(mh_tx_header), hipMemcpyHostToDevice, st));
    if (md_blob && md_blob_len)
        MH_HIP(hipMemcpyAsync(base + b_md, md_blob, md_blob_len, hipMemcpyHostToDevice, st));
    MH_HIP(launch_tx_alh(st, c->tm(), n, (const MhTxHeader *)(base + b_h), base + b_md, nullptr,
                         base + b_s, nullptr, nullptr, base + b_in, base + b_a, nullptr));
    if (inner_out) MH_HIP(hipMemcpyAsync(inner_out, base + b_in, n * 32, hipMemcpyDeviceToHost, st));
    MH_HIP(hipMemcpyAsync(alh_out, base + b_a, n * 32, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    return MH_OK;
}

extern "C" int mh_tx_alh_batch(mh_ctx *c, uint64_t n, const mh_tx_header *hdrs,
                               const uint8_t *md_blob, uint64_t md_blob_len, uint8_t *inner_out,
                               uint8_t *alh_out) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!hdrs || !alh_out))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        for (uint64_t k = 0; k < n; k++)
            if (int e = check_header(hdrs[k], md_blob_len, md_blob != nullptr)) return e;
        std::lock_guard<std::mutex> lk(c->mu);
        return tx_alh_core(c, n, hdrs, md_blob, md_blob_len, inner_out, alh_out);
    });
}

extern "C" int mh_dev_tx_alh_batch(mh_ctx *c, uint64_t n, const mh_tx_header *hdrs,
                                   const uint8_t *md_blob, const uint8_t *eh, uint8_t *scratch,
                                   uint8_t *inner_out, uint8_t *alh_out) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!hdrs || !scratch || !alh_out))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        hipSetDevice(c->device);
        MH_HIP(launch_tx_alh(c->stream, c->tm(), n, hdrs, md_blob, eh, scratch, nullptr, nullptr,
                             inner_out, alh_out, nullptr));
        return MH_OK;
    });
}

// ------------------------------------------------------------------ a3 x many
// Roots of many htrees over device digests d_dig (leaf_off: host, ntrees + 1,
// rebased so leaf_off[0] is d_dig's first digest) into device d_roots, on st;
// scratch: two device buffers of the caller (the small-tree leaves + offsets).
int build_many_dev(mh_ctx *c, hipStream_t st, uint64_t ntrees, const uint64_t *leaf_off,
                   const uint8_t *d_dig, uint8_t *d_roots, DevBuf &s_lv, DevBuf &s_lo) {
    const uint64_t E = leaf_off[ntrees] - leaf_off[0];
    uint64_t wmax = 0;
    for (uint64_t t = 0; t < ntrees; t++) wmax = std::max(wmax, leaf_off[t + 1] - leaf_off[t]);
    if (small_roots_fit(ntrees, wmax)) {  // one lane (or wave) per tree, no host plan
        MH_HIP(s_lv.ensure(std::max<uint64_t>(E, 1) * 32));
        MH_HIP(s_lo.ensure((ntrees + 1) * 8));
        MH_HIP(hipMemcpyAsync(s_lo.p, leaf_off, (ntrees + 1) * 8, hipMemcpyHostToDevice, st));
        MH_HIP(launch_leaf_for(st, c->tm(), E, d_dig, s_lv.as<uint8_t>()));  // htree.go:79-83
        MH_HIP(launch_small_roots(st, c->tm(), ntrees, s_lo.as<uint64_t>(), s_lv.as<uint8_t>(),
                                  d_roots, wmax));
        // leaf_off is the caller's host memory: done with it before returning
        MH_HIP(hipStreamSynchronize(st));
    } else {
        TreePlan P;
        P.build(ntrees, leaf_off);
        if (int e = run_tree_plan(c, st, P, ntrees, E, d_dig, d_roots)) return e;
        MH_HIP(hipStreamSynchronize(st));  // the plan's host vectors go out of scope
    }
    return MH_OK;
}

extern "C" int mh_htree_build_many(mh_ctx *c, uint64_t ntrees, const uint64_t *leaf_off,
                                   const uint8_t *digests, uint8_t *roots) {
    return mh_guard([&]() -> int {
        if (!c || (ntrees && (!leaf_off || !roots))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!ntrees) return MH_OK;
        for (uint64_t t = 0; t < ntrees; t++)
            if (leaf_off[t + 1] < leaf_off[t]) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t E = leaf_off[ntrees] - leaf_off[0];
        if (E && !digests) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        hipSetDevice(c->device);
        hipStream_t st = c->stream;
        Layout L;
        const uint64_t b_d = L.add(std::max<uint64_t>(E, 1) * 32), b_r = L.add(ntrees * 32);
        MH_HIP(c->s_tx.ensure(L.total));
        uint8_t *base = c->s_tx.as<uint8_t>();
        if (E)
            MH_HIP(hipMemcpyAsync(base + b_d, digests + leaf_off[0] * 32, E * 32,
                                  hipMemcpyHostToDevice, st));
        if (int e = build_many_dev(c, st, ntrees, leaf_off, base + b_d, base + b_r, c->s_digests,
                                   c->s_offs))
            return e;
        MH_HIP(hipMemcpyAsync(roots, base + b_r, ntrees * 32, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}

// ------------------------------------------------------------------ a13
extern "C" int mh_verify_linear_proof_batch(mh_ctx *c, uint64_t n, const uint64_t *proof_src,
                                            const uint64_t *proof_tgt, const uint64_t *term_off,
                                            const uint8_t *terms, const uint64_t *src,
                                            const uint64_t *tgt, const uint8_t *src_alh,
                                            const uint8_t *tgt_alh, uint8_t *ok) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!proof_src || !proof_tgt || !term_off || !src || !tgt || !src_alh ||
                         !tgt_alh || !ok)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        if (!monotonic(term_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t nterms = term_off[n] - term_off[0];
        if (nterms && !terms) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        hipSetDevice(c->device);
        hipStream_t st = c->stream;
        std::vector<uint64_t> to(n + 1);
        for (uint64_t p = 0; p <= n; p++) to[p] = term_off[p] - term_off[0];
        Layout L;
        const uint64_t b_ps = L.add(n * 8), b_pt = L.add(n * 8), b_s = L.add(n * 8),
                       b_t = L.add(n * 8), b_off = L.add((n + 1) * 8), b_terms = L.add(nterms * 32),
                       b_sa = L.add(n * 32), b_ta = L.add(n * 32), b_ok = L.add(n);
        MH_HIP(c->s_tx.ensure(L.total));
        uint8_t *base = c->s_tx.as<uint8_t>();
        MH_HIP(hipMemcpyAsync(base + b_ps, proof_src, n * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_pt, proof_tgt, n * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_s, src, n * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_t, tgt, n * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_off, to.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
        if (nterms)
            MH_HIP(hipMemcpyAsync(base + b_terms, terms + term_off[0] * 32, nterms * 32,
                                  hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_sa, src_alh, n * 32, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_ta, tgt_alh, n * 32, hipMemcpyHostToDevice, st));
        MH_HIP(launch_linear_verify(st, c->tm(), n, (const uint64_t *)(base + b_ps),
                                    (const uint64_t *)(base + b_pt), (const uint64_t *)(base + b_s),
                                    (const uint64_t *)(base + b_t), (const uint64_t *)(base + b_off),
                                    base + b_terms, base + b_sa, base + b_ta, base + b_ok));
        MH_HIP(hipMemcpyAsync(ok, base + b_ok, n, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}

// VerifyDualProofV2 (verification.go:305-372) over n proofs whose arguments
// have been checked (offsets monotonic, term arrays present).  The host-built
// arrays are written straight into one pinned staging area laid out like
// their device copies and go up in ONE copy; the results come back the same
// way.  alh_checked: the caller has already matched both headers' Alh with
// src_alh / tgt_alh and rejected unhashable headers (the VerifyDocument batch,
// which hashes every header once) -- the Alh pass (:318-326) is skipped.
// c->mu held by the caller (c->p_stage, c->s_tx).
int dual_proof_v2_core(mh_ctx *c, uint64_t n, const mh_tx_header *sh, const mh_tx_header *th,
                       const uint8_t *md_blob, uint64_t md_blob_len, const uint64_t *incl_off,
                       const uint8_t *incl_terms, const uint64_t *cons_off,
                       const uint8_t *cons_terms, const uint64_t *src, const uint64_t *tgt,
                       const uint8_t *src_alh, const uint8_t *tgt_alh, int32_t *status,
                       bool alh_checked) {
    MH_HIP(hipSetDevice(c->device));
    const uint64_t ni = incl_off[n] - incl_off[0], nc = cons_off[n] - cons_off[0];
    const uint64_t nh = alh_checked ? 0 : 2 * n;  // headers hashed here
    // host-built inputs first (one contiguous upload), then device-only data
    Layout L;
    const uint64_t b_h = L.add(nh * sizeof(mh_tx_header)), b_x = L.add(2 * n * 32),
                   b_sbl = L.add(n * 32), b_tbl = L.add(n * 32), b_sel = L.add(n),
                   b_ii = L.add(n * 8), b_ij = L.add(n * 8), b_ci = L.add(n * 8),
                   b_io = L.add((n + 1) * 8), b_co = L.add((n + 1) * 8);
    const uint64_t up_bytes = L.total;
    const uint64_t b_st = L.add(2 * n * 4), b_oki = L.add(n), b_okc = L.add(n);  // results
    const uint64_t res0 = b_st, res_bytes = L.total - b_st;
    const uint64_t b_md = L.add(alh_checked ? 0 : md_blob_len), b_s = L.add(nh * kTxInnerStride),
                   b_leaf = L.add(n * 32), b_ca = L.add(n * 32), b_it = L.add(ni * 32),
                   b_ct = L.add(nc * 32);
    MH_HIP(c->p_stage.ensure(L.total));
    uint8_t *hp = c->p_stage.as<uint8_t>();
    mh_tx_header *hh = reinterpret_cast<mh_tx_header *>(hp + b_h);
    uint8_t *x = hp + b_x, *sbl = hp + b_sbl, *tbl = hp + b_tbl, *sel = hp + b_sel;
    uint64_t *ii = reinterpret_cast<uint64_t *>(hp + b_ii), *ij = reinterpret_cast<uint64_t *>(hp + b_ij),
             *ci = reinterpret_cast<uint64_t *>(hp + b_ci), *io = reinterpret_cast<uint64_t *>(hp + b_io),
             *co = reinterpret_cast<uint64_t *>(hp + b_co);
    for (uint64_t p = 0; p < n; p++) {
        if (!alh_checked) {
            hh[p] = sh[p];
            hh[n + p] = th[p];
            if (status[p] != MH_OK) {  // keep the kernel's reads inside md_blob; result unused
                hh[p].version = hh[n + p].version = 1;
                hh[p].md_len = hh[n + p].md_len = 0;
            }
        }
        memcpy(x + p * 32, src_alh + p * 32, 32);
        memcpy(x + (n + p) * 32, tgt_alh + p * 32, 32);
        ii[p] = src[p];  // verification.go:342-348
        ij[p] = th[p].bl_tx_id;
        sel[p] = src[p] == 1;  // :354-370
        ci[p] = src[p] == 1 ? src[p] : sh[p].bl_tx_id;
        memcpy(sbl + p * 32, sh[p].bl_root, 32);
        memcpy(tbl + p * 32, th[p].bl_root, 32);
    }
    for (uint64_t p = 0; p <= n; p++) {
        io[p] = incl_off[p] - incl_off[0];
        co[p] = cons_off[p] - cons_off[0];
    }
    MH_HIP(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    MH_HIP(c->s_tx.ensure(L.total));
    uint8_t *base = c->s_tx.as<uint8_t>();
    MH_HIP(hipMemcpyAsync(base, hp, up_bytes, hipMemcpyHostToDevice, st));
    if (ni) MH_HIP(hipMemcpyAsync(base + b_it, incl_terms + incl_off[0] * 32, ni * 32,
                                  hipMemcpyHostToDevice, st));
    if (nc) MH_HIP(hipMemcpyAsync(base + b_ct, cons_terms + cons_off[0] * 32, nc * 32,
                                  hipMemcpyHostToDevice, st));
    if (!alh_checked) {
        if (md_blob && md_blob_len)
            MH_HIP(hipMemcpyAsync(base + b_md, md_blob, md_blob_len, hipMemcpyHostToDevice, st));
        // Alh of both headers vs the given ones (verification.go:318-326)
        MH_HIP(launch_tx_alh(st, c->tm(), 2 * n, (const MhTxHeader *)(base + b_h), base + b_md,
                             nullptr, base + b_s, base + b_x, nullptr, nullptr, nullptr,
                             (int32_t *)(base + b_st)));
    } else {
        MH_HIP(hipMemsetAsync(base + b_st, 0, 2 * n * 4, st));  // every Alh matched (MH_OK)
    }
    // leafFor(sourceAlh) (verification.go:346), then the two ahtree proofs
    MH_HIP(launch_leaf_for(st, c->tm(), n, base + b_x, base + b_leaf));
    MH_HIP(launch_ahtree_verify(st, c->tm(), MH_AHT_INCLUSION, n, (const uint64_t *)(base + b_ii),
                                (const uint64_t *)(base + b_ij), (const uint64_t *)(base + b_io),
                                base + b_it, base + b_leaf, base + b_tbl, base + b_oki, nullptr));
    MH_HIP(launch_select32(st, n, base + b_sel, base + b_leaf, base + b_sbl, base + b_ca));
    MH_HIP(launch_ahtree_verify(st, c->tm(), MH_AHT_CONSISTENCY, n,
                                (const uint64_t *)(base + b_ci), (const uint64_t *)(base + b_ij),
                                (const uint64_t *)(base + b_co), base + b_ct, base + b_ca,
                                base + b_tbl, base + b_okc, nullptr));
    MH_HIP(hipMemcpyAsync(hp + res0, base + res0, res_bytes, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    const int32_t *ast = reinterpret_cast<const int32_t *>(hp + b_st);
    const uint8_t *oki = hp + b_oki, *okc = hp + b_okc;
    for (uint64_t p = 0; p < n; p++) {
        if (status[p] != MH_OK) continue;
        if (ast[p] != MH_OK || ast[n + p] != MH_OK) {
            status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
        } else if (sh[p].id - 1 != sh[p].bl_tx_id || th[p].id - 1 != th[p].bl_tx_id) {
            status[p] = MH_ERR_UNEXPECTED_LINKING;  // :328-330
        } else if (src[p] == tgt[p]) {
            status[p] = MH_OK;  // :332-334
        } else if (!oki[p]) {
            status[p] = MH_ERR_INCLUSION_NOT_VALID;
        } else if (!okc[p]) {
            status[p] = MH_ERR_CONSISTENCY_NOT_VALID;
        }
    }
    return MH_OK;
}

extern "C" int mh_verify_dual_proof_v2_batch(mh_ctx *c, uint64_t n, const mh_tx_header *sh,
                                             const mh_tx_header *th, const uint8_t *md_blob,
                                             uint64_t md_blob_len, const uint64_t *incl_off,
                                             const uint8_t *incl_terms, const uint64_t *cons_off,
                                             const uint8_t *cons_terms, const uint64_t *src,
                                             const uint64_t *tgt, const uint8_t *src_alh,
                                             const uint8_t *tgt_alh, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!sh || !th || !incl_off || !cons_off || !src || !tgt || !src_alh ||
                         !tgt_alh || !status)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        if (!monotonic(incl_off, n) || !monotonic(cons_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t ni = incl_off[n] - incl_off[0], nc = cons_off[n] - cons_off[0];
        if ((ni && !incl_terms) || (nc && !cons_terms)) return MH_ERR_ILLEGAL_ARGUMENTS;
        // verification.go:305-316: argument checks on the host, headers that
        // cannot be hashed (unknown version, bad md) fail as ErrIllegalArguments
        for (uint64_t p = 0; p < n; p++) {
            int32_t s = MH_OK;
            if (sh[p].id == 0 || sh[p].id != src[p] || th[p].id != tgt[p])
                s = MH_ERR_ILLEGAL_ARGUMENTS;
            else if (src[p] > tgt[p])
                s = MH_ERR_SOURCE_TX_NEWER;
            else if (check_header(sh[p], md_blob_len, md_blob != nullptr) ||
                     check_header(th[p], md_blob_len, md_blob != nullptr))
                s = MH_ERR_ILLEGAL_ARGUMENTS;
            status[p] = s;
        }
        std::lock_guard<std::mutex> lk(c->mu);
        return dual_proof_v2_core(c, n, sh, th, md_blob, md_blob_len, incl_off, incl_terms,
                                  cons_off, cons_terms, src, tgt, src_alh, tgt_alh, status, false);
    });
}

extern "C" int mh_verify_dual_proof_batch(mh_ctx *c, const mh_dual_proof_batch *B, uint8_t *ok) {
    return mh_guard([&]() -> int {
        if (!c || !B || (B->n && !ok)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t n = B->n;
        if (!n) return MH_OK;
        if (!B->src_hdr || !B->tgt_hdr || !B->incl_off || !B->cons_off || !B->target_bl_tx_alh ||
            !B->last_off || !B->has_linear || !B->linear_src || !B->linear_tgt || !B->linear_off ||
            !B->has_advance || !B->advance_off || !B->advance_incl_first || !B->advance_incl_off ||
            !B->src || !B->tgt || !B->src_alh || !B->tgt_alh)
            return MH_ERR_ILLEGAL_ARGUMENTS;
        const mh_tx_header *sh = B->src_hdr, *th = B->tgt_hdr;
        if (!monotonic(B->incl_off, n) || !monotonic(B->cons_off, n) ||
            !monotonic(B->last_off, n) || !monotonic(B->linear_off, n) ||
            !monotonic(B->advance_off, n) || !monotonic(B->advance_incl_first, n))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t ni = B->incl_off[n] - B->incl_off[0], nc = B->cons_off[n] - B->cons_off[0],
                       nl = B->last_off[n] - B->last_off[0], nlin = B->linear_off[n] - B->linear_off[0],
                       nadv = B->advance_off[n] - B->advance_off[0],
                       Q = B->advance_incl_first[n] - B->advance_incl_first[0],
                       nq = Q ? B->advance_incl_off[B->advance_incl_first[n]] -
                                    B->advance_incl_off[B->advance_incl_first[0]]
                              : 0;
        if ((ni && !B->incl_terms) || (nc && !B->cons_terms) || (nl && !B->last_terms) ||
            (nlin && !B->linear_terms) || (nadv && !B->advance_terms) ||
            (nq && !B->advance_incl_terms))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t q0 = B->advance_incl_first[0], qt0 = Q ? B->advance_incl_off[q0] : 0;

        // ---- host side: argument checks and per-check operands (verification.go:128-235)
        std::vector<uint8_t> alive(n, 1), adv_state(n, 0);  // 0 run chain, 1 true, 2 false
        std::vector<mh_tx_header> hh(2 * n);
        std::vector<uint8_t> expect(2 * n * 32), lin_sa(n * 32), end_alh(n * 32), sbl(n * 32),
            tbl(n * 32);
        std::vector<uint64_t> ii(n), ij(n), ci(n), li(n), ls(n), lt(n), lo(n + 1), io(n + 1),
            co(n + 1), lso(n + 1);
        std::vector<uint64_t> a_start, a_cnt, a_t0, a_first, a_idx;
        std::vector<uint8_t> a_end;
        for (uint64_t p = 0; p <= n; p++) {
            io[p] = B->incl_off[p] - B->incl_off[0];
            co[p] = B->cons_off[p] - B->cons_off[0];
            lso[p] = B->last_off[p] - B->last_off[0];
            lo[p] = B->linear_off[p] - B->linear_off[0];
        }
        for (uint64_t p = 0; p < n; p++) {
            const uint64_t src = B->src[p], tgt = B->tgt[p];
            if (sh[p].id != src || th[p].id != tgt || sh[p].id == 0 || sh[p].id > th[p].id ||
                check_header(sh[p], B->md_blob_len, B->md_blob != nullptr) ||
                check_header(th[p], B->md_blob_len, B->md_blob != nullptr))
                alive[p] = 0;
            hh[p] = sh[p];
            hh[n + p] = th[p];
            if (!alive[p]) {
                hh[p].version = hh[n + p].version = 1;
                hh[p].md_len = hh[n + p].md_len = 0;
            }
            memcpy(&expect[p * 32], B->src_alh + p * 32, 32);
            memcpy(&expect[(n + p) * 32], B->tgt_alh + p * 32, 32);
            memcpy(&sbl[p * 32], sh[p].bl_root, 32);
            memcpy(&tbl[p * 32], th[p].bl_root, 32);
            const uint64_t tbl_id = th[p].bl_tx_id;
            ii[p] = src;
            ij[p] = tbl_id;
            ci[p] = sh[p].bl_tx_id;
            li[p] = tbl_id;
            const bool a_branch = src < tbl_id;  // verification.go:195 vs :214
            ls[p] = a_branch ? tbl_id : src;
            lt[p] = tgt;
            memcpy(&lin_sa[p * 32], a_branch ? B->target_bl_tx_alh + p * 32 : B->src_alh + p * 32, 32);
            const uint64_t start = sh[p].bl_tx_id, end = a_branch ? src : tbl_id;
            memcpy(&end_alh[p * 32], a_branch ? B->src_alh + p * 32 : B->target_bl_tx_alh + p * 32, 32);
            // VerifyLinearAdvanceProof preconditions (verification.go:90-104)
            const uint64_t f0 = B->advance_incl_first[p], f1 = B->advance_incl_first[p + 1];
            if (end < start) {
                adv_state[p] = 2;
            } else if (end <= start + 1) {
                adv_state[p] = 1;
            } else if (!B->has_advance[p] ||
                       B->advance_off[p + 1] - B->advance_off[p] != end - start ||
                       f1 - f0 != end - start - 1) {
                adv_state[p] = 2;
            } else {
                adv_state[p] = 0;
                a_idx.push_back(p);
                a_start.push_back(start);
                a_cnt.push_back(end - start - 1);
                a_t0.push_back(B->advance_off[p] - B->advance_off[0]);
                a_first.push_back(f0 - q0);
                a_end.insert(a_end.end(), &end_alh[p * 32], &end_alh[p * 32] + 32);
            }
        }
        // nested inclusion proofs (every q; those of proofs not run are ignored)
        std::vector<uint64_t> qi(std::max<uint64_t>(Q, 1)), qj(std::max<uint64_t>(Q, 1)),
            qo(Q + 1);
        std::vector<uint8_t> qroot(std::max<uint64_t>(Q, 1) * 32);
        for (uint64_t q = 0; q <= Q; q++) qo[q] = B->advance_incl_off[q0 + q] - qt0;
        for (uint64_t k = 0; k < a_idx.size(); k++) {
            const uint64_t p = a_idx[k];
            for (uint64_t x = 0; x < a_cnt[k]; x++) {
                const uint64_t q = a_first[k] + x;
                qi[q] = a_start[k] + 1 + x;  // txID, verification.go:108-114
                qj[q] = th[p].bl_tx_id;
                memcpy(&qroot[q * 32], th[p].bl_root, 32);
            }
        }
        const uint64_t na = a_idx.size();

        std::lock_guard<std::mutex> lk(c->mu);
        hipSetDevice(c->device);
        hipStream_t st = c->stream;
        Layout L;
        const uint64_t b_h = L.add(2 * n * sizeof(mh_tx_header)), b_md = L.add(B->md_blob_len),
                       b_s = L.add(2 * n * kTxInnerStride), b_x = L.add(2 * n * 32),
                       b_ast = L.add(2 * n * 4), b_tba = L.add(n * 32), b_lfa = L.add(n * 32),
                       b_lft = L.add(n * 32), b_sbl = L.add(n * 32), b_tbl = L.add(n * 32),
                       b_ii = L.add(n * 8), b_ij = L.add(n * 8), b_ci = L.add(n * 8),
                       b_li = L.add(n * 8), b_io = L.add((n + 1) * 8), b_co = L.add((n + 1) * 8),
                       b_lso = L.add((n + 1) * 8), b_it = L.add(ni * 32), b_ct = L.add(nc * 32),
                       b_lt = L.add(nl * 32), b_oki = L.add(n), b_okc = L.add(n), b_okl = L.add(n),
                       b_ps = L.add(n * 8), b_pt = L.add(n * 8), b_ls = L.add(n * 8),
                       b_ltg = L.add(n * 8), b_lo = L.add((n + 1) * 8), b_lterm = L.add(nlin * 32),
                       b_lsa = L.add(n * 32), b_ta = L.add(n * 32), b_oklin = L.add(n),
                       b_ast0 = L.add(na * 8), b_acnt = L.add(na * 8), b_at0 = L.add(na * 8),
                       b_afirst = L.add(na * 8), b_aend = L.add(na * 32), b_aterm = L.add(nadv * 32),
                       b_aok = L.add(na), b_qsrc = L.add(Q * 32), b_qleaf = L.add(Q * 32),
                       b_qi = L.add(Q * 8), b_qj = L.add(Q * 8), b_qo = L.add((Q + 1) * 8),
                       b_qroot = L.add(Q * 32), b_qterm = L.add(nq * 32), b_qok = L.add(Q);
        MH_HIP(c->s_tx.ensure(L.total));
        uint8_t *base = c->s_tx.as<uint8_t>();
        auto h2d = [&](uint64_t off, const void *p, uint64_t bytes) -> hipError_t {
            return bytes ? hipMemcpyAsync(base + off, p, bytes, hipMemcpyHostToDevice, st)
                         : hipSuccess;
        };
        auto U = [&](uint64_t off) { return (const uint64_t *)(base + off); };
        MH_HIP(h2d(b_h, hh.data(), 2 * n * sizeof(mh_tx_header)));
        if (B->md_blob) MH_HIP(h2d(b_md, B->md_blob, B->md_blob_len));
        MH_HIP(h2d(b_x, expect.data(), 2 * n * 32));
        MH_HIP(h2d(b_tba, B->target_bl_tx_alh, n * 32));
        MH_HIP(h2d(b_sbl, sbl.data(), n * 32));
        MH_HIP(h2d(b_tbl, tbl.data(), n * 32));
        MH_HIP(h2d(b_ii, ii.data(), n * 8));
        MH_HIP(h2d(b_ij, ij.data(), n * 8));
        MH_HIP(h2d(b_ci, ci.data(), n * 8));
        MH_HIP(h2d(b_li, li.data(), n * 8));
        MH_HIP(h2d(b_io, io.data(), (n + 1) * 8));
        MH_HIP(h2d(b_co, co.data(), (n + 1) * 8));
        MH_HIP(h2d(b_lso, lso.data(), (n + 1) * 8));
        MH_HIP(h2d(b_it, ni ? B->incl_terms + B->incl_off[0] * 32 : nullptr, ni * 32));
        MH_HIP(h2d(b_ct, nc ? B->cons_terms + B->cons_off[0] * 32 : nullptr, nc * 32));
        MH_HIP(h2d(b_lt, nl ? B->last_terms + B->last_off[0] * 32 : nullptr, nl * 32));
        MH_HIP(h2d(b_ps, B->linear_src, n * 8));
        MH_HIP(h2d(b_pt, B->linear_tgt, n * 8));
        MH_HIP(h2d(b_ls, ls.data(), n * 8));
        MH_HIP(h2d(b_ltg, lt.data(), n * 8));
        MH_HIP(h2d(b_lo, lo.data(), (n + 1) * 8));
        MH_HIP(h2d(b_lterm, nlin ? B->linear_terms + B->linear_off[0] * 32 : nullptr, nlin * 32));
        MH_HIP(h2d(b_lsa, lin_sa.data(), n * 32));
        MH_HIP(h2d(b_ta, B->tgt_alh, n * 32));
        MH_HIP(h2d(b_ast0, a_start.data(), na * 8));
        MH_HIP(h2d(b_acnt, a_cnt.data(), na * 8));
        MH_HIP(h2d(b_at0, a_t0.data(), na * 8));
        MH_HIP(h2d(b_afirst, a_first.data(), na * 8));
        MH_HIP(h2d(b_aend, a_end.data(), na * 32));
        MH_HIP(h2d(b_aterm, nadv ? B->advance_terms + B->advance_off[0] * 32 : nullptr, nadv * 32));
        MH_HIP(h2d(b_qi, qi.data(), Q * 8));
        MH_HIP(h2d(b_qj, qj.data(), Q * 8));
        MH_HIP(h2d(b_qo, qo.data(), (Q + 1) * 8));
        MH_HIP(h2d(b_qroot, qroot.data(), Q * 32));
        MH_HIP(h2d(b_qterm, nq ? B->advance_incl_terms + qt0 * 32 : nullptr, nq * 32));
        Timer *tm = c->tm();
        // header Alh (verification.go:141-150)
        MH_HIP(launch_tx_alh(st, tm, 2 * n, (const MhTxHeader *)(base + b_h), base + b_md, nullptr,
                             base + b_s, base + b_x, nullptr, nullptr, nullptr,
                             (int32_t *)(base + b_ast)));
        // inclusion / consistency / last inclusion (verification.go:152-190)
        MH_HIP(launch_leaf_for(st, tm, n, base + b_x, base + b_lfa));
        MH_HIP(launch_leaf_for(st, tm, n, base + b_tba, base + b_lft));
        MH_HIP(launch_ahtree_verify(st, tm, MH_AHT_INCLUSION, n, U(b_ii), U(b_ij), U(b_io),
                                    base + b_it, base + b_lfa, base + b_tbl, base + b_oki, nullptr));
        MH_HIP(launch_ahtree_verify(st, tm, MH_AHT_CONSISTENCY, n, U(b_ci), U(b_ij), U(b_co),
                                    base + b_ct, base + b_sbl, base + b_tbl, base + b_okc, nullptr));
        MH_HIP(launch_ahtree_verify(st, tm, MH_AHT_LAST_INCLUSION, n, U(b_li), U(b_li), U(b_lso),
                                    base + b_lt, base + b_lft, base + b_tbl, base + b_okl, nullptr));
        // linear proof (verification.go:195-197 / :214-216)
        MH_HIP(launch_linear_verify(st, tm, n, U(b_ps), U(b_pt), U(b_ls), U(b_ltg), U(b_lo),
                                    base + b_lterm, base + b_lsa, base + b_ta, base + b_oklin));
        // linear advance proofs: chain, then the nested inclusion proofs
        MH_HIP(launch_advance_chain(st, tm, na, U(b_ast0), U(b_acnt), U(b_at0), base + b_aterm,
                                    U(b_afirst), base + b_aend, base + b_qsrc, base + b_aok));
        MH_HIP(launch_leaf_for(st, tm, Q, base + b_qsrc, base + b_qleaf));
        MH_HIP(launch_ahtree_verify(st, tm, MH_AHT_INCLUSION, Q, U(b_qi), U(b_qj), U(b_qo),
                                    base + b_qterm, base + b_qleaf, base + b_qroot, base + b_qok,
                                    nullptr));
        std::vector<int32_t> ast(2 * n);
        std::vector<uint8_t> oki(n), okc(n), okl(n), oklin(n), aok(std::max<uint64_t>(na, 1)),
            qok(std::max<uint64_t>(Q, 1));
        auto d2h = [&](void *dst, uint64_t off, uint64_t bytes) -> hipError_t {
            return bytes ? hipMemcpyAsync(dst, base + off, bytes, hipMemcpyDeviceToHost, st)
                         : hipSuccess;
        };
        MH_HIP(d2h(ast.data(), b_ast, 2 * n * 4));
        MH_HIP(d2h(oki.data(), b_oki, n));
        MH_HIP(d2h(okc.data(), b_okc, n));
        MH_HIP(d2h(okl.data(), b_okl, n));
        MH_HIP(d2h(oklin.data(), b_oklin, n));
        MH_HIP(d2h(aok.data(), b_aok, na));
        MH_HIP(d2h(qok.data(), b_qok, Q));
        MH_HIP(hipStreamSynchronize(st));
        std::vector<uint8_t> adv_ok(n, 0);
        for (uint64_t k = 0; k < na; k++) {
            bool all = aok[k] != 0;
            for (uint64_t x = 0; x < a_cnt[k] && all; x++) all = qok[a_first[k] + x] != 0;
            adv_ok[a_idx[k]] = all;
        }
        for (uint64_t p = 0; p < n; p++) {
            const uint64_t src = B->src[p], tbl_id = th[p].bl_tx_id;
            bool r = alive[p] && ast[p] == MH_OK && ast[n + p] == MH_OK;
            if (r && src < tbl_id) r = oki[p];
            if (r && sh[p].bl_tx_id > 0) r = okc[p];
            if (r && tbl_id > 0) r = okl[p];
            if (r) r = B->has_linear[p] && oklin[p];
            if (r) r = adv_state[p] == 1 || (adv_state[p] == 0 && adv_ok[p]);
            ok[p] = r ? 1 : 0;
        }
        return MH_OK;
    });
}

// ------------------------------------------------------------------ a14
namespace {

inline uint64_t be16p(const uint8_t *q) { return (uint64_t)((uint32_t)q[0] << 8 | q[1]); }

// KVMetadata.unsafeReadFrom + Bytes() (kv_metadata.go:207-256): deleted(0),
// expiresAt(1, 8 bytes), nonIndexable(2); unknown codes and a short expiresAt
// are ErrCorruptedData; a repeated attribute replaces the earlier one; Bytes()
// writes the attributes in code order.
int kv_md_canonical(const uint8_t *md, uint64_t ml, uint8_t out[MH_MAX_KV_METADATA_LEN],
                    uint64_t *ol) {
    if (ml > MH_MAX_KV_METADATA_LEN) return MH_ERR_CORRUPTED_DATA;
    bool has[3] = {false, false, false};
    const uint8_t *exp = nullptr;
    for (uint64_t i = 0; i < ml;) {
        const uint8_t code = md[i++];
        if (code == 1) {
            if (ml - i < 8) return MH_ERR_CORRUPTED_DATA;
            exp = md + i;
            i += 8;
        } else if (code > 2) {
            return MH_ERR_CORRUPTED_DATA;
        }
        has[code] = true;
    }
    uint64_t o = 0;
    if (has[0]) out[o++] = 0;
    if (has[1]) {
        out[o++] = 1;
        memcpy(out + o, exp, 8);
        o += 8;
    }
    if (has[2]) out[o++] = 2;
    *ol = o;
    return MH_OK;
}

// TxMetadata.ReadFrom + Bytes() (tx_metadata.go:145-193): truncatedUptoTx(0,
// 8 bytes), extra(1, BE16 length + up to 256 bytes).  An extra running past
// the metadata (Go indexes past the slice) or longer than 256 bytes (Bytes()
// slices past its array) panics in Go: corrupted data here.
int tx_md_canonical(const uint8_t *md, uint64_t ml, uint8_t out[MH_MAX_TX_METADATA_LEN],
                    uint64_t *ol) {
    if (ml > MH_MAX_TX_METADATA_LEN) return MH_ERR_CORRUPTED_DATA;
    const uint8_t *trunc = nullptr, *extra = nullptr;
    uint64_t el = 0;
    for (uint64_t i = 0; i < ml;) {
        const uint8_t code = md[i++];
        if (code == 0) {
            if (ml - i < 8) return MH_ERR_CORRUPTED_DATA;
            trunc = md + i;
            i += 8;
        } else if (code == 1) {
            if (ml - i < 2) return MH_ERR_CORRUPTED_DATA;
            el = be16p(md + i);
            i += 2;
            if (ml - i < el || el > 256) return MH_ERR_CORRUPTED_DATA;
            extra = md + i;
            i += el;
        } else {
            return MH_ERR_CORRUPTED_DATA;
        }
    }
    uint64_t o = 0;
    if (trunc) {
        out[o++] = 0;
        memcpy(out + o, trunc, 8);
        o += 8;
    }
    if (extra) {
        out[o++] = 1;
        out[o++] = (uint8_t)(el >> 8);
        out[o++] = (uint8_t)el;
        memcpy(out + o, extra, el);
        o += el;
    }
    *ol = o;
    return MH_OK;
}

// Parse the record at p.  Returns MH_OK and fills h / first / alh, or
// the structural error; *eof for an id-0 tail or a buffer too short for an id.
// Checks follow the reader's order (tx.go:419-588): lengths are read before
// the metadata they announce is parsed.  patches (may be null): where to note
// non-canonical metadata of this record (index rec).
int hop_record(const uint8_t *buf, uint64_t len, uint64_t p, const HopLimits &lim,
               mh_tx_header &h, uint64_t &first, uint64_t &alh, bool &eof,
               std::vector<HopPatch> *patches = nullptr, uint64_t rec = 0) {
    eof = false;
    if (p + 8 > len) { eof = true; return MH_OK; }
    memset(&h, 0, sizeof h);
    h.id = be_at(buf + p, 8);
    if (h.id == 0) { eof = true; return MH_OK; }  // preallocated tail, read as EOF (tx.go:427-430)
    if (p + 90 > len) return MH_ERR_TRUNCATED;
    h.ts = (int64_t)be_at(buf + p + 8, 8);
    h.bl_tx_id = be_at(buf + p + 16, 8);
    memcpy(h.bl_root, buf + p + 24, 32);
    memcpy(h.prev_alh, buf + p + 56, 32);
    h.version = (uint32_t)be16p(buf + p + 88);
    uint64_t q = p + 90;
    uint8_t canon[MH_MAX_TX_METADATA_LEN];
    if (h.version == 0) {
        if (q + 2 > len) return MH_ERR_TRUNCATED;
        h.nentries = (uint32_t)be16p(buf + q);
        q += 2;
    } else if (h.version == 1) {
        if (q + 2 > len) return MH_ERR_TRUNCATED;
        h.md_len = (uint32_t)be16p(buf + q);
        q += 2;
        if (h.md_len > MH_MAX_TX_METADATA_LEN) return MH_ERR_CORRUPTED_DATA;
        if (q + h.md_len > len) return MH_ERR_TRUNCATED;
        uint64_t cl = 0;
        if (tx_md_canonical(buf + q, h.md_len, canon, &cl)) return MH_ERR_CORRUPTED_DATA;
        if (patches && (cl != h.md_len || memcmp(canon, buf + q, cl)))
            patches->push_back(HopPatch{rec, 1, 0, std::vector<uint8_t>(canon, canon + cl)});
        if (q + h.md_len + 4 > len) return MH_ERR_TRUNCATED;
        if (q > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;
        h.md_off = (uint32_t)q;
        q += h.md_len;
        h.nentries = (uint32_t)be_at(buf + q, 4);
        q += 4;
    } else {
        return MH_ERR_CORRUPTED_UNKNOWN_VERSION;
    }
    if (h.nentries > lim.max_entries) return MH_ERR_CORRUPTED_MAX_ENTRIES;
    first = q;
    for (uint32_t e = 0; e < h.nentries; e++) {
        if (q + 2 > len) return MH_ERR_TRUNCATED;
        const uint64_t ml = be16p(buf + q);
        if (q + 2 + ml > len) return MH_ERR_TRUNCATED;
        uint64_t cml = 0;
        if (ml && kv_md_canonical(buf + q + 2, ml, canon, &cml)) return MH_ERR_CORRUPTED_DATA;
        if (q + 2 + ml + 2 > len) return MH_ERR_TRUNCATED;
        const uint64_t kl = be16p(buf + q + 2 + ml);
        if (kl > lim.max_key_len) return MH_ERR_CORRUPTED_MAX_KEYLEN;
        if (q + 4 + ml + kl + 12 + 32 > len) return MH_ERR_TRUNCATED;
        // a v0 header cannot carry KV metadata: TxEntryDigest_v1_1 fails the
        // read with ErrMetadataUnsupported (tx.go:690-693, via readEntry)
        if (h.version == 0 && ml > 0) return MH_ERR_METADATA_UNSUPPORTED;
        if (patches && ml && (cml != ml || memcmp(canon, buf + q + 2, cml))) {
            // the entry record re-serialised with canonical metadata
            std::vector<uint8_t> r(4 + cml + kl + 12 + 32);
            r[0] = (uint8_t)(cml >> 8);
            r[1] = (uint8_t)cml;
            memcpy(r.data() + 2, canon, cml);
            memcpy(r.data() + 2 + cml, buf + q + 2 + ml, 2 + kl + 12 + 32);
            patches->push_back(HopPatch{rec, 0, e, std::move(r)});
        }
        q += 4 + ml + kl + 12 + 32;
    }
    if (q + 32 > len) return MH_ERR_TRUNCATED;
    alh = q;
    return MH_OK;
}

// Records starting in [p, stop), at most max_recs of them.
void hop_range(const uint8_t *buf, uint64_t len, uint64_t p, uint64_t stop, uint64_t max_recs,
               const HopLimits &lim, HopOut &o) {
    o.start = p;
    while (p < stop && o.R.size() < max_recs) {
        mh_tx_header h;
        uint64_t first = 0, alh = 0;
        bool eof = false;
        const size_t np = o.P.size();
        const int rc = hop_record(buf, len, p, lim, h, first, alh, eof, &o.P, o.R.size());
        if (rc != MH_OK || eof) {
            o.P.resize(np);  // patches of a record that did not parse
            o.rc = rc;
            o.stopped = true;
            break;
        }
        o.R.push_back(HopRec{p, alh, h.nentries, 0});
        if (o.want_headers) o.H.push_back(h);
        p = alh + 32;
    }
    o.end = p;
}

// A position that parses as 3 consecutive records with consecutive ids (or
// as records up to the end of the log or a zero tail): where a chunk's speculative parse
// starts.  Only a guess -- the merge accepts a chunk only if the previous
// chunk's parse ended exactly there.
bool zero_run(const uint8_t *buf, uint64_t len, uint64_t p, uint64_t n) {
    const uint64_t e = std::min(len, p + n);
    for (uint64_t k = p; k < e; k++)
        if (buf[k]) return false;
    return true;
}

uint64_t find_record_start(const uint8_t *buf, uint64_t len, uint64_t from, uint64_t to,
                           const HopLimits &lim0) {
    // bounded speculation: a 256 KiB window and candidate records of at most
    // 4096 entries (a miss only costs a sequential re-parse of the chunk)
    const HopLimits lim{std::min<uint32_t>(lim0.max_entries, 4096), lim0.max_key_len};
    to = std::min<uint64_t>(to, from + (256u << 10));
    for (uint64_t q = from; q < to; q++) {
        uint64_t p = q, prev_id = 0;
        int ok = 0;
        for (; ok < 3; ok++) {
            mh_tx_header h;
            uint64_t first, alh;
            bool eof;
            if (hop_record(buf, len, p, lim, h, first, alh, eof) != MH_OK) break;
            if (eof) {
                // the end of the log, or a zero-filled preallocated tail after at
                // least one record -- not 8 zero bytes inside a record (a zero
                // vOff field read as an id-0 "tail")
                if (p + 8 <= len && (ok == 0 || !zero_run(buf, len, p, 256))) break;
                ok = 3;
                break;
            }
            if (ok && h.id != prev_id + 1) break;
            prev_id = h.id;
            p = alh + 32;
        }
        if (ok >= 3) return q;
    }
    return ~0ull;
}

// Parked helper threads for the hop (started on first use, kept for the life
// of the process: a validation call runs the hop twice, and starting 15
// threads each time cost about as much as the hop over a quarter of the log).
// run(T, fn) calls fn(k) for k in [0, T): the caller takes tasks too, so a
// pool that could not start threads still finishes.  One run at a time; a
// concurrent caller (another context's hop) gets busy() and starts its own
// threads instead.
class HopPool {
  public:
    static HopPool &get() {
        static HopPool *p = new HopPool();  // never destroyed: its threads stay parked
        return *p;
    }
    bool try_run(unsigned T, const std::function<void(unsigned)> &fn) {
        std::unique_lock<std::mutex> call(call_mu, std::try_to_lock);
        if (!call.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> lk(mu);
            try {
                while (th.size() + 1 < T) {
                    th.emplace_back([this] { loop(); });
                    th.back().detach();
                }
            } catch (...) {  // fewer threads: the caller takes more tasks
            }
            job = &fn;
            next = 0;
            total = T;
            finished = 0;
            failed = false;
        }
        cv_go.notify_all();
        take();
        std::unique_lock<std::mutex> lk(mu);
        cv_done.wait(lk, [&] { return finished == total; });
        job = nullptr;
        if (failed) throw std::bad_alloc();
        return true;
    }

  private:
    std::mutex call_mu, mu;
    std::condition_variable cv_go, cv_done;
    std::vector<std::thread> th;
    const std::function<void(unsigned)> *job = nullptr;
    unsigned next = 0, total = 0, finished = 0;
    bool failed = false;
    // take tasks until none are left (caller and helpers alike)
    void take() {
        std::unique_lock<std::mutex> lk(mu);
        while (job && next < total) {
            const unsigned k = next++;
            const std::function<void(unsigned)> *f = job;
            lk.unlock();
            bool ok = true;
            try {
                (*f)(k);
            } catch (...) {
                ok = false;
            }
            lk.lock();
            failed |= !ok;
            if (++finished == total) cv_done.notify_all();
        }
    }
    void loop() {
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_go.wait(lk, [&] { return job && next < total; });
            }
            take();
        }
    }
};

// The whole hop: one thread below 1 MiB, else up to 16 threads parse chunks
// from speculated record starts; chunks whose start does not match the
// previous chunk's end are re-parsed sequentially, so the result is always
// the sequential parse's.
void hop_all(const uint8_t *buf, uint64_t len, uint64_t max_txs, const HopLimits &lim,
             HopOut &out, bool want_headers) {
    out.want_headers = want_headers;
    // threads: MH_HOP_THREADS from the environment (read once), default 16,
    // never more than the machine has
    static const unsigned kHopThreads = [] {
        const char *e = getenv("MH_HOP_THREADS");
        const long v = e ? strtol(e, nullptr, 10) : 16;
        return (unsigned)std::min(64l, std::max(1l, v));
    }();
    unsigned T = std::min(kHopThreads, std::max(1u, std::thread::hardware_concurrency()));
    // at least 512 KiB per thread (the threads are parked, not started per
    // call: a validation call hops each copy chunk separately, the smallest a
    // few MiB)
    T = (unsigned)std::min<uint64_t>(T, std::max<uint64_t>(1, len >> 19));
    if (T == 1) {
        hop_range(buf, len, 0, ~0ull, max_txs, lim, out);
        return;
    }
    std::vector<uint64_t> cut(T + 1);
    for (unsigned k = 0; k <= T; k++) cut[k] = len / T * k;
    cut[T] = ~0ull;
    std::vector<HopOut> part(T);
    for (auto &pt : part) pt.want_headers = want_headers;
    const std::function<void(unsigned)> work = [&](unsigned k) {
        const uint64_t s = k ? find_record_start(buf, len, cut[k], std::min(cut[k + 1], len), lim) : 0;
        if (s == ~0ull) {
            part[k].start = ~0ull;
            return;
        }
        hop_range(buf, len, s, cut[k + 1], max_txs, lim, part[k]);
    };
    if (!HopPool::get().try_run(T, work)) {
        std::vector<std::thread> th;
        unsigned started = 0;
        try {  // no thread (resource limits): the remaining chunks run on this one
            for (; started + 1 < T; started++) th.emplace_back(work, started + 1);
        } catch (...) {
        }
        work(0);
        for (unsigned k = started + 1; k < T; k++) work(k);
        for (auto &t : th) t.join();
    }
    uint64_t pos = 0;
    out.start = 0;
    for (unsigned k = 0; k < T; k++) {
        if (pos >= cut[k + 1]) continue;  // a record spanning this whole chunk
        HopOut redo, *o = &part[k];
        redo.want_headers = want_headers;
        if (o->start != pos) {            // speculation missed: parse this chunk for real
            hop_range(buf, len, pos, cut[k + 1], max_txs, lim, redo);
            o = &redo;
        }
        const uint64_t room = max_txs - out.R.size();
        const uint64_t take = std::min<uint64_t>(room, o->R.size());
        for (HopPatch &pt : o->P)
            if (pt.rec < take) {
                pt.rec += out.R.size();
                out.P.push_back(std::move(pt));
            }
        out.R.insert(out.R.end(), o->R.begin(), o->R.begin() + take);
        if (want_headers) out.H.insert(out.H.end(), o->H.begin(), o->H.begin() + take);
        // max_txs reached inside or at the end of this chunk: the sequential
        // parse stops before reading the next record, so whatever stopped this
        // chunk's parse after it is not an error of the result
        if (take < o->R.size() || out.R.size() == max_txs) {
            if (take) pos = out.R.back().alh + 32;
            break;
        }
        pos = o->end;
        if (o->stopped) {
            out.rc = o->rc;
            out.stopped = true;
            break;
        }
    }
    out.end = pos;
}

}  // namespace

// Structure-only read of a run of tx records (host, no device): the record
// hop of mh_txlog_validate on its own.
extern "C" int mh_txlog_scan(const uint8_t *buf, uint64_t len, uint32_t max_entries,
                             uint32_t max_key_len, uint64_t max_txs, uint64_t *ntx_out,
                             uint64_t *consumed_out, mh_tx_header *hdrs_out,
                             uint64_t *alh_off_out) {
    return mh_guard([&]() -> int {
        if (len && !buf) return MH_ERR_ILLEGAL_ARGUMENTS;
        HopOut hop;
        hop_all(buf, len, max_txs, HopLimits{max_entries, max_key_len}, hop, hdrs_out != nullptr);
        const uint64_t ntx = hop.R.size();
        if (ntx_out) *ntx_out = ntx;
        if (consumed_out) *consumed_out = hop.end;
        if (hdrs_out && ntx) memcpy(hdrs_out, hop.H.data(), ntx * sizeof(mh_tx_header));
        if (alh_off_out)
            for (uint64_t k = 0; k < ntx; k++) alh_off_out[k] = hop.R[k].alh;
        return hop.rc;
    });
}

// The device address of [p, p + bytes) when the whole range is pinned host
// memory the kernels can store to (one registration or allocation, word
// aligned), else null.
static uint32_t *host_words(void *p, uint64_t bytes) {
    if (!p || !bytes || ((uintptr_t)p & 3) || (bytes & 3)) return nullptr;
    hipPointerAttribute_t a, b;
    if (hipPointerGetAttributes(&a, p) != hipSuccess ||
        hipPointerGetAttributes(&b, (uint8_t *)p + bytes - 1) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || b.type != hipMemoryTypeHost || !a.devicePointer ||
        (uint8_t *)b.devicePointer - (uint8_t *)a.devicePointer != (ptrdiff_t)(bytes - 1))
        return nullptr;
    return (uint32_t *)a.devicePointer;
}

// relative sizes of a pinned log's copy chunks, first to last: 5 : 2 : 1.
// The first two groups take the lane-per-record kernel (k_txlog_lanes, >=
// 16384 records of 2^16), whose launch over 5/8 of the log finishes under the
// next chunk's copy; the last group (1/8) takes the wave kernel, the shorter
// chain per record after the last byte lands.  One chunk boundary fewer than
// round 4's 4 : 2 : 1 : 1: 1.529-1.535 vs 1.555-1.568 ms per call, 3
// interleaved rounds (profiles/txlog_lanes_r05.txt; 6 : 1 : 1 ties, 7 : 1
// and 13 : 2 : 1 overrun the last copy, 11 : 4 : 1 and 9 : 4 : 2 : 1 lose).
// MH_TXLOG_WEIGHTS="w0:w1:..." gives any sizes (read per call, tests: up to
// 16 positive numbers separated by ':' or ',')
static std::vector<double> txlog_weights() {
    std::vector<double> w;
    if (const char *e = getenv("MH_TXLOG_WEIGHTS")) {
        for (const char *p = e; *p && w.size() < 16;) {
            char *q = nullptr;
            const double v = strtod(p, &q);
            if (q == p || !(v > 0)) break;
            w.push_back(v);
            if (*q != ',' && *q != ':') break;
            p = q + 1;
        }
    }
    if (w.empty()) w = {5, 2, 1};
    return w;
}

// The mh_tx_header words of the record at buf + rec other than Eh (words
// 11-14), exactly as k_txlog_wave stores them: id, ts, blTxID (BE64), blRoot
// and prevAlh (raw), version | nentries << 32, v1: mdLen | (rec + 92) << 32.
// The hop has bounds-checked the record.
static void fill_header_host(const uint8_t *buf, uint64_t rec, uint64_t *h) {
    const uint8_t *p = buf + rec;
    auto be = [](const uint8_t *q, int n) {
        uint64_t v = 0;
        for (int i = 0; i < n; i++) v = v << 8 | q[i];
        return v;
    };
    h[0] = be(p, 8);
    h[1] = be(p + 8, 8);
    h[2] = be(p + 16, 8);
    memcpy(h + 3, p + 24, 64);
    const uint32_t ver = (uint32_t)be(p + 88, 2);
    uint32_t nent, ml = 0;
    if (ver == 0) {
        nent = (uint32_t)be(p + 90, 2);
    } else {
        ml = (uint32_t)be(p + 90, 2);
        nent = (uint32_t)be(p + 92 + ml, 4);
    }
    h[15] = (uint64_t)ver | ((uint64_t)nent << 32);
    h[16] = ver ? (uint64_t)ml | ((uint64_t)(uint32_t)(rec + 92) << 32) : 0;
}

// buf: the log in host memory (the hop parses it); dlog: the same bytes
// already resident on the device (no copy; nullptr: copied from buf in chunks)
static int txlog_validate_impl(mh_ctx *c, const uint8_t *buf, const uint8_t *dlog, uint64_t len,
                               uint32_t max_entries, uint32_t max_key_len, uint64_t max_txs,
                               uint64_t *ntx_out, uint64_t *consumed_out, mh_tx_header *hdrs_out,
                               uint8_t *alh_out, int32_t *status_out, bool take_lock = true,
                               const HopOut *parsed = nullptr) {
    return mh_guard([&]() -> int {
        if (!c || (len && !buf)) return MH_ERR_ILLEGAL_ARGUMENTS;
        // The raw records go to the device first, in chunks with an event
        // after each: the copy (DMA when buf is pinned) runs under the host
        // hop, and the device work on the records of a chunk starts as soon as
        // it has landed, under the copy of the rest.
        std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
        if (take_lock) lk.lock();  // (mh_txlog_validate_clog holds it already)
        hipSetDevice(c->device);
        MH_HIP(c->copy_lane());
        hipStream_t st = c->stream;
        // + 256: k_txlog_wave's staging of a wave's records reads up to 128
        // bytes past the last record's stored Alh (16-byte pieces + its
        // unguarded block over-read pad), inside the allocation
        if (len && !dlog) MH_HIP(c->s_txlog.ensure(len + 256));
        uint8_t *dbuf = dlog ? const_cast<uint8_t *>(dlog) : c->s_txlog.as<uint8_t>();
        // A pinned log: 3 chunks from 16 MiB up (txlog_weights: 5 : 2 : 1;
        // the last chunk's device work is the tail after the copy), all
        // queued from this thread at once.  A
        // pageable one is staged by the runtime inside each copy call, so a
        // helper thread (ChunkCopier) issues those under the hop, in two
        // chunks (3/4 + 1/4: every staged call has its own setup).  Events
        // ev_chunks[0, K) mark the chunks' arrival (no system-scope fence: their
        // waiters are device streams), ev_results[0, K) the end of each
        // group's kernels (with the fence: c->d2h_stream's copies of a
        // group's results may run on a DMA engine).
        // the whole range in one pinned allocation (first and last byte)
        const bool pinned = len && !dlog && pinned_same_alloc(buf, buf + len - 1);
        const std::vector<double> wts = pinned ? txlog_weights() : std::vector<double>{3, 1};
        // (a resident log: one chunk without a copy, i.e. one group after the hop)
        const uint64_t K = dlog || len < (16ull << 20) ? 1 : wts.size();
        std::vector<uint64_t> cut(K + 1, 0);
        double wsum = 0, pre = 0;
        for (uint64_t k = 0; k < K; k++) wsum += wts[k];
        for (uint64_t k = 1; k < K; k++) {
            pre += wts[k - 1];  // the first k weights
            cut[k] = std::max<uint64_t>(cut[k - 1], (uint64_t)((double)len * pre / wsum) & ~4095ull);
        }
        cut[K] = len;
        const uint64_t nck = len ? K : 0;
        MH_HIP(ensure_chunk_events(c, nck));
        MH_HIP(ensure_result_events(c, nck));
        // once a group's kernels are queued they may store into the caller's
        // pinned status / alh / header arrays: every exit (errors included)
        // waits for both streams, so nothing writes caller memory after return
        // (every group on the context's stream: a second compute stream for
        // alternate groups slowed the last one, profiles/ab_txlog_streams_r04.txt)
        struct StreamGuard {
            hipStream_t a, b;
            bool armed = true;  // cleared once the call's own final waits ran
            ~StreamGuard() {
                if (!armed) return;
                hipStreamSynchronize(a);
                hipStreamSynchronize(b);
            }
        } stream_guard{st, c->d2h_stream};
        ChunkCopier cc(c);
        cc.chunks.resize(nck);
        for (uint64_t k = 0; k < nck; k++)
            cc.chunks[k] = {{dbuf + cut[k], buf + cut[k], dlog ? 0 : cut[k + 1] - cut[k]}};
        cc.inline_issue = pinned;
        MH_HIP(cc.start());
        auto join_copies = [&]() -> int {
            hipError_t e = cc.join();
            return e == hipSuccess ? MH_OK : -(int)e;
        };
        const HopLimits lim{max_entries, max_key_len};

        // ---- one group of records: its own device arrays (per entry record
        // offset, version, leaf digest; per tx header, entry-count word, record
        // offset, Alh offset, leaf offset, Eh, inner-hash scratch, Alh, status)
        // and pinned index staging, all indexed from the group's first record
        struct Grp {
            uint64_t t0 = 0, t1 = 0, e0 = 0, E = 0, wmax = 0, k = 0;
            bool small = true, fetched = false, host_done = false, early = false, host_hdrs = false;
            uint8_t *base = nullptr;
            uint64_t *pro = nullptr, *pap = nullptr, *plo = nullptr;
            uint64_t b_rec, b_ver, b_lv, b_h, b_es, b_ro, b_ap, b_lo, b_eh, b_s, b_a, b_st, b_pre, b_stats,
                idx_bytes;
            TreePlan P;
        };
        HopOut hop;
        std::vector<Grp> gs;
        gs.reserve(nck + 1);
        // records [t0, t1) of hop.R (entries from e0) as group number gi
        auto prepare = [&](Grp &g, size_t gi, uint64_t t0, uint64_t t1, uint64_t e0) -> int {
            g.t0 = t0;
            g.t1 = t1;
            g.e0 = e0;
            const uint64_t nt = t1 - t0;
            for (uint64_t t = t0; t < t1; t++) {
                g.E += hop.R[t].nent;
                g.wmax = std::max<uint64_t>(g.wmax, hop.R[t].nent);
            }
            g.small = small_roots_fit(nt, g.wmax);
            while (c->s_txg.size() <= gi) c->s_txg.emplace_back();
            while (c->p_txg.size() <= gi) c->p_txg.emplace_back();
            Layout L;
            g.b_rec = L.add(g.E * 8);
            g.b_ver = L.add(g.E);
            g.b_lv = L.add(std::max<uint64_t>(g.E, 1) * 32);
            g.b_h = L.add(nt * sizeof(mh_tx_header));
            g.b_es = L.add(nt * 8);
            g.b_ro = L.add(nt * 8);
            g.b_ap = L.add(nt * 8);
            g.b_lo = L.add((nt + 1) * 8);
            g.b_eh = L.add(nt * 32);
            g.b_s = L.add(nt * kTxInnerStride);
            g.b_a = L.add(nt * 32);
            g.b_st = L.add(nt * 4);
            g.b_pre = L.add(nt * 4);
            g.b_stats = L.add(4 * 8);
            MH_HIP(c->s_txg[gi].ensure(L.total));
            g.base = c->s_txg[gi].as<uint8_t>();
            g.idx_bytes = 3 * (nt + 1) * 8;
            uint64_t pin = g.idx_bytes;
            if (!g.small) {
                std::vector<uint64_t> lof(nt + 1);
                lof[0] = 0;
                for (uint64_t t = 0; t < nt; t++) lof[t + 1] = lof[t] + hop.R[t0 + t].nent;
                g.P.build(nt, lof.data());
                pin += plan_index_bytes(g.P, nt);
            }
            // the previous call's kernels read this staging: done (synced)
            MH_HIP(c->p_txg[gi].ensure(pin));
            g.pro = c->p_txg[gi].as<uint64_t>();
            g.pap = g.pro + (nt + 1);
            g.plo = g.pap + (nt + 1);
            uint64_t acc = 0;
            for (uint64_t t = 0; t < nt; t++) {
                g.pro[t] = hop.R[t0 + t].rec;
                g.pap[t] = hop.R[t0 + t].alh;
                g.plo[t] = acc;
                acc += hop.R[t0 + t].nent;
            }
            g.plo[nt] = acc;
            return MH_OK;
        };
        // ---- its device work, reading the log at db: index arrays up (a
        // kernel reads them from the pinned staging: a DMA copy would wait
        // behind the log chunks still in flight), headers, per-entry index
        // (tx.go:578-585), entry digests hashed in place from the raw entry
        // records (tx.go:690-731), one htree per tx (tx.go:617-621; small
        // trees one lane / wave per tree, a group with a wide tx through the
        // host tree plan), Alh with the rebuilt Eh vs the stored one
        // (tx.go:623-627).  pl: the group's metadata patch lists (below).
        // pre (resident logs): the per-record statuses of the device bytes'
        // structure (txlog_struct.hip) -- filled here for the fused kernels,
        // by the caller for the chain -- so no kernel walks a length of the
        // resident log that differs from the host copy's.
        auto run = [&](Grp &g, const uint8_t *db, const uint64_t *pl, uint64_t npe,
                       uint64_t nph, hipStream_t st, int32_t *pre) -> int {
            const uint64_t nt = g.t1 - g.t0;
            uint8_t *base = g.base;
            uint64_t *ro = (uint64_t *)(base + g.b_ro), *ap = (uint64_t *)(base + g.b_ap),
                     *lo = (uint64_t *)(base + g.b_lo), *es = (uint64_t *)(base + g.b_es),
                     *rec = (uint64_t *)(base + g.b_rec);
            MhTxHeader *hd = (MhTxHeader *)(base + g.b_h);
            if (!g.fetched)
                MH_HIP(launch_fetch_host(st, HostRuns{{g.pro, g.pap, g.plo}, {ro, ap, lo}, {nt, nt, nt + 1}}));
            if (g.small && npe + nph == 0) {  // the whole chain in one launch
                if (pre)  // the resident bytes' structure against the host's
                    MH_HIP(launch_txlog_struct(st, c->tm(), nt, db, len, len, nullptr, 0, ro, ap, lo,
                                               max_entries, max_key_len, pre,
                                               (uint64_t *)(base + g.b_stats)));
                // pinned outputs: the kernel writes the results there itself
                TxlogHostOut ho;
                uint32_t *hs = status_out ? host_words(status_out + g.t0, nt * 4) : nullptr;
                uint32_t *ha = alh_out ? host_words(alh_out + g.t0 * 32, nt * 32) : nullptr;
                uint32_t *hh = hdrs_out ? host_words(hdrs_out + g.t0, nt * sizeof(mh_tx_header)) : nullptr;
                if ((!status_out || hs) && (!alh_out || ha) && (!hdrs_out || hh) &&
                    ((uintptr_t)hh & 7) == 0) {
                    ho.status = hs;
                    ho.alh = ha;
                    ho.hdrs = reinterpret_cast<uint64_t *>(hh);
                    g.host_done = true;
                }
                // a group of >= 16384 records takes the lane-per-record kernel
                // (throughput), a smaller one the wave kernel (its chain per
                // record is shorter: the latency-shaped tail after the last
                // chunk lands).  MH_TXLOG_KERNEL=wave | lanes (read per call)
                // forces one of them: the tests run both on the same logs.
                const char *kn = getenv("MH_TXLOG_KERNEL");
                const bool lanes = kn ? strcmp(kn, "lanes") == 0 : nt >= 16384;
                // The last chunk's group -- its kernel is the tail of the call
                // -- writes only the Eh words of the caller's pinned headers;
                // the host fills the other fields from the log while that
                // kernel runs (32 instead of 136 B per record over PCIe at the
                // end: -4..-10 us per call in 9 of 10 interleaved rounds with
                // the 5 : 2 : 1 chunks, profiles/txlog_lanes_r05.txt).
                if (!lanes && ho.hdrs && g.early && g.k + 1 == nck) {
                    ho.eh_only = 1;
                    g.host_hdrs = true;
                }
                if (lanes)
                    MH_HIP(launch_txlog_lanes(st, c->tm(), nt, db, ro, ap, lo, pre, hd, base + g.b_eh,
                                              base + g.b_a, (int32_t *)(base + g.b_st), ho, g.wmax,
                                              len));
                else
                    MH_HIP(launch_txlog_wave(st, c->tm(), nt, db, ro, ap, lo, pre, hd, base + g.b_eh,
                                             base + g.b_a, (int32_t *)(base + g.b_st), ho, g.wmax,
                                             g.pro, g.pap));
                return MH_OK;
            }
            MH_HIP(launch_tx_hdr_from_raw(st, c->tm(), nt, db, ro, hd, es));
            MH_HIP(launch_txe_index(st, c->tm(), nt, db, hd, es, lo, rec, base + g.b_ver));
            if (npe + nph)
                MH_HIP(launch_txlog_patch(st, npe, pl, pl + npe, rec, nph, pl + 2 * npe,
                                          pl + 2 * npe + nph, hd));
            MH_HIP(launch_txe_leaf(st, c->tm(), g.E, db, rec, base + g.b_ver, g.small, base + g.b_lv));
            if (g.small) {
                MH_HIP(launch_small_roots(st, c->tm(), nt, lo, base + g.b_lv, base + g.b_eh, g.wmax));
            } else if (int e = run_tree_plan_on(c->s_tree, st, c->tm(), g.P, nt, g.E, base + g.b_lv,
                                                base + g.b_eh,
                                                reinterpret_cast<uint8_t *>(g.pro) + g.idx_bytes)) {
                return e;
            }
            MH_HIP(launch_tx_alh(st, c->tm(), nt, hd, db, base + g.b_eh, base + g.b_s, db, ap, nullptr,
                                 base + g.b_a, (int32_t *)(base + g.b_st)));
            if (pre)  // records whose resident bytes differ from the host copy
                MH_HIP(launch_txlog_apply_pre(st, nt, pre, (int32_t *)(base + g.b_st), base + g.b_a));
            if (hdrs_out)  // the device headers with the rebuilt Eh
                MH_HIP(launch_put_eh(st, nt, base + g.b_eh, hd));
            return MH_OK;
        };
        // ---- its results down to the caller's arrays at record t0: by kernel
        // stores when they are pinned host memory (on the results stream,
        // beside the next group's kernels; a D2H copy would wait behind the
        // log chunks on the DMA engine), else by D2H copies.  After event ev.
        // D2H copies into pageable memory return only when done: those of the
        // early groups are issued once every group is queued (late)
        std::vector<std::pair<const Grp *, hipEvent_t>> late;
        bool d2h_used = false;  // anything queued on c->d2h_stream this call
        auto results_dma = [&](const Grp &g, hipEvent_t ev) -> int {
            const uint64_t nt = g.t1 - g.t0, t0 = g.t0;
            hipStream_t ds = c->d2h_stream;
            d2h_used = true;
            MH_HIP(hipStreamWaitEvent(ds, ev, 0));
            if (status_out)
                MH_HIP(hipMemcpyAsync(status_out + t0, g.base + g.b_st, nt * 4, hipMemcpyDeviceToHost, ds));
            if (alh_out)
                MH_HIP(hipMemcpyAsync(alh_out + t0 * 32, g.base + g.b_a, nt * 32, hipMemcpyDeviceToHost, ds));
            if (hdrs_out)
                MH_HIP(hipMemcpyAsync(hdrs_out + t0, g.base + g.b_h, nt * sizeof(mh_tx_header),
                                      hipMemcpyDeviceToHost, ds));
            return MH_OK;
        };
        auto results = [&](const Grp &g, hipEvent_t ev) -> int {
            if (g.host_done) return MH_OK;  // stored by the group's kernel
            const uint64_t nt = g.t1 - g.t0, t0 = g.t0;
            hipStream_t ds = c->d2h_stream;
            uint32_t *hs = status_out ? host_words(status_out + t0, nt * 4) : nullptr;
            uint32_t *ha = alh_out ? host_words(alh_out + t0 * 32, nt * 32) : nullptr;
            uint32_t *hh = hdrs_out ? host_words(hdrs_out + t0, nt * sizeof(mh_tx_header)) : nullptr;
            if ((!status_out || hs) && (!alh_out || ha) && (!hdrs_out || hh)) {
                d2h_used = true;
                MH_HIP(hipStreamWaitEvent(ds, ev, 0));
                MH_HIP(launch_store_host(
                    ds, HostWordRuns{{(const uint32_t *)(g.base + g.b_st), (const uint32_t *)(g.base + g.b_a),
                                      (const uint32_t *)(g.base + g.b_h)},
                                     {hs, ha, hh},
                                     {hs ? nt : 0, ha ? nt * 8 : 0, hh ? nt * sizeof(mh_tx_header) / 4 : 0}}));
                return MH_OK;
            }
            late.emplace_back(&g, ev);
            return MH_OK;
        };

        // ---- host hop (tx.go:419-603): record structure and limits only.  Per
        // entry the host reads the two lengths it needs to find the next entry
        // (parked helper threads over a long stretch, hop_all); the per-entry
        // index (record offsets, versions, message lengths) is rebuilt on the
        // device from each tx's first entry (k_txe_index).
        //
        // It runs in one phase per copy chunk: phase k parses the records
        // that end inside chunk k, from where phase k-1 stopped (a record
        // crossing the chunk's end reads as truncated there and is parsed
        // again by the next phase), and their device work is queued at once
        // behind the chunk's event.  The records and the return code are the
        // one-pass parse's either way: every check of hop_record reads only
        // bytes it has bounds-checked, so a shorter buffer can only end a
        // parse early with TRUNCATED or a short-id EOF.  A phase with
        // non-canonical metadata or a wide tx stops the early groups: the
        // rest goes as one group once the whole log is in.
        // an early group behind the event of its chunk, results on their stream
        auto launch = [&](Grp &g) -> int {
            // the index arrays do not need the chunk: fetched before its event
            const uint64_t nt = g.t1 - g.t0;
            MH_HIP(launch_fetch_host(
                st, HostRuns{{g.pro, g.pap, g.plo},
                             {(uint64_t *)(g.base + g.b_ro), (uint64_t *)(g.base + g.b_ap),
                              (uint64_t *)(g.base + g.b_lo)},
                             {nt, nt, nt + 1}}));
            g.fetched = true;
            g.early = true;
            if (hipError_t e = cc.wait(g.k)) return -(int)e;
            MH_HIP(cc.stream_wait(st, g.k));
            if (int e = run(g, dbuf, nullptr, 0, 0, st, nullptr)) return e;
            MH_HIP(hipEventRecord(c->ev_results[g.k], st));
            return results(g, c->ev_results[g.k]);
        };
        size_t deferred = 0;  // gs[0, deferred) are queued
        uint64_t pos = 0, e_done = 0;
        size_t pre_r = 0, pre_p = 0;  // the next pre-parsed record / patch
        // (a log past 4 GiB is parsed in one phase: hop_record's 32-bit
        // metadata-offset check depends on where the parse starts)
        const uint64_t nphase = len <= 0xffffffffull ? nck : 1;
        bool early = nphase > 1;
        for (uint64_t k = 0; k < nphase; k++) {
            const uint64_t end = k + 1 < nphase ? cut[k + 1] : len;
            const uint64_t r0 = hop.R.size();
            HopOut h;
            if (parsed) {
                // parsed already (the multi-device call): the phase's records
                // are those ending inside it, and the phase reads as truncated
                // while more records follow, as the hop of a cut log does
                for (; pre_r < parsed->R.size() && r0 + h.R.size() < max_txs &&
                       parsed->R[pre_r].alh + 32 <= end;
                     pre_r++) {
                    const HopRec &r = parsed->R[pre_r];
                    for (; pre_p < parsed->P.size() && parsed->P[pre_p].rec == pre_r; pre_p++) {
                        HopPatch pt = parsed->P[pre_p];
                        pt.rec = h.R.size();
                        h.P.push_back(std::move(pt));
                    }
                    h.R.push_back(HopRec{r.rec - pos, r.alh - pos, r.nent, 0});
                }
                h.end = h.R.empty() ? 0 : h.R.back().alh + 32;
                h.rc = pre_r < parsed->R.size() ? MH_ERR_TRUNCATED : MH_OK;
                if (h.rc == MH_OK) h.end = end - pos;  // (the pre-parsed run ends at len)
            } else {
                hop_all(buf + pos, end - pos, max_txs - r0, lim, h, false);
            }
            for (const HopRec &r : h.R) hop.R.push_back(HopRec{r.rec + pos, r.alh + pos, r.nent, 0});
            for (HopPatch &pt : h.P) {
                pt.rec += r0;
                hop.P.push_back(std::move(pt));
            }
            hop.rc = h.rc;
            hop.end = pos + h.end;
            const bool more = k + 1 < nphase && hop.R.size() < max_txs &&
                              (h.rc == MH_ERR_TRUNCATED || (h.rc == MH_OK && hop.end + 8 > end));
            if (early && h.P.empty() && hop.R.size() > r0) {
                gs.emplace_back();
                Grp &g = gs.back();
                if (int e = prepare(g, gs.size() - 1, r0, hop.R.size(), e_done)) return e;
                if (!g.small) {
                    gs.pop_back();
                    early = false;
                } else {
                    g.k = k;
                    e_done += g.E;
                    // queued now if its chunk's copy is (a pageable log's copy
                    // calls block their thread: the remaining phases of the
                    // hop go first, and these groups after them)
                    if (deferred == gs.size() - 1 && cc.issued(k)) {
                        if (int e = launch(g)) return e;
                        deferred++;
                    }
                }
            } else if (!h.P.empty()) {
                early = false;
            }
            if (!more) break;
            pos = hop.end;
        }
        if (!nck && !parsed) hop_all(buf, len, max_txs, lim, hop, false);  // empty log
        for (; deferred < gs.size(); deferred++) {
            if (int e = launch(gs[deferred])) return e;
        }
        // header fields other than Eh of a host_hdrs group (readHeader,
        // tx.go:419-518, as k_txlog_wave lays them out: 17 words per record)
        for (const Grp &g : gs)
            if (g.host_hdrs)
                for (uint64_t t = g.t0; t < g.t1; t++)
                    fill_header_host(buf, hop.R[t].rec, reinterpret_cast<uint64_t *>(hdrs_out + t));
        if (!gs.empty() && mh_fault(MH_FAULT_TXLOG_AFTER_GROUP)) return -(int)hipErrorOutOfMemory;
        const uint64_t ntx = hop.R.size();
        const int rc = hop.rc;
        // on an error hop.end is the failing record's offset = the end of the last good one
        if (ntx_out) *ntx_out = ntx;
        if (consumed_out) *consumed_out = hop.end;
        if (int e = join_copies()) return e;
        const uint64_t t_rest = gs.empty() ? 0 : gs.back().t1;
        if (t_rest < ntx) {
            // ---- the rest as one group once the whole log is in
            if (nck) MH_HIP(cc.stream_wait(st, nck - 1));
            gs.emplace_back();
            Grp &g = gs.back();
            if (int e = prepare(g, gs.size() - 1, t_rest, ntx, e_done)) return e;
            // metadata that parses but is not in canonical form (a log not
            // written by immudb): Go hashes KVMetadata.Bytes() /
            // TxMetadata.Bytes(), so the canonical entry records / tx metadata
            // go after the log bytes in a copy of the log on the device, and
            // the group's entry index / headers point at them
            const uint8_t *db = dbuf;
            const uint64_t *pl = nullptr;
            uint64_t npe = 0, nph = 0;
            int32_t *pre = dlog ? (int32_t *)(g.base + g.b_pre) : nullptr;
            if (dlog && !(g.small && hop.P.empty())) {
                // a resident log whose group the fused kernels do not take
                // (re-encoded metadata, a wide tx): the chain runs over the
                // host copy uploaded beside it, and a record whose resident
                // bytes differ from that copy is corrupted (one byte compare)
                const uint64_t nt = ntx - t_rest;
                uint64_t *ro = (uint64_t *)(g.base + g.b_ro), *ap = (uint64_t *)(g.base + g.b_ap),
                         *lo = (uint64_t *)(g.base + g.b_lo);
                MH_HIP(c->s_txlog.ensure(len + 256));
                MH_HIP(hipMemcpyAsync(c->s_txlog.as<uint8_t>(), buf, len, hipMemcpyHostToDevice, st));
                MH_HIP(launch_fetch_host(st, HostRuns{{g.pro, g.pap, g.plo}, {ro, ap, lo}, {nt, nt, nt + 1}}));
                g.fetched = true;
                MH_HIP(launch_txlog_bytes_cmp(st, nt, dlog, c->s_txlog.as<uint8_t>(), ro, ap, pre));
                db = dbuf = c->s_txlog.as<uint8_t>();
            }
            if (!hop.P.empty()) {
                std::vector<uint64_t> first_leaf(ntx - t_rest);  // group-local entry index
                for (uint64_t t = t_rest, acc = 0; t < ntx; t++) {
                    first_leaf[t - t_rest] = acc;
                    acc += hop.R[t].nent;
                }
                uint64_t side = 0;
                for (const HopPatch &pt : hop.P) {
                    side += pt.bytes.size();
                    (pt.kind == 0 ? npe : nph)++;
                }
                if (len + side > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;
                std::vector<uint8_t> sbuf;
                sbuf.reserve(side);
                std::vector<uint64_t> patch(2 * (npe + nph));  // [ne idx][ne off][nh idx][nh off | len << 32]
                uint64_t ie = 0, ih = 0;
                for (const HopPatch &pt : hop.P) {
                    if (pt.rec < t_rest) return MH_ERR_ILLEGAL_STATE;  // early groups have none
                    const uint64_t off = len + sbuf.size();
                    if (pt.kind == 0) {
                        patch[ie] = first_leaf[pt.rec - t_rest] + pt.entry;
                        patch[npe + ie++] = off;
                    } else {
                        patch[2 * npe + ih] = pt.rec - t_rest;
                        patch[2 * npe + nph + ih++] = off | ((uint64_t)pt.bytes.size() << 32);
                    }
                    sbuf.insert(sbuf.end(), pt.bytes.begin(), pt.bytes.end());
                }
                const uint64_t po = (len + side + 7) & ~7ull;
                MH_HIP(c->s_txpatch.ensure(po + patch.size() * 8));
                uint8_t *nb = c->s_txpatch.as<uint8_t>();
                MH_HIP(hipMemcpyAsync(nb, dbuf, len, hipMemcpyDeviceToDevice, st));
                MH_HIP(hipMemcpyAsync(nb + len, sbuf.data(), side, hipMemcpyHostToDevice, st));
                MH_HIP(hipMemcpyAsync(nb + po, patch.data(), patch.size() * 8, hipMemcpyHostToDevice, st));
                MH_HIP(hipStreamSynchronize(st));  // the host vectors go out of scope
                db = nb;
                pl = reinterpret_cast<const uint64_t *>(nb + po);
            }
            if (int e = run(g, db, pl, npe, nph, st, pre)) return e;
            MH_HIP(hipEventRecord(c->ev_done[1], st));
            if (int e = results(g, c->ev_done[1])) return e;
        }
        for (const auto &r : late)
            if (int e = results_dma(*r.first, r.second)) return e;
        // only the streams this call queued work on (every wait is an API
        // round trip on the critical path of the call)
        MH_HIP(hipStreamSynchronize(st));
        if (d2h_used) MH_HIP(hipStreamSynchronize(c->d2h_stream));
        stream_guard.armed = false;
        // buf stays the caller's once we return
        if (nck) MH_HIP(cc.sync());
        return rc;
    });
}

extern "C" int mh_txlog_validate(mh_ctx *c, const uint8_t *buf, uint64_t len, uint32_t max_entries,
                                 uint32_t max_key_len, uint64_t max_txs, uint64_t *ntx_out,
                                 uint64_t *consumed_out, mh_tx_header *hdrs_out, uint8_t *alh_out,
                                 int32_t *status_out) {
    return txlog_validate_impl(c, buf, nullptr, len, max_entries, max_key_len, max_txs, ntx_out,
                               consumed_out, hdrs_out, alh_out, status_out);
}

void txlog_hop(const uint8_t *buf, uint64_t len, uint32_t max_entries, uint32_t max_key_len,
               uint64_t max_txs, HopOut &out) {
    hop_all(buf, len, max_txs, HopLimits{max_entries, max_key_len}, out, false);
}

int txlog_validate_parsed(mh_ctx *c, const uint8_t *buf, uint64_t len, uint32_t max_entries,
                          uint32_t max_key_len, const HopOut &pre, mh_tx_header *hdrs_out,
                          uint8_t *alh_out, int32_t *status_out) {
    if (pre.rc != MH_OK || pre.end != len) return MH_ERR_ILLEGAL_STATE;
    uint64_t n = 0, used = 0;
    const int rc = txlog_validate_impl(c, buf, nullptr, len, max_entries, max_key_len,
                                       pre.R.size(), &n, &used, hdrs_out, alh_out, status_out,
                                       true, &pre);
    if (rc == MH_OK && (n != pre.R.size() || used != len)) return MH_ERR_ILLEGAL_STATE;
    return rc;
}

extern "C" int mh_txlog_validate_resident(mh_ctx *c, const uint8_t *buf, const uint8_t *dlog,
                                          uint64_t len, uint32_t max_entries, uint32_t max_key_len,
                                          uint64_t max_txs, uint64_t *ntx_out,
                                          uint64_t *consumed_out, mh_tx_header *hdrs_out,
                                          uint8_t *alh_out, int32_t *status_out) {
    return mh_guard([&]() -> int {
        if (!c || (len && (!buf || !dlog))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (len) {
            // the kernels stage 16-byte pieces up to 128 bytes past the last
            // record: the device allocation must extend len + 256 bytes
            hipSetDevice(c->device);
            hipDeviceptr_t base = nullptr;
            size_t size = 0;
            if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)dlog) != hipSuccess) {
                (void)hipGetLastError();
                return MH_ERR_ILLEGAL_ARGUMENTS;
            }
            const uintptr_t b = (uintptr_t)base, d = (uintptr_t)dlog;
            if (d < b || d - b + len + 256 > size) return MH_ERR_ILLEGAL_ARGUMENTS;
        }
        return txlog_validate_impl(c, buf, dlog, len, max_entries, max_key_len, max_txs, ntx_out,
                                   consumed_out, hdrs_out, alh_out, status_out);
    });
}


// The device range [p, p + bytes) lies in one allocation of the context's
// device (hipMemGetAddressRange), or the address is not device memory at all.
static bool dev_range(const void *p, uint64_t bytes) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const uintptr_t b = (uintptr_t)base, d = (uintptr_t)p;
    return d >= b && d - b <= size && bytes <= size - (d - b);
}

// Where a kernel can store the caller's output array p of `bytes`: p itself
// when it is device memory (its whole range in one allocation; *bad when it
// is not), the device alias of pinned host memory, else null (staged on the
// device and copied down).
static void *kernel_dst(void *p, uint64_t bytes, bool *bad, bool *is_dev) {
    *is_dev = false;
    if (!p || !bytes) return nullptr;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;  // pageable host memory
    }
    if (a.type == hipMemoryTypeDevice) {
        if (!dev_range(p, bytes)) *bad = true;
        *is_dev = true;
        return p;
    }
    if (a.type == hipMemoryTypeHost) return host_words(p, bytes);
    return nullptr;
}

// a14 over a tx log indexed by its commit log (txOffsetAndSize,
// immustore.go:2569-2597): no host hop.  The structure pass
// (txlog_struct.hip) parses every record where its cLog entry points, with
// every check of the host hop; the lane kernel hashes the accepted ones (entry
// digests, htree, innerHash, Alh vs the stored Alh); a record whose metadata
// is valid but not canonical (Go hashes the re-serialised form), that is wider
// than the lane kernel takes, or whose read runs past the bytes landed when
// its group ran is re-validated by mh_txlog_validate on a host copy of that
// record alone.
//  * log in device memory: one group, no copy;
//  * log in host memory (pinned: the cgo shim's arena): copied up in chunks
//    (5 : 2 : 1 from 16 MiB, as mh_txlog_validate), each chunk's records --
//    those whose cLog entry ends inside it, when the entries are in log order
//    -- checked as soon as it lands, under the copy of the rest; the lane
//    kernel takes its entries per lane from the structure pass's widest
//    record on the device (launch shape from the cLog sizes), so nothing
//    waits on the host between the chunks.
extern "C" int mh_txlog_validate_clog(mh_ctx *c, const uint8_t *dlog, uint64_t len,
                                      const uint8_t *clog, uint64_t ntx, uint32_t clog_entry_size,
                                      uint32_t max_entries, uint32_t max_key_len,
                                      mh_tx_header *hdrs_out, uint8_t *alh_out,
                                      int32_t *status_out, uint64_t *nbad_out,
                                      uint64_t *first_bad_out) {
    return mh_guard([&]() -> int {
        const uint32_t es = clog_entry_size;
        if (!c || (es != 12 && es != 44) || (ntx && (!dlog || !clog))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (nbad_out) *nbad_out = 0;
        if (first_bad_out) *first_bad_out = ntx;
        if (!ntx) return MH_OK;
        if (ntx > (1ull << 40)) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        hipSetDevice(c->device);
        MH_HIP(c->copy_lane());
        hipStream_t st = c->stream;
        auto is_dev = [](const void *q) {
            hipPointerAttribute_t a;
            const bool d = hipPointerGetAttributes(&a, q) == hipSuccess && a.type == hipMemoryTypeDevice;
            (void)hipGetLastError();
            return d;
        };
        const bool log_dev = is_dev(dlog), clog_dev = is_dev(clog);
        // a resident log: the kernels' unguarded block reads run up to 256
        // bytes past a record, inside the allocation
        if (log_dev && !dev_range(dlog, len + 256)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (clog_dev && !dev_range(clog, ntx * es)) return MH_ERR_ILLEGAL_ARGUMENTS;
        bool bad = false, st_dev, alh_dev, hd_dev;
        uint32_t *k_st = (uint32_t *)kernel_dst(status_out, ntx * 4, &bad, &st_dev);
        uint32_t *k_alh = (uint32_t *)kernel_dst(alh_out, ntx * 32, &bad, &alh_dev);
        uint64_t *k_hd = (uint64_t *)kernel_dst(hdrs_out, ntx * sizeof(mh_tx_header), &bad, &hd_dev);
        if (bad || ((uintptr_t)k_hd & 7)) return MH_ERR_ILLEGAL_ARGUMENTS;
        // ---- copy chunks and record groups of a host log
        const bool pinned = !log_dev && len && pinned_same_alloc(dlog, dlog + len - 1);
        std::vector<uint64_t> cut{0, len};
        if (!log_dev && len >= (16ull << 20)) {
            const std::vector<double> wts = pinned ? txlog_weights() : std::vector<double>{3, 1};
            const uint64_t K = wts.size();
            cut.assign(K + 1, 0);
            double wsum = 0, acc = 0;
            for (double w : wts) wsum += w;
            for (uint64_t k = 1; k < K; k++) {
                acc += wts[k - 1];
                cut[k] = std::max<uint64_t>(cut[k - 1], (uint64_t)((double)len * acc / wsum) & ~4095ull);
            }
            cut[K] = len;
        }
        const uint64_t nck = cut.size() - 1;
        // record groups: one for a resident log, at most one per copy chunk
        const size_t ngmax = log_dev ? 1 : nck;
        Layout L;
        const uint64_t b_ro = L.add(ntx * 8), b_ao = L.add(ntx * 8), b_pre = L.add(ntx * 4),
                       b_st = L.add(ntx * 4), b_eh = L.add(ntx * 32), b_a = L.add(ntx * 32),
                       b_hd = L.add(hdrs_out && !k_hd ? ntx * sizeof(mh_tx_header) : 0),
                       b_cl = L.add(clog_dev ? 0 : ntx * es), b_stats = L.add((4 + 2 * ngmax) * 8);
        MH_HIP(c->s_clog.ensure(L.total));
        uint8_t *base = c->s_clog.as<uint8_t>();
        uint64_t *ro = (uint64_t *)(base + b_ro), *ao = (uint64_t *)(base + b_ao),
                 *stats = (uint64_t *)(base + b_stats), *gstats = stats + 4;
        int32_t *pre = (int32_t *)(base + b_pre), *sts = (int32_t *)(base + b_st);
        MhTxHeader *hd = hdrs_out && !k_hd ? (MhTxHeader *)(base + b_hd) : nullptr;
        const uint8_t *dcl = clog_dev ? clog : base + b_cl;
        if (!log_dev) MH_HIP(c->s_txlog.ensure(len + 256));
        const uint8_t *db = log_dev ? dlog : c->s_txlog.as<uint8_t>();
        MH_HIP(hipMemsetAsync(stats, 0, (4 + 2 * ngmax) * 8, st));
        MH_HIP(hipMemsetAsync(stats + 3, 0xff, 8, st));
        MH_HIP(c->p_small.ensure(64 + 16 * ngmax));
        volatile uint64_t *hs = c->p_small.as<volatile uint64_t>();
        // every exit waits for the streams (kernels may store into the caller's
        // pinned / device arrays; copies read the caller's log)
        struct StreamGuard {
            hipStream_t a;
            bool armed = true;
            ~StreamGuard() {
                if (armed) hipStreamSynchronize(a);
            }
        } guard{st};
        ChunkCopier cc(c);
        if (!log_dev) {
            MH_HIP(ensure_chunk_events(c, nck));
            cc.chunks.resize(nck);
            for (uint64_t k = 0; k < nck; k++)
                cc.chunks[k] = {{const_cast<uint8_t *>(db) + cut[k], dlog + cut[k], cut[k + 1] - cut[k]}};
            cc.inline_issue = pinned;
            MH_HIP(cc.start());
        }
        // (after the chunk copies are issued: they wait for this stream's
        // earlier work, the previous call's readers of the staging buffer)
        if (!clog_dev) MH_HIP(hipMemcpyAsync(base + b_cl, clog, ntx * es, hipMemcpyHostToDevice, st));
        // (the host's pass over the cLog runs under the copies: ~2-3 ns per
        // entry, 0.15-0.2 ms for 65 536 entries, was ahead of them)
        // the host's view of the cLog entries (for the groups and the launch
        // shapes of a host log, and for the host fallback)
        std::vector<uint8_t> hcl_copy;
        const uint8_t *hcl = clog_dev ? nullptr : clog;
        if (clog_dev && !log_dev) {
            // (on this stream, not hipMemcpy's: that one would wait for the
            // copy streams, i.e. for the whole log to land)
            hcl_copy.resize(ntx * es);
            MH_HIP(hipMemcpyAsync(hcl_copy.data(), clog, ntx * es, hipMemcpyDeviceToHost, st));
            MH_HIP(hipStreamSynchronize(st));
            hcl = hcl_copy.data();
        }
        // group g: records [tg[g], tg[g+1]), read within the first lim[g] bytes
        std::vector<uint64_t> tg{0, ntx}, lim{len}, bound{kTxlLanesMaxEntries};
        if (!log_dev) {
            // the widest record a cLog size allows: header + Alh >= 124 bytes,
            // an entry >= 48 (2 + 2 + 4 + 8 + 32)
            auto wbound = [&](uint64_t t) -> uint64_t {
                const uint64_t sz = be_at(hcl + t * es + 8, 4);
                return std::min<uint64_t>(kTxlLanesMaxEntries, sz >= 124 ? (sz - 124) / 48 : 0);
            };
            bool ordered = true;
            uint64_t prev_end = 0;
            std::vector<uint64_t> end(ntx);
            for (uint64_t t = 0; t < ntx; t++) {
                const uint64_t off = be_at(hcl + t * es, 8), sz = be_at(hcl + t * es + 8, 4);
                end[t] = off + sz < off ? ~0ull : off + sz;
                ordered &= end[t] >= prev_end;
                prev_end = end[t];
            }
            if (ordered && nck > 1) {
                tg.assign(nck + 1, 0);
                lim.assign(nck, len);
                for (uint64_t k = 1; k < nck; k++) {
                    tg[k] = (uint64_t)(std::upper_bound(end.begin(), end.end(), cut[k]) - end.begin());
                    lim[k - 1] = cut[k];
                }
                tg[nck] = ntx;
            } else {
                tg = {0, ntx};
                lim = {len};
            }
            bound.assign(tg.size() - 1, 1);
            for (size_t g = 0; g + 1 < tg.size(); g++)
                for (uint64_t t = tg[g]; t < tg[g + 1]; t++) bound[g] = std::max(bound[g], wbound(t));
        }
        const size_t ng = tg.size() - 1;
        TxlogHostOut ho0;
        ho0.status = k_st;
        ho0.alh = k_alh;
        ho0.hdrs = k_hd;
        // stats[0]: a lane launch whose shape was too narrow for its records
        // (the resident form launches on the previous call's widest record
        // without waiting for this one's: a wider log goes again below)
        uint64_t *redo = stats;
        // group g's arrays start at its first record
        auto run_group = [&](size_t g, uint64_t wmax, const uint64_t *wmax_dev) -> int {
            const uint64_t t0 = tg[g], n = tg[g + 1] - t0;
            if (!n) return MH_OK;
            TxlogHostOut ho = ho0;
            if (ho.status) ho.status += t0;
            if (ho.alh) ho.alh += t0 * 8;
            if (ho.hdrs) ho.hdrs += t0 * 17;
            MH_HIP(launch_txlog_lanes(st, c->tm(), n, db, ro + t0, ao + t0, nullptr, pre + t0,
                                      hd ? hd + t0 : nullptr, base + b_eh + t0 * 32,
                                      base + b_a + t0 * 32, sts + t0, ho, std::max<uint64_t>(wmax, 1),
                                      len, wmax_dev, wmax_dev ? redo : nullptr));
            return MH_OK;
        };
        uint64_t nhost = 0;
        if (log_dev) {
            // 1. every record's structure where its cLog entry points
            MH_HIP(launch_txlog_struct(st, c->tm(), ntx, db, len, len, dcl, es, ro, ao, nullptr,
                                       max_entries, max_key_len, pre, gstats));
            // 2. the accepted records hashed and checked, the launch shaped by
            // the previous call's widest record (no wait: 0.264 -> ~0.245 ms
            // on 65 536 records), by this one's on a first call
            if (c->clog_wmax) {
                if (int e = run_group(0, c->clog_wmax, gstats)) return e;
            } else {
                MH_HIP(hipMemcpyAsync((void *)hs, gstats, 2 * 8, hipMemcpyDeviceToHost, st));
                MH_HIP(hipStreamSynchronize(st));
                if (int e = run_group(0, hs[0], nullptr)) return e;
            }
        } else {
            for (size_t g = 0; g < ng; g++) {
                const uint64_t t0 = tg[g], n = tg[g + 1] - t0;
                // the group's bytes have landed: chunk g (or every chunk for the
                // one group of a cLog out of log order)
                const size_t ck = ng == nck ? g : nck - 1;
                if (ng == nck || g == 0) {
                    for (size_t k = ng == nck ? ck : 0; k <= ck; k++) {
                        if (hipError_t e = cc.wait(k)) return -(int)e;
                        MH_HIP(cc.stream_wait(st, k));
                    }
                }
                if (!n) continue;
                MH_HIP(launch_txlog_struct(st, c->tm(), n, db, len, lim[g], dcl + t0 * es, es, ro + t0,
                                           ao + t0, nullptr, max_entries, max_key_len, pre + t0,
                                           gstats + 2 * g));
                if (int e = run_group(g, bound[g], gstats + 2 * g)) return e;
            }
        }
        // 3. how many records failed, and the first (and, for a host log, how
        // many records the host must re-validate); results down
        MH_HIP(launch_txlog_status_summary(st, ntx, sts, stats));
        MH_HIP(hipMemcpyAsync((void *)hs, stats, 4 * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync((void *)(hs + 8), gstats, 2 * ng * 8, hipMemcpyDeviceToHost, st));
        auto results_down = [&]() -> int {
            if (status_out && !k_st) MH_HIP(hipMemcpyAsync(status_out, sts, ntx * 4, hipMemcpyDeviceToHost, st));
            if (alh_out && !k_alh) MH_HIP(hipMemcpyAsync(alh_out, base + b_a, ntx * 32, hipMemcpyDeviceToHost, st));
            if (hdrs_out && !k_hd)
                MH_HIP(hipMemcpyAsync(hdrs_out, hd, ntx * sizeof(mh_tx_header), hipMemcpyDeviceToHost, st));
            return MH_OK;
        };
        if (int e = results_down()) return e;
        MH_HIP(hipStreamSynchronize(st));
        if (!log_dev)
            if (hipError_t e = cc.sync()) return -(int)e;  // the caller's log is no longer read
        if (hs[0]) {  // a launch too narrow for its records: again, shaped by them
            MH_HIP(hipMemsetAsync(stats, 0, 4 * 8, st));
            MH_HIP(hipMemsetAsync(stats + 3, 0xff, 8, st));
            for (size_t g = 0; g < ng; g++)
                if (int e = run_group(g, hs[8 + 2 * g], nullptr)) return e;
            MH_HIP(launch_txlog_status_summary(st, ntx, sts, stats));
            MH_HIP(hipMemcpyAsync((void *)hs, stats, 4 * 8, hipMemcpyDeviceToHost, st));
            if (int e = results_down()) return e;
            MH_HIP(hipStreamSynchronize(st));
        }
        for (size_t g = 0; g < ng; g++) nhost += hs[8 + 2 * g + 1];
        if (log_dev) c->clog_wmax = std::max<uint64_t>((uint64_t)hs[8], 1);
        // 4. records for the host hop (rare: a log not written by immudb, or a
        // record that disagrees with its cLog entry)
        if (nhost) {
            struct Fix {
                uint64_t t;
                int32_t st;
                mh_tx_header h;
                uint8_t alh[32];
            };
            std::vector<Fix> fix;
            std::vector<int32_t> hpre(ntx);
            std::vector<uint64_t> hro(ntx);
            if (clog_dev && hcl_copy.empty()) {
                hcl_copy.resize(ntx * es);
                MH_HIP(hipMemcpyAsync(hcl_copy.data(), clog, ntx * es, hipMemcpyDeviceToHost, st));
                hcl = hcl_copy.data();
            }
            MH_HIP(hipMemcpyAsync(hpre.data(), pre, ntx * 4, hipMemcpyDeviceToHost, st));
            MH_HIP(hipMemcpyAsync(hro.data(), ro, ntx * 8, hipMemcpyDeviceToHost, st));
            MH_HIP(hipStreamSynchronize(st));
            std::vector<uint8_t> rb;
            for (uint64_t t = 0; t < ntx; t++) {
                if (hpre[t] != kTxlNeedsHost) continue;
                const uint64_t off = hro[t], size = be_at(hcl + t * es + 8, 4);
                Fix f{};
                f.t = t;
                int32_t one = 0;
                // the record within its cLog size first (valid records end
                // there); a read past it needs the rest of the log (readTx reads
                // on), for the reader's own verdict
                uint64_t n = 0, used = 0, span = off < len ? std::min(size, len - off) : 0;
                int rc = off >= len || len - off < 8 ? MH_ERR_TRUNCATED : MH_OK;  // the reader's EOF
                for (int pass = 0; pass < 2 && rc == MH_OK; pass++) {
                    const uint8_t *src = dlog + off;
                    if (log_dev) {
                        rb.resize(span);
                        MH_HIP(hipMemcpy(rb.data(), dlog + off, span, hipMemcpyDeviceToHost));
                        src = rb.data();
                    }
                    n = used = 0;
                    memset(&f.h, 0, sizeof f.h);
                    rc = txlog_validate_impl(c, src, nullptr, span, max_entries, max_key_len, 1, &n,
                                             &used, &f.h, f.alh, &one, false);
                    if (rc < 0) return rc;
                    if ((rc != MH_ERR_TRUNCATED && (rc != MH_OK || n == 1)) || span == len - off) break;
                    span = len - off;
                    rc = MH_OK;
                }
                int s1 = rc != MH_OK ? rc : n != 1 ? MH_ERR_TRUNCATED : used != size ? MH_ERR_CORRUPTED_DATA : MH_OK;
                if (s1 == MH_OK && es == 44) {
                    uint8_t a[32];
                    if (log_dev)
                        MH_HIP(hipMemcpy(a, dlog + off + size - 32, 32, hipMemcpyDeviceToHost));
                    else
                        memcpy(a, dlog + off + size - 32, 32);
                    if (memcmp(hcl + t * es + 12, a, 32)) s1 = MH_ERR_CORRUPTED_DATA;
                }
                if (s1 != MH_OK) {
                    memset(&f.h, 0, sizeof f.h);
                    memset(f.alh, 0, 32);
                }
                f.st = s1 != MH_OK ? s1 : one;
                if (f.h.version) f.h.md_off += (uint32_t)off;  // relative to the log, as the kernel's
                fix.push_back(f);
            }
            MH_HIP(c->p_stage.ensure(fix.size() * sizeof(Fix)));
            Fix *pf = c->p_stage.as<Fix>();
            for (size_t k = 0; k < fix.size(); k++) pf[k] = fix[k];
            for (size_t k = 0; k < fix.size(); k++) {  // into the device arrays the summary reads
                const uint64_t t = pf[k].t;
                MH_HIP(hipMemcpyAsync(sts + t, &pf[k].st, 4, hipMemcpyHostToDevice, st));
                MH_HIP(hipMemcpyAsync(base + b_a + t * 32, pf[k].alh, 32, hipMemcpyHostToDevice, st));
                if (hd) MH_HIP(hipMemcpyAsync(hd + t, &pf[k].h, sizeof(mh_tx_header), hipMemcpyHostToDevice, st));
                // device outputs get theirs here, host outputs after the sync
                if (st_dev)
                    MH_HIP(hipMemcpyAsync(status_out + t, &pf[k].st, 4, hipMemcpyHostToDevice, st));
                if (alh_dev)
                    MH_HIP(hipMemcpyAsync(alh_out + t * 32, pf[k].alh, 32, hipMemcpyHostToDevice, st));
                if (hd_dev)
                    MH_HIP(hipMemcpyAsync(hdrs_out + t, &pf[k].h, sizeof(mh_tx_header), hipMemcpyHostToDevice, st));
            }
            MH_HIP(hipMemsetAsync(stats + 2, 0, 8, st));
            MH_HIP(hipMemsetAsync(stats + 3, 0xff, 8, st));
            MH_HIP(launch_txlog_status_summary(st, ntx, sts, stats));
            MH_HIP(hipMemcpyAsync((void *)(hs + 2), stats + 2, 2 * 8, hipMemcpyDeviceToHost, st));
            if (int e = results_down()) return e;
            MH_HIP(hipStreamSynchronize(st));
            for (size_t k = 0; k < fix.size(); k++) {  // host outputs (pinned: the kernel wrote zeros)
                const uint64_t t = pf[k].t;
                if (status_out && !st_dev) status_out[t] = pf[k].st;
                if (alh_out && !alh_dev) memcpy(alh_out + t * 32, pf[k].alh, 32);
                if (hdrs_out && !hd_dev) hdrs_out[t] = pf[k].h;
            }
        }
        guard.armed = false;
        if (nbad_out) *nbad_out = hs[2];
        if (first_bad_out) *first_bad_out = hs[2] ? hs[3] : ntx;
        return MH_OK;
    });
}
