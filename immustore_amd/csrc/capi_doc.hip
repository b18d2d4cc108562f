// capi_doc.hip -- pkg/verification.VerifyDocument (pkg/verification/
// verification.go:37-196), the hashing part, for a batch of documents.
//
// Per document the reference:
//   1. hashes the EncodedDocument and compares it with the HValue of the one
//      tx entry whose key is the document's encoded key (:60-76);
//   2. (decodes the document and compares it with the caller's -- not hashing,
//      left to the caller, :78-110);
//   3. rebuilds the tx's htree from EntrySpecDigestFor(version) over the
//      entries with IsValueTruncated = true and compares the root with Eh
//      (:112-139);
//   4. checks the tx / source / target headers and the known state against
//      the headers' Alh values (:141-183);
//   5. runs VerifyDualProofV2 (:185-194).
// Steps 1, 3, 4 and 5 run here, all on the device: SHA-256 of the documents
// and the entry search, the entry-spec digests (fused entry kernel, HValues
// as hVal overrides) and the per-document htrees, the header checks and Alh
// values, the known-state checks and the dual proofs, each document's verdict
// taken in the reference's order by per-document kernels.  The caller's
// arrays go up as they are (one copy each); the statuses and target Alh come
// back.  The host only validates offsets and plans the many-tree levels.
#include "capi_internal.hpp"

namespace {

// VerifyDocument :60-76, one wave per document: among the tx's entries
// [ent_off[d], ent_off[d+1]) exactly one has the document's encoded key, and
// its HValue is SHA256(EncodedDocument).  Go walks the entries in order and
// stops at the first match whose HValue differs (:63-67); the outcome is the
// same as "exactly one key match, and it is good", which the wave decides
// with one lane per entry and two ballots per 64 entries.  Key / offset arrays
// are the caller's (unrebased offsets, base pointers shifted by the caller's
// first offset).
__global__ __launch_bounds__(256) void k_doc_find(uint64_t n, const uint64_t *__restrict__ ent_off,
                                                  const uint8_t *__restrict__ dkeys,
                                                  const uint64_t *__restrict__ dkey_off,
                                                  const uint8_t *__restrict__ ekeys,
                                                  const uint64_t *__restrict__ ekey_off,
                                                  const uint8_t *__restrict__ ehval,
                                                  const uint8_t *__restrict__ hdoc,
                                                  int32_t *__restrict__ status) {
    const uint64_t d = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (d >= n) return;  // wave-uniform
    const uint8_t *k = dkeys + dkey_off[d];
    const uint64_t kl = dkey_off[d + 1] - dkey_off[d];
    const uint64_t e_end = ent_off[d + 1];
    uint32_t matches = 0, good = 0;
    for (uint64_t e0 = ent_off[d]; e0 < e_end; e0 += 64) {
        const uint64_t e = e0 + lane;
        bool m = false, g = false;
        if (e < e_end && ekey_off[e + 1] - ekey_off[e] == kl) {
            const uint8_t *q = ekeys + ekey_off[e];
            m = true;
            for (uint64_t j = 0; j < kl && m; j++) m = q[j] == k[j];
            if (m) {
                const uint8_t *hv = ehval + 32 * (e - ent_off[0]);
                g = true;
                for (int j = 0; j < 32 && g; j++) g = hv[j] == hdoc[32 * d + j];
            }
        }
        matches += (uint32_t)__popcll(__ballot(m));
        good += (uint32_t)__popcll(__ballot(m && g));
    }
    if (lane == 0) status[d] = (matches == 1 && good == 1) ? MH_OK : MH_ERR_INVALID_PROOF_ENTRY;
}

// Header preconditions of every header the document needs (check_header on
// the device): j < n the tx header, then the source and the target headers.
// A v0 innerHash never reads the metadata (tx.go:258-263): its md_len is
// cleared; a header that cannot be hashed (version not 0/1, metadata out of
// bounds) makes Go's innerHash panic -- flagged, and hashed as an empty v1
// header so the Alh kernel reads nothing outside md_blob.
__global__ __launch_bounds__(256) void k_doc_hdr_prep(uint64_t n, const mh_tx_header *__restrict__ tx,
                                                      const mh_tx_header *__restrict__ src,
                                                      const mh_tx_header *__restrict__ tgt,
                                                      uint64_t md_blob_len, int have_blob,
                                                      mh_tx_header *__restrict__ hfix,
                                                      uint8_t *__restrict__ hashable) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= 3 * n) return;
    mh_tx_header h = j < n ? tx[j] : (j < 2 * n ? src[j - n] : tgt[j - 2 * n]);
    if (h.version == 0) h.md_len = 0;
    bool ok = h.version <= 1;
    if (ok && h.md_len)
        ok = h.md_len <= MH_MAX_TX_METADATA_LEN && have_blob &&
             (uint64_t)h.md_off + h.md_len <= md_blob_len;
    if (!ok) {
        h.version = 1;
        h.md_len = 0;
    }
    hfix[j] = h;
    hashable[j] = ok;
}

__device__ __forceinline__ bool eq32(const uint8_t *a, const uint8_t *b) {
    bool e = true;
    for (int k = 0; k < 32; k++) e &= a[k] == b[k];
    return e;
}

// Steps 3-4 per document (verification.go:112-183) after the entry search
// (status) and the htree roots, and the arguments of its dual proof
// (:185-194 -> VerifyDualProofV2, verification.go:305-372).
__global__ __launch_bounds__(256) void k_doc_state(
    uint64_t n, const mh_tx_header *__restrict__ tx_raw, const mh_tx_header *__restrict__ h3,
    const uint8_t *__restrict__ hashable,
    const uint8_t *__restrict__ alh3, const uint8_t *__restrict__ roots,
    const uint64_t *__restrict__ known_id, const uint8_t *__restrict__ known_alh,
    int32_t *__restrict__ status, uint64_t *__restrict__ ii, uint64_t *__restrict__ ij,
    uint64_t *__restrict__ ci, uint8_t *__restrict__ sel, uint8_t *__restrict__ sbl,
    uint8_t *__restrict__ tbl) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n) return;
    const mh_tx_header &tx = h3[d], &sh = h3[n + d], &th = h3[2 * n + d];
    const uint8_t *xalh = alh3 + 32 * d, *salh = alh3 + 32 * (n + d), *talh = alh3 + 32 * (2 * n + d);
    // step 3 (:112-139): the caller's tx header (h3 holds the prepared copies)
    int32_t s = status[d];
    if (s == MH_OK && tx_raw[d].version > 1) s = MH_ERR_UNSUPPORTED_TX_VERSION;  // :118-121
    if (s == MH_OK && !eq32(roots + 32 * d, tx_raw[d].eh)) s = MH_ERR_INVALID_PROOF;  // :137-139
    const uint64_t srcid = sh.id, tgtid = th.id, id = tx.id;
    if (s == MH_OK) {
        if (tgtid < srcid) {
            s = MH_ERR_INVALID_PROOF;  // :146-148
        } else if (!hashable[n + d] || !hashable[2 * n + d]) {
            s = MH_ERR_ILLEGAL_ARGUMENTS;  // :150-151
        } else if (id != srcid && id != tgtid) {
            s = MH_ERR_INVALID_PROOF;  // :153-155
        } else if (!hashable[d]) {
            s = MH_ERR_ILLEGAL_ARGUMENTS;
        } else if ((id == srcid && !eq32(xalh, salh)) || (id == tgtid && !eq32(xalh, talh))) {
            s = MH_ERR_INVALID_PROOF;  // :157-163
        } else if (known_id[d] == 0) {
            if (srcid != 1) s = MH_ERR_INVALID_PROOF;  // :165-168
        } else {
            const uint64_t k = known_id[d];
            const uint8_t *ka = known_alh + 32 * d;
            if (k != srcid && k != tgtid)
                s = MH_ERR_INVALID_PROOF;  // :170-172
            else if ((k == srcid && !eq32(ka, salh)) || (k == tgtid && !eq32(ka, talh)))
                s = MH_ERR_INVALID_PROOF;  // :174-180
        }
        // VerifyDualProofV2's argument checks (:305-316): sourceID 0; target <
        // source and unhashable headers are already out, and both Alh values
        // passed are the headers' own, so its Alh checks (:318-326) hold
        if (s == MH_OK && srcid == 0) s = MH_ERR_ILLEGAL_ARGUMENTS;
    }
    status[d] = s;
    ii[d] = srcid;  // :342-348
    ij[d] = th.bl_tx_id;
    sel[d] = srcid == 1;  // :354-370
    ci[d] = srcid == 1 ? srcid : sh.bl_tx_id;
    for (int k = 0; k < 32; k++) {
        sbl[32 * d + k] = sh.bl_root[k];
        tbl[32 * d + k] = th.bl_root[k];
    }
}

// The rest of VerifyDualProofV2 (:328-370) and the new state's Alh.
__global__ __launch_bounds__(256) void k_doc_final(uint64_t n, const mh_tx_header *__restrict__ h3,
                                                   const uint8_t *__restrict__ alh3,
                                                   const uint8_t *__restrict__ oki,
                                                   const uint8_t *__restrict__ okc,
                                                   int32_t *__restrict__ status,
                                                   uint8_t *__restrict__ talh_out) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n) return;
    const mh_tx_header &sh = h3[n + d], &th = h3[2 * n + d];
    int32_t s = status[d];
    if (s == MH_OK) {
        if (sh.id - 1 != sh.bl_tx_id || th.id - 1 != th.bl_tx_id)
            s = MH_ERR_UNEXPECTED_LINKING;  // :328-330
        else if (sh.id == th.id)
            s = MH_OK;  // :332-334
        else if (!oki[d])
            s = MH_ERR_INCLUSION_NOT_VALID;
        else if (!okc[d])
            s = MH_ERR_CONSISTENCY_NOT_VALID;
    }
    status[d] = s;
    const uint8_t *talh = alh3 + 32 * (2 * n + d);
    for (int k = 0; k < 32; k++) talh_out[32 * d + k] = s == MH_OK ? talh[k] : 0;
}

}  // namespace

extern "C" int mh_verify_document_batch(mh_ctx *c, const mh_document_batch *B, int32_t *status,
                                        uint8_t *target_alh_out) {
    return mh_guard([&]() -> int {
        if (!c || !B || (B->n && !status)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t n = B->n;
        if (!n) return MH_OK;
        if (!B->doc_off || !B->doc_key_off || !B->tx_hdr || !B->ent_off || !B->ekey_off ||
            !B->ehval || !B->src_hdr || !B->tgt_hdr || !B->incl_off || !B->cons_off ||
            !B->known_tx_id || !B->known_alh)
            return MH_ERR_ILLEGAL_ARGUMENTS;
        // the extents first: every copy below reads [first, last) of an
        // array; that every offset in between is in order is checked on the
        // host while the copies run, before any kernel reads through them
        if (B->doc_off[n] < B->doc_off[0] || B->doc_key_off[n] < B->doc_key_off[0] ||
            B->ent_off[n] < B->ent_off[0] || B->incl_off[n] < B->incl_off[0] ||
            B->cons_off[n] < B->cons_off[0])
            return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t E = B->ent_off[n] - B->ent_off[0];
        if (E && (B->ekey_off[B->ent_off[n]] < B->ekey_off[B->ent_off[0]] ||
                  (B->emd_off && B->emd_off[B->ent_off[n]] < B->emd_off[B->ent_off[0]])))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((B->doc_off[n] > B->doc_off[0] && !B->doc) ||
            (B->doc_key_off[n] > B->doc_key_off[0] && !B->doc_key) ||
            (E && B->ekey_off[B->ent_off[n]] > B->ekey_off[B->ent_off[0]] && !B->ekeys) ||
            (B->emd_off && E && B->emd_off[B->ent_off[n]] > B->emd_off[B->ent_off[0]] && !B->emd))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        const uint64_t e0 = B->ent_off[0];

        // One upload of the caller's arrays as they are (offsets unrebased: the
        // device base pointers are shifted instead), then every step on the
        // device:
        //  1. SHA256(EncodedDocument) vs the HValue of the document's entry (:60-76)
        //  3. htree over EntrySpecDigestFor(version), IsValueTruncated (:112-139):
        //     the fused entry kernel (k_entries_varlen) takes each entry's HValue
        //     as the hVal override and the digest version per entry, one htree
        //     per document.
        //     v1: EntrySpecDigest_v1 (store/verification.go:264-302) =
        //         SHA256(BE16 mdLen || md || BE16 kLen || key || HashValue)
        //     v0: EntrySpecDigest_v0 (:256-262) = SHA256(key || SHA256(Value));
        //         VerifyDocument leaves Value nil, so SHA256(Value) = SHA256(nil)
        //         whatever the entry's HValue (and its metadata is not hashed).
        //     Only a batch that mixes v0 and v1 documents stages per-entry
        //     versions and hVals.
        //  4. header checks, Alh of the tx / source / target headers, the known
        //     state (:141-183)
        //  5. VerifyDualProofV2 (:185-194)
        bool any_v0 = false;
        for (uint64_t d = 0; d < n && !any_v0; d++) any_v0 = B->tx_hdr[d].version == 0;
        const uint64_t k0 = E ? B->ekey_off[e0] : 0, kb = E ? B->ekey_off[e0 + E] - k0 : 0;
        const bool has_md = B->emd_off != nullptr;
        const uint64_t m0 = (has_md && E) ? B->emd_off[e0] : 0,
                       mb = (has_md && E) ? B->emd_off[e0 + E] - m0 : 0;
        const uint64_t dc0 = B->doc_off[0], dcb = B->doc_off[n] - dc0;
        const uint64_t dk0 = B->doc_key_off[0], dkb = B->doc_key_off[n] - dk0;
        const uint64_t i0 = B->incl_off[0], ni = B->incl_off[n] - i0;
        const uint64_t c0 = B->cons_off[0], nc = B->cons_off[n] - c0;
        if ((ni && !B->incl_terms) || (nc && !B->cons_terms)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t mdl = B->md_blob ? B->md_blob_len : 0;
        const uint64_t hb = n * sizeof(mh_tx_header);
        std::lock_guard<std::mutex> lk(c->mu);
        hipStream_t st = c->stream;
        Layout L;
        const uint64_t b_k = L.add(std::max<uint64_t>(kb, 16)), b_m = L.add(mb),
                       b_ko = L.add((E + 1) * 8), b_mo = L.add(has_md ? (E + 1) * 8 : 0),
                       b_hv = L.add(E * 32), b_ov = L.add(any_v0 ? E * 32 : 0),
                       b_ver = L.add(any_v0 ? E : 0), b_dig = L.add(std::max<uint64_t>(E, 1) * 32),
                       b_r = L.add(n * 32), b_doc = L.add(std::max<uint64_t>(dcb, 16)),
                       b_doff = L.add((n + 1) * 8), b_dk = L.add(std::max<uint64_t>(dkb, 16)),
                       b_dko = L.add((n + 1) * 8), b_eo = L.add((n + 1) * 8),
                       b_hdoc = L.add(n * 32), b_st = L.add(n * 4),
                       b_sort = L.add(sha_varlen_scratch_bytes(n)),
                       // steps 4-5
                       b_h3r = L.add(3 * hb), b_h3 = L.add(3 * hb), b_hok = L.add(3 * n),
                       b_md = L.add(std::max<uint64_t>(mdl, 16)), b_hs = L.add(3 * n * kTxInnerStride),
                       b_alh = L.add(3 * n * 32), b_kid = L.add(n * 8), b_kalh = L.add(n * 32),
                       b_io = L.add((n + 1) * 8), b_it = L.add(std::max<uint64_t>(ni, 1) * 32),
                       b_co = L.add((n + 1) * 8), b_ct = L.add(std::max<uint64_t>(nc, 1) * 32),
                       b_ii = L.add(n * 8), b_ij = L.add(n * 8), b_ci = L.add(n * 8),
                       b_sel = L.add(n), b_sbl = L.add(n * 32), b_tbl = L.add(n * 32),
                       b_leaf = L.add(n * 32), b_ca = L.add(n * 32), b_oki = L.add(n),
                       b_okc = L.add(n), b_ta = L.add(n * 32);
        // the caller's arrays: one copy each, or -- when they all lie in one
        // pinned allocation (the shim's packing arena) with little between
        // them -- ONE copy of the whole span, each array then addressed inside
        // it
        struct Up {
            uint64_t off;
            const uint8_t *src;
            uint64_t bytes;
        };
        std::vector<Up> ups;
        auto add = [&](uint64_t off, const void *src, uint64_t bytes) {
            ups.push_back(Up{off, static_cast<const uint8_t *>(src), src ? bytes : 0});
        };
        add(b_doc, B->doc + dc0, dcb);
        add(b_doff, B->doc_off, (n + 1) * 8);
        add(b_dk, B->doc_key + dk0, dkb);
        add(b_dko, B->doc_key_off, (n + 1) * 8);
        add(b_eo, B->ent_off, (n + 1) * 8);
        if (E) {
            add(b_k, B->ekeys + k0, kb);
            add(b_m, B->emd + m0, mb);
            add(b_ko, B->ekey_off + e0, (E + 1) * 8);
            if (has_md) add(b_mo, B->emd_off + e0, (E + 1) * 8);
            add(b_hv, B->ehval + 32 * e0, E * 32);
        }
        add(b_h3r, B->tx_hdr, hb);
        add(b_h3r + hb, B->src_hdr, hb);
        add(b_h3r + 2 * hb, B->tgt_hdr, hb);
        add(b_md, B->md_blob, mdl);
        add(b_kid, B->known_tx_id, n * 8);
        add(b_kalh, B->known_alh, n * 32);
        add(b_io, B->incl_off, (n + 1) * 8);
        add(b_co, B->cons_off, (n + 1) * 8);
        add(b_it, B->incl_terms ? B->incl_terms + 32 * i0 : nullptr, ni * 32);
        add(b_ct, B->cons_terms ? B->cons_terms + 32 * c0 : nullptr, nc * 32);
        const uint8_t *lo = nullptr, *hi = nullptr;
        uint64_t sum = 0;
        for (const Up &u : ups)
            if (u.bytes) {
                lo = lo ? std::min(lo, u.src) : u.src;
                hi = hi ? std::max(hi, u.src + u.bytes) : u.src + u.bytes;
                sum += u.bytes;
            }
        const uint8_t *alo = lo ? reinterpret_cast<const uint8_t *>((uintptr_t)lo & ~(uintptr_t)255) : nullptr;
        const bool arena = lo && (uint64_t)(hi - alo) <= sum + sum / 4 + (1u << 20) &&
                           pinned_same_alloc(alo, hi - 1);
        const uint64_t b_span = L.add(arena ? (uint64_t)(hi - alo) : 0);
        MH_HIP(c->s_msgs.ensure(L.total));
        uint8_t *base = c->s_msgs.as<uint8_t>();
        // the device address of the array uploaded to layout slot off
        auto dp = [&](uint64_t off) -> uint8_t * {
            if (arena)
                for (const Up &u : ups)
                    if (u.off == off && u.bytes) return base + b_span + (u.src - alo);
            return base + off;
        };
        {
            // which upload ran shows in the context's timing records
            // (mh_ctx_timing "doc_upload_arena" / "doc_upload_arrays")
            TimerScope ts(c->tm(), arena ? "doc_upload_arena" : "doc_upload_arrays", st);
            if (arena) {
                MH_HIP(hipMemcpyAsync(base + b_span, alo, (uint64_t)(hi - alo), hipMemcpyHostToDevice, st));
            } else {
                for (const Up &u : ups)
                    if (u.bytes) MH_HIP(hipMemcpyAsync(base + u.off, u.src, u.bytes, hipMemcpyHostToDevice, st));
            }
        }
        // every offset in order (host, under the copies; branch-free loops)
        {
            bool bad = false;
            for (uint64_t d = 0; d < n; d++)
                bad |= (B->doc_off[d + 1] < B->doc_off[d]) | (B->doc_key_off[d + 1] < B->doc_key_off[d]) |
                       (B->ent_off[d + 1] < B->ent_off[d]) | (B->incl_off[d + 1] < B->incl_off[d]) |
                       (B->cons_off[d + 1] < B->cons_off[d]);
            const uint64_t *ko = B->ekey_off, *mo = B->emd_off;
            for (uint64_t e = e0; e < e0 + E; e++) bad |= ko[e + 1] < ko[e];
            if (mo)
                for (uint64_t e = e0; e < e0 + E; e++) bad |= mo[e + 1] < mo[e];
            if (bad) {
                MH_HIP(hipStreamSynchronize(st));  // the copies read the caller's arrays
                return MH_ERR_ILLEGAL_ARGUMENTS;
            }
        }
        std::vector<uint64_t> leaf_off(n + 1);
        for (uint64_t d = 0; d <= n; d++) leaf_off[d] = B->ent_off[d] - e0;
        std::vector<uint8_t> ov, ver;
        if (any_v0 && E) {
            ov.resize(E * 32);
            ver.resize(E);
            for (uint64_t d = 0; d < n; d++) {
                const uint8_t v = B->tx_hdr[d].version == 0 ? 0 : 1;
                for (uint64_t e = B->ent_off[d]; e < B->ent_off[d + 1]; e++) {
                    ver[e - e0] = v;
                    memcpy(&ov[32 * (e - e0)], v ? B->ehval + 32 * e : kEmptyRoot, 32);
                }
            }
            MH_HIP(hipMemcpyAsync(base + b_ov, ov.data(), E * 32, hipMemcpyHostToDevice, st));
            MH_HIP(hipMemcpyAsync(base + b_ver, ver.data(), E, hipMemcpyHostToDevice, st));
        }
        const unsigned g1 = (unsigned)((n + 255) / 256), g3 = (unsigned)((3 * n + 255) / 256);
        // 1.
        MH_HIP(launch_sha256_csr(st, c->tm(), dp(b_doc) - dc0, (const uint64_t *)dp(b_doff),
                                 n, nullptr, nullptr, base + b_hdoc, base + b_sort));
        hipLaunchKernelGGL(k_doc_find, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, n,
                           (const uint64_t *)dp(b_eo), dp(b_dk) - dk0,
                           (const uint64_t *)dp(b_dko), dp(b_k) - k0,
                           (const uint64_t *)dp(b_ko) - e0, dp(b_hv), base + b_hdoc,
                           (int32_t *)(base + b_st));
        MH_HIP(hipGetLastError());
        // 3.
        if (E)
            MH_HIP(launch_entries_varlen(st, c->tm(), 1, E, dp(b_k) - k0,
                                         (const uint64_t *)dp(b_ko),
                                         has_md ? dp(b_m) - m0 : nullptr,
                                         has_md ? (const uint64_t *)dp(b_mo) : nullptr,
                                         nullptr, nullptr, any_v0 ? base + b_ov : dp(b_hv),
                                         nullptr, nullptr, base + b_dig, false, nullptr,
                                         any_v0 ? base + b_ver : nullptr));
        if (int e = build_many_dev(c, st, n, leaf_off.data(), base + b_dig, base + b_r,
                                   c->s_digests, c->s_offs))
            return e;
        // 4.
        const mh_tx_header *htx = reinterpret_cast<const mh_tx_header *>(dp(b_h3r)),
                           *hsrc = reinterpret_cast<const mh_tx_header *>(dp(b_h3r + hb)),
                           *htgt = reinterpret_cast<const mh_tx_header *>(dp(b_h3r + 2 * hb));
        mh_tx_header *h3 = reinterpret_cast<mh_tx_header *>(base + b_h3);
        hipLaunchKernelGGL(k_doc_hdr_prep, dim3(g3), dim3(256), 0, st, n, htx, hsrc, htgt,
                           mdl, B->md_blob != nullptr ? 1 : 0, h3, base + b_hok);
        MH_HIP(hipGetLastError());
        MH_HIP(launch_tx_alh(st, c->tm(), 3 * n, h3, dp(b_md), nullptr, base + b_hs, nullptr,
                             nullptr, nullptr, base + b_alh, nullptr));
        hipLaunchKernelGGL(k_doc_state, dim3(g1), dim3(256), 0, st, n, htx, h3, base + b_hok,
                           base + b_alh, base + b_r, (const uint64_t *)dp(b_kid),
                           dp(b_kalh), (int32_t *)(base + b_st), (uint64_t *)(base + b_ii),
                           (uint64_t *)(base + b_ij), (uint64_t *)(base + b_ci), base + b_sel,
                           base + b_sbl, base + b_tbl);
        MH_HIP(hipGetLastError());
        // 5. leafFor(sourceAlh) (verification.go:346) and the two ahtree proofs
        //    for every document (a document already failed keeps its status);
        //    the caller's term offsets, the terms' base shifted by the first
        MH_HIP(launch_leaf_for(st, c->tm(), n, base + b_alh + 32 * n, base + b_leaf));
        MH_HIP(launch_ahtree_verify(st, c->tm(), MH_AHT_INCLUSION, n, (const uint64_t *)(base + b_ii),
                                    (const uint64_t *)(base + b_ij), (const uint64_t *)dp(b_io),
                                    dp(b_it) - 32 * i0, base + b_leaf, base + b_tbl,
                                    base + b_oki, nullptr));
        MH_HIP(launch_select32(st, n, base + b_sel, base + b_leaf, base + b_sbl, base + b_ca));
        MH_HIP(launch_ahtree_verify(st, c->tm(), MH_AHT_CONSISTENCY, n,
                                    (const uint64_t *)(base + b_ci), (const uint64_t *)(base + b_ij),
                                    (const uint64_t *)dp(b_co), dp(b_ct) - 32 * c0,
                                    base + b_ca, base + b_tbl, base + b_okc, nullptr));
        hipLaunchKernelGGL(k_doc_final, dim3(g1), dim3(256), 0, st, n, h3, base + b_alh,
                           base + b_oki, base + b_okc, (int32_t *)(base + b_st), base + b_ta);
        MH_HIP(hipGetLastError());
        MH_HIP(hipMemcpyAsync(status, base + b_st, n * 4, hipMemcpyDeviceToHost, st));
        if (target_alh_out)
            MH_HIP(hipMemcpyAsync(target_alh_out, base + b_ta, n * 32, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}
