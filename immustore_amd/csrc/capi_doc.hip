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
// Steps 1, 3, 4 and 5 run here: SHA-256 of the documents and the entry
// search, the entry-spec digests (fused entry kernel, HValues as hVal
// overrides) and the per-document htrees, the header Alh values and the dual
// proofs all on the device; the caller's arrays go up as they are and the host
// combines verdicts in the reference's order.
#include "capi_internal.hpp"

namespace {

// VerifyDocument :60-76 per document (one lane): among the tx's entries
// [ent_off[d], ent_off[d+1]) exactly one has the document's encoded key, and
// its HValue is SHA256(EncodedDocument) -- a match whose HValue differs ends
// the search at once (:63-67).  Key / offset arrays are the caller's
// (unrebased offsets, base pointers shifted by the caller's first offset).
__global__ __launch_bounds__(256) void k_doc_find(uint64_t n, const uint64_t *__restrict__ ent_off,
                                                  const uint8_t *__restrict__ dkeys,
                                                  const uint64_t *__restrict__ dkey_off,
                                                  const uint8_t *__restrict__ ekeys,
                                                  const uint64_t *__restrict__ ekey_off,
                                                  const uint8_t *__restrict__ ehval,
                                                  const uint8_t *__restrict__ hdoc,
                                                  int32_t *__restrict__ status) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n) return;
    const uint8_t *k = dkeys + dkey_off[d];
    const uint64_t kl = dkey_off[d + 1] - dkey_off[d];
    int found = 0;
    for (uint64_t e = ent_off[d]; e < ent_off[d + 1]; e++) {
        if (ekey_off[e + 1] - ekey_off[e] != kl) continue;
        const uint8_t *q = ekeys + ekey_off[e];
        bool eq = true;
        for (uint64_t j = 0; j < kl && eq; j++) eq = q[j] == k[j];
        if (!eq) continue;
        bool same = true;
        for (int j = 0; j < 32 && same; j++) same = ehval[32 * (e - ent_off[0]) + j] == hdoc[32 * d + j];
        if (!same) {
            found = -1;
            break;
        }
        found++;
    }
    status[d] = found == 1 ? MH_OK : MH_ERR_INVALID_PROOF_ENTRY;
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
        const uint64_t E = B->ent_off[n] - B->ent_off[0];
        if ((B->doc_off[n] > B->doc_off[0] && !B->doc) ||
            (B->doc_key_off[n] > B->doc_key_off[0] && !B->doc_key) ||
            (E && B->ekey_off[B->ent_off[n]] > B->ekey_off[B->ent_off[0]] && !B->ekeys) ||
            (B->emd_off && E && B->emd_off[B->ent_off[n]] > B->emd_off[B->ent_off[0]] && !B->emd))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        for (uint64_t d = 0; d < n; d++)
            if (B->doc_off[d + 1] < B->doc_off[d] || B->doc_key_off[d + 1] < B->doc_key_off[d] ||
                B->ent_off[d + 1] < B->ent_off[d] || B->incl_off[d + 1] < B->incl_off[d] ||
                B->cons_off[d + 1] < B->cons_off[d])
                return MH_ERR_ILLEGAL_ARGUMENTS;
        for (uint64_t e = B->ent_off[0]; e < B->ent_off[n]; e++)
            if (B->ekey_off[e + 1] < B->ekey_off[e] ||
                (B->emd_off && B->emd_off[e + 1] < B->emd_off[e]))
                return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        for (uint64_t d = 0; d < n; d++) status[d] = MH_OK;
        const uint64_t e0 = B->ent_off[0];

        // ---- 1 + 3 on the device, one upload of the caller's arrays as they
        // are (offsets unrebased: the device base pointers are shifted instead)
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
        std::vector<uint8_t> roots(n * 32);
        {
            bool any_v0 = false;
            for (uint64_t d = 0; d < n && !any_v0; d++) any_v0 = B->tx_hdr[d].version == 0;
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
            }
            const uint64_t k0 = E ? B->ekey_off[e0] : 0, kb = E ? B->ekey_off[e0 + E] - k0 : 0;
            const bool has_md = B->emd_off != nullptr;
            const uint64_t m0 = (has_md && E) ? B->emd_off[e0] : 0,
                           mb = (has_md && E) ? B->emd_off[e0 + E] - m0 : 0;
            const uint64_t dc0 = B->doc_off[0], dcb = B->doc_off[n] - dc0;
            const uint64_t dk0 = B->doc_key_off[0], dkb = B->doc_key_off[n] - dk0;
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
                           b_sort = L.add(sha_varlen_scratch_bytes(n));
            MH_HIP(c->s_msgs.ensure(L.total));
            uint8_t *base = c->s_msgs.as<uint8_t>();
            auto up = [&](uint64_t off, const void *src, uint64_t bytes) -> hipError_t {
                return bytes ? hipMemcpyAsync(base + off, src, bytes, hipMemcpyHostToDevice, st)
                             : hipSuccess;
            };
            MH_HIP(up(b_doc, B->doc + dc0, dcb));
            MH_HIP(up(b_doff, B->doc_off, (n + 1) * 8));
            MH_HIP(up(b_dk, B->doc_key + dk0, dkb));
            MH_HIP(up(b_dko, B->doc_key_off, (n + 1) * 8));
            MH_HIP(up(b_eo, B->ent_off, (n + 1) * 8));
            if (E) {
                MH_HIP(up(b_k, B->ekeys + k0, kb));
                MH_HIP(up(b_m, B->emd + m0, mb));
                MH_HIP(up(b_ko, B->ekey_off + e0, (E + 1) * 8));
                if (has_md) MH_HIP(up(b_mo, B->emd_off + e0, (E + 1) * 8));
                MH_HIP(up(b_hv, B->ehval + 32 * e0, E * 32));
                if (any_v0) {
                    MH_HIP(up(b_ov, ov.data(), E * 32));
                    MH_HIP(up(b_ver, ver.data(), E));
                }
            }
            // 1.
            MH_HIP(launch_sha256_csr(st, c->tm(), base + b_doc - dc0, (const uint64_t *)(base + b_doff),
                                     n, nullptr, nullptr, base + b_hdoc, base + b_sort));
            hipLaunchKernelGGL(k_doc_find, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n,
                               (const uint64_t *)(base + b_eo), base + b_dk - dk0,
                               (const uint64_t *)(base + b_dko), base + b_k - k0,
                               (const uint64_t *)(base + b_ko) - e0, base + b_hv, base + b_hdoc,
                               (int32_t *)(base + b_st));
            MH_HIP(hipGetLastError());
            // 3.
            if (E)
                MH_HIP(launch_entries_varlen(st, c->tm(), 1, E, base + b_k - k0,
                                             (const uint64_t *)(base + b_ko),
                                             has_md ? base + b_m - m0 : nullptr,
                                             has_md ? (const uint64_t *)(base + b_mo) : nullptr,
                                             nullptr, nullptr, any_v0 ? base + b_ov : base + b_hv,
                                             nullptr, nullptr, base + b_dig, false, nullptr,
                                             any_v0 ? base + b_ver : nullptr));
            if (int e = build_many_dev(c, st, n, leaf_off.data(), base + b_dig, base + b_r,
                                       c->s_digests, c->s_offs))
                return e;
            MH_HIP(hipMemcpyAsync(roots.data(), base + b_r, n * 32, hipMemcpyDeviceToHost, st));
            MH_HIP(hipMemcpyAsync(status, base + b_st, n * 4, hipMemcpyDeviceToHost, st));
            MH_HIP(hipStreamSynchronize(st));
        }
        for (uint64_t d = 0; d < n; d++) {
            if (status[d] == MH_OK && B->tx_hdr[d].version > 1)
                status[d] = MH_ERR_UNSUPPORTED_TX_VERSION;  // :118-121
            if (status[d] == MH_OK && memcmp(&roots[32 * d], B->tx_hdr[d].eh, 32))
                status[d] = MH_ERR_INVALID_PROOF;  // :137-139
        }

        // ---- 4. headers and known state (:141-183)
        // Alh of the tx, source and target headers; a header that cannot be
        // hashed (version not 0/1, bad metadata) makes Go's innerHash panic --
        // reported as MH_ERR_ILLEGAL_ARGUMENTS, its Alh is not computed.
        std::vector<mh_tx_header> hh(3 * n);
        std::vector<uint8_t> hashable(3 * n);
        for (uint64_t d = 0; d < n; d++) {
            const mh_tx_header *src3[3] = {&B->tx_hdr[d], &B->src_hdr[d], &B->tgt_hdr[d]};
            for (int k = 0; k < 3; k++) {
                hh[k * n + d] = *src3[k];
                // a v0 innerHash never reads the metadata (tx.go:258-263)
                if (hh[k * n + d].version == 0) hh[k * n + d].md_len = 0;
                hashable[k * n + d] =
                    check_header(hh[k * n + d], B->md_blob_len, B->md_blob != nullptr) == MH_OK;
                if (!hashable[k * n + d]) {
                    hh[k * n + d].version = 1;
                    hh[k * n + d].md_len = 0;
                }
            }
        }
        std::vector<uint8_t> alh(3 * n * 32);
        if (int e = mh_tx_alh_batch(c, 3 * n, hh.data(), B->md_blob, B->md_blob_len, nullptr,
                                    alh.data()))
            return e;
        const uint8_t *xalh = alh.data(), *salh = alh.data() + n * 32, *talh = alh.data() + 2 * n * 32;
        for (uint64_t d = 0; d < n; d++) {
            if (status[d] != MH_OK) continue;
            const uint64_t src = B->src_hdr[d].id, tgt = B->tgt_hdr[d].id, id = B->tx_hdr[d].id;
            int32_t s = MH_OK;
            if (tgt < src) {
                s = MH_ERR_INVALID_PROOF;  // :146-148
            } else if (!hashable[n + d] || !hashable[2 * n + d]) {
                s = MH_ERR_ILLEGAL_ARGUMENTS;  // :150-151
            } else if (id != src && id != tgt) {
                s = MH_ERR_INVALID_PROOF;  // :153-155
            } else if (!hashable[d]) {
                s = MH_ERR_ILLEGAL_ARGUMENTS;
            } else if ((id == src && memcmp(xalh + 32 * d, salh + 32 * d, 32)) ||
                       (id == tgt && memcmp(xalh + 32 * d, talh + 32 * d, 32))) {
                s = MH_ERR_INVALID_PROOF;  // :157-163
            } else if (B->known_tx_id[d] == 0) {
                if (src != 1) s = MH_ERR_INVALID_PROOF;  // :165-168
            } else {
                const uint64_t k = B->known_tx_id[d];
                const uint8_t *ka = B->known_alh + 32 * d;
                if (k != src && k != tgt)
                    s = MH_ERR_INVALID_PROOF;  // :170-172
                else if ((k == src && memcmp(ka, salh + 32 * d, 32)) ||
                         (k == tgt && memcmp(ka, talh + 32 * d, 32)))
                    s = MH_ERR_INVALID_PROOF;  // :174-180
            }
            status[d] = s;
        }

        // ---- 5. VerifyDualProofV2(proof, sourceID, targetID, sourceAlh, targetAlh) (:185-194)
        std::vector<uint64_t> sel;
        for (uint64_t d = 0; d < n; d++)
            if (status[d] == MH_OK) sel.push_back(d);
        if (!sel.empty()) {
            const uint64_t m = sel.size();
            std::vector<mh_tx_header> sh(m), th(m);
            std::vector<uint64_t> io(m + 1, 0), co(m + 1, 0), sv(m), tv(m);
            std::vector<uint8_t> it, ct, sa(m * 32), ta(m * 32);
            std::vector<int32_t> st(m);
            for (uint64_t k = 0; k < m; k++) {
                const uint64_t d = sel[k];
                sh[k] = hh[n + d];
                th[k] = hh[2 * n + d];
                sv[k] = sh[k].id;
                tv[k] = th[k].id;
                memcpy(&sa[32 * k], salh + 32 * d, 32);
                memcpy(&ta[32 * k], talh + 32 * d, 32);
                const uint64_t ni = B->incl_off[d + 1] - B->incl_off[d];
                const uint64_t nc = B->cons_off[d + 1] - B->cons_off[d];
                if ((ni && !B->incl_terms) || (nc && !B->cons_terms)) return MH_ERR_ILLEGAL_ARGUMENTS;
                if (ni) it.insert(it.end(), B->incl_terms + 32 * B->incl_off[d],
                                  B->incl_terms + 32 * B->incl_off[d + 1]);
                if (nc) ct.insert(ct.end(), B->cons_terms + 32 * B->cons_off[d],
                                  B->cons_terms + 32 * B->cons_off[d + 1]);
                io[k + 1] = io[k] + ni;
                co[k + 1] = co[k] + nc;
            }
            if (int e = mh_verify_dual_proof_v2_batch(
                    c, m, sh.data(), th.data(), B->md_blob, B->md_blob_len, io.data(),
                    it.empty() ? nullptr : it.data(), co.data(), ct.empty() ? nullptr : ct.data(),
                    sv.data(), tv.data(), sa.data(), ta.data(), st.data()))
                return e;
            for (uint64_t k = 0; k < m; k++) status[sel[k]] = st[k];
        }
        if (target_alh_out)
            for (uint64_t d = 0; d < n; d++) {
                if (status[d] == MH_OK)
                    memcpy(target_alh_out + 32 * d, talh + 32 * d, 32);
                else
                    memset(target_alh_out + 32 * d, 0, 32);
            }
        return MH_OK;
    });
}
