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
// Steps 1, 3, 4 and 5 run here: SHA-256 of the documents, the entry-spec
// digests and the per-document htrees, the header Alh values and the dual
// proofs all on the device (capi_tx.hip's batch entry points); the host packs
// messages and combines verdicts in the reference's order.
#include "capi_internal.hpp"

namespace {

// SHA-256 of n host byte ranges buf[off[i] .. off[i+1]) on the device.
int sha_batch_host(mh_ctx *c, const uint8_t *buf, const std::vector<uint64_t> &off, uint8_t *out) {
    const uint64_t n = off.size() - 1;
    if (!n) return MH_OK;
    const uint64_t bytes = off[n] - off[0];
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = c->stream;
    Layout L;
    const uint64_t b_buf = L.add(std::max<uint64_t>(bytes, 16)), b_off = L.add((n + 1) * 8),
                   b_out = L.add(n * 32), b_sort = L.add(sha_varlen_scratch_bytes(n));
    MH_HIP(c->s_msgs.ensure(L.total));
    uint8_t *base = c->s_msgs.as<uint8_t>();
    std::vector<uint64_t> rel(n + 1);
    for (uint64_t i = 0; i <= n; i++) rel[i] = off[i] - off[0];
    if (bytes) MH_HIP(hipMemcpyAsync(base + b_buf, buf + off[0], bytes, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(base + b_off, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
    MH_HIP(launch_sha256_csr(st, c->tm(), base + b_buf, (const uint64_t *)(base + b_off), n,
                             nullptr, nullptr, base + b_out, base + b_sort));
    MH_HIP(hipMemcpyAsync(out, base + b_out, n * 32, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    return MH_OK;
}

inline void put16(std::vector<uint8_t> &v, uint64_t x) {
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
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
                B->ent_off[d + 1] < B->ent_off[d])
                return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        for (uint64_t d = 0; d < n; d++) status[d] = MH_OK;
        const uint64_t e0 = B->ent_off[0];

        // ---- 1. SHA256(EncodedDocument) vs the HValue of the document's entry (:60-76)
        std::vector<uint64_t> doff(B->doc_off, B->doc_off + n + 1);
        std::vector<uint8_t> hdoc(n * 32);
        if (int e = sha_batch_host(c, B->doc, doff, hdoc.data())) return e;
        for (uint64_t d = 0; d < n; d++) {
            const uint8_t *k = B->doc_key + B->doc_key_off[d];
            const uint64_t kl = B->doc_key_off[d + 1] - B->doc_key_off[d];
            int found = 0;
            for (uint64_t e = B->ent_off[d]; e < B->ent_off[d + 1]; e++) {
                const uint64_t el = B->ekey_off[e + 1] - B->ekey_off[e];
                if (el != kl || (kl && memcmp(B->ekeys + B->ekey_off[e], k, kl))) continue;
                if (memcmp(B->ehval + 32 * e, &hdoc[32 * d], 32)) {
                    found = -1;  // hash mismatch: returned at once (:63-67)
                    break;
                }
                found++;
            }
            if (found != 1) status[d] = MH_ERR_INVALID_PROOF_ENTRY;
        }

        // ---- 3. htree over EntrySpecDigestFor(version), IsValueTruncated (:112-139)
        //   v1: EntrySpecDigest_v1 (store/verification.go:264-302) =
        //       SHA256(BE16 mdLen || md || BE16 kLen || key || HashValue)
        //   v0: EntrySpecDigest_v0 (:256-262) = SHA256(key || SHA256(Value));
        //       VerifyDocument leaves Value nil, so SHA256(Value) = SHA256(nil)
        //       whatever the entry's HValue (and its metadata is not hashed).
        std::vector<uint8_t> msg;
        std::vector<uint64_t> moff(1, 0);
        std::vector<uint64_t> leaf_off(n + 1, 0);
        for (uint64_t d = 0; d < n; d++) {
            const uint32_t ver = B->tx_hdr[d].version;
            if (status[d] == MH_OK && ver > 1) status[d] = MH_ERR_UNSUPPORTED_TX_VERSION;
            const bool hash = status[d] == MH_OK;
            for (uint64_t e = B->ent_off[d]; hash && e < B->ent_off[d + 1]; e++) {
                const uint8_t *key = B->ekeys ? B->ekeys + B->ekey_off[e] : nullptr;
                const uint64_t kl = B->ekey_off[e + 1] - B->ekey_off[e];
                if (ver == 1) {
                    const uint64_t ml = B->emd_off ? B->emd_off[e + 1] - B->emd_off[e] : 0;
                    put16(msg, ml);
                    if (ml) msg.insert(msg.end(), B->emd + B->emd_off[e], B->emd + B->emd_off[e] + ml);
                    put16(msg, kl);
                    if (kl) msg.insert(msg.end(), key, key + kl);
                    msg.insert(msg.end(), B->ehval + 32 * e, B->ehval + 32 * e + 32);
                } else {
                    if (kl) msg.insert(msg.end(), key, key + kl);
                    msg.insert(msg.end(), kEmptyRoot, kEmptyRoot + 32);
                }
                moff.push_back(msg.size());
            }
            leaf_off[d + 1] = moff.size() - 1;
        }
        (void)e0;
        const uint64_t nd = moff.size() - 1;
        std::vector<uint8_t> digs(std::max<uint64_t>(nd, 1) * 32), roots(n * 32);
        if (nd)
            if (int e = sha_batch_host(c, msg.data(), moff, digs.data())) return e;
        if (int e = mh_htree_build_many(c, n, leaf_off.data(), digs.data(), roots.data())) return e;
        for (uint64_t d = 0; d < n; d++)
            if (status[d] == MH_OK && memcmp(&roots[32 * d], B->tx_hdr[d].eh, 32))
                status[d] = MH_ERR_INVALID_PROOF;

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
