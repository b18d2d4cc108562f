/*
 * mh_client.c -- the C-ABI boundary exercised from plain C, the way the cgo
 * shim of INTEGRATION.md calls it (no Python, no torch): build an htree over
 * digests (htree.New / BuildWith / Root / InclusionProof + VerifyInclusion),
 * append a batch to an ahtree (Append / RootAt / InclusionProof /
 * ConsistencyProof) on one device and across devices (mh_multi_*), and
 * print the results as hex for the test to compare with the oracle.  Input digests / payloads: SHA-256-free deterministic
 * bytes (x[k] = (k * 131 + 7) & 0xff), so the test can rebuild them.
 *
 * usage: mh_client <width> <appends>
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "immustore_merkle.h"

static void hex(const char *tag, const uint8_t *p, size_t n) {
    printf("%s ", tag);
    for (size_t k = 0; k < n; k++) printf("%02x", p[k]);
    printf("\n");
}

#define CHECK(x)                                                            \
    do {                                                                    \
        int st_ = (x);                                                      \
        if (st_ != MH_OK) {                                                 \
            fprintf(stderr, "%s -> %d (%s)\n", #x, st_, mh_status_string(st_)); \
            return 1;                                                       \
        }                                                                   \
    } while (0)

int main(int argc, char **argv) {
    const uint64_t w = argc > 1 ? strtoull(argv[1], 0, 10) : 1000;
    const uint64_t m = argc > 2 ? strtoull(argv[2], 0, 10) : 777;
    uint8_t *d = malloc(w * 32), *p = malloc(m * 32);
    for (uint64_t k = 0; k < w * 32; k++) d[k] = (uint8_t)((k * 131 + 7) & 0xff);
    for (uint64_t k = 0; k < m * 32; k++) p[k] = (uint8_t)((k * 29 + 3) & 0xff);
    printf("abi %d\n", mh_abi_version());

    mh_ctx *ctx;
    CHECK(mh_ctx_create(0, NULL, &ctx));

    /* htree: New / BuildWith / Root / InclusionProof / VerifyInclusion */
    mh_htree *t;
    CHECK(mh_htree_new(ctx, w, &t));
    CHECK(mh_htree_build_with(t, d, w));
    uint8_t root[32];
    CHECK(mh_htree_root(t, root));
    hex("htree_root", root, 32);
    int bad = mh_htree_build_with(t, d, w + 1);  /* ErrMaxWidthExceeded */
    printf("max_width_exceeded %d\n", bad == MH_ERR_MAX_WIDTH_EXCEEDED);
    CHECK(mh_htree_build_with(t, d, w));
    uint8_t terms[64 * 32];
    uint32_t nt = 0;
    const uint64_t leaf = w / 3;
    CHECK(mh_htree_inclusion_proof(t, leaf, terms, 64, &nt));
    hex("htree_proof", terms, nt * 32u);
    uint64_t lf = leaf, wd = w, off[2] = {0, nt};
    uint8_t ok = 0;
    CHECK(mh_htree_verify_inclusion_batch(ctx, 1, &lf, &wd, off, terms, d + leaf * 32, root, &ok));
    printf("htree_verify %d\n", ok);
    terms[5] ^= 1;
    CHECK(mh_htree_verify_inclusion_batch(ctx, 1, &lf, &wd, off, terms, d + leaf * 32, root, &ok));
    printf("htree_verify_tampered %d\n", ok);
    CHECK(mh_htree_free(t));

    /* ahtree: AppendBatch / RootAt / proofs */
    mh_ahtree *a;
    CHECK(mh_ahtree_new(ctx, &a));
    CHECK(mh_ahtree_append_batch(a, p, m, 32, NULL));
    uint64_t n = 0;
    uint8_t r[32];
    CHECK(mh_ahtree_root(a, &n, r));
    printf("ahtree_size %llu\n", (unsigned long long)n);
    hex("ahtree_root", r, 32);
    uint8_t at[32];
    CHECK(mh_ahtree_root_at(a, m / 2, at));
    hex("ahtree_root_half", at, 32);
    uint8_t pt[128 * 32];
    uint32_t pn = 0;
    CHECK(mh_ahtree_inclusion_proof(a, m / 3, m, pt, 128, &pn));
    hex("ahtree_incl", pt, pn * 32u);
    CHECK(mh_ahtree_consistency_proof(a, m / 2, m, pt, 128, &pn));
    hex("ahtree_cons", pt, pn * 32u);
    printf("empty_root_at %d\n", mh_ahtree_root_at(a, m + 1, at) == MH_ERR_UNEXISTENT_DATA);
    const uint64_t nd = mh_ahtree_nodes_upto(m);
    uint8_t *dl1 = malloc(nd * 32), *dl2 = malloc(nd * 32);
    CHECK(mh_ahtree_dlog(a, 0, nd, dl1));
    CHECK(mh_ahtree_free(a));

    /* multi-GPU ahtree AppendBatch (SURVEY.md 8(e), C3 at scale): device 0 as an
     * RCCL clique of one, then listed three times; dLog and RootAt(m) must
     * equal the single-device append above */
    {
        const int one[1] = {0}, three[3] = {0, 0, 0};
        const int *devs[2] = {one, three};
        const int ndv[2] = {1, 3};
        for (int v = 0; v < 2; v++) {
            mh_multi *mm;
            CHECK(mh_multi_create(ndv[v], devs[v], &mm));
            uint8_t mr[32];
            memset(dl2, 0, nd * 32);
            CHECK(mh_multi_ahtree_append_batch(mm, 0, NULL, p, m, 32, dl2, mr));
            printf("%s %d\n", v ? "multi3_ahtree_root_equal" : "multi1_ahtree_root_equal",
                   memcmp(mr, r, 32) == 0);
            printf("%s %d\n", v ? "multi3_ahtree_dlog_equal" : "multi1_ahtree_dlog_equal",
                   memcmp(dl1, dl2, nd * 32) == 0);
            CHECK(mh_multi_destroy(mm));
        }
    }
    free(dl1);
    free(dl2);

    /* multi-GPU htree over entries: an RCCL clique over
     * device 0, then device 0 listed three times (three shards, roots
     * gathered by device copies); entries: key = BE64(k), 64-byte values =
     * the ahtree payload bytes p[2k .. 2k+2) (m >= 2w required, else skipped) */
    if (m >= 2 * w) {
        uint8_t *keys = malloc(w * 8);
        for (uint64_t k = 0; k < w; k++)
            for (int b = 0; b < 8; b++) keys[k * 8 + b] = (uint8_t)(k >> (56 - 8 * b));
        const int one[1] = {0}, three[3] = {0, 0, 0};
        const int *devs[2] = {one, three};
        const int nd[2] = {1, 3};
        for (int v = 0; v < 2; v++) {
            mh_multi *mm;
            CHECK(mh_multi_create(nd[v], devs[v], &mm));
            uint8_t mroot[32];
            CHECK(mh_multi_htree_build_entries_fixed(mm, 1, w, keys, 8, p, 64, NULL, NULL, mroot));
            hex(v ? "multi3_root" : "multi1_root", mroot, 32);
            CHECK(mh_multi_destroy(mm));
        }
        free(keys);
    }
    /* ragged entries (value hash loop + Tx.BuildHashTree, immustore.go:1620-1630,
     * tx.go:332-355) through mh_htree_build_entries: CSR keys / KV metadata /
     * values of varying length, every 5th entry with an IsValueTruncated hVal
     * override; v1 (with metadata) and v0 (without).  Entry e (ne = w):
     *   key   len 1 + (7e mod 40),  byte j = (13e + 5j + 1) & 0xff
     *   md    e%4: none | 00 | 02 | 01 BE64(e)
     *   value len (37e mod 700),    byte j = (3e + 11j) & 0xff
     *   ovr   e%5==0: byte j = (e + j) & 0xff */
    {
        const uint64_t ne = w;
        uint64_t *ko = malloc((ne + 1) * 8), *mo = malloc((ne + 1) * 8), *vo = malloc((ne + 1) * 8);
        ko[0] = mo[0] = vo[0] = 0;
        for (uint64_t e = 0; e < ne; e++) {
            ko[e + 1] = ko[e] + 1 + (7 * e) % 40;
            mo[e + 1] = mo[e] + (e % 4 == 0 ? 0 : e % 4 == 3 ? 9 : 1);
            vo[e + 1] = vo[e] + (37 * e) % 700;
        }
        uint8_t *kb = malloc(ko[ne] + 1), *mb = malloc(mo[ne] + 1), *vb = malloc(vo[ne] + 1);
        uint8_t *ov = malloc(ne * 32), *use = malloc(ne), *hv = malloc(ne * 32);
        for (uint64_t e = 0; e < ne; e++) {
            for (uint64_t j = 0; j < ko[e + 1] - ko[e]; j++) kb[ko[e] + j] = (uint8_t)(13 * e + 5 * j + 1);
            for (uint64_t j = 0; j < vo[e + 1] - vo[e]; j++) vb[vo[e] + j] = (uint8_t)(3 * e + 11 * j);
            uint8_t *m = mb + mo[e];
            if (e % 4 == 1) m[0] = 0x00;
            if (e % 4 == 2) m[0] = 0x02;
            if (e % 4 == 3) {
                m[0] = 0x01;
                for (int b = 0; b < 8; b++) m[1 + b] = (uint8_t)(e >> (56 - 8 * b));
            }
            for (int j = 0; j < 32; j++) ov[e * 32 + j] = (uint8_t)(e + j);
            use[e] = e % 5 == 0;
        }
        mh_htree *et;
        CHECK(mh_htree_new(ctx, ne, &et));
        uint8_t er[32];
        CHECK(mh_htree_build_entries(et, 1, ne, kb, ko, mb, mo, vb, vo, ov, use, hv));
        CHECK(mh_htree_root(et, er));
        hex("entries_v1_root", er, 32);
        hex("entries_v1_hval_mid", hv + (ne / 2) * 32, 32);
        hex("entries_v1_hval_last", hv + (ne - 1) * 32, 32);
        CHECK(mh_htree_build_entries(et, 0, ne, kb, ko, NULL, NULL, vb, vo, NULL, NULL, NULL));
        CHECK(mh_htree_root(et, er));
        hex("entries_v0_root", er, 32);
        printf("entries_v0_md_rejected %d\n",
               mh_htree_build_entries(et, 0, ne, kb, ko, mb, mo, vb, vo, NULL, NULL, NULL) ==
                   (mo[ne] ? MH_ERR_METADATA_UNSUPPORTED : MH_OK));
        if (ne >= 2) {
            const uint64_t save = vo[1];
            vo[1] = vo[2] + 1; /* offsets running backwards */
            printf("entries_backwards_rejected %d\n",
                   mh_htree_build_entries(et, 1, ne, kb, ko, mb, mo, vb, vo, NULL, NULL, NULL) ==
                       MH_ERR_ILLEGAL_ARGUMENTS);
            vo[1] = save;
        }
        CHECK(mh_htree_free(et));
        free(ko); free(mo); free(vo); free(kb); free(mb); free(vb); free(ov); free(use); free(hv);
    }
    {
        /* A self-consistent store, built the way ImmuStore does it: tx k's header
         * links the tree of the first k-1 Alh values (BlTxID k-1, BlRoot), its
         * Alh is appended next.  Then DualProofV2 messages over it
         * (mh_ahtree_dual_proof_v2_pb_batch, the server side) checked by the
         * client side in one call (mh_verify_dual_proof_v2_pb_batch). */
        const uint64_t ntx = 64, np = 40;
        mh_tx_header *h = calloc(ntx, sizeof(mh_tx_header));
        uint8_t *alh = malloc(ntx * 32), inner[32];
        mh_ahtree *st;
        CHECK(mh_ahtree_new(ctx, &st));
        for (uint64_t k = 0; k < ntx; k++) {
            h[k].id = k + 1;
            h[k].ts = (int64_t)(1700000000 + k);
            h[k].bl_tx_id = k;
            h[k].version = 1;
            h[k].nentries = (uint32_t)(1 + k % 7);
            for (int j = 0; j < 32; j++) {
                h[k].eh[j] = (uint8_t)(k * 7 + j);
                h[k].prev_alh[j] = k ? alh[(k - 1) * 32 + j] : 0;
            }
            if (k) CHECK(mh_ahtree_root_at(st, k, h[k].bl_root));
            CHECK(mh_tx_alh_batch(ctx, 1, &h[k], NULL, 0, inner, alh + k * 32));
            CHECK(mh_ahtree_append_batch(st, alh + k * 32, 1, 32, NULL));
        }
        mh_tx_header *sh = malloc(np * sizeof(mh_tx_header)), *th = malloc(np * sizeof(mh_tx_header));
        uint64_t *si = malloc(np * 8), *ti = malloc(np * 8), *off = malloc((np + 1) * 8);
        uint8_t *sa = malloc(np * 32), *ta = malloc(np * 32);
        int32_t *pst = malloc(np * 4), *vst = malloc(np * 4);
        for (uint64_t q = 0; q < np; q++) {
            ti[q] = 2 + (q * 37) % (ntx - 1);
            si[q] = 1 + (q * 11) % ti[q];
            sh[q] = h[si[q] - 1];
            th[q] = h[ti[q] - 1];
            memcpy(sa + q * 32, alh + (si[q] - 1) * 32, 32);
            memcpy(ta + q * 32, alh + (ti[q] - 1) * 32, 32);
        }
        uint64_t cap = 0;
        int r = mh_ahtree_dual_proof_v2_pb_batch(st, np, sh, th, NULL, 0, NULL, 0, off, pst);
        if (r != MH_ERR_BUFFER_TOO_SMALL && r != MH_OK) CHECK(r);
        cap = off[np];
        uint8_t *msgs = malloc(cap ? cap : 1);
        CHECK(mh_ahtree_dual_proof_v2_pb_batch(st, np, sh, th, NULL, 0, msgs, cap, off, pst));
        CHECK(mh_verify_dual_proof_v2_pb_batch(ctx, np, msgs, off, si, ti, sa, ta, vst));
        uint64_t good = 0;
        for (uint64_t q = 0; q < np; q++) good += pst[q] == MH_OK && vst[q] == MH_OK;
        printf("wire_verify_ok %llu/%llu\n", (unsigned long long)good, (unsigned long long)np);
        /* a term byte of the last message flipped: that proof alone fails */
        msgs[off[np] - 1] ^= 1;
        CHECK(mh_verify_dual_proof_v2_pb_batch(ctx, np, msgs, off, si, ti, sa, ta, vst));
        good = 0;
        for (uint64_t q = 0; q + 1 < np; q++) good += vst[q] == MH_OK;
        printf("wire_verify_tampered %d %llu\n", vst[np - 1], (unsigned long long)good);
        {
            /* the same batch over a clique listing device 0 three times
             * (mh_multi_verify_dual_proof_v2_pb_batch: parts of nearly equal
             * message bytes, one per context): the single call's statuses */
            int devs3[3] = {0, 0, 0};
            mh_multi *m3;
            int32_t *mst = malloc(np * 4);
            CHECK(mh_multi_create(3, devs3, &m3));
            CHECK(mh_multi_verify_dual_proof_v2_pb_batch(m3, np, msgs, off, si, ti, sa, ta, mst));
            printf("multi3_wire_verify_equal %d\n", memcmp(mst, vst, np * 4) == 0);
            CHECK(mh_multi_destroy(m3));
            free(mst);
        }
        CHECK(mh_ahtree_free(st));
        free(h); free(alh); free(sh); free(th); free(si); free(ti); free(off); free(sa); free(ta);
        free(pst); free(vst); free(msgs);
    }
    CHECK(mh_ctx_destroy(ctx));
    free(d);
    free(p);
    printf("done\n");
    return 0;
}
