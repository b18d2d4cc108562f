/*
 * mh_client.c -- the C-ABI boundary exercised from plain C, the way the cgo
 * shim of INTEGRATION.md calls it (no Python, no torch): build an htree over
 * digests (htree.New / BuildWith / Root / InclusionProof + VerifyInclusion),
 * append a batch to an ahtree (Append / RootAt / InclusionProof /
 * ConsistencyProof), and print the results as hex for the test to compare
 * with the oracle.  Input digests / payloads: SHA-256-free deterministic
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
    CHECK(mh_ahtree_free(a));

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
    CHECK(mh_ctx_destroy(ctx));
    free(d);
    free(p);
    printf("done\n");
    return 0;
}
