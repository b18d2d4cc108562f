/* txlog_bench.c -- mh_txlog_validate through the C ABI alone, as a cgo caller
 * would drive it (no Python binding between the calls): the a14 workload of
 * bench_workloads.py --workload txlog (2^16 v1 records x 16 entries, 16-byte
 * keys, no metadata, 75.5 MB), the log and the outputs in pinned arenas
 * (mh_host_alloc_pinned).  The stored Alh of every record is sealed from a
 * first validation; after 2 s of untimed calls (GPU clock pre-warm) K calls
 * are timed one by one.  TXB_CLOG=1: mh_txlog_validate_clog over the same
 * pinned log with its commit log (12-byte entries, pinned) -- no host hop.
 *
 * usage: txlog_bench [K=50] [records=65536] [entries=16]
 * prints one JSON line. */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "immustore_merkle.h"

static uint64_t sm(uint64_t *s) { /* splitmix64 */
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static void be(uint8_t *p, uint64_t v, int n) {
    for (int k = n - 1; k >= 0; k--) p[n - 1 - k] = (uint8_t)(v >> (8 * k));
}
static void rnd(uint8_t *p, size_t n, uint64_t *s) {
    for (size_t i = 0; i < n; i++) p[i] = (uint8_t)sm(s);
}
static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}
static int cmp(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}
#define CHECK(x)                                                       \
    do {                                                               \
        int rc_ = (x);                                                 \
        if (rc_ != MH_OK) {                                            \
            fprintf(stderr, "%s: %s (%d)\n", #x, mh_status_string(rc_), rc_); \
            return 1;                                                  \
        }                                                              \
    } while (0)

int main(int argc, char **argv) {
    /* TXB_NO_HDRS=1: no header output (validation only: Alh + statuses) */
    const int nohdr = getenv("TXB_NO_HDRS") && atoi(getenv("TXB_NO_HDRS"));
    const int use_clog = getenv("TXB_CLOG") && atoi(getenv("TXB_CLOG"));
    const int K = argc > 1 ? atoi(argv[1]) : 50;
    const uint64_t ntx = argc > 2 ? strtoull(argv[2], 0, 10) : 65536;
    const uint64_t ne = argc > 3 ? strtoull(argv[3], 0, 10) : 16;
    const uint64_t kl = 16, ent = 2 + 2 + kl + 4 + 8 + 32, hdr = 96, rec = hdr + ne * ent + 32;
    const uint64_t len = ntx * rec;
    mh_ctx *c = NULL;
    CHECK(mh_ctx_create(0, NULL, &c));
    uint8_t *log = NULL, *alh = NULL, *clog = NULL;
    mh_tx_header *hd = NULL;
    int32_t *st = NULL;
    CHECK(mh_host_alloc_pinned(len, (void **)&log));
    CHECK(mh_host_alloc_pinned(ntx * 32, (void **)&alh));
    CHECK(mh_host_alloc_pinned(ntx * sizeof(mh_tx_header), (void **)&hd));
    CHECK(mh_host_alloc_pinned(ntx * 4, (void **)&st));
    CHECK(mh_host_alloc_pinned(ntx * 12, (void **)&clog));
    for (uint64_t t = 0; t < ntx; t++) { /* txOffsetAndSize (immustore.go:2569-2597) */
        be(clog + t * 12, t * rec, 8);
        be(clog + t * 12 + 8, rec, 4);
    }
    uint64_t s = 14;
    for (uint64_t t = 0; t < ntx; t++) {
        uint8_t *r = log + t * rec;
        memset(r, 0, rec);
        be(r, t + 1, 8);                   /* id */
        be(r + 8, 1666885208ull + t, 8);   /* ts */
        be(r + 16, t, 8);                  /* blTxId */
        rnd(r + 24, 64, &s);               /* blRoot, prevAlh */
        be(r + 88, 1, 2);                  /* version 1, mdLen 0 */
        be(r + 92, ne, 4);                 /* nentries */
        for (uint64_t e = 0; e < ne; e++) {
            uint8_t *q = r + hdr + e * ent;
            be(q + 2, kl, 2);
            rnd(q + 4, kl, &s);
            be(q + 4 + kl, 100, 4);
            be(q + 8 + kl, sm(&s) & 0xffffffffffull, 8);
            rnd(q + 16 + kl, 32, &s);
        }
    }
    uint64_t n = 0, used = 0;
    /* seal: the stored Alh of every record is the one validation recomputes */
    mh_txlog_validate(c, log, len, 1024, 1024, ntx, &n, &used, NULL, alh, st);
    for (uint64_t t = 0; t < ntx; t++) memcpy(log + t * rec + rec - 32, alh + t * 32, 32);
    double *ms = malloc(sizeof(double) * (size_t)K);
    uint64_t nbad = 0, first = 0;
#define CALL()                                                                                    \
    (use_clog ? mh_txlog_validate_clog(c, log, len, clog, ntx, 12, 1024, 1024, nohdr ? NULL : hd, \
                                       alh, st, &nbad, &first)                                    \
              : mh_txlog_validate(c, log, len, 1024, 1024, ntx, &n, &used, nohdr ? NULL : hd, alh, st))
    /* clock pre-warm: calls for 2 s first (as bench_workloads.py --prewarm) */
    for (const double tw = now(); now() - tw < 2.0;) CHECK(CALL());
    for (int k = 0; k < K; k++) {
        const double t0 = now();
        CHECK(CALL());
        ms[k] = (now() - t0) * 1e3;
    }
    int bad = 0;
    for (uint64_t t = 0; t < ntx; t++) bad += st[t] != MH_OK;
    if (use_clog) { /* the cLog call reports no count / consumed bytes */
        bad += (int)nbad + (first != ntx);
        n = ntx;
        used = len;
    }
    qsort(ms, (size_t)K, sizeof(double), cmp);
    double sum = 0;
    for (int k = 0; k < K; k++) sum += ms[k];
    printf("{\"metric\": \"tx-log read-path validation (a14) through the C ABI\", \"records\": %llu, "
           "\"entries_per_record\": %llu, \"log_bytes\": %llu, \"calls\": %d, \"ms_median\": %.4f, "
           "\"ms_min\": %.4f, \"ms_mean\": %.4f, \"M_tx_per_s_median\": %.3f, \"ntx\": %llu, "
           "\"consumed\": %llu, \"invalid\": %d, \"pinned\": true, \"headers_out\": %s, \"api\": \"%s\"}\n",
           (unsigned long long)ntx, (unsigned long long)ne, (unsigned long long)len, K, ms[K / 2],
           ms[0], sum / K, ntx / (ms[K / 2] * 1e-3) / 1e6, (unsigned long long)n,
           (unsigned long long)used, bad, nohdr ? "false" : "true",
           use_clog ? "mh_txlog_validate_clog" : "mh_txlog_validate");
    free(ms);
    mh_host_free_pinned(log);
    mh_host_free_pinned(alh);
    mh_host_free_pinned(hd);
    mh_host_free_pinned(st);
    mh_host_free_pinned(clog);
    mh_ctx_destroy(c);
    return bad != 0 || n != ntx || used != len;
}
