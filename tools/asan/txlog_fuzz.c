/* txlog_fuzz.c -- mutation fuzzing of the tx-log record hop (mh_txlog_scan,
 * the host parse of mh_txlog_validate: tx.go:419-603, kv_metadata.go:207-256,
 * tx_metadata.go:159-193) against the oracle's sequential parse
 * (orc_txlog_validate), both built with AddressSanitizer (host code only:
 * tools/asan/Makefile).  Test infrastructure: the oracle is the checker.
 *
 * Every mutant lives in a malloc of exactly its length, so a read one byte
 * past the record run is reported by ASan.  Mutations: bit flips, bytes set
 * to 0x00 / 0xff, BE16 / BE32 length fields overwritten with extreme values,
 * truncation, a splice of another part of the log, a record repeated.
 * For each mutant: (status, ntx, consumed) of the two parses must agree.
 *
 * With MH_FUZZ_DEVICE=1 (on a GPU box) every mutant also goes through
 * mh_txlog_validate -- the device path: raw records to the device, headers,
 * entry digests, trees and Alh rebuilt there, the canonical-metadata side
 * area -- and its status, record count, consumed bytes, Alh values and
 * per-tx statuses must equal the oracle's.  The host code around it still
 * runs under ASan (the device code is built as usual).  Each mutant then goes
 * through mh_txlog_validate_clog too, indexed by the CLEAN log's commit log
 * (12- or 44-byte entries, some of them mutated: sizes, offsets), with the
 * mutant in device memory and in host memory (its exact-size malloc: ASan
 * sees any host over-read of the fallback), against orc_clog below -- the
 * oracle's readTx restatement (oracle.py txlog_validate_clog) in C.
 *
 * usage: txlog_fuzz <iterations per file> <seed> <log file>...
 * prints one line per file; exit 1 on any mismatch. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "immustore_merkle.h"

int orc_txlog_validate(const uint8_t *buf, uint64_t len, uint32_t max_entries, uint32_t max_key_len,
                       uint64_t max_txs, uint64_t *ntx_out, uint64_t *consumed_out,
                       uint8_t *alh_out, int32_t *status_out);

static uint64_t S;
static uint64_t rnd(void) {
    uint64_t z = (S += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint8_t *load(const char *path, uint64_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc(n ? (size_t)n : 1);
    if (n && fread(b, 1, (size_t)n, f) != (size_t)n) n = 0;
    fclose(f);
    *len = (uint64_t)n;
    return b;
}

/* one mutant of src into a fresh exact-size buffer */
static uint8_t *mutate(const uint8_t *src, uint64_t len, uint64_t *out_len) {
    uint64_t n = len;
    uint8_t *b = malloc(n ? n : 1);
    memcpy(b, src, n);
    const int k = 1 + (int)(rnd() % 4);
    for (int m = 0; m < k && n; m++) {
        const uint64_t p = rnd() % n;
        switch (rnd() % 7) {
        case 0: b[p] ^= (uint8_t)(1u << (rnd() % 8)); break;
        case 1: b[p] = 0xff; break;
        case 2: b[p] = 0x00; break;
        case 3: /* a BE16 length field at an extreme */
            if (p + 2 <= n) {
                static const uint16_t v[] = {0, 1, 11, 12, 255, 256, 257, 1024, 1025, 0xffff};
                const uint16_t x = v[rnd() % 10];
                b[p] = (uint8_t)(x >> 8);
                b[p + 1] = (uint8_t)x;
            }
            break;
        case 4: /* a BE32 field at an extreme */
            if (p + 4 <= n) {
                static const uint32_t v[] = {0, 1, 1023, 1024, 1025, 0x10000, 0x7fffffff, 0xffffffff};
                const uint32_t x = v[rnd() % 8];
                for (int j = 0; j < 4; j++) b[p + j] = (uint8_t)(x >> (24 - 8 * j));
            }
            break;
        case 5: /* truncate */
            n = p;
            break;
        case 6: { /* splice: copy a run from elsewhere in the log over p */
            const uint64_t q = rnd() % n, l = 1 + rnd() % 256;
            for (uint64_t j = 0; j < l && p + j < n && q + j < n; j++) b[p + j] = src[q + j < len ? q + j : 0];
            break;
        }
        }
    }
    uint8_t *e = malloc(n ? n : 1); /* exact size: ASan sees any over-read */
    memcpy(e, b, n);
    free(b);
    *out_len = n;
    return e;
}

static mh_ctx *CTX;  /* MH_FUZZ_DEVICE=1: mh_txlog_validate as well */

static uint64_t be_n(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int k = 0; k < n; k++) v = v << 8 | p[k];
    return v;
}

/* ImmuStore.readTx (immustore.go:3048-3060) of entry t of the cLog: the record
 * read at its offset on to the end of the log, plus the open path's cLog
 * checks (:458-528) -- oracle.py txlog_validate_clog */
static void orc_clog(const uint8_t *b, uint64_t n, const uint8_t *cl, uint64_t ntx, int es,
                     uint32_t me, uint32_t mk, uint8_t *alh, int32_t *sts) {
    for (uint64_t t = 0; t < ntx; t++) {
        const uint64_t off = be_n(cl + t * es, 8), size = be_n(cl + t * es + 8, 4);
        memset(alh + 32 * t, 0, 32);
        if (off > n || n - off < 8) {
            sts[t] = MH_ERR_TRUNCATED;
            continue;
        }
        uint64_t k = 0, used = 0;
        uint8_t a[32];
        int32_t s1 = 0;
        int st = orc_txlog_validate(b + off, n - off, me, mk, 1, &k, &used, a, &s1);
        if (st == MH_OK && k == 0) st = MH_ERR_TRUNCATED;
        if (st == MH_OK && used != size) st = MH_ERR_CORRUPTED_DATA;
        if (st == MH_OK && es == 44 && memcmp(cl + t * es + 12, b + off + size - 32, 32)) st = MH_ERR_CORRUPTED_DATA;
        if (st == MH_OK) {
            sts[t] = s1;
            memcpy(alh + 32 * t, a, 32);
        } else {
            sts[t] = st;
        }
    }
}

/* the clean log's commit log (offset, size, Alh per record), from the scan */
static uint8_t *CL;
static uint64_t CL_N;
static void clean_clog(const uint8_t *src, uint64_t len) {
    free(CL);
    CL = NULL;
    CL_N = 0;
    const uint64_t cap = len / 90 + 1;
    uint64_t *ao = malloc(8 * cap), nt = 0, c = 0;
    mh_txlog_scan(src, len, 1024, 1024, cap, &nt, &c, NULL, ao);
    CL = malloc(44 * (nt ? nt : 1));
    for (uint64_t t = 0; t < nt; t++) {
        const uint64_t s0 = t ? ao[t - 1] + 32 : 0, e = ao[t] + 32;
        for (int k = 0; k < 8; k++) CL[44 * t + k] = (uint8_t)(s0 >> (56 - 8 * k));
        for (int k = 0; k < 4; k++) CL[44 * t + 8 + k] = (uint8_t)((e - s0) >> (24 - 8 * k));
        memcpy(CL + 44 * t + 12, src + e - 32, 32);
    }
    CL_N = nt;
    free(ao);
}

/* mh_txlog_validate_clog of mutant b (n bytes) vs orc_clog: the clean cLog,
 * sometimes with mutated entries; the mutant resident and in host memory */
static int check_clog(const uint8_t *b, uint64_t n, uint32_t me, uint32_t mk, long *bad) {
    if (!CL_N) return 1;
    const uint64_t nt = CL_N;
    const int es = (rnd() & 1) ? 12 : 44;
    uint8_t *cl = malloc(es * nt);
    for (uint64_t t = 0; t < nt; t++) memcpy(cl + es * t, CL + 44 * t, es);
    if (rnd() & 1) { /* a few entries that disagree with the log */
        for (int m = 0; m < 3; m++) {
            uint8_t *e = cl + es * (rnd() % nt);
            switch (rnd() % 4) {
            case 0: e[11] ^= (uint8_t)(1 + rnd() % 255); break;        /* size */
            case 1: e[7] ^= (uint8_t)(1 + rnd() % 255); break;         /* offset, low byte */
            case 2: e[8] = 0xff; break;                                 /* size past the log */
            case 3: memcpy(e, cl + es * (rnd() % nt), es); break;       /* another tx's entry */
            }
        }
    }
    uint8_t *a1 = malloc(32 * nt), *a2 = malloc(32 * nt);
    int32_t *s1 = malloc(4 * nt), *s2 = malloc(4 * nt);
    orc_clog(b, n, cl, nt, es, me, mk, a2, s2);
    uint64_t nb2 = 0, f2 = nt;
    for (uint64_t t = 0; t < nt; t++)
        if (s2[t] != MH_OK) {
            if (!nb2) f2 = t;
            nb2++;
        }
    int ok = 1;
    for (int mode = 0; mode < 2; mode++) {
        const uint8_t *src = b;
        void *d = NULL;
        if (mode == 0) { /* resident: an allocation 256 bytes longer */
            if (mh_dev_alloc(CTX, n + 256, &d) != MH_OK) return 0;
            if (n) mh_memcpy_h2d(CTX, d, b, n);
            mh_ctx_synchronize(CTX);
            src = d;
        }
        uint64_t nb1 = 0, f1 = 0;
        memset(s1, 0x55, 4 * nt);
        const int r = mh_txlog_validate_clog(CTX, n ? src : (mode ? b : src), n, cl, nt, es, me, mk,
                                             NULL, a1, s1, &nb1, &f1);
        const int same = r == MH_OK && nb1 == nb2 && f1 == f2 && !memcmp(s1, s2, 4 * nt) &&
                         !memcmp(a1, a2, 32 * nt);
        if (!same && (*bad)++ < 5)
            fprintf(stderr, "clog mismatch (%s, es %d) len %llu: rc %d nbad %llu/%llu first %llu/%llu\n",
                    mode ? "host" : "resident", es, (unsigned long long)n, r,
                    (unsigned long long)nb1, (unsigned long long)nb2, (unsigned long long)f1,
                    (unsigned long long)f2);
        ok &= same;
        if (d) mh_dev_free(CTX, d);
    }
    free(cl); free(a1); free(a2); free(s1); free(s2);
    return ok;
}

static int check_device(const uint8_t *b, uint64_t n, uint32_t me, uint32_t mk, uint64_t cap,
                        int r2, uint64_t n2, uint64_t c2, const uint8_t *alh2,
                        const int32_t *sts2, long *bad) {
    const uint64_t k = cap ? cap : 1;
    mh_tx_header *h = malloc(sizeof(mh_tx_header) * k);
    uint8_t *alh = malloc(32 * k);
    int32_t *sts = malloc(4 * k);
    uint64_t n1 = 0, c1 = 0;
    const int r1 = mh_txlog_validate(CTX, b, n, me, mk, cap, &n1, &c1, h, alh, sts);
    int ok = r1 == r2 && n1 == n2 && c1 == c2;
    if (ok && n1) ok = !memcmp(alh, alh2, 32 * n1) && !memcmp(sts, sts2, 4 * n1);
    if (!ok && (*bad)++ < 5)
        fprintf(stderr, "device mismatch len %llu: validate (%d, %llu, %llu) oracle (%d, %llu, %llu)\n",
                (unsigned long long)n, r1, (unsigned long long)n1, (unsigned long long)c1, r2,
                (unsigned long long)n2, (unsigned long long)c2);
    free(h); free(alh); free(sts);
    return ok;
}

static int check(const uint8_t *b, uint64_t n, uint32_t me, uint32_t mk, uint64_t mt, long *bad) {
    const uint64_t cap = n / 90 + 1 < mt ? n / 90 + 1 : mt;
    mh_tx_header *h = malloc(sizeof(mh_tx_header) * (cap ? cap : 1));
    uint64_t *ao = malloc(8 * (cap ? cap : 1));
    uint8_t *alh = malloc(32 * (cap ? cap : 1));
    int32_t *sts = malloc(4 * (cap ? cap : 1));
    uint64_t n1 = 0, c1 = 0, n2 = 0, c2 = 0;
    const int r1 = mh_txlog_scan(b, n, me, mk, cap, &n1, &c1, h, ao);
    const int r2 = orc_txlog_validate(b, n, me, mk, cap, &n2, &c2, alh, sts);
    int ok = r1 == r2 && n1 == n2 && c1 == c2;
    if (!ok && (*bad)++ < 5)
        fprintf(stderr, "mismatch len %llu: scan (%d, %llu, %llu) oracle (%d, %llu, %llu)\n",
                (unsigned long long)n, r1, (unsigned long long)n1, (unsigned long long)c1, r2,
                (unsigned long long)n2, (unsigned long long)c2);
    if (CTX) ok &= check_device(b, n, me, mk, cap, r2, n2, c2, alh, sts, bad);
    if (CTX && n) ok &= check_clog(b, n, me, mk, bad);
    free(h); free(ao); free(alh); free(sts);
    return ok;
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    const long iters = atol(argv[1]);
    S = strtoull(argv[2], 0, 10);
    const char *dev = getenv("MH_FUZZ_DEVICE");
    if (dev && dev[0] == '1' && mh_ctx_create(0, NULL, &CTX) != MH_OK) {
        fprintf(stderr, "MH_FUZZ_DEVICE=1 but no device context\n");
        return 2;
    }
    long bad = 0;
    for (int a = 3; a < argc; a++) {
        uint64_t len = 0;
        uint8_t *src = load(argv[a], &len);
        if (!src) {
            fprintf(stderr, "cannot read %s\n", argv[a]);
            return 2;
        }
        long agree = 0, accepted = 0;
        if (CTX) clean_clog(src, len);
        check(src, len, 1024, 1024, 1ull << 40, &bad);
        /* large logs: fewer mutants (each parse is ~ms) */
        const long it = len > (4u << 20) ? iters / 50 + 1 : iters;
        for (long i = 0; i < it; i++) {
            uint64_t n;
            uint8_t *m = mutate(src, len, &n);
            const uint32_t me = (rnd() & 3) ? 1024 : (uint32_t)(rnd() % 40);
            const uint32_t mk = (rnd() & 3) ? 1024 : (uint32_t)(rnd() % 70);
            agree += check(m, n, me, mk, 1ull << 40, &bad);
            uint64_t nt = 0, c = 0;
            if (mh_txlog_scan(m, n, me, mk, n / 90 + 1, &nt, &c, NULL, NULL) == MH_OK && nt) accepted++;
            free(m);
        }
        printf("%s: %ld mutants, %ld agree, %ld parsed >= 1 record%s\n", argv[a], it, agree,
               accepted, CTX ? " (device validate and the cLog call too)" : "");
        fflush(stdout);
        free(src);
    }
    if (CTX) {
        mh_ctx_destroy(CTX);
        /* with device allocations made (the cLog check), ASan's device
         * allocator CHECK-fails in the HIP runtime's own static destructors
         * at exit (sanitizer_allocator_device.h: dev_runtime_unloaded_), after
         * every check has passed: leave without running them */
        fflush(stdout);
        fflush(stderr);
        _exit(bad ? 1 : 0);
    }
    return bad ? 1 : 0;
}
