/*
 * mh_committers.c -- concurrent committers of precommit batches from plain C,
 * the shape of the cgo shim's store paths (go/store/precommit_mi355x.go):
 * immudb runs up to MaxConcurrency committers at once, each hashing its own
 * transactions before taking the store lock (immustore.go:1620-1632, :1689;
 * options.go:35).  A pool of `cliques` mh_multi handles (each over the listed
 * devices, default device 0) is shared by `threads` committer threads:
 * checkout, mh_multi_precommit_batch, return -- exactly the pool
 * go/internal/mi355x/device.go keeps (AcquireClique / ReleaseClique).
 *
 * Thread t's batch: ntx transactions of `entries` entries; entry e (global
 * index within the batch) has key BE64((t << 32) | e) and a vlen-byte value
 * with byte j = (7 t + 13 e + 11 j + 1) & 0xff, version 1, no metadata.
 *
 * usage: mh_committers <threads> <cliques> <rounds> <ntx> <entries> <vlen> [device ...]
 * prints per thread (last round): "eh <t> <hex of every Eh>", "hv <t> <hex of
 * the hVals of entries 0, n/2, n-1>", then "rate <GiB/s of values over all
 * threads> <seconds>" for the timed rounds (one untimed round first).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "immustore_merkle.h"

static int T, H, R, ndev = 1, devs[16] = {0};
static uint64_t NTX, NE, VLEN;

/* the clique pool: checkout / return under a mutex, waiting when every
 * handle is out */
static pthread_mutex_t pool_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t pool_cv = PTHREAD_COND_INITIALIZER;
static mh_multi *pool_free[64];
static int pool_nfree;

static mh_multi *acquire(void) {
    pthread_mutex_lock(&pool_mu);
    while (pool_nfree == 0) pthread_cond_wait(&pool_cv, &pool_mu);
    mh_multi *m = pool_free[--pool_nfree];
    pthread_mutex_unlock(&pool_mu);
    return m;
}

static void release(mh_multi *m) {
    pthread_mutex_lock(&pool_mu);
    pool_free[pool_nfree++] = m;
    pthread_cond_signal(&pool_cv);
    pthread_mutex_unlock(&pool_mu);
}

static pthread_barrier_t bar;
static double t_start, t_end;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

typedef struct {
    int t, rc;
    uint8_t *eh, *hv;
} Job;

static void *committer(void *arg) {
    Job *j = (Job *)arg;
    const int t = j->t;
    const uint64_t n = NTX * NE;
    uint8_t *keys = NULL, *vals = NULL;
    if (mh_host_alloc_pinned(n * 8, (void **)&keys) || mh_host_alloc_pinned(n * VLEN, (void **)&vals)) {
        j->rc = MH_ERR_OUT_OF_MEMORY;
        pthread_barrier_wait(&bar);
        pthread_barrier_wait(&bar);
        return NULL;
    }
    uint64_t *tx_off = malloc((NTX + 1) * 8), *key_off = malloc((n + 1) * 8), *val_off = malloc((n + 1) * 8);
    for (uint64_t k = 0; k <= NTX; k++) tx_off[k] = k * NE;
    for (uint64_t e = 0; e < n; e++) {
        const uint64_t key = ((uint64_t)t << 32) | e;
        for (int b = 0; b < 8; b++) keys[e * 8 + b] = (uint8_t)(key >> (56 - 8 * b));
        for (uint64_t q = 0; q < VLEN; q++) vals[e * VLEN + q] = (uint8_t)((7 * t + 13 * e + 11 * q + 1) & 0xff);
    }
    for (uint64_t e = 0; e <= n; e++) {
        key_off[e] = e * 8;
        val_off[e] = e * VLEN;
    }
    int32_t *st = malloc(NTX * 4);
    int rc = MH_OK;
    for (int r = 0; r <= R && rc == MH_OK; r++) {
        if (r == 1) {  /* round 0 untimed: every thread starts the timed rounds together */
            pthread_barrier_wait(&bar);
            if (t == 0) t_start = now();
        }
        mh_multi *m = acquire();
        rc = mh_multi_precommit_batch(m, 1, 0, NTX, tx_off, keys, key_off, NULL, NULL, vals, val_off,
                                      NULL, NULL, NULL, j->hv, j->eh, st);
        release(m);
        for (uint64_t k = 0; k < NTX && rc == MH_OK; k++)
            if (st[k]) rc = st[k];
    }
    pthread_barrier_wait(&bar);
    if (t == 0) t_end = now();
    j->rc = rc;
    free(st);
    free(tx_off);
    free(key_off);
    free(val_off);
    mh_host_free_pinned(keys);
    mh_host_free_pinned(vals);
    return NULL;
}

static void hex(const char *tag, int t, const uint8_t *p, size_t n) {
    printf("%s %d ", tag, t);
    for (size_t k = 0; k < n; k++) printf("%02x", p[k]);
    printf("\n");
}

int main(int argc, char **argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s threads cliques rounds ntx entries vlen [device ...]\n", argv[0]);
        return 2;
    }
    T = atoi(argv[1]);
    H = atoi(argv[2]);
    R = atoi(argv[3]);
    NTX = strtoull(argv[4], 0, 10);
    NE = strtoull(argv[5], 0, 10);
    VLEN = strtoull(argv[6], 0, 10);
    if (argc > 7) {
        ndev = 0;
        for (int k = 7; k < argc && ndev < 16; k++) devs[ndev++] = atoi(argv[k]);
    }
    if (T < 1 || T > 64 || H < 1 || H > 64 || R < 1 || !NTX || !NE) return 2;
    for (int h = 0; h < H; h++) {
        mh_multi *m;
        int rc = mh_multi_create(ndev, devs, &m);
        if (rc != MH_OK) {
            fprintf(stderr, "mh_multi_create -> %d (%s)\n", rc, mh_status_string(rc));
            return 1;
        }
        pool_free[pool_nfree++] = m;
    }
    pthread_barrier_init(&bar, NULL, (unsigned)T);
    pthread_t th[64];
    Job jobs[64];
    for (int t = 0; t < T; t++) {
        jobs[t].t = t;
        jobs[t].rc = 0;
        jobs[t].eh = malloc(NTX * 32);
        jobs[t].hv = malloc(NTX * NE * 32);
        pthread_create(&th[t], NULL, committer, &jobs[t]);
    }
    int bad = 0;
    for (int t = 0; t < T; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) {
            fprintf(stderr, "committer %d -> %d (%s)\n", t, jobs[t].rc, mh_status_string(jobs[t].rc));
            bad = 1;
        }
    }
    if (!bad) {
        const uint64_t n = NTX * NE;
        for (int t = 0; t < T; t++) {
            hex("eh", t, jobs[t].eh, NTX * 32);
            uint8_t s[96];
            memcpy(s, jobs[t].hv, 32);
            memcpy(s + 32, jobs[t].hv + (n / 2) * 32, 32);
            memcpy(s + 64, jobs[t].hv + (n - 1) * 32, 32);
            hex("hv", t, s, 96);
        }
        const double secs = t_end - t_start;
        printf("rate %.3f %.6f\n", (double)T * R * n * VLEN / secs / (double)(1ull << 30), secs);
    }
    for (int t = 0; t < T; t++) {
        free(jobs[t].eh);
        free(jobs[t].hv);
    }
    while (pool_nfree) mh_multi_destroy(pool_free[--pool_nfree]);
    return bad;
}
