/* queue_bench.c -- group commit (mh_commit_queue) under MaxConcurrency
 * committers, as immudb runs precommit (immustore.go:1620-1632, up to
 * options.go:35 DefaultMaxConcurrency = 30 goroutines hashing their own tx
 * before the store lock at :1689).
 *
 * T threads each submit K single transactions of E entries (8-byte keys
 * BE64, V-byte values, v1 digests) and block on their own result; reported:
 * txs/s over the whole run, p50 / p99 / max latency of one submit, batches
 * formed.  Beside it, the same transactions hashed by the oracle (the C
 * restatement in oracle/, SHA-NI when present) on T host threads -- a
 * reported CPU baseline -- and every Eh compared with the oracle's.
 *
 * usage: queue_bench [T=30] [K=2000] [E=16] [V=1024] [wait_us=50] [max_txs=64]
 * prints one JSON line. */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "immustore_merkle.h"

int orc_build_entries(int version, uint64_t n, const uint8_t *keys, const uint64_t *key_off,
                      const uint8_t *md, const uint64_t *md_off, const uint8_t *vals,
                      const uint64_t *val_off, const uint8_t *hval_override,
                      const uint8_t *use_override, uint8_t *hvals_out, uint8_t *levels,
                      uint8_t root[32]);

static int T = 30, K = 2000, E = 16, V = 1024;
static mh_commit_queue *Q;

typedef struct {
    int t;
    uint8_t *keys, *vals;  /* per thread: K txs x E entries */
    uint64_t *koff, *voff; /* E + 1 offsets, shared shape */
    uint8_t *eh_gpu, *eh_cpu;
    double *lat;
    int err;
} job;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static uint64_t splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void *gpu_worker(void *arg) {
    job *j = (job *)arg;
    uint8_t hv[64 * 32];
    for (int k = 0; k < K; k++) {
        const double t0 = now();
        int st = mh_commit_queue_submit(Q, (uint64_t)E, j->keys + (size_t)k * E * 8, j->koff, NULL,
                                        NULL, j->vals + (size_t)k * E * V, j->voff, NULL, NULL, NULL,
                                        hv, j->eh_gpu + (size_t)k * 32);
        j->lat[k] = now() - t0;
        if (st != MH_OK) j->err = st;
    }
    return NULL;
}

static void *cpu_worker(void *arg) {
    job *j = (job *)arg;
    uint8_t hv[64 * 32];
    uint8_t *lv = malloc(2 * 64 * 32 + 64);
    for (int k = 0; k < K; k++) {
        const double t0 = now();
        int st = orc_build_entries(1, (uint64_t)E, j->keys + (size_t)k * E * 8, j->koff, NULL, NULL,
                                   j->vals + (size_t)k * E * V, j->voff, NULL, NULL, hv, lv,
                                   j->eh_cpu + (size_t)k * 32);
        j->lat[k] = now() - t0;
        if (st) j->err = st;
    }
    free(lv);
    return NULL;
}

static int cmpd(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static void run(void *(*fn)(void *), job *J, double *wall, double *p50, double *p99, double *mx) {
    pthread_t th[256];
    const double t0 = now();
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, fn, &J[t]);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    *wall = now() - t0;
    double *all = malloc(sizeof(double) * (size_t)T * K);
    for (int t = 0; t < T; t++) memcpy(all + (size_t)t * K, J[t].lat, sizeof(double) * K);
    qsort(all, (size_t)T * K, sizeof(double), cmpd);
    *p50 = all[(size_t)T * K / 2];
    *p99 = all[(size_t)T * K * 99 / 100];
    *mx = all[(size_t)T * K - 1];
    free(all);
}

int main(int argc, char **argv) {
    int wait_us = 50, max_txs = 64;
    if (argc > 1) T = atoi(argv[1]);
    if (argc > 2) K = atoi(argv[2]);
    if (argc > 3) E = atoi(argv[3]);
    if (argc > 4) V = atoi(argv[4]);
    if (argc > 5) wait_us = atoi(argv[5]);
    if (argc > 6) max_txs = atoi(argv[6]);
    if (T < 1 || T > 256 || K < 1 || E < 1 || E > 64 || V < 0) return 2;
    mh_ctx *ctx;
    int st = mh_ctx_create(0, NULL, &ctx);
    if (st) {
        fprintf(stderr, "mh_ctx_create: %d\n", st);
        return 1;
    }
    st = mh_commit_queue_new(ctx, 1, (uint64_t)E, (uint32_t)max_txs, (uint32_t)wait_us, &Q);
    if (st) {
        fprintf(stderr, "mh_commit_queue_new: %d\n", st);
        return 1;
    }
    job *J = calloc((size_t)T, sizeof(job));
    uint64_t koff[65], voff[65];
    for (int e = 0; e <= E; e++) {
        koff[e] = (uint64_t)e * 8;
        voff[e] = (uint64_t)e * V;
    }
    for (int t = 0; t < T; t++) {
        job *j = &J[t];
        j->t = t;
        j->keys = malloc((size_t)K * E * 8);
        j->vals = malloc((size_t)K * E * V + 8);
        j->koff = koff;
        j->voff = voff;
        j->eh_gpu = malloc((size_t)K * 32);
        j->eh_cpu = malloc((size_t)K * 32);
        j->lat = malloc(sizeof(double) * K);
        uint64_t s = 1000 + t;
        for (size_t b = 0; b < (size_t)K * E * V; b += 8) {
            const uint64_t x = splitmix(&s);
            memcpy(j->vals + b, &x, 8);
        }
        for (int k = 0; k < K; k++)
            for (int e = 0; e < E; e++) {
                const uint64_t id = ((uint64_t)t << 40) | ((uint64_t)k * E + e);
                for (int b = 0; b < 8; b++) j->keys[((size_t)k * E + e) * 8 + b] = (uint8_t)(id >> (56 - 8 * b));
            }
    }
    /* warm-up: one tx per thread through the queue */
    {
        uint8_t hv[64 * 32], eh[32];
        for (int t = 0; t < T; t++)
            mh_commit_queue_submit(Q, (uint64_t)E, J[t].keys, koff, NULL, NULL, J[t].vals, voff, NULL,
                                   NULL, NULL, hv, eh);
    }
    uint64_t b0 = 0, x0 = 0, b1 = 0, x1 = 0;
    mh_commit_queue_stats(Q, &b0, &x0);
    double gw, g50, g99, gmx, cw, c50, c99, cmx;
    run(gpu_worker, J, &gw, &g50, &g99, &gmx);
    mh_commit_queue_stats(Q, &b1, &x1);
    run(cpu_worker, J, &cw, &c50, &c99, &cmx);
    int match = 1, err = 0;
    for (int t = 0; t < T; t++) {
        if (memcmp(J[t].eh_gpu, J[t].eh_cpu, (size_t)K * 32)) match = 0;
        if (J[t].err) err = J[t].err;
    }
    const double ntx = (double)T * K;
    printf("{\"metric\": \"group commit: single-tx precommit hashing from %d committer threads\", "
           "\"threads\": %d, \"txs_per_thread\": %d, \"entries_per_tx\": %d, \"value_len\": %d, "
           "\"wait_us\": %d, \"max_txs\": %d, "
           "\"gpu\": {\"txs_per_s\": %.0f, \"gib_per_s\": %.3f, \"p50_us\": %.1f, \"p99_us\": %.1f, "
           "\"max_us\": %.1f, \"batches\": %llu, \"mean_batch_txs\": %.2f}, "
           "\"cpu_baseline\": {\"kind\": \"port\", \"cores\": %d, \"txs_per_s\": %.0f, "
           "\"gib_per_s\": %.3f, \"p50_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f}, "
           "\"eh_match\": %s, \"status\": %d}\n",
           T, T, K, E, V, wait_us, max_txs, ntx / gw, ntx * E * V / gw / (1u << 30), g50 * 1e6,
           g99 * 1e6, gmx * 1e6, (unsigned long long)(b1 - b0),
           (double)(x1 - x0) / (double)(b1 - b0 ? b1 - b0 : 1), T, ntx / cw,
           ntx * E * V / cw / (1u << 30), c50 * 1e6, c99 * 1e6, cmx * 1e6, match ? "true" : "false",
           err);
    mh_commit_queue_free(Q);
    mh_ctx_destroy(ctx);
    return (match && !err) ? 0 : 1;
}
