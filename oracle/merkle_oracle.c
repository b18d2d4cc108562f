/*
 * merkle_oracle.c -- CPU restatement of immudb's Merkle-hash path.
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle + timed CPU baseline).  See
 * merkle_oracle.h for the pinning evidence and the import rule.  Each
 * function cites the reference file:line it follows (paths relative to the
 * immudb repository root).
 */
#include "merkle_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

enum { OK = 0, ERR_MAX_WIDTH = 1, ERR_ILLEGAL_ARGS = 2, ERR_ILLEGAL_STATE = 3, ERR_EMPTY = 4,
       ERR_UNEXISTENT = 5, ERR_MD_UNSUPPORTED = 6, ERR_SOURCE_TX_NEWER = 10,
       ERR_UNEXPECTED_LINKING = 11, ERR_INCLUSION_NOT_VALID = 12, ERR_CONSISTENCY_NOT_VALID = 13,
       ERR_CORRUPTED_DATA = 14, ERR_CORRUPTED_MAX_ENTRIES = 15, ERR_CORRUPTED_MAX_KEYLEN = 16,
       ERR_CORRUPTED_UNKNOWN_VERSION = 17, ERR_TRUNCATED = 18 };

/* ------------------------------------------------------------------ SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void blocks_portable(uint32_t st[8], const uint8_t *p, size_t nblocks) {
    while (nblocks--) {
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
                   (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
                 h = st[7];
        for (int i = 0; i < 64; i++) {
            uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) +
                          K256[i] + w[i];
            uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d;
        st[4] += e; st[5] += f; st[6] += g; st[7] += h;
        p += 64;
    }
}

#if defined(__x86_64__)
/* Intel SHA extensions (sha256rnds2 / msg1 / msg2).  Same function, ~5x the
 * portable code on one core. */
__attribute__((target("sha,sse4.1,ssse3"))) static void blocks_shani(uint32_t st[8],
                                                                      const uint8_t *p,
                                                                      size_t nblocks) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i tmp = _mm_loadu_si128((const __m128i *)&st[0]);
    __m128i s1 = _mm_loadu_si128((const __m128i *)&st[4]);
    tmp = _mm_shuffle_epi32(tmp, 0xB1);
    s1 = _mm_shuffle_epi32(s1, 0x1B);
    __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);
    s1 = _mm_blend_epi16(s1, tmp, 0xF0);
    while (nblocks--) {
        __m128i abef = s0, cdgh = s1, m[4];
        for (int g = 0; g < 16; g++) {
            __m128i w;
            if (g < 4) {
                m[g] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 16 * g)), MASK);
                w = m[g];
            } else {
                __m128i x = _mm_sha256msg1_epu32(m[g & 3], m[(g + 1) & 3]);
                x = _mm_add_epi32(x, _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4));
                m[g & 3] = _mm_sha256msg2_epu32(x, m[(g + 3) & 3]);
                w = m[g & 3];
            }
            __m128i msg = _mm_add_epi32(w, _mm_loadu_si128((const __m128i *)&K256[4 * g]));
            s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
            msg = _mm_shuffle_epi32(msg, 0x0E);
            s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
        }
        s0 = _mm_add_epi32(s0, abef);
        s1 = _mm_add_epi32(s1, cdgh);
        p += 64;
    }
    tmp = _mm_shuffle_epi32(s0, 0x1B);
    s1 = _mm_shuffle_epi32(s1, 0xB1);
    s0 = _mm_blend_epi16(tmp, s1, 0xF0);
    s1 = _mm_alignr_epi8(s1, tmp, 8);
    _mm_storeu_si128((__m128i *)&st[0], s0);
    _mm_storeu_si128((__m128i *)&st[4], s1);
}

static int detect_shani(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    int sha = (b >> 29) & 1;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    int sse41 = (c >> 19) & 1, ssse3 = (c >> 9) & 1;
    return sha && sse41 && ssse3;
}
#endif

static int g_shani = -1;

int orc_sha256_has_shani(void) {
#if defined(__x86_64__)
    return detect_shani();
#else
    return 0;
#endif
}

void orc_sha256_use_shani(int enable) { g_shani = enable ? orc_sha256_has_shani() : 0; }

static void blocks(uint32_t st[8], const uint8_t *p, size_t nblocks) {
#if defined(__x86_64__)
    if (g_shani < 0) g_shani = detect_shani();
    if (g_shani) {
        blocks_shani(st, p, nblocks);
        return;
    }
#endif
    blocks_portable(st, p, nblocks);
}

void orc_sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
    uint32_t st[8];
    memcpy(st, H0, sizeof st);
    size_t full = len / 64;
    if (full) blocks(st, msg, full);
    uint8_t tail[128];
    size_t rem = len - full * 64;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, msg + full * 64, rem);
    tail[rem] = 0x80;
    size_t tl = (rem < 56) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    blocks(st, tail, tl / 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* leaf = SHA256(0x00 || d) (htree.go:79-83, ahtree.go:288-292, store leafFor) */
static void leaf_hash(const uint8_t d[32], uint8_t out[32]) {
    uint8_t b[33];
    b[0] = 0;
    memcpy(b + 1, d, 32);
    orc_sha256(b, 33, out);
}

/* node = SHA256(0x01 || l || r) (htree.go:89-97) */
static void node_hash(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]) {
    uint8_t b[65];
    b[0] = 1;
    memcpy(b + 1, l, 32);
    memcpy(b + 33, r, 32);
    orc_sha256(b, 65, out);
}

/* ------------------------------------------------------------ entry digest */
int orc_entry_digest(int version, const uint8_t *key, size_t klen, const uint8_t *md,
                     size_t mdlen, const uint8_t hval[32], uint8_t out[32]) {
    uint8_t stackbuf[256];
    size_t len = (version == 0) ? klen + 32 : 2 + mdlen + 2 + klen + 32;
    uint8_t *b = len <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(len);
    size_t i = 0;
    if (version == 0) {
        /* tx.go:690-701 TxEntryDigest_v1_1: key || hVal, md must be empty */
        if (mdlen > 0) {
            if (b != stackbuf) free(b);
            return ERR_MD_UNSUPPORTED;
        }
    } else if (version == 1) {
        /* tx.go:703-731 TxEntryDigest_v1_2: BE16 mdLen || md || BE16 kLen || key || hVal */
        b[i++] = (uint8_t)(mdlen >> 8);
        b[i++] = (uint8_t)mdlen;
        if (mdlen) memcpy(b + i, md, mdlen);
        i += mdlen;
        b[i++] = (uint8_t)(klen >> 8);
        b[i++] = (uint8_t)klen;
    } else {
        if (b != stackbuf) free(b);
        return ERR_ILLEGAL_ARGS;
    }
    if (klen) memcpy(b + i, key, klen);
    i += klen;
    memcpy(b + i, hval, 32);
    orc_sha256(b, len, out);
    if (b != stackbuf) free(b);
    return OK;
}

/* ------------------------------------------------------------------- htree */
uint64_t orc_htree_levels_len(uint64_t n) {
    if (n == 0) return 0;
    uint64_t t = 0, w = n;
    for (;;) {
        t += w;
        if (w == 1) break;
        w = (w + 1) / 2;
    }
    return t;
}

uint64_t orc_htree_level_offset(uint64_t n, int level) {
    uint64_t t = 0, w = n;
    for (int l = 0; l < level; l++) {
        t += w;
        w = (w + 1) / 2;
    }
    return t;
}

/* Levels above the leaves: htree.go:85-110 (pairwise, odd last node promoted). */
static void reduce_levels(uint8_t *lv, uint64_t n, uint8_t root[32]) {
    uint64_t w = n, off = 0;
    while (w > 1) {
        uint64_t noff = off + w, wn = 0;
        for (uint64_t i = 0; i + 1 < w; i += 2, wn++)
            node_hash(lv + (off + i) * 32, lv + (off + i + 1) * 32, lv + (noff + wn) * 32);
        if (w % 2 == 1) {
            memcpy(lv + (noff + wn) * 32, lv + (off + w - 1) * 32, 32);
            wn++;
        }
        off = noff;
        w = wn;
    }
    memcpy(root, lv + off * 32, 32);
}

int orc_htree_build(const uint8_t *digests, uint64_t n, uint8_t *levels, uint8_t root[32]) {
    if (n == 0) { /* htree.go:73-77 */
        orc_sha256(NULL, 0, root);
        return OK;
    }
    uint8_t *lv = levels ? levels : (uint8_t *)malloc(orc_htree_levels_len(n) * 32);
    for (uint64_t i = 0; i < n; i++) leaf_hash(digests + i * 32, lv + i * 32);
    reduce_levels(lv, n, root);
    if (!levels) free(lv);
    return OK;
}

static int bits_len64(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

int orc_htree_inclusion_proof(const uint8_t *levels, uint64_t width, uint64_t i,
                              uint8_t *terms, uint32_t *nterms) {
    /* htree.go:121-164 */
    *nterms = 0;
    if (i >= width) return ERR_ILLEGAL_ARGS;
    if (width == 1) return OK;
    uint64_t m = i, n = width, offset = 0, l, r;
    uint8_t tmp[64][32];
    uint32_t cnt = 0;
    for (;;) {
        int d = bits_len64(n - 1);
        uint64_t k = 1ULL << (d - 1);
        if (m < k) {
            l = offset + k;
            r = offset + n - 1;
            n = k;
        } else {
            l = offset;
            r = offset + k - 1;
            m -= k;
            n -= k;
            offset += k;
        }
        int layer = bits_len64(r - l);
        uint64_t index = l >> layer;
        memcpy(tmp[cnt++], levels + (orc_htree_level_offset(width, layer) + index) * 32, 32);
        if (n < 1 || (n == 1 && m == 0)) break;
    }
    /* terms are prepended in Go: reverse order of discovery */
    for (uint32_t t = 0; t < cnt; t++) memcpy(terms + t * 32, tmp[cnt - 1 - t], 32);
    *nterms = cnt;
    return OK;
}

int orc_htree_verify_inclusion(uint64_t leaf, uint64_t width, const uint8_t *terms,
                               uint32_t nterms, const uint8_t digest[32], const uint8_t root[32]) {
    /* htree.go:166-195 (a nil proof is modelled by the caller).  Leaf and
     * Width are Go ints: signed, truncating % and / (a negative value comes
     * from a decoded wire proof, InclusionProofFromProto) */
    uint8_t calc[32];
    leaf_hash(digest, calc);
    int64_t i = (int64_t)leaf, r = (int64_t)(width - 1);
    for (uint32_t t = 0; t < nterms; t++) {
        if (i % 2 == 0 && i != r)
            node_hash(calc, terms + t * 32, calc);
        else
            node_hash(terms + t * 32, calc, calc);
        i /= 2;
        r /= 2;
    }
    return i == r && memcmp(calc, root, 32) == 0;
}

/* ---------------------------------------------------------- entries -> Eh */
int orc_build_entries(int version, uint64_t n, const uint8_t *keys, const uint64_t *key_off,
                      const uint8_t *md, const uint64_t *md_off, const uint8_t *vals,
                      const uint64_t *val_off, const uint8_t *hval_override,
                      const uint8_t *use_override, uint8_t *hvals_out, uint8_t *levels,
                      uint8_t root[32]) {
    if (n == 0) {
        orc_sha256(NULL, 0, root);
        return OK;
    }
    uint8_t *dig = (uint8_t *)malloc(n * 32);
    int st = OK;
    for (uint64_t i = 0; i < n && st == OK; i++) {
        uint8_t hv[32];
        /* immustore.go:1620-1630 */
        if (use_override && use_override[i])
            memcpy(hv, hval_override + i * 32, 32);
        else
            orc_sha256(vals + val_off[i], val_off[i + 1] - val_off[i], hv);
        if (hvals_out) memcpy(hvals_out + i * 32, hv, 32);
        size_t mdl = md_off ? md_off[i + 1] - md_off[i] : 0;
        st = orc_entry_digest(version, keys + key_off[i], key_off[i + 1] - key_off[i],
                              mdl ? md + md_off[i] : NULL, mdl, hv, dig + i * 32);
    }
    if (st == OK) st = orc_htree_build(dig, n, levels, root);
    free(dig);
    return st;
}

typedef struct {
    int version;
    uint64_t lo, hi;
    const uint8_t *keys, *vals;
    uint32_t key_len, val_len;
    uint8_t *hvals, *lv; /* lv = leaf level base (level 0) */
} fixed_job;

static void *fixed_worker(void *arg) {
    fixed_job *j = (fixed_job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint8_t hv[32], d[32];
        orc_sha256(j->vals + i * (uint64_t)j->val_len, j->val_len, hv);
        if (j->hvals) memcpy(j->hvals + i * 32, hv, 32);
        orc_entry_digest(j->version, j->keys + i * (uint64_t)j->key_len, j->key_len, NULL, 0, hv, d);
        leaf_hash(d, j->lv + i * 32);
    }
    return NULL;
}

int orc_build_entries_fixed(int version, uint64_t n, const uint8_t *keys, uint32_t key_len,
                            const uint8_t *vals, uint32_t val_len, uint8_t *hvals_out,
                            uint8_t *levels, uint8_t root[32], int nthreads) {
    if (version != 0 && version != 1) return ERR_ILLEGAL_ARGS;
    if (n == 0) {
        orc_sha256(NULL, 0, root);
        return OK;
    }
    uint8_t *lv = levels ? levels : (uint8_t *)malloc(orc_htree_levels_len(n) * 32);
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > n) nthreads = (int)n;
    /* leaf hashing split into contiguous ranges; the pairwise levels are
     * independent of how the leaves were produced. */
    fixed_job jobs[256];
    pthread_t th[256];
    if (nthreads > 256) nthreads = 256;
    uint64_t per = (n + nthreads - 1) / nthreads;
    int used = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t lo = (uint64_t)t * per, hi = lo + per > n ? n : lo + per;
        if (lo >= hi) break;
        jobs[t] = (fixed_job){version, lo, hi, keys, vals, key_len, val_len, hvals_out, lv};
        used++;
    }
    if (used == 1) {
        fixed_worker(&jobs[0]);
    } else {
        for (int t = 0; t < used; t++) pthread_create(&th[t], NULL, fixed_worker, &jobs[t]);
        for (int t = 0; t < used; t++) pthread_join(th[t], NULL);
    }
    reduce_levels(lv, n, root);
    if (!levels) free(lv);
    return OK;
}

/* ------------------------------------------------------- value integrity */
/* embedded/store/immustore.go:3183-3240: readValueAt reads vLen bytes of the
 * value (vLog or cache) into b and returns ErrCorruptedData when
 * len(b) != n || hvalue != sha256.Sum256(b[:n]) (:3235). */
typedef struct {
    uint64_t lo, hi;
    const uint8_t *vals;
    const uint64_t *off, *vlen;
    const uint8_t *hv;
    int32_t *st;
    uint64_t bad;
} values_job;

static void *values_worker(void *arg) {
    values_job *j = (values_job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint64_t len = j->off[i + 1] - j->off[i];
        uint8_t h[32];
        orc_sha256(len ? j->vals + j->off[i] : NULL, len, h);
        const int ok = (!j->vlen || j->vlen[i] == len) && memcmp(h, j->hv + 32 * i, 32) == 0;
        j->st[i] = ok ? 0 : 14;
        j->bad += !ok;
    }
    return NULL;
}

uint64_t orc_verify_values(uint64_t n, const uint8_t *vals, const uint64_t *off,
                           const uint64_t *vlen, const uint8_t *hvals, int32_t *status,
                           int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
    values_job jobs[64];
    pthread_t th[64];
    const uint64_t per = (n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        const uint64_t lo = (uint64_t)t * per < n ? (uint64_t)t * per : n;
        const uint64_t hi = lo + per < n ? lo + per : n;
        jobs[t] = (values_job){lo, hi, vals, off, vlen, hvals, status, 0};
    }
    if (nthreads == 1) {
        values_worker(&jobs[0]);
    } else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, values_worker, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    uint64_t bad = 0;
    for (int t = 0; t < nthreads; t++) bad += jobs[t].bad;
    return bad;
}

/* ------------------------------------------------------- precommit batch */
/* ImmuStore.precommit over many transactions (immustore.go:1620-1632, the
 * Eh check of :1649-1654): orc_build_entries per tx, txs spread over
 * nthreads threads (contiguous tx ranges). */
typedef struct {
    int version;
    uint64_t max_width, t0, t1;
    const uint64_t *tx_off;
    const uint8_t *keys, *md, *vals, *ov, *use, *expect;
    const uint64_t *key_off, *md_off, *val_off;
    uint8_t *hvals, *eh;
    int32_t *status;
} pc_job;

static void *pc_worker(void *arg) {
    pc_job *j = (pc_job *)arg;
    const uint64_t E0 = j->tx_off[0];
    for (uint64_t t = j->t0; t < j->t1; t++) {
        const uint64_t e0 = j->tx_off[t], n = j->tx_off[t + 1] - e0;
        int st = OK;
        uint8_t root[32];
        if (j->max_width && n > j->max_width) {
            st = ERR_MAX_WIDTH; /* htree.go:69-71 */
        } else {
            st = orc_build_entries(j->version, n, j->keys, j->key_off + e0, j->md,
                                   j->md_off ? j->md_off + e0 : NULL, j->vals, j->val_off + e0,
                                   j->ov ? j->ov + e0 * 32 : NULL, j->use ? j->use + e0 : NULL,
                                   j->hvals ? j->hvals + (e0 - E0) * 32 : NULL, NULL, root);
        }
        if (st == OK && j->expect && memcmp(j->expect + t * 32, root, 32) != 0)
            st = ERR_ILLEGAL_ARGS; /* "entries hash (Eh) differs" immustore.go:1651 */
        if (j->eh) {
            if (st == OK || st == ERR_ILLEGAL_ARGS)
                memcpy(j->eh + t * 32, root, 32);
            else
                memset(j->eh + t * 32, 0, 32);
        }
        j->status[t] = st;
    }
    return NULL;
}

int orc_precommit_batch(int version, uint64_t max_width, uint64_t ntx, const uint64_t *tx_off,
                        const uint8_t *keys, const uint64_t *key_off, const uint8_t *md,
                        const uint64_t *md_off, const uint8_t *vals, const uint64_t *val_off,
                        const uint8_t *hval_override, const uint8_t *use_override,
                        const uint8_t *expect_eh, uint8_t *hvals_out, uint8_t *eh_out,
                        int32_t *status, int nthreads) {
    if (ntx == 0) return OK;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    if ((uint64_t)nthreads > ntx) nthreads = (int)ntx;
    pc_job jobs[64];
    pthread_t th[64];
    /* split by entry count so threads get similar work */
    const uint64_t E = tx_off[ntx] - tx_off[0];
    uint64_t t = 0;
    for (int k = 0; k < nthreads; k++) {
        pc_job *j = &jobs[k];
        j->version = version;
        j->max_width = max_width;
        j->tx_off = tx_off;
        j->keys = keys; j->md = md; j->vals = vals;
        j->ov = hval_override; j->use = use_override; j->expect = expect_eh;
        j->key_off = key_off; j->md_off = md_off; j->val_off = val_off;
        j->hvals = hvals_out; j->eh = eh_out; j->status = status;
        j->t0 = t;
        const uint64_t target = tx_off[0] + E * (uint64_t)(k + 1) / (uint64_t)nthreads;
        while (t < ntx && (k == nthreads - 1 || tx_off[t + 1] <= target)) t++;
        j->t1 = t;
    }
    if (nthreads == 1) {
        pc_worker(&jobs[0]);
    } else {
        for (int k = 0; k < nthreads; k++) pthread_create(&th[k], NULL, pc_worker, &jobs[k]);
        for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    }
    return OK;
}

/* ------------------------------------------------------------- tx header */
int orc_tx_inner_hash(uint64_t ts, int version, const uint8_t *txmd, size_t txmdlen,
                      uint32_t nentries, const uint8_t eh[32], uint64_t bltxid,
                      const uint8_t blroot[32], uint8_t out[32]) {
    /* tx.go:249-302: ts + version + (v0: BE16 nentries | v1: BE16 mdLen md BE32 nentries)
     * + eh + blTxID + blRoot */
    uint8_t b[8 + 2 + 2 + 268 + 4 + 32 + 8 + 32];
    size_t i = 0;
    for (int k = 7; k >= 0; k--) b[i++] = (uint8_t)(ts >> (8 * k));
    b[i++] = (uint8_t)(version >> 8);
    b[i++] = (uint8_t)version;
    if (version == 0) {
        if (txmdlen) return ERR_MD_UNSUPPORTED;
        b[i++] = (uint8_t)(nentries >> 8);
        b[i++] = (uint8_t)nentries;
    } else if (version == 1) {
        if (txmdlen > 268) return ERR_ILLEGAL_ARGS; /* maxTxMetadataLen, tx_metadata.go:36-39 */
        b[i++] = (uint8_t)(txmdlen >> 8);
        b[i++] = (uint8_t)txmdlen;
        if (txmdlen) memcpy(b + i, txmd, txmdlen);
        i += txmdlen;
        for (int k = 3; k >= 0; k--) b[i++] = (uint8_t)(nentries >> (8 * k));
    } else {
        return ERR_ILLEGAL_ARGS;
    }
    memcpy(b + i, eh, 32);
    i += 32;
    for (int k = 7; k >= 0; k--) b[i++] = (uint8_t)(bltxid >> (8 * k));
    memcpy(b + i, blroot, 32);
    i += 32;
    orc_sha256(b, i, out);
    return OK;
}

void orc_tx_alh(uint64_t id, const uint8_t prev_alh[32], const uint8_t inner[32], uint8_t out[32]) {
    /* tx.go:307-319 and verification.go:32-38 (advanceLinearHash) */
    uint8_t b[72];
    for (int k = 7; k >= 0; k--) b[7 - k] = (uint8_t)(id >> (8 * k));
    memcpy(b + 8, prev_alh, 32);
    memcpy(b + 40, inner, 32);
    orc_sha256(b, 72, out);
}

/* ------------------------------------------------------------------ ahtree */
uint64_t orc_ahtree_nodes_upto(uint64_t n) {
    /* ahtree.go:492-511 */
    uint64_t o = n;
    for (int l = 0; l < 64 && n >= (1ULL << l); l++) {
        o += (n >> (l + 1)) << l;
        if ((n >> l) & 1) o += n & ((1ULL << l) - 1);
    }
    return o;
}

uint64_t orc_ahtree_nodes_until(uint64_t n) { return n == 1 ? 0 : orc_ahtree_nodes_upto(n - 1); }

static void put_be32(uint8_t *b, uint32_t v) {
    for (int k = 0; k < 4; k++) b[k] = (uint8_t)(v >> (24 - 8 * k));
}
static void put_be64(uint8_t *b, uint64_t v) {
    for (int k = 0; k < 8; k++) b[k] = (uint8_t)(v >> (56 - 8 * k));
}

static const uint8_t *aht_node(const uint8_t *dlog, uint64_t k, int l) {
    /* ahtree.go:460-462 node(n,l) = dLog[nodesUntil(n)+l] */
    return dlog + (orc_ahtree_nodes_until(k) + (uint64_t)l) * 32;
}

int orc_ahtree_append(uint8_t *dlog, uint64_t n_before, const uint8_t *payload, size_t plen,
                      uint8_t root[32]) {
    /* ahtree.go:246-322 */
    uint64_t n = n_before + 1;
    uint8_t *out = dlog + orc_ahtree_nodes_until(n) * 32;
    uint8_t stackbuf[129], *b = plen + 1 <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(plen + 1);
    b[0] = 0;
    if (plen) memcpy(b + 1, payload, plen);
    uint8_t h[32];
    orc_sha256(b, plen + 1, h);
    if (b != stackbuf) free(b);
    memcpy(out, h, 32);
    int cnt = 1;
    uint64_t w = n - 1, k = n - 1;
    for (int l = 0; w > 0; l++) {
        if (w & 1) {
            node_hash(aht_node(dlog, k, l), h, h);
            memcpy(out + 32 * cnt++, h, 32);
        }
        k &= ~(1ULL << l);
        w >>= 1;
    }
    if (root) memcpy(root, h, 32);
    return OK;
}

int orc_ahtree_append_batch(uint8_t *dlog, uint64_t n_before, const uint8_t *payloads,
                            uint64_t m, size_t plen) {
    for (uint64_t i = 0; i < m; i++) orc_ahtree_append(dlog, n_before + i, payloads + i * plen, plen, NULL);
    return OK;
}

/* The appendable record streams of m appends of plen-byte payloads
 * (ahtree.go:266-282: pLog gets BE32 len(d) then d; :341-351: cLog gets
 * BE64 poff || BE32 len(d), poff = pLog offset of the length prefix).
 * p_off0 = pLog size before the batch (t.pLogSize).  plog / clog may be NULL. */
void orc_ahtree_log_records(const uint8_t *payloads, uint64_t m, size_t plen, uint64_t p_off0,
                            uint8_t *plog, uint8_t *clog) {
    for (uint64_t i = 0; i < m; i++) {
        const uint64_t poff = p_off0 + i * (4 + (uint64_t)plen);
        if (plog) {
            uint8_t *r = plog + i * (4 + (uint64_t)plen);
            put_be32(r, (uint32_t)plen);
            if (plen) memcpy(r + 4, payloads + i * plen, plen);
        }
        if (clog) {
            uint8_t *c = clog + i * 12;
            put_be64(c, poff);
            put_be32(c + 8, (uint32_t)plen);
        }
    }
}

int orc_ahtree_root_at(const uint8_t *dlog, uint64_t size, uint64_t n, uint8_t out[32]) {
    /* ahtree.go:749-771 */
    if (n == 0) return ERR_ILLEGAL_ARGS;
    if (size == 0) return ERR_EMPTY;
    if (n > size) return ERR_UNEXISTENT;
    memcpy(out, aht_node(dlog, n, __builtin_popcountll(n - 1)), 32);
    return OK;
}

/* proof assembly helpers: terms are prepended in Go; we build into a reversed
 * stack and flip at the end. */
typedef struct {
    uint8_t t[192][32];
    uint32_t n;
} stack_t_;

static void push_front_seq(stack_t_ *s, const uint8_t *d) { memcpy(s->t[s->n++], d, 32); }

static const uint8_t *highest_node(const uint8_t *dlog, uint64_t i, int d) {
    /* ahtree.go:653-661 */
    int l = 0;
    for (int r = d - 1; r >= 0; r--)
        if ((i - 1) & (1ULL << r)) l++;
    return aht_node(dlog, i, l);
}

/* Go inclusionProof (ahtree.go:545-577) returns p ++ proof where proof gets
 * prepends.  Rewritten iteratively: we collect the sequence of prepended
 * terms in "prepend order" (s) so that the final proof is reverse(s). */
static void incl(const uint8_t *dlog, uint64_t i, uint64_t j, int height, stack_t_ *s) {
    for (int h = height - 1; h >= 0; h--) {
        if ((j - 1) & (1ULL << h)) {
            uint64_t k = (j - 1) >> h << h;
            if (i <= k) {
                push_front_seq(s, highest_node(dlog, j, h));
                incl(dlog, i, k, h, s);
                return;
            }
            push_front_seq(s, aht_node(dlog, k, h));
        }
    }
}

static void cons(const uint8_t *dlog, uint64_t i, uint64_t j, int height, stack_t_ *s) {
    /* ahtree.go:596-651 */
    for (int h = height - 1; h >= 0; h--) {
        if ((j - 1) & (1ULL << h)) {
            uint64_t k = (j - 1) >> h << h;
            if (i <= k) {
                push_front_seq(s, highest_node(dlog, j, h));
                if (i < k) cons(dlog, i, k, h, s);
                if (i == k) push_front_seq(s, highest_node(dlog, i, h));
                return;
            }
            push_front_seq(s, aht_node(dlog, k, h));
            if (i == j) {
                push_front_seq(s, highest_node(dlog, i, h));
                return;
            }
        }
    }
}

static int finish_proof(stack_t_ *s, uint8_t *terms, uint32_t *nterms) {
    for (uint32_t t = 0; t < s->n; t++) memcpy(terms + 32 * t, s->t[s->n - 1 - t], 32);
    *nterms = s->n;
    return OK;
}

int orc_ahtree_inclusion_proof(const uint8_t *dlog, uint64_t size, uint64_t i, uint64_t j,
                               uint8_t *terms, uint32_t *nterms) {
    /* ahtree.go:525-543 */
    *nterms = 0;
    if (i > j) return ERR_ILLEGAL_ARGS;
    if (j > size) return ERR_UNEXISTENT;
    stack_t_ s;
    s.n = 0;
    incl(dlog, i, j, bits_len64(j - 1), &s);
    return finish_proof(&s, terms, nterms);
}

int orc_ahtree_consistency_proof(const uint8_t *dlog, uint64_t size, uint64_t i, uint64_t j,
                                 uint8_t *terms, uint32_t *nterms) {
    /* ahtree.go:579-594 */
    *nterms = 0;
    if (i > j) return ERR_ILLEGAL_ARGS;
    if (j > size) return ERR_UNEXISTENT;
    stack_t_ s;
    s.n = 0;
    cons(dlog, i, j, bits_len64(j - 1), &s);
    return finish_proof(&s, terms, nterms);
}

/* Many InclusionProof (kind 0) / ConsistencyProof (kind 1) calls over one
 * dLog (ahtree.go:525-651): proof p into terms + p * cap * 32, its length
 * into nterms[p], the call's status into st[p] (a proof longer than cap:
 * ERR_ILLEGAL_ARGS).  The checker of the device's batch proof generation. */
void orc_ahtree_proof_batch(const uint8_t *dlog, uint64_t size, int kind, uint64_t n,
                            const uint64_t *i, const uint64_t *j, uint8_t *terms, uint32_t cap,
                            uint32_t *nterms, int32_t *st) {
    uint8_t tmp[192 * 32];
    for (uint64_t p = 0; p < n; p++) {
        uint32_t nt = 0;
        int r = kind == 0 ? orc_ahtree_inclusion_proof(dlog, size, i[p], j[p], tmp, &nt)
                          : orc_ahtree_consistency_proof(dlog, size, i[p], j[p], tmp, &nt);
        if (r == OK && nt > cap) r = ERR_ILLEGAL_ARGS;
        st[p] = r;
        nterms[p] = r == OK ? nt : 0;
        if (r == OK) memcpy(terms + p * (uint64_t)cap * 32, tmp, (size_t)nt * 32);
    }
}

void orc_ahtree_eval_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                               const uint8_t leaf[32], uint8_t out[32]) {
    /* ahtree/verification.go:32-56 */
    uint64_t i1 = i - 1, j1 = j - 1;
    uint8_t c[32];
    memcpy(c, leaf, 32);
    for (uint32_t t = 0; t < nterms; t++) {
        if (i1 % 2 == 0 && i1 != j1)
            node_hash(c, terms + 32 * t, c);
        else
            node_hash(terms + 32 * t, c, c);
        i1 >>= 1;
        j1 >>= 1;
    }
    memcpy(out, c, 32);
}

int orc_ahtree_verify_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                                const uint8_t leaf[32], const uint8_t root[32]) {
    /* ahtree/verification.go:21-30 */
    if (i > j || i == 0 || (i < j && nterms == 0)) return 0;
    uint8_t c[32];
    orc_ahtree_eval_inclusion(terms, nterms, i, j, leaf, c);
    return memcmp(c, root, 32) == 0;
}

int orc_ahtree_eval_consistency(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                                uint8_t ci[32], uint8_t cj[32]) {
    /* ahtree/verification.go:72-109.  Go indexes cproof[0] unguarded; we
     * return ERR_ILLEGAL_ARGS for an empty proof instead of panicking. */
    if (nterms == 0) return ERR_ILLEGAL_ARGS;
    uint64_t fn = i - 1, sn = j - 1;
    while (fn % 2 == 1) {
        fn >>= 1;
        sn >>= 1;
    }
    memcpy(ci, terms, 32);
    memcpy(cj, terms, 32);
    for (uint32_t t = 1; t < nterms; t++) {
        const uint8_t *h = terms + 32 * t;
        if (fn % 2 == 1 || fn == sn) {
            node_hash(h, ci, ci);
            node_hash(h, cj, cj);
            while (fn % 2 == 0 && fn != 0) {
                fn >>= 1;
                sn >>= 1;
            }
        } else {
            node_hash(cj, h, cj);
        }
        fn >>= 1;
        sn >>= 1;
    }
    return OK;
}

int orc_ahtree_verify_consistency(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                                  const uint8_t iroot[32], const uint8_t jroot[32]) {
    /* ahtree/verification.go:58-70 */
    if (i > j || i == 0 || (i < j && nterms == 0)) return 0;
    if (i == j && nterms == 0) return memcmp(iroot, jroot, 32) == 0;
    uint8_t ci[32], cj[32];
    orc_ahtree_eval_consistency(terms, nterms, i, j, ci, cj);
    return memcmp(iroot, ci, 32) == 0 && memcmp(jroot, cj, 32) == 0;
}

void orc_ahtree_eval_last_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i,
                                    const uint8_t leaf[32], uint8_t out[32]) {
    /* ahtree/verification.go:120-137 */
    (void)i;
    uint8_t r[32];
    memcpy(r, leaf, 32);
    for (uint32_t t = 0; t < nterms; t++) node_hash(terms + 32 * t, r, r);
    memcpy(out, r, 32);
}

int orc_ahtree_verify_last_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i,
                                     const uint8_t leaf[32], const uint8_t root[32]) {
    /* ahtree/verification.go:111-118 */
    if (i == 0) return 0;
    uint8_t r[32];
    orc_ahtree_eval_last_inclusion(terms, nterms, i, leaf, r);
    return memcmp(r, root, 32) == 0;
}

/* Batch of ahtree VerifyInclusion / VerifyConsistency / VerifyLastInclusion
 * calls (ahtree/verification.go:21-137) over CSR term lists, split over
 * nthreads host threads; ok[p] = the Go verifier's bool.  The CPU side of the
 * ahtree half of BASELINE configs[4].  Returns the number verified. */
typedef struct {
    int kind;
    uint64_t lo, hi;
    const uint64_t *i, *j, *term_off;
    const uint8_t *terms, *a, *b;
    uint8_t *ok;
    uint64_t cnt;
} aht_vjob;

static void *aht_verify_worker(void *arg) {
    aht_vjob *J = (aht_vjob *)arg;
    for (uint64_t p = J->lo; p < J->hi; p++) {
        const uint8_t *t = J->terms + J->term_off[p] * 32;
        const uint32_t nt = (uint32_t)(J->term_off[p + 1] - J->term_off[p]);
        int r;
        if (J->kind == 0)
            r = orc_ahtree_verify_inclusion(t, nt, J->i[p], J->j[p], J->a + 32 * p, J->b + 32 * p);
        else if (J->kind == 1)
            r = orc_ahtree_verify_consistency(t, nt, J->i[p], J->j[p], J->a + 32 * p, J->b + 32 * p);
        else
            r = orc_ahtree_verify_last_inclusion(t, nt, J->i[p], J->a + 32 * p, J->b + 32 * p);
        J->ok[p] = (uint8_t)r;
        J->cnt += (uint64_t)r;
    }
    return NULL;
}

uint64_t orc_ahtree_verify_batch(int kind, uint64_t n, const uint64_t *i, const uint64_t *j,
                                 const uint64_t *term_off, const uint8_t *terms, const uint8_t *a,
                                 const uint8_t *b, uint8_t *ok, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    aht_vjob jobs[64];
    pthread_t th[64];
    for (int t = 0; t < nthreads; t++) {
        aht_vjob J = {kind, n * t / nthreads, n * (t + 1) / nthreads, i, j, term_off, terms, a, b, ok, 0};
        jobs[t] = J;
        pthread_create(&th[t], NULL, aht_verify_worker, &jobs[t]);
    }
    uint64_t cnt = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        cnt += jobs[t].cnt;
    }
    return cnt;
}

/* ------------------------------------------------ streamed ahtree (checker) */
static uint64_t splitmix_word(uint64_t seed, uint64_t w) {
    /* word w of orc_fill_random(seed): splitmix64 output number w+1 */
    uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* The ahtree appends (n_start, n_end] of plen-byte payloads drawn from the
 * orc_fill_random(seed) stream -- append n_start + 1 + x takes payload
 * pay0 + x, i.e. stream bytes [(pay0 + x) plen, (pay0 + x + 1) plen) -- kept
 * as the 64 PEAKS of the current size only, no dLog: peak l of a tree of
 * size n is node(n with the bits below l cleared, l) (ahtree.go:460-462) for
 * every set bit l of n.  Append n (ahtree.go:287-322) hashes the leaf
 * SHA256(0x00 || payload) and then, for every set bit l of n-1 from low to
 * high, h = SHA256(0x01 || node(k, l) || h) with node(k, l) = peak l of n-1;
 * the first tz(n) of those are the perfect nodes ending at n, so the peaks of
 * n are those of n-1 with levels < tz(n) dropped and level tz(n) = h after
 * tz(n) steps.  For each sampled n (strictly ascending, in (n_start, n_end])
 * all 1 + popcount(n-1) digests append n writes to the dLog go to
 * out + s * 65 * 32 and their count to cnt[s] (the last one is RootAt(n)).
 * peaks_in / peaks_out: 64 x 32 B, slot l meaningful for set bits l of
 * n_start / n_end (peaks_in may be NULL when n_start == 0; peaks_out may be
 * NULL).  Test infrastructure: checks device dLogs too large to rebuild. */
int orc_ahtree_stream(uint64_t seed, uint32_t plen, uint64_t pay0, uint64_t n_start,
                      const uint8_t *peaks_in, uint64_t n_end, const uint64_t *samples,
                      uint64_t ns, uint8_t *out, uint32_t *cnt, uint8_t *peaks_out) {
    if (plen % 8 || plen > 1024 || n_end < n_start || (n_start && !peaks_in) ||
        (ns && (!samples || !out || !cnt)))
        return ERR_ILLEGAL_ARGS;
    for (uint64_t s = 0; s < ns; s++)
        if (samples[s] <= n_start || samples[s] > n_end || (s && samples[s] <= samples[s - 1]))
            return ERR_ILLEGAL_ARGS;
    uint8_t pk[64][32];
    memset(pk, 0, sizeof pk);
    if (n_start) memcpy(pk, peaks_in, sizeof pk);
    uint8_t msg[1 + 1024];
    msg[0] = 0;
    const uint32_t words = plen / 8;
    uint64_t s = 0;
    for (uint64_t n = n_start + 1; n <= n_end; n++) {
        const uint64_t w0 = (pay0 + (n - n_start - 1)) * words;
        for (uint32_t q = 0; q < words; q++) {
            const uint64_t z = splitmix_word(seed, w0 + q);
            memcpy(msg + 1 + 8 * q, &z, 8); /* little-endian words, as orc_fill_random */
        }
        uint8_t h[32];
        orc_sha256(msg, 1 + (size_t)plen, h);
        const int sampled = s < ns && samples[s] == n;
        uint8_t *o = sampled ? out + s * 65 * 32 : NULL;
        uint32_t c = 0;
        if (o) memcpy(o + 32 * c++, h, 32);
        const int tz = __builtin_ctzll(n);
        if (tz == 0) memcpy(pk[0], h, 32); /* n odd: the leaf is the level-0 peak */
        const uint64_t prev = n - 1;
        for (int l = 0; l < 64 && (prev >> l); l++) {
            if (!((prev >> l) & 1)) continue;
            if (l >= tz && !o) break; /* past the perfect nodes: only samples need the rest */
            node_hash(pk[l], h, h);
            if (o) memcpy(o + 32 * c++, h, 32);
            if (l == tz - 1) memcpy(pk[tz], h, 32); /* the perfect node ending at n */
        }
        if (o) cnt[s++] = c;
    }
    if (peaks_out) memcpy(peaks_out, pk, sizeof pk);
    return OK;
}

/* ------------------------------------------------------------ synthetic */
void orc_fill_random(uint8_t *dst, uint64_t nbytes, uint64_t seed) {
    /* word w = splitmix64 output number w+1 from state `seed` (little endian) */
    uint64_t nw = (nbytes + 7) / 8;
    for (uint64_t w = 0; w < nw; w++) {
        uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        uint64_t left = nbytes - w * 8;
        if (left >= 8)
            memcpy(dst + w * 8, &z, 8);
        else
            memcpy(dst + w * 8, &z, left);
    }
}

/* Batch of htree.VerifyInclusion calls (htree.go:166-195), fixed term stride;
 * the CPU side of BASELINE configs[4].  Returns the number verified. */
uint64_t orc_htree_verify_batch(uint64_t n, const uint64_t *leaf, uint64_t width,
                                const uint8_t *terms, uint32_t nterms_each,
                                const uint8_t *digests, const uint8_t root[32], uint8_t *ok) {
    uint64_t cnt = 0;
    for (uint64_t p = 0; p < n; p++) {
        const int r = orc_htree_verify_inclusion(leaf[p], width, terms + (uint64_t)p * nterms_each * 32,
                                                 nterms_each, digests + p * 32, root);
        if (ok) ok[p] = (uint8_t)r;
        cnt += (uint64_t)r;
    }
    return cnt;
}

/* ------------------------------------------------------------------ tx layer */
int orc_tx_header_alh(const orc_tx_header *h, const uint8_t *md_blob, uint8_t inner[32],
                      uint8_t alh[32]) {
    /* TxHeader.Alh, tx.go:307-319 over innerHash, tx.go:249-302 */
    uint8_t in[32];
    int st = orc_tx_inner_hash((uint64_t)h->ts, (int)h->version,
                               h->md_len ? md_blob + h->md_off : NULL, h->md_len, h->nentries,
                               h->eh, h->bl_tx_id, h->bl_root, in);
    if (st) return st;
    if (inner) memcpy(inner, in, 32);
    orc_tx_alh(h->id, h->prev_alh, in, alh);
    return OK;
}

int orc_verify_linear_proof(uint64_t p_src, uint64_t p_tgt, const uint8_t *terms, uint32_t nterms,
                            uint64_t src, uint64_t tgt, const uint8_t src_alh[32],
                            const uint8_t tgt_alh[32]) {
    /* store/verification.go:40-64 */
    if (p_src != src || p_tgt != tgt) return 0;
    if (p_src == 0 || p_src > p_tgt || nterms == 0 || memcmp(src_alh, terms, 32) != 0) return 0;
    if ((uint64_t)nterms != tgt - src + 1) return 0;
    uint8_t c[32];
    memcpy(c, terms, 32);
    for (uint32_t i = 1; i < nterms; i++) orc_tx_alh(p_src + i, c, terms + 32 * (size_t)i, c);
    return memcmp(tgt_alh, c, 32) == 0;
}

static void leaf_for(const uint8_t d[32], uint8_t out[32]) { leaf_hash(d, out); }

int orc_verify_linear_advance_proof(int has_proof, const uint8_t *lin_terms, uint32_t nlin,
                                    const uint8_t *incl_terms, const uint32_t *incl_off,
                                    uint32_t nincl, uint64_t start, uint64_t end,
                                    const uint8_t end_alh[32], const uint8_t root[32],
                                    uint64_t size) {
    /* store/verification.go:66-125 */
    if (end < start) return 0;
    if (end <= start + 1) return 1;
    if (!has_proof || (uint64_t)nlin != end - start || (uint64_t)nincl != end - start - 1) return 0;
    uint8_t c[32], lf[32];
    memcpy(c, lin_terms, 32);
    for (uint64_t tx = start + 1; tx < end; tx++) {
        const uint64_t k = tx - start - 1;
        leaf_for(c, lf);
        if (!orc_ahtree_verify_inclusion(incl_terms + 32 * (size_t)incl_off[k],
                                         incl_off[k + 1] - incl_off[k], tx, size, lf, root))
            return 0;
        orc_tx_alh(tx + 1, c, lin_terms + 32 * (size_t)(tx - start), c);
    }
    return memcmp(c, end_alh, 32) == 0;
}

int orc_verify_dual_proof_v2(const orc_tx_header *sh, const orc_tx_header *th,
                             const uint8_t *md_blob, const uint8_t *incl, uint32_t nincl,
                             const uint8_t *cons, uint32_t ncons, uint64_t src, uint64_t tgt,
                             const uint8_t src_alh[32], const uint8_t tgt_alh[32]) {
    /* store/verification.go:304-372 */
    if (!sh || !th || sh->id == 0 || sh->id != src || th->id != tgt) return ERR_ILLEGAL_ARGS;
    if (src > tgt) return ERR_SOURCE_TX_NEWER;
    uint8_t a[32];
    if (orc_tx_header_alh(sh, md_blob, NULL, a) || memcmp(a, src_alh, 32)) return ERR_ILLEGAL_ARGS;
    if (orc_tx_header_alh(th, md_blob, NULL, a) || memcmp(a, tgt_alh, 32)) return ERR_ILLEGAL_ARGS;
    if (sh->id - 1 != sh->bl_tx_id || th->id - 1 != th->bl_tx_id) return ERR_UNEXPECTED_LINKING;
    if (src == tgt) return OK;
    uint8_t lf[32];
    leaf_for(src_alh, lf);
    if (!orc_ahtree_verify_inclusion(incl, nincl, src, th->bl_tx_id, lf, th->bl_root))
        return ERR_INCLUSION_NOT_VALID;
    int ok;
    if (src == 1)
        ok = orc_ahtree_verify_consistency(cons, ncons, src, th->bl_tx_id, lf, th->bl_root);
    else
        ok = orc_ahtree_verify_consistency(cons, ncons, sh->bl_tx_id, th->bl_tx_id, sh->bl_root,
                                           th->bl_root);
    return ok ? OK : ERR_CONSISTENCY_NOT_VALID;
}

int orc_verify_dual_proof(const orc_tx_header *sh, const orc_tx_header *th,
                          const uint8_t *md_blob, const uint8_t *incl, uint32_t nincl,
                          const uint8_t *cons, uint32_t ncons, const uint8_t tbl_alh[32],
                          const uint8_t *last, uint32_t nlast, int has_lin, uint64_t lin_src,
                          uint64_t lin_tgt, const uint8_t *lin, uint32_t nlin, int has_lap,
                          const uint8_t *lap_terms, uint32_t nlap, const uint8_t *lap_incl,
                          const uint32_t *lap_incl_off, uint32_t nlap_incl, uint64_t src,
                          uint64_t tgt, const uint8_t src_alh[32], const uint8_t tgt_alh[32]) {
    /* store/verification.go:127-235 */
    if (!sh || !th || sh->id != src || th->id != tgt) return 0;
    if (sh->id == 0 || sh->id > th->id) return 0;
    uint8_t a[32], lf[32];
    if (orc_tx_header_alh(sh, md_blob, NULL, a) || memcmp(a, src_alh, 32)) return 0;
    if (orc_tx_header_alh(th, md_blob, NULL, a) || memcmp(a, tgt_alh, 32)) return 0;
    if (src < th->bl_tx_id) {
        leaf_for(src_alh, lf);
        if (!orc_ahtree_verify_inclusion(incl, nincl, src, th->bl_tx_id, lf, th->bl_root)) return 0;
    }
    if (sh->bl_tx_id > 0 &&
        !orc_ahtree_verify_consistency(cons, ncons, sh->bl_tx_id, th->bl_tx_id, sh->bl_root,
                                       th->bl_root))
        return 0;
    if (th->bl_tx_id > 0) {
        leaf_for(tbl_alh, lf);
        if (!orc_ahtree_verify_last_inclusion(last, nlast, th->bl_tx_id, lf, th->bl_root)) return 0;
    }
    if (src < th->bl_tx_id) {
        if (!has_lin || !orc_verify_linear_proof(lin_src, lin_tgt, lin, nlin, th->bl_tx_id, tgt,
                                                 tbl_alh, tgt_alh))
            return 0;
        return orc_verify_linear_advance_proof(has_lap, lap_terms, nlap, lap_incl, lap_incl_off,
                                               nlap_incl, sh->bl_tx_id, src, src_alh, th->bl_root,
                                               th->bl_tx_id);
    }
    if (!has_lin ||
        !orc_verify_linear_proof(lin_src, lin_tgt, lin, nlin, src, tgt, src_alh, tgt_alh))
        return 0;
    return orc_verify_linear_advance_proof(has_lap, lap_terms, nlap, lap_incl, lap_incl_off,
                                           nlap_incl, sh->bl_tx_id, th->bl_tx_id, tbl_alh,
                                           th->bl_root, th->bl_tx_id);
}

/* ---- tx log records (immustore.go:1812-1924 writer, tx.go:388-630 reader) */
static int rd(uint64_t len, uint64_t *p, uint64_t n) {
    if (*p + n > len) return 0;
    *p += n;
    return 1;
}
static uint64_t be(const uint8_t *b, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | b[i];
    return v;
}

/* KVMetadata.unsafeReadFrom (kv_metadata.go:221-256) then Bytes()
 * (kv_metadata.go:207-219): attributes deleted(0, no payload),
 * expiresAt(1, BE64), nonIndexable(2, no payload); an unknown code or a short
 * expiresAt is ErrCorruptedData; a repeated attribute overwrites the earlier one
 * (map), and the digest is taken over the re-serialised bytes in code order. */
static int kvmd_canonical(const uint8_t *md, uint64_t ml, uint8_t out[11], uint64_t *outl) {
    int have[3] = {0, 0, 0};
    uint8_t exp[8];
    if (ml > 11) return ERR_CORRUPTED_DATA;
    uint64_t i = 0;
    while (i < ml) {
        const uint8_t code = md[i++];
        if (code == 0) {
            have[0] = 1;
        } else if (code == 1) {
            if (ml - i < 8) return ERR_CORRUPTED_DATA;
            memcpy(exp, md + i, 8);
            i += 8;
            have[1] = 1;
        } else if (code == 2) {
            have[2] = 1;
        } else {
            return ERR_CORRUPTED_DATA;
        }
    }
    uint64_t o = 0;
    if (have[0]) out[o++] = 0;
    if (have[1]) {
        out[o++] = 1;
        memcpy(out + o, exp, 8);
        o += 8;
    }
    if (have[2]) out[o++] = 2;
    *outl = o;
    return OK;
}

/* TxMetadata.ReadFrom (tx_metadata.go:159-193) then Bytes() (:145-157):
 * truncatedUptoTx(0, BE64), extra(1, BE16 length + bytes, <= 256 bytes).  An
 * extra whose length runs past the metadata makes Go's parse index past the
 * slice (a panic), and one longer than 256 bytes panics in Bytes(): both are
 * corrupted data here. */
static int txmd_canonical(const uint8_t *md, uint64_t ml, uint8_t out[268], uint64_t *outl) {
    int have0 = 0, have1 = 0;
    uint8_t trunc[8];
    const uint8_t *extra = NULL;
    uint64_t el = 0;
    if (ml > 268) return ERR_CORRUPTED_DATA;
    uint64_t i = 0;
    while (i < ml) {
        const uint8_t code = md[i++];
        if (code == 0) {
            if (ml - i < 8) return ERR_CORRUPTED_DATA;
            memcpy(trunc, md + i, 8);
            i += 8;
            have0 = 1;
        } else if (code == 1) {
            if (ml - i < 2) return ERR_CORRUPTED_DATA;
            el = be(md + i, 2);
            i += 2;
            if (ml - i < el || el > 256) return ERR_CORRUPTED_DATA;
            extra = md + i;
            i += el;
            have1 = 1;
        } else {
            return ERR_CORRUPTED_DATA;
        }
    }
    uint64_t o = 0;
    if (have0) {
        out[o++] = 0;
        memcpy(out + o, trunc, 8);
        o += 8;
    }
    if (have1) {
        out[o++] = 1;
        out[o++] = (uint8_t)(el >> 8);
        out[o++] = (uint8_t)el;
        memcpy(out + o, extra, el);
        o += el;
    }
    *outl = o;
    return OK;
}

int orc_txlog_validate(const uint8_t *buf, uint64_t len, uint32_t max_entries,
                       uint32_t max_key_len, uint64_t max_txs, uint64_t *ntx_out,
                       uint64_t *consumed_out, uint8_t *alh_out, int32_t *status_out) {
    uint64_t p = 0, ntx = 0;
    int rc = OK;
    uint8_t *digs = (uint8_t *)malloc((size_t)(max_entries ? max_entries : 1) * 32);
    uint8_t *lv = (uint8_t *)malloc((size_t)orc_htree_levels_len(max_entries ? max_entries : 1) * 32);
    while (ntx < max_txs) {
        const uint64_t p0 = p;
        orc_tx_header h;
        memset(&h, 0, sizeof h);
        uint8_t txmd[268];
        /* readHeader, tx.go:419-518 */
        if (p + 8 > len) break;
        h.id = be(buf + p, 8);
        if (h.id == 0) break; /* preallocated tail reads as EOF */
        p += 8;
        if (!rd(len, &p, 16 + 64 + 2)) { rc = ERR_TRUNCATED; p = p0; break; }
        h.ts = (int64_t)be(buf + p0 + 8, 8);
        h.bl_tx_id = be(buf + p0 + 16, 8);
        memcpy(h.bl_root, buf + p0 + 24, 32);
        memcpy(h.prev_alh, buf + p0 + 56, 32);
        h.version = (uint32_t)be(buf + p0 + 88, 2);
        if (h.version == 0) {
            if (!rd(len, &p, 2)) { rc = ERR_TRUNCATED; p = p0; break; }
            h.nentries = (uint32_t)be(buf + p - 2, 2);
        } else if (h.version == 1) {
            if (!rd(len, &p, 2)) { rc = ERR_TRUNCATED; p = p0; break; }
            h.md_len = (uint32_t)be(buf + p - 2, 2);
            if (h.md_len > 268) { rc = ERR_CORRUPTED_DATA; p = p0; break; }
            if (!rd(len, &p, h.md_len)) { rc = ERR_TRUNCATED; p = p0; break; }
            /* TxMetadata.ReadFrom, then Alh over Bytes() (tx.go:483-501, 300-319) */
            uint64_t cl = 0;
            if (txmd_canonical(buf + p - h.md_len, h.md_len, txmd, &cl)) {
                rc = ERR_CORRUPTED_DATA;
                p = p0;
                break;
            }
            h.md_len = (uint32_t)cl;
            if (!rd(len, &p, 4)) { rc = ERR_TRUNCATED; p = p0; break; }
            h.nentries = (uint32_t)be(buf + p - 4, 4);
        } else {
            rc = ERR_CORRUPTED_UNKNOWN_VERSION;
            p = p0;
            break;
        }
        if (h.nentries > max_entries) { rc = ERR_CORRUPTED_MAX_ENTRIES; p = p0; break; }
        /* readEntry, tx.go:520-588 */
        int bad = 0;
        for (uint32_t e = 0; e < h.nentries && !bad; e++) {
            uint64_t q = p;
            if (!rd(len, &p, 2)) { bad = ERR_TRUNCATED; break; }
            const uint64_t ml = be(buf + q, 2);
            if (!rd(len, &p, ml)) { bad = ERR_TRUNCATED; break; }
            /* KVMetadata.unsafeReadFrom (maxKVMetadataLen 11), digest over Bytes() */
            uint8_t cmd[11];
            uint64_t cml = 0;
            if (ml && kvmd_canonical(buf + q + 2, ml, cmd, &cml)) { bad = ERR_CORRUPTED_DATA; break; }
            if (!rd(len, &p, 2)) { bad = ERR_TRUNCATED; break; }
            const uint64_t kl = be(buf + p - 2, 2);
            if (kl > max_key_len) { bad = ERR_CORRUPTED_MAX_KEYLEN; break; }
            if (!rd(len, &p, kl + 4 + 8 + 32)) { bad = ERR_TRUNCATED; break; }
            const uint8_t *key = buf + q + 4 + ml, *hv = buf + p - 32;
            int st = orc_entry_digest((int)h.version, key, kl, cml ? cmd : NULL, cml, hv,
                                      digs + 32 * (size_t)e);
            if (st) { bad = st; break; }
        }
        if (bad) { rc = bad; p = p0; break; }
        /* buildAndValidateHtree, tx.go:605-630 */
        if (!rd(len, &p, 32)) { rc = ERR_TRUNCATED; p = p0; break; }
        orc_htree_build(digs, h.nentries, lv, h.eh);
        uint8_t a[32];
        orc_tx_header_alh(&h, txmd, NULL, a);
        /* the md blob for orc_tx_header_alh is txmd itself at offset 0 */
        if (alh_out) memcpy(alh_out + 32 * ntx, a, 32);
        if (status_out) status_out[ntx] = memcmp(a, buf + p - 32, 32) ? ERR_CORRUPTED_DATA : OK;
        ntx++;
    }
    free(digs);
    free(lv);
    if (ntx_out) *ntx_out = ntx;
    if (consumed_out) *consumed_out = p;
    return rc;
}
