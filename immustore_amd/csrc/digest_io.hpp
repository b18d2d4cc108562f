// digest_io.hpp -- device-side byte <-> SHA word movement shared by the
// kernel translation units.
#pragma once
#include "sha256_cdna.hpp"

namespace mh {

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ void load_digest(const uint8_t *p, uint32_t w[8]) {
    const uint4 a = *reinterpret_cast<const uint4 *>(p);
    const uint4 b = *reinterpret_cast<const uint4 *>(p + 16);
    w[0] = bswap(a.x); w[1] = bswap(a.y); w[2] = bswap(a.z); w[3] = bswap(a.w);
    w[4] = bswap(b.x); w[5] = bswap(b.y); w[6] = bswap(b.z); w[7] = bswap(b.w);
}

__device__ __forceinline__ void store_digest(uint8_t *p, const uint32_t w[8]) {
    uint4 a, b;
    a.x = bswap(w[0]); a.y = bswap(w[1]); a.z = bswap(w[2]); a.w = bswap(w[3]);
    b.x = bswap(w[4]); b.y = bswap(w[5]); b.z = bswap(w[6]); b.w = bswap(w[7]);
    *reinterpret_cast<uint4 *>(p) = a;
    *reinterpret_cast<uint4 *>(p + 16) = b;
}

__device__ __forceinline__ void copy8(uint32_t d[8], const uint32_t s[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++) d[j] = s[j];
}


// ============================================================================
// Generic SHA-256 over one per-lane byte range of any alignment and length,
// optionally preceded by one prefix byte (pre >= 0): SHA256(pre || p[0:len]).
// Used by the general CSR path (values, entry-digest messages) and by ahtree
// leaves of arbitrary payload size (ahtree.go:288-292).
// ============================================================================
__device__ __forceinline__ uint32_t ld_guard(const uint32_t *p, const uint8_t *lo,
                                             const uint8_t *hi) {
    const uint8_t *b = reinterpret_cast<const uint8_t *>(p);
    return (b + 4 > lo && b < hi) ? *p : 0u;
}

// bswap(alignbyte(hi, lo, al)) -- the big-endian message word at byte al of
// the 8 bytes lo || hi -- as ONE v_perm: output byte k is byte 3 - k + al
__device__ __forceinline__ uint32_t be_sel(uint32_t al) { return 0x00010203u + al * 0x01010101u; }

__device__ inline void sha256_bytes(const uint8_t *p, uint64_t len, int pre, uint32_t out[8]) {
    State s;
    s.init();
    const uint64_t L = len + (pre >= 0 ? 1 : 0);   // virtual message length
    const uint8_t *q = p - (pre >= 0 ? 1 : 0);       // virtual byte 0 address
    const uint32_t al = (uint32_t)((uintptr_t)q & 3), sel = be_sel(al);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(q - al);
    const uint8_t *end = p + len;
    const uint64_t nfull = L >> 6;
    for (uint64_t b = 0; b < nfull; b++) {
        const uint32_t *qq = base + b * 16;
        uint32_t d[17], w[16];
        if (b == 0 && pre >= 0) {
#pragma unroll
            for (int j = 0; j < 17; j++) d[j] = ld_guard(qq + j, p, end);
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) d[j] = qq[j];
            d[16] = al ? ld_guard(qq + 16, p, end) : 0u;
        }
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
        if (b == 0 && pre >= 0) w[0] = (w[0] & 0x00ffffffu) | ((uint32_t)pre << 24);
        compress(s, w);
    }
    const uint32_t rem = (uint32_t)(L - nfull * 64);
    const uint32_t *qq = base + nfull * 16;
    uint32_t d[17], w[32];
#pragma unroll
    for (int j = 0; j < 17; j++) d[j] = ld_guard(qq + j, p, end);
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t x = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
        const int v = (int)rem - 4 * j;  // valid bytes in this word
        const uint32_t m = v >= 4 ? 0xffffffffu : (v <= 0 ? 0u : (0xffffffffu << (32 - 8 * v)));
        x &= m;
        if (v >= 0 && v < 4) x |= 0x80u << (24 - 8 * v);
        w[j] = x;
    }
    if (nfull == 0 && pre >= 0) w[0] = (w[0] & 0x00ffffffu) | ((uint32_t)pre << 24);
#pragma unroll
    for (int j = 16; j < 32; j++) w[j] = 0;
    const uint64_t bits = L * 8;
    if (rem < 56) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        compress(s, w);
    } else {
        w[30] = (uint32_t)(bits >> 32);
        w[31] = (uint32_t)bits;
        compress(s, w);
        compress(s, w + 16);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = s.h[j];
}

// ============================================================================
// SHA-256 of p[0:la] || p[la+12 : la+44]: an entry-digest message read in
// place from a raw tx-log entry record (BE16 mdLen | md | BE16 kLen | key |
// BE32 vLen | BE64 vOff | hVal, tx.go:520-588), skipping the 12 bytes of
// vLen / vOff between the head and hVal.  Both views of the record have the
// same alignment (12 = 3 dwords), so every message word is a byte-select of
// two alignbyte words.  Full blocks may read up to 36 bytes past hVal, still
// inside the record (its 32-byte Alh follows the last entry); the last block's
// loads are guarded to [p, p + la + 44).
// ============================================================================
__device__ inline void sha256_skip12(const uint8_t *p, uint32_t la, uint32_t out[8]) {
    State s;
    s.init();
    const uint32_t L = la + 32;
    const uint32_t al = (uint32_t)((uintptr_t)p & 3), sel = be_sel(al);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(p - al);
    const uint8_t *end = p + la + 44;
    const uint32_t nfull = L >> 6;
    auto word = [&](const uint32_t d[20], int j, uint32_t x0) {
        const uint32_t w1 = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
        const uint32_t w2 = __builtin_amdgcn_perm(d[j + 4], d[j + 3], sel);
        const int v = (int)la - (int)(x0 + 4 * j);  // head bytes in this word
        const uint32_t m = v >= 4 ? 0xffffffffu : (v <= 0 ? 0u : (0xffffffffu << (32 - 8 * v)));
        return (w1 & m) | (w2 & ~m);
    };
    for (uint32_t b = 0; b < nfull; b++) {
        const uint32_t *qq = base + b * 16;
        uint32_t d[20], w[16];
#pragma unroll
        for (int j = 0; j < 20; j++) d[j] = qq[j];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = word(d, j, b * 64);
        compress(s, w);
    }
    const uint32_t rem = L - nfull * 64;
    const uint32_t *qq = base + nfull * 16;
    uint32_t d[20], w[32];
#pragma unroll
    for (int j = 0; j < 20; j++) d[j] = ld_guard(qq + j, p, end);
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t x = word(d, j, nfull * 64);
        const int v = (int)rem - 4 * j;  // valid bytes in this word
        const uint32_t m = v >= 4 ? 0xffffffffu : (v <= 0 ? 0u : (0xffffffffu << (32 - 8 * v)));
        x &= m;
        if (v >= 0 && v < 4) x |= 0x80u << (24 - 8 * v);
        w[j] = x;
    }
#pragma unroll
    for (int j = 16; j < 32; j++) w[j] = 0;
    const uint64_t bits = (uint64_t)L * 8;
    if (rem < 56) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        compress(s, w);
    } else {
        w[30] = (uint32_t)(bits >> 32);
        w[31] = (uint32_t)bits;
        compress(s, w);
        compress(s, w + 16);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = s.h[j];
}

}  // namespace mh
