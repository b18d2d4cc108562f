// sha256_cdna.hpp -- SHA-256 compression for CDNA4 (gfx950), one message per lane.
//
// The whole path is 32-bit integer VALU work (add / rotate / xor / bitfield
// select); there is nothing MFMA-shaped in it.  The round function is written
// so that the compiler emits the CDNA4 instructions that fuse the most work:
//   rotr        -> v_alignbit_b32          (1 op)
//   Sigma0/1    -> 3x v_alignbit + v_xor3_b32
//   Ch(e,f,g)   -> v_bfi_b32               (1 op)
//   Maj(a,b,c)  -> v_bfi_b32(a^b, c, b)    (xor + bfi, the xor reused next round)
//   T1 sums     -> v_add3_u32
// Message words are held in VGPRs as a 16-entry rolling window (fully
// unrolled, so no indexing ever reaches scratch).  Blocks whose message
// schedule is a compile-time or launch-time constant (the padding block of a
// 64-byte-multiple value) take a precomputed K+W table from SGPRs instead.
//
// FIPS 180-4; matches Go crypto/sha256 (the reference's only hash primitive,
// SURVEY.md section 1 L0).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mh {

__device__ __constant__ static const uint32_t kK256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

// Compile-time copy for constant folding inside fully unrolled rounds.
#define MH_K(i)                                                                                   \
    ((i) == 0 ? 0x428a2f98u : (i) == 1 ? 0x71374491u : (i) == 2 ? 0xb5c0fbcfu                   \
     : (i) == 3 ? 0xe9b5dba5u : (i) == 4 ? 0x3956c25bu : (i) == 5 ? 0x59f111f1u                  \
     : (i) == 6 ? 0x923f82a4u : (i) == 7 ? 0xab1c5ed5u : (i) == 8 ? 0xd807aa98u                  \
     : (i) == 9 ? 0x12835b01u : (i) == 10 ? 0x243185beu : (i) == 11 ? 0x550c7dc3u                \
     : (i) == 12 ? 0x72be5d74u : (i) == 13 ? 0x80deb1feu : (i) == 14 ? 0x9bdc06a7u               \
     : (i) == 15 ? 0xc19bf174u : (i) == 16 ? 0xe49b69c1u : (i) == 17 ? 0xefbe4786u               \
     : (i) == 18 ? 0x0fc19dc6u : (i) == 19 ? 0x240ca1ccu : (i) == 20 ? 0x2de92c6fu               \
     : (i) == 21 ? 0x4a7484aau : (i) == 22 ? 0x5cb0a9dcu : (i) == 23 ? 0x76f988dau               \
     : (i) == 24 ? 0x983e5152u : (i) == 25 ? 0xa831c66du : (i) == 26 ? 0xb00327c8u               \
     : (i) == 27 ? 0xbf597fc7u : (i) == 28 ? 0xc6e00bf3u : (i) == 29 ? 0xd5a79147u               \
     : (i) == 30 ? 0x06ca6351u : (i) == 31 ? 0x14292967u : (i) == 32 ? 0x27b70a85u               \
     : (i) == 33 ? 0x2e1b2138u : (i) == 34 ? 0x4d2c6dfcu : (i) == 35 ? 0x53380d13u               \
     : (i) == 36 ? 0x650a7354u : (i) == 37 ? 0x766a0abbu : (i) == 38 ? 0x81c2c92eu               \
     : (i) == 39 ? 0x92722c85u : (i) == 40 ? 0xa2bfe8a1u : (i) == 41 ? 0xa81a664bu               \
     : (i) == 42 ? 0xc24b8b70u : (i) == 43 ? 0xc76c51a3u : (i) == 44 ? 0xd192e819u               \
     : (i) == 45 ? 0xd6990624u : (i) == 46 ? 0xf40e3585u : (i) == 47 ? 0x106aa070u               \
     : (i) == 48 ? 0x19a4c116u : (i) == 49 ? 0x1e376c08u : (i) == 50 ? 0x2748774cu               \
     : (i) == 51 ? 0x34b0bcb5u : (i) == 52 ? 0x391c0cb3u : (i) == 53 ? 0x4ed8aa4au               \
     : (i) == 54 ? 0x5b9cca4fu : (i) == 55 ? 0x682e6ff3u : (i) == 56 ? 0x748f82eeu               \
     : (i) == 57 ? 0x78a5636fu : (i) == 58 ? 0x84c87814u : (i) == 59 ? 0x8cc70208u               \
     : (i) == 60 ? 0x90befffau : (i) == 61 ? 0xa4506cebu : (i) == 62 ? 0xbef9a3f7u               \
                 : 0xc67178f2u)

static constexpr uint32_t kH0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
// gfx950 has a 3-input bitwise LUT instruction (v_bitop3_b32).  LUT bits are
// indexed with src0 = 0xF0, src1 = 0xCC, src2 = 0xAA (LOP3 convention).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }
// Ch(e,f,g) = (e&f)^(~e&g): LUT 0xCA
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
// Maj(a,b,c) = (a&b)|(a&c)|(b&c): LUT 0xE8
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// Big-endian load helper: bytes in memory -> SHA word.
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

struct State {
    uint32_t h[8];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int i = 0; i < 8; i++) h[i] = kH0[i];
    }
};

// One round with explicit K+W value.
#define MH_ROUND(a, b, c, d, e, f, g, h, kw)                                                      \
    do {                                                                                          \
        uint32_t t1_ = (h + (kw)) + (bsig1(e) + ch(e, f, g));                                     \
        d += t1_;                                                                                 \
        h = t1_ + (bsig0(a) + maj(a, b, c));                                                      \
    } while (0)

// Compress one block whose 16 message words are in w[] (values, may be
// compile-time constants after inlining: the compiler folds the schedule).
__device__ __forceinline__ void compress(State &s, const uint32_t win[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = win[i];
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6],
             h = s.h[7];
#pragma unroll
    for (int r = 0; r < 64; r += 8) {
        if (r >= 16) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int t = r + j;
                w[t & 15] = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) +
                            w[t & 15];
            }
        }
        MH_ROUND(a, b, c, d, e, f, g, h, MH_K(r + 0) + w[(r + 0) & 15]);
        MH_ROUND(h, a, b, c, d, e, f, g, MH_K(r + 1) + w[(r + 1) & 15]);
        MH_ROUND(g, h, a, b, c, d, e, f, MH_K(r + 2) + w[(r + 2) & 15]);
        MH_ROUND(f, g, h, a, b, c, d, e, MH_K(r + 3) + w[(r + 3) & 15]);
        MH_ROUND(e, f, g, h, a, b, c, d, MH_K(r + 4) + w[(r + 4) & 15]);
        MH_ROUND(d, e, f, g, h, a, b, c, MH_K(r + 5) + w[(r + 5) & 15]);
        MH_ROUND(c, d, e, f, g, h, a, b, MH_K(r + 6) + w[(r + 6) & 15]);
        MH_ROUND(b, c, d, e, f, g, h, a, MH_K(r + 7) + w[(r + 7) & 15]);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// Compress a block whose whole schedule (K[t]+W[t], t = 0..63) is known and
// uniform across the launch: kw[] lives in SGPRs / scalar constant memory.
__device__ __forceinline__ void compress_kw(State &s, const uint32_t *__restrict__ kw) {
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6],
             h = s.h[7];
#pragma unroll
    for (int r = 0; r < 64; r += 8) {
        MH_ROUND(a, b, c, d, e, f, g, h, kw[r + 0]);
        MH_ROUND(h, a, b, c, d, e, f, g, kw[r + 1]);
        MH_ROUND(g, h, a, b, c, d, e, f, kw[r + 2]);
        MH_ROUND(f, g, h, a, b, c, d, e, kw[r + 3]);
        MH_ROUND(e, f, g, h, a, b, c, d, kw[r + 4]);
        MH_ROUND(d, e, f, g, h, a, b, c, kw[r + 5]);
        MH_ROUND(c, d, e, f, g, h, a, b, kw[r + 6]);
        MH_ROUND(b, c, d, e, f, g, h, a, kw[r + 7]);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// leaf = SHA256(0x00 || d), d given as 8 big-endian words (33-byte message,
// one block: htree.go:79-83, ahtree.go:288-292).
__device__ __forceinline__ void leaf_hash(const uint32_t d[8], uint32_t out[8]) {
    uint32_t w[16];
    w[0] = d[0] >> 8;
#pragma unroll
    for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(d[j - 1], d[j], 8);
    w[8] = (d[7] << 24) | 0x00800000u;
#pragma unroll
    for (int j = 9; j < 15; j++) w[j] = 0;
    w[15] = 33u * 8u;
    State s;
    s.init();
    compress(s, w);
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = s.h[j];
}

// node = SHA256(0x01 || l || r) (65-byte message, two blocks: htree.go:89-97).
__device__ __forceinline__ void node_hash(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
    uint32_t w[16];
    w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(l[j - 1], l[j], 8);
    w[8] = __builtin_amdgcn_alignbit(l[7], r[0], 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[8 + j] = __builtin_amdgcn_alignbit(r[j - 1], r[j], 8);
    State s;
    s.init();
    compress(s, w);
    w[0] = (r[7] << 24) | 0x00800000u;
#pragma unroll
    for (int j = 1; j < 15; j++) w[j] = 0;
    w[15] = 65u * 8u;
    compress(s, w);
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = s.h[j];
}

// ---------------------------------------------------------------------------
// Node hashes against a per-workgroup schedule table.
//
// The second block of a node hash (65-byte message) is
//   W0 = r[31] << 24 | 0x80 << 16,  W1..W14 = 0,  W15 = 520,
// so its whole message schedule is a function of ONE byte, r[31].  A
// workgroup that hashes many nodes builds the 256 possible schedules once in
// LDS (K[t] + W[t] for t = 16..63; rounds 0..15 fold to immediates) and the
// block then runs like compress_kw: no schedule expansion, 12 ds_read_b128
// per block instead of ~490 VALU ops (about 17 % of a node hash).  Rows are
// padded to 52 words (13 x 16 B) so rows of different lanes spread over the
// LDS bank groups.
constexpr int kNodeTabStride = 52;
constexpr int kNodeTabWords = 256 * kNodeTabStride;
constexpr int kNodeTabBytes = kNodeTabWords * 4;

// The table is a compile-time constant (constexpr schedule expansion); every
// workgroup copies it from global memory (L2 resident after the first
// touch) into LDS.
struct alignas(16) NodeTab {
    uint32_t w[kNodeTabWords];
};

constexpr NodeTab make_node_tab() {
    constexpr uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
        0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
        0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
        0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
        0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
        0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
        0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
        0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
        0xc67178f2u};
    NodeTab t{};
    for (uint32_t v = 0; v < 256; v++) {
        uint32_t w[64] = {};
        w[0] = (v << 24) | 0x00800000u;
        w[15] = 65u * 8u;
        for (int i = 16; i < 64; i++) {
            const uint32_t x = w[i - 15], y = w[i - 2];
            const uint32_t s0 = ((x >> 7) | (x << 25)) ^ ((x >> 18) | (x << 14)) ^ (x >> 3);
            const uint32_t s1 = ((y >> 17) | (y << 15)) ^ ((y >> 19) | (y << 13)) ^ (y >> 10);
            w[i] = s1 + w[i - 7] + s0 + w[i - 16];
            t.w[v * kNodeTabStride + (i - 16)] = w[i] + K[i];
        }
    }
    return t;
}

__device__ static const NodeTab g_node_tab = make_node_tab();

__device__ __forceinline__ void node_tab_init(uint32_t *tab) {
    const uint4 *src = (const uint4 *)g_node_tab.w;
    uint4 *dst = (uint4 *)tab;
    for (int i = threadIdx.x; i < kNodeTabWords / 4; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

#define MH_ROUNDS8(k0, k1, k2, k3, k4, k5, k6, k7)                                                \
    do {                                                                                          \
        MH_ROUND(a, b, c, d, e, f, g, h, k0);                                                     \
        MH_ROUND(h, a, b, c, d, e, f, g, k1);                                                     \
        MH_ROUND(g, h, a, b, c, d, e, f, k2);                                                     \
        MH_ROUND(f, g, h, a, b, c, d, e, k3);                                                     \
        MH_ROUND(e, f, g, h, a, b, c, d, k4);                                                     \
        MH_ROUND(d, e, f, g, h, a, b, c, k5);                                                     \
        MH_ROUND(c, d, e, f, g, h, a, b, k6);                                                     \
        MH_ROUND(b, c, d, e, f, g, h, a, k7);                                                     \
    } while (0)

// Second block of SHA256(0x01 || l || r) given r's last word.
__device__ __forceinline__ void compress_node_tail(State &s, uint32_t r7,
                                                   const uint32_t *__restrict__ tab) {
    const uint4 *row = (const uint4 *)(tab + (r7 & 0xffu) * kNodeTabStride);
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6],
             h = s.h[7];
    MH_ROUNDS8(MH_K(0) + ((r7 << 24) | 0x00800000u), MH_K(1), MH_K(2), MH_K(3), MH_K(4), MH_K(5),
               MH_K(6), MH_K(7));
    MH_ROUNDS8(MH_K(8), MH_K(9), MH_K(10), MH_K(11), MH_K(12), MH_K(13), MH_K(14),
               MH_K(15) + 65u * 8u);
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const uint4 x = row[2 * q], y = row[2 * q + 1];
        MH_ROUNDS8(x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// node = SHA256(0x01 || l || r) with the second block from the LDS table.
__device__ __forceinline__ void node_hash_tab(const uint32_t l[8], const uint32_t r[8],
                                              uint32_t out[8], const uint32_t *__restrict__ tab) {
    uint32_t w[16];
    w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(l[j - 1], l[j], 8);
    w[8] = __builtin_amdgcn_alignbit(l[7], r[0], 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[8 + j] = __builtin_amdgcn_alignbit(r[j - 1], r[j], 8);
    State s;
    s.init();
    compress(s, w);
    compress_node_tail(s, r[7], tab);
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = s.h[j];
}

// Second block of SHA256(0x01 || l || r) given r's last word, its K+W row
// read from the table in GLOBAL memory (L2-resident): the node hash's
// padding block without the ~480-instruction schedule expansion.
__device__ __forceinline__ void compress_node_tail_g(State &s, uint32_t r7) {
    const uint4 *row = (const uint4 *)(g_node_tab.w + (r7 & 0xffu) * kNodeTabStride);
    uint4 kw[12];
#pragma unroll
    for (int q = 0; q < 12; q++) kw[q] = row[q];
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6],
             h = s.h[7];
    MH_ROUNDS8(MH_K(0) + ((r7 << 24) | 0x00800000u), MH_K(1), MH_K(2), MH_K(3), MH_K(4), MH_K(5),
               MH_K(6), MH_K(7));
    MH_ROUNDS8(MH_K(8), MH_K(9), MH_K(10), MH_K(11), MH_K(12), MH_K(13), MH_K(14),
               MH_K(15) + 65u * 8u);
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const uint4 x = kw[2 * q], y = kw[2 * q + 1];
        MH_ROUNDS8(x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w);
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// node = SHA256(0x01 || l || r) with the second block's K+W row read from
// the table in GLOBAL memory (L2-resident): for latency-bound lone waves at
// the top of a tree, where a workgroup cannot afford the 53 KB LDS copy.  The
// 12 row loads are issued before the first block, whose ~1400 VALU
// instructions hide their latency.
__device__ __forceinline__ void node_hash_g(const uint32_t l[8], const uint32_t r[8],
                                            uint32_t out[8]) {
    const uint4 *row = (const uint4 *)(g_node_tab.w + (r[7] & 0xffu) * kNodeTabStride);
    uint4 kw[12];
#pragma unroll
    for (int q = 0; q < 12; q++) kw[q] = row[q];
    uint32_t w[16];
    w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(l[j - 1], l[j], 8);
    w[8] = __builtin_amdgcn_alignbit(l[7], r[0], 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[8 + j] = __builtin_amdgcn_alignbit(r[j - 1], r[j], 8);
    State s;
    s.init();
    compress(s, w);
    const uint32_t r7 = r[7];
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6],
             h = s.h[7];
    MH_ROUNDS8(MH_K(0) + ((r7 << 24) | 0x00800000u), MH_K(1), MH_K(2), MH_K(3), MH_K(4), MH_K(5),
               MH_K(6), MH_K(7));
    MH_ROUNDS8(MH_K(8), MH_K(9), MH_K(10), MH_K(11), MH_K(12), MH_K(13), MH_K(14),
               MH_K(15) + 65u * 8u);
#pragma unroll
    for (int q = 0; q < 6; q++) {
        const uint4 x = kw[2 * q], y = kw[2 * q + 1];
        MH_ROUNDS8(x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w);
    }
    out[0] = s.h[0] + a; out[1] = s.h[1] + b; out[2] = s.h[2] + c; out[3] = s.h[3] + d;
    out[4] = s.h[4] + e; out[5] = s.h[5] + f; out[6] = s.h[6] + g; out[7] = s.h[7] + h;
}

}  // namespace mh
