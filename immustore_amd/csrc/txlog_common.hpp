// txlog_common.hpp -- device helpers shared by the fused a14 kernels
// (txlog_wave.hip, txlog_lanes.hip, txlog_struct.hip): byte-order reads of the
// raw tx-log records (tx.go:419-588 layout) and the entry-digest block builder
// of TxEntryDigest_v1_1 / _v1_2 (tx.go:690-731) straight from the record.
#pragma once

#include "digest_io.hpp"
#include "mh_internal.hpp"

namespace mh {

__device__ __constant__ static const uint8_t kTxlEmptyRoot[32] = {  // SHA256(nil), htree.go:73-77
    0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4, 0xc8, 0x99, 0x6f, 0xb9, 0x24,
    0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

__device__ __forceinline__ uint32_t rd_le32(const uint8_t *p) {  // 4 bytes of any alignment
    const uint32_t al = (uint32_t)((uintptr_t)p & 3);
    const uint32_t *b = reinterpret_cast<const uint32_t *>(p - al);
    return __builtin_amdgcn_alignbyte(b[1], b[0], al);
}
__device__ __forceinline__ uint32_t rd_be16(const uint8_t *p) {
    return ((uint32_t)p[0] << 8) | p[1];
}
__device__ __forceinline__ uint64_t rd_be64(const uint8_t *p) {
    return ((uint64_t)bswap(rd_le32(p)) << 32) | bswap(rd_le32(p + 4));
}
__device__ __forceinline__ uint64_t rd_raw64(const uint8_t *p) {
    return (uint64_t)rd_le32(p) | ((uint64_t)rd_le32(p + 4) << 32);
}

constexpr int kTxMsgWords = 96;  // innerHash message <= 356 B: 6 blocks
typedef __attribute__((address_space(3))) void tx_lds_void_t;
typedef __attribute__((address_space(1))) void tx_glb_void_t;

// first min(max(n, 0), 4) bytes of a big-endian word: (~0 << 32) >> 8c
__device__ __forceinline__ uint32_t head_mask(int n) {
    const int c = min(max(n, 0), 4);
    return (uint32_t)(0xffffffff00000000ull >> (8 * c));
}

// block b of nb of SHA256(p[0:la] || p[la+12 : la+44]) (sha256_skip12's
// words), padding included: the 20 dwords block b reads from its aligned start
// (unguarded: the caller guarantees >= 96 readable bytes past the message)
__device__ __forceinline__ void skip12_load(const uint8_t *p, uint32_t b, uint32_t d[20]) {
    const uint32_t *qq = reinterpret_cast<const uint32_t *>(p - ((uintptr_t)p & 3)) + b * 16;
#pragma unroll
    for (int j = 0; j < 20; j++) d[j] = qq[j];
}
// Message words j = 0..15 of block b from the 20 dwords d[] read at the
// block's aligned start (al = p & 3, hv0 = la - 64 b): the head bytes, then
// the hVal 12 bytes further on, cut at the message end (la + 32 - 64 b) with
// the 0x80 marker after it.  Each word's bytes come out of one v_perm (the
// byte-aligned window and the big-endian swap in one selector); the end mask
// of word j is the head mask of word j - 8 (the message ends 32 bytes after
// the head), and the marker is the one byte by which the end mask of a
// message one byte longer, (em_j >> 8) | (em_{j-1} << 24), exceeds em_j --
// 25 masks for the 48 masks and markers of the direct form.
__device__ __forceinline__ void skip12_assemble(const uint32_t d[20], uint32_t al, int hv0,
                                                uint32_t w[16]) {
    const uint32_t sel = be_sel(al);
    uint32_t hm[25];  // hm[k] = head_mask(hv0 - 4 (k - 9)): words -9..15
#pragma unroll
    for (int k = 0; k < 25; k++) hm[k] = head_mask(hv0 - 4 * (k - 9));
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t w1 = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
        const uint32_t w2 = __builtin_amdgcn_perm(d[j + 4], d[j + 3], sel);
        const uint32_t x = __builtin_amdgcn_bitop3_b32(hm[j + 9], w1, w2, 0xCA);  // head ? w1 : w2
        const uint32_t em = hm[j + 1], nm = __builtin_amdgcn_alignbit(hm[j], em, 8);
        w[j] = __builtin_amdgcn_bitop3_b32(em, x, nm & 0x80808080u, 0xCA);  // message ? x : marker
    }
}
// the block's message words from those dwords (al = p & 3)
__device__ __forceinline__ void skip12_words(const uint32_t d[20], uint32_t al, uint32_t la,
                                             uint32_t b, uint32_t nb, uint32_t w[16]) {
    const uint32_t L = la + 32;
    skip12_assemble(d, al, (int)la - (int)(b * 64), w);
    if (b + 1 == nb) {
        w[14] = 0;
        w[15] = L * 8;
    }
}
// GUARD: loads confined to [p, p + la + 44) (the log in HBM, no slack assumed)
template <bool GUARD>
__device__ __forceinline__ void skip12_block(const uint8_t *p, uint32_t la, uint32_t b,
                                             uint32_t nb, uint32_t w[16]) {
    const uint32_t al = (uint32_t)((uintptr_t)p & 3);
    const uint32_t *qq = reinterpret_cast<const uint32_t *>(p - al) + b * 16;
    uint32_t d[20];
    if (GUARD) {
        const uint8_t *end = p + la + 44;
#pragma unroll
        for (int j = 0; j < 20; j++) d[j] = ld_guard(qq + j, p, end);
    } else {
#pragma unroll
        for (int j = 0; j < 20; j++) d[j] = qq[j];
    }
    skip12_words(d, al, la, b, nb, w);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, m, 64));
    return x;
}

// a wave's LDS writes complete and visible to its other lanes (each wave
// works in its own LDS slices: no workgroup barrier)
__device__ __forceinline__ void txl_wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

}  // namespace mh
