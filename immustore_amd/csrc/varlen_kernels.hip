// varlen_kernels.hip -- SHA-256 over ragged byte ranges (CSR buffer + u64
// offsets), one message per lane, for the general entry path:
//   value hash          embedded/store/immustore.go:1620-1630 (IsValueTruncated
//                        entries take the caller's hVal instead, :1624-1626)
//   entry digests       embedded/store/tx.go:690-731 (assembled messages)
//   pkg/verification    EntrySpecDigest over document entries
// Real EntrySpecs are ragged (value <= 4096 B, key <= 1024 B, metadata <= 11 B;
// embedded/store/options.go:37-39), so one lane per message in input order
// leaves a wave running as many compressions as its longest message.  Here
// the messages are first bucketed by block count (a counting sort over 1024
// buckets, heaviest first), so every wave hashes messages of one length
// class and runs no idle blocks; the heaviest waves are dispatched first,
// which also balances the tail of the launch.
//
// Per block a lane reads a 68-byte window of its message (dword-aligned
// dwordx4 loads; the next block's window is loaded under the current
// compression), and one v_perm_b32 per word both realigns and byte-swaps it.
// Only the last two blocks of a message need the byte masks, the 0x80 pad
// and the bit length; they run a separate (wave-uniform) branch.
#include <cstdlib>

#include "mh_internal.hpp"
#include "sha256_cdna.hpp"
#include "digest_io.hpp"

namespace mh {

constexpr int kNbBuckets = 1024;     // block-count classes (longer messages share the last)
constexpr int kNbChunk = 256 * 16;   // entries per workgroup of the sort passes

// blocks of SHA256(message of L bytes) incl. padding: (L + 9 + 63) / 64;
// entries hashed from an override count 0 (no compression)
__device__ __forceinline__ uint32_t nb_key(const uint64_t *off, const uint8_t *use, uint64_t i) {
    if (use && use[i]) return 0;
    const uint64_t nb = ((off[i + 1] >= off[i] ? off[i + 1] - off[i] : 0) + 72) >> 6;
    return (uint32_t)(nb < (uint64_t)kNbBuckets ? nb : (uint64_t)kNbBuckets - 1);
}

// bucket slot in sort order: descending block count
__device__ __forceinline__ uint32_t nb_slot(uint32_t key) { return kNbBuckets - 1 - key; }

__global__ __launch_bounds__(256) void k_nb_hist(const uint64_t *__restrict__ off,
                                                 const uint8_t *__restrict__ use, uint64_t n,
                                                 uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[kNbBuckets];
    for (int k = threadIdx.x; k < kNbBuckets; k += 256) h[k] = 0;
    __syncthreads();
    const uint64_t e0 = (uint64_t)blockIdx.x * kNbChunk;
    for (int k = threadIdx.x; k < kNbChunk; k += 256) {
        const uint64_t i = e0 + k;
        if (i < n) atomicAdd(&h[nb_slot(nb_key(off, use, i))], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kNbBuckets; k += 256)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}

// exclusive scan of the bucket counts -> bucket cursors (one workgroup)
__global__ __launch_bounds__(kNbBuckets) void k_nb_scan(const uint32_t *__restrict__ hist,
                                                        uint32_t *__restrict__ cursor) {
    __shared__ uint32_t s[kNbBuckets];
    const int t = threadIdx.x;
    const uint32_t x = hist[t];
    s[t] = x;
    __syncthreads();
    for (int d = 1; d < kNbBuckets; d <<= 1) {
        const uint32_t y = t >= d ? s[t - d] : 0;
        __syncthreads();
        s[t] += y;
        __syncthreads();
    }
    cursor[t] = s[t] - x;
}

// perm[cursor[slot] + rank] = i; ranks inside a bucket are in any order (the
// hash of entry i is written at i, so the result does not depend on it)
__global__ __launch_bounds__(256) void k_nb_scatter(const uint64_t *__restrict__ off,
                                                    const uint8_t *__restrict__ use, uint64_t n,
                                                    uint32_t *__restrict__ cursor,
                                                    uint32_t *__restrict__ perm) {
    __shared__ uint32_t h[kNbBuckets];
    __shared__ uint32_t base[kNbBuckets];
    for (int k = threadIdx.x; k < kNbBuckets; k += 256) h[k] = 0;
    __syncthreads();
    const uint64_t e0 = (uint64_t)blockIdx.x * kNbChunk;
    constexpr int kPer = kNbChunk / 256;
    uint32_t slot[kPer], rank[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint64_t i = e0 + threadIdx.x + r * 256;
        if (i < n) {
            slot[r] = nb_slot(nb_key(off, use, i));
            rank[r] = atomicAdd(&h[slot[r]], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kNbBuckets; k += 256)
        base[k] = h[k] ? atomicAdd(&cursor[k], h[k]) : 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint64_t i = e0 + threadIdx.x + r * 256;
        if (i < n) perm[base[slot[r]] + rank[r]] = (uint32_t)i;
    }
}

// dword-aligned 16-byte load (gfx950 global loads need only dword alignment
// for multi-dword widths)
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ void load_window(const uint32_t *q, uint32_t d[17]) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const u32x4_a4 v = *reinterpret_cast<const u32x4_a4 *>(q + 4 * c);
        d[4 * c + 0] = v.x;
        d[4 * c + 1] = v.y;
        d[4 * c + 2] = v.z;
        d[4 * c + 3] = v.w;
    }
    d[16] = q[16];
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, m, 64));
    return x;
}

// Byte mask of the first v bytes of a big-endian word (v clamped to 0..4).
__device__ __forceinline__ uint32_t hi_mask(int v) {
    return v >= 4 ? 0xffffffffu : (v <= 0 ? 0u : (0xffffffffu << (32 - 8 * v)));
}

__device__ __forceinline__ int clamp_rel(int64_t x) {
    return (int)(x < -8 ? -8 : (x > 72 ? 72 : x));
}

// Per-lane view of one message in memory for the value phase: p = first byte,
// L = length; the block builder keeps the next window prefetched.
struct MsgWalk {
    const uint32_t *q;      // dword holding p
    const uint32_t *qlast;  // dword holding the last byte
    uint32_t sel;           // v_perm selector of p's alignment
    uint64_t L;
    uint32_t d[17];         // window of the current block (loaded one block ahead)
    bool pre;               // d already holds this block's window

    __device__ __forceinline__ void init(const uint8_t *p, uint64_t len) {
        const uint32_t al = (uint32_t)((uintptr_t)p & 3);
        q = reinterpret_cast<const uint32_t *>(p - al);
        qlast = reinterpret_cast<const uint32_t *>((uintptr_t)(p + len - 1) & ~(uintptr_t)3);
        sel = 0x00010203u + al * 0x01010101u;
        L = len;
        pre = false;
    }

    // Message words of block b for the lanes with `on`.  fast (wave-uniform):
    // every active lane has >= 2 more blocks after b, so its 68-byte window
    // and the next one lie inside the message; the words are taken from d and
    // the same registers then receive the next block's window, which lands
    // under this block's compression.  Otherwise the general form (clamped
    // loads, byte masks, 0x80, bit length in the last block nb-1).
    __device__ __forceinline__ void block(uint32_t b, uint32_t nb, bool on, bool fast,
                                          uint32_t w[16]) {
        if (fast) {
            if (!pre && on) load_window(q + 16 * (uint64_t)b, d);
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
            pre = on && b + 3 < nb;
            if (pre) load_window(q + 16 * (uint64_t)(b + 1), d);
            return;
        }
        pre = false;
        uint32_t x[17];
#pragma unroll
        for (int j = 0; j < 17; j++) x[j] = 0;
        if (on && L) {
            const uint32_t *qb = q + 16 * (uint64_t)b;
#pragma unroll
            for (int j = 0; j < 17; j++) x[j] = *(qb + j <= qlast ? qb + j : qlast);
        }
        const int r = clamp_rel((int64_t)L - 64 * (int64_t)b);  // data bytes left at block start
#pragma unroll
        for (int j = 0; j < 16; j++) {
            uint32_t y = __builtin_amdgcn_perm(x[j + 1], x[j], sel);
            const int v = r - 4 * j;  // valid bytes in this word
            y &= hi_mask(v);
            if (v >= 0 && v < 4) y |= 0x80u << (24 - 8 * v);
            w[j] = y;
        }
        if (b + 1 == nb) {
            const uint64_t bits = L * 8;
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
    }
};

// One lane per message; lanes take messages in perm order (or input order
// when perm is null).  out32[i] = SHA256(buf[off[i] .. off[i+1])), or
// override32[i] where use_override[i] != 0.  With cmp.expect (the read-side
// check of readValueAt, immustore.go:3235): status[i] = MH_OK when the
// message's length equals exp_len[i] (when given) and its digest equals
// expect[i], else MH_ERR_CORRUPTED_DATA; out32 may then be null.
struct ShaCompare {
    const uint8_t *expect = nullptr;
    const uint64_t *exp_len = nullptr;
    int32_t *status = nullptr;
};

__global__ __launch_bounds__(256) void k_sha_varlen(const uint8_t *__restrict__ buf,
                                                    const uint64_t *__restrict__ off, uint64_t n,
                                                    const uint32_t *__restrict__ perm,
                                                    const uint8_t *__restrict__ override32,
                                                    const uint8_t *__restrict__ use_override,
                                                    uint8_t *__restrict__ out32, ShaCompare cmp) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool valid = g < n;
    const uint64_t gc = valid ? g : n - 1;
    const uint64_t i = perm ? (uint64_t)perm[gc] : gc;
    const bool ovr = use_override && use_override[i];
    const uint64_t o0 = off[i];
    // offsets that run backwards (a caller bug) hash as empty messages rather
    // than send the lane through a wrapped-around length
    const uint64_t L = off[i + 1] >= o0 ? off[i + 1] - o0 : 0;
    const uint32_t nb = (valid && !ovr) ? (uint32_t)((L + 72) >> 6) : 0u;
    const uint32_t nbmax = wave_max_u32(nb);
    MsgWalk mw;
    mw.init(buf + o0, L);
    State s;
    s.init();
#pragma unroll 1
    for (uint32_t b = 0; b < nbmax; b++) {
        const bool on = b < nb;
        uint32_t w[16];
        mw.block(b, nb, on, __ballot(on && b + 2 >= nb) == 0, w);
        if (on) compress(s, w);
    }
    if (!valid) return;
    if (cmp.expect) {
        uint32_t e[8];
        load_digest(cmp.expect + i * 32, e);
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) diff |= e[j] ^ s.h[j];
        const bool len_ok = !cmp.exp_len || cmp.exp_len[i] == L;
        cmp.status[i] = (diff == 0 && len_ok) ? MH_OK : MH_ERR_CORRUPTED_DATA;
        if (!out32) return;
    }
    if (ovr) {
        reinterpret_cast<uint4 *>(out32 + i * 32)[0] =
            reinterpret_cast<const uint4 *>(override32 + i * 32)[0];
        reinterpret_cast<uint4 *>(out32 + i * 32)[1] =
            reinterpret_cast<const uint4 *>(override32 + i * 32)[1];
    } else {
        store_digest(out32 + i * 32, s.h);
    }
}

// ============================================================================
// Fused ragged entry kernel: per entry (one lane, entries in length-class
// order) the value hash (immustore.go:1620-1630, or the IsValueTruncated
// override), then the entry digest TxEntryDigest_v1_2 / _v1_1 (tx.go:690-731)
// built straight from the key / metadata bytes and the hVal, then the htree
// leaf SHA256(0x00 || digest) (htree.go:79-83) -- one compression per loop
// iteration, the lane's phase given by the iteration index:
//   it in [0, nbv)          value block it
//   it in [nbv, nbv + nbd)  entry-digest block it - nbv
//   it == nbv + nbd         leaf
// The digest message  v1: BE16 ml | md | BE16 kl | key | hVal,  v0: key | hVal
// is never assembled: each of its words is the OR of the key and metadata
// windows (realigned by v_perm, masked to their byte ranges), the two BE16
// lengths and the hVal, which the lane parks in LDS between zero pads so its
// window needs no mask.
// ============================================================================
constexpr int kHvSlot = 10;  // 0 | hVal dwords (memory byte order) | 0

// bytes [S, E) of a memory segment seen through the 17-dword window d of a
// block: rs / re = S / E relative to the block start
__device__ __forceinline__ uint32_t seg_word(const uint32_t d[17], int j, uint32_t sel, int rs,
                                             int re) {
    const uint32_t x = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
    return x & hi_mask(re - 4 * j) & ~hi_mask(rs - 4 * j);
}

// ND-dword window of a segment at byte address a (may start before / run past
// the segment: loads are clamped to [lo, hi], the bytes masked later)
template <int ND = 17>
__device__ __forceinline__ void seg_window(const uint8_t *a, const uint32_t *lo, const uint32_t *hi,
                                           uint32_t d[17], uint32_t *sel) {
    const uint32_t al = (uint32_t)((uintptr_t)a & 3);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(a - al);
    *sel = 0x00010203u + al * 0x01010101u;
#pragma unroll
    for (int j = 0; j < ND; j++) {
        const uint32_t *x = q + j;
        d[j] = *(x < lo ? lo : (x > hi ? hi : x));
    }
}

// BE16 value x at message position rel (relative to the word start 4j)
__device__ __forceinline__ uint32_t be16_word(uint32_t x, int rel) {
    if (rel < -1 || rel > 3) return 0u;
    const uint64_t t = (uint64_t)((x & 0xffffu) << 16) << 8;
    return (uint32_t)(t >> (8 * rel + 8));
}

// OR the v1 digest-message prefix (BE16 ml | md | BE16 kl, message bytes
// [0, 4 + ml)) into 4 words x[0..3] that start at message byte p0.
__device__ __forceinline__ void prefix_words4(uint32_t x[4], const uint8_t *mp, uint64_t ml,
                                              uint64_t kl, int64_t p0) {
    const int r0 = clamp_rel(-p0), r_kl = clamp_rel(2 + (int64_t)ml - p0);
    if (ml) {
        const uint32_t *m_lo = reinterpret_cast<const uint32_t *>((uintptr_t)mp & ~(uintptr_t)3);
        const uint32_t *m_hi =
            reinterpret_cast<const uint32_t *>((uintptr_t)(mp + ml - 1) & ~(uintptr_t)3);
        uint32_t d[17], sel;
        seg_window<5>(mp + (p0 - 2), m_lo, m_hi, d, &sel);
#pragma unroll
        for (int j = 0; j < 4; j++) x[j] |= seg_word(d, j, sel, r0 + 2, r_kl);
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
        x[j] |= be16_word((uint32_t)ml, r0 - 4 * j) | be16_word((uint32_t)kl, r_kl - 4 * j);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_entries_varlen(
    int version, uint64_t n, const uint8_t *__restrict__ keys, const uint64_t *__restrict__ key_off,
    const uint8_t *__restrict__ md, const uint64_t *__restrict__ md_off,
    const uint8_t *__restrict__ vals, const uint64_t *__restrict__ val_off,
    const uint32_t *__restrict__ perm, const uint8_t *__restrict__ override32,
    const uint8_t *__restrict__ use_override, uint8_t *__restrict__ hvals_out,
    uint8_t *__restrict__ out32, int want_leaf, const uint8_t *__restrict__ ver_e) {
    __shared__ uint32_t hv_lds[256 * kHvSlot];
    uint32_t *slot = hv_lds + threadIdx.x * kHvSlot;
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool valid = g < n;
    const uint64_t gc = valid ? g : n - 1;
    const uint64_t i = perm ? (uint64_t)perm[gc] : gc;
    // override32 without use_override: every entry takes its hVal from the
    // caller (val_off may then be null)
    const bool ovr = override32 && (!use_override || use_override[i]);
    // digest version: the launch's, or per entry (documents of several txs)
    const int ver = ver_e ? (int)ver_e[i] : version;
    // offsets that run backwards (a caller bug) read as empty ranges rather
    // than send the lane through a wrapped-around length
    auto span = [](const uint64_t *o, uint64_t k) { return o[k + 1] >= o[k] ? o[k + 1] - o[k] : 0; };
    const uint64_t vo = ovr ? 0 : val_off[i];
    const uint64_t L = ovr ? 0 : span(val_off, i);
    const uint64_t ko = key_off[i];
    const uint64_t kl = span(key_off, i);
    const uint64_t mo = (ver == 1 && md_off) ? md_off[i] : 0;
    const uint64_t ml = (ver == 1 && md_off) ? span(md_off, i) : 0;
    // digest message layout (tx.go:703-731 v1, :690-701 v0)
    const int64_t s_key = ver == 1 ? (int64_t)(4 + ml) : 0;
    const int64_t s_hv = s_key + (int64_t)kl;
    const int64_t ld = s_hv + 32;
    const uint32_t nbv = ovr ? 0u : (uint32_t)((L + 72) >> 6);
    const uint32_t nbd = (uint32_t)((ld + 72) >> 6);
    const uint32_t tot = valid ? nbv + nbd + 1 : 0u;
    const uint32_t itmax = wave_max_u32(tot);

    MsgWalk mw;
    mw.init(vals + vo, L);
    const uint8_t *kp = keys + ko;
    const uint32_t *k_lo = reinterpret_cast<const uint32_t *>((uintptr_t)kp & ~(uintptr_t)3);
    const uint32_t *k_hi =
        reinterpret_cast<const uint32_t *>((uintptr_t)(kp + kl - 1) & ~(uintptr_t)3);
    const uint8_t *mp = md ? md + mo : nullptr;
    slot[0] = 0;
    slot[kHvSlot - 1] = 0;
    State s;
    s.init();
#pragma unroll 1
    for (uint32_t it = 0; it < itmax; it++) {
        const bool live = it < tot;
        if (live && it == nbv) {
            // value done (or overridden): hVal out, parked in LDS for the digest
            uint32_t hv[8];
            if (ovr) load_digest(override32 + i * 32, hv);
            else copy8(hv, s.h);
            if (hvals_out) store_digest(hvals_out + i * 32, hv);
#pragma unroll
            for (int j = 0; j < 8; j++) slot[1 + j] = bswap(hv[j]);
            s.init();
        }
        if (live && it == nbv + nbd) {
            // digest done: parked in the (no longer needed) hVal slot
#pragma unroll
            for (int j = 0; j < 8; j++) slot[1 + j] = s.h[j];
            s.init();
        }
        const bool ph_v = live && it < nbv;
        const bool ph_d = live && it >= nbv && it < nbv + nbd;
        const bool ph_l = live && it == nbv + nbd;
        uint32_t w[16];
        if (__ballot(ph_v)) {
            mw.block(it, nbv, ph_v, __ballot(ph_v && it + 2 >= nbv) == 0, w);
        }
        if (__ballot(ph_d)) {
            if (ph_d) {
                const uint32_t bd = it - nbv;
                const int64_t p0 = 64 * (int64_t)bd;
                const int r_key = clamp_rel(s_key - p0), r_hv = clamp_rel(s_hv - p0);
                uint32_t x[16];
#pragma unroll
                for (int j = 0; j < 16; j++) x[j] = 0;
                // key bytes [s_key, s_hv)
                if (kl && r_hv > 0 && r_key < 64) {
                    uint32_t d[17], sel;
                    seg_window(kp + (p0 - s_key), k_lo, k_hi, d, &sel);
#pragma unroll
                    for (int j = 0; j < 16; j++) x[j] |= seg_word(d, j, sel, r_key, r_hv);
                }
                // v1 prefix: BE16 ml | md | BE16 kl  at [0, s_key): in block 0
                // only, and within its first 4 words whenever every digest lane
                // of the wave has s_key <= 16 (KV metadata <= 11 bytes, always
                // for immudb's attributes)
                if (ver == 1 && p0 < s_key) {
                    prefix_words4(x, mp, ml, kl, p0);
                    if (__ballot(s_key > p0 + 16)) {  // metadata longer than 12 bytes
#pragma unroll
                        for (int c = 1; c < 4; c++) prefix_words4(x + 4 * c, mp, ml, kl, p0 + 16 * c);
                    }
                }
                // hVal bytes [s_hv, s_hv + 32): window over the zero-padded slot
                {
                    const int64_t oh = p0 - s_hv;  // hVal byte of the block's first byte
                    const int64_t k0 = oh >> 2;    // floor
                    const uint32_t sel = 0x00010203u + (uint32_t)(oh & 3) * 0x01010101u;
                    uint32_t hd[17];
#pragma unroll
                    for (int j = 0; j < 17; j++) {
                        const int64_t k = k0 + j;
                        hd[j] = slot[k < -1 ? 0 : (k > 8 ? kHvSlot - 1 : (int)k + 1)];
                    }
#pragma unroll
                    for (int j = 0; j < 16; j++) x[j] |= __builtin_amdgcn_perm(hd[j + 1], hd[j], sel);
                }
                const int r_end = clamp_rel(ld - p0);
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const int v = r_end - 4 * j;
                    if (v >= 0 && v < 4) x[j] |= 0x80u << (24 - 8 * v);
                }
                if (bd + 1 == nbd) {
                    x[14] = (uint32_t)((uint64_t)ld >> 29);
                    x[15] = (uint32_t)((uint64_t)ld << 3);
                }
#pragma unroll
                for (int j = 0; j < 16; j++) w[j] = x[j];
            }
        }
        if (__ballot(ph_l)) {
            if (ph_l) {
                // leaf = SHA256(0x00 || digest)  (htree.go:79-83)
                uint32_t dg[8];
#pragma unroll
                for (int j = 0; j < 8; j++) dg[j] = slot[1 + j];
                w[0] = dg[0] >> 8;
#pragma unroll
                for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(dg[j - 1], dg[j], 8);
                w[8] = (dg[7] << 24) | 0x00800000u;
#pragma unroll
                for (int j = 9; j < 15; j++) w[j] = 0;
                w[15] = 33u * 8u;
            }
        }
        const bool do_c = ph_v || ph_d || (ph_l && want_leaf);
        if (do_c) compress(s, w);
    }
    if (!valid) return;
    // digest (want_leaf == 0, still in the slot) or its leaf
    if (!want_leaf) {
#pragma unroll
        for (int j = 0; j < 8; j++) s.h[j] = slot[1 + j];
    }
    store_digest(out32 + i * 32, s.h);
}

size_t sha_varlen_scratch_bytes(uint64_t n) {
    return 2 * kNbBuckets * sizeof(uint32_t) + n * sizeof(uint32_t);
}

// Length-class order of n messages (perm in scratch), or null when the batch
// is too small to profit (unsorted: 438 vs 1170 GiB/s of ragged values,
// DESIGN.md history, round 2).
static const uint32_t *nb_sort(hipStream_t st, Timer *tm, const uint64_t *off, const uint8_t *use,
                               uint64_t n, uint8_t *scratch, hipError_t *err) {
    *err = hipSuccess;
    // below ~16K messages the four sort launches cost more than the divergence
    if (!scratch || n < 16384 || n >= 0xffffffffull) return nullptr;
    TimerScope ts(tm, "varlen_sort", st);
    uint32_t *hist = reinterpret_cast<uint32_t *>(scratch);
    uint32_t *cursor = hist + kNbBuckets;
    uint32_t *pm = cursor + kNbBuckets;
    const unsigned chunks = (unsigned)((n + kNbChunk - 1) / kNbChunk);
    *err = hipMemsetAsync(hist, 0, kNbBuckets * sizeof(uint32_t), st);
    if (*err != hipSuccess) return nullptr;
    hipLaunchKernelGGL(k_nb_hist, dim3(chunks), dim3(256), 0, st, off, use, n, hist);
    hipLaunchKernelGGL(k_nb_scan, dim3(1), dim3(kNbBuckets), 0, st, hist, cursor);
    hipLaunchKernelGGL(k_nb_scatter, dim3(chunks), dim3(256), 0, st, off, use, n, cursor, pm);
    *err = hipGetLastError();
    return pm;
}

hipError_t launch_sha256_csr(hipStream_t st, Timer *tm, const uint8_t *buf, const uint64_t *off,
                             uint64_t n, const uint8_t *override32, const uint8_t *use_override,
                             uint8_t *out32, uint8_t *scratch) {
    if (!n) return hipSuccess;
    hipError_t e;
    const uint32_t *perm = nb_sort(st, tm, off, use_override, n, scratch, &e);
    if (e != hipSuccess) return e;
    TimerScope ts(tm, "sha256_csr", st);
    hipLaunchKernelGGL(k_sha_varlen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, buf, off, n,
                       perm, override32, use_override, out32, ShaCompare());
    return hipGetLastError();
}

hipError_t launch_verify_values(hipStream_t st, Timer *tm, const uint8_t *buf, const uint64_t *off,
                                uint64_t n, const uint64_t *exp_len, const uint8_t *expect,
                                int32_t *status, uint8_t *scratch) {
    if (!n) return hipSuccess;
    hipError_t e;
    const uint32_t *perm = nb_sort(st, tm, off, nullptr, n, scratch, &e);
    if (e != hipSuccess) return e;
    TimerScope ts(tm, "verify_values", st);
    ShaCompare cmp;
    cmp.expect = expect;
    cmp.exp_len = exp_len;
    cmp.status = status;
    hipLaunchKernelGGL(k_sha_varlen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, buf, off, n,
                       perm, nullptr, nullptr, nullptr, cmp);
    return hipGetLastError();
}

hipError_t launch_entries_varlen(hipStream_t st, Timer *tm, int version, uint64_t n,
                                 const uint8_t *keys, const uint64_t *key_off, const uint8_t *md,
                                 const uint64_t *md_off, const uint8_t *vals,
                                 const uint64_t *val_off, const uint8_t *override32,
                                 const uint8_t *use_override, uint8_t *hvals_out, uint8_t *out32,
                                 bool leaf, uint8_t *scratch, const uint8_t *ver_e) {
    if (!n) return hipSuccess;
    hipError_t e = hipSuccess;
    // every hVal overridden: no value blocks, nothing to sort by
    const uint32_t *perm = (override32 && !use_override)
                               ? nullptr
                               : nb_sort(st, tm, val_off, use_override, n, scratch, &e);
    if (e != hipSuccess) return e;
    TimerScope ts(tm, "entries_varlen", st);
    hipLaunchKernelGGL(k_entries_varlen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       version, n, keys, key_off, md, md_off, vals, val_off, perm, override32,
                       use_override, hvals_out, out32, leaf ? 1 : 0, ver_e);
    return hipGetLastError();
}

}  // namespace mh
