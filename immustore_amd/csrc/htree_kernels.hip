// htree_kernels.hip -- CDNA4 kernels for embedded/htree and the entry hashing
// that feeds it (value hash, TxEntryDigest, leaf hash), plus the level
// reduction.  One SHA-256 message per lane; 32-bit VALU only (no MFMA).
//
// Reference behaviour followed:
//   value hash loop          embedded/store/immustore.go:1620-1630
//   TxEntryDigest_v1_1/_v1_2 embedded/store/tx.go:690-731
//   htree.BuildWith          embedded/htree/htree.go:68-113
//     leaf = SHA256(0x00||d), node = SHA256(0x01||l||r), odd last node promoted
#include <algorithm>
#include <cstring>

#include "mh_internal.hpp"
#include "sha256_cdna.hpp"
#include "digest_io.hpp"

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

namespace mh {

// ------------------------------------------------------------------ host geometry
void LevelGeom::init(uint64_t n_) {
    n = n_;
    nlevels = 0;
    total = 0;
    for (int l = 0; l < kMaxLevels; l++) off[l] = width[l] = 0;
    if (n == 0) return;
    uint64_t w = n;
    for (;;) {
        off[nlevels] = total;
        width[nlevels] = w;
        total += w;
        nlevels++;
        if (w == 1) break;
        w = (w + 1) / 2;
    }
}

static LevelArgs level_args(const LevelGeom &g) {
    LevelArgs a;
    for (int l = 0; l < kMaxLevels; l++) {
        a.off[l] = g.off[l];
        a.width[l] = l < g.nlevels ? g.width[l] : 0;
    }
    return a;
}

void pad_block_kw(uint64_t len, KWTable *out) {
    static const uint32_t K[64] = {
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
    auto ror = [](uint32_t x, int n) { return (x >> n) | (x << (32 - n)); };
    uint32_t w[64] = {0};
    uint64_t bits = len * 8;
    w[0] = 0x80000000u;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    for (int t = 16; t < 64; t++) {
        uint32_t s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    for (int t = 0; t < 64; t++) out->kw[t] = K[t] + w[t];
}

// Offsets / widths of levels 0..10: the levels a leaf workgroup writes (its
// lanes' groups up to level log2(LPL), then its subtree up to 8 more levels).
constexpr int kLaneLevels = 11;
struct LaneLevels {
    uint64_t off[kLaneLevels];
    uint64_t width[kLaneLevels];
};

static LaneLevels lane_levels(const LevelGeom &g) {
    LaneLevels a;
    for (int l = 0; l < kLaneLevels; l++) {
        a.off[l] = l < g.nlevels ? g.off[l] : 0;
        a.width[l] = l < g.nlevels ? g.width[l] : 0;
    }
    return a;
}

__device__ __forceinline__ void store_node(uint8_t *levels, const LaneLevels &la, int l, uint64_t q,
                                           const uint32_t w[8]) {
    if (q < la.width[l]) store_digest(levels + (la.off[l] + q) * 32, w);
}

// Entry digest block for fixed-shape entries without KV metadata
// (tx.go:703-731 v1: BE16 0 || BE16 klen || key || hVal; tx.go:690-701 v0:
// key || hVal).  KW4 = key_len / 4 words, one 64-byte block (<= 55 bytes).
template <int VER, int KW4>
__device__ __forceinline__ void digest_words(const uint32_t key[5], const uint32_t hv[8],
                                             uint32_t w[16]) {
    constexpr int P = VER == 1 ? 1 : 0;  // words before the key
    constexpr int L = (VER == 1 ? 4 : 0) + 4 * KW4 + 32;
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = 0;
    if (VER == 1) w[0] = 4 * KW4;
#pragma unroll
    for (int j = 0; j < KW4; j++) w[P + j] = key[j];
#pragma unroll
    for (int j = 0; j < 8; j++) w[P + KW4 + j] = hv[j];
    w[P + KW4 + 8] = 0x80000000u;
    w[15] = L * 8;
}

__device__ __forceinline__ void digest_block(int version, int kw4, const uint32_t key[5],
                                             const uint32_t hv[8], uint32_t w[16]) {
    if (version == 1) {
        switch (kw4) {
            case 0: digest_words<1, 0>(key, hv, w); break;
            case 1: digest_words<1, 1>(key, hv, w); break;
            case 2: digest_words<1, 2>(key, hv, w); break;
            case 3: digest_words<1, 3>(key, hv, w); break;
            default: digest_words<1, 4>(key, hv, w); break;
        }
    } else {
        switch (kw4) {
            case 0: digest_words<0, 0>(key, hv, w); break;
            case 1: digest_words<0, 1>(key, hv, w); break;
            case 2: digest_words<0, 2>(key, hv, w); break;
            case 3: digest_words<0, 3>(key, hv, w); break;
            case 4: digest_words<0, 4>(key, hv, w); break;
            default: digest_words<0, 5>(key, hv, w); break;
        }
    }
}

// In-lane tree over LPL consecutive leaves [first, first+LPL): the lane writes
// levels 1..log2(LPL) of its aligned group.  The group is aligned, so its
// valid count c decides hashing vs promotion exactly as htree.go:91-104.
template <int LPL>
struct LaneReducer {
    uint32_t A[8], B[8];
    // called with leaf i of the group (i < c); i is a runtime value so that
    // the caller's entry loop is not unrolled (one node_hash call site).
    __device__ __forceinline__ void push(int i, const uint32_t leaf[8]) {
        if (LPL == 1) return;
        if ((i & 1) == 0) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (i == 0) A[j] = leaf[j];
                else B[j] = leaf[j];
            }
        } else {
            uint32_t x[8];
#pragma unroll
            for (int j = 0; j < 8; j++) x[j] = i == 1 ? A[j] : B[j];
            node_hash(x, leaf, x);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (i == 1) A[j] = x[j];
                else B[j] = x[j];
            }
        }
    }
    __device__ __forceinline__ void finish(int c, uint64_t first, uint8_t *levels,
                                           const LaneLevels &la) {
        if (LPL == 1 || c <= 0) return;
        // level 1: node first/2 (A: hashed if c>=2, promoted leaf0 if c==1)
        store_node(levels, la, 1, first >> 1, A);
        if (LPL >= 4) {
            if (c >= 3) {
                store_node(levels, la, 1, (first >> 1) + 1, B);
                node_hash(A, B, A);
            }
            store_node(levels, la, 2, first >> 2, A);
        }
    }
};

template <int LPL>
struct Log2 {
    static constexpr int v = LPL == 1 ? 0 : LPL == 2 ? 1 : 2;
};

// ============================================================================
// Fused fixed-stride entry kernel (BASELINE C1/C2/C4 shape).
//
// Each wave stages its 64 lanes' values through 8 KB of LDS with LDS-DMA
// (global_load_lds_dwordx4): one DMA instruction moves 1 KiB = 8 entries x
// 128 B = 8 full cache lines, so HBM reads are coalesced although every lane
// hashes a different value.  The 16-byte chunk order is XOR-swizzled per
// entry so that the per-lane ds_read_b128 transposition is bank-conflict
// free.  The DMA of the next 2-block step is issued before the current
// step's second compression, so the load latency hides under VALU work.
// ============================================================================
constexpr int kFixedThreads = 256;
constexpr int kWaveLds = 8192;
constexpr uint32_t kFixedMaxValLen = 1u << 24;  // see entries_fixed_supported

// Workgroup timeline probe points of k_entries_fixed (0: start, 3: first value
// block hashed, 1: leaf phase done, 2: end); empty in the library, defined by
// tools/wg_trace.hip.
#ifndef MH_WG_PROBE
#define MH_WG_PROBE(point)
#endif

// Issue the LDS-DMA of one unit (2 blocks = 8 x 1 KiB, or 1 block = 4 x 1 KiB)
// for the wave's 64 lane-slots.  Address = wave-uniform base (SGPRs) + a
// 32-bit per-lane offset; slot entries past the end of the batch are clamped
// to the last entry (`lim`, wave-uniform) so no lane reads out of bounds.
// The empty asm makes the lane index opaque at the call site, so the
// compiler recomputes these few offsets per unit instead of hoisting all of
// them out of the block loop into dozens of live VGPRs.
__device__ __forceinline__ void dma_issue(const uint8_t *__restrict__ vals, uint32_t stride,
                                          uint64_t wave_slot0, int lpl, int i, uint64_t n,
                                          uint32_t byte_off, bool two, char *lds, int lane) {
    uint32_t ln = (uint32_t)lane;
    asm volatile("" : "+v"(ln));
    const uint64_t e0 = wave_slot0 * lpl;                 // first entry of the wave
    const uint32_t lim = (uint32_t)min<uint64_t>(n - 1 - e0, 0xffffffffull);  // last valid rel.
    const uint8_t *g0 = vals + e0 * stride + byte_off;  // uniform
    if (two) {
        const uint32_t k2 = (ln & 7) ^ (ln >> 4);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t rel = min((uint32_t)((j * 8 + (ln >> 3)) * lpl + i), lim);
            const uint32_t off = rel * stride + ((j & 1) ? (k2 ^ 4) : k2) * 16;
            __builtin_amdgcn_global_load_lds((glb_void_t *)(g0 + off),
                                             (lds_void_t *)(lds + j * 1024), 16, 0, 0);
        }
    } else {
        const uint32_t k1 = (ln & 3) ^ ((ln >> 4) & 3);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t rel = min((uint32_t)((j * 16 + (ln >> 2)) * lpl + i), lim);
            const uint32_t off = rel * stride + k1 * 16;
            __builtin_amdgcn_global_load_lds((glb_void_t *)(g0 + off),
                                             (lds_void_t *)(lds + j * 1024), 16, 0, 0);
        }
    }
}

// read block h (0/1) of a 2-block step (layout "two") or the single block
__device__ __forceinline__ void lds_block(const char *lds, int lane, bool two, int h,
                                          uint32_t w[16]) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
        int addr;
        if (two) {
            const int k = 4 * h + c;
            addr = lane * 128 + ((k ^ ((lane >> 1) & 7)) << 4);
        } else {
            addr = lane * 64 + ((c ^ ((lane >> 2) & 3)) << 4);
        }
        const uint4 v = *reinterpret_cast<const uint4 *>(lds + addr);
        w[4 * c + 0] = bswap(v.x);
        w[4 * c + 1] = bswap(v.y);
        w[4 * c + 2] = bswap(v.z);
        w[4 * c + 3] = bswap(v.w);
    }
}

// Per-lane work is a uniform sequence of SHA-256 compressions driven by a
// small state machine with ONE generic compress() call site (plus one
// compress_kw for the constant padding block): value blocks -> padding ->
// entry digest -> leaf -> the in-lane node hashes of the LPL-leaf group.
// A single call site keeps the code ~8 KB of hot instructions and keeps the
// 64 round constants of only one inlined compression live in SGPRs.
enum : int { OP_VALUE = 0, OP_TAIL, OP_DIGEST, OP_LEAF, OP_NODE1, OP_NODE2 };

template <int LPL>
__global__ __launch_bounds__(kFixedThreads) void k_entries_fixed(
    const uint8_t *__restrict__ vals, uint32_t val_len, const uint8_t *__restrict__ keys,
    uint32_t key_len, int version, uint64_t n, uint8_t *__restrict__ hvals_out,
    uint8_t *__restrict__ levels, LaneLevels la, int wg_levels) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // K+W of the constant padding block (value length % 64 == 0), shared by
    // all waves; read back as wave-uniform LDS broadcasts.
    uint32_t *kw_lds = reinterpret_cast<uint32_t *>(smem + (kFixedThreads / 64) * kWaveLds);
    if (threadIdx.x == 0) {
        // constant schedule of the padding block: 0x80, zeros, 64-bit bit length
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = 0;
        w[0] = 0x80000000u;
        const uint64_t bits = (uint64_t)val_len * 8;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
#pragma unroll
        for (int t = 0; t < 64; t++) {
            if (t >= 16)
                w[t & 15] = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) +
                            w[t & 15];
            kw_lds[t] = kK256[t] + w[t & 15];
        }
    }
    __syncthreads();
    MH_WG_PROBE(0);
    char *lds = smem + wave * kWaveLds;
    const uint64_t wave_slot0 = ((uint64_t)blockIdx.x * (kFixedThreads / 64) + wave) * 64;
    const uint64_t first = (wave_slot0 + lane) * LPL;
    const int c = first < n ? (int)min<uint64_t>(LPL, n - first) : 0;
    const bool wave_busy = wave_slot0 * LPL < n;  // wave-uniform

    const uint32_t nfull = val_len >> 6;
    const uint32_t rem = val_len & 63;  // 0, 16, 32 or 48 (fast-path precondition)
    const uint32_t nsteps2 = nfull >> 1;
    const uint32_t units = nsteps2 + (nfull & 1);
    const int kw4 = key_len >> 2;
    State s;
    s.init();
    uint32_t A[8], B[8], ny7 = 0;
    if (wave_busy) {
    if (units) dma_issue(vals, val_len, wave_slot0, LPL, 0, n, 0, nsteps2 > 0, lds, lane);

    int i = 0;         // entry of the lane group (uniform)
    uint32_t b = 0;    // value block (uniform)
    int node = 0;      // node step of the group after leaf i (uniform)
    int op = nfull ? OP_VALUE : (rem ? OP_TAIL : OP_DIGEST);
    if (!nfull && !rem && i < c) compress_kw(s, kw_lds);
    for (;;) {
        const uint64_t idx = first + i;
        bool on = i < c;
        if (op == OP_VALUE) {
            // tight loop over the value's full blocks: its own compress site,
            // no state-machine dispatch per block
#pragma unroll 1
            for (; b < nfull; b++) {
                const uint32_t u = b >> 1;
                const bool two = u < nsteps2;
                const int h = two ? (int)(b & 1) : 0;
                uint32_t w[16];
                lds_block(lds, lane, two, h, w);
                if (!two || h == 1) {
                    // this unit is fully in registers: start the next DMA
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (u + 1 < units)
                        dma_issue(vals, val_len, wave_slot0, LPL, i, n, (u + 1) * 128,
                                  (u + 1) < nsteps2, lds, lane);
                    else if (i + 1 < LPL)
                        dma_issue(vals, val_len, wave_slot0, LPL, i + 1, n, 0, nsteps2 > 0, lds,
                                  lane);
                }
                if (on) compress(s, w);
                if (b == 0 && i == 0) MH_WG_PROBE(3);
            }
            b = 0;
            if (rem) {
                op = OP_TAIL;
            } else {
                if (on) compress_kw(s, kw_lds);
                op = OP_DIGEST;
            }
            continue;
        }
        uint32_t w[16];
        if (op == OP_TAIL) {
            // rem data bytes (16/32/48, dword aligned) + 0x80 + 64-bit length
            const uint32_t rw = rem >> 2;
            const uint32_t *tp =
                reinterpret_cast<const uint32_t *>(vals + idx * val_len + (uint64_t)nfull * 64);
#pragma unroll
            for (int j = 0; j < 12; j++) w[j] = (on && j < (int)rw) ? bswap(tp[j]) : 0u;
#pragma unroll
            for (int j = 12; j < 16; j++) w[j] = 0;
#pragma unroll
            for (int j = 0; j < 13; j++)
                if (j == (int)rw) w[j] = 0x80000000u;
            const uint64_t bits = (uint64_t)val_len * 8;
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        } else if (op == OP_DIGEST) {
            // s holds hVal (immustore.go:1629); TxEntryDigest (tx.go:690-731)
            if (on && hvals_out) store_digest(hvals_out + idx * 32, s.h);
            uint32_t key[5] = {0, 0, 0, 0, 0};
            const uint32_t *kp = reinterpret_cast<const uint32_t *>(keys + idx * key_len);
#pragma unroll
            for (int j = 0; j < 5; j++)
                if (on && j < kw4) key[j] = bswap(kp[j]);
            digest_block(version, kw4, key, s.h, w);
            s.init();
        } else if (op == OP_LEAF) {
            // leaf = SHA256(0x00 || digest)  (htree.go:79-83)
            w[0] = s.h[0] >> 8;
#pragma unroll
            for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(s.h[j - 1], s.h[j], 8);
            w[8] = (s.h[7] << 24) | 0x00800000u;
#pragma unroll
            for (int j = 9; j < 15; j++) w[j] = 0;
            w[15] = 33u * 8u;
            s.init();
        } else if (op == OP_NODE1) {
            // node = SHA256(0x01 || l || r), first block (htree.go:89-97)
            uint32_t l[8], r[8];
            if (LPL >= 2 && node == 0) {
                // (pending left, new right): A|B with the leaf just made
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    l[j] = i == 1 ? A[j] : B[j];
                    r[j] = s.h[j];
                }
                on = i < c;
            } else {
                copy8(l, A);  // (A, B) at the top of a 4-leaf group
                copy8(r, B);
                on = c >= 3;
            }
            w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
            for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(l[j - 1], l[j], 8);
            w[8] = __builtin_amdgcn_alignbit(l[7], r[0], 8);
#pragma unroll
            for (int j = 1; j < 8; j++) w[8 + j] = __builtin_amdgcn_alignbit(r[j - 1], r[j], 8);
            ny7 = r[7];
            s.init();
        } else {  // OP_NODE2: second block, only r[7]'s last byte is data
            w[0] = (ny7 << 24) | 0x00800000u;
#pragma unroll
            for (int j = 1; j < 15; j++) w[j] = 0;
            w[15] = 65u * 8u;
            on = (node == 0) ? (i < c) : (c >= 3);
        }

        if (on) compress(s, w);

        // ---------------------------------------------------------- transition
        bool entry_done = false;
        if (op == OP_TAIL) {
            op = OP_DIGEST;
        } else if (op == OP_DIGEST) {
            op = OP_LEAF;
        } else if (op == OP_LEAF) {
            if (i < c) store_digest(levels + idx * 32, s.h);  // level 0 offset is 0
            if (LPL == 1) break;
            entry_done = true;
            if ((i & 1) == 0) {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    if (i == 0) A[j] = s.h[j];
                    else B[j] = s.h[j];
                }
            } else {
                node = 0;
                op = OP_NODE1;
                continue;
            }
        } else if (op == OP_NODE1) {
            op = OP_NODE2;
            continue;
        } else {  // OP_NODE2 done: node result in s (or unchanged if lane off)
            const bool lane_on = (node == 0) ? (i < c) : (c >= 3);
            if (node == 0) {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    if (lane_on) {
                        if (i == 1) A[j] = s.h[j];
                        else B[j] = s.h[j];
                    }
                }
                // level-1 node of this pair (hashed, or the promoted left leaf)
                if (c > 0) store_node(levels, la, 1, (first >> 1) + (i >> 1), i == 1 ? A : B);
                if (LPL == 4 && i == 3) {
                    node = 1;
                    op = OP_NODE1;
                    continue;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (lane_on) A[j] = s.h[j];
            }
            if (LPL == 4 && i == 3 && c > 0) store_node(levels, la, 2, first >> 2, A);
            if (LPL == 2 || i == LPL - 1) break;
            entry_done = true;
        }
        if (entry_done) {
            // next entry of the group
            if (++i >= LPL) break;
            s.init();
            op = nfull ? OP_VALUE : (rem ? OP_TAIL : OP_DIGEST);
            if (!nfull && !rem && i < c) compress_kw(s, kw_lds);
        }
    }
    }  // wave_busy

    // -------------------------------------------------------- workgroup subtree
    // The workgroup's 256 lane-group nodes (level L0 = log2 LPL) are reduced
    // in LDS to up to 8 more levels (htree.go:85-110), writing every level.
    constexpr int L0 = LPL == 4 ? 2 : (LPL == 2 ? 1 : 0);
    MH_WG_PROBE(1);
    if (wg_levels == 0) return;  // launch-uniform
    const int t = threadIdx.x;
    uint32_t(*buf)[kFixedThreads][9] = reinterpret_cast<uint32_t(*)[kFixedThreads][9]>(smem);
    __syncthreads();  // every wave is done with its staging area
#pragma unroll
    for (int j = 0; j < 8; j++) buf[0][t][j] = LPL == 1 ? s.h[j] : A[j];
    int cur = 0;
#pragma unroll 1
    for (int st = 1; st <= wg_levels; st++) {
        __syncthreads();
        const int active = kFixedThreads >> st;
        const int l = L0 + st;
        if (t < active) {
            const uint64_t q = (uint64_t)blockIdx.x * active + t;
            if (q < la.width[l]) {
                uint32_t lft[8], rgt[8], out[8];
#pragma unroll
                for (int j = 0; j < 8; j++) lft[j] = buf[cur][2 * t][j];
                if (2 * q + 1 < la.width[l - 1]) {
#pragma unroll
                    for (int j = 0; j < 8; j++) rgt[j] = buf[cur][2 * t + 1][j];
                    node_hash(lft, rgt, out);
                } else {
                    copy8(out, lft);
                }
                store_digest(levels + (la.off[l] + q) * 32, out);
#pragma unroll
                for (int j = 0; j < 8; j++) buf[cur ^ 1][t][j] = out[j];
            }
        }
        cur ^= 1;
    }
    MH_WG_PROBE(2);
}

// ============================================================================
// Leaves from digests (htree.BuildWith over caller digests).
// ============================================================================
template <int LPL>
__global__ __launch_bounds__(256) void k_leaves_from_digests(const uint8_t *__restrict__ digests,
                                                             uint64_t n, uint8_t *__restrict__ levels,
                                                             LaneLevels la) {
    const uint64_t lane_id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t first = lane_id * LPL;
    if (first >= n) return;
    const int c = (int)min<uint64_t>(LPL, n - first);
    LaneReducer<LPL> red;
#pragma unroll 1  // one node_hash call site (LaneReducer::push)
    for (int i = 0; i < LPL; i++) {
        if (i < c) {
            uint32_t d[8], leaf[8];
            load_digest(digests + (first + i) * 32, d);
            leaf_hash(d, leaf);
            store_digest(levels + (first + i) * 32, leaf);
            red.push(i, leaf);
        }
    }
    red.finish(c, first, levels, la);
}

// copy nodes to level 0 (reduce_nodes: all-gathered subtree roots)
__global__ void k_copy_nodes(const uint8_t *__restrict__ src, uint64_t n, uint8_t *__restrict__ dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n * 2) reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
}

// ============================================================================
// Level reduction: a 256-thread workgroup turns 512 nodes of level l0 into
// levels l0+1 .. l0+nsteps (<= 9) of its aligned subtree, keeping the
// intermediate levels in LDS and writing every level to HBM (levels are
// needed for InclusionProof, htree.go:158).
// ============================================================================
template <int T>
__global__ __launch_bounds__(T) void k_reduce(uint8_t *__restrict__ levels, LevelArgs la, int l0,
                                              int nsteps, int top, uint8_t *__restrict__ root) {
    __shared__ uint32_t buf[2][T][9];  // +1 word pad: conflict-free 2t / 2t+1 reads
    const int t = threadIdx.x;
    const uint64_t blk = blockIdx.x;
    {
        const uint64_t q = blk * T + t;
        if (q < la.width[l0 + 1]) {
            uint32_t lft[8], rgt[8], out[8];
            load_digest(levels + (la.off[l0] + 2 * q) * 32, lft);
            if (2 * q + 1 < la.width[l0]) {
                load_digest(levels + (la.off[l0] + 2 * q + 1) * 32, rgt);
                node_hash_g(lft, rgt, out);
            } else {
                copy8(out, lft);
            }
            store_digest(levels + (la.off[l0 + 1] + q) * 32, out);
            if (l0 + 1 == top) store_digest(root, out);
#pragma unroll
            for (int j = 0; j < 8; j++) buf[0][t][j] = out[j];
        }
    }
    int cur = 0;
    for (int s = 2; s <= nsteps; s++) {
        __syncthreads();
        const int active = T >> (s - 1);
        const int l = l0 + s;
        if (t < active) {
            const uint64_t q = blk * active + t;
            if (q < la.width[l]) {
                uint32_t lft[8], rgt[8], out[8];
#pragma unroll
                for (int j = 0; j < 8; j++) lft[j] = buf[cur][2 * t][j];
                if (2 * q + 1 < la.width[l - 1]) {
#pragma unroll
                    for (int j = 0; j < 8; j++) rgt[j] = buf[cur][2 * t + 1][j];
                    node_hash_g(lft, rgt, out);
                } else {
                    copy8(out, lft);
                }
                store_digest(levels + (la.off[l] + q) * 32, out);
                if (l == top) store_digest(root, out);
#pragma unroll
                for (int j = 0; j < 8; j++) buf[cur ^ 1][t][j] = out[j];
            }
        }
        cur ^= 1;
    }
}

// Level reduction with two in-lane levels first: a T-thread workgroup turns
// 4T nodes of level l0 into levels l0+1, l0+2 (each lane hashes its own 4
// nodes -> 2 -> 1, every lane busy: three quarters of all the node hashes)
// and then up to nsteps-2 (<= 8) more levels of its aligned subtree in LDS.
// Every level is written (htree.go:158 needs them for InclusionProof).
template <int T>
__global__ __launch_bounds__(T) void k_reduce4(uint8_t *__restrict__ levels, LevelArgs la, int l0,
                                               int nsteps, int top, uint8_t *__restrict__ root) {
    __shared__ uint32_t buf[2][T][9];
    const int t = threadIdx.x;
    const uint64_t q = (uint64_t)blockIdx.x * T + t;  // node of level l0 + 2
    uint32_t A[8], B[8];
    if (q < la.width[l0 + 2]) {
        // k = 0, 1: level l0+1 nodes 2q, 2q+1; k = 2: level l0+2 node q
#pragma unroll 1
        for (int k = 0; k < 3; k++) {
            const int l = k < 2 ? l0 + 1 : l0 + 2;
            const uint64_t p = k < 2 ? 2 * q + k : q;
            if (p >= la.width[l]) break;  // k == 1 only: promoted below
            uint32_t lft[8], rgt[8], out[8];
            if (k < 2) load_digest(levels + (la.off[l0] + 2 * p) * 32, lft);
            else copy8(lft, A);
            const bool pair = 2 * p + 1 < la.width[l - 1];
            if (pair) {
                if (k < 2) load_digest(levels + (la.off[l0] + 2 * p + 1) * 32, rgt);
                else copy8(rgt, B);
                node_hash_g(lft, rgt, out);
            } else {
                copy8(out, lft);
            }
            store_digest(levels + (la.off[l] + p) * 32, out);
            if (l == top) store_digest(root, out);
            if (k == 0) copy8(A, out);
            else if (k == 1) copy8(B, out);
            else copy8(A, out);
        }
        // width[l0+1] odd and 2q+1 past it: node q of level l0+2 is the promoted 2q
        if (2 * q + 1 >= la.width[l0 + 1]) {
            store_digest(levels + (la.off[l0 + 2] + q) * 32, A);
            if (l0 + 2 == top) store_digest(root, A);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) buf[0][t][j] = A[j];
    }
    int cur = 0;
    for (int s = 3; s <= nsteps; s++) {
        __syncthreads();
        const int active = T >> (s - 2);
        const int l = l0 + s;
        if (t < active) {
            const uint64_t qq = (uint64_t)blockIdx.x * active + t;
            if (qq < la.width[l]) {
                uint32_t lft[8], rgt[8], out[8];
#pragma unroll
                for (int j = 0; j < 8; j++) lft[j] = buf[cur][2 * t][j];
                if (2 * qq + 1 < la.width[l - 1]) {
#pragma unroll
                    for (int j = 0; j < 8; j++) rgt[j] = buf[cur][2 * t + 1][j];
                    node_hash_g(lft, rgt, out);
                } else {
                    copy8(out, lft);
                }
                store_digest(levels + (la.off[l] + qq) * 32, out);
                if (l == top) store_digest(root, out);
#pragma unroll
                for (int j = 0; j < 8; j++) buf[cur ^ 1][t][j] = out[j];
            }
        }
        cur ^= 1;
    }
}

// ------------------------------------------------------------------ small helpers
__global__ void k_fill_random(uint8_t *__restrict__ dst, uint64_t nbytes, uint64_t seed) {
    const uint64_t nw = nbytes >> 3;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w <= nw;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        if (w < nw) {
            reinterpret_cast<uint64_t *>(dst)[w] = z;
        } else {
            for (uint64_t b = nw * 8; b < nbytes; b++) dst[b] = (uint8_t)(z >> (8 * (b - nw * 8)));
        }
    }
}

__global__ void k_fill_keys_be64(uint8_t *__restrict__ dst, uint64_t n, uint64_t first) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint64_t v = first + i;
        const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
        reinterpret_cast<uint2 *>(dst)[i] = make_uint2(bswap(hi), bswap(lo));
    }
}

__global__ void k_iota_offsets(uint64_t *__restrict__ off, uint64_t n, uint64_t stride) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) off[i] = i * stride;
}

__global__ void k_gather_nodes(const uint8_t *__restrict__ src, const uint64_t *__restrict__ idx,
                               uint64_t n, uint8_t *__restrict__ dst) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 2) return;
    const uint64_t k = t >> 1;
    reinterpret_cast<uint4 *>(dst)[t] = reinterpret_cast<const uint4 *>(src + idx[k] * 32)[t & 1];
}

// ------------------------------------------------------------------ launchers
static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}


static int choose_lpl(uint64_t n) {
    if (const char *e = getenv("MH_LPL")) {
        int v = atoi(e);
        if (v == 1 || v == 2 || v == 4) return v;
    }
    // Two entries per lane (one in-lane node level) from 2^19 entries up.  At
    // 2^20 that is 2048 workgroups of 256 lanes; each takes 33 KB of LDS and
    // the kernel 104 VGPRs, so 4 workgroups (4 waves per SIMD) are resident
    // per CU and the grid runs as two rounds of 1024, against one round of
    // 1024 with four entries per lane.  The halved work per workgroup halves
    // the straggler tail of the last round and the in-LDS subtree phase
    // (profiles/ab_lpl_wgl_r02.txt: leaf launch 0.835 -> 0.79 ms, single
    // build 0.96-0.97 -> 0.93-0.94 ms, three builds in flight within 0.2 %;
    // residency in profiles/wg_residency_r03.txt).  MH_LPL=4 restores the
    // round-1 shape.
    if (n >= (uint64_t)2 * 262144) return 2;
    return 1;
}

// Leaves from caller digests (one compression per leaf, no value blocks):
// two per lane from 2^19 up, as for entries -- an A/B of the whole
// mh_dev_htree_build_digests (profiles/ab_digest_lpl_r03.txt) gives 1.96 ms
// (LPL 2) / 1.97 (4) / 2.04 (1) at 2^24 digests and 0.250-0.255 ms for all
// three at 2^20 (the in-lane levels only move node hashes between the leaf
// launch and the reduce).  MH_DIGEST_LPL overrides.
static int choose_digest_lpl(uint64_t n) {
    if (const char *e = getenv("MH_DIGEST_LPL")) {
        int v = atoi(e);
        if (v == 1 || v == 2 || v == 4) return v;
    }
    return n >= (uint64_t)2 * 262144 ? 2 : 1;
}

bool entries_fixed_supported(int version, const uint8_t *keys, uint32_t key_len,
                             const uint8_t *vals, uint32_t val_len) {
    if (version != 0 && version != 1) return false;
    if (((uintptr_t)vals & 15) || (val_len & 15)) return false;
    if (((uintptr_t)keys & 3) || (key_len & 3)) return false;
    if (version == 1 && key_len > 16) return false;
    if (version == 0 && key_len > 20) return false;
    // dma_issue forms each lane's offset from the wave's first entry in 32
    // bits: rel * val_len + 112 with rel <= 64 * LPL - 1 <= 255, so values up
    // to 16 MiB (255 * 2^24 + 112 < 2^32).  Go accepts any MaxValueLen
    // (options.go:364-365): longer values take the CSR path (64-bit offsets).
    if (val_len > kFixedMaxValLen) return false;
    return true;
}

hipError_t launch_entries_fixed(hipStream_t st, Timer *tm, int version, uint64_t n,
                                const uint8_t *keys, uint32_t key_len, const uint8_t *vals,
                                uint32_t val_len, uint8_t *hvals_out, uint8_t *levels,
                                const LevelGeom &g, int *levels_done) {
    LaneLevels la = lane_levels(g);
    const int lpl = choose_lpl(n);
    const uint64_t lanes = (n + lpl - 1) / lpl;
    const unsigned grid = grid_for(lanes, kFixedThreads);
    const size_t lds = (kFixedThreads / 64) * kWaveLds + 256;
    // levels each leaf workgroup reduces in LDS after its lanes (0..8); 0
    // leaves the whole upper tree to k_reduce, which a concurrent build on
    // another stream can overlap (MH_WG_LEVELS overrides).  With two entries
    // per lane the default is 1 (profiles/ab_lpl_wgl_r02.txt: LPL 2 / 1 level
    // against LPL 4 / 2 levels); deeper in-kernel subtrees idle most lanes at
    // the end of the leaf kernel.
    int wgl = 1;
    if (const char *e = getenv("MH_WG_LEVELS")) wgl = std::max(0, std::min(8, atoi(e)));
    {
        TimerScope ts(tm, "entries_fixed", st);
        if (lpl == 4)
            hipLaunchKernelGGL(k_entries_fixed<4>, dim3(grid), dim3(kFixedThreads), lds, st, vals,
                               val_len, keys, key_len, version, n, hvals_out, levels, la, wgl);
        else if (lpl == 2)
            hipLaunchKernelGGL(k_entries_fixed<2>, dim3(grid), dim3(kFixedThreads), lds, st, vals,
                               val_len, keys, key_len, version, n, hvals_out, levels, la, wgl);
        else
            hipLaunchKernelGGL(k_entries_fixed<1>, dim3(grid), dim3(kFixedThreads), lds, st, vals,
                               val_len, keys, key_len, version, n, hvals_out, levels, la, wgl);
    }
    *levels_done = std::min((lpl == 4 ? 2 : lpl == 2 ? 1 : 0) + wgl, g.nlevels - 1);
    return hipGetLastError();
}

hipError_t launch_leaves_from_digests(hipStream_t st, Timer *tm, const uint8_t *digests,
                                      uint64_t n, uint8_t *levels, const LevelGeom &g,
                                      int *levels_done) {
    LaneLevels la = lane_levels(g);
    const int lpl = choose_digest_lpl(n);
    const uint64_t lanes = (n + lpl - 1) / lpl;
    {
        TimerScope ts(tm, "leaves", st);
        if (lpl == 4)
            hipLaunchKernelGGL(k_leaves_from_digests<4>, dim3(grid_for(lanes, 256)), dim3(256), 0,
                               st, digests, n, levels, la);
        else if (lpl == 2)
            hipLaunchKernelGGL(k_leaves_from_digests<2>, dim3(grid_for(lanes, 256)), dim3(256), 0,
                               st, digests, n, levels, la);
        else
            hipLaunchKernelGGL(k_leaves_from_digests<1>, dim3(grid_for(lanes, 256)), dim3(256), 0,
                               st, digests, n, levels, la);
    }
    *levels_done = std::min(lpl == 4 ? 2 : lpl == 2 ? 1 : 0, g.nlevels - 1);
    return hipGetLastError();
}

hipError_t launch_reduce(hipStream_t st, Timer *tm, uint8_t *levels, const LevelGeom &g,
                         int from_level, uint8_t *root) {
    // Each launch: a workgroup of T threads turns 2T nodes into log2(2T)
    // levels.  The last (top) launch uses 512 threads = 10 levels, so a
    // 2^20-leaf tree whose leaf kernel stopped at level 10 needs one launch.
    LevelArgs la = level_args(g);
    // the launch that produces the top level also stores the root (saves the
    // 32-byte copy launch after it); -1 = no root pointer
    const int top = root ? g.nlevels - 1 : -1;
    int cur = from_level;
    while (cur < g.nlevels - 1) {
        const int left = g.nlevels - 1 - cur;
        TimerScope ts(tm, "reduce", st);
        if (left <= 10 && g.width[cur] <= 1024) {
            hipLaunchKernelGGL(k_reduce<512>, dim3(1), dim3(512), 0, st, levels, la, cur, left, top, root);
            cur += left;
        } else if (left >= 3 && g.width[cur] >= (uint64_t)4 * 256 * 256) {
            // throughput regime (>= 256 workgroups): two in-lane levels + up
            // to 8 in LDS per launch.  Narrower levels are latency-bound, where
            // one node per lane (k_reduce) is one node-hash latency per level
            // instead of three for the in-lane pair.
            const int steps = std::min(10, left);
            const unsigned grid = grid_for(g.width[cur + 2], 256);
            hipLaunchKernelGGL(k_reduce4<256>, dim3(grid), dim3(256), 0, st, levels, la, cur, steps, top, root);
            cur += steps;
        } else {
            const int steps = std::min(9, left);
            const unsigned grid = grid_for(g.width[cur + 1], 256);
            hipLaunchKernelGGL(k_reduce<256>, dim3(grid), dim3(256), 0, st, levels, la, cur, steps, top, root);
            cur += steps;
        }
    }
    return hipGetLastError();
}

hipError_t launch_fill_random(hipStream_t st, uint8_t *dst, uint64_t nbytes, uint64_t seed) {
    const uint64_t nw = nbytes / 8 + 1;
    const unsigned grid = (unsigned)std::min<uint64_t>(grid_for(nw, 256), 65536);
    hipLaunchKernelGGL(k_fill_random, dim3(grid), dim3(256), 0, st, dst, nbytes, seed);
    return hipGetLastError();
}

hipError_t launch_fill_keys_be64(hipStream_t st, uint8_t *dst, uint64_t n, uint64_t first) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_fill_keys_be64, dim3(grid_for(n, 256)), dim3(256), 0, st, dst, n, first);
    return hipGetLastError();
}

hipError_t launch_iota_offsets(hipStream_t st, uint64_t *off, uint64_t n, uint64_t stride) {
    hipLaunchKernelGGL(k_iota_offsets, dim3(grid_for(n + 1, 256)), dim3(256), 0, st, off, n, stride);
    return hipGetLastError();
}

hipError_t launch_gather_nodes(hipStream_t st, const uint8_t *src, const uint64_t *idx, uint64_t n,
                               uint8_t *dst) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather_nodes, dim3(grid_for(2 * n, 256)), dim3(256), 0, st, src, idx, n,
                       dst);
    return hipGetLastError();
}

hipError_t launch_copy_nodes(hipStream_t st, const uint8_t *src, uint64_t n, uint8_t *dst) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_copy_nodes, dim3(grid_for(2 * n, 256)), dim3(256), 0, st, src, n, dst);
    return hipGetLastError();
}

}  // namespace mh
