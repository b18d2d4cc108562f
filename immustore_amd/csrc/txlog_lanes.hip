// txlog_lanes.hip -- a14 (tx.go:533-630 per record) with every record on
// L = 1, 2, 4, 8 or 16 lanes (k_txlog_lanes<LGL>): the kernel of the bulk
// copy chunks of mh_txlog_validate (>= 16384 records), of a resident log
// (mh_txlog_validate_resident) and of a log indexed by its commit log
// (mh_txlog_validate_clog).
//
// Lane i of a record takes its entries [i EP, (i+1) EP) (EP = P / L, P = the
// widest tx rounded up to a power of two) and builds their subtree itself --
// entry digest (tx.go:690-731) and leaf (htree.go:79-83) per entry, pushed on
// a per-lane stack in LDS; after the c-th leaf, tz(c) merges
// SHA256(0x01 || left || right), and at the end the stack folded from the
// right, which is htree's pairing with the odd last node promoted
// (htree.go:85-110): an aligned block of 2^k leaves of a tree is the htree of
// its leaves (SURVEY.md finding 3).  The L lane roots of a record are then
// paired log2 L more levels, and the record's first lane hashes innerHash
// (tx.go:249-302) and Alh (tx.go:307-319) and compares.  No staging, no
// workgroup barrier before the final stores: a lane is busy on its own record
// for all but the log2 L combine levels and the four innerHash + Alh
// compressions, so with L = 1 every lane of a wave works in every compression
// slot (uniform records).  The price is latency: a record is ~66 dependent
// compressions on L = 1 lane, so the launch picks L from the record count
// (few records: more lanes).
//
// The record structure comes either from the host hop (leaf_off: entry
// counts) or from the device pre-pass of txlog_struct.hip (leaf_off null:
// the entry count is the header's, validated by the pre-pass); records the
// pre-pass rejected (pre[t] != 0) are not walked: status pre[t], Alh, Eh and
// header 0.
//
// `make LANES_CHECK=1` builds the checking form (-DMH_TXLOG_LANES_CHECK):
// every read of the log range-checked against [buf, buf + len + 256), a read
// outside reported and the call failed.  The default library has no checks.
#include <algorithm>
#include <cstdio>

#include "txlog_common.hpp"

#ifndef MH_TXLOG_LANES_CHECK
#define MH_TXLOG_LANES_CHECK 0
#endif

namespace mh {

constexpr int kTxlStackPad = 9;  // words per stack slot (8 + 1: bank spread)
constexpr bool kTxlCheck = MH_TXLOG_LANES_CHECK != 0;

__device__ __forceinline__ void txl_node_first(const uint32_t l[8], const uint32_t r[8], uint32_t w[16]) {
    w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[j] = __builtin_amdgcn_alignbit(l[j - 1], l[j], 8);
    w[8] = __builtin_amdgcn_alignbit(l[7], r[0], 8);
#pragma unroll
    for (int j = 1; j < 8; j++) w[8 + j] = __builtin_amdgcn_alignbit(r[j - 1], r[j], 8);
}

__device__ unsigned g_txl_viol = 0;  // checking build: reported violations

// bytes y, y+1 (y <= 22) of 6 dwords read at an aligned address, as BE16
__device__ __forceinline__ uint32_t be16_of6(const uint32_t x[6], uint32_t y) {
    uint32_t lo = x[0], hi = x[1];
#pragma unroll
    for (int u = 1; u < 5; u++)
        if ((y >> 2) == (uint32_t)u) {
            lo = x[u];
            hi = x[u + 1];
        }
    const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, y & 3);
    return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu);
}

template <int LGL>
__global__ __launch_bounds__(256) void k_txlog_lanes(
    uint64_t ntx, const uint8_t *__restrict__ buf, const uint64_t *__restrict__ rec_off,
    const uint64_t *__restrict__ alh_off, const uint64_t *__restrict__ leaf_off,
    const int32_t *__restrict__ pre, MhTxHeader *__restrict__ hdrs, uint8_t *__restrict__ eh_out,
    uint8_t *__restrict__ alh_out, int32_t *__restrict__ status, TxlogHostOut ho, int lgp,
    int dep, uint64_t blen_, const unsigned long long *__restrict__ wmax_dev,
    unsigned long long *__restrict__ redo) {
    extern __shared__ uint4 lds[];
    constexpr int L = 1 << LGL, R = 64 >> LGL;
    uint32_t *stk = reinterpret_cast<uint32_t *>(lds);  // [dep][256][9]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r = lane >> LGL, i = lane & (L - 1);
    // entries per lane (>= 1): from the widest record, known on the host, or
    // (wmax_dev) found by the structure pass on the device -- the launch's
    // lane count and stack depth were then sized for records up to 2^lgp
    // wide (an upper bound, or the caller's guess): wider ones and the launch
    // does nothing but raise *redo (uniform: every wave returns at once)
    int lgpk = lgp;
    if (wmax_dev) {
        const uint32_t wm = (uint32_t)*wmax_dev;
        lgpk = 0;
        while ((1u << lgpk) < wm) lgpk++;
        if (lgpk > lgp) {
            if (threadIdx.x == 0) atomicOr(redo, 1ull);
            return;
        }
    }
    const int EP = max(1, (1 << lgpk) >> LGL);
    const uint64_t TW = ((uint64_t)blockIdx.x * 4 + wv) * R;  // the wave's first record
    const uint64_t T0 = (uint64_t)blockIdx.x * 4 * R;        // the workgroup's
    const uint64_t t = TW + r;
    const bool valid = t < ntx;
    const int32_t pst = valid && pre ? pre[t] : 0;
    const bool act = valid && pst == 0;
    auto slot = [&](int d) -> uint32_t * { return stk + ((uint32_t)d * 256 + tid) * kTxlStackPad; };
    // checking build: a read range outside [buf, buf + len + 256) is reported
    // and read from buf instead
    auto ok_ = [&](const uint8_t *p, uint32_t n, int tag) -> const uint8_t * {
        if (!kTxlCheck) return p;
        const int64_t o = (int64_t)(p - buf);
        if (o >= 0 && (uint64_t)o + n <= blen_ + 256) return p;
        if (atomicAdd(&g_txl_viol, 1u) < 16)
            printf("txlog_lanes OOB tag=%d blk=%u tid=%d t=%llu off=%lld n=%u len=%llu\n", tag,
                   blockIdx.x, tid, (unsigned long long)t, (long long)o, n, (unsigned long long)blen_);
        return buf;
    };
    // ---- header (tx.go:419-518) and this lane's first entry (tx.go:578-585)
    const uint8_t *rp = act ? buf + rec_off[t] : buf;
    uint32_t ver = 0, ml = 0, nent = 0, w = 0, q = 0;
    if (act) {
        ver = rd_be16(ok_(rp + 88, 4, 1));
        if (ver == 0) {
            nent = rd_be16(ok_(rp + 90, 2, 2));
            q = 92;
        } else {
            ml = rd_be16(ok_(rp + 90, 2, 2));
            nent = bswap(rd_le32(ok_(rp + 92 + ml, 8, 3)));
            q = 96 + ml;
        }
        w = leaf_off ? (uint32_t)(leaf_off[t + 1] - leaf_off[t]) : nent;
    }
    const uint32_t j0 = (uint32_t)i * EP;
    // this lane's entries.  No subtraction under a condition: written as
    // `w > j0 ? min(EP, w - j0) : 0`, LLVM hoisted `sub nuw w, j0` out of its
    // guard and later turned the guard's select into a plain `or`, so for w <
    // j0 the test of ne branched on poison, and IndVarSimplify then dropped
    // the `j < w` bound of round 5's walk -- lanes past a record's last entry
    // walked off the log (profiles/lanes_walk_isa_r06.txt: ISA and IR trace).
    const uint32_t ne = act ? min((uint32_t)EP, w - min(w, j0)) : 0u;
    // skip the j0 entries of the lanes to the left; only a lane with entries
    // walks (a lane past the record's last entry has nothing to find).  Each
    // step reads the entry's first 24 bytes at once (mdLen and, for mdLen <=
    // 16, kLen in them): one load round trip per entry, not two.
    if (ne) {
        for (uint32_t j = 0; j < j0; j++) {
            const uint8_t *e = rp + q;
            const uint32_t o = (uint32_t)((uintptr_t)e & 3);
            const uint32_t *ea = reinterpret_cast<const uint32_t *>(ok_(e - o, 24, 4));
            uint32_t x[6];
#pragma unroll
            for (int u = 0; u < 6; u++) x[u] = ea[u];
            const uint32_t m = be16_of6(x, o);
            const uint32_t k = o + 4 + m <= 24 ? be16_of6(x, o + 2 + m) : rd_be16(ok_(e + 2 + m, 2, 5));
            q += 48 + m + k;
        }
    }
    // ---- 1. this lane's subtree: entries, leaves, merges, the final fold
    State s;
    s.init();
    uint32_t mode = ne ? 0u : 5u;  // 0 digest blocks, 1 leaf, 2 merge / fold (first block), 3 its tail, 5 done
    uint32_t ej = 0, b = 0, nb = 0, la = 0, c = 0, sp = 0, rt7 = 0;
    bool fold = false;
    const uint8_t *mp = rp;
    auto entry_setup = [&]() {  // entry ej of this lane at offset q
        const uint8_t *er = rp + q;
        const uint32_t m = rd_be16(ok_(er, 2, 6)), k = rd_be16(ok_(er + 2 + m, 2, 7));
        mp = ver == 1 ? er : er + 4 + m;  // tx.go:690-731
        la = ver == 1 ? 4 + m + k : k;
        nb = (la + 32 + 8) / 64 + 1;
        q += 48 + m + k;
        b = 0;
    };
    if (ne) entry_setup();
    // the next entry prefetched while this one hashes (a lane's loads are
    // otherwise ~3 dependent round trips per entry with no other wave on the
    // SIMD to cover them at L = 1): its first 24 bytes (mdLen, kLen) issued
    // before one compression, its first message block before the next, each
    // consumed after the compression it was issued before
    uint32_t pfs = ne > 1 ? 0u : 3u;  // 0 issue head, 1 parse head + issue block, 2 block loaded, 3 none
    uint32_t nq = q, n_la = 0, n_nb = 0, n_adv = 0;
    const uint8_t *n_mp = rp;
    uint32_t nx[6], pf[20];
    bool pfok = false;
#pragma unroll 1
    while (__builtin_amdgcn_ballot_w64(mode != 5)) {
        uint32_t wv16[16];
        bool on = true, tail = false;
        if (mode == 0) {
            if (b == 0) s.init();
            uint32_t d[20];
            if (b == 0 && pfok) {
#pragma unroll
                for (int j = 0; j < 20; j++) d[j] = pf[j];
                pfok = false;
            } else {
                const uint8_t *p0 = mp - ((uintptr_t)mp & 3) + 64 * b;
                skip12_load(ok_(p0, 80, 8) == p0 ? mp : buf + 4, b, d);
            }
            skip12_words(d, (uint32_t)((uintptr_t)mp & 3), la, b, nb, wv16);
        } else if (mode == 1) {
            wv16[0] = s.h[0] >> 8;
#pragma unroll
            for (int j = 1; j < 8; j++) wv16[j] = __builtin_amdgcn_alignbit(s.h[j - 1], s.h[j], 8);
            wv16[8] = (s.h[7] << 24) | 0x00800000u;
#pragma unroll
            for (int j = 9; j < 15; j++) wv16[j] = 0;
            wv16[15] = 33u * 8u;
            s.init();
        } else if (mode == 2) {  // pop right and left, SHA256(0x01 || left || right)
            uint32_t lf[8], rg[8];
            const uint32_t *pl = slot(sp - 2), *pr = slot(sp - 1);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) {
                lf[q2] = pl[q2];
                rg[q2] = pr[q2];
            }
            rt7 = rg[7];
            s.init();
            txl_node_first(lf, rg, wv16);
        } else if (mode == 3) {
            tail = true;
        } else {
            on = false;
        }
        // the prefetch stage of this iteration (loads land during the compression)
        if (pfs == 0) {
            const uint8_t *e = rp + nq;
            const uint32_t *ea = reinterpret_cast<const uint32_t *>(ok_(e - ((uintptr_t)e & 3), 24, 17));
#pragma unroll
            for (int j = 0; j < 6; j++) nx[j] = ea[j];
            pfs = 1;
        } else if (pfs == 1) {
            const uint32_t o = (uint32_t)((uintptr_t)(rp + nq) & 3);
            const uint32_t m = be16_of6(nx, o);
            const uint32_t k = o + 4 + m <= 24 ? be16_of6(nx, o + 2 + m) : rd_be16(ok_(rp + nq + 2 + m, 2, 18));
            const uint8_t *er = rp + nq;
            n_mp = ver == 1 ? er : er + 4 + m;  // as entry_setup
            n_la = ver == 1 ? 4 + m + k : k;
            n_nb = (n_la + 32 + 8) / 64 + 1;
            n_adv = 48 + m + k;
            const uint8_t *p0 = n_mp - ((uintptr_t)n_mp & 3);
            skip12_load(ok_(p0, 80, 19) == p0 ? n_mp : buf + 4, 0, pf);
            pfs = 2;
        }
        if (on) {
            if (tail)
                compress_node_tail_g(s, rt7);
            else
                compress(s, wv16);
        }
        // bookkeeping after the block
        if (mode == 0) {
            if (++b == nb) mode = 1;
        } else if (mode == 1 || mode == 3) {
            uint32_t *d = slot(mode == 1 ? sp : sp - 2);  // a leaf is pushed; a node replaces its children
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) d[q2] = s.h[q2];
            if (mode == 1) {
                sp++;
                c++;
                ej++;
            } else {
                sp--;
            }
            // next: the merges the c-th leaf owes (tz(c): the stack holds one
            // perfect subtree per set bit of c once they are done), the next
            // entry, or the fold
            if (!fold && sp > (uint32_t)__builtin_popcount(c)) {
                mode = 2;  // two perfect subtrees of one size on top: merge
            } else if (ej < ne) {
                if (pfs == 2) {  // the prefetched entry (q is at its start)
                    mp = n_mp;
                    la = n_la;
                    nb = n_nb;
                    q += n_adv;
                    b = 0;
                    pfok = true;
                } else {
                    entry_setup();
                }
                nq = q;
                pfs = ej + 1 < ne ? 0u : 3u;
                mode = 0;
            } else if (sp >= 2) {
                fold = true;  // right edge: fold the stack from the right
                mode = 2;
            } else {
                mode = 5;
            }
        } else if (mode == 2) {
            mode = 3;
        }
    }
    // ---- 2. the record's L lane roots paired (htree.go:85-110), via LDS
    // (slot 0 of each lane; a lane without entries holds nothing)
#pragma unroll 1
    for (int l = 0; l < LGL; l++) {
        txl_wave_sync();
        const uint32_t sft = 1u << l;
        const bool me = act && (i & (2 * sft - 1)) == 0 && (uint32_t)(i + sft) * EP < w;
        uint32_t wv16[16];
        if (me) {
            uint32_t lf[8], rg[8];
            const uint32_t *pl = slot(0), *pr = stk + (((uint32_t)0 * 256 + tid + sft) * kTxlStackPad);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) {
                lf[q2] = pl[q2];
                rg[q2] = pr[q2];
            }
            rt7 = rg[7];
            s.init();
            txl_node_first(lf, rg, wv16);
            compress(s, wv16);
            compress_node_tail_g(s, rt7);
        }
        txl_wave_sync();
        if (me) {
            uint32_t *d = slot(0);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) d[q2] = s.h[q2];
        }
    }
    txl_wave_sync();
    // ---- 3. innerHash + Alh on the record's first lane
    const bool head = act && i == 0;
    uint32_t eh[8], a[8];
    const uint32_t blen = ver ? 8 + ml : 4, mlen = 80 + blen;
    // fast path (every v0 record, v1 with mdLen <= 16): the record head
    // [rp, rp + 116) and the stored Alh in ONE batch of aligned dword loads,
    // the innerHash message assembled in this record's LDS row (33 words: no
    // bank conflicts between the wave's rows) with two aligned runs -- ts ||
    // (version ...nentries) and Eh || blTxID || blRoot shifted by blen & 3 --
    // and read back word by word; otherwise message bytes straight from the log
    const bool fast = !ver || ml <= 16;
    const uint32_t al = (uint32_t)((uintptr_t)rp & 3);
    uint32_t hrw[30], av[9];
    if (head && fast) {  // (a record is >= 124 bytes: header + Alh)
        const uint32_t *hb = reinterpret_cast<const uint32_t *>(ok_(rp - al, 120, 20));
#pragma unroll
        for (int j = 0; j < 30; j++) hrw[j] = hb[j];
        const uint8_t *ap = buf + alh_off[t];
        const uint32_t *ab = reinterpret_cast<const uint32_t *>(ok_(ap - ((uintptr_t)ap & 3), 36, 21));
#pragma unroll
        for (int j = 0; j < 9; j++) av[j] = ab[j];
    }
    auto le = [&](int o) -> uint32_t {  // the LE dword at rp + o (o: a constant multiple of 4, <= 112)
        return __builtin_amdgcn_alignbyte(hrw[o / 4 + 1], hrw[o / 4], al);
    };
    uint32_t *msg = stk + (uint32_t)dep * 256 * kTxlStackPad + ((uint32_t)wv * R + r) * 33;
    if (head) {
        if (w == 0) {
            load_digest(kTxlEmptyRoot, eh);  // SHA256(nil), htree.go:73-77
        } else {
            const uint32_t *p0 = slot(0);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) eh[q2] = p0[q2];
        }
        if (fast) {  // message bytes in order: [0,8) ts, [8, 8 + blen) rp[88..), then Eh, rp[16..56)
            msg[0] = le(8);
            msg[1] = le(12);
            const uint32_t nY = blen >> 2, sh = blen & 3;
#pragma unroll
            for (int u = 0; u < 7; u++)
                if ((uint32_t)u <= nY) msg[2 + u] = le(88 + 4 * u);  // u == nY: the partial word
            uint32_t S[18];
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) S[q2] = bswap(eh[q2]);
#pragma unroll
            for (int u = 0; u < 10; u++) S[8 + u] = le(16 + 4 * u);
            uint32_t *dst = msg + 2 + nY;
            const uint32_t prev = sh ? dst[0] << (8 * (4 - sh)) : 0u;  // Y's last sh bytes, on top
#pragma unroll
            for (int t2 = 0; t2 < 19; t2++) {
                const uint32_t lo = t2 ? S[t2 - 1] : prev, hi = t2 < 18 ? S[t2] : 0u;
                dst[t2] = sh ? __builtin_amdgcn_alignbyte(hi, lo, 4 - sh) : hi;
            }
        }
    }
    const uint32_t nbi = head ? (mlen + 8) / 64 + 1 : 0;
    const uint32_t nH = wave_max_u32(head ? nbi + 2 : 0);
#pragma unroll 1
    for (uint32_t k = 0; k < nH; k++) {
        uint32_t wv16[16];
        const bool on = head && k < nbi + 2;
        if (on) {
            if (k < nbi) {  // ts || version || md part || Eh || blTxID || blRoot
                if (k == 0) s.init();
                if (fast) {
#pragma unroll
                    for (int jw = 0; jw < 16; jw++) {
                        const int v = (int)mlen - (int)(64 * k + 4 * jw);  // message bytes left at this word
                        const uint32_t pad = (uint32_t)(0x80000000ull >> (8 * (v < 0 ? 5 : min(v, 4))));
                        wv16[jw] = __builtin_amdgcn_bitop3_b32(bswap(msg[16 * k + jw]), head_mask(v), pad, 0xEA);
                    }
                    if (k + 1 == nbi) {
                        wv16[14] = 0;
                        wv16[15] = mlen * 8;  // the bit length
                    }
                } else {
#pragma unroll 4
                    for (int jw = 0; jw < 16; jw++) {
                        uint32_t v32 = 0;
                        if (jw == 15 && k + 1 == nbi) {
                            v32 = mlen * 8;  // the bit length
                        } else {
#pragma unroll
                            for (int bb = 0; bb < 4; bb++) {
                                const uint32_t kk = 64 * k + 4 * jw + bb;
                                uint32_t v;
                                if (kk < 8) v = *ok_(rp + 8 + kk, 1, 9);
                                else if (kk < 8 + blen) v = *ok_(rp + 80 + kk, 1, 10);
                                else if (kk < 40 + blen) {
                                    const uint32_t o = kk - 8 - blen;
                                    v = (eh[o >> 2] >> (24 - 8 * (o & 3))) & 0xffu;
                                } else if (kk < mlen) v = *ok_(rp + kk - 24 - blen, 1, 11);
                                else v = kk == mlen ? 0x80u : 0u;
                                v32 = v32 << 8 | v;
                            }
                        }
                        wv16[jw] = v32;
                    }
                }
            } else if (k == nbi) {  // BE64 id || prevAlh || innerHash[0:24]
                copy8(a, s.h);      // (a: the innerHash until the Alh is done)
                s.init();
                if (fast) {
                    wv16[0] = bswap(le(0));
                    wv16[1] = bswap(le(4));
#pragma unroll
                    for (int q2 = 0; q2 < 8; q2++) wv16[2 + q2] = bswap(le(56 + 4 * q2));
                } else {
                    const uint64_t id = rd_be64(ok_(rp, 16, 12));
                    wv16[0] = (uint32_t)(id >> 32);
                    wv16[1] = (uint32_t)id;
#pragma unroll
                    for (int q2 = 0; q2 < 8; q2++) wv16[2 + q2] = bswap(rd_le32(ok_(rp + 56 + 4 * q2, 8, 13)));
                }
#pragma unroll
                for (int q2 = 0; q2 < 6; q2++) wv16[10 + q2] = a[q2];
            } else {
                wv16[0] = a[6];
                wv16[1] = a[7];
                wv16[2] = 0x80000000u;
#pragma unroll
                for (int q2 = 3; q2 < 15; q2++) wv16[q2] = 0;
                wv16[15] = 72u * 8u;
            }
            compress(s, wv16);
        }
    }
    copy8(a, s.h);
    int32_t stv = MH_OK;
    uint64_t hw[17];
    const bool fail_head = valid && !act && i == 0;  // rejected by the structure pre-pass
    if (head) {  // tx.go:623-627
        uint32_t xx = 0;
        if (fast) {
            const uint32_t aal = (uint32_t)((uintptr_t)(buf + alh_off[t]) & 3);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++)
                xx |= bswap(__builtin_amdgcn_alignbyte(av[q2 + 1], av[q2], aal)) ^ a[q2];
        } else {
            const uint8_t *ap = ok_(buf + alh_off[t], 40, 14);
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) xx |= bswap(rd_le32(ap + 4 * q2)) ^ a[q2];
        }
        stv = xx ? MH_ERR_CORRUPTED_DATA : MH_OK;
        status[t] = stv;
        store_digest(eh_out + t * 32, eh);
        store_digest(alh_out + t * 32, a);
        if (fast) {
#pragma unroll
            for (int q2 = 0; q2 < 3; q2++)
                hw[q2] = ((uint64_t)bswap(le(8 * q2)) << 32) | bswap(le(8 * q2 + 4));
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++)
                hw[3 + q2] = (uint64_t)le(24 + 8 * q2) | ((uint64_t)le(28 + 8 * q2) << 32);
        } else {
#pragma unroll
            for (int q2 = 0; q2 < 3; q2++) hw[q2] = rd_be64(ok_(rp + 8 * q2, 16, 15));
#pragma unroll
            for (int q2 = 0; q2 < 8; q2++) hw[3 + q2] = rd_raw64(ok_(rp + 24 + 8 * q2, 16, 16));
        }
#pragma unroll
        for (int q2 = 0; q2 < 4; q2++)
            hw[11 + q2] = (uint64_t)bswap(eh[2 * q2]) | ((uint64_t)bswap(eh[2 * q2 + 1]) << 32);
        hw[15] = (uint64_t)ver | ((uint64_t)nent << 32);
        hw[16] = ver ? (uint64_t)ml | ((uint64_t)(uint32_t)(rec_off[t] + 92) << 32) : 0;
    } else if (fail_head) {
#pragma unroll
        for (int q2 = 0; q2 < 8; q2++) a[q2] = 0;
#pragma unroll
        for (int q2 = 0; q2 < 17; q2++) hw[q2] = 0;
        stv = pst;
        status[t] = stv;
        store_digest(eh_out + t * 32, a);
        store_digest(alh_out + t * 32, a);
    }
    // ---- 4. the workgroup's records out as contiguous runs (the stack is free)
    __syncthreads();
    const uint32_t RW = 4 * R;  // records per workgroup
    uint64_t *hst = reinterpret_cast<uint64_t *>(lds);
    uint32_t *ast = reinterpret_cast<uint32_t *>(hst + RW * 17);
    uint32_t *sst = ast + RW * 8;
    const uint32_t rw = (uint32_t)wv * R + r;  // this record in the workgroup
    if (head || fail_head) {
#pragma unroll
        for (int q2 = 0; q2 < 17; q2++) hst[rw * 17 + q2] = hw[q2];
#pragma unroll
        for (int q2 = 0; q2 < 8; q2++) ast[rw * 8 + q2] = bswap(a[q2]);
        sst[rw] = (uint32_t)stv;
    }
    __syncthreads();
    const uint64_t nb_ = T0 < ntx ? min((uint64_t)RW, ntx - T0) : 0;
    uint64_t *hd = ho.hdrs ? ho.hdrs + T0 * 17 : hdrs ? reinterpret_cast<uint64_t *>(hdrs) + T0 * 17 : nullptr;
    if (ho.hdrs && ho.eh_only) {
        for (uint32_t k = tid; k < nb_ * 4; k += 256) {
            const uint32_t rec = k >> 2, j = 11 + (k & 3);
            hd[rec * 17 + j] = hst[rec * 17 + j];
        }
    } else if (hd) {
        for (uint32_t k = tid; k < nb_ * 17; k += 256) hd[k] = hst[k];
    }
    if (ho.alh)
        for (uint32_t k = tid; k < nb_ * 8; k += 256) ho.alh[T0 * 8 + k] = ast[k];
    if (ho.status)
        for (uint32_t k = tid; k < nb_; k += 256) ho.status[T0 + k] = sst[k];
}

// the lane count and stack depth of a launch over ntx records of <= wmax entries
struct TxlShape {
    int lgp, lgl, dep;
    size_t lds;
};
static TxlShape txl_shape(uint64_t ntx, uint64_t wmax) {
    TxlShape sh{};
    while ((1ull << sh.lgp) < wmax) sh.lgp++;
    // lanes per record: the fewest that give every SIMD two waves (2048 waves
    // of 64 lanes: one wave per SIMD issues VALU 0.76 of its cycles, two 0.9,
    // for ~10 % more instructions at L = 2, profiles/txlog_lanes_r05.txt; a
    // record's chain is 2 EP + 2 (EP - 1) + 2 log2 L + 4 compressions, EP = P /
    // L, so fewer records take more lanes: latency), at most 16;
    // MH_TXLOG_LANES=1|2|4|8|16 forces it (read per call, tests)
    int lgl = 0;
    while (lgl < 4 && (ntx << lgl) < 2048ull * 64) lgl++;  // two waves per SIMD (176 VGPRs: at most 2)
    // No LDS cap: from 33 entries a stack of >= 7 slots leaves room for one
    // workgroup per CU (one wave per SIMD), but more lanes per
    // record cost more: a lane past a record's last entry idles in its wave,
    // so the wave-instruction count grows with L unless every record is
    // exactly P wide.  131 072 records, kernel ms at L = 1 / 2 / 4: 40 entries
    // 1.05 / 1.51 / 1.55, 56: 1.46 / 1.53 / 1.62, 64: 1.66 / 1.52 / 1.62
    // (profiles/txlog_wide_r06.txt).
    if (const char *e = getenv("MH_TXLOG_LANES")) {  // exactly this many (the LDS cap too)
        const int v = atoi(e);
        lgl = v >= 16 ? 4 : v >= 8 ? 3 : v >= 4 ? 2 : v >= 2 ? 1 : 0;
    }
    sh.lgl = std::min(lgl, sh.lgp);  // never more lanes than entries
    const int R = 64 >> sh.lgl;
    sh.dep = std::max(1, sh.lgp - sh.lgl + 1);  // stack depth: log2(EP) + 1
    const size_t stack = (size_t)sh.dep * 256 * kTxlStackPad * 4 + (size_t)4 * R * 33 * 4;  // + innerHash rows
    const size_t res = (size_t)4 * R * (17 * 8 + 8 * 4 + 4);
    sh.lds = std::max(stack, res);
    return sh;
}

hipError_t launch_txlog_lanes(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                              const uint64_t *rec_off, const uint64_t *alh_off,
                              const uint64_t *leaf_off, const int32_t *pre, MhTxHeader *hdrs,
                              uint8_t *eh_out, uint8_t *alh_out, int32_t *status,
                              const TxlogHostOut &ho, uint64_t wmax, uint64_t log_len,
                              const uint64_t *wmax_dev, uint64_t *redo) {
    if (!ntx) return hipSuccess;
    if (wmax_dev && !redo) return hipErrorInvalidValue;
    if (wmax > kTxlLanesMaxEntries || ((uintptr_t)ho.hdrs & 7) || ((uintptr_t)ho.alh & 3) ||
        ((uintptr_t)ho.status & 3))
        return hipErrorInvalidValue;
    const TxlShape sh = txl_shape(ntx, wmax);
    static const bool attr = [] {
        const int mx = 160 << 10;
        const void *fs[] = {(const void *)k_txlog_lanes<0>, (const void *)k_txlog_lanes<1>,
                            (const void *)k_txlog_lanes<2>, (const void *)k_txlog_lanes<3>,
                            (const void *)k_txlog_lanes<4>};
        for (const void *f : fs) hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    TimerScope ts(tm, "txlog_lanes", st);
    const int R = 64 >> sh.lgl;
    const dim3 grid((unsigned)((ntx + 4ull * R - 1) / (4ull * R))), blk(256);
    if (kTxlCheck) {
        unsigned zero = 0;
        hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_txl_viol), &zero, sizeof zero, 0,
                                              hipMemcpyHostToDevice, st);
        if (e != hipSuccess) return e;
    }
#define MH_TXL(l_)                                                                                 \
    hipLaunchKernelGGL((k_txlog_lanes<l_>), grid, blk, sh.lds, st, ntx, buf, rec_off, alh_off,   \
                       leaf_off, pre, hdrs, eh_out, alh_out, status, ho, sh.lgp, sh.dep, log_len,   \
                       reinterpret_cast<const unsigned long long *>(wmax_dev),                  \
                       reinterpret_cast<unsigned long long *>(redo))
    if (sh.lgl == 0) MH_TXL(0);
    else if (sh.lgl == 1) MH_TXL(1);
    else if (sh.lgl == 2) MH_TXL(2);
    else if (sh.lgl == 3) MH_TXL(3);
    else MH_TXL(4);
#undef MH_TXL
    hipError_t e = hipGetLastError();
    if (kTxlCheck && e == hipSuccess) {  // the checking build: synchronous, fails on any out-of-range read
        unsigned viol = 0;
        e = hipMemcpyFromSymbolAsync(&viol, HIP_SYMBOL(g_txl_viol), sizeof viol, 0,
                                     hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e == hipSuccess && viol) {
            fprintf(stderr, "txlog_lanes: %u out-of-range reads\n", viol);
            return hipErrorIllegalAddress;
        }
    }
    return e;
}

}  // namespace mh
