// txlog_wave.hip -- a14 (tx.go:533-630 per record), one WAVE per R = 64 / L
// consecutive records with L lanes per record: the kernel of the last copy
// chunk's group of mh_txlog_validate (under 16384 records), whose chain per
// record is the shortest (the latency-shaped tail after the last byte lands).
//
// Four independent waves per 256-thread workgroup (the dispatcher spreads the
// workgroups over the CUs and a workgroup's waves over the CU's four SIMDs,
// so a small launch runs one wave per SIMD):
//   1. the wave's records (contiguous in the log, each ending with its stored
//      Alh) are copied into LDS with 16-byte LDS-DMA loads, one HBM round
//      trip; the header parse, the entry walk and the entry digests then read
//      LDS (a wave whose records do not fit reads the log in HBM instead);
//   2. the record's first lane walks its entries (tx.go:578-585) into an LDS
//      offset table;
//   3. lane i of a record hashes entries 2i and 2i+1 (entry digest
//      tx.go:690-731 + leaf htree.go:79-83, in place from the raw records)
//      and their node; the L lanes then reduce the tree level by level with
//      cross-lane shuffles (htree.go:85-110: node (k, l) hashes its two
//      children when the right one covers any leaf, else it is its left
//      child promoted);
//   4. the record's lanes assemble the innerHash message ts || version ||
//      (mdLen || md)? || nentries || Eh || blTxID || blRoot (tx.go:249-302;
//      every part but Eh is a byte range of the record head) as SHA words in
//      LDS, the first lane hashes it and the Alh (tx.go:307-319) and compares
//      it with the stored one (tx.go:623-627);
//   5. the results are staged in LDS and the whole workgroup stores its
//      records' header words, Alh words and statuses as contiguous runs
//      (device arrays, and the caller's pinned arrays when given).
// Every hash of a record goes through ONE compression site: each lane walks
// its own sequence of message blocks through one loop whose body builds the
// lane's next block (25 KB of code instead of ~20 straight-line copies, 173 KB,
// more than the CU pair's instruction cache).
//
// Records whose structure the device pre-pass rejected (pre[t] != 0,
// txlog_struct.hip) are not walked: their status is pre[t], Alh and header 0.
#include <algorithm>
#include <vector>

#include "txlog_common.hpp"

namespace mh {

// `make WAVE_PROBE=1` (diagnosis only, not in the default library): every
// wave's lane 0 stamps the 100 MHz real-time counter at its phase boundaries
// into g_wave_probe[wave][0..7] (read by mh_debug_txlog_wave_probe):
// 0 start, 1 records staged, 2 entry walk, 3 entry digests + leaves done,
// 4 tree done, 5 innerHash + Alh done, 6 results staged, 7 stores done
#ifndef MH_TXLOG_WAVE_PROBE
#define MH_TXLOG_WAVE_PROBE 0
#endif
#if MH_TXLOG_WAVE_PROBE
constexpr unsigned kWaveProbeWaves = 8192;
__device__ unsigned long long g_wave_probe[kWaveProbeWaves][8];
#define TXW_STAMP(k)                                                                        \
    do {                                                                                    \
        const unsigned wid_ = blockIdx.x * 4 + (threadIdx.x >> 6);                          \
        if ((threadIdx.x & 63) == 0 && wid_ < kWaveProbeWaves)                              \
            g_wave_probe[wid_][k] = __builtin_amdgcn_s_memrealtime();                       \
    } while (0)
#else
#define TXW_STAMP(k) \
    do {             \
    } while (0)
#endif

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

constexpr int kTxwE = 2;  // entries per lane (two leaves and their node in the lane)

template <bool GUARD>
__device__ __forceinline__ void txlog_wave_body(
    const uint8_t *rp, const uint8_t *ap, uint64_t t, uint64_t rec_g, uint64_t w, bool act,
    bool fail, int32_t pst, int lgl, int r, int i, uint32_t *__restrict__ eoff,
    uint32_t *__restrict__ msg, uint32_t *__restrict__ ehb, uint8_t *__restrict__ eh_out,
    uint8_t *__restrict__ alh_out, int32_t *__restrict__ status) {
    constexpr int E = kTxwE;
    const int L = 1 << lgl, P = L * E, R = 64 >> lgl;
    uint32_t ver = 0, ml = 0, nent = 0, q0 = 92;
    if (act) {  // tx.go:419-518
        ver = rd_be16(rp + 88);
        if (ver == 0) {
            nent = rd_be16(rp + 90);
        } else {
            ml = rd_be16(rp + 90);
            nent = bswap(rd_le32(rp + 92 + ml));
            q0 = 96 + ml;
        }
    }
    if (act && i == 0) {  // the entry walk, tx.go:578-585
        uint32_t q = q0;
        for (uint64_t j = 0; j < w; j++) {
            eoff[r * P + j] = q;
            const uint32_t m = rd_be16(rp + q);
            const uint32_t k = rd_be16(rp + q + 2 + m);
            q += 48 + m + k;
        }
    }
    txl_wave_sync();
    TXW_STAMP(2);
    // this lane's entries: digest message start / head length / blocks
    const uint8_t *mp0 = rp, *mp1 = rp;
    uint32_t la0 = 0, la1 = 0, nb0 = 0, nb1 = 0, steps0 = 0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint64_t j = (uint64_t)i * E + e;
        if (act && j < w) {
            const uint8_t *er = rp + eoff[r * P + j];
            const uint32_t m = rd_be16(er), k = rd_be16(er + 2 + m);
            const uint8_t *pp = ver == 1 ? er : er + 4 + m;  // tx.go:690-731
            const uint32_t la = ver == 1 ? 4 + m + k : k;
            const uint32_t nb = (la + 32 + 8) / 64 + 1;
            if (e == 0) { mp0 = pp; la0 = la; nb0 = nb; } else { mp1 = pp; la1 = la; nb1 = nb; }
            steps0 += nb + 1;
        }
    }
    const uint32_t blen = ver ? 8 + ml : 4;  // version || (mdLen || md || nentries) | nentries16
    const uint32_t mlen = 80 + blen;
    const uint32_t nw = ((mlen + 8) / 64 + 1) * 16, nbi = nw / 16;
    const uint32_t n0 = wave_max_u32(steps0);
    const uint32_t n1 = 2 * (1 + lgl);
    const uint32_t n2 = wave_max_u32(act && i == 0 ? nbi + 2 : 0);
    uint32_t *M = msg + r * kTxMsgWords;
    uint32_t *EB = ehb + r * 8;
    State s;
    s.init();
    uint32_t nd[8], lf1[8], rt[8], inner[8];
#pragma unroll
    for (int q = 0; q < 8; q++) nd[q] = lf1[q] = rt[q] = inner[q] = 0;
    uint32_t e = 0, b = 0;
#pragma unroll 1
    for (uint32_t g = 0; g < n0 + n1 + n2; g++) {
        if (MH_TXLOG_WAVE_PROBE && g == n0) TXW_STAMP(3);
        if (MH_TXLOG_WAVE_PROBE && g == n0 + n1) TXW_STAMP(4);
        uint32_t wv[16];
        bool on = false, lev = false;
        uint32_t half = 0;
        if (g < n0) {  // entry digest blocks, then its leaf (htree.go:79-83)
            const bool e1 = e == 1;
            const uint32_t nbe = e1 ? nb1 : nb0;
            if (e < (uint32_t)E && nbe > 0) {
                on = true;
                if (b < nbe) {
                    if (b == 0) s.init();
                    skip12_block<GUARD>(e1 ? mp1 : mp0, e1 ? la1 : la0, b, nbe, wv);
                } else {
                    wv[0] = s.h[0] >> 8;
#pragma unroll
                    for (int j = 1; j < 8; j++) wv[j] = __builtin_amdgcn_alignbit(s.h[j - 1], s.h[j], 8);
                    wv[8] = (s.h[7] << 24) | 0x00800000u;
#pragma unroll
                    for (int j = 9; j < 15; j++) wv[j] = 0;
                    wv[15] = 33u * 8u;
                    s.init();
                }
            }
        } else if (g < n0 + n1) {  // one tree level per two blocks (htree.go:85-110)
            const uint32_t k = g - n0, lv = k >> 1;
            half = k & 1;
            const bool local = lv == 0;  // the lane's own two leaves
            const uint32_t sft = local ? 0 : 1u << (lv - 1);
            if (half == 0) {
                if (local) {
                    copy8(rt, lf1);
                } else {
#pragma unroll
                    for (int q = 0; q < 8; q++) rt[q] = (uint32_t)__shfl_down((int)nd[q], sft, 64);
                }
            }
            const bool h = local ? act && (uint64_t)i * 2 + 1 < w
                                 : act && (i & (2 * sft - 1)) == 0 && (uint64_t)(i + sft) * E < w;
            if (h) {
                on = lev = true;
                if (half == 0) {
                    s.init();
                    wv[0] = 0x01000000u | (nd[0] >> 8);
#pragma unroll
                    for (int j = 1; j < 8; j++) wv[j] = __builtin_amdgcn_alignbit(nd[j - 1], nd[j], 8);
                    wv[8] = __builtin_amdgcn_alignbit(nd[7], rt[0], 8);
#pragma unroll
                    for (int j = 1; j < 8; j++) wv[8 + j] = __builtin_amdgcn_alignbit(rt[j - 1], rt[j], 8);
                }  // half 1: the padding block, from the K+W table below
            }
        } else {  // innerHash (tx.go:249-302) then Alh (tx.go:307-319)
            const uint32_t k = g - n0 - n1;
            if (k == 0) {
                if (act && i == 0) {
                    if (w == 0) load_digest(kTxlEmptyRoot, nd);  // SHA256(nil), htree.go:73-77
#pragma unroll
                    for (int q = 0; q < 8; q++) EB[q] = bswap(nd[q]);
                }
                txl_wave_sync();
                if (act) {
                    const uint8_t *eb = reinterpret_cast<const uint8_t *>(EB);
                    for (uint32_t jw = i; jw < nw; jw += L) {
                        uint32_t x = 0;
                        if (jw == nw - 1) {
                            x = mlen * 8;
                        } else {
#pragma unroll
                            for (int bb = 0; bb < 4; bb++) {
                                const uint32_t kk = 4 * jw + bb;
                                uint32_t v;
                                if (kk < 8) v = rp[8 + kk];
                                else if (kk < 8 + blen) v = rp[80 + kk];
                                else if (kk < 40 + blen) v = eb[kk - 8 - blen];
                                else if (kk < mlen) v = rp[kk - 24 - blen];
                                else v = kk == mlen ? 0x80u : 0u;
                                x = x << 8 | v;
                            }
                        }
                        M[jw] = x;
                    }
                }
                txl_wave_sync();
            }
            if (act && i == 0 && k < nbi + 2) {
                on = true;
                if (k < nbi) {
                    if (k == 0) s.init();
                    const uint4 *m4 = reinterpret_cast<const uint4 *>(M + 16 * k);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint4 y = m4[q];
                        wv[4 * q] = y.x;
                        wv[4 * q + 1] = y.y;
                        wv[4 * q + 2] = y.z;
                        wv[4 * q + 3] = y.w;
                    }
                } else if (k == nbi) {  // BE64 id || prevAlh || innerHash[0:24]
                    copy8(inner, s.h);
                    s.init();
                    const uint64_t id = rd_be64(rp);
                    wv[0] = (uint32_t)(id >> 32);
                    wv[1] = (uint32_t)id;
#pragma unroll
                    for (int q = 0; q < 8; q++) wv[2 + q] = bswap(rd_le32(rp + 56 + 4 * q));
#pragma unroll
                    for (int q = 0; q < 6; q++) wv[10 + q] = inner[q];
                } else {
                    wv[0] = inner[6];
                    wv[1] = inner[7];
                    wv[2] = 0x80000000u;
#pragma unroll
                    for (int q = 3; q < 15; q++) wv[q] = 0;
                    wv[15] = 72u * 8u;
                }
            }
        }
        if (on) {
            if (lev && half == 1)
                compress_node_tail_g(s, rt[7]);
            else
                compress(s, wv);
        }
        if (g < n0) {
            if (on) {
                const bool e1 = e == 1;
                if (b == (e1 ? nb1 : nb0)) {
                    if (e1) copy8(lf1, s.h);
                    else copy8(nd, s.h);
                    e++;
                    b = 0;
                } else {
                    b++;
                }
            }
        } else if (lev && half == 1) {
            copy8(nd, s.h);
        }
    }
    TXW_STAMP(5);
    uint32_t a[8];
    copy8(a, s.h);
    int32_t stv = MH_OK;
    if (act && i == 0) {
        uint32_t x = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) x |= bswap(rd_le32(ap + 4 * q)) ^ a[q];
        stv = x ? MH_ERR_CORRUPTED_DATA : MH_OK;
        status[t] = stv;
        store_digest(eh_out + t * 32, nd);
        store_digest(alh_out + t * 32, a);
    } else if (fail && i == 0) {  // rejected by the structure pre-pass
#pragma unroll
        for (int q = 0; q < 8; q++) a[q] = 0;
        stv = pst;
        status[t] = stv;
        store_digest(eh_out + t * 32, a);
        store_digest(alh_out + t * 32, a);
    }
    txl_wave_sync();  // msg is free: results staged there
    uint64_t *hst = reinterpret_cast<uint64_t *>(msg);  // R x 17 header words
    uint32_t *ast = msg + R * 34;                        // R x 8 Alh words (bytes as stored)
    uint32_t *sst = msg + R * 42;                        // R statuses
    if (act || fail) {
        if (i == 0) {
#pragma unroll
            for (int q = 0; q < 8; q++) ast[r * 8 + q] = bswap(a[q]);
            sst[r] = (uint32_t)stv;
        }
        for (int q = i; q < 17; q += L) {
            uint64_t v = 0;
            if (!act) v = 0;
            else if (q < 3) v = rd_be64(rp + 8 * q);
            else if (q < 11) v = rd_raw64(rp + 24 + 8 * (q - 3));
            else if (q < 15) v = (uint64_t)EB[2 * (q - 11)] | ((uint64_t)EB[2 * (q - 11) + 1] << 32);
            else if (q == 15) v = (uint64_t)ver | ((uint64_t)nent << 32);
            else v = ver ? (uint64_t)ml | ((uint64_t)(uint32_t)(rec_g + 92) << 32) : 0;
            hst[r * 17 + q] = v;
        }
    }
    txl_wave_sync();
    TXW_STAMP(6);
}

constexpr int kTxWaves = 4;  // independent waves per workgroup

// per-wave LDS: [records sbytes][innerHash messages / results R x 384 B]
// [entry offsets 64 E words][Eh R x 32 B]
__host__ __device__ constexpr uint32_t txw_wave_bytes(uint32_t sbytes, int R) {
    return sbytes + R * kTxMsgWords * 4 + 64 * kTxwE * 4 + R * 32;
}

template <bool STAGED>
__global__ __launch_bounds__(256) void k_txlog_wave(
    uint64_t ntx, const uint8_t *__restrict__ buf, const uint64_t *__restrict__ rec_off,
    const uint64_t *__restrict__ alh_off, const uint64_t *__restrict__ leaf_off,
    const int32_t *__restrict__ pre, MhTxHeader *__restrict__ hdrs, uint8_t *__restrict__ eh_out,
    uint8_t *__restrict__ alh_out, int32_t *__restrict__ status, TxlogHostOut ho, int lgl,
    uint32_t sbytes) {
    extern __shared__ uint4 lds[];
    const int R = 64 >> lgl;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane >> lgl, i = lane & ((1 << lgl) - 1);
    const uint32_t wbytes = txw_wave_bytes(sbytes, R);
    uint8_t *wl = reinterpret_cast<uint8_t *>(lds) + wv * wbytes;
    uint32_t *msg = reinterpret_cast<uint32_t *>(wl + sbytes);
    uint32_t *eoff = msg + R * kTxMsgWords, *ehb = eoff + 64 * kTxwE;
    const uint64_t T0 = (uint64_t)blockIdx.x * kTxWaves * R;  // the workgroup's first record
    const uint64_t t0 = T0 + (uint64_t)wv * R;                 // the wave's
    TXW_STAMP(0);
    if (t0 < ntx) {  // wave-uniform
        const uint64_t nmine = min((uint64_t)R, ntx - t0);
        const bool mine = (uint64_t)r < nmine;
        const int32_t pst = mine && pre ? pre[t0 + r] : 0;
        const bool act = mine && pst == 0, fail = mine && pst != 0;
        const uint64_t t = mine ? t0 + r : t0;
        const uint64_t w = act ? leaf_off[t + 1] - leaf_off[t] : 0;
        const uint64_t rec_g = rec_off[t];
        if (STAGED) {
            // 1. the wave's records into LDS by LDS-DMA, every piece in flight
            // at once (+96 bytes: rd_le32 reads a dword ahead, skip12_block a
            // block's 80 bytes from its start unguarded)
            const uint64_t lo = rec_off[t0] & ~15ull, hi = alh_off[t0 + nmine - 1] + 32 + 96;
            const uint8_t *g = buf + lo;
            const uint32_t n16 = (uint32_t)((hi - lo + 15) >> 4);
            for (uint32_t k = 0; k < n16; k += 64) {
                const uint32_t c = min(k + lane, n16 - 1);  // the last lanes repeat the last piece
                __builtin_amdgcn_global_load_lds((tx_glb_void_t *)(g + 16 * (uint64_t)c),
                                                 (tx_lds_void_t *)(wl + 16 * k), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            TXW_STAMP(1);
            txlog_wave_body<false>(wl + (rec_g - lo), wl + (alh_off[t] - lo), t, rec_g, w, act,
                                   fail, pst, lgl, r, i, eoff, msg, ehb, eh_out, alh_out, status);
        } else {
            txlog_wave_body<true>(buf + rec_g, buf + alh_off[t], t, rec_g, w, act, fail, pst, lgl,
                                  r, i, eoff, msg, ehb, eh_out, alh_out, status);
        }
    }
    __syncthreads();  // every wave's results are staged in its msg slice
    // 5. the workgroup's records [T0, T0 + nb) out as contiguous runs
    const uint64_t nb = T0 < ntx ? min((uint64_t)kTxWaves * R, ntx - T0) : 0;
    const uint32_t *m0 = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(lds) + sbytes);
    const uint32_t wwords = wbytes / 4;
    const int lgr = 6 - lgl;
    // the device headers only when the caller's are not written here (they
    // are what a D2H copy takes to pageable outputs)
    uint64_t *hd = ho.hdrs ? ho.hdrs + T0 * 17 : reinterpret_cast<uint64_t *>(hdrs) + T0 * 17;
    if (ho.hdrs && ho.eh_only) {  // words 11-14 of each record's header (Eh); the host fills the rest
        for (uint32_t k = threadIdx.x; k < nb * 4; k += 256) {
            const uint32_t rec = k >> 2, j = 11 + (k & 3);
            hd[rec * 17 + j] = reinterpret_cast<const uint64_t *>(m0 + (rec >> lgr) * wwords)[(rec & (R - 1)) * 17 + j];
        }
    } else {
        for (uint32_t k = threadIdx.x; k < nb * 17; k += 256) {
            const uint32_t rec = k / 17, j = k - rec * 17;
            hd[k] = reinterpret_cast<const uint64_t *>(m0 + (rec >> lgr) * wwords)[(rec & (R - 1)) * 17 + j];
        }
    }
    if (ho.alh)
        for (uint32_t k = threadIdx.x; k < nb * 8; k += 256) {
            const uint32_t rec = k >> 3;
            ho.alh[T0 * 8 + k] = m0[(rec >> lgr) * wwords + R * 34 + (rec & (R - 1)) * 8 + (k & 7)];
        }
    if (ho.status)
        for (uint32_t k = threadIdx.x; k < nb; k += 256)
            ho.status[T0 + k] = m0[(k >> lgr) * wwords + R * 42 + (k & (R - 1))];
    if (MH_TXLOG_WAVE_PROBE) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        TXW_STAMP(7);
    }
    // (no system fence: the caller reads the pinned results only after
    // synchronizing the stream, whose end-of-kernel release is system-scope; a
    // fence here held every wave until its PCIe writes completed)
}

hipError_t launch_txlog_wave(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                             const uint64_t *rec_off, const uint64_t *alh_off,
                             const uint64_t *leaf_off, const int32_t *pre, MhTxHeader *hdrs,
                             uint8_t *eh_out, uint8_t *alh_out, int32_t *status,
                             const TxlogHostOut &ho, uint64_t wmax, const uint64_t *h_rec_off,
                             const uint64_t *h_alh_off) {
    if (!ntx) return hipSuccess;
    if (wmax > 64 || ((uintptr_t)ho.hdrs & 7) || ((uintptr_t)ho.alh & 3) || ((uintptr_t)ho.status & 3))
        return hipErrorInvalidValue;
    int lgp = 0;
    while ((1ull << lgp) < wmax) lgp++;
    const int lgl = std::max(2, lgp - 1);  // >= 4 lanes per record: <= 16 records a wave
    const int R = 64 >> lgl;
    // the widest wave's records (+ alignment and over-read pad) decide whether
    // the waves stage their records in LDS
    uint64_t span = 0;
    for (uint64_t t0 = 0; t0 < ntx; t0 += R) {
        const uint64_t tl = std::min<uint64_t>(ntx, t0 + R) - 1;
        span = std::max<uint64_t>(span, h_alh_off[tl] + 32 + 96 - (h_rec_off[t0] & ~15ull));
    }
    // whole 1 KiB pieces: the LDS-DMA's last pass writes all 64 lanes' slots
    const uint64_t sb = (span + 1023) & ~1023ull;
    // MH_TXLOG_STAGE_MAX (bytes, read per call: tests force the HBM path with 0);
    // four waves' slices must fit the CU's 160 KB
    const char *sm = getenv("MH_TXLOG_STAGE_MAX");
    const uint64_t smax = sm ? strtoull(sm, nullptr, 10) : (32u << 10);
    const bool staged = sb <= std::min<uint64_t>(smax, 32u << 10);
    const uint32_t sbytes = staged ? (uint32_t)sb : 0;
    const size_t sh = (size_t)kTxWaves * txw_wave_bytes(sbytes, R);
    TimerScope ts(tm, "txlog_wave", st);
    const dim3 grid(grid_for(ntx, (unsigned)(kTxWaves * R))), blk(256);
    // up to 160 KB of dynamic LDS (once per instantiation)
    static const bool attr = [] {
        const int mx = 160 << 10;
        hipFuncSetAttribute((const void *)k_txlog_wave<true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        hipFuncSetAttribute((const void *)k_txlog_wave<false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    if (staged)
        hipLaunchKernelGGL(k_txlog_wave<true>, grid, blk, sh, st, ntx, buf, rec_off, alh_off,
                           leaf_off, pre, hdrs, eh_out, alh_out, status, ho, lgl, sbytes);
    else
        hipLaunchKernelGGL(k_txlog_wave<false>, grid, blk, sh, st, ntx, buf, rec_off, alh_off,
                           leaf_off, pre, hdrs, eh_out, alh_out, status, ho, lgl, sbytes);
    return hipGetLastError();
}

}  // namespace mh

#if MH_TXLOG_WAVE_PROBE
// diagnosis build only: the stamps of waves [0, nwaves) (8 x u64 each); reset
// with out == NULL
extern "C" __attribute__((visibility("default"))) int mh_debug_txlog_wave_probe(unsigned long long *out,
                                                                                unsigned nwaves) {
    nwaves = std::min(nwaves, mh::kWaveProbeWaves);
    if (!out) {
        std::vector<unsigned long long> z(mh::kWaveProbeWaves * 8, 0);
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(mh::g_wave_probe), z.data(), z.size() * 8);
    }
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mh::g_wave_probe), (size_t)nwaves * 64);
}
#endif
