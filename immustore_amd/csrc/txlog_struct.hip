// txlog_struct.hip -- the structure of tx-log records checked on the device,
// one lane per record: the record hop of mh_txlog_validate (readHeader /
// readEntry, tx.go:419-588, with the KVMetadata / TxMetadata parses of
// kv_metadata.go:207-256 and tx_metadata.go:145-193) over bytes that are
// already in HBM, so that the fused a14 kernels never walk a length they
// have not seen checked.
//
//  * cLog mode (mh_txlog_validate_clog): record t is read where commit-log
//    entry t points (txOffsetAndSize, immustore.go:2569-2597: BE64 offset ||
//    BE32 size, + the Alh in 44-byte entries, :122-123), as readTx reads it
//    (immustore.go:3048-3060: from that offset on to the end of the log --
//    the reader is not limited to the size; a read past the log is the
//    reader's unexpected EOF).  The store's own consistency checks come on
//    top (the open path, immustore.go:458-528): the record must end exactly
//    at offset + size, and a 44-byte entry's Alh must be the record's.
//  * check mode (mh_txlog_validate_resident): the host hop parsed the host
//    copy; the device bytes must parse to the same records within the same
//    extents, else the record is MH_ERR_CORRUPTED_DATA (the resident bytes
//    drifted from the host copy) -- never a walk past the record.
#include <algorithm>

#include "txlog_common.hpp"

namespace mh {

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

__device__ __forceinline__ uint64_t ld_be(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int k = 0; k < n; k++) v = v << 8 | p[k];
    return v;
}

// KVMetadata.unsafeReadFrom (kv_metadata.go:207-256): deleted(0),
// expiresAt(1, 8 bytes), nonIndexable(2); an unknown code or a short
// expiresAt is ErrCorruptedData.  Bytes() writes each attribute once in code
// order, so the stored form is canonical iff its codes strictly increase.
// Returns MH_OK / MH_ERR_CORRUPTED_DATA; *canon: the canonical form.
__device__ __forceinline__ int kv_md_check(const uint8_t *md, uint32_t ml, bool *canon) {
    if (ml > MH_MAX_KV_METADATA_LEN) return MH_ERR_CORRUPTED_DATA;
    int last = -1;
    bool inc = true;
    for (uint32_t i = 0; i < ml;) {
        const uint32_t code = md[i++];
        if (code == 1) {
            if (ml - i < 8) return MH_ERR_CORRUPTED_DATA;
            i += 8;
        } else if (code > 2) {
            return MH_ERR_CORRUPTED_DATA;
        }
        inc &= (int)code > last;
        last = (int)code;
    }
    *canon = inc;
    return MH_OK;
}

// TxMetadata.ReadFrom (tx_metadata.go:145-193): truncatedUptoTx(0, 8 bytes),
// extra(1, BE16 length + up to 256 bytes); canonical iff the codes strictly
// increase (Bytes() writes each once, in code order)
__device__ __forceinline__ int tx_md_check(const uint8_t *md, uint32_t ml, bool *canon) {
    if (ml > MH_MAX_TX_METADATA_LEN) return MH_ERR_CORRUPTED_DATA;
    int last = -1;
    bool inc = true;
    for (uint32_t i = 0; i < ml;) {
        const uint32_t code = md[i++];
        if (code == 0) {
            if (ml - i < 8) return MH_ERR_CORRUPTED_DATA;
            i += 8;
        } else if (code == 1) {
            if (ml - i < 2) return MH_ERR_CORRUPTED_DATA;
            const uint32_t el = rd_be16(md + i);
            i += 2;
            if (ml - i < el || el > 256) return MH_ERR_CORRUPTED_DATA;
            i += el;
        } else {
            return MH_ERR_CORRUPTED_DATA;
        }
        inc &= (int)code > last;
        last = (int)code;
    }
    *canon = inc;
    return MH_OK;
}

// the record at p read within [p, lim), exactly hop_record's checks in its
// order (capi_tx.hip, tx.go:419-588); eof: no record there (id 0 or no room
// for an id)
__device__ int struct_record(const uint8_t *buf, uint64_t p, uint64_t lim, uint32_t max_entries,
                             uint32_t max_key_len, uint32_t &nent, uint64_t &alh, bool &eof,
                             bool &canon) {
    eof = false;
    canon = true;
    nent = 0;
    if (p >= lim || lim - p < 8) {  // (p from a cLog entry may be anything)
        eof = true;
        return MH_OK;
    }
    if (ld_be(buf + p, 8) == 0) {  // a preallocated tail reads as EOF (tx.go:427-430)
        eof = true;
        return MH_OK;
    }
    if (p + 90 > lim) return MH_ERR_TRUNCATED;
    const uint32_t ver = (uint32_t)ld_be(buf + p + 88, 2);
    uint64_t q = p + 90;
    if (ver == 0) {
        if (q + 2 > lim) return MH_ERR_TRUNCATED;
        nent = (uint32_t)ld_be(buf + q, 2);
        q += 2;
    } else if (ver == 1) {
        if (q + 2 > lim) return MH_ERR_TRUNCATED;
        const uint32_t mdl = (uint32_t)ld_be(buf + q, 2);
        q += 2;
        if (mdl > MH_MAX_TX_METADATA_LEN) return MH_ERR_CORRUPTED_DATA;
        if (q + mdl > lim) return MH_ERR_TRUNCATED;
        bool c = true;
        if (tx_md_check(buf + q, mdl, &c)) return MH_ERR_CORRUPTED_DATA;
        canon &= c;
        if (q + mdl + 4 > lim) return MH_ERR_TRUNCATED;
        if (q > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // md_off is 32-bit
        q += mdl;
        nent = (uint32_t)ld_be(buf + q, 4);
        q += 4;
    } else {
        return MH_ERR_CORRUPTED_UNKNOWN_VERSION;
    }
    if (nent > max_entries) return MH_ERR_CORRUPTED_MAX_ENTRIES;
    for (uint32_t e = 0; e < nent; e++) {
        if (q + 2 > lim) return MH_ERR_TRUNCATED;
        const uint32_t ml = (uint32_t)ld_be(buf + q, 2);
        if (q + 2 + ml > lim) return MH_ERR_TRUNCATED;
        bool c = true;
        if (ml && kv_md_check(buf + q + 2, ml, &c)) return MH_ERR_CORRUPTED_DATA;
        canon &= c;
        if (q + 4 + ml > lim) return MH_ERR_TRUNCATED;
        const uint32_t kl = (uint32_t)ld_be(buf + q + 2 + ml, 2);
        if (kl > max_key_len) return MH_ERR_CORRUPTED_MAX_KEYLEN;
        if (q + 4 + ml + kl + 12 + 32 > lim) return MH_ERR_TRUNCATED;
        // a v0 header cannot carry KV metadata (TxEntryDigest_v1_1, tx.go:690-693)
        if (ver == 0 && ml > 0) return MH_ERR_METADATA_UNSUPPORTED;
        q += 4 + ml + kl + 12 + 32;
    }
    if (q + 32 > lim) return MH_ERR_TRUNCATED;
    alh = q;
    return MH_OK;
}

__global__ __launch_bounds__(256) void k_txlog_struct(
    uint64_t ntx, const uint8_t *__restrict__ buf, uint64_t len, uint64_t lim,
    const uint8_t *__restrict__ clog,
    uint32_t es, uint64_t *__restrict__ rec_off, uint64_t *__restrict__ alh_off,
    uint64_t *__restrict__ leaf_off, uint32_t max_entries, uint32_t max_key_len,
    int32_t *__restrict__ pre, unsigned long long *__restrict__ stats) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx) return;
    uint32_t nent = 0;
    uint64_t alh = 0;
    bool eof = false, canon = true;
    int st;
    if (clog) {
        const uint8_t *ce = clog + t * es;
        const uint64_t p = ld_be(ce, 8), size = ld_be(ce + 8, 4);
        st = struct_record(buf, p, lim, max_entries, max_key_len, nent, alh, eof, canon);
        if (st == MH_OK && eof) st = MH_ERR_TRUNCATED;  // readTx: unexpected EOF (immustore.go:3054-3056)
        // a read past the bytes landed (not past the log's end)
        const bool cut_short = st == MH_ERR_TRUNCATED && lim < len && p < len && len - p >= 8;
        if (st == MH_OK && alh + 32 - p != size) st = MH_ERR_CORRUPTED_DATA;  // the cLog disagrees
        if (st == MH_OK && es == 44) {  // the cLog's Alh (immustore.go:519-527)
            uint32_t x = 0;
            for (int k = 0; k < 32; k++) x |= (uint32_t)(ce[12 + k] ^ buf[alh + k]);
            if (x) st = MH_ERR_CORRUPTED_DATA;
        }
        rec_off[t] = p;
        alh_off[t] = st == MH_OK ? alh : p;
        if (cut_short || (st == MH_OK && (!canon || nent > kTxlLanesMaxEntries))) st = kTxlNeedsHost;
    } else {
        const uint64_t p = rec_off[t], a = alh_off[t];
        st = struct_record(buf, p, a + 32, max_entries, max_key_len, nent, alh, eof, canon);
        // the host copy's structure: the same entry count, the Alh where the
        // host found it, metadata in the form the host hashed
        if (st != MH_OK || eof || !canon || alh != a || nent != leaf_off[t + 1] - leaf_off[t])
            st = MH_ERR_CORRUPTED_DATA;
    }
    pre[t] = st;
    if (st == MH_OK)
        atomicMax(&stats[0], (unsigned long long)nent);
    else if (st == kTxlNeedsHost)
        atomicAdd(&stats[1], 1ull);
}

hipError_t launch_txlog_struct(hipStream_t st, Timer *tm, uint64_t ntx, const uint8_t *buf,
                               uint64_t len, uint64_t lim, const uint8_t *clog, uint32_t clog_es,
                               uint64_t *rec_off, uint64_t *alh_off, uint64_t *leaf_off,
                               uint32_t max_entries, uint32_t max_key_len, int32_t *pre,
                               uint64_t *stats) {
    if (!ntx) return hipSuccess;
    TimerScope ts(tm, "txlog_struct", st);
    hipLaunchKernelGGL(k_txlog_struct, dim3(grid_for(ntx, 256)), dim3(256), 0, st, ntx, buf, len,
                       std::min(lim, len), clog, clog_es, rec_off, alh_off, leaf_off, max_entries, max_key_len, pre,
                       reinterpret_cast<unsigned long long *>(stats));
    return hipGetLastError();
}

// records whose bytes in a differ from b over [rec_off, alh_off + 32): pre =
// MH_ERR_CORRUPTED_DATA (the resident log against the host copy uploaded
// beside it, for the groups the fused kernels do not take).  One wave per
// record, 16-byte pieces where both sides allow.
__global__ __launch_bounds__(256) void k_txlog_bytes_cmp(uint64_t ntx, const uint8_t *__restrict__ a,
                                                         const uint8_t *__restrict__ b,
                                                         const uint64_t *__restrict__ rec_off,
                                                         const uint64_t *__restrict__ alh_off,
                                                         int32_t *__restrict__ pre) {
    const uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= ntx) return;
    const uint64_t lo = rec_off[t], hi = alh_off[t] + 32;
    uint32_t d = 0;
    for (uint64_t p = lo + lane; p < hi; p += 64) d |= (uint32_t)(a[p] ^ b[p]);
    if (__builtin_amdgcn_ballot_w64(d != 0) && lane == 0) pre[t] = MH_ERR_CORRUPTED_DATA;
    else if (lane == 0) pre[t] = MH_OK;
}

// statuses of records whose pre-status is set: pre[t] (Alh zeroed)
__global__ __launch_bounds__(256) void k_txlog_apply_pre(uint64_t ntx, const int32_t *__restrict__ pre,
                                                         int32_t *__restrict__ status,
                                                         uint8_t *__restrict__ alh) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntx || !pre[t]) return;
    status[t] = pre[t];
    uint4 *o = reinterpret_cast<uint4 *>(alh + t * 32);
    o[0] = make_uint4(0, 0, 0, 0);
    o[1] = make_uint4(0, 0, 0, 0);
}

hipError_t launch_txlog_bytes_cmp(hipStream_t st, uint64_t ntx, const uint8_t *a, const uint8_t *b,
                                  const uint64_t *rec_off, const uint64_t *alh_off, int32_t *pre) {
    if (!ntx) return hipSuccess;
    hipLaunchKernelGGL(k_txlog_bytes_cmp, dim3(grid_for(ntx, 4)), dim3(256), 0, st, ntx, a, b,
                       rec_off, alh_off, pre);
    return hipGetLastError();
}

hipError_t launch_txlog_apply_pre(hipStream_t st, uint64_t ntx, const int32_t *pre, int32_t *status,
                                  uint8_t *alh) {
    if (!ntx) return hipSuccess;
    hipLaunchKernelGGL(k_txlog_apply_pre, dim3(grid_for(ntx, 256)), dim3(256), 0, st, ntx, pre,
                       status, alh);
    return hipGetLastError();
}

// stats[2] += non-OK statuses, stats[3] = min(first non-OK record)
__global__ __launch_bounds__(256) void k_txlog_status_summary(uint64_t ntx, const int32_t *__restrict__ status,
                                                              unsigned long long *__restrict__ stats) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool bad = t < ntx && status[t] != MH_OK;
    const uint64_t m = __builtin_amdgcn_ballot_w64(bad);
    if (m && (threadIdx.x & 63) == 0) {
        const uint64_t w0 = t;  // the wave's first record (lane 0)
        atomicAdd(&stats[2], (unsigned long long)__builtin_popcountll(m));
        atomicMin(&stats[3], (unsigned long long)(w0 + __builtin_ctzll(m)));
    }
}

hipError_t launch_txlog_status_summary(hipStream_t st, uint64_t ntx, const int32_t *status,
                                       uint64_t *stats) {
    if (!ntx) return hipSuccess;
    hipLaunchKernelGGL(k_txlog_status_summary, dim3(grid_for(ntx, 256)), dim3(256), 0, st, ntx,
                       status, reinterpret_cast<unsigned long long *>(stats));
    return hipGetLastError();
}

}  // namespace mh
