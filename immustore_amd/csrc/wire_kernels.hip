// wire_kernels.hip -- proofs as protobuf messages, built on the device
// (wire formats; 8(f) row 3, DualProofV2 assembly).
//
// The gRPC server turns every proof into a message of pkg/api/schema/schema.proto
// (Go: pkg/api/schema/database_protoconv.go) and marshals it with protobuf-go.
// These kernels produce the same bytes directly from the device-resident tree:
//
//   InclusionProof  schema.proto:534-540   InclusionProofToProto  database_protoconv.go:115-121
//                   terms = (*HTree).InclusionProof(leaf)          htree.go:121-164
//   DualProofV2     schema.proto:437-445   DualProofV2ToProto     database_protoconv.go:152-159
//   TxHeader        schema.proto:349-367   TxHeaderToProto        database_protoconv.go:161-177
//   TxMetadata      schema.proto:380-383   TxMetadataToProto      database_protoconv.go:179-193
//                   proofs of ImmuStore.DualProofV2                immustore.go:2356-2387
//
// proto3 encoding as protobuf-go marshals generated messages: fields in field
// number order, scalar zero values and empty bytes omitted, sub-messages
// present whenever the Go pointer is non-nil, int32 / int64 negatives as
// 10-byte two's-complement varints.  Every tag here is one byte (field < 16).
//
// Two passes: k_pb_*_size (one lane per message: status + byte size, no
// memory reads beyond the headers), an inclusive scan of the sizes (hipcub)
// into off[1..n], then k_pb_*_write (one wave per message: lane 0 encodes the
// headers, lanes 1/2 walk the proofs into LDS index lists, all lanes gather
// the 32-byte terms into 34-byte records in LDS, then the wave streams the
// message out with consecutive byte stores).
#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "digest_io.hpp"
#include "mh_internal.hpp"
#include "proof_walk.hpp"

namespace mh {

constexpr int kPbMaxMsg = 8192;     // >= 2 x 433 B headers + (63 + 127) x 34 B terms
constexpr int kPbMaxIncl = 64;      // ahtree / htree inclusion proof terms (tree < 2^63)
constexpr int kPbMaxCons = 128;     // ahtree consistency proof terms
constexpr uint64_t kPbGrid = 1u << 16;  // writer workgroups (one wave each), grid-stride

__device__ __forceinline__ uint32_t vlen(uint64_t v) {
    return v ? (uint32_t)((63 - __clzll(v)) / 7 + 1) : 1u;
}
__device__ __forceinline__ uint32_t put_varint(uint8_t *p, uint64_t v) {
    uint32_t k = 0;
    while (v >= 0x80) {
        p[k++] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    p[k++] = (uint8_t)v;
    return k;
}
// int32 field value as protobuf-go encodes it (sign-extended to 64 bits)
__device__ __forceinline__ uint64_t i32v(uint32_t x) { return (uint64_t)(int64_t)(int32_t)x; }

// ------------------------------------------------------------ TxHeader
// TxMetadata.ReadFrom (tx_metadata.go:159-195) of the stored bytes, then
// TxMetadataToProto: truncatedTxID (attribute 0, BE64) and extra (attribute
// 1, BE16 length + bytes); a later attribute of the same code replaces an
// earlier one (Go map assignment).
struct PbHdr {
    uint32_t body = 0;      // TxHeader message length
    uint32_t md_body = 0;   // TxMetadata message length
    uint64_t trunc = 0;
    uint32_t extra_off = 0, extra_len = 0;
    bool has_md = false;
    int32_t st = MH_OK;
};

__device__ inline PbHdr pb_header(const MhTxHeader &h, const uint8_t *md_blob) {
    PbHdr r;
    if (h.md_len) {  // tx.go:483-501: mdLen == 0 leaves Metadata nil
        r.has_md = true;
        if (h.md_len > MH_MAX_TX_METADATA_LEN) {
            r.st = MH_ERR_CORRUPTED_DATA;
            return r;
        }
        const uint8_t *b = md_blob + h.md_off;
        uint32_t i = 0;
        while (i < h.md_len) {
            const uint8_t code = b[i++];
            if (code == 0) {
                if (h.md_len - i < 8) { r.st = MH_ERR_CORRUPTED_DATA; return r; }
                uint64_t v = 0;
                for (int k = 0; k < 8; k++) v = v << 8 | b[i + k];
                r.trunc = v;
                i += 8;
            } else if (code == 1) {
                if (h.md_len - i < 2) { r.st = MH_ERR_CORRUPTED_DATA; return r; }
                const uint32_t L = (uint32_t)b[i] << 8 | b[i + 1];
                if (h.md_len - i - 2 < L) { r.st = MH_ERR_CORRUPTED_DATA; return r; }
                r.extra_off = h.md_off + i + 2;
                r.extra_len = L;
                i += 2 + L;
            } else {
                r.st = MH_ERR_CORRUPTED_DATA;
                return r;
            }
        }
        if (r.trunc) r.md_body += 1 + vlen(r.trunc);
        if (r.extra_len) r.md_body += 1 + vlen(r.extra_len) + r.extra_len;
    }
    uint32_t s = 0;
    if (h.id) s += 1 + vlen(h.id);
    s += 34;                                            // prevAlh
    if (h.ts) s += 1 + vlen((uint64_t)h.ts);
    if (h.nentries) s += 1 + vlen(i32v(h.nentries));
    s += 34;                                            // eH
    if (h.bl_tx_id) s += 1 + vlen(h.bl_tx_id);
    s += 34;                                            // blRoot
    if (h.version) s += 1 + vlen(i32v(h.version));
    if (r.has_md) s += 1 + vlen(r.md_body) + r.md_body;
    r.body = s;
    return r;
}

__device__ inline uint32_t put_bytes32(uint8_t *p, uint8_t tag, const uint8_t *d) {
    p[0] = tag;
    p[1] = 32;
    for (int k = 0; k < 32; k++) p[2 + k] = d[k];
    return 34;
}

// TxHeader as field `tag` of the enclosing message; returns bytes written
__device__ inline uint32_t put_header(uint8_t *p, uint8_t tag, const MhTxHeader &h,
                                      const PbHdr &r, const uint8_t *md_blob) {
    uint32_t k = 0;
    p[k++] = tag;
    k += put_varint(p + k, r.body);
    if (h.id) { p[k++] = 0x08; k += put_varint(p + k, h.id); }
    k += put_bytes32(p + k, 0x12, h.prev_alh);
    if (h.ts) { p[k++] = 0x18; k += put_varint(p + k, (uint64_t)h.ts); }
    if (h.nentries) { p[k++] = 0x20; k += put_varint(p + k, i32v(h.nentries)); }
    k += put_bytes32(p + k, 0x2a, h.eh);
    if (h.bl_tx_id) { p[k++] = 0x30; k += put_varint(p + k, h.bl_tx_id); }
    k += put_bytes32(p + k, 0x3a, h.bl_root);
    if (h.version) { p[k++] = 0x40; k += put_varint(p + k, i32v(h.version)); }
    if (r.has_md) {
        p[k++] = 0x4a;
        k += put_varint(p + k, r.md_body);
        if (r.trunc) { p[k++] = 0x08; k += put_varint(p + k, r.trunc); }
        if (r.extra_len) {
            p[k++] = 0x12;
            k += put_varint(p + k, r.extra_len);
            for (uint32_t q = 0; q < r.extra_len; q++) p[k++] = md_blob[r.extra_off + q];
        }
    }
    return k;
}

__device__ __forceinline__ uint32_t framed(uint32_t body) { return 1 + vlen(body) + body; }

// ------------------------------------------------------------ DualProofV2
// ImmuStore.DualProofV2 (immustore.go:2356-2387) checks and proof bounds.
struct PbDual {
    PbHdr s, t;
    uint64_t ii = 0, ij = 0, ci = 0;  // InclusionProof(ii, ij), ConsistencyProof(ci, ij)
    bool proofs = false;
    int32_t st = MH_OK;
};

__device__ inline PbDual pb_dual(const MhTxHeader &src, const MhTxHeader &tgt,
                                 const uint8_t *md_blob, uint64_t size) {
    PbDual d;
    if (src.id == 0) { d.st = MH_ERR_ILLEGAL_ARGUMENTS; return d; }
    if (src.id > tgt.id) { d.st = MH_ERR_SOURCE_TX_NEWER; return d; }
    if (src.id - 1 != src.bl_tx_id || tgt.id - 1 != tgt.bl_tx_id) {
        d.st = MH_ERR_UNEXPECTED_LINKING;
        return d;
    }
    if (src.id < tgt.id) {
        d.proofs = true;
        d.ii = src.id;
        d.ij = tgt.bl_tx_id;
        d.ci = src.bl_tx_id > 1 ? src.bl_tx_id : 1;  // maxUint64(1, sourceTxHdr.BlTxID)
        // (*AHtree).InclusionProof / ConsistencyProof (ahtree.go:525-545, 579-597):
        // i <= j holds here; j beyond the tree is ErrUnexistentData
        if (d.ij > size) { d.st = MH_ERR_UNEXISTENT_DATA; return d; }
    }
    d.s = pb_header(src, md_blob);
    if (d.s.st) { d.st = d.s.st; return d; }
    d.t = pb_header(tgt, md_blob);
    if (d.t.st) { d.st = d.t.st; return d; }
    return d;
}

__global__ __launch_bounds__(256) void k_pb_dual_size(const uint8_t *__restrict__ dlog, uint64_t size,
                                                      uint64_t n, const MhTxHeader *__restrict__ src,
                                                      const MhTxHeader *__restrict__ tgt,
                                                      const uint8_t *__restrict__ md_blob,
                                                      uint64_t *__restrict__ sizes,
                                                      int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const PbDual d = pb_dual(src[p], tgt[p], md_blob, size);
    uint64_t s = 0;
    int32_t st = d.st;
    if (!st) {
        uint32_t ni = 0, nc = 0;
        if (d.proofs) {
            ni = ahtree_walk(false, d.ii, d.ij, [](uint32_t, uint64_t) {});
            nc = ahtree_walk(true, d.ci, d.ij, [](uint32_t, uint64_t) {});
        }
        s = framed(d.s.body) + framed(d.t.body) + 34ull * (ni + nc);
        if (ni > kPbMaxIncl || nc > kPbMaxCons || s > kPbMaxMsg) {
            st = MH_ERR_ILLEGAL_ARGUMENTS;
            s = 0;
        }
    }
    sizes[p] = s;
    status[p] = st;
}

// Gather the terms named by idx (walk order) into 34-byte records at buf+pre:
// record t holds node idx[cnt-1-t] (Go prepends, proof_walk.hpp).
__device__ __forceinline__ void pb_records(uint8_t *buf, uint32_t pre, uint8_t tag,
                                           const uint64_t *idx, uint32_t cnt,
                                           const uint8_t *__restrict__ nodes, int lane) {
    for (uint32_t t = lane; t < cnt; t += 64) {
        const uint4 *s = reinterpret_cast<const uint4 *>(nodes + idx[cnt - 1 - t] * 32);
        const uint4 a = s[0], b = s[1];
        uint8_t *r = buf + pre + 34 * t;
        r[0] = tag;
        r[1] = 32;
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 8; k++) {
            r[2 + 4 * k] = (uint8_t)w[k];
            r[3 + 4 * k] = (uint8_t)(w[k] >> 8);
            r[4 + 4 * k] = (uint8_t)(w[k] >> 16);
            r[5 + 4 * k] = (uint8_t)(w[k] >> 24);
        }
    }
}

// The wave streams its LDS message out: dword stores for the 4-aligned body,
// bytes for the ends.
__device__ __forceinline__ void pb_flush(uint8_t *__restrict__ out, const uint8_t *buf,
                                         uint32_t len, int lane) {
    const uint32_t head = (uint32_t)((4 - ((uintptr_t)out & 3)) & 3);
    const uint32_t h = head < len ? head : len;
    if ((uint32_t)lane < h) out[lane] = buf[lane];
    const uint32_t nw = (len - h) / 4;
    uint32_t *o32 = reinterpret_cast<uint32_t *>(out + h);
    for (uint32_t k = lane; k < nw; k += 64) {
        const uint8_t *b = buf + h + 4 * k;
        o32[k] = (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
    }
    for (uint32_t k = h + 4 * nw + lane; k < len; k += 64) out[k] = buf[k];
}

__global__ __launch_bounds__(64) void k_pb_dual_write(const uint8_t *__restrict__ dlog, uint64_t size,
                                                      uint64_t n, const MhTxHeader *__restrict__ src,
                                                      const MhTxHeader *__restrict__ tgt,
                                                      const uint8_t *__restrict__ md_blob,
                                                      const uint64_t *__restrict__ off,
                                                      uint8_t *__restrict__ out, uint64_t out_cap,
                                                      int32_t *__restrict__ status) {
    __shared__ uint8_t buf[kPbMaxMsg];
    __shared__ uint64_t idx_i[kPbMaxIncl], idx_c[kPbMaxCons];
    __shared__ uint32_t s_pre, s_ni, s_nc;
    const int lane = threadIdx.x;
    for (uint64_t p = blockIdx.x; p < n; p += gridDim.x) {  // uniform per workgroup
        if (status[p] != MH_OK) continue;
        const uint64_t o = off[p], len = off[p + 1] - o;
        if (off[p + 1] > out_cap) {
            if (lane == 0) status[p] = MH_ERR_BUFFER_TOO_SMALL;
            continue;
        }
        const MhTxHeader &S = src[p], &T = tgt[p];
        if (lane == 0) {
            const PbDual d = pb_dual(S, T, md_blob, size);
            uint32_t k = put_header(buf, 0x0a, S, d.s, md_blob);
            k += put_header(buf + k, 0x12, T, d.t, md_blob);
            s_pre = k;
        } else if (lane == 1 || lane == 2) {
            uint32_t c = 0;
            if (S.id < T.id) {
                if (lane == 1)
                    c = ahtree_walk(false, S.id, T.bl_tx_id,
                                    [&](uint32_t q, uint64_t x) { idx_i[q] = x; });
                else
                    c = ahtree_walk(true, S.bl_tx_id > 1 ? S.bl_tx_id : 1, T.bl_tx_id,
                                    [&](uint32_t q, uint64_t x) { idx_c[q] = x; });
            }
            if (lane == 1) s_ni = c; else s_nc = c;
        }
        __syncthreads();
        const uint32_t pre = s_pre, ni = s_ni, nc = s_nc;
        pb_records(buf, pre, 0x1a, idx_i, ni, dlog, lane);
        pb_records(buf, pre + 34 * ni, 0x22, idx_c, nc, dlog, lane);
        __syncthreads();
        pb_flush(out + o, buf, (uint32_t)len, lane);
        __syncthreads();  // buf / s_* are rewritten by the next message
    }
}

// ------------------------------------------------------------ InclusionProof (htree)
__device__ __forceinline__ uint32_t pb_incl_prefix(uint64_t leaf, uint64_t w) {
    // Leaf: int32(iproof.Leaf), Width: int32(iproof.Width)
    const uint32_t l = (uint32_t)leaf, ww = (uint32_t)w;
    return (l ? 1 + vlen(i32v(l)) : 0) + (ww ? 1 + vlen(i32v(ww)) : 0);
}

__global__ __launch_bounds__(256) void k_pb_incl_size(uint64_t w, uint64_t n,
                                                      const uint64_t *__restrict__ leaf,
                                                      uint64_t *__restrict__ sizes,
                                                      int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t i = leaf[p];
    if (i >= w) {  // htree.go:122-124
        sizes[p] = 0;
        status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
        return;
    }
    const uint32_t c = htree_walk(i, w, [](uint32_t, uint64_t) {});
    sizes[p] = pb_incl_prefix(i, w) + 34ull * c;
    status[p] = MH_OK;
}

__global__ __launch_bounds__(64) void k_pb_incl_write(const uint8_t *__restrict__ levels, uint64_t w,
                                                      uint64_t n, const uint64_t *__restrict__ leaf,
                                                      const uint64_t *__restrict__ off,
                                                      uint8_t *__restrict__ out, uint64_t out_cap,
                                                      int32_t *__restrict__ status) {
    __shared__ uint8_t buf[16 + 34 * kPbMaxIncl];
    __shared__ uint64_t idx[kPbMaxIncl];
    __shared__ uint32_t s_pre, s_c;
    const int lane = threadIdx.x;
    for (uint64_t p = blockIdx.x; p < n; p += gridDim.x) {
        if (status[p] != MH_OK) continue;
        const uint64_t o = off[p], len = off[p + 1] - o;
        if (off[p + 1] > out_cap) {
            if (lane == 0) status[p] = MH_ERR_BUFFER_TOO_SMALL;
            continue;
        }
        const uint64_t i = leaf[p];
        if (lane == 0) {
            uint32_t k = 0;
            if ((uint32_t)i) { buf[k++] = 0x08; k += put_varint(buf + k, i32v((uint32_t)i)); }
            if ((uint32_t)w) { buf[k++] = 0x10; k += put_varint(buf + k, i32v((uint32_t)w)); }
            s_pre = k;
            s_c = htree_walk(i, w, [&](uint32_t q, uint64_t x) { idx[q] = x; });
        }
        __syncthreads();
        pb_records(buf, s_pre, 0x1a, idx, s_c, levels, lane);
        __syncthreads();
        pb_flush(out + o, buf, (uint32_t)len, lane);
        __syncthreads();
    }
}

// ------------------------------------------------------------ launchers
size_t pb_scan_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const uint64_t *)nullptr,
                                     (uint64_t *)nullptr, (int)(n ? n : 1), (hipStream_t)0);
    return bytes;
}

uint64_t pb_scratch_bytes(uint64_t n) {
    return ((n * 8 + 255) & ~255ull) + ((pb_scan_temp_bytes(n) + 255) & ~255ull) + 256;
}

// sizes -> off[0..n] (off[0] = 0)
static hipError_t pb_offsets(hipStream_t st, uint64_t n, const uint64_t *sizes, uint64_t *off,
                             uint8_t *temp) {
    if (hipError_t e = hipMemsetAsync(off, 0, sizeof(uint64_t), st)) return e;
    size_t bytes = pb_scan_temp_bytes(n);
    return hipcub::DeviceScan::InclusiveSum(temp, bytes, sizes, off + 1, (int)n, st);
}

static inline unsigned grid_for(uint64_t threads, unsigned block) {
    return (unsigned)((threads + block - 1) / block);
}

hipError_t launch_pb_dual_v2(hipStream_t st, Timer *tm, int phase, const uint8_t *dlog,
                             uint64_t size, uint64_t n, const MhTxHeader *src,
                             const MhTxHeader *tgt, const uint8_t *md_blob, uint8_t *out,
                             uint64_t out_cap, uint64_t *off, int32_t *status, uint8_t *scratch) {
    if (!n) return hipMemsetAsync(off, 0, sizeof(uint64_t), st);
    uint64_t *sizes = reinterpret_cast<uint64_t *>(scratch);
    uint8_t *temp = scratch + ((n * 8 + 255) & ~255ull);
    if (phase & 1) {
        TimerScope ts(tm, "pb_dual_size", st);
        hipLaunchKernelGGL(k_pb_dual_size, dim3(grid_for(n, 256)), dim3(256), 0, st, dlog, size, n,
                           src, tgt, md_blob, sizes, status);
        if (hipError_t e = hipGetLastError()) return e;
        if (hipError_t e = pb_offsets(st, n, sizes, off, temp)) return e;
    }
    if (phase & 2) {
        TimerScope ts(tm, "pb_dual_write", st);
        hipLaunchKernelGGL(k_pb_dual_write, dim3((unsigned)std::min<uint64_t>(n, kPbGrid)), dim3(64), 0, st, dlog, size, n, src,
                           tgt, md_blob, off, out, out_cap, status);
        if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
}

hipError_t launch_pb_inclusion(hipStream_t st, Timer *tm, int phase, const uint8_t *levels,
                               uint64_t w, uint64_t n, const uint64_t *leaf, uint8_t *out,
                               uint64_t out_cap, uint64_t *off, int32_t *status, uint8_t *scratch) {
    if (!n) return hipMemsetAsync(off, 0, sizeof(uint64_t), st);
    uint64_t *sizes = reinterpret_cast<uint64_t *>(scratch);
    uint8_t *temp = scratch + ((n * 8 + 255) & ~255ull);
    if (phase & 1) {
        TimerScope ts(tm, "pb_incl_size", st);
        hipLaunchKernelGGL(k_pb_incl_size, dim3(grid_for(n, 256)), dim3(256), 0, st, w, n, leaf,
                           sizes, status);
        if (hipError_t e = hipGetLastError()) return e;
        if (hipError_t e = pb_offsets(st, n, sizes, off, temp)) return e;
    }
    if (phase & 2) {
        TimerScope ts(tm, "pb_incl_write", st);
        hipLaunchKernelGGL(k_pb_incl_write, dim3((unsigned)std::min<uint64_t>(n, kPbGrid)), dim3(64), 0, st, levels, w, n, leaf,
                           off, out, out_cap, status);
        if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
}

}  // namespace mh
