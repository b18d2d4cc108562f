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
// Two passes, one lane per message: k_pb_*_size (status, byte size and term
// counts; no memory reads beyond the headers), an inclusive scan of the sizes
// (hipcub) into off[1..n], then k_pb_*_write (headers streamed through a
// register-staged ByteWriter as dword stores; the 34-byte term records built
// per round in LDS and written by the whole wave, staged_records).  Measured
// on MI355X, 10^6 DualProofV2 over a 2^24-append tree: one wave per message
// doing the walks and header encoding itself, 25 ms (64x the serial index
// math); index lists stored by the size pass + one wave per message
// materialising dwords, 8.1 ms; one lane per message storing its own records,
// 4.5 ms (64 scattered lines per store); records staged per wave, 4 per lane
// per round, 3.0 ms (8 per round: 3.7 ms, LDS occupancy; 2: 4.0 ms, flush
// overhead).
#include <algorithm>
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#include "digest_io.hpp"
#include "mh_internal.hpp"
#include "proof_walk.hpp"

namespace mh {


__device__ __forceinline__ uint32_t vlen(uint64_t v) {
    return v ? (uint32_t)((63 - __clzll(v)) / 7 + 1) : 1u;
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
                                                      uint32_t *__restrict__ cnt,
                                                      int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const PbDual d = pb_dual(src[p], tgt[p], md_blob, size);
    uint64_t s = 0;
    uint32_t ni = 0, nc = 0;
    if (!d.st) {
        if (d.proofs) {
            ni = ahtree_walk(false, d.ii, d.ij, [](uint32_t, uint64_t) {});
            nc = ahtree_walk(true, d.ci, d.ij, [](uint32_t, uint64_t) {});
        }
        s = framed(d.s.body) + framed(d.t.body) + 34ull * (ni + nc);
    }
    sizes[p] = s;
    cnt[2 * p] = ni;
    cnt[2 * p + 1] = nc;
    status[p] = d.st;
}

// ------------------------------------------------------------ byte streams
// One lane writes one message.  Bytes collect in a 32-bit register and leave
// as dword stores; only the partial words at the two ends of a run (shared
// with the neighbouring messages / records) are written byte by byte.
// global-memory pointer types: stores through them are global_* rather than
// flat_* (a pointer rebuilt from an integer or read from LDS is generic)
typedef __attribute__((address_space(1))) uint8_t g8;
typedef __attribute__((address_space(1))) uint32_t g32;

struct ByteWriter {
    g32 *w;            // dword that receives the pending bytes
    uint32_t acc = 0;  // pending bytes, little-endian
    uint32_t fill;     // bytes already in *w's slot (pending or not ours)
    uint32_t lo;       // first byte of the current word that is ours
    __device__ explicit ByteWriter(uint8_t *p)
        : w((g32 *)((g8 *)p - ((uintptr_t)p & 3))),
          fill((uint32_t)((uintptr_t)p & 3)), lo((uint32_t)((uintptr_t)p & 3)) {}
    __device__ __forceinline__ void flush_word() {  // fill == 4
        if (lo == 0) {
            *w = acc;
        } else {
            g8 *b = (g8 *)w;
            for (uint32_t k = lo; k < 4; k++) b[k] = (uint8_t)(acc >> (8 * k));
            lo = 0;
        }
        w++;
        acc = 0;
        fill = 0;
    }
    __device__ __forceinline__ void put8(uint32_t b) {
        acc |= (b & 0xff) << (8 * fill);
        if (++fill == 4) flush_word();
    }
    // 4 bytes, little-endian in x (a word as loaded from memory)
    __device__ __forceinline__ void put32(uint32_t x) {
        if (fill == 0) {
            acc = x;
            fill = 4;
            flush_word();
        } else {
            const uint32_t sh = 8 * fill;
            acc |= x << sh;
            const uint32_t rest = x >> (32 - sh);
            fill = 4;
            flush_word();
            acc = rest;
            fill = sh / 8;
        }
    }
    __device__ __forceinline__ void varint(uint64_t v) {
        while (v >= 0x80) {
            put8((uint32_t)(v | 0x80));
            v >>= 7;
        }
        put8((uint32_t)v);
    }
    __device__ __forceinline__ void finish() {  // the trailing partial word
        g8 *b = (g8 *)w;
        for (uint32_t k = lo; k < fill; k++) b[k] = (uint8_t)(acc >> (8 * k));
    }
    __device__ __forceinline__ uint8_t *pos() const { return (uint8_t *)((g8 *)w + fill); }
};

// A 34-byte field `tag, 32, d[0..31]` (repeated-bytes term or a header
// digest) at any alignment without divergent branches: the record is built
// as 9 little-endian words, funnel-shifted to the destination alignment a,
// and stored as 7-8 dwords plus predicated byte / short stores for the
// partial words at the two ends (a = 0: -/short, 1: byte+short/short+byte,
// 2: short/-, 3: byte/byte).
template <int AS>  // address space of the destination: 0 generic, 1 global
__device__ __forceinline__ void put_rec34_as(uint8_t *pg, uint32_t tag, const uint32_t d[8]) {
    typedef __attribute__((address_space(AS))) uint8_t b8;
    typedef __attribute__((address_space(AS))) uint16_t b16;
    typedef __attribute__((address_space(AS))) uint32_t b32;
    b8 *p = (b8 *)pg;
    uint32_t r[10];
    r[0] = (tag & 0xff) | (32u << 8) | (d[0] << 16);
#pragma unroll
    for (int k = 1; k < 8; k++) r[k] = (d[k - 1] >> 16) | (d[k] << 16);
    r[8] = d[7] >> 16;
    r[9] = 0;
    const uint32_t a = (uint32_t)((uintptr_t)p & 3);
    b32 *w = (b32 *)(p - a);
    uint32_t o[10];
    o[0] = r[0] << (8 * a);
#pragma unroll
    for (int j = 1; j < 10; j++)
        o[j] = a ? __builtin_amdgcn_alignbyte(r[j], r[j - 1], 4 - a) : r[j];
    b8 *wb = (b8 *)w;
    // word 0: ours from byte a
    if (a == 0) w[0] = o[0];
    if (a & 1) wb[a] = (uint8_t)(o[0] >> (8 * a));
    if (a == 1 || a == 2) *(b16 *)(wb + 2) = (uint16_t)(o[0] >> 16);
#pragma unroll
    for (int j = 1; j < 8; j++) w[j] = o[j];
    // word 8: ours up to byte a + 34 - 32
    if (a >= 2) w[8] = o[8];
    if (a <= 1) *(b16 *)(wb + 32) = (uint16_t)o[8];
    if (a == 1) wb[34] = (uint8_t)(o[8] >> 16);
    if (a == 3) wb[36] = (uint8_t)o[9];
}

__device__ __forceinline__ void put_rec34(uint8_t *p, uint32_t tag, const uint32_t d[8]) {
    put_rec34_as<0>(p, tag, d);
}

// 32-byte digest field (tag, length 32, bytes; d 8-byte aligned): the byte
// stream is closed, the field stored by put_rec34 and the stream reopened.
__device__ __forceinline__ void put_digest(ByteWriter &bw, uint32_t tag, const uint8_t *d) {
    const uint2 *q = reinterpret_cast<const uint2 *>(d);
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint2 v = q[k];
        x[2 * k] = v.x;
        x[2 * k + 1] = v.y;
    }
    bw.finish();
    uint8_t *p = bw.pos();
    put_rec34_as<1>(p, tag, x);
    bw = ByteWriter(p + 34);
}

// TxHeader as field `tag` of the enclosing message
__device__ inline void put_header(ByteWriter &bw, uint32_t tag, const MhTxHeader &h,
                                  const PbHdr &r, const uint8_t *md_blob) {
    bw.put8(tag);
    bw.varint(r.body);
    if (h.id) { bw.put8(0x08); bw.varint(h.id); }
    put_digest(bw, 0x12, h.prev_alh);
    if (h.ts) { bw.put8(0x18); bw.varint((uint64_t)h.ts); }
    if (h.nentries) { bw.put8(0x20); bw.varint(i32v(h.nentries)); }
    put_digest(bw, 0x2a, h.eh);
    if (h.bl_tx_id) { bw.put8(0x30); bw.varint(h.bl_tx_id); }
    put_digest(bw, 0x3a, h.bl_root);
    if (h.version) { bw.put8(0x40); bw.varint(i32v(h.version)); }
    if (r.has_md) {
        bw.put8(0x4a);
        bw.varint(r.md_body);
        if (r.trunc) { bw.put8(0x08); bw.varint(r.trunc); }
        if (r.extra_len) {
            bw.put8(0x12);
            bw.varint(r.extra_len);
            for (uint32_t q = 0; q < r.extra_len; q++) bw.put8(md_blob[r.extra_off + q]);
        }
    }
}

// ------------------------------------------------------------ staged term records
// Each lane owns one message, but its term records leave through LDS: per
// round a lane builds up to kRpr records of its walk in its LDS slot -- in
// message order, at the byte alignment of their global destination -- and
// then the wave writes every lane's span (up to 272 contiguous bytes) with
// all 64 lanes storing consecutive dwords.  One message per lane keeps the
// serial index walks parallel; the staging turns 64 scattered lines per
// store instruction into 2-3 contiguous ones.
#ifndef MH_PB_RPR
#define MH_PB_RPR 4  // A/B (tools/pb_ab.sh): 4 beats 8 (LDS occupancy) and 2 (flush overhead)
#endif
constexpr uint32_t kRpr = MH_PB_RPR;  // records per lane per round
constexpr uint32_t kSlotBytes = (3 + kRpr * 34 + 15) / 16 * 16;  // + alignment bytes, 16-byte rows

__device__ __forceinline__ void load_node(const uint8_t *node, uint32_t x[8]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(node);  // 32-byte nodes, 16-byte aligned
    const uint4 a = q[0], b = q[1];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
    x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}

// Records q = 0 .. cnt-1 of the walk `gen` (walk order) go to
// rec_base + 34 * (cnt - 1 - q) (proof order, proof_walk.hpp).  Wave-uniform
// control flow: every lane of the wave calls this (inactive lanes with cnt 0).
// A walk that ends before `cnt` terms (the size pass and the writer would
// disagree -- never seen, the two forms are tested against each other) reads
// node 0 instead of faulting and sets *bad.
template <class Gen>
__device__ __forceinline__ void staged_records(uint8_t *rec_base, uint32_t cnt, uint32_t tag,
                                               Gen &gen, const uint8_t *__restrict__ nodes,
                                               uint8_t *wave_lds, int lane, bool *bad) {
    uint8_t *slot = wave_lds + lane * kSlotBytes;
    uint32_t done = 0;
    while (__any(done < cnt)) {
        const uint32_t cr = done < cnt ? min(kRpr, cnt - done) : 0;
        uint8_t *g = rec_base + 34ull * (cnt - done - cr);  // span start (message order)
        const uint32_t a = (uint32_t)((uintptr_t)g & 3);
        // gather in pairs (two node loads in flight), build in LDS
        for (uint32_t k = 0; k < cr; k += 2) {
            uint32_t x[8], y[8];
            uint64_t n0 = gen.next();
            uint64_t n1 = k + 1 < cr ? gen.next() : n0;
            if (n0 == ~0ull || n1 == ~0ull) {
                *bad = true;
                n0 = n1 = 0;
            }
            load_node(nodes + n0 * 32, x);
            load_node(nodes + n1 * 32, y);
            put_rec34(slot + a + 34 * (cr - 1 - k), tag, x);
            if (k + 1 < cr) put_rec34(slot + a + 34 * (cr - 2 - k), tag, y);
        }
        done += cr;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
        __builtin_amdgcn_wave_barrier();
        const uint64_t ga = (uint64_t)(uintptr_t)g;
        const uint32_t len = 34 * cr;
        for (int sl = 0; sl < 64; sl++) {  // span of lane sl, read with v_readlane (scalar)
            const uint32_t ls = (uint32_t)__builtin_amdgcn_readlane((int)len, sl);
            if (!ls) continue;
            const uint64_t gs =
                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ga >> 32), sl) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ga, sl);
            const uint32_t as = (uint32_t)(gs & 3);
            const uint32_t nd = (as + ls + 3) / 4;
            g32 *gw = (g32 *)(uintptr_t)(gs - as);
            const uint32_t *lw = reinterpret_cast<const uint32_t *>(wave_lds + sl * kSlotBytes);
            for (uint32_t d = lane; d < nd; d += 64) {
                const uint32_t lo = d == 0 ? as : 0;
                const uint32_t hi = min(4u, as + ls - 4 * d);
                const uint32_t v = lw[d];
                if (lo == 0 && hi == 4) {
                    gw[d] = v;
                } else {
                    g8 *gb = (g8 *)(gw + d);
                    for (uint32_t e = lo; e < hi; e++) gb[e] = (uint8_t)(v >> (8 * e));
                }
            }
        }
        __builtin_amdgcn_wave_barrier();  // every span is out before the slots are rebuilt
    }
}

// ------------------------------------------------------------ wave-dense term records
// The records of a wave's 64 messages written record-parallel: each lane
// walks its own proof (the loop form, proof_walk.hpp) into an LDS index list
// -- the lists of the wave back to back, at the wave's exclusive prefix of the
// term counts -- and then the wave writes the flattened records with one
// lane per 34-byte record, consecutive records on consecutive lanes, two
// records per lane in flight.  Node indices are 32-bit: the host takes this
// path only when the tree has fewer than 2^32 nodes (else staged_records).
// Lists that do not fit kIdxCap go in chunks of whole messages.
#ifndef MH_PB_IDXCAP
#define MH_PB_IDXCAP 4096
#endif
constexpr uint32_t kIdxCap = MH_PB_IDXCAP;
#ifndef MH_PB_UNROLL
#define MH_PB_UNROLL 2
#endif
constexpr uint32_t kPbUnroll = MH_PB_UNROLL;  // records per lane in flight
static_assert(kIdxCap >= 256, "a message's list (<= 130 terms) must fit a chunk");
struct WaveRecLds {
    uint32_t idx[kIdxCap];
    uint32_t pre[65];
    uint64_t base[64];
};

// walk(emit) runs the loop-form walk of the calling lane and returns its term
// count; emit(q, node) gets the terms in walk order (proof position cnt-1-q).
// Called by the whole wave (blockDim 64); lanes without records pass cnt 0.
template <class Walk>
__device__ __forceinline__ void wave_records(uint8_t *rec_base, uint32_t cnt, uint32_t tag,
                                             Walk &&walk, const uint8_t *__restrict__ nodes,
                                             WaveRecLds &L, int lane, bool *bad) {
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
        if (lane >= d) incl += y;
    }
    const uint32_t excl = incl - cnt;
    __syncthreads();  // a previous call's records are out of L
    L.pre[lane] = excl;
    if (lane == 63) L.pre[64] = incl;
    L.base[lane] = (uint64_t)(uintptr_t)rec_base;
    uint32_t m0 = 0;
    while (m0 < 64) {
        const uint32_t base0 = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)m0);
        const uint64_t fit = __ballot(lane >= (int)m0 && incl - base0 <= kIdxCap);
        const uint32_t m1 = m0 + max(1u, (uint32_t)__popcll(fit));
        const uint32_t T =
            min(kIdxCap, (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)(m1 - 1)) - base0);
        __syncthreads();  // the previous chunk's records are out of L.idx
        if ((uint32_t)lane >= m0 && (uint32_t)lane < m1 && cnt) {
            uint32_t *dst = L.idx + (excl - base0);
            const uint32_t c = walk([&](uint32_t q, uint64_t node) {
                if (q < cnt) dst[cnt - 1 - q] = (uint32_t)node;
            });
            if (c != cnt || cnt > kIdxCap) {  // size pass and writer disagree: never seen
                for (uint32_t k = 0; k < min(cnt, kIdxCap); k++) dst[k] = 0;
                *bad = true;
            }
        }
        __syncthreads();
        uint32_t m = m0;
        auto locate = [&](uint32_t r) {  // message of flattened record r (m only moves forward)
            while (m + 1 < m1 && L.pre[m + 1] - base0 <= r) m++;
            return m;
        };
        for (uint32_t r0 = 0; r0 < T; r0 += 64 * kPbUnroll) {
            uint32_t x[kPbUnroll][8];
            uint8_t *pr[kPbUnroll];
#pragma unroll
            for (uint32_t u = 0; u < kPbUnroll; u++) {  // kPbUnroll gathers in flight
                const uint32_t r = r0 + 64 * u + lane;
                pr[u] = nullptr;
                if (r < T) {
                    const uint32_t mr = locate(r);
                    pr[u] = reinterpret_cast<uint8_t *>(L.base[mr]) + 34ull * (r - (L.pre[mr] - base0));
                    load_node(nodes + (uint64_t)L.idx[r] * 32, x[u]);
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kPbUnroll; u++)
                if (pr[u]) put_rec34_as<1>(pr[u], tag, x[u]);  // global stores
        }
        m0 = m1;
    }
}

// DualProofV2 writer over wave_records: one wave per block, lane per message
// for the headers (ByteWriter) and the walks.
__global__ __launch_bounds__(64) void k_pb_dual_write_w(const uint8_t *__restrict__ dlog,
                                                        uint64_t size, uint64_t n,
                                                        const MhTxHeader *__restrict__ src,
                                                        const MhTxHeader *__restrict__ tgt,
                                                        const uint8_t *__restrict__ md_blob,
                                                        const uint64_t *__restrict__ off,
                                                        const uint32_t *__restrict__ cnt,
                                                        uint8_t *__restrict__ out, uint64_t out_cap,
                                                        int32_t *__restrict__ status) {
    __shared__ WaveRecLds L;
    const uint64_t p = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const int lane = threadIdx.x;
    bool active = p < n && status[p] == MH_OK;
    if (active && off[p + 1] > out_cap) {
        status[p] = MH_ERR_BUFFER_TOO_SMALL;
        active = false;
    }
    uint8_t *rec = out;
    uint32_t ni = 0, nc = 0;
    uint64_t ii = 1, ij = 1, ci = 1;
    if (active) {
        const MhTxHeader &S = src[p], &T = tgt[p];
        const PbDual d = pb_dual(S, T, md_blob, size);
        uint8_t *o = out + off[p];
        ByteWriter bw(o);
        put_header(bw, 0x0a, S, d.s, md_blob);
        put_header(bw, 0x12, T, d.t, md_blob);
        bw.finish();
        rec = o + framed(d.s.body) + framed(d.t.body);
        if (d.proofs) {
            ni = cnt[2 * p];
            nc = cnt[2 * p + 1];
            ii = d.ii;
            ij = d.ij;
            ci = d.ci;
        }
    }
    if (!__any(ni + nc > 0)) return;  // wave-uniform (one wave per block)
    bool bad = false;
    wave_records(rec, ni, 0x1a, [&](auto &&emit) { return ahtree_walk(false, ii, ij, emit); },
                 dlog, L, lane, &bad);
    wave_records(rec + 34ull * ni, nc, 0x22,
                 [&](auto &&emit) { return ahtree_walk(true, ci, ij, emit); }, dlog, L, lane, &bad);
    if (bad) status[p] = MH_ERR_ILLEGAL_STATE;
}

// One lane per message: header fields streamed from registers, term records
// staged per wave (staged_records).
__global__ __launch_bounds__(256) void k_pb_dual_write(const uint8_t *__restrict__ dlog, uint64_t size,
                                                       uint64_t n, const MhTxHeader *__restrict__ src,
                                                       const MhTxHeader *__restrict__ tgt,
                                                       const uint8_t *__restrict__ md_blob,
                                                       const uint64_t *__restrict__ off,
                                                       const uint32_t *__restrict__ cnt,
                                                       uint8_t *__restrict__ out, uint64_t out_cap,
                                                       int32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[256 * kSlotBytes];
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint8_t *wave_lds = lds + (threadIdx.x & ~63) * kSlotBytes;
    bool active = p < n && status[p] == MH_OK;
    if (active && off[p + 1] > out_cap) {
        status[p] = MH_ERR_BUFFER_TOO_SMALL;
        active = false;
    }
    uint8_t *rec = out;
    uint32_t ni = 0, nc = 0;
    uint64_t ii = 1, ij = 1, ci = 1;
    if (active) {
        const MhTxHeader &S = src[p], &T = tgt[p];
        const PbDual d = pb_dual(S, T, md_blob, size);
        uint8_t *o = out + off[p];
        ByteWriter bw(o);
        put_header(bw, 0x0a, S, d.s, md_blob);
        put_header(bw, 0x12, T, d.t, md_blob);
        bw.finish();
        rec = o + framed(d.s.body) + framed(d.t.body);
        if (d.proofs) {
            ni = cnt[2 * p];
            nc = cnt[2 * p + 1];
            ii = d.ii;
            ij = d.ij;
            ci = d.ci;
        }
    }
    if (!__any(ni + nc > 0)) return;  // wave-uniform from here on
    bool bad = false;
    AhtreeWalk gi(false, ii, ij);
    staged_records(rec, ni, 0x1a, gi, dlog, wave_lds, lane, &bad);
    AhtreeWalk gc(true, ci, ij);
    staged_records(rec + 34ull * ni, nc, 0x22, gc, dlog, wave_lds, lane, &bad);
    if (bad) status[p] = MH_ERR_ILLEGAL_STATE;
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
                                                      uint32_t *__restrict__ cnt,
                                                      int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t i = leaf[p];
    if (i >= w) {  // htree.go:122-124
        sizes[p] = 0;
        cnt[2 * p] = 0;
        status[p] = MH_ERR_ILLEGAL_ARGUMENTS;
        return;
    }
    const uint32_t c = htree_walk(i, w, [](uint32_t, uint64_t) {});
    sizes[p] = pb_incl_prefix(i, w) + 34ull * c;
    cnt[2 * p] = c;
    status[p] = MH_OK;
}

__global__ __launch_bounds__(256) void k_pb_incl_write(const uint8_t *__restrict__ levels, uint64_t w,
                                                       uint64_t n, const uint64_t *__restrict__ leaf,
                                                       const uint64_t *__restrict__ off,
                                                       const uint32_t *__restrict__ cnt,
                                                       uint8_t *__restrict__ out, uint64_t out_cap,
                                                       int32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[256 * kSlotBytes];
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint8_t *wave_lds = lds + (threadIdx.x & ~63) * kSlotBytes;
    bool active = p < n && status[p] == MH_OK;
    if (active && off[p + 1] > out_cap) {
        status[p] = MH_ERR_BUFFER_TOO_SMALL;
        active = false;
    }
    uint8_t *rec = out;
    uint32_t c = 0;
    uint64_t i = 0;
    if (active) {
        i = leaf[p];
        uint8_t *o = out + off[p];
        ByteWriter bw(o);
        if ((uint32_t)i) { bw.put8(0x08); bw.varint(i32v((uint32_t)i)); }
        if ((uint32_t)w) { bw.put8(0x10); bw.varint(i32v((uint32_t)w)); }
        bw.finish();
        rec = o + pb_incl_prefix(i, w);
        c = cnt[2 * p];
    }
    if (!__any(c > 0)) return;
    bool bad = false;
    HtreeWalk g(i, active ? w : 0);
    staged_records(rec, c, 0x1a, g, levels, wave_lds, lane, &bad);
    if (bad) status[p] = MH_ERR_ILLEGAL_STATE;
}

__global__ __launch_bounds__(64) void k_pb_incl_write_w(const uint8_t *__restrict__ levels,
                                                        uint64_t w, uint64_t n,
                                                        const uint64_t *__restrict__ leaf,
                                                        const uint64_t *__restrict__ off,
                                                        const uint32_t *__restrict__ cnt,
                                                        uint8_t *__restrict__ out, uint64_t out_cap,
                                                        int32_t *__restrict__ status) {
    __shared__ WaveRecLds L;
    __shared__ uint64_t loff[64];  // level_off(w, l): one table per block
    const uint64_t p = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const int lane = threadIdx.x;
    loff[lane] = level_off(w, lane);
    bool active = p < n && status[p] == MH_OK;
    if (active && off[p + 1] > out_cap) {
        status[p] = MH_ERR_BUFFER_TOO_SMALL;
        active = false;
    }
    uint8_t *rec = out;
    uint32_t c = 0;
    uint64_t i = 0;
    if (active) {
        i = leaf[p];
        uint8_t *o = out + off[p];
        ByteWriter bw(o);
        if ((uint32_t)i) { bw.put8(0x08); bw.varint(i32v((uint32_t)i)); }
        if ((uint32_t)w) { bw.put8(0x10); bw.varint(i32v((uint32_t)w)); }
        bw.finish();
        rec = o + pb_incl_prefix(i, w);
        c = cnt[2 * p];
    }
    if (!__any(c > 0)) return;
    bool bad = false;
    wave_records(rec, c, 0x1a,
                 [&](auto &&emit) {
                     return htree_walk_lo(i, w, [&](int l) { return loff[l]; }, emit);
                 },
                 levels, L, lane, &bad);
    if (bad) status[p] = MH_ERR_ILLEGAL_STATE;
}

// ------------------------------------------------------------ launchers
size_t pb_scan_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const uint64_t *)nullptr,
                                     (uint64_t *)nullptr, (int)(n ? n : 1), (hipStream_t)0);
    return bytes;
}

// scratch: sizes[n] (u64) | term counts[2n] (u32) | scan temp
uint64_t pb_scratch_bytes(uint64_t n) {
    return 2 * ((n * 8 + 255) & ~255ull) + ((pb_scan_temp_bytes(n) + 255) & ~255ull) + 256;
}

// in[0..n) -> out[0..n] with out[0] = 0, out[k+1] = in[0] + ... + in[k]
hipError_t scan_offsets_u64(hipStream_t st, uint64_t n, const uint64_t *in, uint64_t *out,
                            uint8_t *temp) {
    if (hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), st)) return e;
    if (!n) return hipSuccess;
    size_t bytes = pb_scan_temp_bytes(n);
    return hipcub::DeviceScan::InclusiveSum(temp, bytes, in, out + 1, (int)n, st);
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

// MH_PB_STAGED=1 in the environment (read per launch) forces the staged
// writers, the path of trees with >= 2^32 nodes, so the tests cover both.
static bool pb_force_staged() {
    const char *e = getenv("MH_PB_STAGED");
    return e && e[0] == '1';
}

hipError_t launch_pb_dual_v2(hipStream_t st, Timer *tm, int phase, const uint8_t *dlog,
                             uint64_t size, uint64_t n, const MhTxHeader *src,
                             const MhTxHeader *tgt, const uint8_t *md_blob, uint8_t *out,
                             uint64_t out_cap, uint64_t *off, int32_t *status, uint8_t *scratch) {
    if (!n) return hipMemsetAsync(off, 0, sizeof(uint64_t), st);
    uint64_t *sizes = reinterpret_cast<uint64_t *>(scratch);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(scratch + ((n * 8 + 255) & ~255ull));
    uint8_t *temp = scratch + 2 * ((n * 8 + 255) & ~255ull);
    if (phase & 1) {
        TimerScope ts(tm, "pb_dual_size", st);
        hipLaunchKernelGGL(k_pb_dual_size, dim3(grid_for(n, 256)), dim3(256), 0, st, dlog, size, n,
                           src, tgt, md_blob, sizes, cnt, status);
        if (hipError_t e = hipGetLastError()) return e;
        if (hipError_t e = pb_offsets(st, n, sizes, off, temp)) return e;
    }
    if (phase & 2) {
        TimerScope ts(tm, "pb_dual_write", st);
        if (ahtree_nodes_upto(size) < (1ull << 32) && !pb_force_staged())  // 32-bit node indices
            hipLaunchKernelGGL(k_pb_dual_write_w, dim3(grid_for(n, 64)), dim3(64), 0, st, dlog,
                               size, n, src, tgt, md_blob, off, cnt, out, out_cap, status);
        else
            hipLaunchKernelGGL(k_pb_dual_write, dim3(grid_for(n, 256)), dim3(256), 0, st, dlog,
                               size, n, src, tgt, md_blob, off, cnt, out, out_cap, status);
        if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
}

hipError_t launch_pb_inclusion(hipStream_t st, Timer *tm, int phase, const uint8_t *levels,
                               uint64_t w, uint64_t n, const uint64_t *leaf, uint8_t *out,
                               uint64_t out_cap, uint64_t *off, int32_t *status, uint8_t *scratch) {
    if (!n) return hipMemsetAsync(off, 0, sizeof(uint64_t), st);
    uint64_t *sizes = reinterpret_cast<uint64_t *>(scratch);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(scratch + ((n * 8 + 255) & ~255ull));
    uint8_t *temp = scratch + 2 * ((n * 8 + 255) & ~255ull);
    if (phase & 1) {
        TimerScope ts(tm, "pb_incl_size", st);
        hipLaunchKernelGGL(k_pb_incl_size, dim3(grid_for(n, 256)), dim3(256), 0, st, w, n, leaf,
                           sizes, cnt, status);
        if (hipError_t e = hipGetLastError()) return e;
        if (hipError_t e = pb_offsets(st, n, sizes, off, temp)) return e;
    }
    if (phase & 2) {
        TimerScope ts(tm, "pb_incl_write", st);
        if (w < (1ull << 31) && !pb_force_staged())  // < 2^32 level nodes: 32-bit indices
            hipLaunchKernelGGL(k_pb_incl_write_w, dim3(grid_for(n, 64)), dim3(64), 0, st, levels,
                               w, n, leaf, off, cnt, out, out_cap, status);
        else
            hipLaunchKernelGGL(k_pb_incl_write, dim3(grid_for(n, 256)), dim3(256), 0, st, levels,
                               w, n, leaf, off, cnt, out, out_cap, status);
        if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
}

}  // namespace mh
