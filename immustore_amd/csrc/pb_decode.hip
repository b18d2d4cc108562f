// pb_decode.hip -- DualProofV2 protobuf messages decoded on the device
// (the FromProto side of database_protoconv.go): what a
// client / auditor does with every VerifiableTxV2 answer before
// VerifyDualProofV2, for a batch of messages at once.
//
//   DualProofV2FromProto  database_protoconv.go:226-233   schema.proto:437-445
//   TxHeaderFromProto     :235-247                        schema.proto:349-378
//   TxMetadataFromProto   :249-262 (-> TxMetadata.Bytes(), tx_metadata.go:145-157)
//   DigestFromProto / DigestsFromProto  :293-305 (copy of up to 32 bytes)
//   InclusionProofFromProto  :123-129                    schema.proto:534-545
//   DualProofFromProto (v1)  :213-224, LinearProofFromProto :264-270,
//   LinearAdvanceProofFromProto :272-287                 schema.proto:388-434
//
// proto3 wire format as protobuf-go's Unmarshal reads it: fields in any
// order; a scalar or bytes field seen twice keeps the last value; an embedded
// message seen twice is merged (its fields read in turn into the same value);
// a known field with an unexpected wire type, and unknown fields (groups
// included), are skipped; int32 values are the low 32 bits of the varint.
// Malformed bytes (truncation, an over-long varint, wire type 6 / 7, field
// number 0, an unmatched end group) -> MH_ERR_CORRUPTED_DATA.  A message
// without a source or target header -> MH_ERR_ILLEGAL_ARGUMENTS (Go's
// TxHeaderFromProto dereferences the nil header).
//
// One lane per message, two passes: the first validates and counts the
// inclusion / consistency terms and the canonical metadata bytes, the offsets
// are scanned (hipcub), the second writes the headers, the terms and the
// metadata (packed: only the bytes that exist travel back to the host).
#include <hipcub/hipcub.hpp>

#include "capi_internal.hpp"

namespace {

constexpr uint32_t kMdSlot = MH_MAX_TX_METADATA_LEN;  // metadata bytes per header
constexpr uint32_t kMaxExtra = 256;                    // maxExtraLen, tx_metadata.go

struct PbIn {
    const uint8_t *p, *end;
    __device__ __forceinline__ bool varint(uint64_t &v) {
        v = 0;
        for (int i = 0; i < 10; i++) {
            if (p >= end) return false;
            const uint8_t b = *p++;
            if (i == 9 && b > 1) return false;  // beyond 64 bits (protowire)
            v |= (uint64_t)(b & 0x7f) << (7 * i);
            if (!(b & 0x80)) return true;
        }
        return false;
    }
    __device__ __forceinline__ bool bytes(const uint8_t *&q, uint64_t &len) {
        if (!varint(len) || len > (uint64_t)(end - p)) return false;
        q = p;
        p += len;
        return true;
    }
    __device__ __forceinline__ bool skip(uint64_t n) {
        if (n > (uint64_t)(end - p)) return false;
        p += n;
        return true;
    }
    __device__ __forceinline__ bool key(uint32_t &field, uint32_t &wt) {
        uint64_t k;
        if (!varint(k)) return false;
        field = (uint32_t)(k >> 3);
        wt = (uint32_t)(k & 7);
        return (k >> 3) != 0 && (k >> 3) < (1ull << 29);
    }
    // the value of an unknown (or mistyped) field; a group to its end
    __device__ __forceinline__ bool skip_value(uint32_t field, uint32_t wt) {
        uint64_t v;
        const uint8_t *q;
        switch (wt) {
        case 0: return varint(v);
        case 1: return skip(8);
        case 2: return bytes(q, v);
        case 5: return skip(4);
        case 3: return (p = skip_group(p, end, field)) != nullptr;
        default: return false;  // 4: an end group with no start; 6, 7
        }
    }
    // groups (deprecated, seen only as unknown fields) out of line, the reader
    // passed by value (a reference would pin the caller's reader to scratch):
    // -> the position after the group, nullptr if malformed
    static __device__ __noinline__ const uint8_t *skip_group(const uint8_t *p, const uint8_t *end,
                                                             uint32_t field) {
        PbIn in{p, end};
        return in.group_end(field) ? in.p : nullptr;
    }
    __device__ bool group_end(uint32_t field) {
        uint32_t stack[32];
        int depth = 0;
        uint32_t wt = 3;
        for (;;) {
            uint64_t v;
            const uint8_t *q;
            switch (wt) {
            case 0: if (!varint(v)) return false; break;
            case 1: if (!skip(8)) return false; break;
            case 2: if (!bytes(q, v)) return false; break;
            case 5: if (!skip(4)) return false; break;
            case 3:
                if (depth == 32) return false;
                stack[depth++] = field;
                break;
            case 4:
                if (depth == 0 || stack[depth - 1] != field) return false;
                depth--;
                break;
            default: return false;
            }
            if (depth == 0) return true;
            if (!key(field, wt)) return false;
        }
    }
};

// DigestFromProto: the first min(len, 32) bytes, zero padded, into an 8-byte
// aligned destination.  The usual 32-byte case reads nine aligned dwords and
// funnel-shifts them (v_alignbyte) instead of 32 byte loads; the read may run
// up to 3 bytes past the term, inside the padded message area.
__device__ __forceinline__ void digest_from(const uint8_t *q, uint64_t len, uint8_t *d) {
    uint32_t o[8];
    if (len >= 32) {
        const uint32_t *a = (const uint32_t *)((uintptr_t)q & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)((uintptr_t)q & 3);
        uint32_t w[9];
#pragma unroll
        for (int i = 0; i < 9; i++) w[i] = a[i];
#pragma unroll
        for (int i = 0; i < 8; i++) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t v = 0;
            for (int j = 0; j < 4; j++)
                if ((uint64_t)(4 * i + j) < len) v |= (uint32_t)q[4 * i + j] << (8 * j);
            o[i] = v;
        }
    }
    uint2 *dd = (uint2 *)d;
#pragma unroll
    for (int i = 0; i < 4; i++) dd[i] = make_uint2(o[2 * i], o[2 * i + 1]);
}

struct MdState {
    bool present = false;
    uint64_t trunc = 0;
    const uint8_t *extra = nullptr;
    uint64_t extra_len = 0;
};

// TxMetadata fields into md (merged)
__device__ __forceinline__ bool parse_md(const uint8_t *q, uint64_t len, MdState &md) {
    PbIn in{q, q + len};
    md.present = true;
    while (in.p < in.end) {
        uint32_t f, wt;
        if (!in.key(f, wt)) return false;
        if (f == 1 && wt == 0) {
            if (!in.varint(md.trunc)) return false;
        } else if (f == 2 && wt == 2) {
            if (!in.bytes(md.extra, md.extra_len)) return false;
        } else if (!in.skip_value(f, wt)) {
            return false;
        }
    }
    return true;
}

// TxHeader fields (merged); WRITE: stored straight into the output header h
// (zeroed by the caller), else only validated.  md receives the metadata.
template <bool WRITE>
__device__ __forceinline__ bool parse_header(const uint8_t *q, uint64_t len, mh_tx_header *h,
                                             MdState &md) {
    PbIn in{q, q + len};
    while (in.p < in.end) {
        uint32_t f, wt;
        if (!in.key(f, wt)) return false;
        uint64_t v;
        const uint8_t *b;
        uint64_t bl;
        if (wt == 0 && (f == 1 || f == 3 || f == 4 || f == 6 || f == 8)) {
            if (!in.varint(v)) return false;
            if (WRITE) {
                if (f == 1) h->id = v;
                else if (f == 3) h->ts = (int64_t)v;
                else if (f == 4) h->nentries = (uint32_t)v;  // int32: the low 32 bits
                else if (f == 6) h->bl_tx_id = v;
                else h->version = (uint32_t)v;
            }
        } else if (wt == 2 && (f == 2 || f == 5 || f == 7)) {
            if (!in.bytes(b, bl)) return false;
            if (WRITE) digest_from(b, bl, f == 2 ? h->prev_alh : (f == 5 ? h->eh : h->bl_root));
        } else if (wt == 2 && f == 9) {
            if (!in.bytes(b, bl) || !parse_md(b, bl, md)) return false;
        } else if (!in.skip_value(f, wt)) {
            return false;
        }
    }
    return true;
}

// TxMetadataFromProto + Bytes(): truncatedUptoTx (code 0, BE64) when > 0,
// then extra (code 1, BE16 length) when 1..256 bytes (WithExtra rejects
// longer data, and the call's error is ignored)
__device__ __forceinline__ uint32_t md_len(const MdState &md) {
    if (!md.present) return 0;
    return (md.trunc > 0 ? 9u : 0u) +
           (md.extra_len > 0 && md.extra_len <= kMaxExtra ? 3u + (uint32_t)md.extra_len : 0u);
}

__device__ void md_write(const MdState md, uint8_t *out) {  // by value: keeps the caller's state out of scratch
    uint32_t k = 0;
    if (!md.present) return;
    if (md.trunc > 0) {
        out[k++] = 0;
        for (int j = 7; j >= 0; j--) out[k++] = (uint8_t)(md.trunc >> (8 * j));
    }
    if (md.extra_len > 0 && md.extra_len <= kMaxExtra) {
        out[k++] = 1;
        out[k++] = (uint8_t)(md.extra_len >> 8);
        out[k++] = (uint8_t)md.extra_len;
        for (uint64_t j = 0; j < md.extra_len; j++) out[k++] = md.extra[j];
    }
}

// One DualProofV2 message per lane.  WRITE = false: validate, count the
// inclusion / consistency terms and the canonical metadata bytes of the two
// headers; WRITE = true: headers, terms and metadata at the scanned offsets.
// The two headers live in separate variables (no dynamically indexed local
// arrays: those would go to scratch).
template <bool WRITE>
__global__ __launch_bounds__(256) void k_pbd_dual(uint64_t n, const uint8_t *__restrict__ msgs,
                                                  const uint64_t *__restrict__ msg_off,
                                                  uint64_t *__restrict__ cnt_i, uint64_t *__restrict__ cnt_c,
                                                  uint64_t *__restrict__ cnt_m,
                                                  const uint64_t *__restrict__ incl_off,
                                                  const uint64_t *__restrict__ cons_off,
                                                  const uint64_t *__restrict__ md_off,
                                                  uint8_t *__restrict__ incl_terms,
                                                  uint8_t *__restrict__ cons_terms,
                                                  mh_tx_header *__restrict__ src_hdr,
                                                  mh_tx_header *__restrict__ tgt_hdr,
                                                  uint8_t *__restrict__ md_blob,
                                                  int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t o0 = msg_off[p], o1 = msg_off[p + 1] >= o0 ? msg_off[p + 1] : o0;
    mh_tx_header *hs = WRITE ? src_hdr + p : nullptr, *ht = WRITE ? tgt_hdr + p : nullptr;
    // the write pass re-reads only what the first pass accepted: a malformed
    // message was given no term or metadata slots and decodes to zero headers
    const bool corrupt = WRITE && status[p] == MH_ERR_CORRUPTED_DATA;
    if (WRITE) {
        *hs = mh_tx_header{};
        *ht = mh_tx_header{};
    }
    PbIn in{msgs + o0, corrupt ? msgs + o0 : msgs + o1};
    MdState ms, mt;
    bool have_s = false, have_t = false;
    uint64_t ki = 0, kc = 0;
    uint8_t *ti = WRITE ? incl_terms + 32 * incl_off[p] : nullptr;
    uint8_t *tc = WRITE ? cons_terms + 32 * cons_off[p] : nullptr;
    bool ok = true;
    while (ok && in.p < in.end) {
        uint32_t f, wt;
        if (!in.key(f, wt)) {
            ok = false;
            break;
        }
        const uint8_t *b;
        uint64_t bl;
        if (wt == 2 && f == 1) {
            ok = in.bytes(b, bl) && parse_header<WRITE>(b, bl, hs, ms);
            have_s = true;
        } else if (wt == 2 && f == 2) {
            ok = in.bytes(b, bl) && parse_header<WRITE>(b, bl, ht, mt);
            have_t = true;
        } else if (wt == 2 && f == 3) {
            ok = in.bytes(b, bl);
            if (WRITE) digest_from(b, bl, ti + 32 * ki);
            ki++;
        } else if (wt == 2 && f == 4) {
            ok = in.bytes(b, bl);
            if (WRITE) digest_from(b, bl, tc + 32 * kc);
            kc++;
        } else {
            ok = in.skip_value(f, wt);
        }
    }
    if (!WRITE) {
        const int32_t st = !ok ? MH_ERR_CORRUPTED_DATA
                               : (!have_s || !have_t) ? MH_ERR_ILLEGAL_ARGUMENTS : MH_OK;
        status[p] = st;
        // a malformed message contributes no terms and no metadata
        cnt_i[p] = ok ? ki : 0;
        cnt_c[p] = ok ? kc : 0;
        cnt_m[p] = ok ? md_len(ms) + md_len(mt) : 0;
        return;
    }
    const uint64_t m0 = md_off[p];
    const uint32_t ls = corrupt ? 0u : md_len(ms), lt = corrupt ? 0u : md_len(mt);
    hs->md_off = (uint32_t)m0;
    hs->md_len = ls;
    ht->md_off = (uint32_t)(m0 + ls);
    ht->md_len = lt;
    if (ls) md_write(ms, md_blob + m0);
    if (lt) md_write(mt, md_blob + m0 + ls);
}

// One InclusionProof message per lane (InclusionProofFromProto,
// database_protoconv.go:123-129): Leaf / Width are int32 on the wire and Go
// ints after the conversion (sign-extended; stored as their 64-bit pattern).
template <bool WRITE>
__global__ __launch_bounds__(256) void k_pbd_incl(uint64_t n, const uint8_t *__restrict__ msgs,
                                                  const uint64_t *__restrict__ msg_off,
                                                  uint64_t *__restrict__ cnt,
                                                  const uint64_t *__restrict__ term_off,
                                                  uint8_t *__restrict__ terms,
                                                  uint64_t *__restrict__ leaf,
                                                  uint64_t *__restrict__ width,
                                                  int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t o0 = msg_off[p], o1 = msg_off[p + 1] >= o0 ? msg_off[p + 1] : o0;
    const bool corrupt = WRITE && status[p] == MH_ERR_CORRUPTED_DATA;
    PbIn in{msgs + o0, corrupt ? msgs + o0 : msgs + o1};
    uint64_t lf = 0, wd = 0, k = 0;
    uint8_t *t = WRITE ? terms + 32 * term_off[p] : nullptr;
    bool ok = true;
    while (ok && in.p < in.end) {
        uint32_t f, wt;
        if (!in.key(f, wt)) {
            ok = false;
            break;
        }
        uint64_t v;
        const uint8_t *b;
        if (wt == 0 && (f == 1 || f == 2)) {
            ok = in.varint(v);
            const uint64_t x = (uint64_t)(int64_t)(int32_t)(uint32_t)v;  // int(int32)
            if (f == 1) lf = x;
            else wd = x;
        } else if (wt == 2 && f == 3) {
            ok = in.bytes(b, v);
            if (WRITE) digest_from(b, v, t + 32 * k);
            k++;
        } else {
            ok = in.skip_value(f, wt);
        }
    }
    if (!WRITE) {
        status[p] = ok ? MH_OK : MH_ERR_CORRUPTED_DATA;
        cnt[p] = ok ? k : 0;
        return;
    }
    leaf[p] = corrupt ? 0 : lf;
    width[p] = corrupt ? 0 : wd;
}

// ---------------------------------------------------------------- DualProof (v1)
// DualProofFromProto (database_protoconv.go:213-224) with LinearProofFromProto
// (:264-270; not nil-checked: a message without linearProof panics in Go ->
// MH_ERR_ILLEGAL_ARGUMENTS) and LinearAdvanceProofFromProto (:272-287; nil ->
// has_advance 0; only the nested InclusionProofs' terms are kept).
enum : int { kI = 0, kC, kL, kLin, kAdv, kQ, kQT, kMd, kCounts };  // per-message counts

struct Dual1Out {  // device-side outputs of the write pass
    const uint64_t *off[kCounts];  // scanned offsets (n + 1 each)
    uint8_t *terms[5];             // incl, cons, last, linear, advance
    uint8_t *qterms;               // nested inclusion proofs' terms
    uint64_t *qoff;                // nested proofs' term offsets
    mh_tx_header *src_hdr, *tgt_hdr;
    uint8_t *md_blob, *tbl_alh, *has_lin, *has_adv;
    uint64_t *lin_src, *lin_tgt;
};

template <bool WRITE>
__global__ __launch_bounds__(256) void k_pbd_dual1(uint64_t n, const uint8_t *__restrict__ msgs,
                                                   const uint64_t *__restrict__ msg_off,
                                                   uint64_t *__restrict__ cnt,  // kCounts x n
                                                   Dual1Out o, int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t o0 = msg_off[p], o1 = msg_off[p + 1] >= o0 ? msg_off[p + 1] : o0;
    const bool corrupt = WRITE && status[p] == MH_ERR_CORRUPTED_DATA;
    mh_tx_header *hs = WRITE ? o.src_hdr + p : nullptr, *ht = WRITE ? o.tgt_hdr + p : nullptr;
    if (WRITE) {
        *hs = mh_tx_header{};
        *ht = mh_tx_header{};
        uint2 *z = (uint2 *)(o.tbl_alh + 32 * p);
        for (int i = 0; i < 4; i++) z[i] = make_uint2(0, 0);
    }
    PbIn in{msgs + o0, corrupt ? msgs + o0 : msgs + o1};
    MdState ms, mt;
    bool have_s = false, have_t = false, have_lin = false, have_adv = false;
    // running counts (plain scalars: an array or a capturing lambda here sends
    // the readers to scratch)
    uint64_t ki = 0, kc = 0, kl = 0, kln = 0, ka = 0, kq = 0, kqt = 0;
    uint64_t lsrc = 0, ltgt = 0;
    bool ok = true;
#define PBD_TERM(J, CNT, B, BL)                                                          \
    do {                                                                                 \
        if (WRITE) digest_from(B, BL, o.terms[J] + 32 * (o.off[J][p] + CNT));            \
        CNT++;                                                                           \
    } while (0)
    while (ok && in.p < in.end) {
        uint32_t f, wt;
        if (!in.key(f, wt)) {
            ok = false;
            break;
        }
        const uint8_t *b;
        uint64_t bl;
        if (wt == 2 && f == 1) {
            ok = in.bytes(b, bl) && parse_header<WRITE>(b, bl, hs, ms);
            have_s = true;
        } else if (wt == 2 && f == 2) {
            ok = in.bytes(b, bl) && parse_header<WRITE>(b, bl, ht, mt);
            have_t = true;
        } else if (wt == 2 && f == 3) {
            if ((ok = in.bytes(b, bl))) PBD_TERM(kI, ki, b, bl);
        } else if (wt == 2 && f == 4) {
            if ((ok = in.bytes(b, bl))) PBD_TERM(kC, kc, b, bl);
        } else if (wt == 2 && f == 5) {
            if ((ok = in.bytes(b, bl)) && WRITE) digest_from(b, bl, o.tbl_alh + 32 * p);
        } else if (wt == 2 && f == 6) {
            if ((ok = in.bytes(b, bl))) PBD_TERM(kL, kl, b, bl);
        } else if (wt == 2 && f == 7) {  // LinearProof (merged)
            have_lin = true;
            if (!(ok = in.bytes(b, bl))) break;
            PbIn li{b, b + bl};
            while (ok && li.p < li.end) {
                uint32_t g, gt;
                if (!li.key(g, gt)) {
                    ok = false;
                    break;
                }
                const uint8_t *c;
                uint64_t cl;
                if (gt == 0 && g == 1) ok = li.varint(lsrc);
                else if (gt == 0 && g == 2) ok = li.varint(ltgt);
                else if (gt == 2 && g == 3) {
                    if ((ok = li.bytes(c, cl))) PBD_TERM(kLin, kln, c, cl);
                } else ok = li.skip_value(g, gt);
            }
        } else if (wt == 2 && f == 8) {  // LinearAdvanceProof (merged)
            have_adv = true;
            if (!(ok = in.bytes(b, bl))) break;
            PbIn ai{b, b + bl};
            while (ok && ai.p < ai.end) {
                uint32_t g, gt;
                if (!ai.key(g, gt)) {
                    ok = false;
                    break;
                }
                const uint8_t *c;
                uint64_t cl;
                if (gt == 2 && g == 1) {
                    if ((ok = ai.bytes(c, cl))) PBD_TERM(kAdv, ka, c, cl);
                } else if (gt == 2 && g == 2) {  // one more InclusionProof: its terms
                    if (!(ok = ai.bytes(c, cl))) break;
                    if (WRITE) o.qoff[o.off[kQ][p] + kq] = o.off[kQT][p] + kqt;
                    kq++;
                    PbIn qi{c, c + cl};
                    while (ok && qi.p < qi.end) {
                        uint32_t h, htp;
                        if (!qi.key(h, htp)) {
                            ok = false;
                            break;
                        }
                        const uint8_t *d;
                        uint64_t dl;
                        if (htp == 2 && h == 3) {
                            if ((ok = qi.bytes(d, dl))) {
                                if (WRITE) digest_from(d, dl, o.qterms + 32 * (o.off[kQT][p] + kqt));
                                kqt++;
                            }
                        } else ok = qi.skip_value(h, htp);  // leaf / width: not kept
                    }
                } else ok = ai.skip_value(g, gt);
            }
        } else {
            ok = in.skip_value(f, wt);
        }
    }
#undef PBD_TERM
    if (!WRITE) {
        status[p] = !ok ? MH_ERR_CORRUPTED_DATA
                        : (!have_s || !have_t || !have_lin) ? MH_ERR_ILLEGAL_ARGUMENTS : MH_OK;
        const uint64_t v[kCounts] = {ki, kc, kl, kln, ka, kq, kqt, md_len(ms) + md_len(mt)};
#pragma unroll
        for (int j = 0; j < kCounts; j++) cnt[(uint64_t)j * n + p] = ok ? v[j] : 0;
        return;
    }
    o.has_lin[p] = !corrupt && have_lin;
    o.has_adv[p] = !corrupt && have_adv;
    o.lin_src[p] = corrupt ? 0 : lsrc;
    o.lin_tgt[p] = corrupt ? 0 : ltgt;
    const uint64_t m0 = o.off[kMd][p];
    const uint32_t ls = corrupt ? 0u : md_len(ms), lt = corrupt ? 0u : md_len(mt);
    hs->md_off = (uint32_t)m0;
    hs->md_len = ls;
    ht->md_off = (uint32_t)(m0 + ls);
    ht->md_len = lt;
    if (ls) md_write(ms, o.md_blob + m0);
    if (lt) md_write(mt, o.md_blob + m0 + ls);
}

// ------------------------------------------- DualProofV2 from the wire, verified
// VerifyDualProofV2's argument checks (verification.go:303-316) and the arrays
// of its two ahtree proofs (:342-370) from the decoded headers, on the device
// (the host loops of mh_verify_dual_proof_v2_batch); headers that cannot be
// hashed are flagged and hashed as empty v1 headers.  Decoded metadata is
// canonical and at most 268 bytes, so only the version can make a header
// unhashable here.
__global__ __launch_bounds__(256) void k_dpv2_prep(uint64_t n, const mh_tx_header *__restrict__ hd,
                                                   const uint64_t *__restrict__ src,
                                                   const uint64_t *__restrict__ tgt,
                                                   int32_t *__restrict__ status,
                                                   mh_tx_header *__restrict__ hh,
                                                   uint64_t *__restrict__ ii, uint64_t *__restrict__ ij,
                                                   uint64_t *__restrict__ ci, uint8_t *__restrict__ sel,
                                                   uint8_t *__restrict__ sbl, uint8_t *__restrict__ tbl) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    mh_tx_header sh = hd[p], th = hd[n + p];
    int32_t s = status[p];
    // a v0 innerHash never reads the metadata (tx.go:258-263), which a wire
    // header may carry; a version other than 0 / 1 panics in Go's innerHash
    if (sh.version == 0) sh.md_len = 0;
    if (th.version == 0) th.md_len = 0;
    if (s == MH_OK) {
        if (sh.id == 0 || sh.id != src[p] || th.id != tgt[p]) s = MH_ERR_ILLEGAL_ARGUMENTS;
        else if (src[p] > tgt[p]) s = MH_ERR_SOURCE_TX_NEWER;
        else if (sh.version > 1 || th.version > 1) s = MH_ERR_ILLEGAL_ARGUMENTS;
    }
    status[p] = s;
    ii[p] = src[p];
    ij[p] = th.bl_tx_id;
    sel[p] = src[p] == 1;
    ci[p] = src[p] == 1 ? src[p] : sh.bl_tx_id;
    for (int k = 0; k < 32; k++) {
        sbl[32 * p + k] = sh.bl_root[k];
        tbl[32 * p + k] = th.bl_root[k];
    }
    if (s != MH_OK) {  // keep the Alh kernel's reads inside md_blob; result unused
        sh.version = th.version = 1;
        sh.md_len = th.md_len = 0;
    }
    hh[p] = sh;
    hh[n + p] = th;
}

// verification.go:318-370 after the Alh values and the two ahtree proofs
__global__ __launch_bounds__(256) void k_dpv2_final(uint64_t n, const mh_tx_header *__restrict__ hd,
                                                    const uint64_t *__restrict__ src,
                                                    const uint64_t *__restrict__ tgt,
                                                    const int32_t *__restrict__ alh_st,
                                                    const uint8_t *__restrict__ oki,
                                                    const uint8_t *__restrict__ okc,
                                                    int32_t *__restrict__ status) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    int32_t s = status[p];
    if (s == MH_OK) {
        const mh_tx_header &sh = hd[p], &th = hd[n + p];
        if (alh_st[p] != MH_OK || alh_st[n + p] != MH_OK) s = MH_ERR_ILLEGAL_ARGUMENTS;
        else if (sh.id - 1 != sh.bl_tx_id || th.id - 1 != th.bl_tx_id) s = MH_ERR_UNEXPECTED_LINKING;
        else if (src[p] == tgt[p]) s = MH_OK;
        else if (!oki[p]) s = MH_ERR_INCLUSION_NOT_VALID;
        else if (!okc[p]) s = MH_ERR_CONSISTENCY_NOT_VALID;
    }
    status[p] = s;
}

// Two device words into pinned host memory by a kernel store: a small
// read-back without a DMA copy, which would queue behind the large
// host-to-device chunks in flight on the copy engine.
__global__ void k_put2_host(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b,
                            volatile uint64_t *out) {
    if (threadIdx.x == 0) {
        out[0] = *a;
        out[1] = *b;
        __threadfence_system();
    }
}

}  // namespace

extern "C" int mh_dual_proof_v2_pb_decode_batch(
    mh_ctx *c, uint64_t n, const uint8_t *msgs, const uint64_t *msg_off, mh_tx_header *src_hdr,
    mh_tx_header *tgt_hdr, uint8_t *md_blob, uint64_t *incl_off, uint8_t *incl_terms,
    uint64_t incl_cap, uint64_t *cons_off, uint8_t *cons_terms, uint64_t cons_cap,
    int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!msg_off || !src_hdr || !tgt_hdr || !md_blob || !incl_off || !cons_off ||
                         !status)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n == 0) {
            if (incl_off) incl_off[0] = 0;
            if (cons_off) cons_off[0] = 0;
            return MH_OK;
        }
        if (2 * n * (uint64_t)kMdSlot > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // md_off
        if (n > 0x7fffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // hipcub's int item count
        if (!monotonic(msg_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t m0 = msg_off[0], mb = msg_off[n] - m0;
        if (mb && !msgs) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        size_t scan_bytes = 0;
        MH_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (const uint64_t *)nullptr,
                                                (uint64_t *)nullptr, (int)n, st));
        Layout L;
        const uint64_t b_msg = L.add(mb + 16), b_off = L.add((n + 1) * 8), b_ni = L.add(n * 8),
                       b_nc = L.add(n * 8), b_nm = L.add(n * 8), b_io = L.add((n + 1) * 8),
                       b_co = L.add((n + 1) * 8), b_mo = L.add((n + 1) * 8), b_st = L.add(n * 4),
                       b_scan = L.add(scan_bytes), b_h = L.add(2 * n * sizeof(mh_tx_header)),
                       b_md = L.add(2 * n * (uint64_t)kMdSlot);
        MH_HIP(c->s_tx.ensure(L.total));
        uint8_t *base = c->s_tx.as<uint8_t>();
        if (mb) MH_HIP(hipMemcpyAsync(base + b_msg, msgs + m0, mb, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_off, msg_off, (n + 1) * 8, hipMemcpyHostToDevice, st));
        const unsigned grid = (unsigned)((n + 255) / 256);
        const uint8_t *dmsg = base + b_msg - m0;
        uint64_t *io = (uint64_t *)(base + b_io), *co = (uint64_t *)(base + b_co),
                 *mo = (uint64_t *)(base + b_mo);
        hipLaunchKernelGGL(k_pbd_dual<false>, dim3(grid), dim3(256), 0, st, n, dmsg,
                           (const uint64_t *)(base + b_off), (uint64_t *)(base + b_ni),
                           (uint64_t *)(base + b_nc), (uint64_t *)(base + b_nm), nullptr, nullptr,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           (int32_t *)(base + b_st));
        MH_HIP(hipGetLastError());
        const uint64_t cnt[3] = {b_ni, b_nc, b_nm};
        uint64_t *outs[3] = {io, co, mo};
        for (int k = 0; k < 3; k++) {
            MH_HIP(hipMemsetAsync(outs[k], 0, 8, st));
            size_t sb = scan_bytes;
            MH_HIP(hipcub::DeviceScan::InclusiveSum(base + b_scan, sb,
                                                    (const uint64_t *)(base + cnt[k]), outs[k] + 1,
                                                    (int)n, st));
        }
        uint64_t md_total = 0;
        MH_HIP(hipMemcpyAsync(incl_off, io, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(cons_off, co, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(&md_total, mo + n, 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(status, base + b_st, n * 4, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        const uint64_t ti = incl_off[n], tc = cons_off[n];
        if (ti > incl_cap || tc > cons_cap) return MH_ERR_BUFFER_TOO_SMALL;
        if ((ti && !incl_terms) || (tc && !cons_terms)) return MH_ERR_ILLEGAL_ARGUMENTS;
        DevBuf &tb = c->s_tree;
        MH_HIP(tb.ensure(std::max<uint64_t>(ti + tc, 1) * 32));
        uint8_t *dti = tb.as<uint8_t>(), *dtc = dti + ti * 32;
        hipLaunchKernelGGL(k_pbd_dual<true>, dim3(grid), dim3(256), 0, st, n, dmsg,
                           (const uint64_t *)(base + b_off), nullptr, nullptr, nullptr, io, co, mo,
                           dti, dtc, (mh_tx_header *)(base + b_h),
                           (mh_tx_header *)(base + b_h) + n, base + b_md, (int32_t *)(base + b_st));
        MH_HIP(hipGetLastError());
        MH_HIP(hipMemcpyAsync(src_hdr, base + b_h, n * sizeof(mh_tx_header), hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(tgt_hdr, base + b_h + n * sizeof(mh_tx_header),
                              n * sizeof(mh_tx_header), hipMemcpyDeviceToHost, st));
        if (md_total) MH_HIP(hipMemcpyAsync(md_blob, base + b_md, md_total, hipMemcpyDeviceToHost, st));
        if (ti) MH_HIP(hipMemcpyAsync(incl_terms, dti, ti * 32, hipMemcpyDeviceToHost, st));
        if (tc) MH_HIP(hipMemcpyAsync(cons_terms, dtc, tc * 32, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}

extern "C" int mh_htree_inclusion_proof_pb_decode_batch(mh_ctx *c, uint64_t n, const uint8_t *msgs,
                                                        const uint64_t *msg_off, uint64_t *leaf,
                                                        uint64_t *width, uint64_t *term_off,
                                                        uint8_t *terms, uint64_t term_cap,
                                                        int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!msg_off || !leaf || !width || !term_off || !status)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n == 0) {
            if (term_off) term_off[0] = 0;
            return MH_OK;
        }
        if (n > 0x7fffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // hipcub's int item count
        if (!monotonic(msg_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t m0 = msg_off[0], mb = msg_off[n] - m0;
        if (mb && !msgs) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        size_t scan_bytes = 0;
        MH_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (const uint64_t *)nullptr,
                                                (uint64_t *)nullptr, (int)n, st));
        Layout L;
        const uint64_t b_msg = L.add(mb + 16), b_off = L.add((n + 1) * 8), b_cnt = L.add(n * 8),
                       b_to = L.add((n + 1) * 8), b_st = L.add(n * 4), b_scan = L.add(scan_bytes),
                       b_lw = L.add(2 * n * 8);
        MH_HIP(c->s_tx.ensure(L.total));
        uint8_t *base = c->s_tx.as<uint8_t>();
        if (mb) MH_HIP(hipMemcpyAsync(base + b_msg, msgs + m0, mb, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_off, msg_off, (n + 1) * 8, hipMemcpyHostToDevice, st));
        const unsigned grid = (unsigned)((n + 255) / 256);
        const uint8_t *dmsg = base + b_msg - m0;
        uint64_t *to = (uint64_t *)(base + b_to), *lw = (uint64_t *)(base + b_lw);
        hipLaunchKernelGGL(k_pbd_incl<false>, dim3(grid), dim3(256), 0, st, n, dmsg,
                           (const uint64_t *)(base + b_off), (uint64_t *)(base + b_cnt), nullptr,
                           nullptr, nullptr, nullptr, (int32_t *)(base + b_st));
        MH_HIP(hipGetLastError());
        MH_HIP(hipMemsetAsync(to, 0, 8, st));
        size_t sb = scan_bytes;
        MH_HIP(hipcub::DeviceScan::InclusiveSum(base + b_scan, sb, (const uint64_t *)(base + b_cnt),
                                                to + 1, (int)n, st));
        MH_HIP(hipMemcpyAsync(term_off, to, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(status, base + b_st, n * 4, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        const uint64_t tt = term_off[n];
        if (tt > term_cap) return MH_ERR_BUFFER_TOO_SMALL;
        if (tt && !terms) return MH_ERR_ILLEGAL_ARGUMENTS;
        DevBuf &tb = c->s_tree;
        MH_HIP(tb.ensure(std::max<uint64_t>(tt, 1) * 32));
        hipLaunchKernelGGL(k_pbd_incl<true>, dim3(grid), dim3(256), 0, st, n, dmsg,
                           (const uint64_t *)(base + b_off), nullptr, to, tb.as<uint8_t>(), lw,
                           lw + n, (int32_t *)(base + b_st));
        MH_HIP(hipGetLastError());
        MH_HIP(hipMemcpyAsync(leaf, lw, n * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(width, lw + n, n * 8, hipMemcpyDeviceToHost, st));
        if (tt) MH_HIP(hipMemcpyAsync(terms, tb.as<uint8_t>(), tt * 32, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}

extern "C" int mh_dual_proof_pb_decode_batch(mh_ctx *c, uint64_t n, const uint8_t *msgs,
                                             const uint64_t *msg_off, mh_dual_proof_decoded *out,
                                             int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || !out) return MH_ERR_ILLEGAL_ARGUMENTS;
        uint64_t *offs[kCounts - 1] = {out->incl_off,   out->cons_off,           out->last_off,
                                       out->linear_off, out->advance_off,        out->advance_incl_first,
                                       nullptr};  // nested term offsets: advance_incl_off below
        if (n && (!msg_off || !status || !out->src_hdr || !out->tgt_hdr || !out->md_blob ||
                  !out->target_bl_tx_alh || !out->has_linear || !out->linear_src ||
                  !out->linear_tgt || !out->has_advance || !out->advance_incl_off))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        for (int j = 0; j < kQT; j++)
            if (!offs[j]) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n == 0) {
            for (int j = 0; j < kQT; j++) offs[j][0] = 0;
            if (out->advance_incl_off) out->advance_incl_off[0] = 0;
            out->nested_proofs = out->nested_terms = 0;
            return MH_OK;
        }
        if (2 * n * (uint64_t)kMdSlot > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // md_off
        if (n > 0x7fffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // hipcub's int item count
        if (!monotonic(msg_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t m0 = msg_off[0], mb = msg_off[n] - m0;
        if (mb && !msgs) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        size_t scan_bytes = 0;
        MH_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (const uint64_t *)nullptr,
                                                (uint64_t *)nullptr, (int)n, st));
        Layout L;
        const uint64_t b_msg = L.add(mb + 16), b_off = L.add((n + 1) * 8),
                       b_cnt = L.add(kCounts * n * 8), b_so = L.add(kCounts * (n + 1) * 8),
                       b_st = L.add(n * 4), b_scan = L.add(scan_bytes),
                       b_h = L.add(2 * n * sizeof(mh_tx_header)), b_md = L.add(2 * n * (uint64_t)kMdSlot),
                       b_tba = L.add(n * 32), b_flags = L.add(2 * n), b_ls = L.add(2 * n * 8);
        MH_HIP(c->s_tx.ensure(L.total));
        uint8_t *base = c->s_tx.as<uint8_t>();
        if (mb) MH_HIP(hipMemcpyAsync(base + b_msg, msgs + m0, mb, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_off, msg_off, (n + 1) * 8, hipMemcpyHostToDevice, st));
        const unsigned grid = (unsigned)((n + 255) / 256);
        const uint8_t *dmsg = base + b_msg - m0;
        uint64_t *cnt = (uint64_t *)(base + b_cnt), *so = (uint64_t *)(base + b_so);
        hipLaunchKernelGGL(k_pbd_dual1<false>, dim3(grid), dim3(256), 0, st, n, dmsg,
                           (const uint64_t *)(base + b_off), cnt, Dual1Out{},
                           (int32_t *)(base + b_st));
        MH_HIP(hipGetLastError());
        for (int j = 0; j < kCounts; j++) {
            uint64_t *sj = so + (uint64_t)j * (n + 1);
            MH_HIP(hipMemsetAsync(sj, 0, 8, st));
            size_t sb = scan_bytes;
            MH_HIP(hipcub::DeviceScan::InclusiveSum(base + b_scan, sb, (const uint64_t *)(cnt + j * n),
                                                    sj + 1, (int)n, st));
        }
        for (int j = 0; j < kQT; j++)
            MH_HIP(hipMemcpyAsync(offs[j], so + (uint64_t)j * (n + 1), (n + 1) * 8,
                                  hipMemcpyDeviceToHost, st));
        uint64_t tot[2] = {0, 0};  // nested terms, metadata bytes
        MH_HIP(hipMemcpyAsync(&tot[0], so + (uint64_t)kQT * (n + 1) + n, 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(&tot[1], so + (uint64_t)kMd * (n + 1) + n, 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(status, base + b_st, n * 4, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        const uint64_t caps[kCounts - 1] = {out->incl_cap,   out->cons_cap,        out->last_cap,
                                            out->linear_cap, out->advance_cap,     out->advance_incl_cap,
                                            out->advance_incl_terms_cap};
        uint8_t *hterms[5] = {out->incl_terms, out->cons_terms, out->last_terms, out->linear_terms,
                              out->advance_terms};
        uint64_t totals[kCounts - 1];
        for (int j = 0; j < kQT; j++) totals[j] = offs[j][n];
        totals[kQT] = tot[0];
        out->nested_proofs = totals[kQ];
        out->nested_terms = totals[kQT];
        for (int j = 0; j < kCounts - 1; j++)
            if (totals[j] > caps[j]) return MH_ERR_BUFFER_TOO_SMALL;
        for (int j = 0; j < 5; j++)
            if (totals[j] && !hterms[j]) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (totals[kQT] && !out->advance_incl_terms) return MH_ERR_ILLEGAL_ARGUMENTS;
        // device term area: the five lists, the nested terms, the nested offsets
        uint64_t tpos[6], tall = 0;
        for (int j = 0; j < 5; j++) {
            tpos[j] = tall;
            tall += totals[j];
        }
        tpos[5] = tall;
        tall += totals[kQT];
        const uint64_t nq = totals[kQ];
        DevBuf &tb = c->s_tree;
        MH_HIP(tb.ensure(tall * 32 + (nq + 1) * 8 + 8));
        uint8_t *dt = tb.as<uint8_t>();
        uint64_t *dq = (uint64_t *)(dt + tall * 32);
        Dual1Out o;
        for (int j = 0; j < kCounts; j++) o.off[j] = so + (uint64_t)j * (n + 1);
        for (int j = 0; j < 5; j++) o.terms[j] = dt + tpos[j] * 32;
        o.qterms = dt + tpos[5] * 32;
        o.qoff = dq;
        o.src_hdr = (mh_tx_header *)(base + b_h);
        o.tgt_hdr = o.src_hdr + n;
        o.md_blob = base + b_md;
        o.tbl_alh = base + b_tba;
        o.has_lin = base + b_flags;
        o.has_adv = base + b_flags + n;
        o.lin_src = (uint64_t *)(base + b_ls);
        o.lin_tgt = o.lin_src + n;
        hipLaunchKernelGGL(k_pbd_dual1<true>, dim3(grid), dim3(256), 0, st, n, dmsg,
                           (const uint64_t *)(base + b_off), nullptr, o, (int32_t *)(base + b_st));
        MH_HIP(hipGetLastError());
        const size_t hb = n * sizeof(mh_tx_header);
        MH_HIP(hipMemcpyAsync(out->src_hdr, base + b_h, hb, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(out->tgt_hdr, base + b_h + hb, hb, hipMemcpyDeviceToHost, st));
        if (tot[1]) MH_HIP(hipMemcpyAsync(out->md_blob, base + b_md, tot[1], hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(out->target_bl_tx_alh, base + b_tba, n * 32, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(out->has_linear, base + b_flags, n, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(out->has_advance, base + b_flags + n, n, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(out->linear_src, base + b_ls, n * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(out->linear_tgt, base + b_ls + n * 8, n * 8, hipMemcpyDeviceToHost, st));
        for (int j = 0; j < 5; j++)
            if (totals[j])
                MH_HIP(hipMemcpyAsync(hterms[j], dt + tpos[j] * 32, totals[j] * 32,
                                      hipMemcpyDeviceToHost, st));
        if (totals[kQT])
            MH_HIP(hipMemcpyAsync(out->advance_incl_terms, dt + tpos[5] * 32, totals[kQT] * 32,
                                  hipMemcpyDeviceToHost, st));
        if (nq) MH_HIP(hipMemcpyAsync(out->advance_incl_off, dq, nq * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        out->advance_incl_off[nq] = totals[kQT];
        return MH_OK;
    });
}

// The fused call is bound by the copy of the messages (1.8 GB for 10^6
// DualProofV2 at ~54 GB/s against ~11.5 ms of device work), so the batch is
// cut into chunks of ~64 MiB of messages (MH_PB_CHUNK_MIB): a helper thread
// issues every chunk's copies on the context's copy stream (a pageable copy
// holds its issuing thread until it is staged) and records one event per
// chunk, while this thread decodes and verifies chunk k on the compute stream
// as soon as its event fires -- only the last chunk's device work is exposed.
extern "C" int mh_verify_dual_proof_v2_pb_batch(mh_ctx *c, uint64_t n, const uint8_t *msgs,
                                                const uint64_t *msg_off, const uint64_t *src,
                                                const uint64_t *tgt, const uint8_t *src_alh,
                                                const uint8_t *tgt_alh, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!msg_off || !src || !tgt || !src_alh || !tgt_alh || !status)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n == 0) return MH_OK;
        if (2 * n * (uint64_t)kMdSlot > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // md_off
        if (n > 0x7fffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;  // hipcub's int item count
        if (!monotonic(msg_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t m0 = msg_off[0], mb = msg_off[n] - m0;
        if (mb && !msgs) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(hipSetDevice(c->device));
        MH_HIP(c->copy_lane());
        MH_HIP(c->p_small.ensure(64));
        hipStream_t st = c->stream;
        // chunks: consecutive messages up to chunk_bytes (one at least)
        uint64_t chunk_bytes = 128ull << 20;
        if (const char *e = getenv("MH_PB_CHUNK_MIB")) chunk_bytes = std::max(1, atoi(e)) * (1ull << 20);
        std::vector<uint64_t> cut{0};
        for (uint64_t i = 0; i < n;) {
            uint64_t j = i + 1;
            while (j < n && msg_off[j + 1] - msg_off[i] <= chunk_bytes) j++;
            cut.push_back(j);
            i = j;
        }
        const int nch = (int)cut.size() - 1;
        uint64_t max_nk = 0;
        for (int k = 0; k < nch; k++) max_nk = std::max(max_nk, cut[k + 1] - cut[k]);
        MH_HIP(ensure_chunk_events(c, nch));
        size_t scan_bytes = 0;
        MH_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (const uint64_t *)nullptr,
                                                (uint64_t *)nullptr, (int)max_nk, st));
        Layout L;
        // caller arrays (x = per chunk: its source Alh values then its target
        // Alh values, as the Alh kernel expects them), then device-only data;
        // per-chunk offset arrays hold n_k + 1 entries at [lo + k, hi + k]
        const uint64_t nc = n + (uint64_t)nch;
        const uint64_t b_msg = L.add(mb + 16), b_off = L.add((n + 1) * 8), b_src = L.add(n * 8),
                       b_tgt = L.add(n * 8), b_xa = L.add(2 * n * 32), b_x = L.add(2 * n * 32),
                       b_cnt = L.add(3 * n * 8), b_io = L.add(nc * 8), b_co = L.add(nc * 8), b_mo = L.add(nc * 8),
                       b_st = L.add(n * 4), b_scan = L.add(scan_bytes),
                       b_hd = L.add(2 * n * sizeof(mh_tx_header)), b_hh = L.add(2 * n * sizeof(mh_tx_header)),
                       b_md = L.add(2 * n * (uint64_t)kMdSlot), b_s = L.add(2 * n * kTxInnerStride),
                       b_ast = L.add(2 * n * 4), b_ii = L.add(n * 8), b_ij = L.add(n * 8),
                       b_ci = L.add(n * 8), b_sel = L.add(n), b_sbl = L.add(n * 32), b_tbl = L.add(n * 32),
                       b_leaf = L.add(n * 32), b_ca = L.add(n * 32), b_oki = L.add(n), b_okc = L.add(n);
        MH_HIP(c->s_tx.ensure(L.total));
        // term area reused chunk after chunk: a well-formed term costs >= 34
        // message bytes (tag, length, 32-byte digest), so this rarely grows;
        // sized from the batch itself when it is smaller than one chunk
        DevBuf &tb = c->s_tree;
        MH_HIP(tb.ensure(std::max<uint64_t>(std::min(mb, chunk_bytes) / 34 + 64, 1) * 32));
        uint8_t *base = c->s_tx.as<uint8_t>();
        // the copies, one helper thread: chunk 0 = the per-message arrays
        // whole (offsets, ids, Alh values: few large copies -- each copy call
        // costs the DMA engine ~0.1 ms of setup) and the first messages, chunk
        // k = its messages
        ChunkCopier cc(c);
        cc.chunks.resize(nch);
        cc.chunks[0] = {{base + b_off, msg_off, (n + 1) * 8},
                        {base + b_src, src, n * 8},
                        {base + b_tgt, tgt, n * 8},
                        {base + b_xa, src_alh, n * 32},
                        {base + b_xa + n * 32, tgt_alh, n * 32}};
        for (int k = 0; k < nch; k++) {
            const uint64_t lo = cut[k], hi = cut[k + 1];
            const uint64_t b0 = msg_off[lo] - m0, bb = msg_off[hi] - msg_off[lo];
            cc.chunks[k].push_back({base + b_msg + b0, msgs + msg_off[lo], bb});
        }
        MH_HIP(cc.start());
        const uint8_t *dmsg = base + b_msg - m0;
        int32_t *dst_all = (int32_t *)(base + b_st);
        for (int k = 0; k < nch; k++) {
            MH_HIP(cc.wait(k));
            MH_HIP(hipStreamWaitEvent(st, c->ev_chunks[k], 0));
            const uint64_t lo = cut[k], nk = cut[k + 1] - lo;
            const unsigned grid = (unsigned)((nk + 255) / 256);
            const uint64_t *doff = (const uint64_t *)(base + b_off) + lo;
            uint64_t *cnt = (uint64_t *)(base + b_cnt);
            uint64_t *io = (uint64_t *)(base + b_io) + lo + k, *co = (uint64_t *)(base + b_co) + lo + k,
                     *mo = (uint64_t *)(base + b_mo) + lo + k;
            int32_t *dst = dst_all + lo;
            uint8_t *md = base + b_md + 2 * lo * (uint64_t)kMdSlot;
            // decode: validate + count, scans
            hipLaunchKernelGGL(k_pbd_dual<false>, dim3(grid), dim3(256), 0, st, nk, dmsg, doff,
                               cnt + lo, cnt + n + lo, cnt + 2 * n + lo, nullptr, nullptr, nullptr,
                               nullptr, nullptr, nullptr, nullptr, nullptr, dst);
            MH_HIP(hipGetLastError());
            uint64_t *outs[3] = {io, co, mo};
            for (int q = 0; q < 3; q++) {
                MH_HIP(hipMemsetAsync(outs[q], 0, 8, st));
                size_t sb = scan_bytes;
                MH_HIP(hipcub::DeviceScan::InclusiveSum(base + b_scan, sb,
                                                        (const uint64_t *)(cnt + q * n + lo),
                                                        outs[q] + 1, (int)nk, st));
            }
            // the chunk's term totals size its term area: one small read-back
            // (waits for this chunk only; later chunks keep copying), stored
            // by a kernel into pinned memory rather than copied by the DMA
            // engine that is busy with the next chunks
            volatile uint64_t *tot = c->p_small.as<volatile uint64_t>();
            hipLaunchKernelGGL(k_put2_host, dim3(1), dim3(64), 0, st, io + nk, co + nk,
                               (uint64_t *)c->p_small.p);
            MH_HIP(hipGetLastError());
            MH_HIP(hipStreamSynchronize(st));
            MH_HIP(tb.ensure(std::max<uint64_t>(tot[0] + tot[1], 1) * 32));
            uint8_t *dti = tb.as<uint8_t>(), *dtc = dti + tot[0] * 32;
            mh_tx_header *hd = (mh_tx_header *)(base + b_hd) + 2 * lo,
                         *hh = (mh_tx_header *)(base + b_hh) + 2 * lo;
            hipLaunchKernelGGL(k_pbd_dual<true>, dim3(grid), dim3(256), 0, st, nk, dmsg, doff,
                               nullptr, nullptr, nullptr, io, co, mo, dti, dtc, hd, hd + nk, md, dst);
            MH_HIP(hipGetLastError());
            // VerifyDualProofV2 (verification.go:303-370)
            uint64_t *ii = (uint64_t *)(base + b_ii) + lo, *ij = (uint64_t *)(base + b_ij) + lo,
                     *ci = (uint64_t *)(base + b_ci) + lo;
            const uint64_t *dsrc = (const uint64_t *)(base + b_src) + lo,
                           *dtgt = (const uint64_t *)(base + b_tgt) + lo;
            uint8_t *x = base + b_x + 2 * lo * 32, *leaf = base + b_leaf + lo * 32,
                    *sbl = base + b_sbl + lo * 32, *tbl = base + b_tbl + lo * 32,
                    *ca = base + b_ca + lo * 32, *sel = base + b_sel + lo, *oki = base + b_oki + lo,
                    *okc = base + b_okc + lo;
            int32_t *ast = (int32_t *)(base + b_ast) + 2 * lo;
            // the chunk's Alh values source-then-target, as the Alh kernel reads them
            MH_HIP(hipMemcpyAsync(x, base + b_xa + lo * 32, nk * 32, hipMemcpyDeviceToDevice, st));
            MH_HIP(hipMemcpyAsync(x + nk * 32, base + b_xa + (n + lo) * 32, nk * 32,
                                  hipMemcpyDeviceToDevice, st));
            hipLaunchKernelGGL(k_dpv2_prep, dim3(grid), dim3(256), 0, st, nk, hd, dsrc, dtgt, dst, hh,
                               ii, ij, ci, sel, sbl, tbl);
            MH_HIP(hipGetLastError());
            MH_HIP(launch_tx_alh(st, c->tm(), 2 * nk, hh, md, nullptr,
                                 base + b_s + 2 * lo * kTxInnerStride, x, nullptr, nullptr, nullptr,
                                 ast));
            MH_HIP(launch_leaf_for(st, c->tm(), nk, x, leaf));
            MH_HIP(launch_ahtree_verify(st, c->tm(), MH_AHT_INCLUSION, nk, ii, ij, io, dti, leaf,
                                        tbl, oki, nullptr));
            MH_HIP(launch_select32(st, nk, sel, leaf, sbl, ca));
            MH_HIP(launch_ahtree_verify(st, c->tm(), MH_AHT_CONSISTENCY, nk, ci, ij, co, dtc, ca,
                                        tbl, okc, nullptr));
            hipLaunchKernelGGL(k_dpv2_final, dim3(grid), dim3(256), 0, st, nk, hd, dsrc, dtgt, ast,
                               oki, okc, dst);
            MH_HIP(hipGetLastError());
        }
        MH_HIP(cc.join());
        MH_HIP(hipMemcpyAsync(status, dst_all, n * 4, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}
