// capi_wire.hip -- C ABI of the wire-format writers:
// protobuf InclusionProof / DualProofV2 messages built on the device
// (wire_kernels.hip).  Host variants: inputs copied in, sizes pass, one
// 8-byte read of the total, write pass, one copy of the packed messages out.
#include "capi_internal.hpp"

extern "C" uint64_t mh_pb_scratch_size(uint64_t n) { return pb_scratch_bytes(n); }

extern "C" int mh_dev_htree_inclusion_proof_pb_batch(mh_ctx *c, int phase, const uint8_t *levels,
                                                     uint64_t width, uint64_t n,
                                                     const uint64_t *leaf, uint8_t *out,
                                                     uint64_t out_cap, uint64_t *off,
                                                     int32_t *status, void *scratch) {
    return mh_guard([&]() -> int {
        if (!c || phase < 1 || phase > 3 || !off) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n && (!leaf || !status || !scratch || (width && !levels) || ((phase & 2) && !out && out_cap)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        hipSetDevice(c->device);
        MH_HIP(launch_pb_inclusion(c->stream, c->tm(), phase, levels, width, n, leaf, out, out_cap, off,
                                   status, (uint8_t *)scratch));
        return MH_OK;
    });
}

extern "C" int mh_dev_dual_proof_v2_pb_batch(mh_ctx *c, int phase, const uint8_t *dlog,
                                             uint64_t size, uint64_t n, const mh_tx_header *src,
                                             const mh_tx_header *tgt, const uint8_t *md_blob,
                                             uint8_t *out, uint64_t out_cap, uint64_t *off,
                                             int32_t *status, void *scratch) {
    return mh_guard([&]() -> int {
        if (!c || phase < 1 || phase > 3 || !off) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n && (!src || !tgt || !status || !scratch || (size && !dlog) ||
                  ((phase & 2) && !out && out_cap)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        hipSetDevice(c->device);
        MH_HIP(launch_pb_dual_v2(c->stream, c->tm(), phase, dlog, size, n, src, tgt, md_blob, out,
                                 out_cap, off, status, (uint8_t *)scratch));
        return MH_OK;
    });
}

// Shared host flow: launch(phase) runs on st with device off / status;
// returns after out / off / status are in host memory.
template <class Launch>
static int pb_host(hipStream_t st, DevBuf &wout, uint64_t n, uint64_t *d_off, int32_t *d_status,
                   uint8_t *out, uint64_t out_cap, uint64_t *off, int32_t *status,
                   Launch &&launch) {
    MH_HIP(launch(1, nullptr, 0));
    uint64_t total = 0;
    MH_HIP(hipMemcpyAsync(&total, d_off + n, 8, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    if (total > out_cap || (total && !out)) {
        MH_HIP(hipMemcpyAsync(off, d_off, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(status, d_status, n * 4, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_ERR_BUFFER_TOO_SMALL;
    }
    MH_HIP(wout.ensure(total ? total : 16));
    MH_HIP(launch(2, wout.as<uint8_t>(), total));
    if (total) MH_HIP(hipMemcpyAsync(out, wout.p, total, hipMemcpyDeviceToHost, st));
    MH_HIP(hipMemcpyAsync(off, d_off, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    MH_HIP(hipMemcpyAsync(status, d_status, n * 4, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    return MH_OK;
}

extern "C" int mh_htree_inclusion_proof_pb_batch(mh_htree *t, uint64_t n, const uint64_t *leaf,
                                                 uint8_t *out, uint64_t out_cap, uint64_t *off,
                                                 int32_t *status) {
    return mh_guard([&]() -> int {
        if (!t || !off || (n && (!leaf || !status))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) {
            off[0] = 0;
            return MH_OK;
        }
        hipSetDevice(t->ctx->device);
        hipStream_t st = t->stream;
        Layout L;
        const uint64_t b_leaf = L.add(n * 8), b_off = L.add((n + 1) * 8), b_st = L.add(n * 4),
                       b_s = L.add(pb_scratch_bytes(n));
        MH_HIP(t->w_in.ensure(L.total));
        uint8_t *base = t->w_in.as<uint8_t>();
        MH_HIP(hipMemcpyAsync(base + b_leaf, leaf, n * 8, hipMemcpyHostToDevice, st));
        uint64_t *d_off = (uint64_t *)(base + b_off);
        int32_t *d_st = (int32_t *)(base + b_st);
        const uint8_t *lv = t->levels.as<uint8_t>();
        const uint64_t w = t->width;
        Timer *tm = t->ctx->tm();
        return pb_host(st, t->w_out, n, d_off, d_st, out, out_cap, off, status,
                       [&](int phase, uint8_t *dout, uint64_t cap) {
                           return launch_pb_inclusion(st, tm, phase, lv, w, n,
                                                      (const uint64_t *)(base + b_leaf), dout, cap,
                                                      d_off, d_st, base + b_s);
                       });
    });
}

extern "C" int mh_ahtree_dual_proof_v2_pb_batch(mh_ahtree *t, uint64_t n, const mh_tx_header *src,
                                                const mh_tx_header *tgt, const uint8_t *md_blob,
                                                uint64_t md_blob_len, uint8_t *out,
                                                uint64_t out_cap, uint64_t *off, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!t || !off || (n && (!src || !tgt || !status))) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        if (!n) {
            off[0] = 0;
            return MH_OK;
        }
        for (uint64_t k = 0; k < n; k++) {
            if (int e = check_header(src[k], md_blob_len, md_blob != nullptr)) return e;
            if (int e = check_header(tgt[k], md_blob_len, md_blob != nullptr)) return e;
        }
        hipSetDevice(t->ctx->device);
        hipStream_t st = t->stream;
        Layout L;
        const uint64_t b_src = L.add(n * sizeof(mh_tx_header)), b_tgt = L.add(n * sizeof(mh_tx_header)),
                       b_md = L.add(md_blob_len), b_off = L.add((n + 1) * 8), b_st = L.add(n * 4),
                       b_s = L.add(pb_scratch_bytes(n));
        MH_HIP(t->w_in.ensure(L.total));
        uint8_t *base = t->w_in.as<uint8_t>();
        MH_HIP(hipMemcpyAsync(base + b_src, src, n * sizeof(mh_tx_header), hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_tgt, tgt, n * sizeof(mh_tx_header), hipMemcpyHostToDevice, st));
        if (md_blob && md_blob_len)
            MH_HIP(hipMemcpyAsync(base + b_md, md_blob, md_blob_len, hipMemcpyHostToDevice, st));
        uint64_t *d_off = (uint64_t *)(base + b_off);
        int32_t *d_st = (int32_t *)(base + b_st);
        const uint8_t *dl = t->dlog.as<uint8_t>();
        const uint64_t size = t->size;
        Timer *tm = t->ctx->tm();
        return pb_host(st, t->w_out, n, d_off, d_st, out, out_cap, off, status,
                       [&](int phase, uint8_t *dout, uint64_t cap) {
                           return launch_pb_dual_v2(st, tm, phase, dl, size, n,
                                                    (const MhTxHeader *)(base + b_src),
                                                    (const MhTxHeader *)(base + b_tgt), base + b_md,
                                                    dout, cap, d_off, d_st, base + b_s);
                       });
    });
}
