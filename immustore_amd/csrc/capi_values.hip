// capi_values.hip -- the read-side value integrity check behind the C ABI.
//
// readValueAt (embedded/store/immustore.go:3183-3240) reads an entry's value
// into a buffer of its stored length vLen (from the vLog or the value cache)
// and rejects it with ErrCorruptedData when the bytes read are not vLen long
// or their SHA-256 is not the entry's stored hVal (:3235).  Every reader of
// values goes through it -- Get/ReadValue (:3173), the export path (:2694),
// the indexer (indexer.go:547), key readers (key_reader.go:359) -- so a batch
// of them (replay, export, a full-store scrub) is one pass over the values:
// hashes in length-class order (k_sha_varlen) with the compare fused in.
#include "capi_internal.hpp"

extern "C" int mh_dev_verify_values_batch(mh_ctx *c, uint64_t n, const uint8_t *vals,
                                          const uint64_t *off, const uint64_t *vlen,
                                          const uint8_t *hvals, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!off || !hvals || !status))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        MH_HIP(hipSetDevice(c->device));
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->s_sort.ensure(sha_varlen_scratch_bytes(n)));
        MH_HIP(launch_verify_values(c->stream, c->tm(), vals, off, n, vlen, hvals, status,
                                    c->s_sort.as<uint8_t>()));
        return MH_OK;
    });
}

namespace {
constexpr uint64_t kValChunk = 64ull << 20;  // value bytes per pipelined chunk
}

// Host memory in and out.  The per-entry arrays go up once; the value bytes
// go up in chunks of ~64 MiB on the context's copy stream, double-buffered,
// while the compute stream checks the previous chunk (the call is bound by
// the PCIe copy of the values; the hashing hides under it).
extern "C" int mh_verify_values_batch(mh_ctx *c, uint64_t n, const uint8_t *vals,
                                      const uint64_t *off, const uint64_t *vlen,
                                      const uint8_t *hvals, int32_t *status,
                                      uint64_t *ncorrupted) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!off || !hvals || !status))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (ncorrupted) *ncorrupted = 0;
        if (!n) return MH_OK;
        if (!monotonic(off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (off[n] > off[0] && !vals) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->copy_lane());
        // chunk plan: consecutive entries up to kValChunk value bytes (an
        // entry longer than that is a chunk of its own)
        std::vector<uint64_t> cut{0};
        uint64_t maxb = 0;
        for (uint64_t i = 0; i < n;) {
            uint64_t j = i + 1;
            while (j < n && off[j + 1] - off[cut.back()] <= kValChunk) j++;
            maxb = std::max(maxb, off[j] - off[i]);
            cut.push_back(j);
            i = j;
        }
        Layout L;
        const uint64_t b_off = L.add((n + 1) * 8), b_len = L.add(vlen ? n * 8 : 0),
                       b_hv = L.add(n * 32), b_st = L.add(n * 4);
        MH_HIP(c->s_msgs.ensure(L.total));
        MH_HIP(c->s_sort.ensure(sha_varlen_scratch_bytes(n)));
        for (int s = 0; s < 2; s++) MH_HIP(c->s_chunk[s].ensure(maxb + 16));
        uint8_t *base = c->s_msgs.as<uint8_t>();
        uint64_t *d_off = reinterpret_cast<uint64_t *>(base + b_off);
        uint64_t *d_len = vlen ? reinterpret_cast<uint64_t *>(base + b_len) : nullptr;
        uint8_t *d_hv = base + b_hv;
        int32_t *d_st = reinterpret_cast<int32_t *>(base + b_st);
        hipStream_t cs = c->copy_stream, st = c->stream;
        // an error below may leave copies of the caller's values in flight:
        // wait for them on every way out
        struct CopyGuard {
            hipStream_t s;
            ~CopyGuard() { hipStreamSynchronize(s); }
        } copy_guard{cs};
        MH_HIP(hipMemcpyAsync(d_off, off, (n + 1) * 8, hipMemcpyHostToDevice, st));
        if (vlen) MH_HIP(hipMemcpyAsync(d_len, vlen, n * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(d_hv, hvals, n * 32, hipMemcpyHostToDevice, st));
        // the slots are free once the compute stream has passed everything
        // queued on it so far
        for (int s = 0; s < 2; s++) MH_HIP(hipEventRecord(c->ev_done[s], st));
        for (size_t k = 0; k + 1 < cut.size(); k++) {
            const int s = (int)(k & 1);
            const uint64_t lo = cut[k], hi = cut[k + 1], bytes = off[hi] - off[lo];
            uint8_t *slot = c->s_chunk[s].as<uint8_t>();
            MH_HIP(hipStreamWaitEvent(cs, c->ev_done[s], 0));
            if (bytes) MH_HIP(hipMemcpyAsync(slot, vals + off[lo], bytes, hipMemcpyHostToDevice, cs));
            MH_HIP(hipEventRecord(c->ev_copied[s], cs));
            MH_HIP(hipStreamWaitEvent(st, c->ev_copied[s], 0));
            // absolute offsets: the slot seen through a base shifted by off[lo]
            const uint8_t *vb = reinterpret_cast<const uint8_t *>((uintptr_t)slot - (uintptr_t)off[lo]);
            MH_HIP(launch_verify_values(st, c->tm(), vb, d_off + lo, hi - lo,
                                        d_len ? d_len + lo : nullptr, d_hv + lo * 32, d_st + lo,
                                        c->s_sort.as<uint8_t>()));
            MH_HIP(hipEventRecord(c->ev_done[s], st));
        }
        MH_HIP(hipMemcpyAsync(status, d_st, n * 4, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        if (ncorrupted) {
            uint64_t bad = 0;
            for (uint64_t i = 0; i < n; i++) bad += status[i] != MH_OK;
            *ncorrupted = bad;
        }
        return MH_OK;
    });
}
