// capi_app.hip -- the appendable file framing around the ahtree record
// streams ("stream GPU dLog output straight into the
// ahtree appendables"), host code only.
//
// An ahtree keeps three multi-file appendables, data/ (pLog), tree/ (dLog)
// and commit/ (cLog) (ahtree.go:106-140).  Each is a multiapp
// (multi_app.go:120-196): file NNNNNNNN.<ext> holds logical bytes
// [id * fileSize, (id + 1) * fileSize) of the log (appendableID, :208-214),
// and every file is a singleapp (single_app.go:116-171) that starts with
//   BE32 len(m) || m,   m = appendable.Metadata.Bytes() (metadata.go) of
//   { PREALLOC_SIZE, COMPRESSION_FORMAT, COMPRESSION_LEVEL,
//     WRAPPED_METADATA = { FILE_SIZE, WRAPPED_METADATA = { VERSION: 1 } } }
// followed by the log bytes at fileBaseOffset = 4 + len(m).  With these and
// the record streams the device already produces (mh_ahtree_append_batch_logs,
// mh_dev_ahtree_append_batch_logs, the dLog), a caller can place a batch's
// bytes at their file positions directly.
//
// Metadata.Bytes(): field(BE32 count) then field(key) field(value) per entry,
// field(x) = BE32 len(x) || x, integers as BE64 (metadata.go:33-110).  Go
// writes the entries in map order, which varies run to run; any order reads
// back the same.  Here they are written in the caller's order (the header
// helper uses sorted keys).
#include <cstdint>

#include "capi_internal.hpp"

namespace {

struct Out {  // bounded writer: counts every byte, copies while they fit
    uint8_t *p;
    uint64_t cap, len = 0;
    void put(const void *src, uint64_t n) {
        if (p && len + n <= cap) memcpy(p + len, src, n);
        len += n;
    }
    void be32(uint32_t x) {
        const uint8_t b[4] = {(uint8_t)(x >> 24), (uint8_t)(x >> 16), (uint8_t)(x >> 8), (uint8_t)x};
        put(b, 4);
    }
};

using Bytes = std::vector<uint8_t>;

Bytes be64v(int64_t v) {
    Bytes b(8);
    for (int k = 0; k < 8; k++) b[k] = (uint8_t)((uint64_t)v >> (56 - 8 * k));
    return b;
}

void field(Bytes &b, const void *src, uint64_t n) {
    for (int k = 3; k >= 0; k--) b.push_back((uint8_t)(n >> (8 * k)));
    b.insert(b.end(), (const uint8_t *)src, (const uint8_t *)src + n);
}

// Metadata.Bytes() (metadata.go:33-80) of (key, value) pairs in the given order
Bytes metadata_bytes(const std::vector<std::pair<std::string, Bytes>> &kv) {
    Bytes b;
    const uint32_t c = (uint32_t)kv.size();
    const uint8_t cnt[4] = {(uint8_t)(c >> 24), (uint8_t)(c >> 16), (uint8_t)(c >> 8), (uint8_t)c};
    field(b, cnt, 4);
    for (auto &e : kv) {
        field(b, e.first.data(), e.first.size());
        field(b, e.second.data(), e.second.size());
    }
    return b;
}

}  // namespace

extern "C" int mh_appendable_metadata(uint32_t n, const char *const *keys,
                                      const uint8_t *const *vals, const uint64_t *val_len,
                                      uint8_t *out, uint64_t cap, uint64_t *len) {
    return mh_guard([&]() -> int {
        if (!len || (n && (!keys || !vals || !val_len))) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::vector<std::pair<std::string, Bytes>> kv;
        for (uint32_t k = 0; k < n; k++) {
            if (!keys[k] || (val_len[k] && !vals[k])) return MH_ERR_ILLEGAL_ARGUMENTS;
            if (val_len[k] > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;
            kv.emplace_back(keys[k], Bytes(vals[k], vals[k] + val_len[k]));
        }
        const Bytes b = metadata_bytes(kv);
        *len = b.size();
        if (!out || cap < b.size()) return MH_ERR_BUFFER_TOO_SMALL;
        memcpy(out, b.data(), b.size());
        return MH_OK;
    });
}

extern "C" int mh_ahtree_log_header(uint64_t file_size, int64_t prealloc_size,
                                    int32_t compression_format, int32_t compression_level,
                                    uint8_t *out, uint64_t cap, uint64_t *len) {
    return mh_guard([&]() -> int {
        if (!len || file_size == 0 || file_size > (uint64_t)INT64_MAX) return MH_ERR_ILLEGAL_ARGUMENTS;
        // innermost: the ahtree's own metadata (ahtree.go:106-107)
        const Bytes aht = metadata_bytes({{"VERSION", be64v(1)}});
        // multiapp.OpenWithHooks (multi_app.go:152-154)
        const Bytes multi =
            metadata_bytes({{"FILE_SIZE", be64v((int64_t)file_size)}, {"WRAPPED_METADATA", aht}});
        // singleapp.Open of a new file (single_app.go:116-121); PREALLOC_SIZE
        // is absent from files written before it existed (prealloc_size < 0)
        std::vector<std::pair<std::string, Bytes>> top = {
            {"COMPRESSION_FORMAT", be64v(compression_format)},
            {"COMPRESSION_LEVEL", be64v(compression_level)}};
        if (prealloc_size >= 0) top.push_back({"PREALLOC_SIZE", be64v(prealloc_size)});
        top.push_back({"WRAPPED_METADATA", multi});
        const Bytes m = metadata_bytes(top);
        Out o{out, cap};
        o.be32((uint32_t)m.size());
        o.put(m.data(), m.size());
        *len = o.len;
        if (!out || cap < o.len) return MH_ERR_BUFFER_TOO_SMALL;
        return MH_OK;
    });
}

extern "C" int mh_multiapp_segments(uint64_t off, uint64_t n, uint64_t file_size,
                                    uint64_t header_len, uint64_t *seg, uint32_t cap,
                                    uint32_t *nseg) {
    return mh_guard([&]() -> int {
        if (!nseg || file_size == 0) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n && off + n < off) return MH_ERR_ILLEGAL_ARGUMENTS;  // wraps around
        const uint64_t total = n ? (off + n - 1) / file_size - off / file_size + 1 : 0;
        if (total > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint32_t k = (uint32_t)total;
        uint64_t done = 0;
        for (uint32_t j = 0; seg && j < k && j < cap; j++) {
            const uint64_t o = off + done;
            const uint64_t id = o / file_size, in = o % file_size;  // appendableID
            const uint64_t take = std::min(n - done, file_size - in);
            seg[4 * j + 0] = id;
            seg[4 * j + 1] = header_len + in;  // fileBaseOffset + offset in the file
            seg[4 * j + 2] = done;
            seg[4 * j + 3] = take;
            done += take;
        }
        *nseg = k;
        return (!seg || k <= cap) ? MH_OK : MH_ERR_BUFFER_TOO_SMALL;
    });
}
