// capi.hip -- implementation of the C ABI declared in include/immustore_merkle.h.
//
// Host-side mirror of the reference's Go objects (embedded/htree.HTree,
// embedded/ahtree.AHtree) written in C++ (the reference is compiled Go; no Go
// toolchain exists in this image).  All hashing runs in the HIP kernels of
// htree_kernels.hip / ahtree_kernels.hip / verify_kernels.hip; the host code
// here only moves bytes, computes indices and reports errors.  There is no
// CPU hashing fallback: without a usable device every entry point returns
// MH_ERR_NO_DEVICE.
#include <atomic>
#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "capi_internal.hpp"


namespace mh {
hipError_t launch_copy_nodes(hipStream_t st, const uint8_t *src, uint64_t n, uint8_t *dst);
}

// ------------------------------------------------------------------ misc
extern "C" int mh_abi_version(void) { return MH_ABI_VERSION; }

namespace {
std::atomic<int> g_fault[4];
}

bool mh_fault(int site) {
    if (site <= 0 || site >= 4 || g_fault[site].load(std::memory_order_relaxed) <= 0) return false;
    return g_fault[site].fetch_sub(1) == 1;
}

extern "C" int mh_debug_fail_at(int site, int countdown) {
    if (site <= 0 || site >= 4 || countdown < 0) return MH_ERR_ILLEGAL_ARGUMENTS;
    g_fault[site].store(countdown);
    return MH_OK;
}

extern "C" const char *mh_status_string(int st) {
    switch (st) {
        case MH_OK: return "ok";
        case MH_ERR_MAX_WIDTH_EXCEEDED: return "htree: max width exceeded";
        case MH_ERR_ILLEGAL_ARGUMENTS: return "illegal arguments";
        case MH_ERR_ILLEGAL_STATE: return "htree: illegal state";
        case MH_ERR_EMPTY_TREE: return "ahtree: empty tree";
        case MH_ERR_UNEXISTENT_DATA: return "ahtree: attempt to read unexistent data";
        case MH_ERR_METADATA_UNSUPPORTED: return "metadata is unsupported when in 1.1 compatibility mode";
        case MH_ERR_CANNOT_RESET_TO_LARGER: return "ahtree: can not reset the tree to a larger size";
        case MH_ERR_NO_DEVICE: return "no usable gfx950 device";
        case MH_ERR_OUT_OF_MEMORY: return "out of device memory";
        case MH_ERR_SOURCE_TX_NEWER: return "illegal arguments: source tx is newer than target tx";
        case MH_ERR_UNEXPECTED_LINKING:
            return "internal inconsistency between linear and binary linking";
        case MH_ERR_INCLUSION_NOT_VALID: return "inclusion proof does NOT validate";
        case MH_ERR_CONSISTENCY_NOT_VALID: return "consistency proof does NOT validate";
        case MH_ERR_CORRUPTED_DATA: return "data is corrupted";
        case MH_ERR_CORRUPTED_MAX_ENTRIES:
            return "tx data is corrupted: maximum number of TX entries exceeded";
        case MH_ERR_CORRUPTED_MAX_KEYLEN: return "tx data is corrupted: maximum key length exceeded";
        case MH_ERR_CORRUPTED_UNKNOWN_VERSION: return "tx data is corrupted: unknown TX header version";
        case MH_ERR_TRUNCATED: return "unexpected EOF";
        case MH_ERR_BUFFER_TOO_SMALL: return "output buffer too small";
        case MH_ERR_INVALID_PROOF: return "invalid proof";
        case MH_ERR_UNSUPPORTED_TX_VERSION: return "unsupported tx version";
        case MH_ERR_INVALID_PROOF_ENTRY: return "invalid proof: document entry";
        case MH_ERR_COLLECTIVE: return "RCCL collective failed or RCCL not available";
        default: return st < 0 ? hipGetErrorString((hipError_t)(-st)) : "unknown status";
    }
}

extern "C" int mh_device_count(int *count) {
    return mh_guard([&]() -> int {
        if (!count) return MH_ERR_ILLEGAL_ARGUMENTS;
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess) {
            *count = 0;
            return MH_ERR_NO_DEVICE;
        }
        *count = n;
        return MH_OK;
    });
}

static int map_alloc(hipError_t e) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return MH_ERR_OUT_OF_MEMORY;
    return e == hipSuccess ? MH_OK : -(int)e;
}

// ------------------------------------------------------------------ context
extern "C" int mh_ctx_create(int device_ordinal, void *hip_stream, mh_ctx **out) {
    return mh_guard([&]() -> int {
        if (!out) return MH_ERR_ILLEGAL_ARGUMENTS;
        *out = nullptr;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return MH_ERR_NO_DEVICE;
        if (device_ordinal < 0 || device_ordinal >= n) return MH_ERR_ILLEGAL_ARGUMENTS;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device_ordinal) != hipSuccess) return MH_ERR_NO_DEVICE;
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return MH_ERR_NO_DEVICE;
        MH_HIP(hipSetDevice(device_ordinal));
        mh_ctx *c = new (std::nothrow) mh_ctx();
        if (!c) return MH_ERR_OUT_OF_MEMORY;
        c->device = device_ordinal;
        if (hip_stream) {
            c->stream = (hipStream_t)hip_stream;
        } else {
            hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
            if (e != hipSuccess) {
                delete c;
                return -(int)e;
            }
            c->own_stream = true;
        }
        *out = c;
        return MH_OK;
    });
}

extern "C" int mh_ctx_destroy(mh_ctx *c) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        hipSetDevice(c->device);
        hipStreamSynchronize(c->stream);
        if (c->own_stream) hipStreamDestroy(c->stream);
        delete c;
        return MH_OK;
    });
}

extern "C" int mh_ctx_synchronize(mh_ctx *c) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        MH_HIP(hipStreamSynchronize(c->stream));
        return MH_OK;
    });
}

extern "C" void *mh_ctx_stream(mh_ctx *c) { return c ? (void *)c->stream : nullptr; }

extern "C" int mh_ctx_set_timing(mh_ctx *c, int enable) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        c->timer.enabled = enable != 0;
        return MH_OK;
    });
}

extern "C" int mh_ctx_timing(mh_ctx *c, const char *prefix, double *total_ms, uint64_t *launches) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        return c->timer.sum(prefix, total_ms, launches);
    });
}

extern "C" int mh_ctx_timing_reset(mh_ctx *c) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        c->timer.reset();
        return MH_OK;
    });
}

extern "C" int mh_dev_alloc(mh_ctx *c, uint64_t bytes, void **dptr) {
    return mh_guard([&]() -> int {
        if (!c || !dptr) return MH_ERR_ILLEGAL_ARGUMENTS;
        hipSetDevice(c->device);
        return map_alloc(hipMalloc(dptr, std::max<uint64_t>(bytes, 1)));
    });
}

extern "C" int mh_dev_free(mh_ctx *c, void *dptr) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        MH_HIP(hipFree(dptr));
        return MH_OK;
    });
}

extern "C" int mh_host_alloc_pinned(uint64_t bytes, void **hptr) {
    return mh_guard([&]() -> int {
        if (!hptr) return MH_ERR_ILLEGAL_ARGUMENTS;
        return map_alloc(hipHostMalloc(hptr, std::max<uint64_t>(bytes, 1), hipHostMallocDefault));
    });
}

extern "C" int mh_host_free_pinned(void *hptr) {
    return mh_guard([&]() -> int {
        MH_HIP(hipHostFree(hptr));
        return MH_OK;
    });
}

extern "C" int mh_memcpy_h2d(mh_ctx *c, void *dst, const void *src, uint64_t bytes) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (!bytes) return MH_OK;
        MH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
        return MH_OK;
    });
}

extern "C" int mh_memcpy_d2h(mh_ctx *c, void *dst, const void *src, uint64_t bytes) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (!bytes) return MH_OK;
        MH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
        return MH_OK;
    });
}

extern "C" int mh_dev_fill_random(mh_ctx *c, void *dptr, uint64_t nbytes, uint64_t seed) {
    return mh_guard([&]() -> int {
        if (!c || (!dptr && nbytes)) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (!nbytes) return MH_OK;
        MH_HIP(launch_fill_random(c->stream, (uint8_t *)dptr, nbytes, seed));
        return MH_OK;
    });
}

extern "C" int mh_dev_fill_keys_be64(mh_ctx *c, void *dptr, uint64_t n, uint64_t first) {
    return mh_guard([&]() -> int {
        if (!c || (!dptr && n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (((uintptr_t)dptr) & 7) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(launch_fill_keys_be64(c->stream, (uint8_t *)dptr, n, first));
        return MH_OK;
    });
}

// ------------------------------------------------------------------ htree core
extern "C" uint64_t mh_htree_levels_len(uint64_t n) {
    LevelGeom g;
    g.init(n);
    return g.total;
}

extern "C" uint64_t mh_htree_level_offset(uint64_t n, int level) {
    LevelGeom g;
    g.init(n);
    if (level < 0 || level >= kMaxLevels) return 0;
    if (level >= g.nlevels) return g.total;
    return g.off[level];
}

static int write_root(hipStream_t st, const LevelGeom &g, uint8_t *levels, uint8_t *root,
                      bool in_kernel = false) {
    if (!root || in_kernel) return MH_OK;
    if (g.n == 0) {
        MH_HIP(hipMemcpyAsync(root, kEmptyRoot, 32, hipMemcpyHostToDevice, st));
        return MH_OK;
    }
    MH_HIP(hipMemcpyAsync(root, levels + g.off[g.nlevels - 1] * 32, 32, hipMemcpyDeviceToDevice, st));
    return MH_OK;
}

// Fused fixed-stride path (device pointers, stream st).
static int build_fixed(hipStream_t st, Timer *tm, int version, uint64_t n, const uint8_t *keys,
                       uint32_t key_len, const uint8_t *vals, uint32_t val_len, uint8_t *hvals_out,
                       uint8_t *levels, const LevelGeom &g, uint8_t *root = nullptr,
                       bool *root_done = nullptr) {
    int done = 0;
    MH_HIP(launch_entries_fixed(st, tm, version, n, keys, key_len, vals, val_len, hvals_out, levels,
                                g, &done));
    // the last k_reduce launch stores the root itself when there is one
    MH_HIP(launch_reduce(st, tm, levels, g, done, root));
    if (root_done) *root_done = root && done < g.nlevels - 1;
    return MH_OK;
}

static int build_digests(hipStream_t st, Timer *tm, const uint8_t *digests, uint64_t n,
                         uint8_t *levels, const LevelGeom &g, uint8_t *root = nullptr,
                         bool *root_done = nullptr) {
    int done = 0;
    MH_HIP(launch_leaves_from_digests(st, tm, digests, n, levels, g, &done));
    MH_HIP(launch_reduce(st, tm, levels, g, done, root));
    if (root_done) *root_done = root && done < g.nlevels - 1;
    return MH_OK;
}

// General CSR path (ragged keys / metadata / values, hVal overrides): value
// hashes, entry digests and leaves in one fused launch (varlen_kernels.hip),
// then the levels above the leaves.
static int build_csr(hipStream_t st, Timer *tm, int version, uint64_t n, const uint8_t *keys,
                     const uint64_t *key_off, const uint8_t *md, const uint64_t *md_off,
                     const uint8_t *vals, const uint64_t *val_off, const uint8_t *ov,
                     const uint8_t *use, uint8_t *hvals, uint8_t *levels, const LevelGeom &g,
                     DevBuf &sort) {
    MH_HIP(sort.ensure(sha_varlen_scratch_bytes(n)));
    MH_HIP(launch_entries_varlen(st, tm, version, n, keys, key_off, md, md_off, vals, val_off, ov,
                                 use, hvals, levels, true, sort.as<uint8_t>()));
    MH_HIP(launch_reduce(st, tm, levels, g, 0));
    return MH_OK;
}

extern "C" int mh_dev_htree_build_digests(mh_ctx *c, const uint8_t *digests, uint64_t n,
                                          uint8_t *levels, uint8_t *root) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!digests || !levels))) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (((uintptr_t)digests & 15) || ((uintptr_t)levels & 15)) return MH_ERR_ILLEGAL_ARGUMENTS;
        LevelGeom g;
        g.init(n);
        bool rk = false;
        if (n) {
            int st = build_digests(c->stream, c->tm(), digests, n, levels, g, root, &rk);
            if (st) return st;
        }
        return write_root(c->stream, g, levels, root, rk);
    });
}

extern "C" int mh_dev_htree_build_entries_fixed(mh_ctx *c, int version, uint64_t n,
                                                const uint8_t *keys, uint32_t key_len,
                                                const uint8_t *vals, uint32_t val_len,
                                                uint8_t *hvals_out, uint8_t *levels, uint8_t *root) {
    return mh_guard([&]() -> int {
        if (!c || (version != 0 && version != 1)) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (n && (!levels || (!keys && key_len) || (!vals && val_len))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (((uintptr_t)levels & 15) || ((uintptr_t)hvals_out & 15)) return MH_ERR_ILLEGAL_ARGUMENTS;
        LevelGeom g;
        g.init(n);
        bool rk = false;
        if (n) {
            if (entries_fixed_supported(version, keys, key_len, vals, val_len)) {
                int st = build_fixed(c->stream, c->tm(), version, n, keys, key_len, vals, val_len,
                                     hvals_out, levels, g, root, &rk);
                if (st) return st;
            } else {
                // odd shapes: general CSR path over generated offsets
                std::lock_guard<std::mutex> lk(c->mu);
                MH_HIP(c->s_offs.ensure(2 * (n + 1) * sizeof(uint64_t)));
                uint64_t *koff = c->s_offs.as<uint64_t>(), *voff = koff + (n + 1);
                MH_HIP(launch_iota_offsets(c->stream, koff, n, key_len));
                MH_HIP(launch_iota_offsets(c->stream, voff, n, val_len));
                int st = build_csr(c->stream, c->tm(), version, n, keys, koff, nullptr, nullptr, vals,
                                   voff, nullptr, nullptr, hvals_out, levels, g, c->s_sort);
                if (st) return st;
            }
        }
        return write_root(c->stream, g, levels, root, rk);
    });
}

extern "C" int mh_dev_htree_build_entries(mh_ctx *c, int version, uint64_t n, const uint8_t *keys,
                                          const uint64_t *key_off, const uint8_t *md,
                                          const uint64_t *md_off, const uint8_t *vals,
                                          const uint64_t *val_off, const uint8_t *hval_override,
                                          const uint8_t *use_override, uint8_t *hvals_out,
                                          uint8_t *levels, uint8_t *root) {
    return mh_guard([&]() -> int {
        if (!c || (version != 0 && version != 1)) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (n && (!levels || !key_off || !val_off)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((hval_override == nullptr) != (use_override == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        LevelGeom g;
        g.init(n);
        if (n) {
            if (version == 0 && md_off) {
                // v0 + KV metadata is rejected up front (tx.go:691-693): one
                // small D2H of the metadata bounds
                uint64_t mb[2] = {0, 0};
                MH_HIP(hipMemcpyAsync(&mb[0], md_off, 8, hipMemcpyDeviceToHost, c->stream));
                MH_HIP(hipMemcpyAsync(&mb[1], md_off + n, 8, hipMemcpyDeviceToHost, c->stream));
                MH_HIP(hipStreamSynchronize(c->stream));
                if (mb[1] != mb[0]) return MH_ERR_METADATA_UNSUPPORTED;
            }
            std::lock_guard<std::mutex> lk(c->mu);
            int st = build_csr(c->stream, c->tm(), version, n, keys, key_off, md, md_off, vals, val_off,
                               hval_override, use_override, hvals_out, levels, g, c->s_sort);
            if (st) return st;
        }
        return write_root(c->stream, g, levels, root);
    });
}

extern "C" int mh_dev_htree_reduce_nodes(mh_ctx *c, const uint8_t *nodes, uint64_t w,
                                         uint8_t *levels, uint8_t *root) {
    return mh_guard([&]() -> int {
        if (!c || (w && (!nodes || !levels))) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (((uintptr_t)nodes & 15) || ((uintptr_t)levels & 15)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (w >= 1 && w <= kSmallTreeMax) {  // one launch (every multi-GPU step)
            MH_HIP(launch_reduce_small(c->stream, nodes, w, levels, root));
            return MH_OK;
        }
        LevelGeom g;
        g.init(w);
        if (w) {
            MH_HIP(launch_copy_nodes(c->stream, nodes, w, levels));
            MH_HIP(launch_reduce(c->stream, c->tm(), levels, g, 0));
        }
        return write_root(c->stream, g, levels, root);
    });
}

extern "C" int mh_dev_sha256_batch(mh_ctx *c, const uint8_t *buf, const uint64_t *off, uint64_t n,
                                   uint8_t *out) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!off || !out))) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->s_sort.ensure(sha_varlen_scratch_bytes(n)));
        MH_HIP(launch_sha256_csr(c->stream, c->tm(), buf, off, n, nullptr, nullptr, out,
                                 c->s_sort.as<uint8_t>()));
        return MH_OK;
    });
}

// ------------------------------------------------------------------ htree handle
extern "C" int mh_htree_new(mh_ctx *c, uint64_t max_width, mh_htree **out) {
    return mh_guard([&]() -> int {
        if (!c || !out) return MH_ERR_ILLEGAL_ARGUMENTS;
        *out = nullptr;
        hipSetDevice(c->device);
        mh_htree *t = new (std::nothrow) mh_htree();
        if (!t) return MH_ERR_OUT_OF_MEMORY;
        t->ctx = c;
        t->max_width = max_width;
        memcpy(t->root, kEmptyRoot, 32);
        hipError_t e = hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete t;
            return -(int)e;
        }
        if (max_width) {
            e = t->levels.ensure(mh_htree_levels_len(max_width) * 32);
            if (e != hipSuccess) {
                hipStreamDestroy(t->stream);
                delete t;
                return map_alloc(e);
            }
        }
        *out = t;
        return MH_OK;
    });
}

extern "C" int mh_htree_free(mh_htree *t) {
    return mh_guard([&]() -> int {
        if (!t) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(t->ctx->device));
        hipStreamSynchronize(t->stream);
        hipStreamDestroy(t->stream);
        if (t->pinned) hipHostFree(t->pinned);
        delete t;
        return MH_OK;
    });
}

static int stage_h2d(mh_htree *t, DevBuf &dst, const void *src, uint64_t bytes) {
    MH_HIP(dst.ensure(bytes));
    if (bytes) MH_HIP(hipMemcpyAsync(dst.p, src, bytes, hipMemcpyHostToDevice, t->stream));
    return MH_OK;
}

static int finish_build(mh_htree *t, uint64_t n) {
    t->geom.init(n);
    t->width = n;
    if (n == 0) {
        memcpy(t->root, kEmptyRoot, 32);
        return MH_OK;
    }
    MH_HIP(hipMemcpyAsync(t->root, t->levels.as<uint8_t>() + t->geom.off[t->geom.nlevels - 1] * 32, 32,
                          hipMemcpyDeviceToHost, t->stream));
    MH_HIP(hipStreamSynchronize(t->stream));
    return MH_OK;
}

extern "C" int mh_htree_build_with(mh_htree *t, const uint8_t *digests, uint64_t n) {
    return mh_guard([&]() -> int {
        if (!t || (n && !digests)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n > t->max_width) return MH_ERR_MAX_WIDTH_EXCEEDED;  // htree.go:69-71
        if (n == 0) return finish_build(t, 0);                    // htree.go:73-77
        hipSetDevice(t->ctx->device);
        int st = stage_h2d(t, t->in_a, digests, n * 32);
        if (st) return st;
        LevelGeom g;
        g.init(n);
        st = build_digests(t->stream, t->ctx->tm(), t->in_a.as<uint8_t>(), n, t->levels.as<uint8_t>(), g);
        if (st) return st;
        return finish_build(t, n);
    });
}

static bool is_progression(const uint64_t *off, uint64_t n, uint64_t *stride) {
    if (!off) return false;
    if (off[0] != 0) return false;
    const uint64_t s = n ? off[1] - off[0] : 0;
    for (uint64_t i = 1; i <= n; i++)
        if (off[i] - off[i - 1] != s) return false;
    *stride = s;
    return true;
}

extern "C" int mh_htree_build_entries(mh_htree *t, int version, uint64_t n, const uint8_t *keys,
                                      const uint64_t *key_off, const uint8_t *md,
                                      const uint64_t *md_off, const uint8_t *vals,
                                      const uint64_t *val_off, const uint8_t *hval_override,
                                      const uint8_t *use_override, uint8_t *hvals_out) {
    return mh_guard([&]() -> int {
        if (!t || (version != 0 && version != 1)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n && (!key_off || !val_off)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((hval_override == nullptr) != (use_override == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n > t->max_width) return MH_ERR_MAX_WIDTH_EXCEEDED;
        for (uint64_t i = 0; i < n; i++)
            if (key_off[i + 1] < key_off[i] || val_off[i + 1] < val_off[i] ||
                (md_off && md_off[i + 1] < md_off[i]))
                return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t md_bytes = md_off && n ? md_off[n] - md_off[0] : 0;
        if (version == 0 && md_bytes) return MH_ERR_METADATA_UNSUPPORTED;  // tx.go:691-693
        if (n == 0) return finish_build(t, 0);
        hipSetDevice(t->ctx->device);
        Timer *tm = t->ctx->tm();
        const uint64_t kbytes = key_off[n] - key_off[0], vbytes = val_off[n] - val_off[0];
        LevelGeom g;
        g.init(n);
        int st;
        bool any_override = false;
        if (use_override)
            for (uint64_t i = 0; i < n && !any_override; i++) any_override = use_override[i] != 0;
        uint64_t kstride = 0, vstride = 0;
        uint8_t *hv_dev = nullptr;
        MH_HIP(t->hv.ensure(n * 32));
        hv_dev = t->hv.as<uint8_t>();
        if (!md_bytes && !any_override && is_progression(key_off, n, &kstride) &&
            is_progression(val_off, n, &vstride) && kstride <= 0xffffffffull &&
            vstride <= 0xffffffffull) {
            // uniform shapes: fused kernel (same as BASELINE C1/C2)
            if ((st = stage_h2d(t, t->in_a, keys, kbytes))) return st;
            if ((st = stage_h2d(t, t->in_b, vals, vbytes))) return st;
            if (entries_fixed_supported(version, t->in_a.as<uint8_t>(), (uint32_t)kstride,
                                        t->in_b.as<uint8_t>(), (uint32_t)vstride)) {
                st = build_fixed(t->stream, tm, version, n, t->in_a.as<uint8_t>(), (uint32_t)kstride,
                                 t->in_b.as<uint8_t>(), (uint32_t)vstride, hv_dev,
                                 t->levels.as<uint8_t>(), g);
                if (st) return st;
                goto done;
            }
        }
        {
            // general CSR path: rebase offsets to 0 and stage everything
            std::vector<uint64_t> ko(n + 1), vo(n + 1), mo;
            for (uint64_t i = 0; i <= n; i++) {
                ko[i] = key_off[i] - key_off[0];
                vo[i] = val_off[i] - val_off[0];
            }
            if ((st = stage_h2d(t, t->in_a, keys ? keys + key_off[0] : nullptr, kbytes))) return st;
            if ((st = stage_h2d(t, t->in_b, vals ? vals + val_off[0] : nullptr, vbytes))) return st;
            if ((st = stage_h2d(t, t->off_a, ko.data(), (n + 1) * 8))) return st;
            if ((st = stage_h2d(t, t->off_b, vo.data(), (n + 1) * 8))) return st;
            uint64_t *mo_dev = nullptr;
            if (md_off) {
                mo.resize(n + 1);
                for (uint64_t i = 0; i <= n; i++) mo[i] = md_off[i] - md_off[0];
                if ((st = stage_h2d(t, t->in_c, md ? md + md_off[0] : nullptr, md_bytes))) return st;
                if ((st = stage_h2d(t, t->off_c, mo.data(), (n + 1) * 8))) return st;
                mo_dev = t->off_c.as<uint64_t>();
            }
            const uint8_t *ovd = nullptr, *used = nullptr;
            if (any_override) {
                if ((st = stage_h2d(t, t->ov, hval_override, n * 32))) return st;
                if ((st = stage_h2d(t, t->use, use_override, n))) return st;
                ovd = t->ov.as<uint8_t>();
                used = t->use.as<uint8_t>();
            }
            st = build_csr(t->stream, tm, version, n, t->in_a.as<uint8_t>(), t->off_a.as<uint64_t>(),
                           md_off ? t->in_c.as<uint8_t>() : nullptr, mo_dev, t->in_b.as<uint8_t>(),
                           t->off_b.as<uint64_t>(), ovd, used, hv_dev, t->levels.as<uint8_t>(), g,
                           t->sort);
            if (st) return st;
        }
    done:
        if (hvals_out) MH_HIP(hipMemcpyAsync(hvals_out, hv_dev, n * 32, hipMemcpyDeviceToHost, t->stream));
        return finish_build(t, n);
    });
}

extern "C" int mh_htree_root(mh_htree *t, uint8_t root[32]) {
    return mh_guard([&]() -> int {
        if (!t || !root) return MH_ERR_ILLEGAL_ARGUMENTS;
        memcpy(root, t->root, 32);
        return MH_OK;
    });
}

extern "C" int mh_htree_width(mh_htree *t, uint64_t *width) {
    return mh_guard([&]() -> int {
        if (!t || !width) return MH_ERR_ILLEGAL_ARGUMENTS;
        *width = t->width;
        return MH_OK;
    });
}

static int bits_len64(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

extern "C" int mh_htree_inclusion_proof(mh_htree *t, uint64_t i, uint8_t *terms, uint32_t cap,
                                        uint32_t *nterms) {
    return mh_guard([&]() -> int {
        // htree.go:121-164: index walk on the host, terms gathered from HBM.
        if (!t || !nterms) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(t->ctx->device));
        *nterms = 0;
        if (i >= t->width) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (t->width == 1) return MH_OK;
        uint64_t m = i, n = t->width, offset = 0, l, r;
        uint64_t idx[64];
        uint32_t cnt = 0;
        for (;;) {
            const int d = bits_len64(n - 1);
            const uint64_t k = 1ull << (d - 1);
            if (m < k) {
                l = offset + k;
                r = offset + n - 1;
                n = k;
            } else {
                l = offset;
                r = offset + k - 1;
                m -= k;
                n -= k;
                offset += k;
            }
            const int layer = bits_len64(r - l);
            idx[cnt++] = t->geom.off[layer] + (l >> layer);
            if (n < 1 || (n == 1 && m == 0)) break;
        }
        if (cnt > cap || !terms) return MH_ERR_ILLEGAL_ARGUMENTS;
        // Go prepends each term: output is the reverse discovery order
        for (uint32_t k = 0; k < cnt; k++)
            MH_HIP(hipMemcpyAsync(terms + 32 * k, t->levels.as<uint8_t>() + idx[cnt - 1 - k] * 32, 32,
                                  hipMemcpyDeviceToHost, t->stream));
        MH_HIP(hipStreamSynchronize(t->stream));
        *nterms = cnt;
        return MH_OK;
    });
}

// Batch proof generation on the device.
static int proof_batch_host(mh_ctx *c, hipStream_t st, uint64_t n, const uint64_t *a,
                            const uint64_t *b, uint32_t max_terms, uint8_t *terms,
                            uint32_t *nterms, int32_t *status,
                            const std::function<hipError_t(const uint64_t *, const uint64_t *,
                                                           uint8_t *, uint32_t *, int32_t *)> &run) {
    std::lock_guard<std::mutex> lk(c->mu);
    hipSetDevice(c->device);
    const uint64_t b_a = 0, b_b = (n * 8 + 255) & ~255ull, b_t = b_b + ((n * 8 + 255) & ~255ull),
                   b_n = b_t + ((n * max_terms * 32 + 255) & ~255ull),
                   b_s = b_n + ((n * 4 + 255) & ~255ull), total = b_s + n * 4 + 64;
    MH_HIP(c->s_msgs.ensure(total));
    uint8_t *base = c->s_msgs.as<uint8_t>();
    MH_HIP(hipMemcpyAsync(base + b_a, a, n * 8, hipMemcpyHostToDevice, st));
    if (b) MH_HIP(hipMemcpyAsync(base + b_b, b, n * 8, hipMemcpyHostToDevice, st));
    MH_HIP(run((const uint64_t *)(base + b_a), (const uint64_t *)(base + b_b), base + b_t,
               (uint32_t *)(base + b_n), (int32_t *)(base + b_s)));
    MH_HIP(hipMemcpyAsync(terms, base + b_t, n * max_terms * 32, hipMemcpyDeviceToHost, st));
    MH_HIP(hipMemcpyAsync(nterms, base + b_n, n * 4, hipMemcpyDeviceToHost, st));
    MH_HIP(hipMemcpyAsync(status, base + b_s, n * 4, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    return MH_OK;
}

extern "C" int mh_htree_inclusion_proof_batch(mh_htree *t, uint64_t n, const uint64_t *leaf,
                                              uint8_t *terms, uint32_t max_terms, uint32_t *nterms,
                                              int32_t *status) {
    return mh_guard([&]() -> int {
        if (!t || (n && (!leaf || !terms || !nterms || !status || !max_terms)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(t->ctx->device));
        if (!n) return MH_OK;
        const uint8_t *lv = t->levels.as<uint8_t>();
        const uint64_t w = t->width;
        // the context's scratch is used, so run on the context's stream (after
        // any mh_dev_* work queued there); the handle's own stream is idle
        // between host calls (each one synchronises it before returning)
        hipStream_t st = t->ctx->stream;
        Timer *tm = t->ctx->tm();
        return proof_batch_host(t->ctx, st, n, leaf, nullptr, max_terms, terms, nterms, status,
                                [&](const uint64_t *a, const uint64_t *, uint8_t *tt, uint32_t *nt,
                                    int32_t *ss) {
                                    return launch_htree_proof(st, tm, lv, w, n, a, tt, max_terms, nt,
                                                              ss);
                                });
    });
}

extern "C" int mh_dev_htree_inclusion_proof_batch(mh_ctx *c, const uint8_t *levels, uint64_t width,
                                                  uint64_t n, const uint64_t *leaf, uint8_t *terms,
                                                  uint32_t max_terms, uint32_t *nterms,
                                                  int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!levels || !leaf || !terms || !nterms || !status || !max_terms)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        hipSetDevice(c->device);
        MH_HIP(launch_htree_proof(c->stream, c->tm(), levels, width, n, leaf, terms, max_terms, nterms,
                                  status));
        return MH_OK;
    });
}

extern "C" int mh_htree_levels(mh_htree *t, uint8_t *out, uint64_t cap_nodes) {
    return mh_guard([&]() -> int {
        if (!t) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(t->ctx->device));
        const uint64_t total = mh_htree_levels_len(t->width);
        if (cap_nodes < total || (total && !out)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!total) return MH_OK;
        MH_HIP(hipMemcpyAsync(out, t->levels.p, total * 32, hipMemcpyDeviceToHost, t->stream));
        MH_HIP(hipStreamSynchronize(t->stream));
        return MH_OK;
    });
}

extern "C" int mh_htree_levels_device(mh_htree *t, const uint8_t **dptr) {
    return mh_guard([&]() -> int {
        if (!t || !dptr) return MH_ERR_ILLEGAL_ARGUMENTS;
        *dptr = t->levels.as<uint8_t>();
        return MH_OK;
    });
}

// ------------------------------------------------------------------ verification
extern "C" int mh_dev_htree_verify_inclusion_batch(mh_ctx *c, uint64_t np, const uint64_t *leaf,
                                                   const uint64_t *width, const uint64_t *term_off,
                                                   const uint8_t *terms, const uint8_t *digests,
                                                   const uint8_t *roots, uint8_t *ok) {
    return mh_guard([&]() -> int {
        if (!c || (np && (!leaf || !width || !term_off || !digests || !roots || !ok)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (!np) return MH_OK;
        MH_HIP(launch_htree_verify(c->stream, c->tm(), np, leaf, width, term_off, terms, digests, roots,
                                   ok));
        return MH_OK;
    });
}

// host wrapper: stage, run on the context stream, copy back
extern "C" int mh_htree_verify_inclusion_batch(mh_ctx *c, uint64_t np, const uint64_t *leaf,
                                               const uint64_t *width, const uint64_t *term_off,
                                               const uint8_t *terms, const uint8_t *digests,
                                               const uint8_t *roots, uint8_t *ok) {
    return mh_guard([&]() -> int {
        if (!c || (np && (!leaf || !width || !term_off || !digests || !roots || !ok)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!np) return MH_OK;
        if (!monotonic(term_off, np)) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        hipSetDevice(c->device);
        const uint64_t nterms = term_off[np] - term_off[0];
        std::vector<uint64_t> to(np + 1);
        for (uint64_t p = 0; p <= np; p++) to[p] = term_off[p] - term_off[0];
        // layout in one scratch buffer: leaf | width | off | digests | roots | terms | ok
        const uint64_t b_leaf = 0, b_width = b_leaf + np * 8, b_off = b_width + np * 8,
                       b_dig = (b_off + (np + 1) * 8 + 15) & ~15ull, b_root = b_dig + np * 32,
                       b_terms = b_root + np * 32, b_ok = b_terms + nterms * 32,
                       total = b_ok + np + 16;
        MH_HIP(c->s_msgs.ensure(total));
        uint8_t *base = c->s_msgs.as<uint8_t>();
        hipStream_t st = c->stream;
        MH_HIP(hipMemcpyAsync(base + b_leaf, leaf, np * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_width, width, np * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_off, to.data(), (np + 1) * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_dig, digests, np * 32, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_root, roots, np * 32, hipMemcpyHostToDevice, st));
        if (nterms)
            MH_HIP(hipMemcpyAsync(base + b_terms, terms + term_off[0] * 32, nterms * 32,
                                  hipMemcpyHostToDevice, st));
        MH_HIP(launch_htree_verify(st, c->tm(), np, (const uint64_t *)(base + b_leaf),
                                   (const uint64_t *)(base + b_width), (const uint64_t *)(base + b_off),
                                   base + b_terms, base + b_dig, base + b_root, base + b_ok));
        MH_HIP(hipMemcpyAsync(ok, base + b_ok, np, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}

extern "C" int mh_dev_ahtree_verify_batch(mh_ctx *c, int kind, uint64_t np, const uint64_t *i,
                                          const uint64_t *j, const uint64_t *term_off,
                                          const uint8_t *terms, const uint8_t *a, const uint8_t *b,
                                          uint8_t *ok, uint8_t *eval_out) {
    return mh_guard([&]() -> int {
        if (!c || kind < 0 || kind > 2) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        if (np && (!i || !j || !term_off || !a || !b || !ok)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!np) return MH_OK;
        MH_HIP(launch_ahtree_verify(c->stream, c->tm(), kind, np, i, j, term_off, terms, a, b, ok,
                                    eval_out));
        return MH_OK;
    });
}

extern "C" int mh_ahtree_verify_batch(mh_ctx *c, int kind, uint64_t np, const uint64_t *i,
                                      const uint64_t *j, const uint64_t *term_off,
                                      const uint8_t *terms, const uint8_t *a, const uint8_t *b,
                                      uint8_t *ok, uint8_t *eval_out) {
    return mh_guard([&]() -> int {
        if (!c || kind < 0 || kind > 2) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (np && (!i || !j || !term_off || !a || !b || !ok)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!np) return MH_OK;
        if (!monotonic(term_off, np)) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(c->mu);
        hipSetDevice(c->device);
        const uint64_t nterms = term_off[np] - term_off[0];
        std::vector<uint64_t> to(np + 1);
        for (uint64_t p = 0; p <= np; p++) to[p] = term_off[p] - term_off[0];
        const uint64_t eval_w = kind == MH_AHT_CONSISTENCY ? 64 : 32;
        const uint64_t b_i = 0, b_j = np * 8, b_off = 2 * np * 8,
                       b_a = (b_off + (np + 1) * 8 + 15) & ~15ull, b_b = b_a + np * 32,
                       b_terms = b_b + np * 32, b_eval = b_terms + nterms * 32,
                       b_ok = b_eval + (eval_out ? np * eval_w : 0), total = b_ok + np + 16;
        MH_HIP(c->s_msgs.ensure(total));
        uint8_t *base = c->s_msgs.as<uint8_t>();
        hipStream_t st = c->stream;
        MH_HIP(hipMemcpyAsync(base + b_i, i, np * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_j, j, np * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_off, to.data(), (np + 1) * 8, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_a, a, np * 32, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(base + b_b, b, np * 32, hipMemcpyHostToDevice, st));
        if (nterms)
            MH_HIP(hipMemcpyAsync(base + b_terms, terms + term_off[0] * 32, nterms * 32,
                                  hipMemcpyHostToDevice, st));
        MH_HIP(launch_ahtree_verify(st, c->tm(), kind, np, (const uint64_t *)(base + b_i),
                                    (const uint64_t *)(base + b_j), (const uint64_t *)(base + b_off),
                                    base + b_terms, base + b_a, base + b_b, base + b_ok,
                                    eval_out ? base + b_eval : nullptr));
        MH_HIP(hipMemcpyAsync(ok, base + b_ok, np, hipMemcpyDeviceToHost, st));
        if (eval_out)
            MH_HIP(hipMemcpyAsync(eval_out, base + b_eval, np * eval_w, hipMemcpyDeviceToHost, st));
        MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    });
}

// ------------------------------------------------------------------ ahtree
extern "C" uint64_t mh_ahtree_nodes_upto(uint64_t n) { return ahtree_nodes_upto(n); }

extern "C" int mh_dev_ahtree_append_batch(mh_ctx *c, uint8_t *dlog, uint64_t n0,
                                          const uint8_t *payloads, uint64_t m, uint32_t plen,
                                          uint8_t *roots_out) {
    return mh_guard([&]() -> int {
        if (!c || (m && (!dlog || (!payloads && plen)))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((uintptr_t)dlog & 15) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!m) return MH_OK;
        hipSetDevice(c->device);
        // the work-queue counter is ctx scratch: reset + launch are enqueued
        // under the lock so concurrent callers on this ctx never share one
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->s_ctr.ensure(256));
        MH_HIP(launch_ahtree_append(c->stream, c->tm(), dlog, n0, payloads, m, plen, roots_out,
                                    c->s_ctr.as<uint32_t>()));
        return MH_OK;
    });
}

// the pLog / cLog records of a batch (ahtree.go:266-282,
// 341-351), alone or fused into the append's leaf phase.
static bool logs_ok(const uint8_t *payloads, uint64_t m, uint32_t plen, uint64_t p_off0) {
    if (m && !payloads && plen) return false;
    const uint64_t rec = 4 + (uint64_t)plen;
    return !m || (m <= (~0ull - p_off0) / rec);  // offsets stay in uint64
}

extern "C" int mh_dev_ahtree_log_records(mh_ctx *c, const uint8_t *payloads, uint64_t m,
                                         uint32_t plen, uint64_t p_off0, uint8_t *plog,
                                         uint8_t *clog) {
    return mh_guard([&]() -> int {
        if (!c || !logs_ok(payloads, m, plen, p_off0)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!m || (!plog && !clog)) return MH_OK;
        hipSetDevice(c->device);
        AhtLogs lg;
        lg.plog = plog;
        lg.clog = clog;
        lg.p_off0 = p_off0;
        MH_HIP(launch_ahtree_leaves(c->stream, c->tm(), nullptr, 0, payloads, m, plen, lg));
        return MH_OK;
    });
}

extern "C" int mh_dev_ahtree_append_batch_logs(mh_ctx *c, uint8_t *dlog, uint64_t n0,
                                               const uint8_t *payloads, uint64_t m, uint32_t plen,
                                               uint64_t p_off0, uint8_t *plog, uint8_t *clog,
                                               uint8_t *roots_out) {
    return mh_guard([&]() -> int {
        if (!c || (m && !dlog) || !logs_ok(payloads, m, plen, p_off0)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((uintptr_t)dlog & 15) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!m) return MH_OK;
        hipSetDevice(c->device);
        AhtLogs lg;
        lg.plog = plog;
        lg.clog = clog;
        lg.p_off0 = p_off0;
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->s_ctr.ensure(256));
        MH_HIP(launch_ahtree_append(c->stream, c->tm(), dlog, n0, payloads, m, plen, roots_out,
                                    c->s_ctr.as<uint32_t>(), lg));
        return MH_OK;
    });
}

extern "C" uint64_t mh_ahtree_node_index(uint64_t n, int level) {
    return ahtree_nodes_until(n) + (uint64_t)level;
}

extern "C" int mh_dev_ahtree_append_range(mh_ctx *c, uint8_t *dlog_range, uint64_t n0,
                                          const uint8_t *peaks, const uint8_t *payloads,
                                          uint64_t m, uint32_t plen, uint8_t *roots_out) {
    return mh_guard([&]() -> int {
        if (!c || (m && (!dlog_range || (!payloads && plen))) || (n0 && !peaks))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (((uintptr_t)dlog_range & 15) || m > ~0ull - n0) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!m) return MH_OK;
        hipSetDevice(c->device);
        AhtSlots slots;
        memset(slots.b, 0, sizeof slots.b);
        for (int l = 0, q = 0; l < 64; l++)
            if ((n0 >> l) & 1) memcpy(slots.b + l * 32, peaks + 32 * (q++), 32);
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->s_ctr.ensure(256));
        MH_HIP(c->s_edge.ensure(64 * 32));
        MH_HIP(launch_ahtree_put_slots(c->stream, slots, c->s_edge.as<uint8_t>()));
        AhtEdge edge;
        edge.fr = c->s_edge.as<uint8_t>();
        edge.lo = n0;
        // dLog index x lives at dlog_range + (x - nodesUpto(n0)) * 32
        uint8_t *vb = reinterpret_cast<uint8_t *>((uintptr_t)dlog_range -
                                                  (uintptr_t)(ahtree_nodes_upto(n0) * 32));
        MH_HIP(launch_ahtree_append(c->stream, c->tm(), vb, n0, payloads, m, plen, roots_out,
                                    c->s_ctr.as<uint32_t>(), AhtLogs(), edge));
        return MH_OK;
    });
}

extern "C" int mh_dev_ahtree_peaks(mh_ctx *c, const uint8_t *dlog, uint64_t n, uint8_t *peaks_out) {
    return mh_guard([&]() -> int {
        if (!c || (n && (!dlog || !peaks_out))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((uintptr_t)dlog & 15) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        hipSetDevice(c->device);
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->s_edge.ensure(64 * 32));
        MH_HIP(launch_ahtree_peaks(c->stream, dlog, n, c->s_edge.as<uint8_t>()));
        uint8_t slots[64 * 32];
        MH_HIP(hipMemcpyAsync(slots, c->s_edge.p, sizeof slots, hipMemcpyDeviceToHost, c->stream));
        MH_HIP(hipStreamSynchronize(c->stream));
        for (int l = 0, q = 0; l < 64; l++)
            if ((n >> l) & 1) memcpy(peaks_out + 32 * (q++), slots + l * 32, 32);
        return MH_OK;
    });
}

extern "C" int mh_dev_ahtree_append_local(mh_ctx *c, uint8_t *dlog, uint64_t n0,
                                          const uint8_t *payloads, uint64_t m, uint32_t plen,
                                          int shard_bits) {
    return mh_guard([&]() -> int {
        if (!c || shard_bits < 0 || shard_bits > 62 || (m && (!dlog || (!payloads && plen))))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((uintptr_t)dlog & 15) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n0 & ((1ull << shard_bits) - 1)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!m) return MH_OK;
        hipSetDevice(c->device);
        MH_HIP(launch_ahtree_leaves(c->stream, c->tm(), dlog, n0, payloads, m, plen));
        MH_HIP(launch_ahtree_perfect(c->stream, c->tm(), dlog, n0, n0 + m, 1, shard_bits));
        return MH_OK;
    });
}

extern "C" int mh_dev_ahtree_put_shard_roots(mh_ctx *c, uint8_t *dlog, int shard_bits,
                                             uint64_t count, const uint8_t *roots) {
    return mh_guard([&]() -> int {
        if (!c || shard_bits < 0 || shard_bits > 62 || (count && (!dlog || !roots)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!count) return MH_OK;
        hipSetDevice(c->device);
        MH_HIP(launch_ahtree_put_shard_roots(c->stream, c->tm(), dlog, shard_bits, count, roots));
        return MH_OK;
    });
}

extern "C" int mh_dev_ahtree_append_spine(mh_ctx *c, uint8_t *dlog, uint64_t n0, uint64_t m,
                                          uint8_t *roots_out) {
    return mh_guard([&]() -> int {
        if (!c || (m && !dlog)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((uintptr_t)dlog & 15) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!m) return MH_OK;
        hipSetDevice(c->device);
        std::lock_guard<std::mutex> lk(c->mu);
        MH_HIP(c->s_ctr.ensure(256));
        MH_HIP(launch_ahtree_spine(c->stream, c->tm(), dlog, n0, m, roots_out,
                                   c->s_ctr.as<uint32_t>()));
        return MH_OK;
    });
}

extern "C" int mh_ahtree_new(mh_ctx *c, mh_ahtree **out) {
    return mh_guard([&]() -> int {
        if (!c || !out) return MH_ERR_ILLEGAL_ARGUMENTS;
        *out = nullptr;
        hipSetDevice(c->device);
        mh_ahtree *t = new (std::nothrow) mh_ahtree();
        if (!t) return MH_ERR_OUT_OF_MEMORY;
        t->ctx = c;
        hipError_t e = hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete t;
            return -(int)e;
        }
        *out = t;
        return MH_OK;
    });
}

extern "C" int mh_ahtree_free(mh_ahtree *t) {
    return mh_guard([&]() -> int {
        if (!t) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(t->ctx->device));
        hipStreamSynchronize(t->stream);
        hipStreamDestroy(t->stream);
        delete t;
        return MH_OK;
    });
}

static int aht_reserve(mh_ahtree *t, uint64_t new_size) {
    const uint64_t need = ahtree_nodes_upto(new_size) * 32;
    if (need <= t->dlog.cap && t->dlog.p) return MH_OK;
    uint64_t cap = std::max<uint64_t>(need, t->dlog.cap * 2);
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, cap);
    if (e != hipSuccess) {
        cap = need;  // retry exact
        e = hipMalloc(&p, cap);
        if (e != hipSuccess) return map_alloc(e);
    }
    const uint64_t used = ahtree_nodes_upto(t->size) * 32;
    if (used) MH_HIP(hipMemcpyAsync(p, t->dlog.p, used, hipMemcpyDeviceToDevice, t->stream));
    MH_HIP(hipStreamSynchronize(t->stream));
    if (t->dlog.p) hipFree(t->dlog.p);
    t->dlog.p = p;
    t->dlog.cap = cap;
    return MH_OK;
}

static int aht_append_batch(mh_ahtree *t, const uint8_t *payloads, uint64_t m, uint32_t plen,
                            uint64_t p_off0, uint8_t *plog_out, uint8_t *clog_out,
                            uint8_t *roots_out) {
    if (!t || !logs_ok(payloads, m, plen, p_off0)) return MH_ERR_ILLEGAL_ARGUMENTS;
    std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
    if (!m) return MH_OK;
    hipSetDevice(t->ctx->device);
    int st = aht_reserve(t, t->size + m);
    if (st) return st;
    const uint64_t rec = 4 + (uint64_t)plen;
    // one device buffer: payloads | pLog records | cLog entries | roots
    const uint64_t b_pay = 0, b_plog = (m * plen + 15) & ~15ull;
    const uint64_t b_clog = b_plog + (plog_out ? (m * rec + 15) & ~15ull : 0);
    const uint64_t b_end = b_clog + (clog_out ? (m * 12 + 15) & ~15ull : 0);
    MH_HIP(t->in.ensure(b_end ? b_end : 16));
    uint8_t *base = t->in.as<uint8_t>();
    if (plen)
        MH_HIP(hipMemcpyAsync(base + b_pay, payloads, m * plen, hipMemcpyHostToDevice, t->stream));
    uint8_t *rd = nullptr;
    if (roots_out) {
        MH_HIP(t->roots.ensure(m * 32));
        rd = t->roots.as<uint8_t>();
    }
    AhtLogs lg;
    lg.plog = plog_out ? base + b_plog : nullptr;
    lg.clog = clog_out ? base + b_clog : nullptr;
    lg.p_off0 = p_off0;
    MH_HIP(t->ctr.ensure(256));
    MH_HIP(launch_ahtree_append(t->stream, t->ctx->tm(), t->dlog.as<uint8_t>(), t->size,
                                base + b_pay, m, plen, rd, t->ctr.as<uint32_t>(), lg));
    if (roots_out) MH_HIP(hipMemcpyAsync(roots_out, rd, m * 32, hipMemcpyDeviceToHost, t->stream));
    if (plog_out)
        MH_HIP(hipMemcpyAsync(plog_out, lg.plog, m * rec, hipMemcpyDeviceToHost, t->stream));
    if (clog_out)
        MH_HIP(hipMemcpyAsync(clog_out, lg.clog, m * 12, hipMemcpyDeviceToHost, t->stream));
    MH_HIP(hipStreamSynchronize(t->stream));
    t->size += m;
    return MH_OK;
}

extern "C" int mh_ahtree_append_batch(mh_ahtree *t, const uint8_t *payloads, uint64_t m,
                                      uint32_t plen, uint8_t *roots_out) {
    return mh_guard([&]() -> int {
        return aht_append_batch(t, payloads, m, plen, 0, nullptr, nullptr, roots_out);
    });
}

extern "C" int mh_ahtree_append_batch_logs(mh_ahtree *t, const uint8_t *payloads, uint64_t m,
                                           uint32_t plen, uint64_t p_off0, uint8_t *plog_out,
                                           uint8_t *clog_out, uint8_t *roots_out) {
    return mh_guard([&]() -> int {
        return aht_append_batch(t, payloads, m, plen, p_off0, plog_out, clog_out, roots_out);
    });
}

extern "C" int mh_ahtree_append(mh_ahtree *t, const uint8_t *payload, uint64_t plen, uint64_t *n,
                                uint8_t h[32]) {
    return mh_guard([&]() -> int {
        // ahtree.go:246-373 (d == nil -> ErrIllegalArguments, ahtree.go:258-261)
        if (!t || (!payload && plen)) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        MH_HIP(hipSetDevice(t->ctx->device));
        if (!payload) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (plen > 0xffffffffull) return MH_ERR_ILLEGAL_ARGUMENTS;
        uint8_t root[32];
        int st = mh_ahtree_append_batch(t, payload, 1, (uint32_t)plen, root);
        if (st) return st;
        if (n) *n = t->size;
        if (h) memcpy(h, root, 32);
        return MH_OK;
    });
}

extern "C" int mh_ahtree_size(mh_ahtree *t, uint64_t *size) {
    return mh_guard([&]() -> int {
        if (!t || !size) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        *size = t->size;
        return MH_OK;
    });
}

static int aht_read_nodes(mh_ahtree *t, const uint64_t *idx, uint32_t cnt, uint8_t *out) {
    for (uint32_t k = 0; k < cnt; k++)
        MH_HIP(hipMemcpyAsync(out + 32 * k, t->dlog.as<uint8_t>() + idx[k] * 32, 32,
                              hipMemcpyDeviceToHost, t->stream));
    MH_HIP(hipStreamSynchronize(t->stream));
    return MH_OK;
}

extern "C" int mh_ahtree_root_at(mh_ahtree *t, uint64_t n, uint8_t root[32]) {
    return mh_guard([&]() -> int {
        // ahtree.go:749-771
        if (!t || !root) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        MH_HIP(hipSetDevice(t->ctx->device));
        if (n == 0) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (t->size == 0) return MH_ERR_EMPTY_TREE;
        if (n > t->size) return MH_ERR_UNEXISTENT_DATA;
        const uint64_t idx = ahtree_nodes_until(n) + (uint64_t)__builtin_popcountll(n - 1);
        return aht_read_nodes(t, &idx, 1, root);
    });
}

extern "C" int mh_ahtree_root(mh_ahtree *t, uint64_t *n, uint8_t root[32]) {
    return mh_guard([&]() -> int {
        if (!t) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        MH_HIP(hipSetDevice(t->ctx->device));
        if (t->size == 0) return MH_ERR_EMPTY_TREE;  // ahtree.go:731-734
        if (n) *n = t->size;
        return mh_ahtree_root_at(t, t->size, root);
    });
}

// Proof index walks: ahtree.go:545-577 / 596-661, node(k,l) = nodesUntil(k)+l.
static uint64_t aht_node_idx(uint64_t k, int l) { return ahtree_nodes_until(k) + (uint64_t)l; }

static uint64_t aht_highest(uint64_t i, int d) {
    int l = 0;
    for (int r = d - 1; r >= 0; r--)
        if ((i - 1) & (1ull << r)) l++;
    return aht_node_idx(i, l);
}

static void aht_incl(uint64_t i, uint64_t j, int height, std::vector<uint64_t> &s) {
    for (int h = height - 1; h >= 0; h--) {
        if ((j - 1) & (1ull << h)) {
            const uint64_t k = (j - 1) >> h << h;
            if (i <= k) {
                s.push_back(aht_highest(j, h));
                aht_incl(i, k, h, s);
                return;
            }
            s.push_back(aht_node_idx(k, h));
        }
    }
}

static void aht_cons(uint64_t i, uint64_t j, int height, std::vector<uint64_t> &s) {
    for (int h = height - 1; h >= 0; h--) {
        if ((j - 1) & (1ull << h)) {
            const uint64_t k = (j - 1) >> h << h;
            if (i <= k) {
                s.push_back(aht_highest(j, h));
                if (i < k) aht_cons(i, k, h, s);
                if (i == k) s.push_back(aht_highest(i, h));
                return;
            }
            s.push_back(aht_node_idx(k, h));
            if (i == j) {
                s.push_back(aht_highest(i, h));
                return;
            }
        }
    }
}

static int aht_emit(mh_ahtree *t, std::vector<uint64_t> &s, uint8_t *terms, uint32_t cap,
                    uint32_t *nterms) {
    std::reverse(s.begin(), s.end());  // Go prepends every term
    if (s.size() > cap || (!terms && !s.empty())) return MH_ERR_ILLEGAL_ARGUMENTS;
    int st = aht_read_nodes(t, s.data(), (uint32_t)s.size(), terms);
    if (st) return st;
    *nterms = (uint32_t)s.size();
    return MH_OK;
}

extern "C" int mh_ahtree_inclusion_proof(mh_ahtree *t, uint64_t i, uint64_t j, uint8_t *terms,
                                         uint32_t cap, uint32_t *nterms) {
    return mh_guard([&]() -> int {
        if (!t || !nterms) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        MH_HIP(hipSetDevice(t->ctx->device));
        *nterms = 0;
        if (i > j) return MH_ERR_ILLEGAL_ARGUMENTS;    // ahtree.go:534-536
        if (j > t->size) return MH_ERR_UNEXISTENT_DATA;  // ahtree.go:538-540
        if (j == 0) return MH_ERR_UNEXISTENT_DATA;       // Go fails reading node(0, .)
        std::vector<uint64_t> s;
        aht_incl(i, j, bits_len64(j - 1), s);
        return aht_emit(t, s, terms, cap, nterms);
    });
}

extern "C" int mh_ahtree_consistency_proof(mh_ahtree *t, uint64_t i, uint64_t j, uint8_t *terms,
                                           uint32_t cap, uint32_t *nterms) {
    return mh_guard([&]() -> int {
        if (!t || !nterms) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        MH_HIP(hipSetDevice(t->ctx->device));
        *nterms = 0;
        if (i > j) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (j > t->size) return MH_ERR_UNEXISTENT_DATA;
        if (j == 0) return MH_ERR_UNEXISTENT_DATA;
        std::vector<uint64_t> s;
        aht_cons(i, j, bits_len64(j - 1), s);
        return aht_emit(t, s, terms, cap, nterms);
    });
}

extern "C" int mh_ahtree_proof_batch(mh_ahtree *t, int kind, uint64_t n, const uint64_t *i,
                                     const uint64_t *j, uint8_t *terms, uint32_t max_terms,
                                     uint32_t *nterms, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!t || (kind != MH_AHT_INCLUSION && kind != MH_AHT_CONSISTENCY) ||
            (n && (!i || !j || !terms || !nterms || !status || !max_terms)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        MH_HIP(hipSetDevice(t->ctx->device));
        if (!n) return MH_OK;
        const uint8_t *dl = t->dlog.as<uint8_t>();
        const uint64_t size = t->size;
        hipStream_t st = t->ctx->stream;  // ctx scratch: see mh_htree_inclusion_proof_batch
        Timer *tm = t->ctx->tm();
        return proof_batch_host(t->ctx, st, n, i, j, max_terms, terms, nterms, status,
                                [&](const uint64_t *a, const uint64_t *b, uint8_t *tt, uint32_t *nt,
                                    int32_t *ss) {
                                    return launch_ahtree_proof(st, tm, kind, dl, size, n, a, b, tt,
                                                               max_terms, nt, ss);
                                });
    });
}

extern "C" int mh_dev_ahtree_proof_batch(mh_ctx *c, int kind, const uint8_t *dlog, uint64_t size,
                                         uint64_t n, const uint64_t *i, const uint64_t *j,
                                         uint8_t *terms, uint32_t max_terms, uint32_t *nterms,
                                         int32_t *status) {
    return mh_guard([&]() -> int {
        if (!c || (kind != MH_AHT_INCLUSION && kind != MH_AHT_CONSISTENCY) ||
            (n && (!dlog || !i || !j || !terms || !nterms || !status || !max_terms)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!n) return MH_OK;
        hipSetDevice(c->device);
        MH_HIP(launch_ahtree_proof(c->stream, c->tm(), kind, dlog, size, n, i, j, terms, max_terms,
                                   nterms, status));
        return MH_OK;
    });
}

extern "C" int mh_ahtree_reset_size(mh_ahtree *t, uint64_t new_size) {
    return mh_guard([&]() -> int {
        // ahtree.go:375-458 (file-size checks belong to the Go appendables)
        if (!t) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        if (new_size > t->size) return MH_ERR_CANNOT_RESET_TO_LARGER;
        t->size = new_size;
        return MH_OK;
    });
}

extern "C" int mh_ahtree_dlog(mh_ahtree *t, uint64_t first, uint64_t count, uint8_t *out) {
    return mh_guard([&]() -> int {
        if (!t) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        MH_HIP(hipSetDevice(t->ctx->device));
        const uint64_t total = ahtree_nodes_upto(t->size);
        if (first > total || count > total - first) return MH_ERR_UNEXISTENT_DATA;
        if (!count) return MH_OK;
        if (!out) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipMemcpyAsync(out, t->dlog.as<uint8_t>() + first * 32, count * 32, hipMemcpyDeviceToHost,
                              t->stream));
        MH_HIP(hipStreamSynchronize(t->stream));
        return MH_OK;
    });
}

extern "C" int mh_ahtree_dlog_device(mh_ahtree *t, const uint8_t **dptr) {
    return mh_guard([&]() -> int {
        if (!t || !dptr) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::recursive_mutex> lk_(t->mu);  // AHtree.mutex (ahtree.go:60-84)
        *dptr = t->dlog.as<uint8_t>();
        return MH_OK;
    });
}
