// capi_multi.hip -- the multi-GPU htree build and ahtree batch append behind
// the C ABI.
//
// One process drives K devices -- what a cgo caller (one Go process, the
// commit path of immustore.go:1620-1632) needs -- with one mh_ctx (HIP
// stream) per device and an RCCL clique over them (ncclCommInitAll).  The
// leaves are cut into power-of-two aligned shards of S = 2^k entries; device
// g builds the subtree over [gS, min((g+1)S, n)) with every level (levels
// 0..k of the global tree restricted to the shard are exactly the shard's own
// levels, htree.go:85-110, the right edge included); the G <= K subtree roots
// are all-gathered (32 bytes per device, RCCL over xGMI) and the top
// ceil(log2 G) levels are reduced on every device.
//
// RCCL is loaded on first use (dlopen of librccl.so.1), so single-device
// users of the library never need it.
#include <dlfcn.h>

#include <memory>
#include <thread>

#include <rccl/rccl.h>

#include "capi_internal.hpp"

namespace {

struct Rccl {
    bool ok = false;
    ncclResult_t (*init_all)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.ok = r.init_all && r.destroy && r.all_gather && r.group_start && r.group_end;
    });
    return r;
}

#define MH_NCCL(expr)                                      \
    do {                                                   \
        if ((expr) != ncclSuccess) return MH_ERR_COLLECTIVE; \
    } while (0)

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace

struct mh_multi {
    int K = 0;
    std::vector<int> dev;
    std::vector<mh_ctx *> ctx;
    std::vector<ncclComm_t> comm;
    // false when a device is listed more than once (more shards than
    // devices): RCCL wants one rank per device, so the 32-byte roots are then
    // gathered with device-to-device copies instead
    bool use_rccl = true;
    struct Dev {
        DevBuf keys, vals, hv, levels, send, recv, top, dlog, ovr;
    };
    std::vector<std::unique_ptr<Dev>> buf;
    std::mutex mu;  // one build at a time per mh_multi
};

extern "C" int mh_multi_shard_plan(uint64_t n, int ndev, uint64_t *shard, uint64_t *nshards) {
    if (ndev < 1 || !shard || !nshards) return MH_ERR_ILLEGAL_ARGUMENTS;
    if (n == 0) {
        *shard = 1;
        *nshards = 0;
        return MH_OK;
    }
    const uint64_t S = next_pow2((n + (uint64_t)ndev - 1) / (uint64_t)ndev);
    *shard = S;
    *nshards = (n + S - 1) / S;
    return MH_OK;
}

extern "C" int mh_multi_create(int ndev, const int *devices, mh_multi **out) {
    return mh_guard([&]() -> int {
        if (ndev < 1 || !devices || !out) return MH_ERR_ILLEGAL_ARGUMENTS;
        *out = nullptr;
        int have = 0;
        if (hipGetDeviceCount(&have) != hipSuccess || have < 1) return MH_ERR_NO_DEVICE;
        for (int d = 0; d < ndev; d++)
            if (devices[d] < 0 || devices[d] >= have) return MH_ERR_ILLEGAL_ARGUMENTS;
        bool distinct = true;
        for (int a = 0; a < ndev; a++)
            for (int b = a + 1; b < ndev; b++) distinct &= devices[a] != devices[b];
        const Rccl &R = rccl();
        if (distinct && !R.ok) return MH_ERR_COLLECTIVE;
        mh_multi *m = new mh_multi();
        m->use_rccl = distinct;
        m->K = ndev;
        m->dev.assign(devices, devices + ndev);
        m->ctx.assign(ndev, nullptr);
        for (int d = 0; d < ndev; d++) m->buf.emplace_back(new mh_multi::Dev());
        for (int d = 0; d < ndev; d++) {
            int st = mh_ctx_create(devices[d], nullptr, &m->ctx[d]);
            if (st != MH_OK) {
                mh_multi_destroy(m);
                return st;
            }
        }
        if (!distinct) {
            *out = m;
            return MH_OK;
        }
        m->comm.assign(ndev, nullptr);
        if (R.init_all(m->comm.data(), ndev, devices) != ncclSuccess) {
            m->comm.clear();
            mh_multi_destroy(m);
            return MH_ERR_COLLECTIVE;
        }
        *out = m;
        return MH_OK;
    });
}

extern "C" int mh_multi_destroy(mh_multi *m) {
    return mh_guard([&]() -> int {
        if (!m) return MH_OK;
        for (int d = 0; d < m->K; d++)
            if (m->ctx[d]) mh_ctx_synchronize(m->ctx[d]);
        const Rccl &R = rccl();
        for (ncclComm_t c : m->comm)
            if (c && R.ok) R.destroy(c);
        for (int d = 0; d < (int)m->buf.size(); d++) {
            hipSetDevice(m->dev[d]);
            m->buf[d].reset();  // frees on the owning device
        }
        for (mh_ctx *c : m->ctx)
            if (c) mh_ctx_destroy(c);
        delete m;
        return MH_OK;
    });
}

extern "C" int mh_multi_size(mh_multi *m, int *ndev) {
    if (!m || !ndev) return MH_ERR_ILLEGAL_ARGUMENTS;
    *ndev = m->K;
    return MH_OK;
}

extern "C" mh_ctx *mh_multi_ctx(mh_multi *m, int d) {
    return (m && d >= 0 && d < m->K) ? m->ctx[d] : nullptr;
}

extern "C" int mh_multi_synchronize(mh_multi *m) {
    return mh_guard([&]() -> int {
        if (!m) return MH_ERR_ILLEGAL_ARGUMENTS;
        for (int d = 0; d < m->K; d++)
            if (int st = mh_ctx_synchronize(m->ctx[d])) return st;
        return MH_OK;
    });
}

namespace {

// fn(d) for d in [0, n) on n threads (this one included): each device's host
// copies go over its own PCIe link at once, and a pageable copy, which holds
// the issuing thread until it is staged, never serialises the devices.
// Returns the first non-zero status.
template <class F>
int per_device(int n, F &&fn) {
    std::vector<int> st(n, MH_OK);
    std::vector<std::thread> th;
    auto run = [&](int d) {
        try {
            st[d] = fn(d);
        } catch (const std::bad_alloc &) {
            st[d] = MH_ERR_OUT_OF_MEMORY;
        } catch (...) {
            st[d] = MH_ERR_ILLEGAL_STATE;
        }
    };
    int d = 1;
    try {
        for (; d < n; d++) th.emplace_back(run, d);
    } catch (...) {  // no thread: the rest run here
    }
    run(0);
    for (int k = d; k < n; k++) run(k);
    for (auto &t : th) t.join();
    for (int k = 0; k < n; k++)
        if (st[k]) return st[k];
    return MH_OK;
}

// All-gather of one 32-byte root per device (send[d] -> recv[d] = K x 32 B),
// on each device's context stream.
int gather_roots(mh_multi *m, const std::vector<const uint8_t *> &send,
                 const std::vector<uint8_t *> &recv) {
    if (!m->use_rccl) {
        // shards sharing devices: wait for every subtree, then copy the roots
        for (int d = 0; d < m->K; d++)
            if (int st = mh_ctx_synchronize(m->ctx[d])) return st;
        for (int d = 0; d < m->K; d++) {
            MH_HIP(hipSetDevice(m->dev[d]));
            for (int s = 0; s < m->K; s++)
                MH_HIP(hipMemcpyAsync(recv[d] + 32 * s, send[s], 32, hipMemcpyDefault,
                                      m->ctx[d]->stream));
        }
        return MH_OK;
    }
    const Rccl &R = rccl();
    MH_NCCL(R.group_start());
    for (int d = 0; d < m->K; d++) {
        MH_HIP(hipSetDevice(m->dev[d]));
        if (R.all_gather(send[d], recv[d], 32, ncclUint8, m->comm[d], m->ctx[d]->stream) !=
            ncclSuccess) {
            R.group_end();
            return MH_ERR_COLLECTIVE;
        }
    }
    MH_NCCL(R.group_end());
    return MH_OK;
}

}  // namespace

extern "C" int mh_multi_dev_htree_build_entries_fixed(
    mh_multi *m, int version, uint64_t n_per_dev, const uint8_t *const *keys, uint32_t key_len,
    const uint8_t *const *vals, uint32_t val_len, uint8_t *const *hvals_out,
    uint8_t *const *levels, uint8_t *const *top_levels, uint8_t *const *root) {
    return mh_guard([&]() -> int {
        if (!m || (version != 0 && version != 1) || !keys || !vals || !levels || !top_levels ||
            !root || n_per_dev == 0)
            return MH_ERR_ILLEGAL_ARGUMENTS;
        const int K = m->K;
        if (K > 1 && (n_per_dev & (n_per_dev - 1))) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(m->mu);
        // 1. every device: its subtree (levels 0..log2 n_per_dev, root at root[d])
        for (int d = 0; d < K; d++) {
            int st = mh_dev_htree_build_entries_fixed(m->ctx[d], version, n_per_dev, keys[d],
                                                      key_len, vals[d], val_len,
                                                      hvals_out ? hvals_out[d] : nullptr,
                                                      levels[d], root[d]);
            if (st) return st;
        }
        // 2. all-gather the K subtree roots (32 B each) over RCCL
        std::vector<const uint8_t *> send(K);
        std::vector<uint8_t *> recv(K);
        for (int d = 0; d < K; d++) {
            MH_HIP(hipSetDevice(m->dev[d]));
            MH_HIP(m->buf[d]->recv.ensure(32 * (uint64_t)K));
            send[d] = root[d];
            recv[d] = m->buf[d]->recv.as<uint8_t>();
        }
        if (int st = gather_roots(m, send, recv)) return st;
        // 3. every device: the top log2(K) levels over the gathered roots
        //    (replicated, identical), the global root into root[d]
        for (int d = 0; d < K; d++) {
            int st = mh_dev_htree_reduce_nodes(m->ctx[d], recv[d], (uint64_t)K, top_levels[d],
                                               root[d]);
            if (st) return st;
        }
        return MH_OK;
    });
}

namespace {

// Steps 2-4 of a host-memory multi build once every shard's subtree is built
// on its device (B.hv, B.levels, B.send = subtree root): all-gather of the
// subtree roots (devices without a shard send zeros), the top levels over the
// G roots on device 0 (global levels kS+1 ..), then the results back -- hVals
// and each shard's slice of every level <= kS from every device's own
// thread, the top levels and the root from device 0.
int multi_htree_finish(mh_multi *m, uint64_t n, uint64_t S, uint64_t G, int kS,
                       uint8_t *hvals_out, uint8_t *levels_out, uint8_t root[32]) {
    const int K = m->K;
    LevelGeom gg;
    gg.init(n);
    std::vector<const uint8_t *> send(K);
    std::vector<uint8_t *> recv(K);
    for (int d = 0; d < K; d++) {
        mh_multi::Dev &B = *m->buf[d];
        MH_HIP(hipSetDevice(m->dev[d]));
        if ((uint64_t)d >= G) {
            MH_HIP(B.send.ensure(32));
            MH_HIP(hipMemsetAsync(B.send.p, 0, 32, m->ctx[d]->stream));
        }
        MH_HIP(B.recv.ensure(32 * (uint64_t)K));
        send[d] = B.send.as<uint8_t>();
        recv[d] = B.recv.as<uint8_t>();
    }
    if (int st = gather_roots(m, send, recv)) return st;
    mh_multi::Dev &B0 = *m->buf[0];
    MH_HIP(hipSetDevice(m->dev[0]));
    MH_HIP(B0.top.ensure(mh_htree_levels_len(G) * 32 + 32));
    uint8_t *d_root = B0.top.as<uint8_t>() + mh_htree_levels_len(G) * 32;
    if (int e = mh_dev_htree_reduce_nodes(m->ctx[0], recv[0], G, B0.top.as<uint8_t>(), d_root))
        return e;
    if (int e = per_device((int)G, [&](int d) -> int {
            const uint64_t g = (uint64_t)d;
            mh_multi::Dev &B = *m->buf[d];
            const uint64_t lo = g * S, ng = std::min(S, n - lo);
            MH_HIP(hipSetDevice(m->dev[d]));
            hipStream_t st = m->ctx[d]->stream;
            if (hvals_out)
                MH_HIP(hipMemcpyAsync(hvals_out + lo * 32, B.hv.p, ng * 32,
                                      hipMemcpyDeviceToHost, st));
            if (levels_out) {
                // global level l <= kS restricted to this shard = the shard's
                // level l; above the (short) last shard's own root, that root
                // is promoted unchanged (htree.go:100-103)
                LevelGeom lg;
                lg.init(ng);
                for (int l = 0; l <= kS && l < gg.nlevels; l++) {
                    const int ll = std::min(l, lg.nlevels - 1);
                    MH_HIP(hipMemcpyAsync(levels_out + (gg.off[l] + (lo >> l)) * 32,
                                          B.levels.as<uint8_t>() + lg.off[ll] * 32,
                                          (l < lg.nlevels ? lg.width[l] : 1) * 32,
                                          hipMemcpyDeviceToHost, st));
                }
            }
            return MH_OK;
        }))
        return e;
    hipStream_t st0 = m->ctx[0]->stream;
    if (levels_out && G > 1) {
        LevelGeom tg;
        tg.init(G);
        for (int j = 1; j < tg.nlevels; j++)
            MH_HIP(hipMemcpyAsync(levels_out + gg.off[kS + j] * 32,
                                  B0.top.as<uint8_t>() + tg.off[j] * 32, tg.width[j] * 32,
                                  hipMemcpyDeviceToHost, st0));
    }
    MH_HIP(hipMemcpyAsync(root, d_root, 32, hipMemcpyDeviceToHost, st0));
    for (int d = 0; d < K; d++)
        if (int e = mh_ctx_synchronize(m->ctx[d])) return e;
    return MH_OK;
}

int log2_exact(uint64_t S) {
    int k = 0;
    while ((1ull << k) < S) k++;
    return k;
}

}  // namespace

extern "C" int mh_multi_htree_build_entries_fixed(mh_multi *m, int version, uint64_t n,
                                                  const uint8_t *keys, uint32_t key_len,
                                                  const uint8_t *vals, uint32_t val_len,
                                                  uint8_t *hvals_out, uint8_t *levels_out,
                                                  uint8_t root[32]) {
    return mh_guard([&]() -> int {
        if (!m || (version != 0 && version != 1) || !root) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n && ((key_len && !keys) || (val_len && !vals))) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n == 0) {
            memcpy(root, kEmptyRoot, 32);  // htree.go:73-77
            return MH_OK;
        }
        std::lock_guard<std::mutex> lk(m->mu);
        uint64_t S = 0, G = 0;
        mh_multi_shard_plan(n, m->K, &S, &G);
        // 1. shards in, subtree per device (host copies on each device's stream,
        //    every device from its own thread)
        if (int e = per_device((int)G, [&](int d) -> int {
                const uint64_t g = (uint64_t)d;
                mh_multi::Dev &B = *m->buf[d];
                const uint64_t lo = g * S, ng = std::min(S, n - lo);
                MH_HIP(hipSetDevice(m->dev[d]));
                MH_HIP(B.keys.ensure(ng * key_len + 16));
                MH_HIP(B.vals.ensure(ng * val_len + 16));
                MH_HIP(B.hv.ensure(ng * 32));
                MH_HIP(B.levels.ensure(mh_htree_levels_len(ng) * 32));
                MH_HIP(B.send.ensure(32));
                hipStream_t st = m->ctx[d]->stream;
                if (key_len)
                    MH_HIP(hipMemcpyAsync(B.keys.p, keys + lo * key_len, ng * key_len,
                                          hipMemcpyHostToDevice, st));
                if (val_len)
                    MH_HIP(hipMemcpyAsync(B.vals.p, vals + lo * val_len, ng * val_len,
                                          hipMemcpyHostToDevice, st));
                return mh_dev_htree_build_entries_fixed(m->ctx[d], version, ng,
                                                        B.keys.as<uint8_t>(), key_len,
                                                        B.vals.as<uint8_t>(), val_len,
                                                        B.hv.as<uint8_t>(), B.levels.as<uint8_t>(),
                                                        B.send.as<uint8_t>());
            }))
            return e;
        return multi_htree_finish(m, n, S, G, log2_exact(S), hvals_out, levels_out, root);
    });
}

extern "C" int mh_multi_htree_build_entries(mh_multi *m, int version, uint64_t n,
                                            const uint8_t *keys, const uint64_t *key_off,
                                            const uint8_t *md, const uint64_t *md_off,
                                            const uint8_t *vals, const uint64_t *val_off,
                                            const uint8_t *hval_override,
                                            const uint8_t *use_override, uint8_t *hvals_out,
                                            uint8_t *levels_out, uint8_t root[32]) {
    return mh_guard([&]() -> int {
        if (!m || (version != 0 && version != 1) || !root) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((hval_override == nullptr) != (use_override == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((md == nullptr) != (md_off == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n == 0) {
            memcpy(root, kEmptyRoot, 32);  // htree.go:73-77
            return MH_OK;
        }
        if (!key_off || !val_off || !keys || !vals) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(key_off, n) || !monotonic(val_off, n) || (md_off && !monotonic(md_off, n)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (version == 0 && md_off && md_off[n] != md_off[0])
            return MH_ERR_METADATA_UNSUPPORTED;  // tx.go:691-693
        std::lock_guard<std::mutex> lk(m->mu);
        uint64_t S = 0, G = 0;
        mh_multi_shard_plan(n, m->K, &S, &G);
        // 1. each shard's CSR slices in (bytes [off[lo], off[hi]) and the
        //    offsets [lo, hi] unchanged, read through base pointers shifted by
        //    off[lo]), subtree per device, every device from its own thread
        if (int e = per_device((int)G, [&](int d) -> int {
                const uint64_t g = (uint64_t)d;
                mh_multi::Dev &B = *m->buf[d];
                const uint64_t lo = g * S, ng = std::min(S, n - lo), hi = lo + ng;
                const uint64_t kb = key_off[hi] - key_off[lo], vb = val_off[hi] - val_off[lo];
                // v0 never has metadata (checked above): no md arrays for it
                const bool use_md = md_off && version == 1;
                const uint64_t mb = use_md ? md_off[hi] - md_off[lo] : 0;
                const uint64_t offb = (ng + 1) * 8;
                auto pad8 = [](uint64_t x) { return (x + 16 + 7) & ~7ull; };
                MH_HIP(hipSetDevice(m->dev[d]));
                // keys | key offsets | md | md offsets  in B.keys; vals | val offsets in B.vals
                MH_HIP(B.keys.ensure(pad8(kb) + offb + (use_md ? pad8(mb) + offb : 0)));
                MH_HIP(B.vals.ensure(pad8(vb) + offb));
                MH_HIP(B.hv.ensure(ng * 32));
                MH_HIP(B.levels.ensure(mh_htree_levels_len(ng) * 32));
                MH_HIP(B.send.ensure(32));
                if (hval_override) MH_HIP(B.ovr.ensure(ng * 33 + 16));
                hipStream_t st = m->ctx[d]->stream;
                uint8_t *kd = B.keys.as<uint8_t>();
                uint64_t *kod = reinterpret_cast<uint64_t *>(kd + pad8(kb));
                uint8_t *mdd = reinterpret_cast<uint8_t *>(kod + ng + 1);
                uint64_t *mod = reinterpret_cast<uint64_t *>(mdd + pad8(mb));
                uint8_t *vd = B.vals.as<uint8_t>();
                uint64_t *vod = reinterpret_cast<uint64_t *>(vd + pad8(vb));
                if (kb) MH_HIP(hipMemcpyAsync(kd, keys + key_off[lo], kb, hipMemcpyHostToDevice, st));
                MH_HIP(hipMemcpyAsync(kod, key_off + lo, offb, hipMemcpyHostToDevice, st));
                if (vb) MH_HIP(hipMemcpyAsync(vd, vals + val_off[lo], vb, hipMemcpyHostToDevice, st));
                MH_HIP(hipMemcpyAsync(vod, val_off + lo, offb, hipMemcpyHostToDevice, st));
                if (use_md) {
                    if (mb) MH_HIP(hipMemcpyAsync(mdd, md + md_off[lo], mb, hipMemcpyHostToDevice, st));
                    MH_HIP(hipMemcpyAsync(mod, md_off + lo, offb, hipMemcpyHostToDevice, st));
                }
                uint8_t *ovd = nullptr, *used = nullptr;
                if (hval_override) {
                    ovd = B.ovr.as<uint8_t>();
                    used = ovd + ng * 32;
                    MH_HIP(hipMemcpyAsync(ovd, hval_override + lo * 32, ng * 32,
                                          hipMemcpyHostToDevice, st));
                    MH_HIP(hipMemcpyAsync(used, use_override + lo, ng, hipMemcpyHostToDevice, st));
                }
                return mh_dev_htree_build_entries(
                    m->ctx[d], version, ng, kd - key_off[lo], kod,
                    use_md ? mdd - md_off[lo] : nullptr, use_md ? mod : nullptr, vd - val_off[lo],
                    vod, ovd, used, B.hv.as<uint8_t>(), B.levels.as<uint8_t>(),
                    B.send.as<uint8_t>());
            }))
            return e;
        return multi_htree_finish(m, n, S, G, log2_exact(S), hvals_out, levels_out, root);
    });
}

// ============================================================================
// Sharded ahtree batch append (C3 at scale; ahtree.go:246-373 over K devices).
// A batch of `total` appends to an EMPTY tree is cut into K ranges of S = 2^k
// appends (the smallest S with K*S >= total); device d appends (dS, dS + m_d]
// into its own globally indexed dLog: the leaves, the perfect nodes of levels
// <= k and every spine node below level k lie inside its range; only the
// nodes above level k need the other ranges, and they are built from the
// complete shards' roots, all-gathered once (32 B per device, RCCL).  The
// phases are the ones mh_dev_ahtree_append_local / put_shard_roots /
// append_spine expose to torch.distributed ranks.
// ============================================================================
namespace {

int ahtree_shard_bits(uint64_t total, int K) {
    int k = 0;
    while ((uint64_t)K * (1ull << k) < total) k++;
    return k;
}

// phases 2-3 once every device has run phase 1 into dlog[d]: shard roots
// all-gathered, the nodes above shard level, then each device's spine
int ahtree_multi_finish(mh_multi *m, uint64_t total, int k, uint8_t *const *dlog,
                        uint8_t *const *roots_out) {
    const int K = m->K;
    const uint64_t S = 1ull << k;
    std::vector<const uint8_t *> send(K);
    std::vector<uint8_t *> recv(K);
    for (int d = 0; d < K; d++) {
        mh_multi::Dev &B = *m->buf[d];
        MH_HIP(hipSetDevice(m->dev[d]));
        const uint64_t n0 = std::min((uint64_t)d * S, total), md = std::min(S, total - n0);
        if (md == S) {
            send[d] = dlog[d] + 32 * mh_ahtree_node_index(n0 + S, k);
        } else {  // a short or empty last range has no shard root: zeros, unused
            MH_HIP(B.send.ensure(32));
            MH_HIP(hipMemsetAsync(B.send.p, 0, 32, m->ctx[d]->stream));
            send[d] = B.send.as<uint8_t>();
        }
        MH_HIP(B.recv.ensure(32 * (uint64_t)K));
        recv[d] = B.recv.as<uint8_t>();
    }
    if (int st = gather_roots(m, send, recv)) return st;
    const uint64_t complete = std::min<uint64_t>(total / S, (uint64_t)K);
    for (int d = 0; d < K; d++) {
        const uint64_t n0 = std::min((uint64_t)d * S, total), md = std::min(S, total - n0);
        if (!md) continue;
        if (int st = mh_dev_ahtree_put_shard_roots(m->ctx[d], dlog[d], k, complete, recv[d]))
            return st;
        if (int st = mh_dev_ahtree_append_spine(m->ctx[d], dlog[d], n0, md,
                                                roots_out ? roots_out[d] : nullptr))
            return st;
    }
    return MH_OK;
}

}  // namespace

extern "C" int mh_multi_dev_ahtree_append_batch(mh_multi *m, uint64_t total,
                                                const uint8_t *const *payloads, uint32_t plen,
                                                uint8_t *const *dlog, uint8_t *const *roots_out) {
    return mh_guard([&]() -> int {
        if (!m || !dlog || (total && !payloads)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (total == 0) return MH_OK;
        std::lock_guard<std::mutex> lk(m->mu);
        const int K = m->K;
        const int k = ahtree_shard_bits(total, K);
        const uint64_t S = 1ull << k;
        for (int d = 0; d < K; d++) {
            const uint64_t n0 = std::min((uint64_t)d * S, total), md = std::min(S, total - n0);
            if (!md) continue;
            if (!dlog[d] || (plen && !payloads[d])) return MH_ERR_ILLEGAL_ARGUMENTS;
            if (int st = mh_dev_ahtree_append_local(m->ctx[d], dlog[d], n0, payloads[d], md, plen,
                                                    k))
                return st;
        }
        return ahtree_multi_finish(m, total, k, dlog, roots_out);
    });
}

extern "C" int mh_multi_ahtree_append_batch(mh_multi *m, const uint8_t *payloads, uint64_t total,
                                            uint32_t plen, uint8_t *dlog_out, uint8_t root[32]) {
    return mh_guard([&]() -> int {
        if (!m || !root || (total && plen && !payloads)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (total == 0) return MH_ERR_UNEXISTENT_DATA;  // RootAt(0) of an empty tree
        std::lock_guard<std::mutex> lk(m->mu);
        const int K = m->K;
        const int k = ahtree_shard_bits(total, K);
        const uint64_t S = 1ull << k;
        const uint64_t nd = mh_ahtree_nodes_upto(total);
        int last = 0;  // device of the last append: its final root is RootAt(total)
        for (int d = 0; d < K; d++)
            if ((uint64_t)d * S < total) last = d;
        std::vector<uint8_t *> dl(K, nullptr), ro(K, nullptr);
        // 1. payload ranges in, leaves + perfect nodes up to shard level (every
        //    device from its own thread: each range crosses its own PCIe link)
        if (int e = per_device(K, [&](int d) -> int {
                const uint64_t n0 = std::min((uint64_t)d * S, total), md = std::min(S, total - n0);
                if (!md) return MH_OK;
                mh_multi::Dev &B = *m->buf[d];
                MH_HIP(hipSetDevice(m->dev[d]));
                MH_HIP(B.dlog.ensure(nd * 32));
                MH_HIP(B.vals.ensure(md * plen + 16));
                if (d == last) MH_HIP(B.hv.ensure(md * 32));
                dl[d] = B.dlog.as<uint8_t>();
                if (d == last) ro[d] = B.hv.as<uint8_t>();
                hipStream_t st = m->ctx[d]->stream;
                if (plen)
                    MH_HIP(hipMemcpyAsync(B.vals.p, payloads + n0 * plen, md * plen,
                                          hipMemcpyHostToDevice, st));
                return mh_dev_ahtree_append_local(m->ctx[d], dl[d], n0, B.vals.as<uint8_t>(), md,
                                                  plen, k);
            }))
            return e;
        // 2-3. shard roots exchanged, nodes above shard level, spines
        if (int st = ahtree_multi_finish(m, total, k, dl.data(), ro.data())) return st;
        // 4. every device's own dLog range back (ranges tile [0, nodesUpto(total)))
        if (int e = per_device(K, [&](int d) -> int {
                const uint64_t n0 = std::min((uint64_t)d * S, total), md = std::min(S, total - n0);
                if (!md) return MH_OK;
                MH_HIP(hipSetDevice(m->dev[d]));
                hipStream_t st = m->ctx[d]->stream;
                if (dlog_out) {
                    const uint64_t lo = mh_ahtree_node_index(n0 + 1, 0);
                    const uint64_t hi = mh_ahtree_nodes_upto(n0 + md);
                    MH_HIP(hipMemcpyAsync(dlog_out + lo * 32, dl[d] + lo * 32, (hi - lo) * 32,
                                          hipMemcpyDeviceToHost, st));
                }
                if (d == last)
                    MH_HIP(hipMemcpyAsync(root, ro[d] + (md - 1) * 32, 32, hipMemcpyDeviceToHost,
                                          st));
                return mh_ctx_synchronize(m->ctx[d]);
            }))
            return e;
        return MH_OK;
    });
}
