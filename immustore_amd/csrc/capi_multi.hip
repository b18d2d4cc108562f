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
    ncclResult_t (*abort)(ncclComm_t) = nullptr;
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
        r.abort = (decltype(r.abort))dlsym(h, "ncclCommAbort");
        r.ok = r.init_all && r.destroy && r.all_gather && r.group_start && r.group_end && r.abort;
    });
    return r;
}

#define MH_NCCL(expr)                                      \
    do {                                                   \
        if ((expr) != ncclSuccess) return MH_ERR_COLLECTIVE; \
    } while (0)

// Ends an open RCCL group on scope exit unless end() already did.
struct RcclGroup {
    const Rccl &r;
    bool open = true;
    explicit RcclGroup(const Rccl &rr) : r(rr) {}
    ncclResult_t end() {
        open = false;
        return r.group_end();
    }
    ~RcclGroup() {
        if (open) r.group_end();
    }
};

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
    // the clique was aborted (a collective failed after others of the same
    // group were queued): every later collective returns MH_ERR_COLLECTIVE
    bool broken = false;
    struct Dev {
        DevBuf keys, vals, hv, levels, send, recv, top, dlog, ovr;
        DevBuf fr, pk, ctr;  // ranged ahtree append: frontier, old peaks, work queue
    };
    std::vector<std::unique_ptr<Dev>> buf;
    std::vector<hipEvent_t> ev;  // duplicate-device gathers (one per context)
    std::vector<mh_commit_pipe *> pipe;  // mh_multi_precommit_batch: one per context, made on first use
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
            if (c && R.ok && !m->broken) R.destroy(c);  // aborted comms are gone
        for (int d = 0; d < (int)m->buf.size(); d++) {
            hipSetDevice(m->dev[d]);
            m->buf[d].reset();  // frees on the owning device
            if (d < (int)m->ev.size()) hipEventDestroy(m->ev[d]);
        }
        for (mh_commit_pipe *p : m->pipe)
            if (p) mh_commit_pipe_free(p);
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

// All-gather of `bytes` per device (send[d] -> recv[d] = K x bytes), on each
// device's context stream.
int gather_bytes(mh_multi *m, const std::vector<const uint8_t *> &send,
                 const std::vector<uint8_t *> &recv, uint64_t bytes) {
    if (!m->use_rccl) {
        // shards sharing devices: wait for every subtree, then copy the
        // slices; every stream then waits for every stream's copies, so no
        // later work on stream s (which may overwrite send[s]) can overtake a
        // copy that reads it
        for (int d = 0; d < m->K; d++)
            if (int st = mh_ctx_synchronize(m->ctx[d])) return st;
        if ((int)m->ev.size() < m->K) {
            for (int d = (int)m->ev.size(); d < m->K; d++) {
                MH_HIP(hipSetDevice(m->dev[d]));
                hipEvent_t e;
                MH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                m->ev.push_back(e);
            }
        }
        for (int d = 0; d < m->K; d++) {
            MH_HIP(hipSetDevice(m->dev[d]));
            for (int s = 0; s < m->K; s++)
                MH_HIP(hipMemcpyAsync(recv[d] + bytes * s, send[s], bytes, hipMemcpyDefault,
                                      m->ctx[d]->stream));
            MH_HIP(hipEventRecord(m->ev[d], m->ctx[d]->stream));
        }
        for (int s = 0; s < m->K; s++) {
            MH_HIP(hipSetDevice(m->dev[s]));
            for (int d = 0; d < m->K; d++)
                if (d != s) MH_HIP(hipStreamWaitEvent(m->ctx[s]->stream, m->ev[d], 0));
        }
        return MH_OK;
    }
    const Rccl &R = rccl();
    if (m->broken) return MH_ERR_COLLECTIVE;
    // every device selectable before the group opens, so a plain HIP error
    // cannot stop the loop below half way
    for (int d = 0; d < m->K; d++) MH_HIP(hipSetDevice(m->dev[d]));
    MH_NCCL(R.group_start());
    // every exit after ncclGroupStart ends the group: an open group would
    // defer every later RCCL call of this thread into it (the next build
    // would hang instead of failing)
    RcclGroup group(R);
    int queued = 0, st = MH_OK;
    for (int d = 0; d < m->K && st == MH_OK; d++) {
        if (mh_fault(MH_FAULT_RCCL_GROUP) || hipSetDevice(m->dev[d]) != hipSuccess ||
            R.all_gather(send[d], recv[d], bytes, ncclUint8, m->comm[d], m->ctx[d]->stream) !=
                ncclSuccess)
            st = MH_ERR_COLLECTIVE;
        else
            queued++;
    }
    if (st == MH_OK && mh_fault(MH_FAULT_RCCL_GROUP_LATE)) st = MH_ERR_COLLECTIVE;
    const ncclResult_t ge = group.end();
    if (st == MH_OK && ge == ncclSuccess) return MH_OK;
    if (queued > 0) {
        // the collectives queued for devices 0..queued-1 were launched by
        // ncclGroupEnd and wait for peers that never join: abort the clique
        // (ncclCommAbort ends its pending operations) so those streams drain,
        // and refuse every later collective on this handle
        m->broken = true;
        for (ncclComm_t c : m->comm)
            if (c) R.abort(c);
    }
    return MH_ERR_COLLECTIVE;
}

int gather_roots(mh_multi *m, const std::vector<const uint8_t *> &send,
                 const std::vector<uint8_t *> &recv) {
    return gather_bytes(m, send, recv, 32);
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
// Sharded ahtree batch append onto a tree of any size n0 (C3 at scale, and
// the replay of syncBinaryLinking, immustore.go:1198-1232, which resumes at
// aht.Size()+1 on every open, :686-693): ahtree.go:246-373 over K devices.
//
// The batch (n0, n0 + total] is cut at multiples of S = 2^k into G <= K
// ranges (b[d], b[d+1]] of nearly equal size (S <= total / 8K, so each range
// holds >= 8 aligned pieces of S appends and the split is within 1/8 of even).
// Every node an append reads is either inside its own range or a PEAK of the
// range's left end b[d] (the perfect subtree of a set bit of b[d]; for the
// first range these are the old tree's peaks, which the caller passes), so a
// device keeps only its own dLog range plus a 64-slot frontier:
//   1. leaves + perfect nodes of levels 1..k ending in (b[d], b[d+1]]
//      (range 0 reads the old peaks below level k; the others read nothing
//      outside their range);
//   2. all-gather of the level-k roots of the complete pieces (<= Pmax per
//      device; RCCL, 32 B each);
//   3. the piece tree above level k (replicated, tens of nodes), its nodes
//      that end in the device's range into its dLog range, the peaks of
//      b[d] into its frontier;
//   4. the spine chains of the range (left nodes at or before b[d] from the
//      frontier).
// ============================================================================
namespace {

struct AhtPlan {
    int k = 0, G = 0;
    uint64_t b[kAhtMaxRanges + 1] = {};
};

int aht_plan(uint64_t n0, uint64_t total, int ndev, AhtPlan &p) {
    if (ndev < 1 || ndev > kAhtMaxRanges || total > ~0ull - n0) return MH_ERR_ILLEGAL_ARGUMENTS;
    p = AhtPlan();
    p.b[0] = n0;
    if (!total) return MH_OK;
    const uint64_t target = total / (uint64_t)ndev + (total % (uint64_t)ndev != 0);
    while (p.k < 62 && (16ull << p.k) <= target) p.k++;  // largest S with 8 S <= target
    const uint64_t S = 1ull << p.k, end = n0 + total;
    for (int d = 1; d < ndev; d++) {
        const unsigned __int128 x = (unsigned __int128)total * (unsigned)d + (unsigned)ndev / 2;
        const uint64_t want = n0 + (uint64_t)(x / (unsigned)ndev);
        uint64_t r = (want >> p.k) << p.k;  // nearest multiple of S
        if (S > 1 && want - r >= S / 2) r += S;
        if (r > p.b[p.G] && r < end) p.b[++p.G] = r;
    }
    p.b[++p.G] = end;
    return MH_OK;
}

// packed peaks of n (lowest level first, popcount(n) x 32 B) -> 64 slots
void expand_peaks(uint64_t n, const uint8_t *packed, AhtSlots &slots) {
    memset(slots.b, 0, sizeof slots.b);
    int q = 0;
    for (int l = 0; l < 64; l++)
        if ((n >> l) & 1) memcpy(slots.b + l * 32, packed + 32 * (q++), 32);
}

inline uint8_t *range_base(uint8_t *buf, uint64_t lo) {
    // dLog index x of the range lives at buf + (x - nodesUpto(lo)) * 32
    return reinterpret_cast<uint8_t *>((uintptr_t)buf - (uintptr_t)(ahtree_nodes_upto(lo) * 32));
}

// The piece-tree geometry of a plan (shared by every range): send slots per
// device (Pmax) and the slot count of the replicated top buffer.
AhtTopArgs aht_top_args(const AhtPlan &p, uint64_t *top_slots) {
    const int G = p.G, k = p.k;
    const uint64_t n0 = p.b[0];
    uint64_t Pmax = 1;
    AhtTopArgs ta;
    ta.k = k;
    ta.G = G;
    ta.n0 = n0;
    ta.N0 = n0 >> k;
    ta.Pend = p.b[G] >> k;
    for (int d = 0; d <= G; d++) ta.pe0[d] = p.b[d] >> k;
    for (int d = 0; d < G; d++) Pmax = std::max<uint64_t>(Pmax, ta.pe0[d + 1] - ta.pe0[d]);
    ta.Pmax = Pmax;
    uint64_t slots = 0;
    ta.nlev = 0;
    while (ta.nlev < 64 - k && (ta.Pend >> ta.nlev) != 0) {
        ta.lev_off[ta.nlev] = slots;
        slots += (ta.Pend >> ta.nlev) - (ta.N0 >> ta.nlev) + 1;
        ta.nlev++;
    }
    *top_slots = slots;
    return ta;
}

// Device buffers of one range: the old peaks of n0 (pk) and the frontier of
// its left end (fr), 64 slots each, the spine work queue and the top tree.
struct AhtRangeBufs {
    uint8_t *pk = nullptr, *fr = nullptr, *top = nullptr;
    uint32_t *ctr = nullptr;
};

// Phase 1 of range d on its context's stream: the old peaks in, leaves +
// perfect levels (all of them when one range holds the batch), then -- with
// more than one range -- the level-k roots of its complete pieces into send
// (Pmax slots).
int aht_range_local(mh_ctx *c, const AhtPlan &p, const AhtTopArgs &ta, int d,
                    const AhtSlots &slots, const uint8_t *payload, uint32_t plen, uint8_t *dlog,
                    const AhtRangeBufs &B, uint8_t *send) {
    hipStream_t st = c->stream;
    // by value through the kernel arguments: nothing host-side to outlive
    MH_HIP(launch_ahtree_put_slots(st, slots, B.pk));
    const uint64_t lo = p.b[d], hi = p.b[d + 1];
    uint8_t *vb = range_base(dlog, lo);
    AhtEdge edge;
    edge.fr = d ? B.fr : B.pk;
    edge.lo = lo;
    MH_HIP(launch_ahtree_leaves(st, c->tm(), vb, lo, payload, hi - lo, plen));
    MH_HIP(launch_ahtree_perfect(st, c->tm(), vb, lo, hi, 1, p.G == 1 ? 63 : p.k, edge));
    if (p.G > 1 && send)
        MH_HIP(launch_ahtree_gather_pieces(st, vb, p.k, ta.pe0[d] + 1, ta.pe0[d + 1] - ta.pe0[d],
                                           send));
    return MH_OK;
}

// Phases 3-4 of range d once recv holds every range's piece roots (range r
// at r * Pmax slots): the piece tree, its nodes ending in the range, the
// frontier, then the spines.
int aht_range_finish(mh_ctx *c, const AhtPlan &p, const AhtTopArgs &ta, int d,
                     const uint8_t *recv, uint8_t *dlog, const AhtRangeBufs &B,
                     uint8_t *roots_out) {
    hipStream_t st = c->stream;
    uint8_t *vb = range_base(dlog, p.b[d]);
    if (p.G > 1) {
        AhtTopArgs a = ta;
        a.lo = p.b[d];
        a.hi = p.b[d + 1];
        MH_HIP(launch_ahtree_top(st, a, recv, B.pk, B.top, vb, B.fr));
    }
    AhtEdge edge;
    edge.fr = d ? B.fr : B.pk;
    edge.lo = p.b[d];
    MH_HIP(launch_ahtree_spine(st, c->tm(), vb, p.b[d], p.b[d + 1] - p.b[d], roots_out, B.ctr,
                               edge));
    return MH_OK;
}

// Phases 1-4 for ranges already planned; payload[d] / dlog[d] are device
// pointers of range d (dlog[d] holds nodesUpto(b[d+1]) - nodesUpto(b[d])
// digests), slots = the old peaks of n0 in the 64-slot layout (host).
int aht_multi_run(mh_multi *m, const AhtPlan &p, const AhtSlots &slots,
                  const std::vector<const uint8_t *> &payload, uint32_t plen,
                  const std::vector<uint8_t *> &dlog, const std::vector<uint8_t *> &roots_out) {
    const int K = m->K, G = p.G;
    uint64_t top_slots = 0;
    const AhtTopArgs ta = aht_top_args(p, &top_slots);
    const uint64_t Pmax = ta.Pmax;
    std::vector<AhtRangeBufs> rb(K);
    std::vector<const uint8_t *> send(K);
    std::vector<uint8_t *> recv(K);
    for (int d = 0; d < K; d++) {
        mh_multi::Dev &B = *m->buf[d];
        MH_HIP(hipSetDevice(m->dev[d]));
        MH_HIP(B.pk.ensure(64 * 32));
        MH_HIP(B.fr.ensure(64 * 32));
        MH_HIP(B.ctr.ensure(256));
        MH_HIP(B.top.ensure(top_slots * 32));
        MH_HIP(B.send.ensure(Pmax * 32));
        MH_HIP(B.recv.ensure((uint64_t)K * Pmax * 32));
        rb[d].pk = B.pk.as<uint8_t>();
        rb[d].fr = B.fr.as<uint8_t>();
        rb[d].top = B.top.as<uint8_t>();
        rb[d].ctr = B.ctr.as<uint32_t>();
        send[d] = B.send.as<uint8_t>();
        recv[d] = B.recv.as<uint8_t>();
    }
    // 1. leaves + perfect levels, the pieces' level-k roots into send
    for (int d = 0; d < G; d++) {
        MH_HIP(hipSetDevice(m->dev[d]));
        if (int st = aht_range_local(m->ctx[d], p, ta, d, slots, payload[d], plen, dlog[d], rb[d],
                                     m->buf[d]->send.as<uint8_t>()))
            return st;
    }
    // 2. all-gather of Pmax slots per device
    if (G > 1)
        if (int st = gather_bytes(m, send, recv, Pmax * 32)) return st;
    // 3-4. piece tree, the device's nodes above level k, its frontier; spines
    for (int d = 0; d < G; d++) {
        MH_HIP(hipSetDevice(m->dev[d]));
        if (int st = aht_range_finish(m->ctx[d], p, ta, d, recv[d], dlog[d], rb[d], roots_out[d]))
            return st;
    }
    return MH_OK;
}

// The work buffer of the one-range-per-process form: pk | fr | ctr | top.
constexpr uint64_t kAhtWorkHead = 64 * 32 * 2 + 256;

AhtRangeBufs aht_work_bufs(uint8_t *work) {
    AhtRangeBufs B;
    B.pk = work;
    B.fr = work + 64 * 32;
    B.ctr = reinterpret_cast<uint32_t *>(work + 64 * 32 * 2);
    B.top = work + kAhtWorkHead;
    return B;
}

int peaks_ok(uint64_t n0, const uint8_t *peaks) { return n0 == 0 || peaks != nullptr; }

}  // namespace

extern "C" int mh_ahtree_range_plan(uint64_t n0, uint64_t total, int ndev, int *shard_bits,
                                    uint64_t *bounds, int *nranges) {
    return mh_guard([&]() -> int {
        if (!shard_bits || !bounds || !nranges) return MH_ERR_ILLEGAL_ARGUMENTS;
        AhtPlan p;
        if (int st = aht_plan(n0, total, ndev, p)) return st;
        *shard_bits = p.k;
        *nranges = p.G;
        for (int d = 0; d <= p.G; d++) bounds[d] = p.b[d];
        return MH_OK;
    });
}

extern "C" int mh_ahtree_range_sizes(uint64_t n0, uint64_t total, int ndev, uint64_t *send_bytes,
                                     uint64_t *work_bytes) {
    return mh_guard([&]() -> int {
        if (!send_bytes || !work_bytes) return MH_ERR_ILLEGAL_ARGUMENTS;
        AhtPlan p;
        if (int st = aht_plan(n0, total, ndev, p)) return st;
        uint64_t top_slots = 0;
        const AhtTopArgs ta = aht_top_args(p, &top_slots);
        *send_bytes = ta.Pmax * 32;
        *work_bytes = kAhtWorkHead + top_slots * 32;
        return MH_OK;
    });
}

namespace {

// Arguments shared by the two per-rank calls: the plan, the range, the old
// peaks and the work buffer.
int aht_rank_setup(uint64_t n0, const uint8_t *peaks, uint64_t total, int world, int rank,
                   uint8_t *dlog_range, uint8_t *work, AhtPlan &p, AhtTopArgs &ta) {
    if (!peaks_ok(n0, peaks) || !work || world < 1 || rank < 0 || rank >= world || total == 0)
        return MH_ERR_ILLEGAL_ARGUMENTS;
    if (((uintptr_t)work & 15) || ((uintptr_t)dlog_range & 15)) return MH_ERR_ILLEGAL_ARGUMENTS;
    if (int st = aht_plan(n0, total, world, p)) return st;
    uint64_t top_slots = 0;
    ta = aht_top_args(p, &top_slots);
    if (rank < p.G && !dlog_range) return MH_ERR_ILLEGAL_ARGUMENTS;
    return MH_OK;
}

}  // namespace

extern "C" int mh_dev_ahtree_range_local(mh_ctx *c, uint64_t n0, const uint8_t *peaks,
                                         uint64_t total, int world, int rank,
                                         const uint8_t *payloads, uint32_t plen,
                                         uint8_t *dlog_range, uint8_t *work, uint8_t *send) {
    return mh_guard([&]() -> int {
        if (!c || !send) return MH_ERR_ILLEGAL_ARGUMENTS;
        AhtPlan p;
        AhtTopArgs ta;
        if (int st = aht_rank_setup(n0, peaks, total, world, rank, dlog_range, work, p, ta))
            return st;
        if (rank >= p.G) return MH_OK;  // no range: its send slots are never read
        if (plen && !payloads) return MH_ERR_ILLEGAL_ARGUMENTS;
        AhtSlots slots;
        expand_peaks(n0, peaks, slots);
        MH_HIP(hipSetDevice(c->device));
        std::lock_guard<std::mutex> lk(c->mu);
        return aht_range_local(c, p, ta, rank, slots, payloads, plen, dlog_range,
                               aht_work_bufs(work), send);
    });
}

extern "C" int mh_dev_ahtree_range_finish(mh_ctx *c, uint64_t n0, const uint8_t *peaks,
                                          uint64_t total, int world, int rank,
                                          const uint8_t *recv, uint8_t *dlog_range, uint8_t *work,
                                          uint8_t *roots_out) {
    return mh_guard([&]() -> int {
        if (!c) return MH_ERR_ILLEGAL_ARGUMENTS;
        AhtPlan p;
        AhtTopArgs ta;
        if (int st = aht_rank_setup(n0, peaks, total, world, rank, dlog_range, work, p, ta))
            return st;
        if (rank >= p.G) return MH_OK;
        if (p.G > 1 && !recv) return MH_ERR_ILLEGAL_ARGUMENTS;
        MH_HIP(hipSetDevice(c->device));
        std::lock_guard<std::mutex> lk(c->mu);
        return aht_range_finish(c, p, ta, rank, recv, dlog_range, aht_work_bufs(work), roots_out);
    });
}

extern "C" int mh_multi_dev_ahtree_append_batch(mh_multi *m, uint64_t n0, const uint8_t *peaks,
                                                uint64_t total, const uint8_t *const *payloads,
                                                uint32_t plen, uint8_t *const *dlog,
                                                uint8_t *const *roots_out) {
    return mh_guard([&]() -> int {
        if (!m || !dlog || (total && !payloads) || !peaks_ok(n0, peaks))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (total == 0) return MH_OK;
        AhtPlan p;
        if (int st = aht_plan(n0, total, m->K, p)) return st;
        std::vector<const uint8_t *> pay(m->K, nullptr);
        std::vector<uint8_t *> dl(m->K, nullptr), ro(m->K, nullptr);
        for (int d = 0; d < p.G; d++) {
            if (!dlog[d] || ((uintptr_t)dlog[d] & 15) || (plen && !payloads[d]))
                return MH_ERR_ILLEGAL_ARGUMENTS;
            pay[d] = payloads[d];
            dl[d] = dlog[d];
            ro[d] = roots_out ? roots_out[d] : nullptr;
        }
        AhtSlots slots;
        expand_peaks(n0, peaks, slots);
        std::lock_guard<std::mutex> lk(m->mu);
        return aht_multi_run(m, p, slots, pay, plen, dl, ro);
    });
}

extern "C" int mh_multi_ahtree_append_batch(mh_multi *m, uint64_t n0, const uint8_t *peaks,
                                            const uint8_t *payloads, uint64_t total, uint32_t plen,
                                            uint8_t *dlog_out, uint8_t root[32]) {
    return mh_guard([&]() -> int {
        if (!m || !root || (total && plen && !payloads) || !peaks_ok(n0, peaks))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        // nothing appended: RootAt(0) of an empty tree, or nothing to compute
        if (total == 0) return n0 ? MH_ERR_ILLEGAL_ARGUMENTS : MH_ERR_UNEXISTENT_DATA;
        AhtPlan p;
        if (int st = aht_plan(n0, total, m->K, p)) return st;
        AhtSlots slots;
        expand_peaks(n0, peaks, slots);
        std::lock_guard<std::mutex> lk(m->mu);
        const int G = p.G;
        const uint64_t base = ahtree_nodes_upto(n0);
        std::vector<const uint8_t *> pay(m->K, nullptr);
        std::vector<uint8_t *> dl(m->K, nullptr), ro(m->K, nullptr);
        // 0. each range's payloads in (every device from its own thread: each
        //    range crosses its own PCIe link)
        if (int e = per_device(G, [&](int d) -> int {
                mh_multi::Dev &B = *m->buf[d];
                const uint64_t lo = p.b[d], md = p.b[d + 1] - lo;
                MH_HIP(hipSetDevice(m->dev[d]));
                MH_HIP(B.dlog.ensure((ahtree_nodes_upto(p.b[d + 1]) - ahtree_nodes_upto(lo)) * 32));
                MH_HIP(B.vals.ensure(md * plen + 16));
                if (d == G - 1) MH_HIP(B.hv.ensure(md * 32));
                dl[d] = B.dlog.as<uint8_t>();
                pay[d] = B.vals.as<uint8_t>();
                if (d == G - 1) ro[d] = B.hv.as<uint8_t>();
                if (plen)
                    MH_HIP(hipMemcpyAsync(B.vals.p, payloads + (lo - n0) * plen, md * plen,
                                          hipMemcpyHostToDevice, m->ctx[d]->stream));
                return MH_OK;
            }))
            return e;
        if (int st = aht_multi_run(m, p, slots, pay, plen, dl, ro)) return st;
        // 5. every range's digests back (the ranges tile the new dLog stream)
        if (int e = per_device(G, [&](int d) -> int {
                MH_HIP(hipSetDevice(m->dev[d]));
                hipStream_t st = m->ctx[d]->stream;
                const uint64_t lo = ahtree_nodes_upto(p.b[d]), hi = ahtree_nodes_upto(p.b[d + 1]);
                if (dlog_out)
                    MH_HIP(hipMemcpyAsync(dlog_out + (lo - base) * 32, dl[d], (hi - lo) * 32,
                                          hipMemcpyDeviceToHost, st));
                if (d == G - 1)
                    MH_HIP(hipMemcpyAsync(root, ro[d] + (p.b[d + 1] - p.b[d] - 1) * 32, 32,
                                          hipMemcpyDeviceToHost, st));
                return mh_ctx_synchronize(m->ctx[d]);
            }))
            return e;
        return MH_OK;
    });
}

// ============================================================================
// The PCIe-bound batch paths over the node's GPUs (one Go process = one
// process: only mh_multi gives it more than one device).  Each call cuts its
// batch into K contiguous parts -- by index for proofs, at record boundaries
// for a tx log -- and runs the single-context call of part d on device d from
// its own thread, so every part crosses its own PCIe link; the outputs are the
// parts' outputs side by side, byte-equal to one single-context call over the
// whole batch.  K = 1 is that call.
// ============================================================================
namespace {

// [lo, hi) of part d of n items over K parts (nearly equal)
inline void split_part(uint64_t n, int K, int d, uint64_t &lo, uint64_t &hi) {
    lo = (uint64_t)((unsigned __int128)n * (unsigned)d / (unsigned)K);
    hi = (uint64_t)((unsigned __int128)n * (unsigned)(d + 1) / (unsigned)K);
}

// K + 1 item bounds splitting n items into K parts of nearly equal bytes,
// bytes(i) = the byte offset where item i starts (non-decreasing, i <= n)
template <class B>
std::vector<uint64_t> split_by_bytes(uint64_t n, int K, B bytes) {
    std::vector<uint64_t> t(K + 1, 0);
    t[K] = n;
    const uint64_t b0 = bytes(0), tot = bytes(n) - b0;
    for (int d = 1; d < K; d++) {
        const uint64_t want = b0 + (uint64_t)((unsigned __int128)tot * (unsigned)d / (unsigned)K);
        uint64_t lo = t[d - 1], hi = n;  // the first item starting at or after want
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if (bytes(mid) < want) lo = mid + 1;
            else hi = mid;
        }
        t[d] = lo;
    }
    return t;
}

}  // namespace

// htree.VerifyInclusion over n proofs (htree.go:166-195), split by index.
extern "C" int mh_multi_htree_verify_inclusion_batch(mh_multi *m, uint64_t n, const uint64_t *leaf,
                                                     const uint64_t *width, const uint64_t *term_off,
                                                     const uint8_t *terms, const uint8_t *digests,
                                                     const uint8_t *roots, uint8_t *ok) {
    return mh_guard([&]() -> int {
        if (!m) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (m->K == 1 || n < (uint64_t)m->K)
            return mh_htree_verify_inclusion_batch(m->ctx[0], n, leaf, width, term_off, terms,
                                                   digests, roots, ok);
        if (!leaf || !width || !term_off || !digests || !roots || !ok) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(term_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;  // before any part writes ok
        std::lock_guard<std::mutex> lk(m->mu);
        return per_device(m->K, [&](int d) -> int {
            uint64_t lo, hi;
            split_part(n, m->K, d, lo, hi);
            return mh_htree_verify_inclusion_batch(m->ctx[d], hi - lo, leaf + lo, width + lo,
                                                   term_off + lo, terms, digests + 32 * lo,
                                                   roots + 32 * lo, ok + lo);
        });
    });
}

// store.VerifyDualProofV2 over n proofs (verification.go:303-372), split by index.
extern "C" int mh_multi_verify_dual_proof_v2_batch(
    mh_multi *m, uint64_t n, const mh_tx_header *src_hdr, const mh_tx_header *tgt_hdr,
    const uint8_t *md_blob, uint64_t md_blob_len, const uint64_t *incl_off,
    const uint8_t *incl_terms, const uint64_t *cons_off, const uint8_t *cons_terms,
    const uint64_t *src, const uint64_t *tgt, const uint8_t *src_alh, const uint8_t *tgt_alh,
    int32_t *status) {
    return mh_guard([&]() -> int {
        if (!m) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (m->K == 1 || n < (uint64_t)m->K)
            return mh_verify_dual_proof_v2_batch(m->ctx[0], n, src_hdr, tgt_hdr, md_blob,
                                                 md_blob_len, incl_off, incl_terms, cons_off,
                                                 cons_terms, src, tgt, src_alh, tgt_alh, status);
        if (!src_hdr || !tgt_hdr || !incl_off || !cons_off || !src || !tgt || !src_alh ||
            !tgt_alh || !status)
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(incl_off, n) || !monotonic(cons_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(m->mu);
        return per_device(m->K, [&](int d) -> int {
            uint64_t lo, hi;
            split_part(n, m->K, d, lo, hi);
            return mh_verify_dual_proof_v2_batch(m->ctx[d], hi - lo, src_hdr + lo, tgt_hdr + lo,
                                                 md_blob, md_blob_len, incl_off + lo, incl_terms,
                                                 cons_off + lo, cons_terms, src + lo, tgt + lo,
                                                 src_alh + 32 * lo, tgt_alh + 32 * lo, status + lo);
        });
    });
}

// The read path's re-hash of a tx log (tx.go:388-630: replay,
// immustore.go:1198-1223; the indexer's readTx, indexer.go:570) over the
// devices: the host hop parses the record structure ONCE (txlog_hop: the
// call's structural status, the records, any re-encoded metadata), the
// records are cut into K parts of nearly equal bytes at record boundaries --
// every record carries its prevAlh, so the parts are independent -- and part
// d is validated by device d from that parse (txlog_validate_parsed: its own
// copy over its own link, no second hop).  A v1 header's md_off is
// relative to buf, as in the single call.
extern "C" int mh_multi_txlog_validate(mh_multi *m, const uint8_t *buf, uint64_t len,
                                       uint32_t max_entries, uint32_t max_key_len,
                                       uint64_t max_txs, uint64_t *ntx_out,
                                       uint64_t *consumed_out, mh_tx_header *hdrs_out,
                                       uint8_t *alh_out, int32_t *status_out) {
    return mh_guard([&]() -> int {
        if (!m) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (m->K == 1)
            return mh_txlog_validate(m->ctx[0], buf, len, max_entries, max_key_len, max_txs,
                                     ntx_out, consumed_out, hdrs_out, alh_out, status_out);
        if (len && !buf) return MH_ERR_ILLEGAL_ARGUMENTS;
        HopOut all;
        txlog_hop(buf, len, max_entries, max_key_len, max_txs, all);
        const uint64_t cnt = all.R.size(), used = all.end;
        const int rc = all.rc;
        if (ntx_out) *ntx_out = cnt;
        if (consumed_out) *consumed_out = used;
        if (!cnt) return rc;
        // part d: records [t[d], t[d+1]), bytes [start(t[d]), start(t[d+1]))
        const int K = m->K;
        auto start = [&](uint64_t t) -> uint64_t { return t ? all.R[t - 1].alh + 32 : 0; };
        std::vector<uint64_t> t(K + 1, 0);
        t[K] = cnt;
        for (int d = 1; d < K; d++) {
            const uint64_t want = (uint64_t)((unsigned __int128)used * (unsigned)d / (unsigned)K);
            uint64_t lo = 0, hi = cnt;  // the first record ending at or after want
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                if (all.R[mid].alh < want) lo = mid + 1; else hi = mid;
            }
            t[d] = std::max(t[d - 1], std::min(lo, cnt));
        }
        // each part's records and patches, rebased to the part
        std::vector<HopOut> part(K);
        size_t p = 0;
        for (int d = 0; d < K; d++) {
            const uint64_t t0 = t[d], t1 = t[d + 1], b0 = start(t0);
            HopOut &o = part[d];
            o.R.reserve(t1 - t0);
            for (uint64_t k = t0; k < t1; k++)
                o.R.push_back(HopRec{all.R[k].rec - b0, all.R[k].alh - b0, all.R[k].nent, 0});
            for (; p < all.P.size() && all.P[p].rec < t1; p++) {
                HopPatch pt = all.P[p];
                pt.rec -= t0;
                o.P.push_back(std::move(pt));
            }
            o.rc = MH_OK;
            o.end = start(t1) - b0;
        }
        std::lock_guard<std::mutex> lk(m->mu);
        const int st = per_device(K, [&](int d) -> int {
            const uint64_t t0 = t[d], t1 = t[d + 1];
            if (t1 == t0) return MH_OK;
            const uint64_t b0 = start(t0), b1 = start(t1);
            const int r = txlog_validate_parsed(m->ctx[d], buf + b0, b1 - b0, max_entries,
                                                max_key_len, part[d],
                                                hdrs_out ? hdrs_out + t0 : nullptr,
                                                alh_out ? alh_out + 32 * t0 : nullptr,
                                                status_out ? status_out + t0 : nullptr);
            if (r != MH_OK) return r < 0 ? r : MH_ERR_ILLEGAL_STATE;
            if (hdrs_out)
                for (uint64_t k = t0; k < t1; k++)
                    if (hdrs_out[k].version == 1) hdrs_out[k].md_off += (uint32_t)b0;
            return MH_OK;
        });
        if (st) return st;
        // a header whose tx metadata was re-encoded points at the canonical
        // copy placed after the log (md_off >= len): where the one-device call
        // places it, i.e. after the whole log, the patches in log order
        if (hdrs_out) {
            uint64_t side = 0;
            for (const HopPatch &pt : all.P) {
                if (pt.kind == 1 && pt.rec < cnt) hdrs_out[pt.rec].md_off = (uint32_t)(len + side);
                side += pt.bytes.size();
            }
        }
        return rc;
    });
}

// readValueAt's hVal check (immustore.go:3183-3240, the compare at :3235)
// over a batch of values, split into K parts of nearly equal value bytes.
// *ncorrupted (may be NULL) is the sum over the parts.
extern "C" int mh_multi_verify_values_batch(mh_multi *m, uint64_t n, const uint8_t *vals,
                                            const uint64_t *off, const uint64_t *vlen,
                                            const uint8_t *hvals, int32_t *status,
                                            uint64_t *ncorrupted) {
    return mh_guard([&]() -> int {
        if (!m) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (m->K == 1 || n < (uint64_t)m->K)
            return mh_verify_values_batch(m->ctx[0], n, vals, off, vlen, hvals, status, ncorrupted);
        if (!off || !vlen || !hvals || !status) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const std::vector<uint64_t> t = split_by_bytes(n, m->K, [&](uint64_t i) { return off[i]; });
        std::vector<uint64_t> bad(m->K, 0);
        std::lock_guard<std::mutex> lk(m->mu);
        const int st = per_device(m->K, [&](int d) -> int {
            const uint64_t lo = t[d], hi = t[d + 1];
            if (hi == lo) return MH_OK;
            return mh_verify_values_batch(m->ctx[d], hi - lo, vals, off + lo, vlen + lo,
                                          hvals + 32 * lo, status + lo, &bad[d]);
        });
        if (st) return st;
        if (ncorrupted) {
            uint64_t c = 0;
            for (uint64_t b : bad) c += b;
            *ncorrupted = c;
        }
        return MH_OK;
    });
}

// The fused DualProofV2 wire verify (DualProofV2FromProto,
// database_protoconv.go:226-262, + VerifyDualProofV2, verification.go:303-372)
// over n messages, split into K parts of nearly equal message bytes.
extern "C" int mh_multi_verify_dual_proof_v2_pb_batch(mh_multi *m, uint64_t n, const uint8_t *msgs,
                                                      const uint64_t *msg_off, const uint64_t *src,
                                                      const uint64_t *tgt, const uint8_t *src_alh,
                                                      const uint8_t *tgt_alh, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!m) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (m->K == 1 || n < (uint64_t)m->K)
            return mh_verify_dual_proof_v2_pb_batch(m->ctx[0], n, msgs, msg_off, src, tgt, src_alh,
                                                    tgt_alh, status);
        if (!msg_off || !src || !tgt || !src_alh || !tgt_alh || !status) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(msg_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const std::vector<uint64_t> t =
            split_by_bytes(n, m->K, [&](uint64_t i) { return msg_off[i]; });
        std::lock_guard<std::mutex> lk(m->mu);
        return per_device(m->K, [&](int d) -> int {
            const uint64_t lo = t[d], hi = t[d + 1];
            if (hi == lo) return MH_OK;
            return mh_verify_dual_proof_v2_pb_batch(m->ctx[d], hi - lo, msgs, msg_off + lo, src + lo,
                                                    tgt + lo, src_alh + 32 * lo,
                                                    tgt_alh + 32 * lo, status + lo);
        });
    });
}

// precommit's hashing (immustore.go:1620-1632, 2301-2313 -> tx.go:332-355) for
// a batch of transactions, split into K parts of whole transactions with
// nearly equal value bytes; part d runs on device d's own commit pipe (made
// on first use with the default chunk size).  Arguments and outputs as
// mh_precommit_batch; entry-indexed inputs keep their absolute indexing.
extern "C" int mh_multi_precommit_batch(mh_multi *m, int version, uint64_t max_width, uint64_t ntx,
                                        const uint64_t *tx_off, const uint8_t *keys,
                                        const uint64_t *key_off, const uint8_t *md,
                                        const uint64_t *md_off, const uint8_t *vals,
                                        const uint64_t *val_off, const uint8_t *hval_override,
                                        const uint8_t *use_override, const uint8_t *expect_eh,
                                        uint8_t *hvals_out, uint8_t *eh_out, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!m) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(m->mu);
        if (m->pipe.empty()) m->pipe.assign(m->K, nullptr);
        auto pipe = [&](int d) -> int {
            return m->pipe[d] ? MH_OK : mh_commit_pipe_new(m->ctx[d], 0, &m->pipe[d]);
        };
        if (m->K == 1 || ntx < (uint64_t)m->K) {
            if (int e = pipe(0)) return e;
            return mh_precommit_batch(m->pipe[0], version, max_width, ntx, tx_off, keys, key_off, md,
                                      md_off, vals, val_off, hval_override, use_override, expect_eh,
                                      hvals_out, eh_out, status);
        }
        if (!tx_off || !val_off || !status) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(tx_off, ntx)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(val_off + tx_off[0], tx_off[ntx] - tx_off[0])) return MH_ERR_ILLEGAL_ARGUMENTS;
        const std::vector<uint64_t> t =
            split_by_bytes(ntx, m->K, [&](uint64_t i) { return val_off[tx_off[i]]; });
        return per_device(m->K, [&](int d) -> int {
            const uint64_t lo = t[d], hi = t[d + 1];
            if (hi == lo) return MH_OK;
            if (int e = pipe(d)) return e;
            return mh_precommit_batch(m->pipe[d], version, max_width, hi - lo, tx_off + lo, keys,
                                      key_off, md, md_off, vals, val_off, hval_override, use_override,
                                      expect_eh ? expect_eh + 32 * lo : nullptr,
                                      hvals_out ? hvals_out + 32 * (tx_off[lo] - tx_off[0]) : nullptr,
                                      eh_out ? eh_out + 32 * lo : nullptr, status + lo);
        });
    });
}

// pkg/verification.VerifyDocument's hashing part (verification.go:37-196)
// for n documents, split into K parts of nearly equal work (entries + document
// bytes): part d is the same batch with its per-document arrays advanced to
// its first document; entry, term and byte arrays are indexed through the
// offsets, which index them directly, so they are shared.
extern "C" int mh_multi_verify_document_batch(mh_multi *m, const mh_document_batch *batch,
                                              int32_t *status, uint8_t *target_alh_out) {
    return mh_guard([&]() -> int {
        if (!m || !batch) return MH_ERR_ILLEGAL_ARGUMENTS;
        const uint64_t n = batch->n;
        if (m->K == 1 || n < (uint64_t)m->K)
            return mh_verify_document_batch(m->ctx[0], batch, status, target_alh_out);
        const mh_document_batch &B = *batch;
        if (!B.doc_off || !B.doc_key_off || !B.tx_hdr || !B.ent_off || !B.src_hdr || !B.tgt_hdr ||
            !B.incl_off || !B.cons_off || !B.known_tx_id || !B.known_alh || !status)
            return MH_ERR_ILLEGAL_ARGUMENTS;
        if (!monotonic(B.ent_off, n) || !monotonic(B.doc_off, n)) return MH_ERR_ILLEGAL_ARGUMENTS;
        const std::vector<uint64_t> t = split_by_bytes(n, m->K, [&](uint64_t i) {
            return (B.ent_off[i] - B.ent_off[0]) * 64 + (B.doc_off[i] - B.doc_off[0]);
        });
        std::lock_guard<std::mutex> lk(m->mu);
        return per_device(m->K, [&](int d) -> int {
            const uint64_t lo = t[d], hi = t[d + 1];
            if (hi == lo) return MH_OK;
            mh_document_batch P = B;
            P.n = hi - lo;
            P.doc_off = B.doc_off + lo;
            P.doc_key_off = B.doc_key_off + lo;
            P.tx_hdr = B.tx_hdr + lo;
            P.ent_off = B.ent_off + lo;
            P.src_hdr = B.src_hdr + lo;
            P.tgt_hdr = B.tgt_hdr + lo;
            P.incl_off = B.incl_off + lo;
            P.cons_off = B.cons_off + lo;
            P.known_tx_id = B.known_tx_id + lo;
            P.known_alh = B.known_alh + 32 * lo;
            return mh_verify_document_batch(m->ctx[d], &P, status + lo,
                                            target_alh_out ? target_alh_out + 32 * lo : nullptr);
        });
    });
}
