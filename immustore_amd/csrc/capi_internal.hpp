// capi_internal.hpp -- host-side objects shared by the C-ABI translation
// units (capi.hip: htree / ahtree handles; capi_tx.hip: tx layer).
#pragma once
#include <algorithm>
#include <condition_variable>
#include <deque>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <new>
#include <string>
#include <vector>

#include "mh_internal.hpp"

using namespace mh;

// Every extern "C" int entry point runs its body through mh_guard: a C++
// exception (std::bad_alloc from a host vector, std::system_error from a
// thread) becomes a status instead of crossing the C ABI.
template <class F>
inline int mh_guard(F &&f) noexcept {
    try {
        return f();
    } catch (const std::bad_alloc &) {
        return MH_ERR_OUT_OF_MEMORY;
    } catch (...) {
        return MH_ERR_ILLEGAL_STATE;
    }
}

#define MH_HIP(expr)                                        \
    do {                                                    \
        hipError_t e_ = (expr);                             \
        if (e_ != hipSuccess) return -(int)e_;              \
    } while (0)

// Test-only fault sites (mh_debug_fail_at, include/immustore_merkle.h):
// true exactly once, when the armed countdown of `site` reaches zero.
bool mh_fault(int site);

// CSR offsets off[0..n] never run backwards (checked before a host wrapper
// rebases them and sizes the device copies from off[n] - off[0])
inline bool monotonic(const uint64_t *off, uint64_t n) {
    for (uint64_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) return false;
    return true;
}

static const uint8_t kEmptyRoot[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14,
                                       0x9a, 0xfb, 0xf4, 0xc8, 0x99, 0x6f, 0xb9, 0x24,
                                       0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c,
                                       0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

// ------------------------------------------------------------------ timing
struct EventTimer : Timer {
    struct Rec {
        std::string name;
        hipEvent_t a, b;
    };
    std::mutex mu;
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    bool enabled = false;
    hipEvent_t take() {
        hipEvent_t e;
        if (!pool.empty()) {
            e = pool.back();
            pool.pop_back();
        } else {
            hipEventCreate(&e);
        }
        return e;
    }
    // launches from several threads may interleave: end() closes the record
    // its own thread opened last (a stack per thread, so scopes may nest)
    std::unordered_map<std::thread::id, std::vector<size_t>> open;
    void begin(const char *name, hipStream_t st) override {
        std::lock_guard<std::mutex> g(mu);
        Rec r;
        r.name = name;
        r.a = take();
        r.b = take();
        hipEventRecord(r.a, st);
        open[std::this_thread::get_id()].push_back(recs.size());
        recs.push_back(r);
    }
    void end(hipStream_t st) override {
        std::lock_guard<std::mutex> g(mu);
        auto it = open.find(std::this_thread::get_id());
        if (it == open.end() || it->second.empty()) return;
        hipEventRecord(recs[it->second.back()].b, st);
        it->second.pop_back();
    }
    int sum(const char *prefix, double *ms, uint64_t *cnt) {
        std::lock_guard<std::mutex> g(mu);
        double tot = 0;
        uint64_t c = 0;
        size_t pl = prefix ? strlen(prefix) : 0;
        for (auto &r : recs) {
            if (pl && r.name.compare(0, pl, prefix) != 0) continue;
            hipError_t e = hipEventSynchronize(r.b);
            if (e != hipSuccess) return -(int)e;
            float x = 0;
            hipEventElapsedTime(&x, r.a, r.b);
            tot += x;
            c++;
        }
        if (ms) *ms = tot;
        if (cnt) *cnt = c;
        return MH_OK;
    }
    void reset() {
        std::lock_guard<std::mutex> g(mu);
        for (auto &r : recs) {
            hipEventSynchronize(r.b);
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        recs.clear();
        open.clear();
    }
    ~EventTimer() {
        for (auto &r : recs) {
            hipEventDestroy(r.a);
            hipEventDestroy(r.b);
        }
        for (auto e : pool) hipEventDestroy(e);
    }
};

// ------------------------------------------------------------------ buffers
struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        uint64_t c = std::max<uint64_t>(bytes + 64, 256);
        hipError_t e = hipMalloc(&p, c);
        if (e == hipSuccess) cap = c;
        return e;
    }
    template <class T>
    T *as() const {
        return reinterpret_cast<T *>(p);
    }
    ~DevBuf() {
        if (p) hipFree(p);
    }
};

// Pinned host staging (hipHostMalloc), grown on demand.
struct PinBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        const uint64_t c = std::max<uint64_t>(bytes + 64, 4096);
        hipError_t e = hipHostMalloc(&p, c, hipHostMallocDefault);
        if (e == hipSuccess) cap = c;
        return e;
    }
    template <class T>
    T *as() const {
        return reinterpret_cast<T *>(p);
    }
    ~PinBuf() {
        if (p) hipHostFree(p);
    }
};

struct mh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    EventTimer timer;
    std::mutex mu;  // guards scratch for mh_dev_* calls
    DevBuf s_hvals, s_msgoff, s_msgs, s_digests, s_idx, s_offs, s_ctr;
    DevBuf s_edge;        // ahtree frontier of a ranged append (64 x 32 B)
    DevBuf s_sort;        // length-class sort of ragged messages (varlen_kernels.hip)
    DevBuf s_tx, s_tree;  // tx layer (capi_tx.hip)
    DevBuf s_txlog;       // raw tx-log bytes of mh_txlog_validate
    DevBuf s_txpatch;     // the same + canonical metadata records (rare)
    DevBuf s_clog;        // mh_txlog_validate_clog's per-record arrays
    uint64_t clog_wmax = 0;  // the widest record of its last resident call (the next launch's guess)
    PinBuf p_tx;          // its pinned staging of the parsed index arrays
    // mh_txlog_validate's groups (one per copy chunk): device arrays and
    // pinned index staging of each, kept across calls
    std::deque<DevBuf> s_txg;
    std::deque<PinBuf> p_txg;
    PinBuf p_stage;       // host-built arrays of one call, staged for a single upload
    PinBuf p_small;       // a few words a kernel stores straight into host memory
    // second stream for host->device copies that overlap the compute stream
    // (chunked pipelines), its events, and the double-buffered chunk slots
    hipStream_t copy_stream = nullptr;
    hipStream_t copy_stream2 = nullptr;  // a second copy lane (ChunkCopier)
    hipStream_t d2h_stream = nullptr;  // device->host results of an early part of a call
    hipStream_t stream2 = nullptr;     // a second compute stream (tx-log groups)
    hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
    DevBuf s_chunk[2];
    std::vector<hipEvent_t> ev_chunks;  // one per chunk of a pipelined call (arrivals)
    std::vector<hipEvent_t> ev_results; // one per group: its results are complete
    Timer *tm() { return timer.enabled ? &timer : nullptr; }
    // creates copy_stream and the events on first use (c->mu held)
    hipError_t copy_lane() {
        if (copy_stream) return hipSuccess;
        hipError_t e = hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&copy_stream2, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&d2h_stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking);
        for (int k = 0; k < 2 && e == hipSuccess; k++) {
            e = hipEventCreateWithFlags(&ev_copied[k], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming);
        }
        return e;
    }
    ~mh_ctx() {
        for (int k = 0; k < 2; k++) {
            if (ev_copied[k]) hipEventDestroy(ev_copied[k]);
            if (ev_done[k]) hipEventDestroy(ev_done[k]);
        }
        for (hipEvent_t e : ev_chunks) hipEventDestroy(e);
        for (hipEvent_t e : ev_results) hipEventDestroy(e);
        if (copy_stream) hipStreamDestroy(copy_stream);
        if (copy_stream2) hipStreamDestroy(copy_stream2);
        if (d2h_stream) hipStreamDestroy(d2h_stream);
        if (stream2) hipStreamDestroy(stream2);
    }
};

// ---- the tx-log record hop (capi_tx.hip), shared with the multi-device call
// Records of one stretch of a tx log (the structure readHeader / readEntry
// read, tx.go:419-603; no hashing).
// Per record: where it starts, where its stored Alh is, its entry count and
// the bytes of its entry-digest messages.  The headers themselves are only
// kept when asked (mh_txlog_scan); the validation path rebuilds them on the
// device from the raw record bytes (k_tx_hdr_from_raw).
struct HopRec {
    uint64_t rec, alh;
    uint32_t nent, pad;
};

// A record whose metadata is valid but not in the canonical form Go hashes
// (the reader re-serialises parsed metadata: KVMetadata.Bytes() in the entry
// digest, TxMetadata.Bytes() in the inner hash): the canonical bytes the
// device hashes instead.  kind 0: entry `entry` of the record, bytes = the
// whole entry record with canonical KV metadata; kind 1: the tx metadata.
struct HopPatch {
    uint64_t rec;  // index into HopOut::R
    uint32_t kind, entry;
    std::vector<uint8_t> bytes;
};

struct HopOut {
    std::vector<HopRec> R;
    std::vector<HopPatch> P;
    std::vector<mh_tx_header> H;  // want_headers only
    bool want_headers = false;
    uint64_t start = 0, end = 0;  // first record parsed / where parsing stopped
    int rc = MH_OK;
    bool stopped = false;  // EOF (id 0 / end of buffer) or a structural error
};

struct HopLimits {
    uint32_t max_entries, max_key_len;
};

// The whole hop of a run of records (no headers kept), as mh_txlog_validate
// runs it: out.R, out.P, out.rc (the structural status), out.end (consumed).
void txlog_hop(const uint8_t *buf, uint64_t len, uint32_t max_entries, uint32_t max_key_len,
               uint64_t max_txs, HopOut &out);
// mh_txlog_validate with the record structure parsed already (pre: every
// record of [buf, buf + len) with offsets relative to buf, patches indexed by
// record, rc MH_OK, end == len): no host hop in the call.
int txlog_validate_parsed(mh_ctx *c, const uint8_t *buf, uint64_t len, uint32_t max_entries,
                          uint32_t max_key_len, const HopOut &pre, mh_tx_header *hdrs_out,
                          uint8_t *alh_out, int32_t *status_out);

// Host-to-device copies of a call cut into chunks, issued from one helper
// thread (or two, chunk k on lane k % 2) onto the context's copy stream(s)
// with an event after each chunk.  A copy call from pinned memory holds its
// caller until the transfer is done, so every chunk boundary leaves the DMA
// engine idle for the next call's setup (60-100 us measured,
// profiles/txlog_copy_trace_r03.txt): few, large chunks.  The consumer
// waits for chunk k (wait(k): the copy and its event are enqueued) and then
// orders its stream after event ev(k).  c->mu must be held; both lanes start
// after everything queued on c->stream before start().
struct ChunkCopier {
    struct Piece {
        void *dst;
        const void *src;
        uint64_t bytes;
    };
    mh_ctx *c = nullptr;
    std::vector<std::vector<Piece>> chunks;
    std::mutex m;
    std::condition_variable cv;
    std::vector<uint8_t> done;  // chunk k enqueued (guarded by m)
    hipError_t err = hipSuccess;
    std::thread th[2];
    int lanes = 1;  // 1: one helper thread / copy stream; 2: two
    bool inline_issue = false;  // issue every copy from the caller (pinned sources: no blocking)

    bool started = false, synced = false;
    explicit ChunkCopier(mh_ctx *ctx) : c(ctx) {}
    // every copy is complete: none reads the caller's host memory any more
    // (the second lane's stream holds copies only with lanes == 2)
    hipError_t sync() {
        if (hipError_t e = join()) return e;
        if (started) {
            if (hipError_t e = hipStreamSynchronize(c->copy_stream)) return e;
            if (lanes == 2)
                if (hipError_t e = hipStreamSynchronize(c->copy_stream2)) return e;
        }
        synced = true;
        return hipSuccess;
    }
    // on every way out of the call: no copy may still read the caller's
    // host memory once it returns (an error path skips the final sync)
    ~ChunkCopier() {
        join();
        if (started && !synced) {
            hipStreamSynchronize(c->copy_stream);
            hipStreamSynchronize(c->copy_stream2);
        }
    }
    // chunks must be filled; events for every chunk must exist in c->ev_chunks
    hipError_t start() {
        done.assign(chunks.size(), 0);
        started = true;
        const bool idle = hipStreamQuery(c->stream) == hipSuccess;
        (void)hipGetLastError();  // hipErrorNotReady is not an error here
        // the copies overwrite device buffers that work queued earlier on the
        // context's stream may still read: the copy streams wait for it, unless
        // that stream is idle already (a cross-queue wait ahead of the first
        // copy delays its start: -20..-50 us per a14 call,
        // profiles/ab_txlog_wait0_flags_r04.txt; and the event itself is then
        // not recorded: ~3 us of host time ahead of the first copy)
        if (!idle) {
            if (hipError_t e = hipEventRecord(c->ev_done[0], c->stream)) return e;
            if (hipError_t e = hipStreamWaitEvent(c->copy_stream, c->ev_done[0], 0)) return e;
            if (hipError_t e = hipStreamWaitEvent(c->copy_stream2, c->ev_done[0], 0)) return e;
        }
        for (int j = 0; j < lanes; j++) {
            auto lane = [this, j]() {
                hipError_t e = hipSetDevice(c->device);
                hipStream_t s = j ? c->copy_stream2 : c->copy_stream;
                for (size_t k = (size_t)j; k < chunks.size(); k += (size_t)lanes) {
                    for (const Piece &p : chunks[k])
                        if (!e && p.bytes) e = hipMemcpyAsync(p.dst, p.src, p.bytes, hipMemcpyHostToDevice, s);
                    if (!e) e = hipEventRecord(c->ev_chunks[k], s);
                    std::lock_guard<std::mutex> g(m);
                    if (e) {
                        err = e;
                        cv.notify_all();
                        return;
                    }
                    done[k] = 1;
                    cv.notify_all();
                }
            };
            if (chunks.size() <= 1 || inline_issue) {  // no thread worth starting
                lane();
                continue;
            }
            try {
                th[j] = std::thread(lane);
            } catch (...) {
                lane();  // no thread: issue this lane's copies here
            }
        }
        return hipSuccess;
    }
    // chunk k's copies and event are enqueued (or an error happened)
    hipError_t wait(size_t k) {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return done[k] || err != hipSuccess; });
        return err;
    }
    // stream st waits until chunk k has landed (after wait(k) succeeded: its
    // copies and event are enqueued).  Events, not stream-written words:
    // ROCclr runs hipStreamWriteValue32 / WaitValue32 as blit kernels, no
    // faster (profiles/ab_txlog_wait0_flags_r04.txt)
    hipError_t stream_wait(hipStream_t st, size_t k) { return hipStreamWaitEvent(st, c->ev_chunks[k], 0); }
    // chunk k's copies and event are enqueued already (no waiting)
    bool issued(size_t k) {
        std::lock_guard<std::mutex> g(m);
        return done[k] || err != hipSuccess;
    }
    hipError_t join() {
        for (auto &t : th)
            if (t.joinable()) t.join();
        return err;
    }
};

// [a, b] (b >= a) lies inside ONE pinned host allocation: the allocation's
// address range as the runtime reports it for a (HIP_POINTER_ATTRIBUTE_
// RANGE_START_ADDR / _RANGE_SIZE, in the host or the device view of the
// allocation) must hold both ends.  Two separate hipHostMalloc blocks are not
// one allocation even when their device addresses are as far apart as their
// host addresses (on ROCm they usually are: same virtual address), and a copy
// of a span crossing them could read a gap.  Any query that
// fails means "no", i.e. one copy per array.
inline bool pinned_same_alloc(const void *a, const void *b) {
    hipPointerAttribute_t x;
    void *start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttributes(&x, a) != hipSuccess || x.type != hipMemoryTypeHost ||
        hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)a) !=
            hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)a) !=
            hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const uintptr_t s = (uintptr_t)start, ua = (uintptr_t)a, ub = (uintptr_t)b,
                    ud = (uintptr_t)x.devicePointer;
    if (ub < ua || !size) return false;
    uintptr_t off;
    if (ua >= s && ua - s < size)
        off = ua - s;
    else if (ud && ud >= s && ud - s < size)
        off = ud - s;
    else
        return false;
    return ub - ua < size - off;
}

// events for n chunks in c->ev_chunks
// Without the system-scope fence: every waiter on these events is a device
// stream (the host waits on streams), and the fence held each chunk's
// consumer ~4 us longer (-12..-19 us per a14 call in three interleaved
// rounds, profiles/ab_txlog_evfence_r04.txt).
inline hipError_t ensure_chunk_events(mh_ctx *c, size_t n) {
    const unsigned flags = hipEventDisableTiming | hipEventDisableSystemFence;
    while (c->ev_chunks.size() < n) {
        hipEvent_t e;
        if (hipError_t r = hipEventCreateWithFlags(&e, flags)) return r;
        c->ev_chunks.push_back(e);
    }
    return hipSuccess;
}

// events for the results of n groups in c->ev_results: default flags, i.e.
// WITH the system-scope release -- the copies that wait on them may read the
// results through a DMA engine rather than a kernel
inline hipError_t ensure_result_events(mh_ctx *c, size_t n) {
    while (c->ev_results.size() < n) {
        hipEvent_t e;
        if (hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming)) return r;
        c->ev_results.push_back(e);
    }
    return hipSuccess;
}

struct mh_htree {
    mh_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    uint64_t max_width = 0;
    uint64_t width = 0;
    uint8_t root[32];
    DevBuf levels, in_a, in_b, in_c, off_a, off_b, off_c, ov, use, hv, msgoff, msgs, digests;
    DevBuf sort;  // length-class sort of ragged messages
    DevBuf w_in, w_out;  // wire formats (capi_wire.hip)
    void *pinned = nullptr;
    uint64_t pinned_cap = 0;
    LevelGeom geom;
};

struct mh_ahtree {
    mh_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    uint64_t size = 0;
    // every mh_ahtree_* call holds this for its whole duration, like the Go
    // AHtree's t.mutex (ahtree.go:60-84): readers (Root, proofs, dLog reads)
    // may run concurrently with a committer's Append, which can reallocate
    // the dLog.  Recursive: Append / Root call other locked entry points.
    std::recursive_mutex mu;
    DevBuf dlog, in, roots, idx, out, ctr;
    DevBuf w_in, w_out;  // wire formats (capi_wire.hip)
};

// Header preconditions shared by every entry point that reads headers.
inline int check_header(const mh_tx_header &h, uint64_t md_blob_len, bool have_blob) {
    if (h.version > 1) return MH_ERR_ILLEGAL_ARGUMENTS;
    if (h.md_len) {
        if (h.version == 0) return MH_ERR_METADATA_UNSUPPORTED;
        if (h.md_len > MH_MAX_TX_METADATA_LEN || !have_blob) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((uint64_t)h.md_off + h.md_len > md_blob_len) return MH_ERR_ILLEGAL_ARGUMENTS;
    }
    return MH_OK;
}

// ---------------------------------------------------------------- tx layer helpers
// Sub-allocations of one device scratch buffer (256-byte aligned).
struct Layout {
    uint64_t total = 0;
    uint64_t add(uint64_t bytes) {
        const uint64_t o = total;
        total = (total + bytes + 255) & ~255ull;
        return o;
    }
};

// ---------------------------------------------------------------- many trees
// Level plan of a batch of htrees (htree.go:85-110 per tree): level 0 are the
// leaves of all trees back to back, every further level appends the nodes of
// the trees that still have more than one node.
struct TreePlan {
    std::vector<uint64_t> cur, prev, prevw;  // items, grouped by level
    struct Level {
        uint64_t base, nodes, item0, nitems;
    };
    std::vector<Level> levels;
    std::vector<uint64_t> root_idx;  // per tree: node index of the root, ~0 = empty tree
    uint64_t total_nodes = 0;

    void build(uint64_t ntrees, const uint64_t *leaf_off) {
        const uint64_t o0 = leaf_off[0];
        root_idx.assign(ntrees, ~0ull);
        struct Act {
            uint64_t t, base, w;
        };
        std::vector<Act> act, nxt;
        for (uint64_t t = 0; t < ntrees; t++) {
            const uint64_t w = leaf_off[t + 1] - leaf_off[t];
            if (w == 1) root_idx[t] = leaf_off[t] - o0;
            if (w > 1) act.push_back({t, leaf_off[t] - o0, w});
        }
        uint64_t next = leaf_off[ntrees] - o0;
        while (!act.empty()) {
            Level L{next, 0, cur.size(), act.size()};
            nxt.clear();
            for (const Act &a : act) {
                const uint64_t cw = (a.w + 1) / 2;
                cur.push_back(next);
                prev.push_back(a.base);
                prevw.push_back(a.w);
                if (cw == 1)
                    root_idx[a.t] = next;
                else
                    nxt.push_back({a.t, next, cw});
                next += cw;
                L.nodes += cw;
            }
            levels.push_back(L);
            act.swap(nxt);
        }
        total_nodes = next;
    }
};

// bytes of pinned staging run_tree_plan_on needs for plan P over ntrees trees
inline uint64_t plan_index_bytes(const TreePlan &P, uint64_t ntrees) {
    return (3 * P.cur.size() + ntrees) * 8;
}

// Leaves + levels + roots of a planned batch (capi_tx.hip).
// roots of many htrees over device digests (capi_tx.hip)
// innerHash / Alh of checked headers (capi_tx.hip); c->mu held by the caller.
int tx_alh_core(mh_ctx *c, uint64_t n, const mh_tx_header *hdrs, const uint8_t *md_blob,
                uint64_t md_blob_len, uint8_t *inner_out, uint8_t *alh_out);
// VerifyDualProofV2 over checked arguments (capi_tx.hip); alh_checked skips
// the header Alh pass when the caller has matched them already; c->mu held.
int dual_proof_v2_core(mh_ctx *c, uint64_t n, const mh_tx_header *sh, const mh_tx_header *th,
                       const uint8_t *md_blob, uint64_t md_blob_len, const uint64_t *incl_off,
                       const uint8_t *incl_terms, const uint64_t *cons_off,
                       const uint8_t *cons_terms, const uint64_t *src, const uint64_t *tgt,
                       const uint8_t *src_alh, const uint8_t *tgt_alh, int32_t *status,
                       bool alh_checked);
int build_many_dev(mh_ctx *c, hipStream_t st, uint64_t ntrees, const uint64_t *leaf_off,
                   const uint8_t *d_dig, uint8_t *d_roots, DevBuf &s_lv, DevBuf &s_lo);
int run_tree_plan(mh_ctx *c, hipStream_t st, const TreePlan &P, uint64_t ntrees, uint64_t nleaves,
                  const uint8_t *d_digests, uint8_t *d_roots);
int run_tree_plan_on(DevBuf &scratch, hipStream_t st, Timer *tm, const TreePlan &P, uint64_t ntrees,
                     uint64_t nleaves, const uint8_t *d_digests, uint8_t *d_roots, uint8_t *pinned);
