// capi_internal.hpp -- host-side objects shared by the C-ABI translation
// units (capi.hip: htree / ahtree handles; capi_tx.hip: tx layer).
#pragma once
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "mh_internal.hpp"

using namespace mh;

#define MH_HIP(expr)                                        \
    do {                                                    \
        hipError_t e_ = (expr);                             \
        if (e_ != hipSuccess) return -(int)e_;              \
    } while (0)

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
    void begin(const char *name, hipStream_t st) override {
        std::lock_guard<std::mutex> g(mu);
        Rec r;
        r.name = name;
        r.a = take();
        r.b = take();
        hipEventRecord(r.a, st);
        recs.push_back(r);
    }
    void end(hipStream_t st) override {
        std::lock_guard<std::mutex> g(mu);
        hipEventRecord(recs.back().b, st);
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

struct mh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    EventTimer timer;
    std::mutex mu;  // guards scratch for mh_dev_* calls
    DevBuf s_hvals, s_msgoff, s_msgs, s_digests, s_idx, s_offs, s_ctr;
    DevBuf s_tx, s_tree;  // tx layer (capi_tx.hip)
    Timer *tm() { return timer.enabled ? &timer : nullptr; }
};

struct mh_htree {
    mh_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    uint64_t max_width = 0;
    uint64_t width = 0;
    uint8_t root[32];
    DevBuf levels, in_a, in_b, in_c, off_a, off_b, off_c, ov, use, hv, msgoff, msgs, digests;
    void *pinned = nullptr;
    uint64_t pinned_cap = 0;
    LevelGeom geom;
};

struct mh_ahtree {
    mh_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    uint64_t size = 0;
    DevBuf dlog, in, roots, idx, out, ctr;
};

