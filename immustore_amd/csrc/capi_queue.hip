// capi_queue.hip -- group commit for the single-transaction precommit path.
//
// In the reference every committer hashes its own transaction before taking
// the store lock: precommit's value-hash loop and Tx.BuildHashTree
// (immustore.go:1620-1632, the lock is taken at :1689), from up to
// MaxConcurrency = 30 goroutines at once (options.go:35).  One transaction of
// a few entries is far too little work for a GPU launch sequence, so the
// library coalesces them: every committer submits its one transaction and
// blocks; a worker thread gathers what arrives within a short window (or a
// full batch), packs it into one pinned arena, runs one mh_precommit_batch
// over the commit pipe (value hashes, entry digests, one htree per tx -- all
// on the device) and hands each committer its own hVals, Eh and status.
// Two workers, each with its own pipe (HIP streams) and arenas, take turns:
// while one batch is packed, hashed and scattered, the other worker gathers
// the next one, so the host work of one batch runs under the device work of
// the other (MH_QUEUE_WORKERS = 1..8 overrides the count).
//
// Lock order: q->mu is never held while the device works.
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <memory>

#include "capi_internal.hpp"

struct mh_commit_queue {
    mh_ctx *ctx = nullptr;
    int version = 1;
    uint64_t max_width = 0;
    uint32_t max_txs = 64;
    uint32_t wait_us = 50;

    struct Req {
        uint64_t n;
        const uint8_t *keys, *md, *vals, *ov, *use, *expect;
        const uint64_t *key_off, *md_off, *val_off;
        uint8_t *hvals_out, *eh_out;
        int32_t status = MH_OK;
        bool done = false;
    };
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::deque<Req *> pending;
    bool stop = false;
    uint32_t submitters = 0;  // inside mh_commit_queue_submit (free waits for 0)
    bool gathering = false;  // one worker at a time collects the next batch
    struct Worker {
        mh_commit_pipe *pipe = nullptr;
        PinBuf in, out;  // packing arenas (pinned: the pipe's copies are then DMA)
        std::thread th;
    };
    std::vector<std::unique_ptr<Worker>> workers;
    // counters (mh_commit_queue_stats)
    uint64_t batches = 0, txs = 0;
};

namespace {

// One batch: pack, hash on the device, scatter.
int run_batch(mh_commit_queue *q, mh_commit_queue::Worker &W,
              std::vector<mh_commit_queue::Req *> &B) {
    const uint64_t nt = B.size();
    uint64_t ne = 0, kb = 0, mb = 0, vb = 0;
    bool any_md = false, any_ov = false;
    for (auto *r : B) {
        ne += r->n;
        if (r->n) {
            kb += r->key_off[r->n] - r->key_off[0];
            vb += r->val_off[r->n] - r->val_off[0];
            if (r->md_off) mb += r->md_off[r->n] - r->md_off[0];
        }
        any_md |= r->md_off != nullptr;
        any_ov |= r->use != nullptr;
    }
    Layout L;
    const uint64_t b_tx = L.add((nt + 1) * 8), b_ko = L.add((ne + 1) * 8),
                   b_mo = L.add(any_md ? (ne + 1) * 8 : 0), b_vo = L.add((ne + 1) * 8),
                   b_k = L.add(kb), b_m = L.add(mb), b_v = L.add(vb),
                   b_ov = L.add(any_ov ? ne * 32 : 0), b_use = L.add(any_ov ? ne : 0);
    Layout O;
    const uint64_t o_hv = O.add(ne * 32), o_eh = O.add(nt * 32), o_st = O.add(nt * 4);
    MH_HIP(W.in.ensure(L.total));
    MH_HIP(W.out.ensure(O.total));
    uint8_t *in = W.in.as<uint8_t>(), *out = W.out.as<uint8_t>();
    uint64_t *tx_off = (uint64_t *)(in + b_tx), *ko = (uint64_t *)(in + b_ko),
             *mo = any_md ? (uint64_t *)(in + b_mo) : nullptr, *vo = (uint64_t *)(in + b_vo);
    uint64_t e = 0, kp = 0, mp = 0, vp = 0;
    tx_off[0] = 0;
    ko[0] = mo ? (mo[0] = 0) : 0;
    vo[0] = 0;
    for (uint64_t t = 0; t < nt; t++) {
        const mh_commit_queue::Req *r = B[t];
        for (uint64_t i = 0; i < r->n; i++, e++) {
            const uint64_t kl = r->key_off[i + 1] - r->key_off[i];
            const uint64_t vl = r->val_off[i + 1] - r->val_off[i];
            if (kl) memcpy(in + b_k + kp, r->keys + r->key_off[i], kl);
            if (vl) memcpy(in + b_v + vp, r->vals + r->val_off[i], vl);
            kp += kl;
            vp += vl;
            ko[e + 1] = kp;
            vo[e + 1] = vp;
            if (mo) {
                const uint64_t ml = r->md_off ? r->md_off[i + 1] - r->md_off[i] : 0;
                if (ml) memcpy(in + b_m + mp, r->md + r->md_off[i], ml);
                mp += ml;
                mo[e + 1] = mp;
            }
            if (any_ov) {
                const bool u = r->use && r->use[i];
                in[b_use + e] = u ? 1 : 0;
                if (u) memcpy(in + b_ov + e * 32, r->ov + i * 32, 32);
            }
        }
        tx_off[t + 1] = e;
    }
    int32_t *st = (int32_t *)(out + o_st);
    int rc = mh_precommit_batch(W.pipe, q->version, q->max_width, nt, tx_off, in + b_k, ko,
                                any_md ? in + b_m : nullptr, mo, in + b_v, vo,
                                any_ov ? in + b_ov : nullptr, any_ov ? in + b_use : nullptr,
                                nullptr, out + o_hv, out + o_eh, st);
    if (rc != MH_OK) return rc;
    e = 0;
    for (uint64_t t = 0; t < nt; t++) {
        mh_commit_queue::Req *r = B[t];
        int32_t s = st[t];
        const uint8_t *eh = out + o_eh + t * 32;
        // ReplicateTx's check, immustore.go:1649-1654
        if (s == MH_OK && r->expect && memcmp(r->expect, eh, 32)) s = MH_ERR_ILLEGAL_ARGUMENTS;
        if (r->hvals_out && r->n) memcpy(r->hvals_out, out + o_hv + e * 32, r->n * 32);
        if (r->eh_out) memcpy(r->eh_out, eh, 32);
        r->status = s;
        e += r->n;
    }
    return MH_OK;
}

void worker_loop(mh_commit_queue *q, mh_commit_queue::Worker *W) {
    hipSetDevice(q->ctx->device);
    std::vector<mh_commit_queue::Req *> B;
    for (;;) {
        std::unique_lock<std::mutex> lk(q->mu);
        q->cv_work.wait(lk, [&] { return q->stop || (!q->gathering && !q->pending.empty()); });
        if (q->pending.empty()) {
            if (q->stop) break;  // stop requested, nothing left
            continue;
        }
        // gather: until the window closes or a full batch is waiting
        q->gathering = true;
        const auto deadline =
            std::chrono::steady_clock::now() + std::chrono::microseconds(q->wait_us);
        while (!q->stop && q->pending.size() < q->max_txs) {
            if (q->cv_work.wait_until(lk, deadline) == std::cv_status::timeout) break;
        }
        B.clear();
        while (!q->pending.empty() && B.size() < q->max_txs) {
            B.push_back(q->pending.front());
            q->pending.pop_front();
        }
        q->gathering = false;
        lk.unlock();
        q->cv_work.notify_all();  // another worker may gather the next batch now
        int rc = MH_ERR_ILLEGAL_STATE;
        try {
            rc = run_batch(q, *W, B);
        } catch (const std::bad_alloc &) {
            rc = MH_ERR_OUT_OF_MEMORY;
        } catch (...) {
            rc = MH_ERR_ILLEGAL_STATE;
        }
        lk.lock();
        for (auto *r : B) {
            if (rc != MH_OK) r->status = rc;
            r->done = true;
        }
        q->batches++;
        q->txs += B.size();
        lk.unlock();
        q->cv_done.notify_all();
    }
}

int queue_workers() {
    if (const char *e = getenv("MH_QUEUE_WORKERS")) {
        const int v = atoi(e);
        if (v >= 1 && v <= 8) return v;
    }
    return 2;
}

}  // namespace

extern "C" int mh_commit_queue_new(mh_ctx *c, int version, uint64_t max_width, uint32_t max_txs,
                                   uint32_t wait_us, mh_commit_queue **out) {
    return mh_guard([&]() -> int {
        if (!c || !out || (version != 0 && version != 1)) return MH_ERR_ILLEGAL_ARGUMENTS;
        *out = nullptr;
        MH_HIP(hipSetDevice(c->device));
        mh_commit_queue *q = new mh_commit_queue();
        q->ctx = c;
        q->version = version;
        q->max_width = max_width;
        q->max_txs = max_txs ? max_txs : 64;
        q->wait_us = wait_us;
        const int nw = queue_workers();
        for (int k = 0; k < nw; k++) {
            q->workers.emplace_back(new mh_commit_queue::Worker());
            int st = mh_commit_pipe_new(c, 0, &q->workers.back()->pipe);
            if (st != MH_OK) {
                for (auto &w : q->workers)
                    if (w->pipe) mh_commit_pipe_free(w->pipe);
                delete q;
                return st;
            }
        }
        for (auto &w : q->workers) w->th = std::thread(worker_loop, q, w.get());
        *out = q;
        return MH_OK;
    });
}

extern "C" int mh_commit_queue_free(mh_commit_queue *q) {
    return mh_guard([&]() -> int {
        if (!q) return MH_OK;
        {
            std::lock_guard<std::mutex> lk(q->mu);
            q->stop = true;
        }
        q->cv_work.notify_all();
        for (auto &w : q->workers)
            if (w->th.joinable()) w->th.join();  // the workers drain what is pending first
        {
            // a submitter woken by the last batch still re-takes q->mu on its
            // way out: the queue must outlive every one of them
            std::unique_lock<std::mutex> lk(q->mu);
            q->cv_done.wait(lk, [&] { return q->submitters == 0; });
        }
        for (auto &w : q->workers) mh_commit_pipe_free(w->pipe);
        delete q;
        return MH_OK;
    });
}

extern "C" int mh_commit_queue_submit(mh_commit_queue *q, uint64_t n, const uint8_t *keys,
                                      const uint64_t *key_off, const uint8_t *md,
                                      const uint64_t *md_off, const uint8_t *vals,
                                      const uint64_t *val_off, const uint8_t *hval_override,
                                      const uint8_t *use_override, const uint8_t *expect_eh,
                                      uint8_t *hvals_out, uint8_t *eh_out) {
    return mh_guard([&]() -> int {
        if (!q) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n && (!key_off || !val_off)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((hval_override == nullptr) != (use_override == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((md == nullptr) != (md_off == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        for (uint64_t i = 0; i < n; i++)
            if (key_off[i + 1] < key_off[i] || val_off[i + 1] < val_off[i] ||
                (md_off && md_off[i + 1] < md_off[i]))
                return MH_ERR_ILLEGAL_ARGUMENTS;
        if (n && ((key_off[n] > key_off[0] && !keys) || (val_off[n] > val_off[0] && !vals)))
            return MH_ERR_ILLEGAL_ARGUMENTS;
        mh_commit_queue::Req r;
        r.n = n;
        r.keys = keys;
        r.key_off = key_off;
        r.md = md;
        r.md_off = md_off;
        r.vals = vals;
        r.val_off = val_off;
        r.ov = hval_override;
        r.use = use_override;
        r.expect = expect_eh;
        r.hvals_out = hvals_out;
        r.eh_out = eh_out;
        std::unique_lock<std::mutex> lk(q->mu);
        if (q->stop) return MH_ERR_ILLEGAL_STATE;
        q->pending.push_back(&r);
        q->submitters++;
        // all: the worker gathering a batch must see it, not only an idle one
        q->cv_work.notify_all();
        q->cv_done.wait(lk, [&] { return r.done; });
        const int st = r.status;
        // the last one out wakes a waiting mh_commit_queue_free (notified
        // under the lock: free cannot delete q between this and unlock)
        if (--q->submitters == 0 && q->stop) q->cv_done.notify_all();
        return st;
    });
}

extern "C" int mh_commit_queue_stats(mh_commit_queue *q, uint64_t *batches, uint64_t *txs) {
    return mh_guard([&]() -> int {
        if (!q) return MH_ERR_ILLEGAL_ARGUMENTS;
        std::lock_guard<std::mutex> lk(q->mu);
        if (batches) *batches = q->batches;
        if (txs) *txs = q->txs;
        return MH_OK;
    });
}
