// capi_commit.hip -- the commit path's hashing for many transactions at once
// (SURVEY.md 8(f) row 1): ImmuStore.precommit / preCommitWith compute
// hVal = SHA256(value) for every EntrySpec (or take HashValue when the value
// is truncated, immustore.go:1620-1630 and 2301-2311), then
// Tx.BuildHashTree (tx.go:332-355) gives the header's Eh; a replicated tx's
// Eh is compared with the one it came with (immustore.go:1649-1654).  Up to
// MaxConcurrency commits run that concurrently, and replication / replay feed
// whole batches of transactions; here a batch of transactions is cut into
// chunks of whole transactions: one HIP stream copies chunk k+1 in while a
// second hashes chunk k and copies its hVals / Eh back.
//
// Inputs are host memory; in pinned memory (mh_host_alloc_pinned) the copies
// are DMA at full PCIe rate and asynchronous.  Every SHA-256 runs on the
// device (htree_kernels.hip: k_sha256_csr, k_digest_assemble; tx_kernels.hip:
// the many-tree level kernels); the host only cuts chunks and plans trees.
#include <cstring>
#include <vector>

#include "capi_internal.hpp"

namespace {

// off[0..n] -= off[0] for up to three CSR offset arrays (chunk slices of the
// caller's arrays, copied verbatim).
__global__ void k_rebase3(uint64_t n, uint64_t *__restrict__ a, uint64_t *__restrict__ b,
                          uint64_t *__restrict__ c, uint64_t a0, uint64_t b0, uint64_t c0) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    a[i] -= a0;
    if (b) b[i] -= b0;
    c[i] -= c0;
}

}  // namespace

// Three slots of device / pinned buffers; one copy stream carries every
// chunk's host->device copies back to back (the PCIe link is the bound), one
// compute stream hashes chunk k while chunk k+1 is copied in.  The host
// waits only before reusing a slot (chunk k-3's results).
constexpr int kSlots = 3;

struct mh_commit_pipe {
    mh_ctx *ctx = nullptr;
    uint64_t chunk_bytes = 0;
    hipStream_t copy = nullptr, comp = nullptr;
    struct Slot {
        hipEvent_t in = nullptr, done = nullptr;
        DevBuf arena, tree;
        PinBuf pin;  // tree-plan index arrays + results staging
        bool busy = false;
        uint64_t t0 = 0, t1 = 0, e0 = 0, e1 = 0;
        uint64_t res_off = 0;  // offset of the results in pin
    } slot[kSlots];
};

namespace {

struct Req {
    int version;
    uint64_t max_width;
    const uint64_t *tx_off;
    const uint8_t *keys;
    const uint64_t *key_off;
    const uint8_t *md;
    const uint64_t *md_off;
    const uint8_t *vals;
    const uint64_t *val_off;
    const uint8_t *ov;
    const uint8_t *use;
    const uint8_t *expect_eh;
    uint8_t *hvals_out;
    uint8_t *eh_out;
    int32_t *status;
    bool hv_pinned, eh_pinned;  // outputs in pinned host memory: D2H lands there directly
};

bool is_pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Copy a finished chunk's results out of the slot's pinned staging and set
// the per-tx statuses (hashing errors are decided on the host, the Eh
// comparison needs the device result).
int drain(mh_commit_pipe::Slot &s, const Req &R) {
    if (!s.busy) return MH_OK;
    s.busy = false;
    MH_HIP(hipEventSynchronize(s.done));
    const uint64_t ne = s.e1 - s.e0, nt = s.t1 - s.t0;
    const uint8_t *hv = reinterpret_cast<const uint8_t *>(s.pin.p) + s.res_off;
    const uint8_t *eh = R.eh_pinned ? R.eh_out + s.t0 * 32 : hv + ne * 32;
    if (R.hvals_out && !R.hv_pinned) memcpy(R.hvals_out + (s.e0 - R.tx_off[0]) * 32, hv, ne * 32);
    for (uint64_t k = 0; k < nt; k++) {
        const uint64_t t = s.t0 + k;
        int32_t st = R.status ? R.status[t] : MH_OK;
        if (st == MH_OK && R.expect_eh && memcmp(R.expect_eh + t * 32, eh + k * 32, 32) != 0)
            st = MH_ERR_ILLEGAL_ARGUMENTS;  // "entries hash (Eh) differs" immustore.go:1651
        if (R.status) R.status[t] = st;
        if (R.eh_out) {
            if (st != MH_OK && st != MH_ERR_ILLEGAL_ARGUMENTS)
                memset(R.eh_out + t * 32, 0, 32);
            else if (!R.eh_pinned)
                memcpy(R.eh_out + t * 32, eh + k * 32, 32);
        }
    }
    return MH_OK;
}

// Enqueue the chunk of transactions [t0, t1) on slot s.
int enqueue(mh_commit_pipe *p, mh_commit_pipe::Slot &s, const Req &R, uint64_t t0, uint64_t t1) {
    const uint64_t e0 = R.tx_off[t0], e1 = R.tx_off[t1], n = e1 - e0, nt = t1 - t0;
    const hipStream_t cp = p->copy, st = p->comp;
    Timer *tm = p->ctx->tm();
    const uint64_t k0 = R.key_off[e0], kb = R.key_off[e1] - k0;
    const uint64_t v0 = R.val_off[e0], vb = R.val_off[e1] - v0;
    const uint64_t m0 = R.md_off ? R.md_off[e0] : 0, mb = R.md_off ? R.md_off[e1] - m0 : 0;
    // trees of this chunk (leaf offsets relative to the chunk)
    std::vector<uint64_t> loff(nt + 1);
    uint64_t wmax = 0;
    for (uint64_t k = 0; k <= nt; k++) loff[k] = R.tx_off[t0 + k] - e0;
    for (uint64_t k = 0; k < nt; k++) wmax = std::max(wmax, loff[k + 1] - loff[k]);
    // small trees (every tx of the chunk <= kSmallTreeMax entries): one lane
    // per tree on the device, no host tree plan
    const bool small = small_roots_fit(nt, wmax);
    TreePlan P;
    if (!small) P.build(nt, loff.data());
    Layout L;
    const uint64_t b_k = L.add(kb), b_m = L.add(mb), b_v = L.add(vb);
    const uint64_t b_ko = L.add((n + 1) * 8), b_mo = L.add(R.md_off ? (n + 1) * 8 : 0),
                   b_vo = L.add((n + 1) * 8);
    const uint64_t b_ov = L.add(R.use ? n * 32 : 0), b_use = L.add(R.use ? n : 0);
    const uint64_t b_hv = L.add(n * 32),
                   b_dig = L.add(std::max<uint64_t>(n, 1) * 32), b_eh = L.add(nt * 32),
                   b_lv = L.add(small ? std::max<uint64_t>(n, 1) * 32 : 0),
                   b_lo = L.add(small ? (nt + 1) * 8 : 0),
                   b_sort = L.add(sha_varlen_scratch_bytes(n));
    MH_HIP(s.arena.ensure(L.total));
    const uint64_t idx_bytes = ((small ? (nt + 1) * 8 : plan_index_bytes(P, nt)) + 255) & ~255ull;
    MH_HIP(s.pin.ensure(idx_bytes + n * 32 + nt * 32));
    s.res_off = idx_bytes;
    uint8_t *base = s.arena.as<uint8_t>();
    // ---- host -> device on the copy stream (the caller's slices, verbatim)
    if (kb) MH_HIP(hipMemcpyAsync(base + b_k, R.keys + k0, kb, hipMemcpyHostToDevice, cp));
    if (mb) MH_HIP(hipMemcpyAsync(base + b_m, R.md + m0, mb, hipMemcpyHostToDevice, cp));
    if (vb) MH_HIP(hipMemcpyAsync(base + b_v, R.vals + v0, vb, hipMemcpyHostToDevice, cp));
    if (n) {
        MH_HIP(hipMemcpyAsync(base + b_ko, R.key_off + e0, (n + 1) * 8, hipMemcpyHostToDevice, cp));
        if (R.md_off)
            MH_HIP(hipMemcpyAsync(base + b_mo, R.md_off + e0, (n + 1) * 8, hipMemcpyHostToDevice,
                                  cp));
        MH_HIP(hipMemcpyAsync(base + b_vo, R.val_off + e0, (n + 1) * 8, hipMemcpyHostToDevice, cp));
        if (R.use) {
            MH_HIP(hipMemcpyAsync(base + b_ov, R.ov + e0 * 32, n * 32, hipMemcpyHostToDevice, cp));
            MH_HIP(hipMemcpyAsync(base + b_use, R.use + e0, n, hipMemcpyHostToDevice, cp));
        }
    }
    MH_HIP(hipEventRecord(s.in, cp));
    MH_HIP(hipStreamWaitEvent(st, s.in, 0));
    if (n) {
        uint64_t *ko = (uint64_t *)(base + b_ko), *vo = (uint64_t *)(base + b_vo);
        uint64_t *mo = R.md_off ? (uint64_t *)(base + b_mo) : nullptr;
        hipLaunchKernelGGL(k_rebase3, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, st, n, ko, mo,
                           vo, k0, m0, v0);
        MH_HIP(hipGetLastError());
        // ---- hVal (immustore.go:1624-1629) and entry digests (tx.go:690-731)
        // in one fused launch (varlen_kernels.hip)
        MH_HIP(launch_entries_varlen(st, tm, R.version, n, base + b_k, ko,
                                     R.version == 1 ? base + b_m : nullptr,
                                     R.version == 1 ? mo : nullptr, base + b_v, vo,
                                     R.use ? base + b_ov : nullptr, R.use ? base + b_use : nullptr,
                                     base + b_hv, base + b_dig, false, base + b_sort));
    }
    // ---- one htree per tx (tx.go:347 -> htree.go:68-113), Eh = root
    if (small) {
        memcpy(s.pin.p, loff.data(), (nt + 1) * 8);
        MH_HIP(hipMemcpyAsync(base + b_lo, s.pin.p, (nt + 1) * 8, hipMemcpyHostToDevice, st));
        MH_HIP(launch_leaf_for(st, tm, n, base + b_dig, base + b_lv));  // htree.go:79-83
        MH_HIP(launch_small_roots(st, tm, nt, (const uint64_t *)(base + b_lo), base + b_lv,
                                  base + b_eh, wmax));
    } else if (int e = run_tree_plan_on(s.tree, st, tm, P, nt, n, base + b_dig, base + b_eh,
                                        reinterpret_cast<uint8_t *>(s.pin.p))) {
        return e;
    }
    // ---- device -> the caller's pinned outputs, or pinned staging
    uint8_t *res = reinterpret_cast<uint8_t *>(s.pin.p) + s.res_off;
    uint8_t *hv_dst = R.hv_pinned ? R.hvals_out + (e0 - R.tx_off[0]) * 32 : res;
    uint8_t *eh_dst = R.eh_pinned ? R.eh_out + t0 * 32 : res + n * 32;
    if (n && (R.hvals_out || !R.hv_pinned))
        MH_HIP(hipMemcpyAsync(hv_dst, base + b_hv, n * 32, hipMemcpyDeviceToHost, st));
    MH_HIP(hipMemcpyAsync(eh_dst, base + b_eh, nt * 32, hipMemcpyDeviceToHost, st));
    MH_HIP(hipEventRecord(s.done, st));
    s.busy = true;
    s.t0 = t0;
    s.t1 = t1;
    s.e0 = e0;
    s.e1 = e1;
    return MH_OK;
}

}  // namespace

extern "C" int mh_commit_pipe_new(mh_ctx *c, uint64_t chunk_bytes, mh_commit_pipe **out) {
    return mh_guard([&]() -> int {
        if (!c || !out) return MH_ERR_ILLEGAL_ARGUMENTS;
        *out = nullptr;
        MH_HIP(hipSetDevice(c->device));
        mh_commit_pipe *p = new mh_commit_pipe();
        p->ctx = c;
        p->chunk_bytes = chunk_bytes ? chunk_bytes : (64ull << 20);
        hipError_t e = hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->comp, hipStreamNonBlocking);
        for (auto &s : p->slot) {
            if (e == hipSuccess) e = hipEventCreateWithFlags(&s.in, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        }
        if (e != hipSuccess) {
            mh_commit_pipe_free(p);
            return -(int)e;
        }
        *out = p;
        return MH_OK;
    });
}

extern "C" int mh_commit_pipe_free(mh_commit_pipe *p) {
    return mh_guard([&]() -> int {
        if (!p) return MH_OK;
        hipSetDevice(p->ctx->device);
        if (p->copy) hipStreamSynchronize(p->copy);
        if (p->comp) hipStreamSynchronize(p->comp);
        for (auto &s : p->slot) {
            if (s.in) hipEventDestroy(s.in);
            if (s.done) hipEventDestroy(s.done);
        }
        if (p->copy) hipStreamDestroy(p->copy);
        if (p->comp) hipStreamDestroy(p->comp);
        delete p;
        return MH_OK;
    });
}

extern "C" int mh_precommit_batch(mh_commit_pipe *p, int version, uint64_t max_width,
                                  uint64_t ntx, const uint64_t *tx_off, const uint8_t *keys,
                                  const uint64_t *key_off, const uint8_t *md,
                                  const uint64_t *md_off, const uint8_t *vals,
                                  const uint64_t *val_off, const uint8_t *hval_override,
                                  const uint8_t *use_override, const uint8_t *expect_eh,
                                  uint8_t *hvals_out, uint8_t *eh_out, int32_t *status) {
    return mh_guard([&]() -> int {
        if (!p || (version != 0 && version != 1)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if (ntx == 0) return MH_OK;
        if (!tx_off || !key_off || !val_off || !status) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((hval_override == nullptr) != (use_override == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        if ((md == nullptr) != (md_off == nullptr)) return MH_ERR_ILLEGAL_ARGUMENTS;
        for (uint64_t t = 0; t < ntx; t++)
            if (tx_off[t + 1] < tx_off[t]) return MH_ERR_ILLEGAL_ARGUMENTS;
        // per-tx errors decided on the host (the Go call would return them):
        // htree.ErrMaxWidthExceeded (htree.go:69-71), ErrMetadataUnsupported for
        // KV metadata under a v0 header (tx.go:691-693)
        for (uint64_t t = 0; t < ntx; t++) {
            int32_t st = MH_OK;
            if (max_width && tx_off[t + 1] - tx_off[t] > max_width) st = MH_ERR_MAX_WIDTH_EXCEEDED;
            if (st == MH_OK && version == 0 && md_off && md_off[tx_off[t + 1]] > md_off[tx_off[t]])
                st = MH_ERR_METADATA_UNSUPPORTED;
            status[t] = st;
        }
        MH_HIP(hipSetDevice(p->ctx->device));
        Req R{version, max_width, tx_off, keys, key_off, md, md_off, vals, val_off, hval_override,
              use_override, expect_eh, hvals_out, eh_out, status, is_pinned(hvals_out),
              is_pinned(eh_out)};
        // chunks of whole transactions, ~chunk_bytes of keys + values (and at
        // most 2^22 entries) each, round robin over the slots; each chunk's
        // offsets are checked just before it is enqueued, under the GPU work of
        // the chunks before it
        constexpr uint64_t kMaxChunkEntries = 1ull << 22;
        uint64_t t = 0;
        int k = 0, rc = MH_OK;
        while (t < ntx) {
            uint64_t t1 = t + 1;
            while (t1 < ntx) {
                const uint64_t e0 = tx_off[t], e1 = tx_off[t1 + 1];
                if (val_off[e1] - val_off[e0] + (key_off[e1] - key_off[e0]) > p->chunk_bytes) break;
                if (e1 - e0 > kMaxChunkEntries) break;
                t1++;
            }
            bool ok = true;
            for (uint64_t e = tx_off[t]; e < tx_off[t1] && ok; e++) {
                ok = key_off[e + 1] >= key_off[e] && val_off[e + 1] >= val_off[e] &&
                     (!md_off || md_off[e + 1] >= md_off[e]);
            }
            if (ok && tx_off[t1] > tx_off[t]) {
                const uint64_t e0 = tx_off[t], e1 = tx_off[t1];
                ok = !((key_off[e1] > key_off[e0] && !keys) || (val_off[e1] > val_off[e0] && !vals) ||
                       (md_off && md_off[e1] > md_off[e0] && !md));
            }
            if (!ok) {
                rc = MH_ERR_ILLEGAL_ARGUMENTS;
                break;
            }
            mh_commit_pipe::Slot &s = p->slot[k % kSlots];
            if ((rc = drain(s, R))) break;
            if ((rc = enqueue(p, s, R, t, t1))) break;
            t = t1;
            k++;
        }
        // drain every slot in chunk order (also after an error: nothing is left
        // in flight)
        for (int j = 0; j < kSlots; j++) {
            int e = drain(p->slot[(k + j) % kSlots], R);
            if (!rc) rc = e;
        }
        return rc;
    });
}
