"""Concurrent use of one mh_ctx from many threads (SURVEY.md 8(b) threading:
up to MaxConcurrency = 30 goroutines run BuildHashTree on different trees at
once, immustore.go:1632; one handle per goroutine, a context shared).

Every thread owns an mh_htree and an mh_ahtree on the shared context and
loops build / proofs / appends; one more thread queues asynchronous mh_dev_*
builds on the context's stream (sharing its scratch with the host-pointer
proof batches and verifications of the others).  Per-kernel timing is on, so
the event records of interleaved launches are exercised too.  Every result
must equal the oracle's (ctypes releases the GIL, so the calls overlap)."""
import ctypes as C
import threading

import numpy as np
import pytest

import oracle as O

THREADS = 8
ROUNDS = 12


def _case(seed):
    rng = np.random.default_rng(seed)
    w = int(rng.integers(1, 3000))
    d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
    lv, root = O.htree_build(d)
    leaves = rng.integers(0, w, 16).astype(np.uint64)
    proofs = [O.htree_inclusion_proof(lv, w, int(i))[1] for i in leaves]
    m = int(rng.integers(1, 500))
    p = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    return w, d, root, leaves, proofs, m, p


@pytest.mark.gpu
def test_threads_share_one_context():
    import torch
    import immustore_amd as m
    from immustore_amd import _native as N
    if m.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    L = N.load()
    ctx = m.Context(0)
    ctx.set_timing(True)
    cases = [[_case(1000 * t + r) for r in range(ROUNDS)] for t in range(THREADS)]
    # the ahtree every thread ends with, from the oracle
    final = []
    for t in range(THREADS):
        a = O.AHtree()
        for c in cases[t]:
            a.append_batch(c[6])
        final.append(a)

    # device-resident CSR entries for the mh_dev_* thread
    rng = np.random.default_rng(7)
    dev_cases = []
    for r in range(ROUNDS):
        n = int(rng.integers(1, 2000))
        keys = [rng.bytes(int(rng.integers(1, 40))) for _ in range(n)]
        vals = [rng.bytes(int(rng.integers(0, 300))) for _ in range(n)]
        st, _, _, root = O.build_entries(1, keys, [b""] * n, vals)
        assert st == 0

        def csr(items):
            off = np.zeros(n + 1, np.uint64)
            off[1:] = np.cumsum([len(x) for x in items])
            buf = np.frombuffer(b"".join(items) + b"\0", np.uint8)
            return (torch.from_numpy(buf.copy()).cuda(), torch.from_numpy(off.view(np.int64)).cuda())

        kb, ko = csr(keys)
        vb, vo = csr(vals)
        lv = torch.zeros(m.levels_len(n) * 32, dtype=torch.uint8, device="cuda")
        rt = torch.zeros(32, dtype=torch.uint8, device="cuda")
        dev_cases.append((n, kb, ko, vb, vo, lv, rt, root))
    torch.cuda.synchronize()

    errors = []

    def worker(t):
        try:
            ht = m.HTree(4096, ctx)
            ah = m.AHtree(ctx)
            try:
                for (w, d, root, leaves, proofs, mm, p) in cases[t]:
                    ht.build_with(d)
                    assert ht.root() == root
                    terms, nt, st = ht.inclusion_proof_batch(leaves)
                    assert (st == 0).all()
                    for k, pr in enumerate(proofs):
                        assert nt[k] == len(pr) and terms[k, :nt[k]].tobytes() == pr.tobytes()
                    ok = m.verify_inclusion_batch([ht.inclusion_proof(int(i)) for i in leaves[:4]],
                                                  d[leaves[:4].astype(np.int64)], [root] * 4, ctx=ctx)
                    assert all(ok)
                    ah.append_batch(p)
                o = final[t]
                assert ah.size() == o.size
                assert ah.root_at(o.size) == o.root_at(o.size)[1]
                j = np.full(8, o.size, np.uint64)
                i = np.linspace(1, o.size, 8).astype(np.uint64)
                terms, nt, st = ah.proof_batch(0, i, j)
                assert (st == 0).all()
                for k in range(8):
                    s, ref = o.inclusion_proof(int(i[k]), int(j[k]))
                    assert s == 0 and terms[k, :nt[k]].tobytes() == ref.tobytes()
            finally:
                ht.close()
                ah.close()
        except BaseException as e:  # noqa: BLE001 -- reported by the main thread
            errors.append((t, repr(e)))

    def dev_worker():
        try:
            for (n, kb, ko, vb, vo, lv, rt, root) in dev_cases:
                N.check(L.mh_dev_htree_build_entries(
                    ctx.handle, 1, n, C.c_void_p(kb.data_ptr()), C.c_void_p(ko.data_ptr()), None,
                    None, C.c_void_p(vb.data_ptr()), C.c_void_p(vo.data_ptr()), None, None, None,
                    C.c_void_p(lv.data_ptr()), C.c_void_p(rt.data_ptr())))
            ctx.synchronize()
            for (n, kb, ko, vb, vo, lv, rt, root) in dev_cases[-1:]:
                assert bytes(rt.cpu().numpy()) == root
        except BaseException as e:  # noqa: BLE001
            errors.append(("dev", repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    ths.append(threading.Thread(target=dev_worker))
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths), "worker threads did not finish"
    assert not errors, errors
    ms, launches = ctx.timing()
    assert launches > 0 and ms > 0
    ctx.close()
