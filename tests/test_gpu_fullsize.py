"""BASELINE.json configs at their full sizes, compared bit for bit with the
oracle (configs[1], 2^20 x 1 KiB, is in test_gpu_parity.py):

- configs[2]: ahtree append of 10^7 x 32 B payloads -- the whole 3.98 GB dLog
  stream (124,434,624 digests) and RootAt(10^7);
- configs[3] per GPU: 2^23 x 4 KiB entries (32 GiB of values generated in HBM
  from the same splitmix64 stream the oracle generates on the host) -- every
  level, every hVal and the subtree root.

Each takes tens of seconds of oracle time on the host (16 threads for the
htree, the ahtree append is serial as in Go)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import torch  # noqa: F401
    import immustore_amd as m
    if m.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return m


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def test_c3_full_dlog_vs_oracle(m, ctx, orc):
    import torch
    from immustore_amd import _native as N
    L = N.load()
    M = 10 ** 7
    dev = torch.device("cuda", 0)
    pay = torch.empty(M * 32, dtype=torch.uint8, device=dev)
    N.check(L.mh_dev_fill_random(ctx.handle, pay.data_ptr(), pay.numel(), 3))
    nd = m.nodes_upto(M)
    assert nd == 124_434_624
    dlog = torch.empty(nd * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    N.check(L.mh_dev_ahtree_append_batch(ctx.handle, dlog.data_ptr(), 0, pay.data_ptr(), M, 32,
                                         None))
    ctx.synchronize()
    got = dlog.cpu().numpy().reshape(nd, 32)
    hp = orc.fill_random(M * 32, 3).reshape(M, 32)
    assert np.array_equal(pay.cpu().numpy().reshape(M, 32), hp)
    o = orc.AHtree(M)
    o.append_batch(hp)
    assert np.array_equal(got, o.dlog[:nd])
    st, r = o.root_at(M)
    assert st == 0 and got[orc.nodes_until(M) + bin(M - 1).count("1")].tobytes() == r


def test_c4_per_gpu_full_vs_oracle(m, ctx, orc):
    import torch
    from immustore_amd import _native as N
    L = N.load()
    n, vlen = 1 << 23, 4096
    dev = torch.device("cuda", 0)
    vals = torch.empty(n * vlen, dtype=torch.uint8, device=dev)
    keys = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    N.check(L.mh_dev_fill_random(ctx.handle, vals.data_ptr(), vals.numel(), 4))
    N.check(L.mh_dev_fill_keys_be64(ctx.handle, keys.data_ptr(), n, 0))
    lv = torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device=dev)
    hv = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    root = torch.empty(32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    N.check(L.mh_dev_htree_build_entries_fixed(ctx.handle, 1, n, keys.data_ptr(), 8,
                                               vals.data_ptr(), vlen, hv.data_ptr(),
                                               lv.data_ptr(), root.data_ptr()))
    ctx.synchronize()
    del vals
    hk = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).reshape(n, 8)
    hvals = orc.fill_random(n * vlen, 4).reshape(n, vlen)
    ohv, olv, oroot = orc.build_entries_fixed(1, hk, hvals, nthreads=min(16, os.cpu_count() or 1))
    del hvals
    assert root.cpu().numpy().tobytes() == oroot
    assert np.array_equal(hv.cpu().numpy().reshape(n, 32), ohv)
    assert np.array_equal(lv.cpu().numpy().reshape(-1, 32), olv)


# ------------------------------------------------- values past the 32-bit lane offsets
# Go accepts any positive MaxValueLen (embedded/store/options.go:364-365); the
# fixed-stride kernel forms each lane's DMA offset from the wave's first entry
# in 32 bits (rel * val_len, rel <= 64 * LPL - 1), so values above 16 MiB must
# take the CSR path.  Each case hashes ~4.3 GB of values (immustore.go:1620-1630).
@pytest.mark.parametrize("n,vlen,lpl", [
    (64, (64 << 20) + 16, None),      # 63 * vlen alone is past 2^32
    (128, 33818640, "2"),             # LPL 2: 127 * vlen = 2^32 - 16, chunks wrap
    (256, 1 << 24, "4"),              # the largest fast-path value, rel up to 255
])
def test_big_values_vs_oracle(m, ctx, orc, n, vlen, lpl):
    import torch
    from immustore_amd import _native as N
    L = N.load()
    old = os.environ.get("MH_LPL")
    if lpl:
        os.environ["MH_LPL"] = lpl
    try:
        dev = torch.device("cuda", 0)
        vals = torch.empty(n * vlen, dtype=torch.uint8, device=dev)
        keys = torch.empty(n * 8, dtype=torch.uint8, device=dev)
        N.check(L.mh_dev_fill_random(ctx.handle, vals.data_ptr(), vals.numel(), 21))
        N.check(L.mh_dev_fill_keys_be64(ctx.handle, keys.data_ptr(), n, 0))
        lv = torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device=dev)
        hv = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        root = torch.empty(32, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        N.check(L.mh_dev_htree_build_entries_fixed(ctx.handle, 1, n, keys.data_ptr(), 8,
                                                   vals.data_ptr(), vlen, hv.data_ptr(),
                                                   lv.data_ptr(), root.data_ptr()))
        ctx.synchronize()
        del vals
    finally:
        if old is None:
            os.environ.pop("MH_LPL", None)
        else:
            os.environ["MH_LPL"] = old
    hk = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).reshape(n, 8)
    hvals = orc.fill_random(n * vlen, 21).reshape(n, vlen)
    ohv, olv, oroot = orc.build_entries_fixed(1, hk, hvals, nthreads=min(16, os.cpu_count() or 1))
    del hvals
    assert np.array_equal(hv.cpu().numpy().reshape(n, 32), ohv)
    assert np.array_equal(lv.cpu().numpy().reshape(-1, 32), olv)
    assert root.cpu().numpy().tobytes() == oroot


# ---------------------------------------------------------------- configs[4]
P_C5, D_C5 = 10 ** 6, 24


def _nodes_until(n):
    """nodesUntil(n) = nodesUpto(n-1) (ahtree.go:485-511) for a uint64 array."""
    x = np.asarray(n, np.uint64) - np.uint64(1)
    s = x.copy()
    for k in range(63):
        hi = (x >> np.uint64(k + 1)) << np.uint64(k)
        lo = x & np.uint64((1 << (k + 1)) - 1)
        s += hi + np.where(lo > np.uint64(1 << k), lo - np.uint64(1 << k), np.uint64(0))
    return s


def _popcount(v):
    v = np.asarray(v, np.uint64)
    c = np.zeros(v.shape, np.uint64)
    for k in range(64):
        c += (v >> np.uint64(k)) & np.uint64(1)
    return c


def _tamper(rng, terms_host, off, frac=0.10):
    """Flip one random bit of one random term in `frac` of the proofs (in place)."""
    n = len(off) - 1
    cnt = off[1:] - off[:-1]
    sel = np.nonzero((rng.random(n) < frac) & (cnt > 0))[0]
    t = off[sel] + (rng.random(len(sel)) * cnt[sel]).astype(np.int64)
    byte = rng.integers(0, 32, len(sel))
    bit = rng.integers(0, 8, len(sel)).astype(np.uint8)
    terms_host[t, byte] ^= (np.uint8(1) << bit)
    mask = np.zeros(n, bool)
    mask[sel] = True
    return mask


@pytest.mark.timeout(900)
def test_c5_htree_full_vs_oracle(m, ctx, orc):
    """configs[4], htree half at full size: a 2^24-leaf tree over seed-5
    digests built on the device (every level vs the oracle), 10^6 random-leaf
    depth-24 proofs generated on the device (htree.go:121-164; 10^4 sampled
    term lists vs the oracle), 10 % tampered (one bit of one term), and the
    whole 10^6-entry htree.VerifyInclusion bitmap (htree.go:166-195) vs the
    oracle's on the same inputs."""
    import torch
    from immustore_amd import _native as N
    L = N.load()
    W, P, D = 1 << D_C5, P_C5, D_C5
    dev = torch.device("cuda", 0)
    dig = torch.empty(W * 32, dtype=torch.uint8, device=dev)
    N.check(L.mh_dev_fill_random(ctx.handle, dig.data_ptr(), dig.numel(), 5))
    lv = torch.empty(m.levels_len(W) * 32, dtype=torch.uint8, device=dev)
    root = torch.empty(32, dtype=torch.uint8, device=dev)
    N.check(L.mh_dev_htree_build_digests(ctx.handle, dig.data_ptr(), W, lv.data_ptr(),
                                         root.data_ptr()))
    rng = np.random.default_rng(5)
    leaf = rng.integers(0, W, P, dtype=np.int64)
    leaf_t = torch.from_numpy(leaf).to(dev)
    terms = torch.empty(P * D * 32, dtype=torch.uint8, device=dev)
    nt = torch.empty(P, dtype=torch.int32, device=dev)
    pst = torch.empty(P, dtype=torch.int32, device=dev)
    N.check(L.mh_dev_htree_inclusion_proof_batch(ctx.handle, lv.data_ptr(), W, P,
                                                 leaf_t.data_ptr(), terms.data_ptr(), D,
                                                 nt.data_ptr(), pst.data_ptr()))
    ctx.synchronize()
    assert int(pst.abs().sum().item()) == 0 and int((nt != D).sum().item()) == 0
    hd = orc.fill_random(W * 32, 5).reshape(W, 32)
    assert np.array_equal(dig.cpu().numpy().reshape(W, 32), hd)
    olv, oroot = orc.htree_build(hd)
    assert root.cpu().numpy().tobytes() == oroot
    assert np.array_equal(lv.cpu().numpy().reshape(-1, 32), olv)
    th = terms.cpu().numpy().reshape(P, D, 32)
    for p in rng.choice(P, 10_000, replace=False):
        st, ot = orc.htree_inclusion_proof(olv, W, int(leaf[p]))
        assert st == 0 and np.array_equal(th[p], ot), p
    flat = th.reshape(P * D, 32)
    tam = _tamper(rng, flat, np.arange(0, (P + 1) * D, D, dtype=np.int64))
    # device verify of the tampered set (the terms go back to HBM)
    terms.copy_(torch.from_numpy(flat.reshape(-1)).to(dev))
    digs = dig.view(W, 32)[leaf_t].contiguous()
    width_t = torch.full((P,), W, dtype=torch.int64, device=dev)
    toff = torch.arange(0, (P + 1) * D, D, dtype=torch.int64, device=dev)
    roots = root.view(1, 32).expand(P, 32).contiguous()
    ok = torch.zeros(P, dtype=torch.uint8, device=dev)
    N.check(L.mh_dev_htree_verify_inclusion_batch(ctx.handle, P, leaf_t.data_ptr(),
                                                  width_t.data_ptr(), toff.data_ptr(),
                                                  terms.data_ptr(), digs.data_ptr(),
                                                  roots.data_ptr(), ok.data_ptr()))
    ctx.synchronize()
    c, ook = orc.htree_verify_batch(leaf.astype(np.uint64), W, flat.reshape(P, D, 32), hd[leaf],
                                    oroot)
    got = ok.cpu().numpy()
    assert np.array_equal(got, ook)
    assert c == P - int(tam.sum()) and np.array_equal(got.astype(bool), ~tam)


@pytest.mark.timeout(1200)
def test_c5_ahtree_full_vs_oracle(m, ctx, orc):
    """configs[4], ahtree half at full size: 2^24 appends (the device dLog, 6.98 GB,
    vs the oracle's), then 10^6 inclusion and 10^6 consistency proofs with
    j = 2^24 and random i, generated on the device (ahtree.go:525-661; 10^4
    sampled term lists each vs the oracle), 10 % tampered, and the device
    VerifyInclusion / VerifyConsistency bitmaps (ahtree/verification.go:21-109)
    vs the oracle's on the same inputs."""
    import torch
    from immustore_amd import _native as N
    L = N.load()
    W, P = 1 << D_C5, P_C5
    dev = torch.device("cuda", 0)
    pay = torch.empty(W * 32, dtype=torch.uint8, device=dev)
    N.check(L.mh_dev_fill_random(ctx.handle, pay.data_ptr(), pay.numel(), 55))
    nd = m.nodes_upto(W)
    dlog = torch.empty(nd * 32, dtype=torch.uint8, device=dev)
    N.check(L.mh_dev_ahtree_append_batch(ctx.handle, dlog.data_ptr(), 0, pay.data_ptr(), W, 32,
                                         None))
    ctx.synchronize()
    hp = orc.fill_random(W * 32, 55).reshape(W, 32)
    o = orc.AHtree(W)
    o.append_batch(hp)
    dl_h = dlog.cpu().numpy().reshape(nd, 32)
    assert np.array_equal(dl_h, o.dlog[:nd])
    del dl_h
    rng = np.random.default_rng(55)
    jv = np.full(P, W, np.uint64)
    root_idx = lambda v: _nodes_until(v) + _popcount(np.asarray(v, np.uint64) - np.uint64(1))  # noqa: E731
    jroot = o.dlog[root_idx(jv)]
    for kind, S in ((0, 64), (1, 128)):
        iv = rng.integers(1, W + 1, P).astype(np.uint64)
        it = torch.from_numpy(iv.view(np.int64)).to(dev)
        jt = torch.from_numpy(jv.view(np.int64)).to(dev)
        terms = torch.empty(P * S * 32, dtype=torch.uint8, device=dev)
        nt = torch.empty(P, dtype=torch.int32, device=dev)
        st = torch.empty(P, dtype=torch.int32, device=dev)
        N.check(L.mh_dev_ahtree_proof_batch(ctx.handle, kind, dlog.data_ptr(), W, P, it.data_ptr(),
                                            jt.data_ptr(), terms.data_ptr(), S, nt.data_ptr(),
                                            st.data_ptr()))
        ctx.synchronize()
        assert int(st.abs().sum().item()) == 0
        cnt = nt.cpu().numpy().astype(np.int64)
        th = terms.cpu().numpy().reshape(P, S, 32)
        del terms
        for p in rng.choice(P, 10_000, replace=False):
            prf = o.inclusion_proof if kind == 0 else o.consistency_proof
            s, ot = prf(int(iv[p]), W)
            assert s == 0 and cnt[p] == len(ot) and np.array_equal(th[p, :cnt[p]], ot), (kind, p)
        off = np.zeros(P + 1, np.int64)
        off[1:] = np.cumsum(cnt)
        flat = th[np.repeat(np.arange(P), cnt), np.arange(off[-1]) - np.repeat(off[:-1], cnt)]
        del th
        tam = _tamper(rng, flat, off)
        if kind == 0:
            a = o.dlog[_nodes_until(iv)]  # leaf digests SHA256(0x00 || payload)
        else:
            a = o.dlog[root_idx(iv)]      # RootAt(i)
        ok = torch.zeros(P, dtype=torch.uint8, device=dev)
        off_t = torch.from_numpy(off).to(dev)
        flat_t = torch.from_numpy(flat.reshape(-1)).to(dev)
        a_t = torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(dev)
        b_t = torch.from_numpy(np.ascontiguousarray(jroot).reshape(-1)).to(dev)
        N.check(L.mh_dev_ahtree_verify_batch(ctx.handle, kind, P, it.data_ptr(), jt.data_ptr(),
                                             off_t.data_ptr(), flat_t.data_ptr(), a_t.data_ptr(),
                                             b_t.data_ptr(), ok.data_ptr(), None))
        ctx.synchronize()
        c, ook = orc.ahtree_verify_batch(kind, iv, jv, off.astype(np.uint64), flat, a, jroot,
                                         nthreads=min(16, os.cpu_count() or 1))
        got = ok.cpu().numpy()
        assert np.array_equal(got, ook), kind
        # untampered proofs verify; every tampered one fails (a flipped term
        # bit changes the recomputed root(s)) -- except consistency proofs
        # whose tampered term is unused when i == j
        assert got[~tam].all() and c == int(got.sum())
        assert not got[tam & (iv != jv)].any()


def test_ragged_full_size_vs_oracle(m, ctx, orc):
    """The ragged workload of bench_workloads.py at its size: 2^20 entries,
    values 0-4096 B, keys 8-64 B, KV metadata 0-11 B, v1 -- every hVal, every
    level and the root through mh_dev_htree_build_entries."""
    import sys
    import torch
    from immustore_amd import _native as N
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench_workloads import ragged_inputs
    n = 1 << 20
    R = ragged_inputs(n, 4096)
    dev = torch.device("cuda", 0)
    d = {k: (torch.from_numpy(b).to(dev), torch.from_numpy(o.view(np.int64)).to(dev))
         for k, (b, o) in R.items()}
    nl = m.levels_len(n)
    lv = torch.empty(nl * 32, dtype=torch.uint8, device=dev)
    hv = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    root = torch.empty(32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    N.check(N.load().mh_dev_htree_build_entries(
        ctx.handle, 1, n, d["k"][0].data_ptr(), d["k"][1].data_ptr(), d["m"][0].data_ptr(),
        d["m"][1].data_ptr(), d["v"][0].data_ptr(), d["v"][1].data_ptr(), None, None,
        hv.data_ptr(), lv.data_ptr(), root.data_ptr()))
    ctx.synchronize()
    st, ohv, olv, oroot = orc.build_entries_csr(1, R["k"][0], R["k"][1], R["m"][0], R["m"][1],
                                                R["v"][0], R["v"][1])
    assert st == 0
    assert root.cpu().numpy().tobytes() == oroot
    assert np.array_equal(hv.cpu().numpy().reshape(n, 32), ohv)
    assert np.array_equal(lv.cpu().numpy().reshape(nl, 32), olv)
