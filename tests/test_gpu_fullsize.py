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
