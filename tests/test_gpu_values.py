"""The read-side value integrity check on the device (mh_verify_values_batch /
mh_dev_verify_values_batch) against the oracle's restatement of
ImmuStore.readValueAt (embedded/store/immustore.go:3183-3240): a value is
corrupted when the bytes read are not vLen long or their SHA-256 is not the
stored hVal (:3235).  Flipped bytes, short and long reads, wrong hVals, empty
values; batches large enough for the chunked host pipeline (several 64 MiB
chunks, one value larger than a chunk)."""
import os

import numpy as np
import pytest

from test_oracle import _values_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import torch  # noqa: F401
    import immustore_amd as m
    if m.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return m


def test_verify_values_small_vs_oracle(m, orc):
    for seed in (1, 2, 3):
        vb, off, hv, vlen, bad = _values_case(seed)
        c, st = m.verify_values(vb, off, hv, vlen)
        oc, ost = orc.verify_values(vb, off, hv, vlen)
        assert c == oc == int(bad.sum())
        assert np.array_equal(st, ost)
        c2, st2 = m.verify_values(vb, off, hv, None)
        oc2, ost2 = orc.verify_values(vb, off, hv, None)
        assert c2 == oc2 and np.array_equal(st2, ost2)
    # offsets need not start at 0; every value empty; nothing at all
    vb, off, hv, vlen, bad = _values_case(4, 50)
    pad = np.concatenate([np.zeros(7, np.uint8), vb])
    c, st = m.verify_values(pad, off + np.uint64(7), hv, vlen)
    assert np.array_equal(st != 0, bad)
    import hashlib
    e = np.frombuffer(hashlib.sha256(b"").digest() * 5, np.uint8).reshape(5, 32).copy()
    e[3, 0] ^= 1
    c, st = m.verify_values(np.zeros(0, np.uint8), np.zeros(6, np.uint64), e,
                            np.array([0, 0, 0, 0, 1], np.uint64))
    assert c == 2 and list(st != 0) == [False, False, False, True, True]
    c, st = m.verify_values(np.zeros(0, np.uint8), np.zeros(1, np.uint64), np.zeros((0, 32), np.uint8))
    assert c == 0 and len(st) == 0


def test_verify_values_chunked_vs_oracle(m, orc):
    """2^19 ragged values (0..4096 B, ~1 GiB) plus one 80 MiB value: the host
    call crosses many 64 MiB chunks of its copy / check pipeline."""
    rng = np.random.default_rng(9)
    n = (1 << 19) + 1
    lens = rng.integers(0, 4097, n).astype(np.uint64)
    lens[n // 3] = 80 << 20
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    vb = orc.fill_random(int(off[-1]), 17)
    hv = np.zeros((n, 32), np.uint8)
    # stored hVals from the oracle itself on the clean values (status 14 is
    # written for every entry whose hVal is zeros, so compute them first)
    ctx = m.default_context()
    import torch
    from immustore_amd import _native as N
    L = N.load()
    dv = torch.from_numpy(vb).cuda()
    do = torch.from_numpy(off.view(np.int64)).cuda()
    dh = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    N.check(L.mh_dev_sha256_batch(ctx.handle, dv.data_ptr(), do.data_ptr(), n, dh.data_ptr()))
    ctx.synchronize()
    hv[:] = dh.cpu().numpy().reshape(n, 32)
    vlen = lens.copy()
    sel = rng.choice(n, 3000, replace=False)
    for i in sel[:1000]:
        hv[i, int(rng.integers(0, 32))] ^= 1
    for i in sel[1000:2000]:
        vlen[i] += np.uint64(1)
    flip = [int(i) for i in sel[2000:] if lens[i] > 0] + [n // 3]
    for i in flip:
        vb[int(off[i]) + int(rng.integers(0, int(lens[i])))] ^= 0x40
    oc, ost = orc.verify_values(vb, off, hv, vlen, nthreads=min(16, os.cpu_count() or 1))
    c, st = m.verify_values(vb, off, hv, vlen)
    assert c == oc and np.array_equal(st, ost)
    assert st[n // 3] != 0
    # the device variant over the same (now corrupted) bytes
    dv = torch.from_numpy(vb).cuda()
    dh = torch.from_numpy(hv.reshape(-1)).cuda()
    dl = torch.from_numpy(vlen.view(np.int64)).cuda()
    ds = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    N.check(L.mh_dev_verify_values_batch(ctx.handle, n, dv.data_ptr(), do.data_ptr(),
                                         dl.data_ptr(), dh.data_ptr(), ds.data_ptr()))
    ctx.synchronize()
    assert np.array_equal(ds.cpu().numpy(), ost)
