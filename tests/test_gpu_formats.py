"""GPU parity for SURVEY.md 8(f) row 4, the formats either side of the path:
the ahtree appendable record streams (pLog / cLog / dLog, ahtree.go:266-351)
written by the device next to the dLog.

Pinned by the Go-written aht/{data,commit,tree} files of the reference's test
stores (tests/golden/immudb_fixtures.json) and by the oracle's restatement
(orc_ahtree_log_records).  Bit-exact.
"""
import ctypes as C

import numpy as np
import pytest

from gpu_util import DevBuf

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


def expected_logs(pay, p_off0):
    """numpy restatement of the record streams for a fixed payload size."""
    mm, plen = pay.shape
    rec = 4 + plen
    plog = np.zeros((mm, rec), np.uint8)
    plog[:, :4] = np.frombuffer(np.uint32(plen).byteswap().tobytes(), np.uint8)
    plog[:, 4:] = pay
    clog = np.zeros((mm, 12), np.uint8)
    off = (p_off0 + np.arange(mm, dtype=np.uint64) * np.uint64(rec)).astype(">u8")
    clog[:, :8] = off.view(np.uint8).reshape(mm, 8)
    clog[:, 8:] = np.frombuffer(np.uint32(plen).byteswap().tobytes(), np.uint8)
    return plog.tobytes(), clog.tobytes()


@pytest.mark.parametrize("split", [0, 1, 5, 1000])
def test_go_fixture_appendables(m, ctx, fixtures, split):
    for name, fx in fixtures.items():
        pay = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
        k = min(split, len(pay))
        t = m.AHtree(ctx)
        p1, c1 = t.append_batch_logs(pay[:k], 0)
        p2, c2 = t.append_batch_logs(pay[k:], len(p1))
        assert p1 + p2 == bytes.fromhex(fx["aht_plog"]), name
        assert c1 + c2 == bytes.fromhex(fx["aht_clog"]), name
        assert t.dlog() == bytes.fromhex(fx["aht_dlog"]), name


def test_appendables_random_batches_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(44)
    t = m.AHtree(ctx)
    o = orc.AHtree()
    poff = 0
    for bs in [1, 255, 256, 257, 3, 4096, 70001, 2]:
        p = rng.integers(0, 256, (bs, 32), dtype=np.uint8)
        pl, cl = t.append_batch_logs(p, poff)
        opl, ocl = o.append_batch_logs(p, poff)
        assert pl == opl and cl == ocl, bs
        assert t.dlog() == o.dlog_bytes()
        poff += len(pl)
    # other payload sizes take the per-lane byte path
    for plen in [0, 1, 31, 33, 100]:
        p = rng.integers(0, 256, (300, plen), dtype=np.uint8)
        pl, cl = t.append_batch_logs(p, poff)
        opl, ocl = o.append_batch_logs(p, poff)
        assert pl == opl and cl == ocl, plen
        assert t.dlog() == o.dlog_bytes()
        poff += len(pl)


def test_appendables_large_offsets(m, ctx):
    """10^6 appends with a pLog offset above 2^32 (BE64 high word in use)."""
    from immustore_amd import _native as N
    M = 10 ** 6
    pay = np.random.default_rng(5).integers(0, 256, (M, 32), dtype=np.uint8)
    p0 = (1 << 32) + 12345 * 36
    t = m.AHtree(ctx)
    pl, cl = t.append_batch_logs(pay, p0)
    epl, ecl = expected_logs(pay, p0)
    assert pl == epl and cl == ecl
    # fused device call == separate append + records-only call
    L = N.load()
    dpay = DevBuf.from_host(ctx, pay)
    dl = DevBuf(ctx, orc_nodes_upto(M) * 32)
    dpl, dcl = DevBuf(ctx, M * 36), DevBuf(ctx, M * 12)
    N.check(L.mh_dev_ahtree_append_batch_logs(ctx.handle, C.c_void_p(dl.ptr), 0,
                                              C.c_void_p(dpay.ptr), M, 32, p0,
                                              C.c_void_p(dpl.ptr), C.c_void_p(dcl.ptr), None))
    ctx.synchronize()
    assert dpl.to_host().tobytes() == epl and dcl.to_host().tobytes() == ecl
    assert dl.to_host().tobytes() == t.dlog()


def orc_nodes_upto(n):
    from immustore_amd import _native as N
    return N.load().mh_ahtree_nodes_upto(n)


@pytest.mark.parametrize("shift", [0, 4, 1])
def test_records_only_alignment(m, ctx, shift):
    """mh_dev_ahtree_log_records at 16-, 4- and 1-byte aligned outputs (LDS
    staged dword stores vs the byte path) and with m not a multiple of 256."""
    from immustore_amd import _native as N
    L = N.load()
    M = 1000
    pay = np.random.default_rng(shift).integers(0, 256, (M, 32), dtype=np.uint8)
    dpay = DevBuf.from_host(ctx, pay)
    dpl, dcl = DevBuf(ctx, M * 36 + 32), DevBuf(ctx, M * 12 + 32)
    N.check(L.mh_dev_ahtree_log_records(ctx.handle, C.c_void_p(dpay.ptr), M, 32, 777,
                                        C.c_void_p(dpl.ptr + shift), C.c_void_p(dcl.ptr + shift)))
    ctx.synchronize()
    epl, ecl = expected_logs(pay, 777)
    assert dpl.to_host()[shift:shift + M * 36].tobytes() == epl
    assert dcl.to_host()[shift:shift + M * 12].tobytes() == ecl
    # NULL outputs and m = 0 are no-ops; offsets that overflow uint64 are rejected
    N.check(L.mh_dev_ahtree_log_records(ctx.handle, C.c_void_p(dpay.ptr), M, 32, 0, None, None))
    N.check(L.mh_dev_ahtree_log_records(ctx.handle, None, 0, 32, 0, C.c_void_p(dpl.ptr), None))
    assert L.mh_dev_ahtree_log_records(ctx.handle, C.c_void_p(dpay.ptr), M, 32, (1 << 64) - 100,
                                       C.c_void_p(dpl.ptr), None) == N.MH_ERR_ILLEGAL_ARGUMENTS
