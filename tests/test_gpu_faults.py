"""Error paths through the C ABI on the MI355X:
a failure injected with the test-only hook mh_debug_fail_at must return a
status, leave no RCCL group open and no kernel writing caller memory, and the
next call on the same handle must succeed and match the oracle.  Also the
ahtree batch shapes the Go shim now passes (zero-length payloads with no
payload pointer; mixed payload lengths as runs onto the previous peaks,
ahtree.go:260-263, 279)."""
import ctypes as C

import numpy as np
import pytest

from tx_util import _bulk_txlog

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import torch  # noqa: F401
    import immustore_amd as m
    if m.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return m


def test_rccl_group_closed_after_injected_failure(m, orc):
    """A failure inside the RCCL group of the all-gather (after
    ncclGroupStart) returns an error; the group is ended on that path, so the
    next mh_multi_dev_htree_build_entries_fixed on the same one-device RCCL
    clique completes (no hang) and its root equals the oracle's."""
    import torch
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    L = N.load()
    n, vl, kl = 1 << 12, 256, 8
    vals = orc.fill_random(n * vl, 21).reshape(n, vl)
    keys = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).reshape(n, kl)
    _, _, want = orc.build_entries_fixed(1, keys, vals)
    md = MultiDevice([0])
    assert md.uses_rccl()
    try:
        dk = torch.from_numpy(keys.reshape(-1).copy()).cuda()
        dv = torch.from_numpy(vals.reshape(-1).copy()).cuda()
        lv = torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device="cuda")
        top = torch.empty(32 * 2, dtype=torch.uint8, device="cuda")
        rt = torch.empty(32, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        args = (1, n, [dk.data_ptr()], kl, [dv.data_ptr()], vl, [lv.data_ptr()],
                [top.data_ptr()], [rt.data_ptr()])
        N.check(L.mh_debug_fail_at(N.MH_FAULT_RCCL_GROUP, 1))
        try:
            with pytest.raises(N.MerkleError):
                md.dev_build_entries_fixed(*args)
        finally:
            N.check(L.mh_debug_fail_at(N.MH_FAULT_RCCL_GROUP, 0))
        md.synchronize()
        rt.zero_()
        torch.cuda.synchronize()
        md.dev_build_entries_fixed(*args)
        md.synchronize()
        assert rt.cpu().numpy().tobytes() == want
        # and once more, host variant through the same clique
        _, _, r2 = md.build_entries_fixed(1, keys, vals, want_levels=False)
        assert r2 == want
    finally:
        md.close()


def test_rccl_clique_aborted_after_late_failure(m, orc):
    """A failure after the group's collectives were queued (on
    K > 1 devices those would wait for peers that never join) aborts the
    clique: the call returns MH_ERR_COLLECTIVE, every later collective on the
    handle returns it too (no hang), the handle still closes, and a new
    clique on the same device builds the oracle's root."""
    import torch
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    L = N.load()
    n, vl, kl = 1 << 12, 256, 8
    vals = orc.fill_random(n * vl, 22).reshape(n, vl)
    keys = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).reshape(n, kl)
    _, _, want = orc.build_entries_fixed(1, keys, vals)
    dk = torch.from_numpy(keys.reshape(-1).copy()).cuda()
    dv = torch.from_numpy(vals.reshape(-1).copy()).cuda()
    lv = torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device="cuda")
    top = torch.empty(32 * 2, dtype=torch.uint8, device="cuda")
    rt = torch.empty(32, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    args = (1, n, [dk.data_ptr()], kl, [dv.data_ptr()], vl, [lv.data_ptr()],
            [top.data_ptr()], [rt.data_ptr()])
    md = MultiDevice([0])
    assert md.uses_rccl()
    try:
        N.check(L.mh_debug_fail_at(N.MH_FAULT_RCCL_GROUP_LATE, 1))
        try:
            with pytest.raises(N.MerkleError) as e:
                md.dev_build_entries_fixed(*args)
            assert e.value.status == N.MH_ERR_COLLECTIVE
        finally:
            N.check(L.mh_debug_fail_at(N.MH_FAULT_RCCL_GROUP_LATE, 0))
        with pytest.raises(N.MerkleError) as e:
            md.dev_build_entries_fixed(*args)
        assert e.value.status == N.MH_ERR_COLLECTIVE
    finally:
        md.close()
    md = MultiDevice([0])
    try:
        rt.zero_()
        torch.cuda.synchronize()
        md.dev_build_entries_fixed(*args)
        md.synchronize()
        assert rt.cpu().numpy().tobytes() == want
    finally:
        md.close()


def test_debug_fail_at_arguments(m):
    from immustore_amd import _native as N
    L = N.load()
    assert L.mh_debug_fail_at(0, 1) == N.MH_ERR_ILLEGAL_ARGUMENTS
    assert L.mh_debug_fail_at(99, 1) == N.MH_ERR_ILLEGAL_ARGUMENTS
    assert L.mh_debug_fail_at(N.MH_FAULT_RCCL_GROUP, -1) == N.MH_ERR_ILLEGAL_ARGUMENTS
    assert L.mh_debug_fail_at(N.MH_FAULT_RCCL_GROUP, 0) == N.MH_OK


def test_txlog_failure_after_early_groups(m, orc):
    """mh_txlog_validate failing after its first chunk groups were queued
    (their kernels store into the caller's pinned outputs): the call returns
    an error only after those kernels are done -- the outputs do not change
    after the return -- and the next call on the context matches the oracle."""
    import time

    import torch
    from immustore_amd import _native as N
    from immustore_amd.txlayer import TX_HEADER
    L = N.load()
    rng = np.random.default_rng(44)
    raw, starts = _bulk_txlog(rng, 9000)
    assert len(raw) >= (16 << 20)  # several copy chunks, early groups
    pin = torch.empty(len(raw), dtype=torch.uint8).pin_memory()
    pin.numpy()[:] = np.frombuffer(raw, np.uint8)
    cap = 9100
    hd = torch.empty(cap * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER)
    alh = torch.empty(cap * 32, dtype=torch.uint8).pin_memory().numpy().reshape(cap, 32)
    sts = torch.empty(cap, dtype=torch.int32).pin_memory().numpy()
    ctx = m.Context(0)
    try:
        alh[:] = 0
        sts[:] = -7
        ntx, used = C.c_uint64(), C.c_uint64()
        N.check(L.mh_debug_fail_at(N.MH_FAULT_TXLOG_AFTER_GROUP, 1))
        try:
            rc = L.mh_txlog_validate(ctx.handle, pin.numpy().ctypes.data, len(raw), 1024, 1024,
                                     cap, C.byref(ntx), C.byref(used), hd.ctypes.data,
                                     alh.ctypes.data, sts.ctypes.data)
        finally:
            N.check(L.mh_debug_fail_at(N.MH_FAULT_TXLOG_AFTER_GROUP, 0))
        assert rc < 0  # the injected HIP out-of-memory
        snap = (alh.copy(), sts.copy())
        time.sleep(0.05)
        assert np.array_equal(alh, snap[0]) and np.array_equal(sts, snap[1])
        # the early groups were the ones written: some results landed
        assert (sts != -7).any()
        a = m.txlog_validate(pin.numpy(), ctx=ctx, out=(hd, alh, sts))
        o = orc.txlog_validate(raw)
        assert (a[0], a[1], a[2]) == (o[0], o[1], o[2])
        assert np.array_equal(a[4], o[3]) and list(a[5]) == list(o[4])
    finally:
        ctx.close()


def test_multi_ahtree_zero_length_payloads_null_pointer(m, orc):
    """plen 0 with payloads == NULL (what the Go shim passes for empty
    payloads): the same dLog and root as the oracle's appends of b''."""
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    L = N.load()
    M = 1000
    o = orc.AHtree(M)
    for _ in range(M):
        o.append(b"")
    nd = L.mh_ahtree_nodes_upto(M)
    dl = np.zeros((nd, 32), np.uint8)
    root = np.zeros(32, np.uint8)
    md = MultiDevice([0])
    try:
        N.check(L.mh_multi_ahtree_append_batch(md.handle, 0, None, None, M, 0, dl.ctypes.data,
                                                root.ctypes.data))
    finally:
        md.close()
    assert dl.tobytes() == o.dlog_bytes()
    assert root.tobytes() == bytes(o.root_at(M)[1])


def test_multi_ahtree_mixed_lengths_as_runs(m, orc):
    """Mixed payload lengths (AppendBatch's runs): each run of equal length
    one mh_multi_ahtree_append_batch onto the previous peaks; the dLog and
    roots equal single Appends of the whole mixed sequence."""
    from immustore_amd.multi import MultiDevice, peaks_of
    rng = np.random.default_rng(5)
    lens = [32] * 700 + [7] * 300 + [0] * 5 + [32] * 1000 + [100] * 33
    pays = [orc.fill_random(ln + 1, 1000 + i)[:ln].tobytes() for i, ln in enumerate(lens)]
    o = orc.AHtree(len(pays))
    for p in pays:
        o.append(p)
    full = np.frombuffer(o.dlog_bytes(), np.uint8).reshape(-1, 32)
    from immustore_amd import _native as N
    L = N.load()
    md = MultiDevice([0, 0])
    try:
        n0, got = 0, []
        i = 0
        while i < len(pays):
            j = i
            while j < len(pays) and len(pays[j]) == len(pays[i]):
                j += 1
            run = np.frombuffer(b"".join(pays[i:j]), np.uint8).reshape(j - i, len(pays[i]))
            dl, root = md.ahtree_append_batch(run, n0=n0, peaks=peaks_of(full, n0) if n0 else None)
            got.append(dl.tobytes())
            assert root == bytes(o.root_at(j)[1]), (i, j)
            n0, i = j, j
        assert b"".join(got) == o.dlog_bytes()
        del rng
    finally:
        md.close()
    assert L.mh_ahtree_nodes_upto(len(pays)) == full.shape[0]
