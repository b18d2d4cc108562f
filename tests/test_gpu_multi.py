"""The multi-GPU htree build behind the C ABI (mh_multi_*) on
the one-GPU box: an RCCL clique of size 1 (devices [0]) exercises the real
ncclCommInitAll / ncclAllGather path; the same device listed several times
(more shards than devices, roots gathered by device copies) exercises the
shard plan, the per-shard level slices and the top levels with G > 1 -- all
against the oracle's build of the whole tree (htree.go:68-113,
immustore.go:1620-1630, tx.go:332-355)."""
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


def _inputs(orc, n, klen, vlen, seed):
    vals = orc.fill_random(n * vlen, seed).reshape(n, vlen)
    keys = orc.fill_random(n * klen, seed + 1).reshape(n, klen)
    return keys, vals


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_multi_host_build_vs_oracle(m, orc, devices):
    from immustore_amd.multi import MultiDevice, shard_plan
    md = MultiDevice(devices)
    try:
        for n in (1, 2, 3, 7, 8, 9, 1000, 4097, 65537, (1 << 18) + 3):
            keys, vals = _inputs(orc, n, 8, 256, n)
            hv, lv, root = md.build_entries_fixed(1, keys, vals)
            ohv, olv, oroot = orc.build_entries_fixed(1, keys, vals, nthreads=8)
            S, G = shard_plan(n, len(devices))
            assert root == oroot, (devices, n, S, G)
            assert np.array_equal(lv, olv), (devices, n)
            assert np.array_equal(hv, ohv), (devices, n)
        # odd shapes go through the device's general path shard by shard
        keys, vals = _inputs(orc, 3001, 5, 77, 9)
        hv, lv, root = md.build_entries_fixed(0, keys, vals)
        ohv, olv, oroot = orc.build_entries_fixed(0, keys, vals)
        assert root == oroot and np.array_equal(lv, olv) and np.array_equal(hv, ohv)
        # empty tree: SHA256(nil), htree.go:73-77
        _, _, root = md.build_entries_fixed(1, np.zeros((0, 8), np.uint8),
                                            np.zeros((0, 16), np.uint8))
        assert root == orc.sha256(b"")
    finally:
        md.close()


@pytest.mark.parametrize("devices,n_per_dev", [([0], 1 << 16), ([0, 0, 0, 0], 1 << 14),
                                               ([0, 0, 0, 0, 0, 0, 0, 0], 1 << 12)])
def test_multi_device_resident_vs_oracle(m, orc, devices, n_per_dev):
    """Device-resident shards (the configs[3] shape): every device's subtree
    levels are its slice of the global levels, and every device ends with the
    same top levels and the global root."""
    import torch
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    K = len(devices)
    n = K * n_per_dev
    keys, vals = _inputs(orc, n, 8, 1024, 77)
    md = MultiDevice(devices)
    try:
        dk = [torch.from_numpy(keys[d * n_per_dev:(d + 1) * n_per_dev].reshape(-1).copy()).cuda()
              for d in range(K)]
        dv = [torch.from_numpy(vals[d * n_per_dev:(d + 1) * n_per_dev].reshape(-1).copy()).cuda()
              for d in range(K)]
        lv = [torch.empty(m.levels_len(n_per_dev) * 32, dtype=torch.uint8, device="cuda")
              for _ in range(K)]
        top = [torch.empty(m.levels_len(K) * 32, dtype=torch.uint8, device="cuda")
               for _ in range(K)]
        rt = [torch.empty(32, dtype=torch.uint8, device="cuda") for _ in range(K)]
        hv = [torch.empty(n_per_dev * 32, dtype=torch.uint8, device="cuda") for _ in range(K)]
        torch.cuda.synchronize()
        ptr = lambda ts: [t.data_ptr() for t in ts]  # noqa: E731
        md.dev_build_entries_fixed(1, n_per_dev, ptr(dk), 8, ptr(dv), 1024, ptr(lv), ptr(top),
                                   ptr(rt), ptr(hv))
        md.synchronize()
        ohv, olv, oroot = orc.build_entries_fixed(1, keys, vals, nthreads=8)
        k = n_per_dev.bit_length() - 1
        for d in range(K):
            assert rt[d].cpu().numpy().tobytes() == oroot, d
            got = lv[d].cpu().numpy().reshape(-1, 32)
            for l in range(k + 1):
                w = n_per_dev >> l
                src = got[m.level_offset(n_per_dev, l):m.level_offset(n_per_dev, l) + w]
                o = m.level_offset(n, l) + d * w
                assert np.array_equal(src, olv[o:o + w]), (d, l)
            assert np.array_equal(hv[d].cpu().numpy().reshape(-1, 32),
                                  ohv[d * n_per_dev:(d + 1) * n_per_dev])
            tg = top[d].cpu().numpy().reshape(-1, 32)
            for j in range(1, (K - 1).bit_length() + 1):
                w = -(-K // (1 << j))
                o = m.level_offset(n, k + j)
                assert np.array_equal(tg[m.level_offset(K, j):m.level_offset(K, j) + w],
                                      olv[o:o + w]), (d, j)
        N.check(0)
    finally:
        md.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_multi_ahtree_append_vs_oracle(m, orc, devices):
    """mh_multi_ahtree_append_batch: the whole dLog (tree/*.sha stream) and
    RootAt(m) equal the oracle's single AppendBatch (ahtree.go:246-373,
    :727-771) -- ranges of 2^k appends per device, the shard roots exchanged
    (RCCL for [0], device copies when the device repeats)."""
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    md = MultiDevice(devices)
    try:
        for total in (1, 2, 3, 5, 8, 9, 1000, 4096, 70001, (1 << 17) + 5):
            pay = orc.fill_random(32 * total, total).reshape(total, 32)
            dl, root = md.ahtree_append_batch(pay)
            o = orc.AHtree(total)
            o.append_batch(pay)
            assert dl.tobytes() == o.dlog_bytes(), (devices, total)
            assert root == bytes(o.root_at(total)[1]), (devices, total)
        # other payload sizes (the leaf kernel's per-lane byte path)
        for plen in (0, 1, 100):
            pay = orc.fill_random(plen * 777 + 1, plen)[:plen * 777].reshape(777, plen)
            dl, root = md.ahtree_append_batch(pay)
            o = orc.AHtree(777)
            o.append_batch(pay)
            assert dl.tobytes() == o.dlog_bytes() and root == bytes(o.root_at(777)[1]), plen
        with pytest.raises(N.MerkleError):
            md.ahtree_append_batch(np.zeros((0, 32), np.uint8))
    finally:
        md.close()


@pytest.mark.parametrize("devices,total", [([0], 1 << 14), ([0, 0, 0, 0], 1 << 16),
                                           ([0, 0, 0, 0], 3 * (1 << 14) + 5)])
def test_multi_dev_ahtree_append_vs_oracle(m, orc, devices, total):
    """Device-resident ranges (the configs[2]-at-scale shape): device d fills
    its range of a globally indexed dLog byte-identically to one device's
    append; its roots_out are RootAt after each of its appends."""
    import torch
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    L = N.load()
    K = len(devices)
    k = 0
    while K * (1 << k) < total:
        k += 1
    S = 1 << k
    pay = orc.fill_random(32 * total, 5).reshape(total, 32)
    nd = L.mh_ahtree_nodes_upto(total)
    o = orc.AHtree(total)
    o.append_batch(pay)
    ref = np.frombuffer(o.dlog_bytes(), np.uint8).reshape(-1, 32)
    md = MultiDevice(devices)
    try:
        spans = [(min(d * S, total), min(S, max(total - d * S, 0))) for d in range(K)]
        dp = [torch.from_numpy(pay[n0:n0 + c].reshape(-1).copy()).cuda() if c else None
              for n0, c in spans]
        dl = [torch.empty(nd * 32, dtype=torch.uint8, device="cuda") if c else None
              for _, c in spans]
        ro = [torch.empty(c * 32, dtype=torch.uint8, device="cuda") if c else None
              for _, c in spans]
        torch.cuda.synchronize()
        ptr = lambda ts: [t.data_ptr() if t is not None else None for t in ts]  # noqa: E731
        md.dev_ahtree_append_batch(total, ptr(dp), 32, ptr(dl), ptr(ro))
        md.synchronize()
        covered = 0
        for d, (n0, c) in enumerate(spans):
            if not c:
                continue
            lo, hi = L.mh_ahtree_node_index(n0 + 1, 0), L.mh_ahtree_nodes_upto(n0 + c)
            got = dl[d].cpu().numpy().reshape(-1, 32)
            assert np.array_equal(got[lo:hi], ref[lo:hi]), d
            covered += hi - lo
            r = ro[d].cpu().numpy().reshape(-1, 32)
            for j in (0, c // 2, c - 1):
                assert r[j].tobytes() == bytes(o.root_at(n0 + j + 1)[1]), (d, j)
        assert covered == nd
    finally:
        md.close()


def _ragged(orc, n, seed, md=True):
    rng = np.random.default_rng(seed)
    out = []
    for lo, hi in ((8, 64), (0, 11), (0, 3000)):
        ln = rng.integers(lo, hi + 1, n).astype(np.uint64)
        off = np.zeros(n + 1, np.uint64)
        np.cumsum(ln, out=off[1:])
        off += np.uint64(rng.integers(0, 5))  # offsets need not start at 0
        out.append((orc.fill_random(int(off[-1]) + 16, seed + len(out)), off))
    (kb, ko), (mb, mo), (vb, vo) = out
    return kb, ko, (mb if md else None), (mo if md else None), vb, vo


@pytest.mark.parametrize("devices", [[0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_multi_ragged_build_vs_oracle(m, orc, devices):
    """mh_multi_htree_build_entries: ragged CSR entries (key 8-64 B, KV
    metadata 0-11 B, value 0-3000 B, offsets not starting at 0), some with
    IsValueTruncated overrides, v1 and v0, sharded over the devices: hVals,
    every level and the root equal the oracle's single build (immustore.go:
    1620-1630, tx.go:332-355, htree.go:68-113)."""
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice
    md = MultiDevice(devices)
    try:
        for n in (1, 2, 3, 1000, 20001):
            kb, ko, mb, mo, vb, vo = _ragged(orc, n, n)
            rng = np.random.default_rng(n)
            ov = rng.integers(0, 256, (n, 32), dtype=np.uint8)
            use = (rng.random(n) < 0.2).astype(np.uint8)
            for version, mdd, ovv in ((1, True, False), (1, True, True), (0, False, True)):
                args = (kb, ko, mb if mdd else None, mo if mdd else None, vb, vo)
                hv, lv, root = md.build_entries(version, *args, ov=ov if ovv else None,
                                                use=use if ovv else None)
                st, ohv, olv, oroot = orc.build_entries_csr(version, *args,
                                                            ov=ov if ovv else None,
                                                            use=use if ovv else None)
                assert st == 0
                assert root == oroot, (devices, n, version)
                assert np.array_equal(lv, olv) and np.array_equal(hv, ohv), (devices, n, version)
        # v0 with KV metadata: ErrMetadataUnsupported (tx.go:691-693)
        kb, ko, mb, mo, vb, vo = _ragged(orc, 100, 3)
        with pytest.raises(N.MerkleError):
            md.build_entries(0, kb, ko, mb, mo, vb, vo)
        _, _, root = md.build_entries(1, kb, ko[:1], None, None, vb, vo[:1])
        assert root == orc.sha256(b"")
    finally:
        md.close()
