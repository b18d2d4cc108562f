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
