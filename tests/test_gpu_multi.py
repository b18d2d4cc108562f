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
        # back-to-back builds with no host sync between them: on repeated
        # devices every stream's top reduce (which overwrites root[s]) must
        # wait for the other streams' copies of root[s]
        for rep in range(8):
            md.dev_build_entries_fixed(1, n_per_dev, ptr(dk), 8, ptr(dv), 1024, ptr(lv), ptr(top),
                                       ptr(rt), None)
        md.synchronize()
        for d in range(K):
            assert rt[d].cpu().numpy().tobytes() == oroot, ("repeat", d)
        N.check(0)
    finally:
        md.close()


# one oracle tree long enough for every (n0, total) below: the dLog of the
# first n appends is the same prefix whatever comes after
_AHT_N0S = (0, 1, (1 << 13) - 1, 10 ** 6 + 3)
_AHT_TOTALS = (1, 2, 3, 5, 8, 9, 1000, 4096, 70001, (1 << 17) + 5)


@pytest.fixture(scope="module")
def aht_ref(orc):
    N_all = max(_AHT_N0S) + max(_AHT_TOTALS)
    pay = orc.fill_random(32 * N_all, 123).reshape(N_all, 32)
    o = orc.AHtree(N_all)
    o.append_batch(pay)
    return pay, o, np.frombuffer(o.dlog_bytes(), np.uint8).reshape(-1, 32)


@pytest.mark.parametrize("devices", [[0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_multi_ahtree_append_vs_oracle(m, orc, aht_ref, devices):
    """mh_multi_ahtree_append_batch onto trees of n0 in {0, 1, 2^13-1,
    10^6+3} (the replay of syncBinaryLinking resumes at aht.Size()+1,
    immustore.go:1198-1232): the new dLog digests (tree/*.sha stream) and
    RootAt(n0 + total) equal the oracle's single AppendBatch (ahtree.go:246-373,
    :727-771) -- nearly equal ranges per device, each device holding only its
    own range; the piece roots exchanged over RCCL for [0], by device copies
    when the device repeats."""
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice, peaks_of
    L = N.load()
    pay, o, ref = aht_ref
    md = MultiDevice(devices)
    try:
        for n0 in _AHT_N0S:
            pk = peaks_of(ref, n0)
            for total in _AHT_TOTALS:
                dl, root = md.ahtree_append_batch(pay[n0:n0 + total], n0=n0, peaks=pk)
                lo, hi = L.mh_ahtree_nodes_upto(n0), L.mh_ahtree_nodes_upto(n0 + total)
                assert np.array_equal(dl, ref[lo:hi]), (devices, n0, total)
                assert root == bytes(o.root_at(n0 + total)[1]), (devices, n0, total)
        # other payload sizes (the leaf kernel's per-lane byte path)
        for plen in (0, 1, 100):
            p2 = orc.fill_random(plen * 777 + 1, plen)[:plen * 777].reshape(777, plen)
            dl, root = md.ahtree_append_batch(p2)
            o2 = orc.AHtree(777)
            o2.append_batch(p2)
            assert dl.tobytes() == o2.dlog_bytes() and root == bytes(o2.root_at(777)[1]), plen
            # the same batch in two calls: the second onto the first's peaks
            full = np.frombuffer(o2.dlog_bytes(), np.uint8).reshape(-1, 32)
            dl2, root2 = md.ahtree_append_batch(p2[300:], n0=300, peaks=peaks_of(full, 300))
            assert dl2.tobytes() == o2.dlog_bytes()[L.mh_ahtree_nodes_upto(300) * 32:], plen
            assert root2 == root
        with pytest.raises(N.MerkleError):
            md.ahtree_append_batch(np.zeros((0, 32), np.uint8))
        with pytest.raises(N.MerkleError):  # n0 > 0 needs the old peaks
            md.ahtree_append_batch(pay[:5], n0=5)
    finally:
        md.close()


@pytest.mark.parametrize("devices,total", [([0], 1 << 14), ([0, 0, 0, 0], 1 << 16),
                                           ([0, 0, 0, 0], 3 * (1 << 14) + 5),
                                           ([0] * 8, 100003)])
@pytest.mark.parametrize("n0", _AHT_N0S)
def test_multi_dev_ahtree_append_vs_oracle(m, orc, aht_ref, devices, total, n0):
    """Device-resident ranges (the configs[2]-at-scale shape, and replay):
    device d holds only its range's digests [nodesUpto(b[d]), nodesUpto(b[d+1]))
    -- memory O(total / K) -- byte-identical to one device's append of the
    whole batch; its roots_out are RootAt after each of its appends."""
    import torch
    from immustore_amd import _native as N
    from immustore_amd.multi import MultiDevice, ahtree_range_plan, peaks_of
    L = N.load()
    K = len(devices)
    pay, o, ref = aht_ref
    _, b = ahtree_range_plan(n0, total, K)
    G = len(b) - 1
    md = MultiDevice(devices)
    try:
        up = L.mh_ahtree_nodes_upto
        dp = [torch.from_numpy(pay[b[d]:b[d + 1]].reshape(-1).copy()).cuda() if d < G else None
              for d in range(K)]
        dl = [torch.empty((up(b[d + 1]) - up(b[d])) * 32, dtype=torch.uint8, device="cuda")
              if d < G else None for d in range(K)]
        ro = [torch.empty((b[d + 1] - b[d]) * 32, dtype=torch.uint8, device="cuda")
              if d < G else None for d in range(K)]
        torch.cuda.synchronize()
        ptr = lambda ts: [t.data_ptr() if t is not None else None for t in ts]  # noqa: E731
        md.dev_ahtree_append_batch(total, ptr(dp), 32, ptr(dl), ptr(ro), n0=n0,
                                   peaks=peaks_of(ref, n0))
        md.synchronize()
        for d in range(G):
            got = dl[d].cpu().numpy().reshape(-1, 32)
            assert np.array_equal(got, ref[up(b[d]):up(b[d + 1])]), (d, b)
            r = ro[d].cpu().numpy().reshape(-1, 32)
            c = b[d + 1] - b[d]
            for j in (0, c // 2, c - 1):
                assert r[j].tobytes() == bytes(o.root_at(b[d] + j + 1)[1]), (d, j)
    finally:
        md.close()


@pytest.mark.parametrize("world,total", [(1, 1 << 14), (2, 1 << 16), (3, 3 * (1 << 14) + 5),
                                         (4, 1000), (8, 100003), (8, 5)])
@pytest.mark.parametrize("n0", _AHT_N0S)
def test_rank_ahtree_range_append_vs_oracle(m, orc, aht_ref, world, total, n0):
    """The one-process-per-GPU form (mh_dev_ahtree_range_local / _finish,
    what bench_workloads.py --workload c3 runs under torch.distributed): the
    `world` ranks played one after the other on one device, each with its own
    context, work buffer and range, the all-gather done by hand in rank order
    between the two calls -- every rank's range and roots equal the oracle's
    single AppendBatch (ahtree.go:246-373); ranks past the plan's ranges
    (total = 5 over 8 ranks) do nothing."""
    import torch
    from immustore_amd import _native as N
    from immustore_amd import sharding
    from immustore_amd.multi import ahtree_range_plan, peaks_of
    L = N.load()
    up = L.mh_ahtree_nodes_upto
    pay, o, ref = aht_ref
    _, b = ahtree_range_plan(n0, total, world)
    G = len(b) - 1
    send_b, work_b = sharding.ahtree_range_sizes(n0, total, world)
    pk = peaks_of(ref, n0) if n0 else None
    ctxs = [m.Context(0) for _ in range(world)]
    try:
        rng = lambda r: (b[r], b[r + 1]) if r < G else (b[G], b[G])  # noqa: E731
        dp = [torch.from_numpy(pay[rng(r)[0]:rng(r)[1]].reshape(-1).copy()).cuda()
              if r < G else torch.empty(32, dtype=torch.uint8, device="cuda") for r in range(world)]
        dl = [torch.empty(max(up(rng(r)[1]) - up(rng(r)[0]), 1) * 32, dtype=torch.uint8,
                          device="cuda") for r in range(world)]
        ro = [torch.empty(max(rng(r)[1] - rng(r)[0], 1) * 32, dtype=torch.uint8, device="cuda")
              for r in range(world)]
        work = [torch.empty(work_b, dtype=torch.uint8, device="cuda") for _ in range(world)]
        send = [torch.zeros(send_b, dtype=torch.uint8, device="cuda") for _ in range(world)]
        recv = [torch.empty(world * send_b, dtype=torch.uint8, device="cuda") for _ in range(world)]
        pkb = np.frombuffer(pk, np.uint8) if pk else None
        pkp = pkb.ctypes.data if pk else None
        torch.cuda.synchronize()
        for _rep in range(2):  # a second append of the same batch reuses the work buffers
            for r in range(world):
                N.check(L.mh_dev_ahtree_range_local(ctxs[r].handle, n0, pkp, total, world, r,
                                                    dp[r].data_ptr(), 32, dl[r].data_ptr(),
                                                    work[r].data_ptr(), send[r].data_ptr()))
            for c in ctxs:
                c.synchronize()
            gathered = torch.cat(send)
            for r in range(world):
                recv[r].copy_(gathered)
            torch.cuda.synchronize()
            for r in range(world):
                N.check(L.mh_dev_ahtree_range_finish(ctxs[r].handle, n0, pkp, total, world, r,
                                                     recv[r].data_ptr(), dl[r].data_ptr(),
                                                     work[r].data_ptr(), ro[r].data_ptr()))
            for c in ctxs:
                c.synchronize()
            for r in range(G):
                lo, hi = b[r], b[r + 1]
                got = dl[r].cpu().numpy().reshape(-1, 32)
                assert np.array_equal(got, ref[up(lo):up(hi)]), (world, n0, total, r)
                rr = ro[r].cpu().numpy().reshape(-1, 32)
                assert all(rr[j].tobytes() == bytes(o.root_at(lo + j + 1)[1])
                           for j in (0, (hi - lo) // 2, hi - lo - 1)), (world, n0, total, r)
        with pytest.raises(N.MerkleError):  # n0 > 0 needs the old peaks on every rank
            N.check(L.mh_dev_ahtree_range_local(ctxs[0].handle, 7, None, total, world, 0,
                                                dp[0].data_ptr(), 32, dl[0].data_ptr(),
                                                work[0].data_ptr(), send[0].data_ptr()))
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("n0", _AHT_N0S + (2 ** 20, 2 ** 20 - 1))
def test_dev_ahtree_append_range_vs_oracle(m, orc, aht_ref, n0):
    """One device, the dLog kept as a range (mh_dev_ahtree_append_range):
    only the old tree's peaks on the device (read back from a resident dLog
    with mh_dev_ahtree_peaks), the new digests and roots equal the oracle's."""
    import torch
    from immustore_amd import _native as N
    from immustore_amd.multi import peaks_of
    L = N.load()
    pay, o, ref = aht_ref
    ctx = m.Context(0)
    up = L.mh_ahtree_nodes_upto
    pk = peaks_of(ref, n0)
    if n0:
        dref = torch.from_numpy(ref[:up(n0)].reshape(-1).copy()).cuda()
        got = np.zeros(len(pk), np.uint8)
        N.check(L.mh_dev_ahtree_peaks(ctx.handle, dref.data_ptr(), n0, got.ctypes.data))
        assert got.tobytes() == pk
        del dref
    for total in (1, 2, 777, 70001):
        dp = torch.from_numpy(pay[n0:n0 + total].reshape(-1).copy()).cuda()
        dl = torch.empty((up(n0 + total) - up(n0)) * 32, dtype=torch.uint8, device="cuda")
        ro = torch.empty(total * 32, dtype=torch.uint8, device="cuda")
        pkb = np.frombuffer(pk, np.uint8) if n0 else None
        N.check(L.mh_dev_ahtree_append_range(ctx.handle, dl.data_ptr(), n0,
                                             pkb.ctypes.data if n0 else None, dp.data_ptr(),
                                             total, 32, ro.data_ptr()))
        ctx.synchronize()
        assert np.array_equal(dl.cpu().numpy().reshape(-1, 32), ref[up(n0):up(n0 + total)])
        r = ro.cpu().numpy().reshape(-1, 32)
        for j in (0, total // 2, total - 1):
            assert r[j].tobytes() == bytes(o.root_at(n0 + j + 1)[1]), (n0, total, j)


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


# ------------------------------------------------- PCIe-bound batch paths, split
_SPLIT_DEVICES = [[0], [0, 0], [0, 0, 0, 0], [0] * 8]


@pytest.mark.parametrize("devices", _SPLIT_DEVICES)
def test_multi_txlog_validate_vs_single_and_oracle(m, orc, fixtures, devices):
    """mh_multi_txlog_validate (the log cut at record boundaries, part d on
    device d): status, count, consumed bytes, every header (md_off relative to
    the whole log), Alh and per-tx status byte-equal to one mh_txlog_validate
    call and to the oracle -- synthetic logs with metadata and mixed versions,
    corrupted records, a log cut inside a record (structural error), the
    Go-written fixture log (tx.go:388-630)."""
    from immustore_amd.multi import MultiDevice
    from tx_util import _synthetic_txlog
    rng = np.random.default_rng(len(devices))
    logs = [_synthetic_txlog(rng, 700, orc, max_entries=16),
            _synthetic_txlog(rng, 500, orc, max_entries=64)]
    bad = bytearray(logs[0])
    for p in rng.integers(0, len(bad), 30):
        bad[int(p)] ^= 0x20
    logs += [bytes(bad), logs[1][:len(logs[1]) * 2 // 3],
             bytes.fromhex(fixtures["long_linear_proof"]["txlog"]), b""]
    # round 6: the parts are validated from the one host parse (no second hop)
    # -- re-encoded metadata in several parts, and a > 16 MiB log whose parts
    # are copied in chunks
    from tx_util import _bulk_txlog, metadata_logs
    nc = b"".join(r for n, r in metadata_logs(orc) if n == "noncanonical_sealed_canonical")
    logs += [nc * 40 + logs[0] + nc * 40, _bulk_txlog(rng, 9000)[0]]
    ctx = m.Context(0)
    md = MultiDevice(devices)
    try:
        for k, raw in enumerate(logs):
            single = m.txlog_validate(raw, ctx=ctx)
            got = md.txlog_validate(raw)
            assert got[:3] == single[:3], (devices, k)
            assert np.array_equal(got[3], single[3]) and np.array_equal(got[4], single[4])
            assert np.array_equal(got[5], single[5]), (devices, k)
            o = orc.txlog_validate(raw)
            assert got[:3] == (o[0], o[1], o[2]) and np.array_equal(got[4], o[3][:got[1]])
            assert list(got[5]) == list(o[4][:got[1]])
    finally:
        md.close()
        ctx.close()


@pytest.mark.parametrize("devices", _SPLIT_DEVICES)
def test_multi_verify_batches_vs_single_and_oracle(m, orc, fixtures, devices):
    """mh_multi_htree_verify_inclusion_batch and
    mh_multi_verify_dual_proof_v2_batch, split by index: the same verdicts as
    one single-context call and the oracle -- 3001 htree proofs over a 5000-leaf
    tree (10 % tampered) and every fixture DualProofV2 case with tampered
    variants (htree.go:166-195, verification.go:303-372)."""
    from immustore_amd import txlayer
    from immustore_amd.multi import MultiDevice
    from tx_util import headers_from_fixture
    rng = np.random.default_rng(3)
    W, n = 5000, 3001
    dig = orc.fill_random(W * 32, 41).reshape(W, 32)
    lv, root = orc.htree_build(dig)
    leaf = rng.integers(0, W, n)
    proofs = [orc.htree_inclusion_proof(lv, W, int(i))[1] for i in leaf]
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(p) for p in proofs])
    terms = np.concatenate(proofs)
    tamper = rng.random(n) < 0.1
    digs = dig[np.where(tamper, (leaf + 1) % W, leaf)]
    roots = np.tile(np.frombuffer(root, np.uint8), (n, 1))
    want = np.array([orc.htree_verify_inclusion(int(leaf[p]), W, proofs[p], digs[p], root)
                     for p in range(n)])
    assert (want == ~tamper).all()
    ctx = m.Context(0)
    md = MultiDevice(devices)
    try:
        ok = md.htree_verify_inclusion_batch(leaf.astype(np.uint64), np.full(n, W, np.uint64), off,
                                             terms, digs, roots)
        assert np.array_equal(ok, want), devices
        for name, fx in fixtures.items():
            recs, blob, alhs = headers_from_fixture(fx["txs"])
            S, T, I, Cn, SA, TA = [], [], [], [], [], []
            for c in fx["dual_v2"]:
                for variant in range(3):
                    ii = [bytes.fromhex(x) for x in c["incl"]]
                    cc = [bytes.fromhex(x) for x in c["cons"]]
                    if variant == 1 and ii:
                        ii[0] = bytes([ii[0][0] ^ 1]) + ii[0][1:]
                    if variant == 2 and cc:
                        cc[-1] = bytes([cc[-1][0] ^ 1]) + cc[-1][1:]
                    S.append(c["src"])
                    T.append(c["tgt"])
                    I.append(ii)
                    Cn.append(cc)
                    SA.append(alhs[c["src"] - 1])
                    TA.append(alhs[c["tgt"] - 1])
            SH = np.array([recs[s - 1] for s in S])
            TH = np.array([recs[t - 1] for t in T])
            single = txlayer.verify_dual_proof_v2_batch(SH, TH, blob, I, Cn, S, T, SA, TA, ctx)
            got = md.verify_dual_proof_v2_batch(SH, TH, blob, I, Cn, S, T, SA, TA)
            assert np.array_equal(got, single), (devices, name)
            exp = [orc.verify_dual_proof_v2(SH[p], TH[p], blob, I[p], Cn[p], S[p], T[p], SA[p], TA[p])
                   for p in range(len(S))]
            assert list(got) == exp, (devices, name)
    finally:
        md.close()
        ctx.close()


@pytest.mark.parametrize("devices", _SPLIT_DEVICES)
def test_multi_values_wire_precommit_vs_single_and_oracle(m, orc, fixtures, devices):
    """mh_multi_verify_values_batch, mh_multi_verify_dual_proof_v2_pb_batch
    and mh_multi_precommit_batch (parts of nearly equal input bytes, one per
    listed device): the same statuses / hashes as one single-context call and
    the oracle -- ragged values with 10 % corrupted and offsets not starting
    at 0 (immustore.go:3235), the fixture stores' device-written DualProofV2
    messages with flipped bytes (verification.go:303-372), and 300 random
    transactions with KV metadata, truncated values and two expected-Eh
    mismatches (immustore.go:1620-1654)."""
    from immustore_amd import txlayer
    from immustore_amd.multi import MultiDevice
    from commit_util import random_batch
    from test_oracle import _values_case
    from tx_util import headers_from_fixture
    ctx = m.Context(0)
    md = MultiDevice(devices)
    try:
        # values
        vb, off, hv, vlen, bad = _values_case(11, 2000)
        pad = np.concatenate([np.zeros(5, np.uint8), vb])
        c, st = md.verify_values(pad, off + np.uint64(5), hv, vlen)
        oc, ost = orc.verify_values(vb, off, hv, vlen)
        assert c == oc == int(bad.sum()) and np.array_equal(st, ost), devices
        c1, st1 = m.verify_values(pad, off + np.uint64(5), hv, vlen, ctx=ctx)
        assert c1 == c and np.array_equal(st1, st)
        # DualProofV2 messages over the wire form
        rng = np.random.default_rng(5)
        for name, fx in fixtures.items():
            pay = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
            t = m.AHtree(ctx)
            try:
                t.append_batch(pay)
                recs, blob, alhs = headers_from_fixture(fx["txs"])
                cases = [(c_["src"], c_["tgt"]) for c_ in fx["dual_v2"] if c_["src"] <= c_["tgt"]]
                S = np.array([a for a, _ in cases], np.uint64)
                T = np.array([b for _, b in cases], np.uint64)
                msgs, _ = t.dual_proof_v2_pb_batch(recs[S.astype(int) - 1], recs[T.astype(int) - 1],
                                                   blob)
            finally:
                t.close()
            msgs = list(msgs)
            for k in range(0, len(msgs), 3):  # every third message with a flipped byte
                b = bytearray(msgs[k])
                b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
                msgs[k] = bytes(b)
            SA = [alhs[int(x) - 1] for x in S]
            TA = [alhs[int(x) - 1] for x in T]
            single = txlayer.verify_dual_proof_v2_pb_batch(msgs, S, T, SA, TA, ctx=ctx)
            got = md.verify_dual_proof_v2_pb_batch(msgs, S, T, SA, TA)
            assert np.array_equal(got, single), (devices, name)
            assert (got[1::3] == 0).all() or len(got) < 2
        # precommit
        for version in (0, 1):
            b = random_batch(np.random.default_rng(40 + version), 300, version=version,
                             md_prob=0.2 if version else 0.0)
            hv_o, eh_o, st_o = orc.precommit_batch(version, **b)
            hv2, eh2, st2 = md.precommit_csr(version, **b)
            assert np.array_equal(st2, st_o) and np.array_equal(eh2, eh_o), (devices, version)
            assert np.array_equal(hv2, hv_o), (devices, version)
            exp = eh_o.copy()
            exp[[7, 250], 1] ^= 0x40
            _, eh3, st3 = md.precommit_csr(version, expect_eh=exp, **b)
            assert sorted(np.nonzero(st3)[0].tolist()) == [7, 250] and np.array_equal(eh3, eh_o)
    finally:
        md.close()
        ctx.close()


@pytest.mark.parametrize("devices", _SPLIT_DEVICES)
def test_multi_verify_document_batch_vs_single_and_oracle(m, orc, devices):
    """mh_multi_verify_document_batch (parts of nearly equal entries +
    document bytes; each part's per-document arrays start past 0, the shared
    entry / byte arrays are indexed through them): the statuses and new-state
    Alh values of one single-context call and of the oracle's VerifyDocument
    (verification.go:37-196) -- 60 documents of 1-700 entries, every third
    with a tampered entry."""
    import struct
    from immustore_amd import txlayer
    from immustore_amd.multi import MultiDevice
    from tx_util import TX_HEADER
    rng = np.random.default_rng(23)
    docs = []
    for k in range(60):
        ne = int(rng.integers(1, 700)) if k % 4 else int(rng.integers(1, 5))
        ents = []
        for e in range(ne):
            key = b"doc/%d/%d" % (k, e)
            md_ = [b"", b"\x00", b"\x02", b"\x01" + struct.pack(">Q", e)][e % 4]
            ents.append((key, md_, bytes(rng.integers(0, 256, 32, dtype=np.uint8))))
        j = int(rng.integers(0, ne))
        doc = bytes(rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8))
        ents[j] = (ents[j][0], ents[j][1], orc.sha256(doc))
        digs = np.frombuffer(b"".join(orc.entry_digest(1, a, b_, c)[1] for a, b_, c in ents),
                             np.uint8).reshape(-1, 32)
        eh = orc.htree_build(digs)[1]
        h = np.zeros(1, TX_HEADER)
        h["id"], h["bl_tx_id"], h["version"], h["nentries"] = 100 + k, 99 + k, 1, ne
        h["eh"] = np.frombuffer(eh, np.uint8)
        h["ts"] = 1_700_000_000 + k
        alh = orc.tx_header_alh(h[0])[2]
        if k % 3 == 2:
            i = (j + 1) % ne
            ents[i] = (ents[i][0], ents[i][1], bytes([ents[i][2][0] ^ 0x80]) + ents[i][2][1:])
        docs.append({"encoded_document": doc, "doc_key": ents[j][0], "tx_hdr": h[0],
                     "entries": ents, "src_hdr": h[0], "tgt_hdr": h[0], "incl": [], "cons": [],
                     "known_tx_id": 100 + k, "known_alh": alh})
    ctx = m.Context(0)
    md = MultiDevice(devices)
    try:
        st1, alh1 = txlayer.verify_document_batch(docs, ctx=ctx)
        st, alh = md.verify_document_batch(docs)
        assert np.array_equal(st, st1) and np.array_equal(alh, alh1), devices
        for k, d in enumerate(docs):
            ost, oalh = orc.verify_document(d)
            assert int(st[k]) == ost, (devices, k)
            assert alh[k].tobytes() == (oalh if ost == 0 else bytes(32))
    finally:
        md.close()
        ctx.close()
