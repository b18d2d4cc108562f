"""GPU parity of the commit path over many transactions (SURVEY.md 8(f) row 1,
mh_precommit_batch): the Go stores' own Eh (tests/golden) and the oracle's
orc_precommit_batch on seeded ragged batches, bit-exact hVals / Eh and the
same per-tx statuses, through the two-stream chunked pipeline (small chunk
sizes force many chunks through both slots)."""
import numpy as np
import pytest

from commit_util import fixture_batch, random_batch

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


@pytest.mark.parametrize("store", ["long_linear_proof", "v110_defaultdb", "v110_systemdb"])
@pytest.mark.parametrize("trunc", [0, 3])
@pytest.mark.parametrize("chunk", [0, 1])
def test_precommit_fixture_stores(m, ctx, fixtures, store, trunc, chunk):
    version, b, eh_ref = fixture_batch(fixtures[store], trunc)
    p = m.CommitPipe(ctx, chunk_bytes=chunk)
    try:
        hv, eh, st = p.precommit_csr(version, **b)
        assert (st == 0).all()
        assert np.array_equal(eh, eh_ref)
        _, _, st2 = p.precommit_csr(version, expect_eh=eh_ref, **b)
        assert (st2 == 0).all()
    finally:
        p.close()


@pytest.mark.parametrize("version", [0, 1])
@pytest.mark.parametrize("chunk", [1 << 10, 1 << 16, 0])
def test_precommit_random_vs_oracle(m, ctx, orc, version, chunk):
    rng = np.random.default_rng(100 + version * 7 + chunk % 97)
    b = random_batch(rng, 300, version=version, md_prob=0.2 if version else 0.0)
    hv_o, eh_o, st_o = orc.precommit_batch(version, **b)
    p = m.CommitPipe(ctx, chunk_bytes=chunk)
    try:
        hv, eh, st = p.precommit_csr(version, **b)
        assert np.array_equal(st, st_o)
        assert np.array_equal(eh, eh_o)
        assert np.array_equal(hv, hv_o)
        # the same pipe again (buffers reused), with an expected-Eh mismatch
        bad = eh_o.copy()
        bad[[3, 150], 0] ^= 0x80
        _, eh2, st2 = p.precommit_csr(version, expect_eh=bad, **b)
        assert sorted(np.nonzero(st2)[0].tolist()) == [3, 150] and (st2[[3, 150]] == 2).all()
        assert np.array_equal(eh2, eh_o)
    finally:
        p.close()


@pytest.mark.parametrize("max_entries", [64, 65, 300, 1024])
def test_precommit_tree_paths_vs_oracle(m, ctx, orc, max_entries):
    """Chunks whose widest tx has <= 64 entries get one-lane-per-tree roots,
    wider ones the host tree plan (both within one batch when chunks differ)."""
    rng = np.random.default_rng(max_entries)
    b = random_batch(rng, 60, version=1, max_entries=max_entries, vlens=(0, 33, 100))
    hv_o, eh_o, st_o = orc.precommit_batch(1, **b)
    for chunk in (1 << 12, 0):
        p = m.CommitPipe(ctx, chunk_bytes=chunk)
        try:
            hv, eh, st = p.precommit_csr(1, **b)
        finally:
            p.close()
        assert np.array_equal(st, st_o) and np.array_equal(eh, eh_o)
        assert np.array_equal(hv, hv_o)


def test_precommit_max_sizes_vs_oracle(m, ctx, orc):
    """The reference's limits (options.go:35-39): MaxTxEntries 1024 entries in
    one tx, keys up to MaxKeyLen 1024 and values up to MaxValueLen 4096 bytes,
    KV metadata up to 11 bytes, truncated values among them."""
    rng = np.random.default_rng(1024)
    b = random_batch(rng, 24, version=1, max_entries=1024, md_prob=0.5, trunc_prob=0.2,
                     vlens=(0, 1, 63, 64, 4031, 4032, 4095, 4096),
                     klens=(1, 55, 56, 119, 120, 1000, 1023, 1024))
    hv_o, eh_o, st_o = orc.precommit_batch(1, **b)
    assert (st_o == 0).all()
    p = m.CommitPipe(ctx)
    try:
        hv, eh, st = p.precommit_csr(1, **b)
        assert np.array_equal(st, st_o) and np.array_equal(eh, eh_o)
        assert np.array_equal(hv, hv_o)
    finally:
        p.close()


def test_precommit_statuses_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(5)
    b = random_batch(rng, 120, version=1, md_prob=0.3)
    p = m.CommitPipe(ctx, chunk_bytes=1 << 12)
    try:
        for version, mw in ((1, 16), (0, 0), (0, 25)):
            hv_o, eh_o, st_o = orc.precommit_batch(version, max_width=mw, **b)
            hv, eh, st = p.precommit_csr(version, max_width=mw, **b)
            assert np.array_equal(st, st_o), (version, mw)
            assert np.array_equal(eh, eh_o), (version, mw)
            ok = np.repeat(st_o == 0, np.diff(b["tx_off"].astype(np.int64)))
            assert np.array_equal(hv[ok], hv_o[ok])
    finally:
        p.close()


def test_precommit_entryspec_api(m, ctx, orc):
    """The EntrySpec-list mirror; empty txs give SHA256(nil) (htree.go:73-77)."""
    E = m.EntrySpec
    txs = [[E(b"k1", b"v1"), E(b"k2", b"", md=b"\x00\x01"), E(b"k3", hash_value=b"\x11" * 32)],
           [],
           [E(b"key", b"x" * 5000)]]
    p = m.CommitPipe(ctx)
    try:
        hvs, eh, st = p.precommit(1, txs)
    finally:
        p.close()
    assert (st == 0).all()
    import hashlib
    assert eh[1].tobytes() == hashlib.sha256(b"").digest()
    for t, es in enumerate(txs):
        s, hv, _, root = orc.build_entries(1, [e.key for e in es], [e.md for e in es],
                                           [e.value for e in es],
                                           [e.hash_value for e in es])
        assert s == 0 and root == eh[t].tobytes()
        assert np.array_equal(hv, hvs[t])


def test_precommit_large_batch_pinned(m, ctx, orc):
    """~96 MiB of values in pinned host memory through 64 MiB chunks: both
    slots busy, results identical to the oracle (4 host threads)."""
    import torch
    ntx, per, vlen = 3072, 32, 1024
    n = ntx * per
    vals = torch.empty(n * vlen, dtype=torch.uint8).pin_memory()
    vals.copy_(torch.randint(0, 256, (n * vlen,), dtype=torch.uint8,
                             generator=torch.Generator().manual_seed(9)))
    keys = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).copy()
    b = dict(tx_off=np.arange(0, n + 1, per, dtype=np.uint64), keys=keys,
             key_off=np.arange(0, 8 * n + 1, 8, dtype=np.uint64), vals=vals.numpy(),
             val_off=np.arange(0, vlen * n + 1, vlen, dtype=np.uint64))
    hv_o, eh_o, st_o = orc.precommit_batch(1, nthreads=4, **b)
    p = m.CommitPipe(ctx)
    try:
        hv, eh, st = p.precommit_csr(1, **b)
    finally:
        p.close()
    assert (st == 0).all() and (st_o == 0).all()
    assert np.array_equal(eh, eh_o) and np.array_equal(hv, hv_o)


def test_commit_queue_30_threads_vs_oracle(m, ctx, orc):
    """Group commit (mh_commit_queue): 30 threads -- MaxConcurrency
    (options.go:35) -- each submit single 16-entry transactions
    (immustore.go:1620-1632) with 1 KiB values, KV metadata, truncated values
    and ReplicateTx Eh checks mixed in; every tx's hVals, Eh and status equal
    the oracle's, and the queue really coalesced them into fewer batches."""
    import threading
    from immustore_amd.commit import CommitQueue, EntrySpec
    q = CommitQueue(ctx, version=1, max_width=24, max_txs=64, wait_us=100)
    rng = np.random.default_rng(30)
    per_thread = 12
    txs = []
    for k in range(30 * per_thread):
        ne = 16 if k % 7 else int(rng.integers(0, 30))  # some empty / over max_width
        es = []
        for e in range(ne):
            key = b"k/%d/%d" % (k, e)
            val = bytes(rng.integers(0, 256, 1024 if e % 5 else int(rng.integers(0, 3000)),
                                     dtype=np.uint8))
            md = [b"", b"", b"\x00", b"\x01" + bytes(8)][e % 4]
            hv = orc.sha256(val + b"!") if (k + e) % 11 == 0 else None
            es.append(EntrySpec(key, val, md, hv))
        txs.append(es)
    exp = []
    for k, es in enumerate(txs):
        ovs = [e.hash_value for e in es]
        st, hv, _, root = orc.build_entries(1, [e.key for e in es], [e.md for e in es],
                                            [e.value for e in es], ovs)
        if len(es) > 24:
            st, root = 1, None
        exp.append((st, hv, root))
    out = [None] * len(txs)

    def run(t):
        for k in range(t, len(txs), 30):
            want = exp[k][2] if (k % 13 == 0 and exp[k][0] == 0) else None
            if want is not None and k % 26 == 0:
                want = bytes([want[0] ^ 1]) + want[1:]  # a replicated tx whose Eh differs
            out[k] = (q.submit(txs[k], expect_eh=want), want)

    ths = [threading.Thread(target=run, args=(t,)) for t in range(30)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for k, ((st, hv, eh), want) in enumerate(out):
        est, ehv, eroot = exp[k]
        if est == 1:
            assert st == 1, k  # MH_ERR_MAX_WIDTH_EXCEEDED
            continue
        assert np.array_equal(hv, ehv.reshape(-1, 32)), k
        assert eh == eroot, k
        if want is not None and want != eroot:
            assert st == 2, k  # "entries hash (Eh) differs"
        else:
            assert st == 0, k
    batches, n = q.stats()
    assert n == len(txs) and batches < n
    q.close()


def test_commit_queue_small_batches_and_large_txs(m, ctx, orc):
    """Committers copy their own txs into the open batch's arena and their
    results out of it: max_txs 4 under 12 threads (several batches in flight
    over the two workers, arenas reused as soon as every committer has read),
    and txs larger than the default arena (5000 entries; a 20 MiB value; 2 MiB
    of keys) that open a batch of their own -- every result equal to the
    oracle's."""
    import threading
    from immustore_amd.commit import CommitQueue, EntrySpec
    q = CommitQueue(ctx, version=1, max_width=0, max_txs=4, wait_us=30)
    rng = np.random.default_rng(31)
    txs = []
    for k in range(96):
        if k == 17:
            es = [EntrySpec(b"w%d" % e, bytes([e % 251]) * 8) for e in range(5000)]
        elif k == 40:
            es = [EntrySpec(b"big", orc.fill_random(20 << 20, 3).tobytes(), b"\x02")]
        elif k == 63:
            es = [EntrySpec(bytes([e % 256, e // 256]) * 500, b"v") for e in range(2100)]
        else:
            es = [EntrySpec(b"k%d/%d" % (k, e), bytes(rng.integers(0, 256, int(rng.integers(0, 2000)),
                                                                    dtype=np.uint8)),
                            [b"", b"\x00"][e % 2]) for e in range(int(rng.integers(0, 9)))]
        txs.append(es)
    out = [None] * len(txs)

    def run(t):
        for k in range(t, len(txs), 12):
            out[k] = q.submit(txs[k])

    ths = [threading.Thread(target=run, args=(t,)) for t in range(12)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for k, es in enumerate(txs):
        st, hv, eh = out[k]
        s2, ehv, _, root = orc.build_entries(1, [e.key for e in es], [e.md for e in es],
                                             [e.value for e in es])
        assert st == 0 and eh == root, k
        assert np.array_equal(hv, ehv.reshape(-1, 32)), k
    batches, n = q.stats()
    assert n == len(txs) and batches >= len(txs) // 4
    q.close()


def test_commit_queue_v0_metadata_and_free(m, ctx, orc):
    from immustore_amd.commit import CommitQueue, EntrySpec
    q = CommitQueue(ctx, version=0)
    st, hv, eh = q.submit([EntrySpec(b"a", b"x", b"\x00")])
    assert st == 6  # MH_ERR_METADATA_UNSUPPORTED (tx.go:691-693)
    st, hv, eh = q.submit([EntrySpec(b"a", b"x"), EntrySpec(b"bb", b"")])
    s2, hv2, _, root = orc.build_entries(0, [b"a", b"bb"], [b"", b""], [b"x", b""])
    assert st == 0 and eh == root and np.array_equal(hv, hv2.reshape(-1, 32))
    st, hv, eh = q.submit([])
    assert st == 0 and eh == orc.sha256(b"")
    q.close()
