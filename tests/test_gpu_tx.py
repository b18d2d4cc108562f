"""GPU parity of the tx layer (SURVEY.md 8(a) a7, a13, a14 and a3 over many
trees) through the C ABI, against the reference's Go-written stores
(tests/golden/immudb_fixtures.json: raw tx logs, stored Alh, DualProofV2 and
linear proofs built from the stores' own dLog) and the oracle on synthetic
logs.  Bit-exact digests and identical statuses.
"""
import struct

import numpy as np
import pytest

from tx_util import _bulk_txlog, _synthetic_txlog, headers_from_fixture

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


def test_tx_alh_batch_fixture_headers(m, ctx, fixtures):
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        inner, alh = m.tx_alh_batch(recs, blob, ctx)
        assert [a.tobytes() for a in alh] == alhs, name


def test_tx_alh_batch_synthetic_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(7)
    n = 3000
    recs = np.zeros(n, m.TX_HEADER)
    blob = bytearray()
    for k in range(n):
        r = recs[k]
        r["id"] = int(rng.integers(1, 1 << 62))
        r["ts"] = int(rng.integers(-(1 << 62), 1 << 62))
        r["bl_tx_id"] = int(rng.integers(0, 1 << 62))
        for f in ("bl_root", "prev_alh", "eh"):
            r[f] = rng.integers(0, 256, 32, dtype=np.uint8)
        r["version"] = k % 2
        r["nentries"] = int(rng.integers(0, 1 << 31))
        if r["version"] == 1:
            ml = [0, 1, 9, 12, 100, 268][k % 6]
            r["md_len"], r["md_off"] = ml, len(blob)
            blob += rng.integers(0, 256, ml, dtype=np.uint8).tobytes()
        else:
            r["nentries"] &= 0xFFFF
    inner, alh = m.tx_alh_batch(recs, bytes(blob), ctx)
    for k in range(0, n, 7):
        st, oi, oa = orc.tx_header_alh(recs[k], bytes(blob))
        assert st == 0 and inner[k].tobytes() == oi and alh[k].tobytes() == oa, k
    bad = recs[:2].copy()
    bad[0]["version"] = 2
    with pytest.raises(m.ErrIllegalArguments):
        m.tx_alh_batch(bad, bytes(blob), ctx)
    bad = recs[:2].copy()
    bad[0]["version"], bad[0]["md_len"] = 0, 3
    with pytest.raises(m.ErrMetadataUnsupported):
        m.tx_alh_batch(bad, bytes(blob), ctx)


def test_htree_build_many_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(8)
    widths = [0, 1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 31, 33, 100, 1000, 1024, 1025, 1, 1, 0, 2] + \
        list(rng.integers(1, 300, 400))
    trees = [rng.integers(0, 256, (w, 32), dtype=np.uint8) for w in widths]
    roots = m.htree_build_many(trees, ctx)
    for t, r in zip(trees, roots):
        assert r.tobytes() == orc.htree_build(t)[1]
    # every width <= 64: the one-lane-per-tree kernel instead of the host plan
    small = [t for t in trees if len(t) <= 64] + [rng.integers(0, 256, (64, 32), dtype=np.uint8)]
    roots = m.htree_build_many(small, ctx)
    for t, r in zip(small, roots):
        assert r.tobytes() == orc.htree_build(t)[1]
    # every shape class of the many-tree dispatch (small_roots_fit): few trees
    # up to 64 wide (a wave per tree), many trees up to 16 wide (a lane per
    # tree), many trees of 17..64 (level-parallel through the plan)
    for count, lo, hi in ((2048, 1, 65), (3000, 1, 17), (3000, 17, 65), (2049, 60, 65)):
        ts = [rng.integers(0, 256, (int(w), 32), dtype=np.uint8)
              for w in rng.integers(lo, hi, count)]
        roots = m.htree_build_many(ts, ctx)
        for t, r in zip(ts, roots):
            assert r.tobytes() == orc.htree_build(t)[1], (count, lo, hi, len(t))


def test_txlog_validate_fixture_stores(m, ctx, fixtures):
    for name, fx in fixtures.items():
        raw = bytes.fromhex(fx["txlog"])
        rc, n, used, hdrs, alh, sts = m.txlog_validate(raw, ctx=ctx)
        assert rc == 0 and n == len(fx["txs"]) and used <= len(raw)
        assert list(sts) == [0] * n
        assert [a.tobytes().hex() for a in alh] == [t["header"]["alh"] for t in fx["txs"]]
        assert [h["eh"].tobytes().hex() for h in hdrs] == [t["header"]["eh"] for t in fx["txs"]]
        assert [int(h["id"]) for h in hdrs] == [t["header"]["id"] for t in fx["txs"]]


def test_txlog_validate_synthetic_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(11)
    raw = _synthetic_txlog(rng, 300, orc)
    rc, n, used, hdrs, alh, sts = m.txlog_validate(raw, ctx=ctx)
    o = orc.txlog_validate(raw)
    assert (rc, n, used) == (o[0], o[1], o[2]) == (0, 300, len(raw))
    assert np.array_equal(alh, o[3]) and list(sts) == list(o[4]) == [0] * 300
    # corrupt a few hVals / stored alhs / a header field: per-tx statuses match
    bad = bytearray(raw)
    rng2 = np.random.default_rng(3)
    for pos in rng2.integers(0, len(raw), 40):
        bad[int(pos)] ^= 0x10
    r1 = m.txlog_validate(bytes(bad), ctx=ctx)
    r2 = orc.txlog_validate(bytes(bad))
    assert (r1[0], r1[1], r1[2]) == (r2[0], r2[1], r2[2])
    assert list(r1[5]) == list(r2[4])
    assert np.array_equal(r1[4], r2[3])
    # structural errors and limits agree
    for kw in ({"max_entries": 5}, {"max_key_len": 10}, {"max_txs": 17}):
        a = m.txlog_validate(raw, ctx=ctx, **kw)
        b = orc.txlog_validate(raw, **kw)
        assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]) and list(a[5]) == list(b[4]), kw
    for cut in (1, 50, 91, len(raw) // 2, len(raw) - 1):
        a = m.txlog_validate(raw[:cut], ctx=ctx)
        b = orc.txlog_validate(raw[:cut])
        assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]), cut


def test_txlog_validate_v0_entry_with_kv_metadata(m, ctx, orc):
    """a v0 record whose entry carries KV metadata fails the
    read with ErrMetadataUnsupported (tx.go:690-693); validation stops there
    with the records before it validated, as in the oracle."""
    import struct
    rng = np.random.default_rng(12)
    good = _synthetic_txlog(rng, 9, orc, version_mix=False)
    for md in (b"\x00", b"\x02", b"\x00\x02"):
        ent = struct.pack(">H", len(md)) + md + struct.pack(">H", 4) + b"keyz"
        ent += struct.pack(">IQ", 5, 9) + bytes(32)
        rec = struct.pack(">QQQ", 10, 1, 0) + bytes(64) + struct.pack(">HH", 0, 1) + ent + bytes(32)
        a = m.txlog_validate(good + rec, ctx=ctx)
        b = orc.txlog_validate(good + rec)
        assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]) == (6, 9, len(good))
        assert list(a[5]) == list(b[4]) == [0] * 9 and np.array_equal(a[4], b[3])


def test_txlog_validate_message_lengths(m, ctx, orc):
    """Entry-digest messages hashed in place from the raw records
    (k_txe_leaf): every key length 0..140 (all padding remainders, one-, two-
    and three-block messages, each byte alignment) and keys up to the 1024-byte
    limit, v0 and v1 with every KV-metadata shape."""
    rng = np.random.default_rng(77)
    lens = list(range(141)) + [255, 256, 511, 1000, 1019, 1020, 1021, 1022, 1023, 1024]
    raw = _synthetic_txlog(rng, 200, orc, max_entries=12,
                           key_len=lambda k, e: lens[(k * 12 + e) % len(lens)])
    rc, n, used, hdrs, alh, sts = m.txlog_validate(raw, ctx=ctx)
    o = orc.txlog_validate(raw)
    assert (rc, n, used) == (o[0], o[1], o[2]) == (0, 200, len(raw))
    assert np.array_equal(alh, o[3]) and list(sts) == [0] * 200


@pytest.mark.parametrize("max_entries", [64, 65, 300, 1024])
def test_txlog_validate_tree_paths(m, ctx, orc, max_entries):
    """Batches whose widest tx has <= 64 entries take the one-lane-per-tree
    root kernel, wider ones the host tree plan: both agree with the oracle."""
    rng = np.random.default_rng(max_entries)
    raw = _synthetic_txlog(rng, 60, orc, max_entries=max_entries)
    rc, n, used, hdrs, alh, sts = m.txlog_validate(raw, ctx=ctx)
    o = orc.txlog_validate(raw)
    assert (rc, n, used) == (o[0], o[1], o[2]) == (0, 60, len(raw))
    assert np.array_equal(alh, o[3]) and list(sts) == [0] * 60


def test_txlog_validate_parallel_hop(m, ctx, orc):
    """The multi-threaded record hop equals the sequential parse (the oracle)
    on a ~20 MB log: clean, with a structural error deep inside, cut short,
    with a zeroed (preallocated) tail and with max_txs inside a chunk."""
    rng = np.random.default_rng(77)
    raw, starts = _bulk_txlog(rng, 9000)
    assert len(raw) > (8 << 20)

    def same(buf, **kw):
        a = m.txlog_validate(buf, ctx=ctx, **kw)
        b = orc.txlog_validate(buf, **kw)
        assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]), kw
        assert list(a[5]) == list(b[4]) and np.array_equal(a[4], b[3])
        return a

    a = same(raw)
    assert (a[0], a[1], a[2]) == (0, 9000, len(raw))
    bad = bytearray(raw)
    bad[starts[6543] + 89] = 7  # unknown header version
    a = same(bytes(bad))
    assert (a[0], a[1], a[2]) == (17, 6543, starts[6543])
    same(raw[:len(raw) - 100])
    same(raw[:starts[5000]] + bytes(3 << 20))
    same(raw, max_txs=4321)


def _chunk_cuts(n, weights=(5, 2, 1)):
    """mh_txlog_validate's copy chunks of a pinned n-byte log (from 16 MiB,
    sizes 5 : 2 : 1 by default, cut at 4 KiB multiples)."""
    tot, pre, cuts = float(sum(weights)), 0.0, []
    for w in weights[:-1]:
        pre += w
        cuts.append(max(cuts[-1] if cuts else 0, int(float(n) * pre / tot) & ~4095))
    return cuts


@pytest.mark.parametrize("weights", [None, "4:2:1:1"])
def test_txlog_validate_chunk_phases(m, ctx, orc, monkeypatch, weights):
    """From 16 MiB the log goes up in copy chunks (5 : 2 : 1 by default, and
    round 4's 4 : 2 : 1 : 1 through MH_TXLOG_WEIGHTS) and the hop runs in one
    phase per chunk (the records ending inside a chunk are validated while the
    rest is copied and parsed): errors on either side of every cut and in the
    records that straddle them, max_txs at a cut, a cut short of a record,
    non-canonical metadata (patched records) and wide txs (tree plan) in the
    first or the last chunk -- all equal to the one-pass oracle."""
    from tx_util import metadata_logs
    if weights:
        monkeypatch.setenv("MH_TXLOG_WEIGHTS", weights)
    wts = tuple(int(x) for x in weights.split(":")) if weights else (5, 2, 1)
    rng = np.random.default_rng(5)
    raw, starts = _bulk_txlog(rng, 9000)
    assert len(raw) >= (16 << 20)

    def same(buf, **kw):
        a = m.txlog_validate(buf, ctx=ctx, **kw)
        b = orc.txlog_validate(buf, **kw)
        assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]), kw
        assert list(a[5]) == list(b[4]) and np.array_equal(a[4], b[3]), kw
        return a

    for cut in _chunk_cuts(len(raw), wts):
        j = max(k for k in range(len(starts)) if starts[k] < cut)  # straddles the cut
        for k in (j - 1, j, j + 1):
            bad = bytearray(raw)
            bad[starts[k] + 89] = 7  # unknown header version
            a = same(bytes(bad))
            assert (a[0], a[1], a[2]) == (17, k, starts[k])
        bad = bytearray(raw)  # hVal of the straddling record's last entry
        bad[starts[j + 1] - 33] ^= 1
        same(bytes(bad))
        for mt in (j - 1, j, j + 1):
            a = same(raw, max_txs=mt)
            assert a[1] == mt
    cut = _chunk_cuts(len(raw), wts)[0]
    j = max(k for k in range(len(starts)) if starts[k] < cut)
    same(raw[:starts[j + 1]] + bytes(len(raw) - starts[j + 1]))  # zero tail from the first cut
    same(raw[:len(raw) - 5])
    # patched records / wide txs at the start or the end
    md = b"".join(r for name, r in metadata_logs(orc) if name == "noncanonical_sealed_canonical")
    same(raw + md * 50)
    same(md * 50 + raw)
    wide = _synthetic_txlog(rng, 20, orc, max_entries=300)
    same(raw + wide)
    same(wide + raw)


def test_txlog_validate_chunked_mutants(m, ctx, orc):
    """Random damage to a ~24 MiB log (chunked copy, one hop phase per chunk):
    byte flips anywhere, bursts of zeros, a cut at a random length -- status,
    count, consumed bytes, every Alh and per-tx status equal to the oracle's
    one-pass parse, with pageable and with pinned outputs."""
    import torch
    from immustore_amd.txlayer import TX_HEADER
    rng = np.random.default_rng(21)
    raw, starts = _bulk_txlog(rng, 11000)
    assert len(raw) >= (16 << 20)
    cap = 11100
    outs = (torch.empty(cap * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER),
            torch.empty(cap * 32, dtype=torch.uint8).pin_memory().numpy().reshape(cap, 32),
            torch.empty(cap, dtype=torch.int32).pin_memory().numpy())
    for case in range(24):
        b = bytearray(raw)
        kind = case % 3
        if kind == 0:
            for p in rng.integers(0, len(b), int(rng.integers(1, 40))):
                b[int(p)] ^= int(rng.integers(1, 256))
        elif kind == 1:
            p = int(rng.integers(0, len(b) - 4096))
            w = int(rng.integers(8, 4096))
            b[p:p + w] = bytes(w)
        else:
            b = b[:int(rng.integers(len(b) // 2, len(b)))]
        buf = bytes(b)
        o = orc.txlog_validate(buf)
        for out in (None, outs):
            a = m.txlog_validate(buf, ctx=ctx, out=out)
            assert (a[0], a[1], a[2]) == (o[0], o[1], o[2]), (case, out is None)
            assert np.array_equal(a[4], o[3]) and list(a[5]) == list(o[4]), (case, out is None)


@pytest.mark.parametrize("hdrs", [True, False])
def test_txlog_validate_pinned_buffers(m, ctx, orc, hdrs):
    """The log and the outputs in pinned host memory (as the cgo shim's arena
    holds them): the index arrays go up and the results come down by kernel
    loads / stores over PCIe instead of DMA copies.  Equal to the oracle and
    to the pageable call, for a clean log, one with corrupted records in every
    copy chunk, and an output arena larger than the result."""
    import torch
    from immustore_amd.txlayer import TX_HEADER
    rng = np.random.default_rng(8)
    raw, starts = _bulk_txlog(rng, 9000)
    bad = bytearray(raw)
    for k in (3, 2500, 4700, 7000, 8999):
        bad[starts[k] + 100] ^= 1  # inside the record: an Alh mismatch
    for buf in (raw, bytes(bad)):
        pin = torch.empty(len(buf), dtype=torch.uint8).pin_memory()
        pin.numpy()[:] = np.frombuffer(buf, np.uint8)
        cap = 9100
        outs = (torch.empty(cap * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy()
                .view(TX_HEADER) if hdrs else None,
                torch.empty(cap * 32, dtype=torch.uint8).pin_memory().numpy().reshape(cap, 32),
                torch.empty(cap, dtype=torch.int32).pin_memory().numpy())
        a = m.txlog_validate(pin.numpy(), ctx=ctx, out=outs)
        b = orc.txlog_validate(buf)
        c = m.txlog_validate(buf, ctx=ctx)
        assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]) == (c[0], c[1], c[2])
        assert np.array_equal(a[4], b[3]) and list(a[5]) == list(b[4])
        if hdrs:
            assert np.array_equal(a[3], c[3])


def test_txlog_validate_pinned_last_chunk(m, ctx, orc):
    """The last copy chunk of a pinned log (its group's kernel runs right
    after it lands and stores the results into the pinned outputs itself; the
    header fields other than Eh are filled by the host meanwhile): ends that
    are not 16-byte multiples, errors / max_txs / a corrupted hVal inside the
    last chunk, and a wide tx or re-encoded metadata at the end (the
    rest-group path) -- equal to the oracle and to the pageable call, headers
    included."""
    import torch
    from tx_util import metadata_logs
    from immustore_amd.txlayer import TX_HEADER
    rng = np.random.default_rng(31)
    raw, starts = _bulk_txlog(rng, 9500)
    assert len(raw) >= (16 << 20)
    last_cut = _chunk_cuts(len(raw))[-1]
    late = [k for k in range(len(starts)) if starts[k] > last_cut + 4096]
    assert len(late) > 50
    cap = 20000
    outs = (torch.empty(cap * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER),
            torch.empty(cap * 32, dtype=torch.uint8).pin_memory().numpy().reshape(cap, 32),
            torch.empty(cap, dtype=torch.int32).pin_memory().numpy())

    def same(buf, **kw):
        pin = torch.empty(len(buf), dtype=torch.uint8).pin_memory()
        pin.numpy()[:] = np.frombuffer(buf, np.uint8)
        a = m.txlog_validate(pin.numpy(), ctx=ctx, out=outs, **kw)
        b = orc.txlog_validate(buf, **kw)
        c = m.txlog_validate(buf, ctx=ctx, **kw)
        assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]) == (c[0], c[1], c[2]), kw
        assert np.array_equal(a[4], b[3]) and list(a[5]) == list(b[4]), kw
        assert np.array_equal(a[3], c[3]), kw
        return a

    same(raw)
    odd = [k for k in late if starts[k] % 16][-1]
    a = same(raw[:starts[odd]])  # ends mid 16-byte piece
    assert a[1] == odd
    k = late[len(late) // 2]
    bad = bytearray(raw)
    bad[starts[k] + 89] = 7  # unknown header version inside the last chunk
    a = same(bytes(bad))
    assert (a[0], a[1], a[2]) == (17, k, starts[k])
    bad = bytearray(raw)
    bad[starts[k + 1] - 33] ^= 1  # the last hVal of record k
    a = same(bytes(bad))
    same(raw, max_txs=k)
    same(raw[:len(raw) - 7])
    md = b"".join(r for name, r in metadata_logs(orc) if name == "noncanonical_sealed_canonical")
    same(raw + md * 50)
    same(raw + _synthetic_txlog(rng, 20, orc, max_entries=300))


def test_dual_proof_v2_fixture_cases(m, ctx, orc, fixtures):
    seen = set()
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        S, T, I, Cn, SA, TA, exp = [], [], [], [], [], [], []

        def add(s, t, incl, cons, sa, ta, sh=None, th=None):
            S.append(s)
            T.append(t)
            I.append(incl)
            Cn.append(cons)
            SA.append(sa)
            TA.append(ta)
            sh_ = recs[s - 1] if sh is None else sh
            th_ = recs[t - 1] if th is None else th
            exp.append(orc.verify_dual_proof_v2(sh_, th_, blob, incl, cons, s, t, sa, ta))
            return sh_, th_

        SH, TH = [], []
        for c in fx["dual_v2"]:
            s, t = c["src"], c["tgt"]
            incl = [bytes.fromhex(x) for x in c["incl"]]
            cons = [bytes.fromhex(x) for x in c["cons"]]
            for variant in range(4):
                ii, cc, sa = list(incl), list(cons), alhs[s - 1]
                if variant == 1 and ii:
                    ii[0] = bytes([ii[0][0] ^ 1]) + ii[0][1:]
                if variant == 2 and cc:
                    cc[-1] = bytes([cc[-1][0] ^ 1]) + cc[-1][1:]
                if variant == 3:
                    sa = bytes(32)
                a, b = add(s, t, ii, cc, sa, alhs[t - 1])
                SH.append(a)
                TH.append(b)
        st = m.verify_dual_proof_v2_batch(np.array(SH), np.array(TH), blob, I, Cn, S, T, SA, TA,
                                          ctx)
        assert list(st) == exp, name
        seen |= set(exp)
    assert {0, 2, 12, 13} <= seen
    # Go-shaped wrapper raises the Go error
    fx = fixtures["long_linear_proof"]
    recs, blob, alhs = headers_from_fixture(fx["txs"])
    c = [x for x in fx["dual_v2"] if x["src"] < x["tgt"]][0]
    s, t = c["src"], c["tgt"]
    incl = [bytes.fromhex(x) for x in c["incl"]]
    cons = [bytes.fromhex(x) for x in c["cons"]]
    m.VerifyDualProofV2(recs[s - 1], recs[t - 1], blob, incl, cons, s, t, alhs[s - 1],
                        alhs[t - 1], ctx)
    with pytest.raises(m._native.ErrSourceTxNewerThanTargetTx):
        m.VerifyDualProofV2(recs[t - 1], recs[s - 1], blob, incl, cons, t, s, alhs[t - 1],
                            alhs[s - 1], ctx)


def test_linear_proofs_fixture_and_random(m, ctx, orc, fixtures):
    items, exp = [], []
    for name, fx in fixtures.items():
        alhs = [bytes.fromhex(t["header"]["alh"]) for t in fx["txs"]]
        for c in fx["linear"]:
            s, t = c["src"], c["tgt"]
            terms = [bytes.fromhex(x) for x in c["terms"]]
            for v in range(3):
                tt = list(terms)
                tgt = t
                if v == 1 and len(tt) > 1:
                    tt[-1] = bytes([tt[-1][0] ^ 2]) + tt[-1][1:]
                if v == 2:
                    tgt = t + 1
                items.append((s, t, tt, s, tgt, alhs[s - 1], alhs[t - 1]))
                exp.append(orc.verify_linear_proof(s, t, tt, s, tgt, alhs[s - 1], alhs[t - 1]))
    z = bytes(32)
    for it in [(0, 1, [z], 0, 1, z, z), (2, 1, [z], 2, 1, z, z), (1, 1, [], 1, 1, z, z),
               (1, 1, [z], 1, 1, z, z)]:
        items.append(it)
        exp.append(orc.verify_linear_proof(*it))
    got = m.verify_linear_proof_batch(items, ctx)
    assert list(got) == exp
    assert any(exp) and not all(exp)


def test_dual_proof_v1_fixture_cases(m, ctx, orc, fixtures):
    from test_tx_oracle import dual_v1_args
    cols = [[] for _ in range(13)]
    exp = []
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        assert blob == b""  # all fixture headers carry no tx metadata: one shared blob
        for c in fx["dual_v1"]:
            for tamper in (None, "lap", "lin", "last", "tbl"):
                a = dual_v1_args(c, recs, blob, alhs, tamper)
                exp.append(orc.verify_dual_proof(*a))
                for i, v in enumerate(a):
                    cols[i].append(v)
    got = m.verify_dual_proof_batch(np.array(cols[0]), np.array(cols[1]), b"", cols[3], cols[4],
                                    cols[5], cols[6], cols[7], cols[8], cols[9], cols[10],
                                    cols[11], cols[12], ctx)
    assert list(got) == exp
    assert sum(exp) > 400 and not all(exp)


def test_verify_document_batch_vs_oracle(m, ctx, orc, fixtures):
    """pkg/verification.VerifyDocument (verification.go:37-196), hashing part,
    on the device for every document case built from the Go-written stores
    (tests/tx_util.document_cases: untampered and 12 tampered variants each)
    -- per-document status and new-state Alh equal the oracle's."""
    from immustore_amd import txlayer
    from tx_util import document_cases
    docs, blob = document_cases(fixtures, orc)
    docs[0]["md_blob"] = blob
    st, alh = txlayer.verify_document_batch(docs, ctx=ctx)
    for k, d in enumerate(docs):
        ost, oalh = orc.verify_document(d, blob)
        assert int(st[k]) == ost, (k, k % 13)
        assert alh[k].tobytes() == (oalh if ost == 0 else bytes(32)), k
    assert (st == 0).sum() >= 40


@pytest.mark.parametrize("pinned", [True, "arena"])
def test_verify_document_batch_pinned_and_arena(m, ctx, orc, fixtures, pinned):
    """The same document cases packed in pinned memory, one allocation per
    array or every array in ONE pinned allocation (the shim's arena: one
    upload of the whole span, each array addressed inside it) -- per-document
    status and Alh equal to the oracle and to the pageable call."""
    from immustore_amd import txlayer
    from tx_util import document_cases
    docs, blob = document_cases(fixtures, orc)
    docs[0]["md_blob"] = blob
    ref = txlayer.verify_document_batch(docs, ctx=ctx)
    b, keep = txlayer.pack_document_batch(docs, pinned=pinned)
    ctx.timing_reset()
    ctx.set_timing(True)
    st, alh = txlayer.call_document_batch(b, len(docs), ctx)
    ctx.set_timing(False)
    assert np.array_equal(st, ref[0]) and np.array_equal(alh, ref[1])
    # one upload of the arena's span only when every array is inside ONE
    # pinned allocation; separately pinned arrays (adjacent or not) go one
    # copy per array, never one span across allocations
    n_arena, n_arrays = ctx.timing("doc_upload_arena")[1], ctx.timing("doc_upload_arrays")[1]
    assert (n_arena > 0 and n_arrays == 0) if pinned == "arena" else (n_arena == 0 and n_arrays > 0), \
        (pinned, n_arena, n_arrays)
    for k, d in enumerate(docs):
        ost, oalh = orc.verify_document(d, blob)
        assert int(st[k]) == ost, k
        assert alh[k].tobytes() == (oalh if ost == 0 else bytes(32)), k
    del keep


def test_verify_document_batch_offsets_running_backwards(m, ctx, orc, fixtures):
    """Offsets that run backwards (document, key, entry and proof-term CSR)
    are rejected with ErrIllegalArguments before anything is read through
    them; restored, the same batch verifies."""
    import ctypes as C
    from immustore_amd import _native as N
    from immustore_amd import txlayer
    from tx_util import document_cases
    docs, blob = document_cases(fixtures, orc)
    docs = docs[:13]
    docs[0]["md_blob"] = blob
    b, keep = txlayer.pack_document_batch(docs)
    n = len(docs)
    st0, _ = txlayer.call_document_batch(b, n, ctx)
    for field in ("doc_off", "doc_key_off", "ent_off", "incl_off", "cons_off"):
        off = (C.c_uint64 * (n + 1)).from_address(getattr(b, field))
        saved = list(off)
        off[1] = off[2] + 5
        with pytest.raises(N.MerkleError):
            txlayer.call_document_batch(b, n, ctx)
        for i, v in enumerate(saved):
            off[i] = v
    st1, _ = txlayer.call_document_batch(b, n, ctx)
    assert np.array_equal(st0, st1)


def test_verify_document_batch_wide_txs(m, ctx, orc):
    """Synthetic v1 documents in transactions of up to 700 entries (the
    htrees take the planned many-tree path), with KV metadata, a trivial
    DualProofV2 (source = target = the document's tx) and the tx as known
    state; a third of them with one entry's hValue flipped."""
    import struct
    from immustore_amd import txlayer
    from tx_util import TX_HEADER
    rng = np.random.default_rng(21)
    docs = []
    for k in range(60):
        ne = int(rng.integers(1, 700)) if k % 4 else int(rng.integers(1, 5))
        ents = []
        for e in range(ne):
            key = b"doc/%d/%d" % (k, e)
            md = [b"", b"\x00", b"\x02", b"\x01" + struct.pack(">Q", e)][e % 4]
            ents.append((key, md, bytes(rng.integers(0, 256, 32, dtype=np.uint8))))
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
    st, alh = txlayer.verify_document_batch(docs, ctx=ctx)
    for k, d in enumerate(docs):
        ost, oalh = orc.verify_document(d)
        assert int(st[k]) == ost, k
        assert alh[k].tobytes() == (oalh if ost == 0 else bytes(32))
        if k % 3 == 2 and len(d["entries"]) > 1:
            assert ost in (orc.ERR_INVALID_PROOF, orc.ERR_INVALID_PROOF_ENTRY)
        elif k % 3 != 2:
            assert ost == 0


def test_txlog_validate_metadata_parse_vs_oracle(m, ctx, orc):
    """Metadata as the reader parses it: valid non-canonical
    KV / tx metadata is hashed in its re-serialised form (Go hashes Bytes()):
    the device hashes canonical entry records / tx metadata placed after the
    log; invalid metadata stops the read with ErrCorruptedData.  Also a
    > 8 MiB log of such records (the multi-threaded hop merges the patches)."""
    from tx_util import metadata_logs
    logs = metadata_logs(orc)
    big = b"".join(raw for name, raw in logs if name == "noncanonical_sealed_canonical") * 4200
    assert len(big) > (8 << 20)
    for name, raw in logs + [("big", big)]:
        rc, n, used, hdrs, alh, sts = m.txlog_validate(raw, ctx=ctx)
        o = orc.txlog_validate(raw)
        assert (rc, n, used) == (o[0], o[1], o[2]), name
        assert np.array_equal(alh, o[3][:n]) and np.array_equal(sts, o[4][:n]), name
    rc, n, _, _, _, sts = m.txlog_validate(big, ctx=ctx)
    assert rc == 0 and n == 42000 and not sts.any()


def _record_heads(raw, n):
    """The TxHeader fields of the first n records, parsed in Python from the
    raw log (tx.go:419-518) -- what mh_txlog_validate returns besides Eh."""
    out, p = [], 0
    for _ in range(n):
        tid, ts, bl = struct.unpack_from(">QQQ", raw, p)
        ver, = struct.unpack_from(">H", raw, p + 88)
        if ver == 0:
            ne, = struct.unpack_from(">H", raw, p + 90)
            ml, mo, q = 0, 0, p + 92
        else:
            ml, = struct.unpack_from(">H", raw, p + 90)
            ne, = struct.unpack_from(">I", raw, p + 92 + ml)
            mo, q = p + 92, p + 96 + ml
        out.append((tid, ts, bl, raw[p + 24:p + 56], raw[p + 56:p + 88], ver, ne, ml, mo))
        for _ in range(ne):
            m_, = struct.unpack_from(">H", raw, q)
            k_, = struct.unpack_from(">H", raw, q + 2 + m_)
            q += 4 + m_ + k_ + 44
        p = q + 32
    return out


@pytest.mark.parametrize("max_entries", [1, 2, 3, 5, 8, 16, 17, 40, 64])
def test_txlog_fused_kernels_vs_oracle(m, ctx, orc, monkeypatch, max_entries):
    """k_txlog_wave (one wave per 64 / L records, L lanes per record: every
    lane-count the widest tx can pick; the records staged in LDS and read from
    HBM) and k_txlog_lanes (1, 2, 4, 8 and 16 lanes per record, each lane's
    subtree serial) against the oracle and the record heads parsed in Python:
    Alh and per-tx statuses equal to the oracle's, headers (every field, Eh
    included) equal across kernels and to the Python parse, clean and with
    corrupted records, with pageable and pinned outputs."""
    import torch
    from immustore_amd.txlayer import TX_HEADER
    rng = np.random.default_rng(100 + max_entries)
    raw = _synthetic_txlog(rng, 700, orc, max_entries=max_entries)
    bad = bytearray(raw)
    for p in rng.integers(0, len(raw), 25):
        bad[int(p)] ^= 0x40
    cap = 800
    pin = (torch.empty(cap * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER),
           torch.empty(cap * 32, dtype=torch.uint8).pin_memory().numpy().reshape(cap, 32),
           torch.empty(cap, dtype=torch.int32).pin_memory().numpy())
    for buf in (raw, bytes(bad)):
        o = orc.txlog_validate(buf)
        res = {}
        for kern, smax in (("wave", None), ("wave", "0"), ("lanes", "L1"), ("lanes", "L2"),
                           ("lanes", "L4"), ("lanes", "L8"), ("lanes", "L16")):
            monkeypatch.setenv("MH_TXLOG_KERNEL", kern)
            monkeypatch.delenv("MH_TXLOG_STAGE_MAX", raising=False)
            monkeypatch.delenv("MH_TXLOG_LANES", raising=False)
            if smax is not None and smax.startswith("L"):
                monkeypatch.setenv("MH_TXLOG_LANES", smax[1:])
            elif smax is not None:
                monkeypatch.setenv("MH_TXLOG_STAGE_MAX", smax)
            for out in (None, pin):
                a = m.txlog_validate(buf, ctx=ctx, out=out)
                assert (a[0], a[1], a[2]) == (o[0], o[1], o[2]), (kern, smax)
                assert np.array_equal(a[4], o[3]) and list(a[5]) == list(o[4]), (kern, smax)
                res[(kern, smax, out is None)] = a[3][:a[1]].copy()
        ref = res[("wave", None, True)]
        for key, h in res.items():
            assert np.array_equal(h, ref), key
        if buf is raw:
            heads = _record_heads(buf, o[1])
            for h, x in zip(ref, heads):
                got = (int(h["id"]), int(h["ts"]), int(h["bl_tx_id"]), h["bl_root"].tobytes(),
                       h["prev_alh"].tobytes(), int(h["version"]), int(h["nentries"]),
                       int(h["md_len"]), int(h["md_off"]))
                assert got == x
    monkeypatch.delenv("MH_TXLOG_KERNEL", raising=False)
    monkeypatch.delenv("MH_TXLOG_LANES", raising=False)


@pytest.mark.parametrize("kern", ["wave", "lanes"])
def test_txlog_validate_resident_vs_host_path(m, ctx, orc, monkeypatch, kern):
    """mh_txlog_validate_resident (the log already in HBM: scrub / re-validate
    of what was just written, one group, no copy) equals the copying call and
    the oracle -- clean and corrupted logs, the Go-written fixture log, pinned
    and pageable outputs; a device allocation ending less than 256 bytes past
    the log, or a host pointer, is refused."""
    import ctypes as C
    import torch
    from immustore_amd import _native as N
    from immustore_amd.txlayer import TX_HEADER
    monkeypatch.setenv("MH_TXLOG_KERNEL", kern)
    rng = np.random.default_rng(7)
    logs = [_synthetic_txlog(rng, 900, orc, max_entries=16),
            _synthetic_txlog(rng, 300, orc, max_entries=64)]
    bad = bytearray(logs[0])
    for p in rng.integers(0, len(bad), 20):
        bad[int(p)] ^= 0x08
    logs.append(bytes(bad))
    cap = 1000
    pin = (torch.empty(cap * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER),
           torch.empty(cap * 32, dtype=torch.uint8).pin_memory().numpy().reshape(cap, 32),
           torch.empty(cap, dtype=torch.int32).pin_memory().numpy())
    for raw in logs:
        d = torch.zeros(len(raw) + 256, dtype=torch.uint8, device="cuda")
        d[:len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
        torch.cuda.synchronize()
        o = orc.txlog_validate(raw)
        want = m.txlog_validate(raw, ctx=ctx)
        for out in (None, pin):
            got = m.txlog_validate(raw, ctx=ctx, out=out, dev=d.data_ptr())
            assert (got[0], got[1], got[2]) == (o[0], o[1], o[2])
            assert np.array_equal(got[4], o[3]) and list(got[5]) == list(o[4])
            assert np.array_equal(got[3], want[3][:want[1]])
    L = N.load()
    raw = logs[0]
    p = C.c_void_p()
    size = (len(raw) + 65535) & ~65535
    N.check(L.mh_dev_alloc(ctx.handle, size, C.byref(p)))
    try:
        hb = np.frombuffer(raw, np.uint8)
        ntx, used = C.c_uint64(), C.c_uint64()
        alh = np.zeros((cap, 32), np.uint8)
        sts = np.zeros(cap, np.int32)
        args = lambda dp: (ctx.handle, hb.ctypes.data, dp, len(raw), 1024, 1024, cap, C.byref(ntx),  # noqa: E731
                           C.byref(used), None, alh.ctypes.data, sts.ctypes.data)
        assert L.mh_txlog_validate_resident(*args(p.value + size - len(raw))) == N.MH_ERR_ILLEGAL_ARGUMENTS
        assert L.mh_txlog_validate_resident(*args(hb.ctypes.data)) == N.MH_ERR_ILLEGAL_ARGUMENTS
    finally:
        L.mh_dev_free(ctx.handle, p.value)
