"""GPU parity of a14 over a tx log already in HBM (SURVEY.md 8(a) a14, 8(f)
row 2), through the C ABI:

* mh_txlog_validate_clog -- the log located by its commit log (readTx,
  immustore.go:3048-3060 -> txOffsetAndSize :2569-2597 -> Tx.readFrom
  tx.go:388-630), no host hop, the log resident in HBM or in host memory
  (pageable or pinned; copied up in chunks, each checked as it lands): against the reference's Go-written stores with
  their Go-written commit logs (tests/golden: tx/00000000.tx +
  commit/00000000.txi), against mh_txlog_validate and against the oracle's
  restatement (oracle.txlog_validate_clog) on synthetic logs, corrupted
  records, wide and metadata-bearing records and mutated cLog entries;
* mh_txlog_validate_resident with resident bytes that drifted from the host
  copy: the drifted record is reported, nothing walks past it.
"""
import numpy as np
import pytest

from tx_util import _bulk_txlog, _synthetic_txlog, clog_for, metadata_logs, record_spans

pytestmark = pytest.mark.gpu

OK, CORRUPTED, TRUNCATED, ILLEGAL = 0, 14, 18, 2


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


def _dev(raw, pad=256):
    import torch
    d = torch.zeros(len(raw) + pad, dtype=torch.uint8, device="cuda")
    if len(raw):
        d[:len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    return d


MODES = ("dev", "host", "pinned")


def _pinned(raw):
    import torch
    t = torch.empty(max(len(raw), 1), dtype=torch.uint8).pin_memory()
    a = t.numpy()
    a[:len(raw)] = np.frombuffer(raw, np.uint8)
    return a[:len(raw)]


def _clog(ctx, raw, d, clog, es=12, out=None, mode="dev", **kw):
    """mode: the log resident (d), pageable host bytes, or a pinned host copy."""
    from immustore_amd.txlayer import txlog_validate_clog
    src = d.data_ptr() if mode == "dev" else np.frombuffer(raw, np.uint8) if mode == "host" \
        else _pinned(raw)
    return txlog_validate_clog(src, len(raw), clog, clog_entry_size=es, ctx=ctx, out=out, **kw)


def _same_as_oracle(orc, raw, clog, es, r, **kw):
    o_alh, o_sts = orc.txlog_validate_clog(raw, clog, es, **kw)
    rc, nbad, first, hd, alh, sts = r
    assert rc == 0
    assert list(sts) == list(o_sts)
    assert np.array_equal(alh, o_alh)
    bad = np.nonzero(o_sts)[0]
    assert nbad == len(bad) and first == (bad[0] if len(bad) else len(o_sts))
    return o_sts


def test_clog_fixture_stores(m, ctx, orc, fixtures):
    """The reference's three Go-written stores, each validated from its own
    commit log: every stored Alh reproduced, headers equal to
    mh_txlog_validate's; the 44-byte form (cLogEntrySizeV2) built from the same
    entries and the stored Alh values too."""
    for name, fx in fixtures.items():
        raw = bytes.fromhex(fx["txlog"])
        txi = bytes.fromhex(fx["txi"])
        want = m.txlog_validate(raw, ctx=ctx)
        d = _dev(raw)
        for es, cl, mode in ((12, txi, "dev"), (44, clog_for(raw, record_spans(raw), 44), "dev"),
                             (12, txi, "host"), (12, txi, "pinned")):
            r = _clog(ctx, raw, d, cl, es, mode=mode)
            _same_as_oracle(orc, raw, cl, es, r)
            assert r[1] == 0 and r[2] == len(fx["txs"])
            for k, tx in enumerate(fx["txs"]):
                assert r[4][k].tobytes().hex() == tx["header"]["alh"], (name, k)
            assert np.array_equal(r[3], want[3]), name
            assert np.array_equal(r[4], want[4])


@pytest.mark.parametrize("max_entries", [1, 5, 16, 64, 300])
def test_clog_synthetic_vs_validate_and_oracle(m, ctx, orc, max_entries):
    """Synthetic logs (v0 / v1 headers, KV / tx metadata, empty txs, up to 300
    entries per tx: every lane count and stack depth of the lane kernel):
    clean -- equal to mh_txlog_validate (headers, Alh, statuses) and to the
    oracle; with byte flips -- equal to the oracle (structural errors per
    record, Alh mismatches), with pageable, pinned and device outputs and 12-
    and 44-byte cLog entries."""
    import torch
    from immustore_amd.txlayer import TX_HEADER
    rng = np.random.default_rng(300 + max_entries)
    raw = _synthetic_txlog(rng, 600, orc, max_entries=max_entries)
    spans = record_spans(raw)
    assert len(spans) == 600
    want = m.txlog_validate(raw, ctx=ctx)
    n = len(spans)
    pin = (torch.empty(n * TX_HEADER.itemsize, dtype=torch.uint8).pin_memory().numpy().view(TX_HEADER),
           torch.empty(n * 32, dtype=torch.uint8).pin_memory().numpy().reshape(n, 32),
           torch.empty(n, dtype=torch.int32).pin_memory().numpy())
    dh = torch.zeros(n * TX_HEADER.itemsize, dtype=torch.uint8, device="cuda")
    da = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    ds = torch.zeros(n, dtype=torch.int32, device="cuda")
    bad = bytearray(raw)
    for p in rng.integers(0, len(raw), 30):
        bad[int(p)] ^= 0x20
    for buf in (raw, bytes(bad)):
        d = _dev(buf)
        for es in (12, 44):
            cl = clog_for(raw, spans, es)  # the clean log's cLog: flips may break records
            for out in (None, pin, "dev"):
                if out == "dev":
                    r = _clog(ctx, buf, d, cl, es, out=(dh.data_ptr(), da.data_ptr(), ds.data_ptr()))
                    r = r[:3] + (dh.cpu().numpy().view(TX_HEADER), da.view(n, 32).cpu().numpy(),
                                 ds.cpu().numpy())
                else:
                    r = _clog(ctx, buf, d, cl, es, out=out)
                for md in ("dev", "host", "pinned"):
                    if md != "dev":
                        if out == "dev" or (out is not None and es == 44):
                            continue
                        r = _clog(ctx, buf, d, cl, es, out=out, mode=md)
                    _same_as_oracle(orc, buf, cl, es, r)
                    if buf is raw:
                        assert r[1] == 0
                        assert np.array_equal(r[3], want[3]) and np.array_equal(r[4], want[4])
                        assert list(r[5]) == list(want[5])


def test_clog_entry_mutations(m, ctx, orc):
    """cLog entries that disagree with the log: a size one byte short or long
    (the record does not end at offset + size: corrupted), an offset past the
    log or into its zero tail (the reader's EOF: truncated), an offset into the
    middle of a record, two entries for one record, entries out of log order,
    a 44-byte entry whose Alh is not the record's -- every status and Alh
    equal to the oracle's."""
    import struct
    rng = np.random.default_rng(41)
    raw = _synthetic_txlog(rng, 400, orc, max_entries=20) + bytes(4096)
    spans = record_spans(raw)
    d = _dev(raw)
    ent = [bytearray(struct.pack(">QI", s, e - s) + raw[e - 32:e]) for s, e in spans]

    def run(entries, es):
        cl = b"".join(bytes(x[:es]) for x in entries)
        for mode in MODES:
            sts = _same_as_oracle(orc, raw, cl, es, _clog(ctx, raw, d, cl, es, mode=mode))
        return sts

    e = [bytearray(x) for x in ent]
    e[3][8:12] = struct.pack(">I", spans[3][1] - spans[3][0] - 1)
    e[7][8:12] = struct.pack(">I", spans[7][1] - spans[7][0] + 1)
    e[11][0:8] = struct.pack(">Q", len(raw) + 1000)
    e[12][0:8] = struct.pack(">Q", len(raw) - 100)  # the zero tail
    e[13][0:8] = struct.pack(">Q", spans[13][0] + 77)
    e[20] = bytearray(e[21])
    e[30][20] ^= 1  # the cLog's Alh (44-byte form only)
    e[50][0:8] = struct.pack(">Q", (1 << 64) - 16)  # offset + 8 wraps
    e[51][8:12] = struct.pack(">I", 0xffffffff)  # offset + size past any log
    e[52][0:12] = struct.pack(">QI", (1 << 64) - 64, 0xffffffff)  # both, the end wraps
    for es in (12, 44):
        sts = run(e, es)
        assert (sts[3], sts[7], sts[11], sts[12]) == (CORRUPTED, CORRUPTED, TRUNCATED, TRUNCATED)
        assert sts[13] != OK and sts[20] == OK and sts[21] == OK
        assert sts[30] == (CORRUPTED if es == 44 else OK)
        assert (sts[50], sts[51], sts[52]) == (TRUNCATED, CORRUPTED, TRUNCATED)
    perm = rng.permutation(len(ent))
    for es in (12, 44):
        assert not run([ent[k] for k in perm], es).any()


def test_clog_metadata_and_wide_records(m, ctx, orc):
    """Records the device hands to the host hop (metadata valid but not in
    Go's canonical form; more than 1024 entries) and records with invalid
    metadata (structural errors on the device): statuses and Alh equal to the
    oracle, canonical and non-canonical records mixed in one log."""
    rng = np.random.default_rng(5)
    for name, raw in metadata_logs(orc):
        spans = record_spans(raw)
        if not spans:
            continue
        d = _dev(raw)
        for es in (12, 44):
            cl = clog_for(raw, spans, es)
            for mode in MODES:
                _same_as_oracle(orc, raw, cl, es, _clog(ctx, raw, d, cl, es, mode=mode))
    mixed = b"".join(r for _, r in metadata_logs(orc))
    wide = _synthetic_txlog(rng, 12, orc, max_entries=1500)
    for raw, kw in ((mixed, {}), (wide, {"max_entries": 1500}),
                    (wide + _synthetic_txlog(rng, 50, orc, max_entries=8), {"max_entries": 1500})):
        spans = record_spans(raw)
        d = _dev(raw)
        cl = clog_for(raw, spans, 12)
        for mode in MODES:
            _same_as_oracle(orc, raw, cl, 12, _clog(ctx, raw, d, cl, 12, mode=mode, **kw), **kw)
    # the wide log with the default limit: MAX_ENTRIES per record, as the reader
    spans = record_spans(wide)
    cl = clog_for(wide, spans, 12)
    _same_as_oracle(orc, wide, cl, 12, _clog(ctx, wide, _dev(wide), cl, 12))


def test_clog_bulk_log(m, ctx, orc):
    """9000 ragged records (> 8 MiB, unsealed Alh values: every record an Alh
    mismatch except where the flips below break its structure) from a cLog in
    device memory; equal to the oracle and to mh_txlog_validate."""
    import torch
    rng = np.random.default_rng(9)
    raw, starts = _bulk_txlog(rng, 9000)
    spans = record_spans(raw)
    assert [s for s, _ in spans] == starts
    cl = clog_for(raw, spans, 12)
    dcl = torch.frombuffer(bytearray(cl), dtype=torch.uint8).cuda()
    from immustore_amd.txlayer import txlog_validate_clog
    d = _dev(raw)
    r = txlog_validate_clog(d.data_ptr(), len(raw), None, ntx=len(spans), clog_dev=dcl.data_ptr(),
                            ctx=ctx)
    _same_as_oracle(orc, raw, cl, 12, r)
    want = m.txlog_validate(raw, ctx=ctx)
    assert np.array_equal(r[4], want[4]) and np.array_equal(r[3], want[3])
    for mode in ("host", "pinned"):  # > 16 MiB: copied up in 3 (pageable: 2) chunks
        r = _clog(ctx, raw, d, cl, 12, mode=mode)
        _same_as_oracle(orc, raw, cl, 12, r)
        assert np.array_equal(r[4], want[4]) and np.array_equal(r[3], want[3])


def test_clog_host_log_chunk_edges(m, ctx, orc):
    """A host log > 16 MiB copied up in chunks, its records grouped by the
    chunk their cLog entry ends in: entries whose size reaches past the chunk
    boundary (a read past the bytes landed: the host takes the record, as the
    reader would see the whole log), past the log's end, entries out of log
    order (one group after every chunk), a 44-byte entry's Alh flipped, and
    non-canonical metadata records in the middle -- equal to the oracle and to
    the resident log's results, pageable and pinned."""
    import struct
    rng = np.random.default_rng(19)
    raw, _ = _bulk_txlog(rng, 8000)
    raw += b"".join(r for n, r in metadata_logs(orc) if n == "noncanonical_sealed_canonical")
    raw += _synthetic_txlog(rng, 200, orc, max_entries=40)
    spans = record_spans(raw)
    assert len(raw) > (16 << 20)
    d = _dev(raw)
    ent = [bytearray(struct.pack(">QI", s, e - s) + raw[e - 32:e]) for s, e in spans]
    # a record near each 5:2:1 / 3:1 cut (4 KiB aligned)
    cuts = [(int(len(raw) * f) & ~4095) for f in (5 / 8, 7 / 8, 3 / 4)]
    e = [bytearray(x) for x in ent]
    for c in cuts:
        t = next(k for k, (s, en) in enumerate(spans) if en > c)
        e[t - 1][8:12] = struct.pack(">I", spans[t - 1][1] - spans[t - 1][0] + 5000)  # past the cut
        e[t + 2][8:12] = struct.pack(">I", spans[t + 2][1] - spans[t + 2][0] - 1)
    e[len(e) - 3][8:12] = struct.pack(">I", 1 << 30)  # past the log's end
    e[100][12] ^= 1
    for es in (12, 44):
        cl = b"".join(bytes(x[:es]) for x in e)
        want = _same_as_oracle(orc, raw, cl, es, _clog(ctx, raw, d, cl, es))
        assert want.any()
        for mode in ("host", "pinned"):
            _same_as_oracle(orc, raw, cl, es, _clog(ctx, raw, d, cl, es, mode=mode))
    perm = np.concatenate([np.arange(1, 50), [0], np.arange(50, len(ent))])
    cl = b"".join(bytes(ent[k][:12]) for k in perm)
    for mode in MODES:
        _same_as_oracle(orc, raw, cl, 12, _clog(ctx, raw, d, cl, 12, mode=mode))


def test_clog_resident_launch_guess(m, ctx, orc):
    """The resident form shapes its lane launch by the previous call's widest
    record (no wait for this call's structure pass): a log wider than the
    guess is launched again at its own shape (the kernel raises a redo flag
    and writes nothing), a narrower one runs at the wider shape -- every call
    equal to the oracle, with host and device outputs."""
    import torch
    rng = np.random.default_rng(61)
    logs = [_synthetic_txlog(rng, 200, orc, max_entries=w) for w in (2, 40, 3, 300, 1, 64)]
    for raw in logs:
        spans = record_spans(raw)
        d = _dev(raw)
        cl = clog_for(raw, spans, 12)
        _same_as_oracle(orc, raw, cl, 12, _clog(ctx, raw, d, cl, 12))
        n = len(spans)
        da = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        ds = torch.zeros(n, dtype=torch.int32, device="cuda")
        r = _clog(ctx, raw, d, cl, 12, out=(None, da.data_ptr(), ds.data_ptr()))
        _same_as_oracle(orc, raw, cl, 12, r[:3] + (None, da.view(n, 32).cpu().numpy(), ds.cpu().numpy()))


def test_clog_arguments(m, ctx, orc):
    """A device allocation ending less than 256 bytes past the log, an entry
    size other than 12 / 44: illegal arguments; a host pointer as the log: the
    host-log mode; no records: MH_OK with nothing bad."""
    import ctypes as C
    from immustore_amd import _native as N
    rng = np.random.default_rng(2)
    raw = _synthetic_txlog(rng, 20, orc, max_entries=4)
    cl = clog_for(raw, record_spans(raw), 12)
    L = N.load()
    nb, fb = C.c_uint64(), C.c_uint64()
    cb = np.frombuffer(cl, np.uint8)
    p = C.c_void_p()
    size = (len(raw) + 65535) & ~65535  # an allocation of its own (not torch's cache)
    N.check(L.mh_dev_alloc(ctx.handle, size, C.byref(p)))
    try:
        assert L.mh_txlog_validate_clog(ctx.handle, p.value + size - len(raw) - 100, len(raw),
                                        cb.ctypes.data, 20, 12, 1024, 1024, None, None, None,
                                        C.byref(nb), C.byref(fb)) == ILLEGAL
    finally:
        L.mh_dev_free(ctx.handle, p.value)
    hb = np.frombuffer(raw, np.uint8)
    assert L.mh_txlog_validate_clog(ctx.handle, hb.ctypes.data, len(raw), cb.ctypes.data, 20, 12,
                                    1024, 1024, None, None, None, C.byref(nb), C.byref(fb)) == OK
    assert nb.value == 0 and fb.value == 20
    d = _dev(raw)
    assert L.mh_txlog_validate_clog(ctx.handle, d.data_ptr(), len(raw), cb.ctypes.data, 20, 13,
                                    1024, 1024, None, None, None, C.byref(nb), C.byref(fb)) == ILLEGAL
    assert L.mh_txlog_validate_clog(ctx.handle, d.data_ptr(), len(raw), cb.ctypes.data, 0, 12,
                                    1024, 1024, None, None, None, C.byref(nb), C.byref(fb)) == OK
    assert nb.value == 0 and fb.value == 0


@pytest.mark.parametrize("kern", ["wave", "lanes", "chain"])
def test_resident_log_drifted_from_host_copy(m, ctx, orc, monkeypatch, kern):
    """mh_txlog_validate_resident when the resident bytes are NOT the host
    copy: a length field flipped in the device copy only (an
    entry's key length, an mdLen, the entry count) and a flipped hVal -- the
    drifted records are MH_ERR_CORRUPTED_DATA, every other record equals the
    host call's, and nothing faults.  kern: the fused kernels (structure
    checked on the device first) and the chain of a group with re-encoded
    metadata (a byte compare against the uploaded host copy)."""
    import struct
    rng = np.random.default_rng(77)
    if kern == "chain":
        raw = _synthetic_txlog(rng, 300, orc, max_entries=16) + \
            b"".join(r for n, r in metadata_logs(orc) if n == "noncanonical_sealed_canonical")
    else:
        monkeypatch.setenv("MH_TXLOG_KERNEL", kern)
        raw = _synthetic_txlog(rng, 300, orc, max_entries=16)
    spans = record_spans(raw)
    want = m.txlog_validate(raw, ctx=ctx)
    assert want[0] == 0 and want[1] == len(spans)
    drift = bytearray(raw)
    hit = {}
    for t in (5, 40, 77, 120):
        s, e = spans[t]
        ver, = struct.unpack_from(">H", raw, s + 88)
        q = s + 92 if ver == 0 else s + 96 + struct.unpack_from(">H", raw, s + 90)[0]
        if q + 4 >= e - 32:  # no entries: flip the entry count instead
            drift[s + 90 if ver == 0 else q - 1] ^= 0x7f
        elif t % 2:
            ml, = struct.unpack_from(">H", raw, q)
            drift[q + 2 + ml] ^= 0xff  # the first entry's kLen, high byte
        else:
            drift[q] ^= 0x80  # the first entry's mdLen, high byte
        hit[t] = True
    drift[spans[200][1] - 40] ^= 1  # an hVal byte of record 200's last entry (or its vOff)
    hit[200] = True
    d = _dev(bytes(drift))
    got = m.txlog_validate(raw, ctx=ctx, dev=d.data_ptr())
    assert (got[0], got[1], got[2]) == (want[0], want[1], want[2])
    for t in range(len(spans)):
        if t in hit:
            assert got[5][t] == CORRUPTED, t
        else:
            assert got[5][t] == want[5][t] and np.array_equal(got[4][t], want[4][t]), t
    monkeypatch.delenv("MH_TXLOG_KERNEL", raising=False)
