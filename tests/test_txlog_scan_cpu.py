"""The tx-log record hop (mh_txlog_scan: the structure-only part of
mh_txlog_validate, host code, no device) against the oracle's sequential parse
(orc_txlog_validate, tx.go:419-603): the reference's Go-written tx logs,
synthetic records with every structural error, and > 8 MiB logs that take the
multi-threaded hop from speculated record starts."""
import numpy as np
import pytest

from tx_util import _bulk_txlog, _synthetic_txlog


@pytest.fixture(scope="module")
def txl():
    from immustore_amd import txlayer
    return txlayer


def same(txl, orc, buf, **kw):
    a = txl.txlog_scan(buf, **kw)
    b = orc.txlog_validate(buf, **kw)
    assert (a[0], a[1], a[2]) == (b[0], b[1], b[2]), kw
    ao = a[4]
    if a[1]:
        # every record ends with its stored Alh: the parse stops right after the last one
        assert int(ao[-1]) + 32 == a[2]
        assert np.all(np.diff(ao.astype(np.int64)) > 0)
    return a


def test_scan_fixture_logs(txl, orc, fixtures):
    for name, fx in fixtures.items():
        raw = bytes.fromhex(fx["txlog"])
        a = same(txl, orc, raw)
        assert a[0] == 0 and a[1] == len(fx["txs"])
        assert [int(v) for v in a[3]["version"]] == [t["header"]["version"] for t in fx["txs"]]


def test_scan_synthetic_errors(txl, orc):
    rng = np.random.default_rng(5)
    raw = _synthetic_txlog(rng, 120, orc)
    same(txl, orc, raw)
    for kw in ({"max_entries": 5}, {"max_key_len": 10}, {"max_txs": 17}, {"max_txs": 0}):
        same(txl, orc, raw, **kw)
    for cut in (0, 1, 7, 8, 50, 89, 90, 91, len(raw) // 3, len(raw) - 33, len(raw) - 1):
        same(txl, orc, raw[:cut])
    bad = bytearray(raw)
    for pos in np.random.default_rng(9).integers(0, len(raw), 60):
        bad[int(pos)] ^= 0x40
        same(txl, orc, bytes(bad))


def test_scan_parallel_hop_matches_sequential(txl, orc):
    rng = np.random.default_rng(78)
    raw, starts = _bulk_txlog(rng, 9000)
    assert len(raw) > (8 << 20)
    a = same(txl, orc, raw)
    assert (a[0], a[1], a[2]) == (0, 9000, len(raw))
    for k, code in ((1, 17), (4444, 17), (8999, 17)):  # unknown version in chunk 0 / middle / last
        bad = bytearray(raw)
        bad[starts[k] + 89] = 9
        a = same(txl, orc, bytes(bad))
        assert (a[0], a[1], a[2]) == (code, k, starts[k])
    bad = bytearray(raw)
    bad[starts[6000] + 95] = 0xFF  # nentries of a v1 record beyond max_entries (or truncation)
    same(txl, orc, bytes(bad))
    same(txl, orc, raw[:len(raw) - 100])
    same(txl, orc, raw[:starts[5000]] + bytes(3 << 20))
    for mt in (1, 4321, 8999, 9000, 10 ** 6):
        same(txl, orc, raw, max_txs=mt)
    # max_txs reached right before a structural error / a cut: the sequential
    # parse never reads the bad record (the merge once reported the error of
    # the hop chunk that holds it)
    bad = bytearray(raw)
    bad[starts[4444] + 89] = 9
    for mt in (4443, 4444, 4445):
        a = same(txl, orc, bytes(bad), max_txs=mt)
        assert a[0] == (0 if mt <= 4444 else 17)
    for cut in range(starts[6000] + 1, starts[6000] + 100, 33):
        same(txl, orc, raw[:cut], max_txs=6000)
    # records that span whole hop chunks: 3 txs of 90 000 entries (~4.6 MB each)
    import struct
    recs = bytearray()
    for k in range(3):
        ne = 90000
        recs += struct.pack(">QQQ", k + 1, 5, k) + bytes(64) + struct.pack(">HHI", 1, 0, ne)
        ent = struct.pack(">HH", 0, 8) + b"k" * 8 + struct.pack(">IQ", 1, 2) + bytes(32)
        recs += ent * ne + bytes(32)
    recs = bytes(recs)
    assert len(recs) > (8 << 20)
    a = same(txl, orc, recs, max_entries=1 << 20)
    assert (a[0], a[1]) == (0, 3)
    same(txl, orc, recs, max_entries=1000)  # MaxTxEntries exceeded in the first record
    same(txl, orc, recs[:len(recs) // 2], max_entries=1 << 20)


def test_scan_concurrent_callers(txl, orc):
    """The hop's parked helper threads serve one call at a time; concurrent
    callers (other contexts, other goroutines) start their own threads. Six
    threads scanning different logs at once (some 1-8 MiB: the pool's smaller
    chunks) all get the sequential parse's result."""
    import threading
    rng = np.random.default_rng(91)
    raw, starts = _bulk_txlog(rng, 6000)
    bad = bytearray(raw)
    bad[starts[3333] + 89] = 9
    cases = [(raw, {}), (bytes(bad), {}), (raw[:len(raw) - 77], {}), (raw[:starts[700]], {}),
             (raw, {"max_txs": 2500}), (raw[:(3 << 20) + 5], {})]
    want = [orc.txlog_validate(b, **kw)[:3] for b, kw in cases]
    got = [None] * len(cases)

    def run(i):
        b, kw = cases[i]
        for _ in range(5):
            a = txl.txlog_scan(b, **kw)
            got[i] = (a[0], a[1], a[2]) if got[i] in (None, (a[0], a[1], a[2])) else "mismatch"

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(cases))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert got == [tuple(w) for w in want]


def test_scan_v0_entry_with_kv_metadata(txl, orc):
    """A v0 record whose entry carries KV metadata: TxEntryDigest_v1_1 fails
    the read with ErrMetadataUnsupported (tx.go:690-693 via readEntry,
    tx.go:582-588); the hop stops before that record."""
    import struct
    rng = np.random.default_rng(11)
    good = _synthetic_txlog(rng, 6, orc, version_mix=False)
    for md in (b"\x00", b"\x02", b"\x01" + struct.pack(">Q", 7)):
        ent = struct.pack(">H", len(md)) + md + struct.pack(">H", 3) + b"key"
        ent += struct.pack(">IQ", 5, 9) + bytes(32)
        rec = struct.pack(">QQQ", 7, 1, 0) + bytes(64) + struct.pack(">HH", 0, 1) + ent + bytes(32)
        for buf in (rec, good + rec):
            a = same(txl, orc, buf)
            assert a[0] == 6  # MH_ERR_METADATA_UNSUPPORTED
            assert a[1] == (0 if buf is rec else 6)


def test_scan_metadata_parse(txl, orc):
    """KV / tx metadata parsed as the reader does (kv_metadata.go:221-256,
    tx_metadata.go:159-193): unknown attribute codes, short payloads and an
    extra running past the metadata stop the read with ErrCorruptedData;
    valid non-canonical metadata parses."""
    from tx_util import metadata_logs
    for name, raw in metadata_logs(orc):
        a = same(txl, orc, raw)
        if name.startswith("bad"):
            assert (a[0], a[1]) == (14, 1), name
        else:
            assert (a[0], a[1]) == (0, 10), name


def test_oracle_metadata_canonical_hashing(orc):
    """Go hashes the re-serialised metadata: a log sealed over the canonical
    bytes validates, the same log sealed over the raw non-canonical bytes gives
    an ALH mismatch on exactly the non-canonical records."""
    from tx_util import metadata_logs
    logs = dict(metadata_logs(orc))
    rc, n, _, _, sts = orc.txlog_validate(logs["noncanonical_sealed_canonical"])
    assert rc == 0 and n == 10 and not np.any(sts)
    rc, n, _, _, sts = orc.txlog_validate(logs["noncanonical_sealed_raw"])
    assert rc == 0 and n == 10
    assert list(sts) == [0] + [14] * 8 + [0]
