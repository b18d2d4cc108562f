"""The oracle's restatement of readTx over the commit log
(oracle.txlog_validate_clog: immustore.go:3048-3060 -> txOffsetAndSize
:2569-2597 -> Tx.readFrom tx.go:388-630, plus the open path's cLog checks
:458-528), pinned by the reference's Go-written stores: each store's
commit/00000000.txi locates every record of its tx/00000000.tx, and every
stored Alh is reproduced (tests/golden/immudb_fixtures.json, written by
make_golden.py, which also checks each entry against the parsed record)."""
import struct

import numpy as np

from tx_util import _synthetic_txlog, clog_for, record_spans


def test_go_written_commit_logs_locate_every_record(orc, fixtures):
    for name, fx in fixtures.items():
        raw = bytes.fromhex(fx["txlog"])
        txi = bytes.fromhex(fx["txi"])
        assert len(txi) == 12 * len(fx["txs"])
        spans = record_spans(raw)
        assert clog_for(raw, spans, 12) == txi, name  # the Go writer's entries, byte for byte
        alh, sts = orc.txlog_validate_clog(raw, txi, 12)
        assert not sts.any(), name
        for k, tx in enumerate(fx["txs"]):
            assert alh[k].tobytes().hex() == tx["header"]["alh"], (name, k)
        # the cLog's own appendable header (singleapp, single_app.go:116-171)
        h = bytes.fromhex(fx["txi_header"])
        assert struct.unpack(">I", h[:4])[0] == len(h) - 4


def test_oracle_clog_checks(orc, fixtures):
    """Each cLog check on the Go-written store: a size one short / long is
    corrupted, an offset past the log truncated, a 44-byte entry with a
    foreign Alh corrupted, the same entries out of order all valid."""
    fx = fixtures["long_linear_proof"]
    raw = bytes.fromhex(fx["txlog"])
    txi = bytearray(bytes.fromhex(fx["txi"]))
    e = [txi[12 * k:12 * k + 12] for k in range(len(txi) // 12)]
    bad = [bytearray(x) for x in e]
    bad[2][8:12] = struct.pack(">I", struct.unpack(">I", e[2][8:12])[0] - 1)
    bad[4][8:12] = struct.pack(">I", struct.unpack(">I", e[4][8:12])[0] + 1)
    bad[6][0:8] = struct.pack(">Q", len(raw) + 5)
    _, sts = orc.txlog_validate_clog(raw, b"".join(bad), 12)
    assert (sts[2], sts[4], sts[6]) == (orc.ERR_CORRUPTED_DATA, orc.ERR_CORRUPTED_DATA,
                                        orc.ERR_TRUNCATED)
    assert not np.delete(sts, [2, 4, 6]).any()
    c44 = clog_for(raw, record_spans(raw), 44)
    alh, sts = orc.txlog_validate_clog(raw, c44, 44)
    assert not sts.any()
    m = bytearray(c44)
    m[44 * 9 + 12:44 * 9 + 44] = c44[44 * 10 + 12:44 * 10 + 44]
    alh2, sts = orc.txlog_validate_clog(raw, bytes(m), 44)
    assert sts[9] == orc.ERR_CORRUPTED_DATA and not alh2[9].any()
    perm = np.random.default_rng(1).permutation(len(e))
    alh3, sts = orc.txlog_validate_clog(raw, b"".join(bytes(e[k]) for k in perm), 12)
    assert not sts.any() and np.array_equal(alh3, alh[perm])


def test_oracle_clog_equals_sequential_read(orc):
    """On a clean synthetic log the per-record read equals the sequential
    one (orc.txlog_validate), record for record."""
    rng = np.random.default_rng(4)
    raw = _synthetic_txlog(rng, 200, orc, max_entries=30)
    a1, s1 = orc.txlog_validate_clog(raw, clog_for(raw, record_spans(raw), 12), 12)
    rc, n, _, a2, s2 = orc.txlog_validate(raw)
    assert rc == 0 and n == 200
    assert np.array_equal(a1, a2) and np.array_equal(s1, s2)
