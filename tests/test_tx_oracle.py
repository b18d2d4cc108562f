"""Oracle restatement of the tx layer against
the reference's Go-written test stores: every stored Alh, the raw tx-log
records, and DualProofV2 / linear proofs built from the stores' own headers
and dLog (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from tx_util import headers_from_fixture


def test_header_alh_matches_stored(orc, fixtures):
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        for k in range(len(recs)):
            st, _, a = orc.tx_header_alh(recs[k], blob)
            assert st == 0 and a == alhs[k], (name, k)


def test_txlog_validate_fixture_stores(orc, fixtures):
    for name, fx in fixtures.items():
        raw = bytes.fromhex(fx["txlog"])
        st, n, used, alh, sts = orc.txlog_validate(raw)
        assert st == 0 and n == len(fx["txs"]), name
        assert all(s == 0 for s in sts)
        assert [a.tobytes().hex() for a in alh] == [t["header"]["alh"] for t in fx["txs"]]


def _record_spans(raw):
    """byte offset of every tx record (walks the same format)."""
    import struct
    p, spans = 0, []
    while p + 8 <= len(raw) and struct.unpack(">Q", raw[p:p + 8])[0]:
        s = p
        p += 8 + 16 + 64
        ver = struct.unpack(">H", raw[p:p + 2])[0]
        p += 2
        if ver == 0:
            ne = struct.unpack(">H", raw[p:p + 2])[0]
            p += 2
        else:
            ml = struct.unpack(">H", raw[p:p + 2])[0]
            p += 2 + ml
            ne = struct.unpack(">I", raw[p:p + 4])[0]
            p += 4
        for _ in range(ne):
            ml = struct.unpack(">H", raw[p:p + 2])[0]
            p += 2 + ml
            kl = struct.unpack(">H", raw[p:p + 2])[0]
            p += 2 + kl + 12 + 32
        p += 32
        spans.append((s, p))
    return spans


def test_txlog_validate_detects_corruption(orc, fixtures):
    raw = bytes.fromhex(fixtures["long_linear_proof"]["txlog"])
    spans = _record_spans(raw)
    assert len(spans) == len(fixtures["long_linear_proof"]["txs"])
    # flip one bit of tx 5's last stored hVal (just before its stored alh)
    s, e = spans[4]
    bad = bytearray(raw)
    bad[e - 32 - 1] ^= 1
    st, n, _, _, sts = orc.txlog_validate(bytes(bad))
    assert st == 0 and n == len(spans)
    assert [k for k, x in enumerate(sts) if x] == [4] and sts[4] == 14
    # stored alh flipped: same per-tx status
    bad = bytearray(raw)
    bad[e - 1] ^= 0x80
    assert list(orc.txlog_validate(bytes(bad))[4]).count(14) == 1
    # unknown header version -> structural error at that record
    bad = bytearray(raw)
    bad[s + 88:s + 90] = b"\x00\x07"
    st, n, used, _, _ = orc.txlog_validate(bytes(bad))
    assert st == 17 and n == 4 and used == s
    # too many entries for the reader's limit
    st, n, _, _, _ = orc.txlog_validate(raw, max_entries=0)
    assert st == 15 and n == 0
    # key longer than MaxKeyLen
    st, n, _, _, _ = orc.txlog_validate(raw, max_key_len=3)
    assert st == 16 and n == 0
    # truncated record
    st, n, used, _, _ = orc.txlog_validate(raw[:e - 5])
    assert st == 18 and n == 4 and used == s
    # preallocated zero tail ends the log cleanly
    st, n, _, _, _ = orc.txlog_validate(raw + b"\0" * 64)
    assert st == 0 and n == len(spans)
    assert orc.txlog_validate(raw, max_txs=3)[1] == 3


def test_dual_proof_v2_fixture_cases(orc, fixtures):
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        for c in fx["dual_v2"]:
            s, t = c["src"], c["tgt"]
            incl = [bytes.fromhex(x) for x in c["incl"]]
            cons = [bytes.fromhex(x) for x in c["cons"]]
            args = (recs[s - 1], recs[t - 1], blob, incl, cons, s, t, alhs[s - 1], alhs[t - 1])
            assert orc.verify_dual_proof_v2(*args) == 0, (name, s, t)
            if incl:
                bad = [bytes([incl[0][0] ^ 1]) + incl[0][1:]] + incl[1:]
                assert orc.verify_dual_proof_v2(recs[s - 1], recs[t - 1], blob, bad, cons, s, t,
                                                alhs[s - 1], alhs[t - 1]) == 12
            if cons:
                bad = cons[:-1] + [bytes([cons[-1][0] ^ 1]) + cons[-1][1:]]
                assert orc.verify_dual_proof_v2(recs[s - 1], recs[t - 1], blob, incl, bad, s, t,
                                                alhs[s - 1], alhs[t - 1]) == 13
            # wrong source alh, swapped ids, mismatching header ids
            assert orc.verify_dual_proof_v2(recs[s - 1], recs[t - 1], blob, incl, cons, s, t,
                                            alhs[t - 1] if s != t else b"\0" * 32,
                                            alhs[t - 1]) == 2
            if s < t:
                assert orc.verify_dual_proof_v2(recs[t - 1], recs[s - 1], blob, incl, cons, t, s,
                                                alhs[t - 1], alhs[s - 1]) == 10
            assert orc.verify_dual_proof_v2(recs[s - 1], recs[t - 1], blob, incl, cons, s + 1, t,
                                            alhs[s - 1], alhs[t - 1]) == 2


def test_linear_proofs_fixture_cases(orc, fixtures):
    for name, fx in fixtures.items():
        alhs = [bytes.fromhex(t["header"]["alh"]) for t in fx["txs"]]
        for c in fx["linear"]:
            s, t = c["src"], c["tgt"]
            terms = [bytes.fromhex(x) for x in c["terms"]]
            assert orc.verify_linear_proof(s, t, terms, s, t, alhs[s - 1], alhs[t - 1])
            assert not orc.verify_linear_proof(s, t, terms, s, t + 1, alhs[s - 1], alhs[t - 1])
            assert not orc.verify_linear_proof(s, t, terms[:-1], s, t, alhs[s - 1], alhs[t - 1]) or \
                len(terms) == 1
            if len(terms) > 1:
                bad = terms[:1] + [bytes([terms[1][0] ^ 4]) + terms[1][1:]] + terms[2:]
                assert not orc.verify_linear_proof(s, t, bad, s, t, alhs[s - 1], alhs[t - 1])
        # verification.go:43-49 edge rules
        assert not orc.verify_linear_proof(0, 1, [alhs[0]], 0, 1, alhs[0], alhs[0])
        assert not orc.verify_linear_proof(2, 1, [alhs[0]], 2, 1, alhs[0], alhs[0])
        assert not orc.verify_linear_proof(1, 1, [], 1, 1, alhs[0], alhs[0])
        assert orc.verify_linear_proof(1, 1, [alhs[0]], 1, 1, alhs[0], alhs[0])


def test_linear_advance_proof_edges(orc):
    z = b"\0" * 32
    # verification.go:90-104: end < start false, end <= start+1 true, nil proof false
    assert not orc.verify_linear_advance_proof(None, 5, 4, z, z, 10)
    assert orc.verify_linear_advance_proof(None, 5, 6, z, z, 10)
    assert not orc.verify_linear_advance_proof(None, 5, 7, z, z, 10)
    assert not orc.verify_linear_advance_proof(([z, z], []), 5, 7, z, z, 10)


def dual_v1_args(c, recs, blob, alhs, tamper=None):
    """Fixture DualProof (v1) case -> orc.verify_dual_proof arguments."""
    s, t = c["src"], c["tgt"]
    dec = lambda xs: [bytes.fromhex(x) for x in xs]  # noqa: E731
    incl, cons, last = dec(c["incl"]), dec(c["cons"]), dec(c["last"])
    lin = (c["lin_src"], t, dec(c["lin"]))
    lap = None if c["lap"] is None else (dec(c["lap"]["terms"]), [dec(x) for x in c["lap"]["incl"]])
    tbl = bytes.fromhex(c["tbl_alh"])
    if tamper == "lap" and lap and lap[1] and any(lap[1]):
        k = next(i for i, x in enumerate(lap[1]) if x)
        lap[1][k] = [bytes([lap[1][k][0][0] ^ 1]) + lap[1][k][0][1:]] + lap[1][k][1:]
    if tamper == "lin" and len(lin[2]) > 1:
        lin = (lin[0], lin[1], lin[2][:-1] + [bytes([lin[2][-1][0] ^ 8]) + lin[2][-1][1:]])
    if tamper == "last" and last:
        last = [bytes([last[0][0] ^ 1]) + last[0][1:]] + last[1:]
    if tamper == "tbl":
        tbl = bytes(32)
    return (recs[s - 1], recs[t - 1], blob, incl, cons, tbl, last, lin, lap, s, t, alhs[s - 1],
            alhs[t - 1])


def test_dual_proof_v1_fixture_cases(orc, fixtures):
    n_lap = 0
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        for c in fx["dual_v1"]:
            assert orc.verify_dual_proof(*dual_v1_args(c, recs, blob, alhs)), (name, c["src"],
                                                                               c["tgt"])
            if c["lap"] and any(c["lap"]["incl"]):
                n_lap += 1
                assert not orc.verify_dual_proof(*dual_v1_args(c, recs, blob, alhs, "lap"))
            if len(c["lin"]) > 1:
                assert not orc.verify_dual_proof(*dual_v1_args(c, recs, blob, alhs, "lin"))
            if c["last"]:
                assert not orc.verify_dual_proof(*dual_v1_args(c, recs, blob, alhs, "last"))
            if recs[c["tgt"] - 1]["bl_tx_id"] > 0:
                assert not orc.verify_dual_proof(*dual_v1_args(c, recs, blob, alhs, "tbl"))
    assert n_lap > 10


# ---------------------------------------------------------- precommit (8(f) row 1)
@pytest.mark.parametrize("store", ["long_linear_proof", "v110_defaultdb", "v110_systemdb"])
@pytest.mark.parametrize("trunc", [0, 3])
def test_precommit_batch_fixture_stores(orc, fixtures, store, trunc):
    """Every stored Eh from the Go stores' own entries (values or, for every
    third entry, the stored hVal as a truncated value), 1 and 4 threads."""
    from commit_util import fixture_batch
    version, b, eh_ref = fixture_batch(fixtures[store], trunc)
    for th in (1, 4):
        hv, eh, st = orc.precommit_batch(version, nthreads=th, **b)
        assert (st == 0).all()
        assert np.array_equal(eh, eh_ref)
        _, eh2, st2 = orc.precommit_batch(version, expect_eh=eh_ref, **b)
        assert (st2 == 0).all()


def test_precommit_batch_statuses(orc):
    from commit_util import random_batch
    rng = np.random.default_rng(11)
    b = random_batch(rng, 50, version=1)
    hv, eh, st = orc.precommit_batch(1, **b)
    assert (st == 0).all()
    # per-tx restatement: orc.build_entries over each tx's entries
    to = b["tx_off"]
    for t in range(50):
        e0, e1 = int(to[t]), int(to[t + 1])
        ks = [b["keys"][int(b["key_off"][e]):int(b["key_off"][e + 1])].tobytes() for e in range(e0, e1)]
        vs = [b["vals"][int(b["val_off"][e]):int(b["val_off"][e + 1])].tobytes() for e in range(e0, e1)]
        mds = [b["md"][int(b["md_off"][e]):int(b["md_off"][e + 1])].tobytes() if "md" in b else b""
               for e in range(e0, e1)]
        ovs = None
        if "use_override" in b:
            ovs = [b["hval_override"][e].tobytes() if b["use_override"][e] else None
                   for e in range(e0, e1)]
        s1, hv1, _, root = orc.build_entries(1, ks, mds, vs, ovs)
        assert s1 == 0 and root == eh[t].tobytes()
        assert np.array_equal(hv1, hv[e0:e1])
    # expected-Eh mismatch -> ErrIllegalArguments, max width, v0 + metadata
    bad = eh.copy()
    bad[7, 3] ^= 1
    _, eh2, st2 = orc.precommit_batch(1, expect_eh=bad, **b)
    assert list(np.nonzero(st2)[0]) == [7] and st2[7] == 2 and np.array_equal(eh2, eh)
    widths = np.diff(to.astype(np.int64))
    _, eh3, st3 = orc.precommit_batch(1, max_width=20, **b)
    assert ((st3 == 1) == (widths > 20)).all()
    assert not eh3[widths > 20].any()
    _, eh4, st4 = orc.precommit_batch(0, **b)
    has_md = np.array([int(b["md_off"][int(to[t + 1])] - b["md_off"][int(to[t])]) > 0
                       for t in range(50)])
    assert ((st4 == 6) == has_md).all()


def test_verify_document_oracle_on_go_stores(orc, fixtures):
    """pkg/verification.VerifyDocument restated (oracle.verify_document) on
    documents taken from the Go-written stores: every untampered v1 document
    verifies and yields the target's stored Alh; v0 txs fail the Eh check
    because EntrySpecDigest_v0 hashes SHA256(Value) of the nil Value
    (store/verification.go:256-262); every tampered check fails."""
    from tx_util import document_cases
    docs, blob = document_cases(fixtures, orc)
    seen = {}
    for k, d in enumerate(docs):
        st, alh = orc.verify_document(d, blob)
        v = k % 13
        ver = int(d["src_hdr"]["version"])
        seen.setdefault((ver, v), set()).add(st)
        if v == 0:
            if ver == 1 and (d["known_tx_id"] or int(d["src_hdr"]["id"]) == 1):
                assert st == 0
                # new state = target Alh
                assert alh == orc.tx_header_alh(d["tgt_hdr"], blob)[2]
            else:  # v0 quirk, or no known state with a source other than tx 1 (:165-168)
                assert st == orc.ERR_INVALID_PROOF
        elif v in (1, 2, 3):
            assert st == orc.ERR_INVALID_PROOF_ENTRY
        elif v == 11:
            assert st == orc.ERR_UNSUPPORTED_TX_VERSION
        elif v in (4, 5, 6, 7, 10) or (v == 12 and d["src_hdr"]["id"] != d["tgt_hdr"]["id"]):
            assert st != 0
    assert (1, 0) in seen and (0, 0) in seen
