"""DualProofV2 protobuf messages decoded on the device
(mh_dual_proof_v2_pb_decode_batch: DualProofV2FromProto, TxHeaderFromProto,
TxMetadataFromProto, DigestsFromProto, database_protoconv.go:226-305) against
the protobuf runtime's own parse of the same bytes (oracle/wire.py's
descriptors of schema.proto), then fed to VerifyDualProofV2."""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MAX_EXTRA = 256


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


@pytest.fixture(scope="module")
def wire(orc):
    import wire
    return wire


def d32(b):
    return (bytes(b) + bytes(32))[:32]


def _go_varints_ok(b, kind="top"):
    """protobuf-go rejects a 10-byte varint whose last byte is above 1
    (protowire.ConsumeVarint: errCodeOverflow); the upb runtime behind python
    protobuf drops the excess bits instead.  This walk applies Go's rule to
    every varint the decoder reads (keys, scalars, lengths, unknown fields
    and groups, inside the headers and their metadata); all else is left to
    the protobuf runtime's parse."""
    def varint(i):
        v = 0
        for k in range(10):
            if i >= len(b):
                raise IndexError
            c = b[i]
            i += 1
            if k == 9 and c > 1:
                raise OverflowError
            v |= (c & 0x7f) << (7 * k)
            if not c & 0x80:
                return v, i
        raise OverflowError
    try:
        i, groups = 0, []
        while i < len(b):
            key, i = varint(i)
            f, wt = key >> 3, key & 7
            if wt == 0:
                _, i = varint(i)
            elif wt == 1:
                i += 8
            elif wt == 5:
                i += 4
            elif wt == 2:
                ln, i = varint(i)
                sub, i = b[i:i + ln], i + ln
                # DualProofV2 ("top") -> TxHeader -> TxMetadata; "incl" (an
                # InclusionProof) has no sub-messages
                # DualProof v1 ("top1") adds LinearProof / LinearAdvanceProof
                nested = {"top": {1: "hdr", 2: "hdr"}, "hdr": {9: "md"},
                          "top1": {1: "hdr", 2: "hdr", 7: "lin", 8: "adv"},
                          "adv": {2: "incl"}}.get(kind, {})
                if not groups and f in nested and not _go_varints_ok(sub, nested[f]):
                    return False
            elif wt == 3:
                groups.append(f)
            elif wt == 4 and groups:
                groups.pop()
            if i > len(b):
                return True  # truncated: the runtime's parse rejects it too
        return True
    except OverflowError:
        return False
    except IndexError:
        return True


def expect(wire, raw):
    """What DualProofV2FromProto gives for `raw` per the protobuf runtime:
    (status, src, tgt, incl, cons); src / tgt = dict of header fields and the
    metadata's Bytes()."""
    from google.protobuf.message import DecodeError
    if not _go_varints_ok(raw):
        return 14, None, None, [], []
    try:
        mm = wire.MSG["DualProofV2"].FromString(raw)
    except DecodeError:
        return 14, None, None, [], []
    if not (mm.HasField("sourceTxHeader") and mm.HasField("targetTxHeader")):
        return 2, None, None, [d32(x) for x in mm.inclusionProof], [d32(x) for x in mm.consistencyProof]

    def hdr(h):
        md = b""
        if h.HasField("metadata"):
            if h.metadata.truncatedTxID > 0:
                md += b"\x00" + struct.pack(">Q", h.metadata.truncatedTxID)
            if 0 < len(h.metadata.extra) <= MAX_EXTRA:
                md += b"\x01" + struct.pack(">H", len(h.metadata.extra)) + h.metadata.extra
        return {"id": h.id, "ts": h.ts, "bl_tx_id": h.blTxId, "bl_root": d32(h.blRoot),
                "prev_alh": d32(h.prevAlh), "eh": d32(h.eH), "version": h.version & 0xFFFFFFFF,
                "nentries": h.nentries & 0xFFFFFFFF, "md": md}
    return (0, hdr(mm.sourceTxHeader), hdr(mm.targetTxHeader),
            [d32(x) for x in mm.inclusionProof], [d32(x) for x in mm.consistencyProof])


def got_hdr(r, md, k):
    off, ln = int(r["md_off"]), int(r["md_len"])
    return {"id": int(r["id"]), "ts": int(r["ts"]), "bl_tx_id": int(r["bl_tx_id"]),
            "bl_root": r["bl_root"].tobytes(), "prev_alh": r["prev_alh"].tobytes(),
            "eh": r["eh"].tobytes(), "version": int(r["version"]), "nentries": int(r["nentries"]),
            "md": md[off:off + ln]}


def check(wire, raws, out):
    st, sh, th, md, io, it, co, ct = out
    # metadata packed in message order, source before target
    ends = [0]
    for k in range(len(raws)):
        assert int(sh[k]["md_off"]) == ends[-1], k
        assert int(th[k]["md_off"]) == int(sh[k]["md_off"]) + int(sh[k]["md_len"]), k
        ends.append(int(th[k]["md_off"]) + int(th[k]["md_len"]))
    for k, raw in enumerate(raws):
        est, es, et, ei, ec = expect(wire, raw)
        assert int(st[k]) == est, (k, raw.hex())
        if est == 14:
            assert io[k + 1] == io[k] and co[k + 1] == co[k]
            continue
        assert [x.tobytes() for x in it[int(io[k]):int(io[k + 1])]] == ei, k
        assert [x.tobytes() for x in ct[int(co[k]):int(co[k + 1])]] == ec, k
        if est == 0:
            assert got_hdr(sh[k], md, 2 * k) == es, k
            assert got_hdr(th[k], md, 2 * k + 1) == et, k


def tag(f, wt):
    """a field key as its varint bytes"""
    v, out = f << 3 | wt, bytearray()
    while v >= 0x80:
        out.append(v & 0x7f | 0x80)
        v >>= 7
    return bytes(out + bytes([v]))


def random_msg(wire, rng):
    """A DualProofV2 message with random field values, the protobuf runtime's
    bytes, optionally with extra wire-level twists (unknown fields, a header
    split in two occurrences, fields out of order)."""
    M = wire.MSG

    def header():
        h = M["TxHeader"]()
        for f, v in (("id", int(rng.integers(0, 1 << 62))), ("ts", int(rng.integers(-(1 << 40), 1 << 40))),
                     ("blTxId", int(rng.integers(0, 1 << 40))),
                     ("version", int(rng.choice([0, 1, 2, -1]))),
                     ("nentries", int(rng.integers(-(1 << 31), 1 << 31)))):
            if rng.random() < 0.85:
                setattr(h, f, v)
        for f in ("prevAlh", "eH", "blRoot"):
            if rng.random() < 0.9:
                setattr(h, f, bytes(rng.integers(0, 256, int(rng.choice([32, 32, 32, 0, 5, 40])),
                                                 dtype=np.uint8)))
        if rng.random() < 0.5:
            md = M["TxMetadata"]()
            if rng.random() < 0.6:
                md.truncatedTxID = int(rng.integers(0, 1 << 50))
            if rng.random() < 0.6:
                md.extra = bytes(rng.integers(0, 256, int(rng.choice([0, 1, 100, 256, 257])),
                                              dtype=np.uint8))
            h.metadata.CopyFrom(md)
        return h

    mm = M["DualProofV2"]()
    if rng.random() < 0.95:
        mm.sourceTxHeader.CopyFrom(header())
    if rng.random() < 0.95:
        mm.targetTxHeader.CopyFrom(header())
    for _ in range(int(rng.integers(0, 30))):
        mm.inclusionProof.append(bytes(rng.integers(0, 256, int(rng.choice([32, 32, 31, 33, 0])),
                                                    dtype=np.uint8)))
    for _ in range(int(rng.integers(0, 30))):
        mm.consistencyProof.append(bytes(rng.integers(0, 256, 32, dtype=np.uint8)))
    raw = mm.SerializeToString()
    r = rng.random()
    if r < 0.15:
        # unknown fields: varint, fixed64, bytes, fixed32, a group (fields 50-54)
        raw += tag(50, 0) + bytes([0x96, 0x01]) + tag(51, 1) + bytes(8) + \
            tag(52, 2) + bytes([3, 1, 2, 3]) + tag(53, 5) + bytes(4) + \
            tag(54, 3) + tag(1, 0) + bytes([7]) + tag(54, 4)
    elif r < 0.3 and mm.HasField("sourceTxHeader"):
        # a second source header occurrence: merged into the first
        h2 = M["TxHeader"](id=int(rng.integers(1, 1 << 30)), blRoot=bytes(range(32)))
        b = h2.SerializeToString()
        raw += tag(1, 2) + bytes([len(b)]) + b
    elif r < 0.4:
        # a known field with the wrong wire type (skipped as unknown)
        raw = bytes([3 << 3 | 0, 5]) + raw
    return raw


def test_decode_random_messages_vs_protobuf(m, ctx, wire):
    from immustore_amd import txlayer
    rng = np.random.default_rng(2024)
    raws = [random_msg(wire, rng) for _ in range(3000)]
    raws += [b"", bytes([1 << 3 | 2, 0, 2 << 3 | 2, 0])]  # empty message; two empty headers
    check(wire, raws, txlayer.decode_dual_proof_v2_pb(raws, ctx=ctx))


def test_decode_corrupted_messages_vs_protobuf(m, ctx, wire):
    """Truncations and byte flips: the status is CORRUPTED exactly when the
    protobuf runtime rejects the bytes, else the fields agree."""
    from immustore_amd import txlayer
    rng = np.random.default_rng(7)
    base = [random_msg(wire, rng) for _ in range(400)]
    raws = []
    for raw in base:
        if not raw:
            continue
        b = bytearray(raw)
        if rng.random() < 0.5:
            raws.append(bytes(b[:int(rng.integers(0, len(b)))]))
        else:
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            raws.append(bytes(b))
    raws += [bytes([0x80] * 11), bytes([0x07]), bytes([1 << 3 | 2, 200]), bytes([0, 0]),
             tag(54, 3) + tag(1, 0) + bytes([7]), tag(54, 4), tag(1 << 29, 0) + bytes([1]), tag((1 << 29) - 1, 0) + bytes([1]),
             tag(7, 6), tag(2, 2) + bytes([0x80] * 9 + [2])]
    check(wire, raws, txlayer.decode_dual_proof_v2_pb(raws, ctx=ctx))


def _canonical_md(b):
    """TxMetadata.ReadFrom then Bytes() (tx_metadata.go:145-193): a zero
    truncated id and an empty extra are not written back"""
    out, i = b"", 0
    while i < len(b):
        if b[i] == 0:
            v = int.from_bytes(b[i + 1:i + 9], "big")
            out += b[i:i + 9] if v else b""
            i += 9
        else:
            ln = int.from_bytes(b[i + 1:i + 3], "big")
            out += b[i:i + 3 + ln] if ln else b""
            i += 3 + ln
    return out


def _same_hdr(a, b, md, blob):
    for f in ("id", "ts", "bl_tx_id", "version", "nentries"):
        assert int(a[f]) == int(b[f]), f
    for f in ("bl_root", "prev_alh", "eh"):
        assert a[f].tobytes() == b[f].tobytes(), f
    assert md[int(a["md_off"]):int(a["md_off"]) + int(a["md_len"])] == \
        _canonical_md(blob[int(b["md_off"]):int(b["md_off"]) + int(b["md_len"])])


def test_decode_device_encoded_random_headers(m, ctx, wire):
    """Round trip at scale: 3000 DualProofV2 messages written on the device
    (mh_ahtree_dual_proof_v2_pb_batch) from a 70 000-leaf tree and random
    headers with every metadata shape decode to the headers and proof terms
    they were written from."""
    from immustore_amd import txlayer
    from test_gpu_formats import _random_headers
    rng = np.random.default_rng(91)
    N_TX = 70000
    t = m.AHtree(ctx)
    t.append_batch(rng.integers(0, 256, (N_TX, 32), dtype=np.uint8))
    recs, blob = _random_headers(rng, N_TX + 10)
    tgt = rng.integers(1, N_TX + 1, 3000)
    src = np.array([int(rng.integers(1, x + 1)) for x in tgt])
    s, g = recs[src - 1].copy(), recs[tgt - 1].copy()
    msgs, st = t.dual_proof_v2_pb_batch(s, g, blob)
    assert (st == 0).all()
    out = txlayer.decode_dual_proof_v2_pb(msgs, ctx=ctx)
    dst, sh, th, md, io, it, co, ct = out
    assert (dst == 0).all()
    for k in range(len(msgs)):
        _same_hdr(sh[k], s[k], md, blob)
        _same_hdr(th[k], g[k], md, blob)
    check(wire, msgs, out)  # and the terms, against the protobuf runtime


def test_decode_then_verify_fixture_stores(m, ctx, orc, fixtures):
    """Real immudb stores (the golden fixtures): DualProofV2 messages written on
    the device, decoded on the device, then VerifyDualProofV2 over the decoded
    arrays gives the oracle's verdict on the fixture's own proof (0 for every
    proof the store emits), and a flipped term is rejected."""
    from immustore_amd import txlayer
    from tx_util import headers_from_fixture
    n_ok = 0
    for name, fx in fixtures.items():
        pay = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
        t = m.AHtree(ctx)
        t.append_batch(pay)
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        cases = [(c["src"], c["tgt"]) for c in fx["dual_v2"] if c["src"] <= c["tgt"]]
        S = np.array([a for a, _ in cases], np.uint64)
        T = np.array([b for _, b in cases], np.uint64)
        msgs, st = t.dual_proof_v2_pb_batch(recs[S.astype(int) - 1], recs[T.astype(int) - 1], blob)
        assert (st == 0).all(), name
        dst, sh, th, md, io, it, co, ct = txlayer.decode_dual_proof_v2_pb(msgs, ctx=ctx)
        assert (dst == 0).all(), name
        incl = [it[int(io[k]):int(io[k + 1])] for k in range(len(msgs))]
        cons = [ct[int(co[k]):int(co[k + 1])] for k in range(len(msgs))]
        sa = [alhs[int(x) - 1] for x in S]
        ta = [alhs[int(x) - 1] for x in T]
        vs = txlayer.verify_dual_proof_v2_batch(sh, th, md, incl, cons, S, T, sa, ta, ctx=ctx)
        exp = [orc.verify_dual_proof_v2(sh[k], th[k], md, [x.tobytes() for x in incl[k]],
                                        [x.tobytes() for x in cons[k]], int(S[k]), int(T[k]),
                                        sa[k], ta[k]) for k in range(len(msgs))]
        assert list(vs) == exp == [0] * len(msgs), name
        n_ok += len(msgs)
        flip = [k for k in range(len(msgs)) if len(incl[k])]
        if flip:
            k = flip[0]
            incl[k] = incl[k].copy()
            incl[k][0, 0] ^= 1
            vs = txlayer.verify_dual_proof_v2_batch(sh, th, md, incl, cons, S, T, sa, ta, ctx=ctx)
            assert vs[k] != 0 and (np.delete(vs, k) == 0).all(), name
    assert n_ok > 10


def test_decode_capacity_and_arguments(m, ctx, wire):
    """The C-ABI's two phases: short term capacity -> BUFFER_TOO_SMALL with
    the offsets and statuses filled (the size query), then the write; bad
    offsets -> ILLEGAL_ARGUMENTS; n = 0 -> OK."""
    from immustore_amd import _native as N
    from immustore_amd.merkle import _addr
    from immustore_amd.txlayer import TX_HEADER
    rng = np.random.default_rng(5)
    raws = [random_msg(wire, rng) for _ in range(50)]
    n = len(raws)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in raws])
    buf = np.frombuffer(b"".join(raws), np.uint8).copy()
    sh, th = np.zeros(n, TX_HEADER), np.zeros(n, TX_HEADER)
    md = np.zeros(2 * n * 268, np.uint8)
    io, co = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.int32)
    L, h = N.load(), ctx.handle

    def call(it, icap, ct, ccap, o=off):
        return L.mh_dual_proof_v2_pb_decode_batch(h, n, _addr(buf), _addr(o), _addr(sh), _addr(th),
                                                  _addr(md), _addr(io), _addr(it), icap, _addr(co),
                                                  _addr(ct), ccap, _addr(st))
    assert call(None, 0, None, 0) == 19
    ti, tc = int(io[n]), int(co[n])
    exp = [sum(1 for _ in wire.MSG["DualProofV2"].FromString(r).inclusionProof) for r in raws]
    assert list(np.diff(io)) == exp and ti > 0 and tc > 0
    it, ct = np.zeros((ti, 32), np.uint8), np.zeros((tc, 32), np.uint8)
    assert call(it, ti - 1, ct, tc) == 19
    assert call(it, ti, ct, tc - 1) == 19
    assert call(it, ti, ct, tc) == 0
    check(wire, raws, (st, sh, th, md.tobytes(), io, it, co, ct))
    bad = off.copy()
    bad[3], bad[4] = bad[4], bad[3]
    if bad[3] != bad[4]:
        assert call(it, ti, ct, tc, bad) == 2
    assert L.mh_dual_proof_v2_pb_decode_batch(h, 0, None, _addr(off), None, None, None, _addr(io),
                                              None, 0, _addr(co), None, 0, None) == 0


# ------------------------------------------------------------ InclusionProof
def go_verify_inclusion(leaf, width, terms, digest, root):
    """htree.VerifyInclusion (htree.go:166-195) with Go's int arithmetic
    (truncating / and %), in Python: the checker for negative leaf / width."""
    import hashlib
    calc = hashlib.sha256(b"\0" + digest).digest()
    i, r = leaf, width - 1
    tdiv = lambda x: -((-x) // 2) if x < 0 else x // 2  # noqa: E731
    for t in terms:
        if i % 2 == 0 and i != r:
            calc = hashlib.sha256(b"\1" + calc + t).digest()
        else:
            calc = hashlib.sha256(b"\1" + t + calc).digest()
        i, r = tdiv(i), tdiv(r)
    return i == r and calc == root


def random_incl_msg(wire, rng):
    M = wire.MSG["InclusionProof"]()
    if rng.random() < 0.9:
        M.leaf = int(rng.choice([0, 1, 5, (1 << 31) - 1, -1, -2, -(1 << 31)]) if rng.random() < 0.3
                     else rng.integers(0, 1 << 24))
    if rng.random() < 0.9:
        M.width = int(rng.choice([0, 1, 2, -1, -(1 << 31)]) if rng.random() < 0.3
                      else rng.integers(1, 1 << 24))
    for _ in range(int(rng.integers(0, 26))):
        M.terms.append(bytes(rng.integers(0, 256, int(rng.choice([32, 32, 32, 0, 7, 33])),
                                          dtype=np.uint8)))
    raw = M.SerializeToString()
    r = rng.random()
    if r < 0.1:
        raw += tag(9, 0) + bytes([1]) + tag(10, 3) + tag(1, 2) + bytes([0]) + tag(10, 4)
    elif r < 0.2:
        raw += tag(1, 0) + bytes([0xff] * 9 + [1])  # leaf again (last wins), 10-byte varint
    elif r < 0.25:
        raw = tag(3, 0) + bytes([3]) + raw  # terms with the wrong wire type: skipped
    return raw


def expect_incl(wire, raw):
    from google.protobuf.message import DecodeError
    if not _go_varints_ok(raw, "incl"):
        return 14, None
    try:
        mm = wire.MSG["InclusionProof"].FromString(raw)
    except DecodeError:
        return 14, None
    return 0, (mm.leaf, mm.width, [d32(x) for x in mm.terms])


def test_inclusion_decode_random_vs_protobuf(m, ctx, wire):
    rng = np.random.default_rng(404)
    raws = [random_incl_msg(wire, rng) for _ in range(3000)]
    for raw in list(raws[:600]):
        b = bytearray(raw or b"\x08")
        if rng.random() < 0.5:
            raws.append(bytes(b[:int(rng.integers(0, len(b)))]))
        else:
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            raws.append(bytes(b))
    raws += [b"", tag(1, 0) + bytes([0x80] * 9 + [2]), tag(2, 0) + bytes([0xff] * 5 + [0x0f])]
    st, proofs = m.decode_inclusion_proof_pb(raws, ctx=ctx)
    seen = set()
    for k, raw in enumerate(raws):
        est, e = expect_incl(wire, raw)
        assert int(st[k]) == est, (k, raw.hex())
        seen.add(est)
        if est == 0:
            p = proofs[k]
            assert (p.leaf, p.width, p.terms) == e, k
        else:
            assert proofs[k] is None
    assert seen == {0, 14}


def test_inclusion_decode_then_verify(m, ctx, orc):
    """InclusionProof messages written on the device (HTree.inclusion_proof_pb_batch)
    decode back to the proofs the tree gives, and every one verifies on the
    device; a flipped term or a wrong leaf does not."""
    rng = np.random.default_rng(8)
    for w in [1, 2, 3, 1000, (1 << 17) + 5]:
        d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
        h = m.HTree(w, ctx)
        h.build_with(d)
        root = h.root()
        leaves = np.concatenate([rng.integers(0, w, 300), [0, w - 1]]).astype(np.uint64)
        msgs, st = h.inclusion_proof_pb_batch(leaves)
        assert (st == 0).all()
        dst, proofs = m.decode_inclusion_proof_pb(msgs, ctx=ctx)
        assert (dst == 0).all()
        for k in (0, 1, len(leaves) - 1):
            want = h.inclusion_proof(int(leaves[k]))
            assert (proofs[k].leaf, proofs[k].width, proofs[k].terms) == (want.leaf, want.width, want.terms)
        dig = d[leaves.astype(int)]
        ok = m.verify_inclusion_batch(proofs, dig, [root] * len(proofs), ctx=ctx)
        assert ok.all(), w
        if w > 2:
            bad = [m.InclusionProof(p.leaf, p.width, [bytes([p.terms[0][0] ^ 1]) + p.terms[0][1:]] + p.terms[1:])
                   for p in proofs[:20]]
            bad += [m.InclusionProof(p.leaf ^ 1, p.width, p.terms) for p in proofs[20:40]]
            # a changed leaf can still verify where Go's walk takes the same
            # branches (e.g. leaf 3 of width 3): the restatement decides
            exp = [go_verify_inclusion(p.leaf, p.width, p.terms, dig[k].tobytes(), root)
                   for k, p in enumerate(bad)]
            assert not any(exp[:20])
            assert list(m.verify_inclusion_batch(bad, dig[:40], [root] * 40, ctx=ctx)) == exp


def test_inclusion_verify_negative_leaf_width(m, ctx, orc, wire):
    """Wire proofs may carry negative int32 leaf / width (Go ints after
    InclusionProofFromProto); VerifyInclusion then runs Go's signed arithmetic.
    Roots are computed with the Python restatement, so some of these verify only
    under signed semantics (leaf -2, width 1, two terms)."""
    import hashlib
    rng = np.random.default_rng(12)
    cases = []
    for leaf, width, nt in [(-2, 1, 2), (-1, 0, 1), (-5, -3, 3), (-(1 << 31), 4, 31), (3, -7, 4),
                            (-2, 1, 1), (6, 7, 3), (-3, -3, 2)]:
        digest = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        terms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(nt)]
        # the root the proof's own hash walk yields
        calc = hashlib.sha256(b"\0" + digest).digest()
        i, r = leaf, width - 1
        for t in terms:
            calc = hashlib.sha256(b"\1" + (calc + t if i % 2 == 0 and i != r else t + calc)).digest()
            i, r = (-((-i) // 2) if i < 0 else i // 2), (-((-r) // 2) if r < 0 else r // 2)
        for root in (calc, bytes(32)):
            cases.append((leaf, width, terms, digest, root))
    msgs = [wire.MSG["InclusionProof"](leaf=c[0], width=c[1], terms=c[2]).SerializeToString()
            for c in cases]
    st, proofs = m.decode_inclusion_proof_pb(msgs, ctx=ctx)
    assert (st == 0).all()
    assert [(p.leaf, p.width) for p in proofs] == [(c[0], c[1]) for c in cases]
    ok = m.verify_inclusion_batch(proofs, [c[3] for c in cases], [c[4] for c in cases], ctx=ctx)
    exp = [go_verify_inclusion(*c) for c in cases]
    orc_ok = [orc.htree_verify_inclusion(c[0] & 0xFFFFFFFFFFFFFFFF, c[1] & 0xFFFFFFFFFFFFFFFF,
                                         c[2], c[3], c[4]) for c in cases]
    assert list(ok) == exp == orc_ok
    assert exp[0] and sum(exp) >= 4  # (-2, 1) verifies: signed arithmetic


# ------------------------------------------------------------ DualProof (v1)
def dual_v1_msg(wire, a):
    """DualProofToProto (database_protoconv.go:131-142, LinearProofToProto,
    LinearAdvanceProofToProto) of orc.verify_dual_proof arguments -> bytes"""
    from test_gpu_formats import _rec_hdr
    sh, th, blob, incl, cons, tbl, last, lin, lap = a[:9]
    M = wire.MSG["DualProof"]()
    M.sourceTxHeader.CopyFrom(wire.tx_header_msg(_rec_hdr(sh, blob))[1])
    M.targetTxHeader.CopyFrom(wire.tx_header_msg(_rec_hdr(th, blob))[1])
    M.inclusionProof.extend(incl)
    M.consistencyProof.extend(cons)
    M.targetBlTxAlh = tbl
    M.lastInclusionProof.extend(last)
    if lin is not None:
        M.linearProof.SetInParent()
        M.linearProof.sourceTxId, M.linearProof.TargetTxId = lin[0], lin[1]
        M.linearProof.terms.extend(lin[2])
    if lap is not None:
        M.LinearAdvanceProof.SetInParent()
        M.LinearAdvanceProof.linearProofTerms.extend(lap[0])
        for ip in lap[1]:
            M.LinearAdvanceProof.inclusionProofs.add(terms=ip)
    return M.SerializeToString()


def test_dual_v1_decode_then_verify_fixture_cases(m, ctx, orc, wire, fixtures):
    """The Go stores' v1 DualProofs (with tampered linear, linear-advance, last
    inclusion and TargetBlTxAlh parts) marshalled as DualProof messages, decoded
    on the device, verified straight from the decoded arrays: the verdicts are
    the oracle's on the original proofs."""
    from immustore_amd import txlayer
    from test_tx_oracle import dual_v1_args
    from tx_util import headers_from_fixture
    args = []
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        for c in fx["dual_v1"]:
            for tamper in (None, "lap", "lin", "last", "tbl"):
                args.append(dual_v1_args(c, recs, blob, alhs, tamper))
    msgs = [dual_v1_msg(wire, a) for a in args]
    st, dec = txlayer.decode_dual_proof_pb(msgs, ctx=ctx)
    assert (st == 0).all()
    for k in range(0, len(args), 37):  # decoded arrays == the proof's parts
        a = args[k]
        assert dec["src_hdr"][k].tobytes()[:128] == np.asarray(a[0]).tobytes()[:128]
        assert dec["target_bl_tx_alh"][k].tobytes() == a[5]
        lo = dec["linear_off"]
        assert [x.tobytes() for x in dec["linear_terms"][int(lo[k]):int(lo[k + 1])]] == a[7][2]
        assert (int(dec["linear_src"][k]), int(dec["linear_tgt"][k])) == a[7][:2]
        assert bool(dec["has_advance"][k]) == (a[8] is not None)
    ok = txlayer.verify_decoded_dual_proof_batch(dec, [a[9] for a in args], [a[10] for a in args],
                                                 [a[11] for a in args], [a[12] for a in args],
                                                 ctx=ctx)
    exp = [orc.verify_dual_proof(*a) for a in args]
    assert list(ok) == exp
    assert sum(exp) > 400 and not all(exp)


def random_dual_v1_msg(wire, rng):
    M = wire.MSG["DualProof"]()
    rb = lambda: bytes(rng.integers(0, 256, int(rng.choice([32, 32, 32, 0, 9, 40])),  # noqa: E731
                                    dtype=np.uint8))

    def hdr(h):
        h.id = int(rng.integers(0, 1 << 40))
        h.blTxId = int(rng.integers(0, 1 << 40))
        h.version = int(rng.choice([0, 1, 2]))
        h.nentries = int(rng.integers(-5, 1 << 20))
        h.prevAlh, h.eH, h.blRoot = rb(), rb(), rb()
        if rng.random() < 0.4:
            h.metadata.truncatedTxID = int(rng.integers(0, 1 << 30))
            if rng.random() < 0.5:
                h.metadata.extra = rb()
    if rng.random() < 0.95:
        hdr(M.sourceTxHeader)
    if rng.random() < 0.95:
        hdr(M.targetTxHeader)
    for fld in (M.inclusionProof, M.consistencyProof, M.lastInclusionProof):
        fld.extend(rb() for _ in range(int(rng.integers(0, 12))))
    if rng.random() < 0.8:
        M.targetBlTxAlh = rb()
    if rng.random() < 0.9:
        M.linearProof.SetInParent()
        M.linearProof.sourceTxId = int(rng.integers(0, 1 << 40))
        M.linearProof.TargetTxId = int(rng.integers(0, 1 << 40))
        M.linearProof.terms.extend(rb() for _ in range(int(rng.integers(0, 10))))
    if rng.random() < 0.6:
        M.LinearAdvanceProof.SetInParent()
        M.LinearAdvanceProof.linearProofTerms.extend(rb() for _ in range(int(rng.integers(0, 6))))
        for _ in range(int(rng.integers(0, 5))):
            ip = M.LinearAdvanceProof.inclusionProofs.add(leaf=int(rng.integers(-3, 100)),
                                                           width=int(rng.integers(0, 100)))
            ip.terms.extend(rb() for _ in range(int(rng.integers(0, 6))))
    raw = M.SerializeToString()
    r = rng.random()
    if r < 0.1:  # unknown fields at the top, a group inside
        raw += tag(20, 2) + bytes([2, 8, 1]) + tag(21, 3) + tag(3, 5) + bytes(4) + tag(21, 4)
    elif r < 0.2:  # a second LinearAdvanceProof occurrence: merged (lists appended)
        la = wire.MSG["LinearAdvanceProof"](linearProofTerms=[bytes(range(32))])
        la.inclusionProofs.add(terms=[bytes(32), b"x"])
        b = la.SerializeToString()
        raw += tag(8, 2) + bytes([len(b)]) + b
    elif r < 0.3:  # a second LinearProof occurrence: ids replaced, terms appended
        lp = wire.MSG["LinearProof"](sourceTxId=7, terms=[bytes(range(1, 33))])
        b = lp.SerializeToString()
        raw += tag(7, 2) + bytes([len(b)]) + b
    return raw


def expect_v1(wire, raw):
    from google.protobuf.message import DecodeError
    if not _go_varints_ok(raw, "top1"):
        return 14, None
    try:
        M = wire.MSG["DualProof"].FromString(raw)
    except DecodeError:
        return 14, None
    ok = M.HasField("sourceTxHeader") and M.HasField("targetTxHeader") and M.HasField("linearProof")
    e = {"incl": [d32(x) for x in M.inclusionProof], "cons": [d32(x) for x in M.consistencyProof],
         "last": [d32(x) for x in M.lastInclusionProof], "tbl": d32(M.targetBlTxAlh),
         "has_linear": M.HasField("linearProof"), "has_advance": M.HasField("LinearAdvanceProof"),
         "linear": (M.linearProof.sourceTxId, M.linearProof.TargetTxId,
                    [d32(x) for x in M.linearProof.terms]),
         "advance": [d32(x) for x in M.LinearAdvanceProof.linearProofTerms],
         "nested": [[d32(x) for x in ip.terms] for ip in M.LinearAdvanceProof.inclusionProofs],
         "src_id": M.sourceTxHeader.id, "tgt_bl": M.targetTxHeader.blTxId}
    return (0 if ok else 2), e


def test_dual_v1_decode_random_vs_protobuf(m, ctx, wire):
    from immustore_amd import txlayer
    rng = np.random.default_rng(1001)
    raws = [random_dual_v1_msg(wire, rng) for _ in range(1500)]
    for raw in list(raws[:400]):
        b = bytearray(raw)
        if rng.random() < 0.5:
            raws.append(bytes(b[:int(rng.integers(0, len(b)))]))
        else:
            for _ in range(int(rng.integers(1, 3))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            raws.append(bytes(b))
    raws += [b"", tag(7, 2) + bytes([0]) + tag(1, 2) + bytes([0]) + tag(2, 2) + bytes([0])]
    st, d = txlayer.decode_dual_proof_pb(raws, ctx=ctx)
    seen = set()

    def terms(name, k):
        o = d[name + "_off"]
        return [x.tobytes() for x in d[name + "_terms"][int(o[k]):int(o[k + 1])]]

    for k, raw in enumerate(raws):
        est, e = expect_v1(wire, raw)
        assert int(st[k]) == est, (k, raw.hex())
        seen.add(est)
        if est == 14:
            assert all(int(d[t + "_off"][k]) == int(d[t + "_off"][k + 1])
                       for t in ("incl", "cons", "last", "linear", "advance"))
            continue
        assert terms("incl", k) == e["incl"] and terms("cons", k) == e["cons"], k
        assert terms("last", k) == e["last"] and terms("advance", k) == e["advance"], k
        assert d["target_bl_tx_alh"][k].tobytes() == e["tbl"], k
        assert bool(d["has_linear"][k]) == e["has_linear"], k
        assert bool(d["has_advance"][k]) == e["has_advance"], k
        assert (int(d["linear_src"][k]), int(d["linear_tgt"][k]), terms("linear", k)) == e["linear"], k
        q0, q1 = int(d["advance_incl_first"][k]), int(d["advance_incl_first"][k + 1])
        qo, qt = d["advance_incl_off"], d["advance_incl_terms"]
        got = [[x.tobytes() for x in qt[int(qo[q]):int(qo[q + 1])]] for q in range(q0, q1)]
        assert got == e["nested"], k
        assert int(d["src_hdr"][k]["id"]) == e["src_id"] and int(d["tgt_hdr"][k]["bl_tx_id"]) == e["tgt_bl"]
    assert seen == {0, 2, 14}


# ------------------------------------------- DualProofV2 from the wire, verified
def _compose(txlayer, msgs, S, T, SA, TA, ctx):
    """decode, then mh_verify_dual_proof_v2_batch, with Go's v0 rule (a v0
    header's metadata is not hashed): the fused call must agree"""
    dst, sh, th, md, io, it, co, ct = txlayer.decode_dual_proof_v2_pb(msgs, ctx=ctx)
    for h in (sh, th):
        h["md_len"][h["version"] == 0] = 0
    incl = [it[int(io[k]):int(io[k + 1])] for k in range(len(msgs))]
    cons = [ct[int(co[k]):int(co[k + 1])] for k in range(len(msgs))]
    vs = txlayer.verify_dual_proof_v2_batch(sh, th, md, incl, cons, S, T, SA, TA, ctx=ctx)
    return np.where(dst != 0, dst, vs)


def test_verify_from_wire_fixture_stores(m, ctx, fixtures):
    """mh_verify_dual_proof_v2_pb_batch over the device-written DualProofV2
    messages of the Go stores: every proof verifies; flipped message bytes,
    wrong ids / Alh and swapped source / target give the decode-then-verify
    composition's verdicts."""
    from immustore_amd import txlayer
    from tx_util import headers_from_fixture
    rng = np.random.default_rng(3)
    seen = set()
    for name, fx in fixtures.items():
        pay = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
        t = m.AHtree(ctx)
        t.append_batch(pay)
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        cases = [(c["src"], c["tgt"]) for c in fx["dual_v2"] if c["src"] <= c["tgt"]]
        S = np.array([a for a, _ in cases], np.uint64)
        T = np.array([b for _, b in cases], np.uint64)
        msgs, st = t.dual_proof_v2_pb_batch(recs[S.astype(int) - 1], recs[T.astype(int) - 1], blob)
        SA = [alhs[int(x) - 1] for x in S]
        TA = [alhs[int(x) - 1] for x in T]
        fused = txlayer.verify_dual_proof_v2_pb_batch(msgs, S, T, SA, TA, ctx=ctx)
        assert (fused == 0).all(), name
        # variants: flipped bytes, wrong target id, zero source Alh, swapped pair
        M2, S2, T2, SA2, TA2 = [], [], [], [], []
        for k, msg in enumerate(msgs):
            for v in range(4):
                b = bytearray(msg)
                s_, t_, sa, ta = int(S[k]), int(T[k]), SA[k], TA[k]
                if v == 0:
                    for _ in range(2):
                        b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
                elif v == 1:
                    t_ += 1
                elif v == 2:
                    sa = bytes(32)
                else:
                    s_, t_, sa, ta = t_, s_, ta, sa
                M2.append(bytes(b))
                S2.append(s_)
                T2.append(t_)
                SA2.append(sa)
                TA2.append(ta)
        fused = txlayer.verify_dual_proof_v2_pb_batch(M2, S2, T2, SA2, TA2, ctx=ctx)
        comp = _compose(txlayer, M2, S2, T2, SA2, TA2, ctx)
        assert list(fused) == list(comp), name
        seen |= set(comp.tolist())
    assert len(seen) >= 3


def test_verify_from_wire_random_vs_composition(m, ctx, orc, wire):
    """Messages over a 70 000-append tree with random headers (every metadata
    shape) plus random protobuf-built and mutated ones: the fused call equals
    decode + mh_verify_dual_proof_v2_batch on every message."""
    from immustore_amd import txlayer
    from test_gpu_formats import _random_headers
    rng = np.random.default_rng(44)
    N_TX = 70000
    t = m.AHtree(ctx)
    t.append_batch(rng.integers(0, 256, (N_TX, 32), dtype=np.uint8))
    recs, blob = _random_headers(rng, N_TX + 10)
    tgt = rng.integers(1, N_TX + 1, 1500)
    src = np.array([int(rng.integers(1, x + 1)) for x in tgt])
    msgs, st = t.dual_proof_v2_pb_batch(recs[src - 1], recs[tgt - 1], blob)
    msgs = list(msgs)
    S, T = list(src), list(tgt)
    SA = [orc.tx_header_alh(recs[int(x) - 1], blob)[2] for x in src]
    TA = [orc.tx_header_alh(recs[int(x) - 1], blob)[2] for x in tgt]
    for k in range(500):  # mutated copies
        b = bytearray(msgs[k])
        b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        msgs.append(bytes(b))
        S.append(S[k])
        T.append(T[k])
        SA.append(SA[k])
        TA.append(TA[k])
    for _ in range(500):  # random protobuf messages (ids mostly mismatched)
        msgs.append(random_msg(wire, rng))
        S.append(int(rng.integers(1, 5)))
        T.append(int(rng.integers(1, 5)))
        SA.append(bytes(32))
        TA.append(bytes(32))
    fused = txlayer.verify_dual_proof_v2_pb_batch(msgs, S, T, SA, TA, ctx=ctx)
    comp = _compose(txlayer, msgs, S, T, SA, TA, ctx)
    assert list(fused) == list(comp)
    # the tree's payloads are not these headers' Alh: inclusion fails (12) where
    # the arguments pass; plus ILLEGAL_ARGUMENTS and CORRUPTED_DATA
    assert {2, 12, 14} <= set(comp.tolist())
