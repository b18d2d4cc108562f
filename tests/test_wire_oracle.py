"""The wire-format oracle (oracle/wire.py) on the CPU:
hand-derived protobuf bytes, DualProofV2 messages of the reference's test
stores round-tripped through decode + the oracle's VerifyDualProofV2, and the
Go error cases of ImmuStore.DualProofV2 (immustore.go:2356-2387)."""
import struct

import numpy as np
import pytest

from tx_util import headers_from_fixture


@pytest.fixture(scope="module")
def wire(orc):
    import wire
    return wire


def hdr(h):
    """fixture header (hex strings) -> wire.tx_header_msg input"""
    return {"id": h["id"], "ts": h["ts"], "bltxid": h["bltxid"], "blroot": bytes.fromhex(h["blroot"]),
            "prevalh": bytes.fromhex(h["prevalh"]), "eh": bytes.fromhex(h["eh"]),
            "version": h["version"], "nentries": h["nentries"], "md": bytes.fromhex(h["md"])}


def test_hand_derived_encodings(wire):
    # proto3: zero scalars omitted, tags (field << 3 | wire type), varints
    assert wire.inclusion_proof_pb(0, 1, []) == bytes([0x10, 0x01])
    t = bytes(range(32))
    assert wire.inclusion_proof_pb(3, 300, [t]) == bytes([0x08, 3, 0x10, 0xAC, 0x02, 0x1A, 0x20]) + t
    # int32(width) of 2^31 is negative: a 10-byte two's-complement varint
    assert wire.inclusion_proof_pb(0, 1 << 31, []) == bytes([0x10] + [0x80] * 4 + [0xF8] + [0xFF] * 4
                                                            + [0x01])
    z = bytes(32)
    st, m = wire.tx_header_msg({"id": 1, "ts": 0, "bltxid": 0, "blroot": z, "prevalh": z, "eh": z,
                                "version": 0, "nentries": 0, "md": b""})
    assert st == 0
    # the three digests are always present (Go slices of [32]byte arrays)
    assert m.SerializeToString() == (bytes([0x08, 1, 0x12, 32]) + z + bytes([0x2A, 32]) + z
                                     + bytes([0x3A, 32]) + z)
    # metadata: truncatedTxID attribute (0) and extra attribute (1), tx_metadata.go:145-157
    md = bytes([0]) + struct.pack(">Q", 7) + bytes([1]) + struct.pack(">H", 2) + b"hi"
    st, m = wire.tx_header_msg({"id": 0, "ts": -1, "bltxid": 0, "blroot": z, "prevalh": z, "eh": z,
                                "version": 1, "nentries": 0, "md": md})
    b = m.SerializeToString()
    assert b[:2] == bytes([0x12, 32])  # id 0 omitted
    assert bytes([0x18] + [0xFF] * 9 + [0x01]) in b  # ts = -1
    assert b.endswith(bytes([0x40, 1, 0x4A, 6, 0x08, 7, 0x12, 2]) + b"hi")


def test_metadata_parse(wire):
    ok = wire.parse_tx_metadata
    assert ok(b"") == (0, None, None)
    assert ok(bytes([1, 0, 0])) == (0, None, b"")
    assert ok(bytes([0]) + bytes(8) + bytes([0]) + struct.pack(">Q", 9)) == (0, 9, None)  # last wins
    for bad in [bytes([2]), bytes([0, 1, 2]), bytes([1, 0]), bytes([1, 0, 5, 1]), bytes(269)]:
        assert ok(bad)[0] == wire.MH_ERR_CORRUPTED_DATA


@pytest.mark.parametrize("store", ["long_linear_proof", "v110_defaultdb", "v110_systemdb"])
def test_dual_proof_v2_fixture_round_trip(orc, wire, fixtures, store):
    fx = fixtures[store]
    aht = orc.AHtree()
    aht.append_batch(np.stack([np.frombuffer(bytes.fromhex(p), np.uint8)
                               for p in fx["aht_payloads"]]))
    hs = [hdr(t["header"]) for t in fx["txs"]]
    recs, blob, alhs = headers_from_fixture(fx["txs"])
    for c in fx["dual_v2"]:
        s, t = c["src"], c["tgt"]
        st, b = wire.dual_proof_v2_pb(hs[s - 1], hs[t - 1], aht)
        assert st == 0
        m = wire.MSG["DualProofV2"].FromString(b)
        assert [x.hex() for x in m.inclusionProof] == c["incl"]
        assert [x.hex() for x in m.consistencyProof] == c["cons"]
        for mh, h in ((m.sourceTxHeader, hs[s - 1]), (m.targetTxHeader, hs[t - 1])):
            assert (mh.id, mh.ts, mh.blTxId, mh.nentries, mh.version) == \
                (h["id"], h["ts"], h["bltxid"], h["nentries"], h["version"])
            assert (mh.prevAlh, mh.eH, mh.blRoot) == (h["prevalh"], h["eh"], h["blroot"])
            assert not mh.HasField("metadata")
        # the decoded proof verifies against the stored Alh values
        assert orc.verify_dual_proof_v2(recs[s - 1], recs[t - 1], blob, list(m.inclusionProof),
                                        list(m.consistencyProof), s, t, alhs[s - 1],
                                        alhs[t - 1]) == 0


def test_dual_proof_v2_errors(orc, wire, fixtures):
    fx = fixtures["long_linear_proof"]
    aht = orc.AHtree()
    aht.append_batch(np.stack([np.frombuffer(bytes.fromhex(p), np.uint8)
                               for p in fx["aht_payloads"]]))
    hs = [hdr(t["header"]) for t in fx["txs"]]
    assert wire.dual_proof_v2_pb(dict(hs[0], id=0), hs[3], aht)[0] == wire.MH_ERR_ILLEGAL_ARGUMENTS
    assert wire.dual_proof_v2_pb(hs[5], hs[3], aht)[0] == wire.MH_ERR_SOURCE_TX_NEWER
    assert wire.dual_proof_v2_pb(hs[2], dict(hs[5], bltxid=3), aht)[0] == \
        wire.MH_ERR_UNEXPECTED_LINKING
    far = dict(hs[-1], id=len(fx["aht_payloads"]) + 5, bltxid=len(fx["aht_payloads"]) + 4)
    assert wire.dual_proof_v2_pb(hs[2], far, aht)[0] == wire.MH_ERR_UNEXISTENT_DATA
    st, b = wire.dual_proof_v2_pb(hs[4], hs[4], aht)  # same tx: headers only
    m = wire.MSG["DualProofV2"].FromString(b)
    assert st == 0 and not m.inclusionProof and not m.consistencyProof


def test_htree_inclusion_proof_pb(orc, wire):
    rng = np.random.default_rng(8)
    for w in [1, 2, 3, 5, 64, 1000]:
        d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
        lv, root = orc.htree_build(d)
        for i in sorted({0, w - 1, w // 2}):
            st, b = wire.htree_inclusion_proof_pb(lv, w, i)
            assert st == 0
            m = wire.MSG["InclusionProof"].FromString(b)
            assert (m.leaf, m.width) == (i, w)
            assert orc.htree_verify_inclusion(i, w, list(m.terms), d[i].tobytes(), root)
        assert wire.htree_inclusion_proof_pb(lv, w, w)[0] == wire.MH_ERR_ILLEGAL_ARGUMENTS


def test_wire_descriptor_matches_reference_generated_descriptor():
    """oracle/wire.py's hand-declared messages == the reference's own compiled
    descriptor (pkg/api/schema/schema.pb.go file_schema_proto_rawDesc, decoded
    by tests/golden/make_golden.py into schema_fields.json): every field's
    name, number, type, label and message type."""
    import json
    import os
    import wire
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "schema_fields.json")))
    assert ref["package"] == "immudb.schema" and ref["syntax"] == "proto3"
    for name, fields in ref["messages"].items():
        from google.protobuf import descriptor_pb2
        d = wire.MSG[name].DESCRIPTOR
        assert d.full_name == "immudb.schema." + name
        dp = descriptor_pb2.DescriptorProto()
        d.CopyToProto(dp)
        got = [[f.name, f.number, f.type, f.label, f.type_name] for f in dp.field]
        assert got == fields, name
    assert set(ref["messages"]) == set(wire.MSG)
