"""CPU restatement of the proof wire formats.

TEST INFRASTRUCTURE ONLY: the parity oracle for the device protobuf writers
(immustore_amd/csrc/wire_kernels.hip).  Only tests/ may import it.

The reference marshals proofs with protobuf-go after converting them
(pkg/api/schema/database_protoconv.go).  This module declares the same
messages (field names, numbers and types of pkg/api/schema/schema.proto) as a
descriptor for the protobuf runtime in this image (python protobuf, proto3
serialisation in field-number order, as protobuf-go's), rebuilds each proof
with the C oracle (oracle.py) the way the Go server does, and serialises it:

  InclusionProof  schema.proto:534-540, InclusionProofToProto database_protoconv.go:115-121
  DualProofV2     schema.proto:437-445, DualProofV2ToProto    database_protoconv.go:152-159
  TxHeader        schema.proto:349-367, TxHeaderToProto       database_protoconv.go:161-177
  TxMetadata      schema.proto:380-383, TxMetadataToProto     database_protoconv.go:179-193
  DualProof (v1), LinearProof, LinearAdvanceProof  schema.proto:388-434
                  (the decode direction: DualProofFromProto database_protoconv.go:211-224)
  ImmuStore.DualProofV2                                        immustore.go:2356-2387
  TxMetadata.ReadFrom                                          tx_metadata.go:159-195

Parity note: the reference holds no Go-marshalled protobuf bytes for these
messages, so the encoding is pinned by the protobuf wire-format rules as the
python runtime implements them (protobuf 7.x), and the message CONTENT (terms,
headers) by the C oracle, itself pinned by the Go-written fixtures.  The
declarations below are checked field by field (name, number, type, label,
message type) against the reference's own compiled descriptor
(schema.pb.go file_schema_proto_rawDesc, decoded into
tests/golden/schema_fields.json; tests/test_wire_oracle.py).
"""
import struct

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

import oracle as O

MH_OK = 0
MH_ERR_ILLEGAL_ARGUMENTS = 2
MH_ERR_UNEXISTENT_DATA = 5
MH_ERR_SOURCE_TX_NEWER = 10
MH_ERR_UNEXPECTED_LINKING = 11
MH_ERR_CORRUPTED_DATA = 14
MAX_TX_METADATA_LEN = 268  # tx_metadata.go:36-39

_F = descriptor_pb2.FieldDescriptorProto


def _build():
    fdp = descriptor_pb2.FileDescriptorProto(name="immudb_schema_subset.proto",
                                             package="immudb.schema", syntax="proto3")

    def msg(name, fields):
        m = fdp.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = ".immudb.schema." + tname

    O_, R_ = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    msg("TxMetadata", [("truncatedTxID", 1, _F.TYPE_UINT64, O_, None),
                       ("extra", 2, _F.TYPE_BYTES, O_, None)])
    msg("TxHeader", [("id", 1, _F.TYPE_UINT64, O_, None),
                     ("prevAlh", 2, _F.TYPE_BYTES, O_, None),
                     ("ts", 3, _F.TYPE_INT64, O_, None),
                     ("nentries", 4, _F.TYPE_INT32, O_, None),
                     ("eH", 5, _F.TYPE_BYTES, O_, None),
                     ("blTxId", 6, _F.TYPE_UINT64, O_, None),
                     ("blRoot", 7, _F.TYPE_BYTES, O_, None),
                     ("version", 8, _F.TYPE_INT32, O_, None),
                     ("metadata", 9, _F.TYPE_MESSAGE, O_, "TxMetadata")])
    msg("DualProofV2", [("sourceTxHeader", 1, _F.TYPE_MESSAGE, O_, "TxHeader"),
                        ("targetTxHeader", 2, _F.TYPE_MESSAGE, O_, "TxHeader"),
                        ("inclusionProof", 3, _F.TYPE_BYTES, R_, None),
                        ("consistencyProof", 4, _F.TYPE_BYTES, R_, None)])
    msg("InclusionProof", [("leaf", 1, _F.TYPE_INT32, O_, None),
                           ("width", 2, _F.TYPE_INT32, O_, None),
                           ("terms", 3, _F.TYPE_BYTES, R_, None)])
    msg("LinearProof", [("sourceTxId", 1, _F.TYPE_UINT64, O_, None),
                        ("TargetTxId", 2, _F.TYPE_UINT64, O_, None),
                        ("terms", 3, _F.TYPE_BYTES, R_, None)])
    msg("LinearAdvanceProof", [("linearProofTerms", 1, _F.TYPE_BYTES, R_, None),
                               ("inclusionProofs", 2, _F.TYPE_MESSAGE, R_, "InclusionProof")])
    msg("DualProof", [("sourceTxHeader", 1, _F.TYPE_MESSAGE, O_, "TxHeader"),
                      ("targetTxHeader", 2, _F.TYPE_MESSAGE, O_, "TxHeader"),
                      ("inclusionProof", 3, _F.TYPE_BYTES, R_, None),
                      ("consistencyProof", 4, _F.TYPE_BYTES, R_, None),
                      ("targetBlTxAlh", 5, _F.TYPE_BYTES, O_, None),
                      ("lastInclusionProof", 6, _F.TYPE_BYTES, R_, None),
                      ("linearProof", 7, _F.TYPE_MESSAGE, O_, "LinearProof"),
                      ("LinearAdvanceProof", 8, _F.TYPE_MESSAGE, O_, "LinearAdvanceProof")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName("immudb.schema." + n))
    return {n: get(n) for n in ("TxMetadata", "TxHeader", "DualProofV2", "InclusionProof",
                                "DualProof", "LinearProof", "LinearAdvanceProof")}


MSG = _build()


def _i32(x):
    """Go int32(x) of a non-negative int."""
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def parse_tx_metadata(b):
    """TxMetadata.ReadFrom (tx_metadata.go:159-195) -> (status, truncated or None, extra or None)."""
    if len(b) > MAX_TX_METADATA_LEN:
        return MH_ERR_CORRUPTED_DATA, None, None
    i, trunc, extra = 0, None, None
    while i < len(b):
        code = b[i]
        i += 1
        if code == 0:
            if len(b) - i < 8:
                return MH_ERR_CORRUPTED_DATA, None, None
            trunc = struct.unpack(">Q", b[i:i + 8])[0]
            i += 8
        elif code == 1:
            if len(b) - i < 2:
                return MH_ERR_CORRUPTED_DATA, None, None
            ln = struct.unpack(">H", b[i:i + 2])[0]
            if len(b) - i - 2 < ln:
                return MH_ERR_CORRUPTED_DATA, None, None
            extra = bytes(b[i + 2:i + 2 + ln])
            i += 2 + ln
        else:
            return MH_ERR_CORRUPTED_DATA, None, None
    return MH_OK, trunc, extra


def tx_header_msg(h):
    """TxHeaderToProto (database_protoconv.go:161-177).  h: dict with id, ts,
    bltxid, blroot, prevalh, eh (bytes), version, nentries, md (bytes; empty =
    nil Metadata as read from the tx log, tx.go:483-501)."""
    m = MSG["TxHeader"](id=h["id"], prevAlh=h["prevalh"], ts=h["ts"], nentries=_i32(h["nentries"]),
                        eH=h["eh"], blTxId=h["bltxid"], blRoot=h["blroot"],
                        version=_i32(h["version"]))
    if h["md"]:
        st, trunc, extra = parse_tx_metadata(h["md"])
        if st:
            return st, None
        md = MSG["TxMetadata"]()
        if trunc is not None:
            md.truncatedTxID = trunc
        if extra is not None:
            md.extra = extra
        m.metadata.CopyFrom(md)
    return MH_OK, m


def dual_proof_v2_pb(src, tgt, aht):
    """ImmuStore.DualProofV2 (immustore.go:2356-2387) over the oracle ahtree
    `aht`, then DualProofV2ToProto + Marshal -> (status, bytes)."""
    if src["id"] == 0:
        return MH_ERR_ILLEGAL_ARGUMENTS, b""
    if src["id"] > tgt["id"]:
        return MH_ERR_SOURCE_TX_NEWER, b""
    if src["id"] - 1 != src["bltxid"] or tgt["id"] - 1 != tgt["bltxid"]:
        return MH_ERR_UNEXPECTED_LINKING, b""
    incl, cons = [], []
    if src["id"] < tgt["id"]:
        st, t = aht.inclusion_proof(src["id"], tgt["bltxid"])
        if st:
            return st, b""
        incl = [bytes(x) for x in t]
        st, t = aht.consistency_proof(max(1, src["bltxid"]), tgt["bltxid"])
        if st:
            return st, b""
        cons = [bytes(x) for x in t]
    st, hs = tx_header_msg(src)
    if st:
        return st, b""
    st, ht = tx_header_msg(tgt)
    if st:
        return st, b""
    m = MSG["DualProofV2"](inclusionProof=incl, consistencyProof=cons)
    m.sourceTxHeader.CopyFrom(hs)
    m.targetTxHeader.CopyFrom(ht)
    return MH_OK, m.SerializeToString()


def inclusion_proof_pb(leaf, width, terms):
    """InclusionProofToProto (database_protoconv.go:115-121) + Marshal."""
    return MSG["InclusionProof"](leaf=_i32(leaf), width=_i32(width),
                                 terms=[bytes(x) for x in terms]).SerializeToString()


def htree_inclusion_proof_pb(levels, width, leaf):
    """(*HTree).InclusionProof (htree.go:121-164) via the C oracle, encoded."""
    if leaf >= width:
        return MH_ERR_ILLEGAL_ARGUMENTS, b""
    st, terms = O.htree_inclusion_proof(levels, width, leaf)
    if st:
        return st, b""
    return MH_OK, inclusion_proof_pb(leaf, width, terms)
