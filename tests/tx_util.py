"""Helpers shared by the tx-layer tests: fixture headers -> TX_HEADER records."""
import struct

import numpy as np

TX_HEADER = np.dtype([("id", "<u8"), ("ts", "<i8"), ("bl_tx_id", "<u8"), ("bl_root", "u1", 32),
                      ("prev_alh", "u1", 32), ("eh", "u1", 32), ("version", "<u4"),
                      ("nentries", "<u4"), ("md_len", "<u4"), ("md_off", "<u4")])


def headers_from_fixture(txs):
    """-> (records[n] of TX_HEADER, md_blob bytes, stored alh[n] as bytes)"""
    recs = np.zeros(len(txs), TX_HEADER)
    blob = bytearray()
    alhs = []
    for k, t in enumerate(txs):
        h = t["header"]
        r = recs[k]
        r["id"], r["ts"], r["bl_tx_id"] = h["id"], h["ts"], h["bltxid"]
        r["bl_root"] = np.frombuffer(bytes.fromhex(h["blroot"]), np.uint8)
        r["prev_alh"] = np.frombuffer(bytes.fromhex(h["prevalh"]), np.uint8)
        r["eh"] = np.frombuffer(bytes.fromhex(h["eh"]), np.uint8)
        r["version"], r["nentries"] = h["version"], h["nentries"]
        md = bytes.fromhex(h["md"])
        r["md_len"], r["md_off"] = len(md), len(blob)
        blob += md
        alhs.append(bytes.fromhex(h["alh"]))
    return recs, bytes(blob), alhs


def inner_hashes(orc, recs, blob):
    return [orc.tx_header_alh(recs[k], blob)[1] for k in range(len(recs))]


def _txmd(rng, kind):
    """TxMetadata.Bytes() (tx_metadata.go:145-157): none, truncatedUptoTx,
    extra (short), or both attributes at the 268-byte maximum."""
    rb = lambda n: bytes(rng.integers(0, 256, n, dtype=np.uint8))  # noqa: E731
    trunc = b"\x00" + rb(8)
    if kind == 2:
        return trunc
    if kind == 3:  # 8..11 bytes: every alignment of what follows it in the header
        n = int(rng.integers(5, 9))
        return b"\x01" + struct.pack(">H", n) + rb(n)
    if kind == 4:
        return trunc + b"\x01" + struct.pack(">H", 256) + rb(256)
    return b""


def _synthetic_txlog(rng, ntx, orc, max_entries=40, version_mix=True, key_len=None):
    """Tx records in the immustore.go:1812-1924 layout with a valid Alh chain
    (the stored alh of each record is the oracle's Alh over its own fields)."""
    out = bytearray()
    prev = orc.sha256(b"")
    for k in range(ntx):
        ver = int(rng.integers(0, 2)) if version_mix else 1
        ne = int(rng.integers(0, max_entries + 1)) if k % 5 else int(rng.integers(1, 3))
        txmd = b"" if ver == 0 else _txmd(rng, k % 5)
        ents, digs = bytearray(), []
        for e in range(ne):
            md = b"" if ver == 0 else [b"", b"\x00", b"\x01" + struct.pack(">Q", e), b"\x02",
                                       b"\x00\x01" + struct.pack(">Q", k) + b"\x02"][(k + e) % 5]
            kl = key_len(k, e) if key_len else int(rng.integers(0, 70))
            key = bytes(rng.integers(0, 256, kl, dtype=np.uint8))
            hv = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
            ents += struct.pack(">H", len(md)) + md + struct.pack(">H", len(key)) + key
            ents += struct.pack(">IQ", int(rng.integers(0, 1 << 20)), int(rng.integers(0, 1 << 40)))
            ents += hv
            digs.append(orc.entry_digest(ver, key, md, hv)[1])
        eh = orc.htree_build(np.frombuffer(b"".join(digs), np.uint8).reshape(-1, 32))[1] if ne \
            else orc.sha256(b"")
        ts, bl = int(rng.integers(0, 1 << 40)), int(rng.integers(0, k + 1))
        blroot = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        st, inner = orc.tx_inner_hash(ts, ver, txmd, ne, eh, bl, blroot)
        assert st == 0
        alh = orc.tx_alh(k + 1, prev, inner)
        hdr = struct.pack(">QQQ", k + 1, ts, bl) + blroot + prev + struct.pack(">H", ver)
        hdr += struct.pack(">H", ne) if ver == 0 else struct.pack(">H", len(txmd)) + txmd + \
            struct.pack(">I", ne)
        out += hdr + ents + alh
        prev = alh
    return bytes(out)


def _bulk_txlog(rng, ntx):
    """A long run of structurally valid records (ragged entry counts, key and
    metadata sizes, v0/v1) with unsealed Alh values: > 8 MiB, so the host
    parse runs on several threads from speculated record starts."""
    out = bytearray()
    starts = []
    for k in range(ntx):
        starts.append(len(out))
        ver = 1 if k % 3 else 0
        ne = int(rng.integers(0, 24))
        txmd = b"" if ver == 0 else bytes([1, 0, k % 7]) + bytes(k % 7)
        hdr = struct.pack(">QQQ", k + 1, 1000 + k, k) + bytes(64) + struct.pack(">H", ver)
        hdr += struct.pack(">H", ne) if ver == 0 else struct.pack(">H", len(txmd)) + txmd + \
            struct.pack(">I", ne)
        ents = bytearray()
        for e in range(ne):
            md = b"" if ver == 0 else bytes([0]) * ((k + e) % 2)
            key = bytes([e % 251]) * int(rng.integers(1, 400))
            ents += struct.pack(">H", len(md)) + md + struct.pack(">H", len(key)) + key
            ents += struct.pack(">IQ", 10, e) + bytes([k % 256]) * 32
        out += hdr + ents + bytes([7]) * 32
    return bytes(out), starts


def document_cases(fixtures, orc, per_store=60, seed=7):
    """VerifyDocument inputs built from the reference's Go-written stores: the
    "document" of tx t is a stored value of one of t's entries whose key is
    unique in t (so SHA256(document) is that entry's stored hVal), proven by a
    fixture DualProofV2 whose source or target is t, with and without a
    known state, plus tampered variants of every check
    (pkg/verification/verification.go:60-194).  -> (docs, md_blob)."""
    rng = np.random.default_rng(seed)
    docs = []
    blob_all = bytearray()
    for name, fx in fixtures.items():
        recs, blob, alhs = headers_from_fixture(fx["txs"])
        recs = recs.copy()
        recs["md_off"] += len(blob_all)
        blob_all += blob
        cases = [c for c in fx["dual_v2"]]
        rng.shuffle(cases)
        made = 0
        for c in cases:
            if made >= per_store:
                break
            s, t = c["src"], c["tgt"]
            tid = [s, t][int(rng.integers(0, 2))]
            ents = fx["txs"][tid - 1]["entries"]
            keys = [e["key"] for e in ents]
            cand = [e for e in ents if e.get("value") is not None and keys.count(e["key"]) == 1]
            if not cand:
                continue
            e = cand[int(rng.integers(0, len(cand)))]
            entries = [(bytes.fromhex(x["key"]), bytes.fromhex(x["md"]), bytes.fromhex(x["hval"]))
                       for x in ents]
            kid = [0, s, t][made % 3]
            base = {"encoded_document": bytes.fromhex(e["value"]),
                    "doc_key": bytes.fromhex(e["key"]), "tx_hdr": recs[tid - 1].copy(),
                    "entries": entries, "src_hdr": recs[s - 1].copy(), "tgt_hdr": recs[t - 1].copy(),
                    "incl": [bytes.fromhex(x) for x in c["incl"]],
                    "cons": [bytes.fromhex(x) for x in c["cons"]],
                    "known_tx_id": kid, "known_alh": alhs[kid - 1] if kid else bytes(32)}
            made += 1
            docs.append(base)
            for v in range(1, 13):
                d = dict(base)
                d["tx_hdr"] = base["tx_hdr"].copy()
                d["src_hdr"] = base["src_hdr"].copy()
                d["tgt_hdr"] = base["tgt_hdr"].copy()
                d["entries"] = list(base["entries"])
                if v == 1:    # document bytes changed: hVal mismatch (:63-67)
                    d["encoded_document"] = base["encoded_document"] + b"x"
                elif v == 2:  # key not in the tx (:74-76)
                    d["doc_key"] = base["doc_key"] + b"\0"
                elif v == 3:  # key twice (:74-76)
                    d["entries"] = d["entries"] + [next(x for x in entries if x[0] == d["doc_key"])]
                elif v == 4:  # Eh changed (:137-139)
                    d["tx_hdr"]["eh"][0] ^= 1
                elif v == 5:  # another entry's hValue changed (:137-139) or the doc's own
                    i = int(rng.integers(0, len(entries)))
                    k_, m_, h_ = d["entries"][i]
                    d["entries"][i] = (k_, m_, bytes([h_[0] ^ 1]) + h_[1:])
                elif v == 6:  # known state names another tx (:170-172)
                    d["known_tx_id"] = t + 1
                    d["known_alh"] = bytes(32)
                elif v == 7:  # known state with a wrong Alh (:174-180)
                    d["known_tx_id"] = s
                    d["known_alh"] = bytes(32)
                elif v == 8:  # no known state (:165-168)
                    d["known_tx_id"] = 0
                elif v == 9 and d["incl"]:  # inclusion term changed
                    d["incl"] = [bytes([d["incl"][0][0] ^ 1]) + d["incl"][0][1:]] + d["incl"][1:]
                elif v == 10:  # the tx is neither source nor target (:153-155)
                    d["tx_hdr"]["id"] = t + 5
                elif v == 11:  # unsupported version (:118-121)
                    d["tx_hdr"]["version"] = 2
                elif v == 12:  # source newer than target (:146-148)
                    d["src_hdr"], d["tgt_hdr"] = base["tgt_hdr"].copy(), base["src_hdr"].copy()
                docs.append(d)
    return docs, bytes(blob_all)


def md_record(orc, txid, prev, ver, txmd_raw, txmd_hash, entries, seal_raw=False):
    """One tx record whose metadata is stored as given (txmd_raw, and per
    entry md_raw) while the Alh is sealed over txmd_hash / md_hash (what Go
    hashes: the re-serialised Bytes(), tx.go:300-319, 703-731), or over the raw
    bytes when seal_raw.  entries: [(md_raw, md_hash, key, hval)].
    -> (record bytes, alh)"""
    digs = []
    ents = bytearray()
    for md_raw, md_hash, key, hv in entries:
        digs.append(orc.entry_digest(ver, key, md_raw if seal_raw else md_hash, hv)[1])
        ents += struct.pack(">H", len(md_raw)) + md_raw + struct.pack(">H", len(key)) + key
        ents += struct.pack(">IQ", 3, 77) + hv
    ne = len(entries)
    eh = orc.htree_build(np.frombuffer(b"".join(digs), np.uint8).reshape(-1, 32))[1] if ne \
        else orc.sha256(b"")
    st, inner = orc.tx_inner_hash(1000 + txid, ver, txmd_raw if seal_raw else txmd_hash, ne, eh,
                                  0, bytes(32))
    assert st == 0
    alh = orc.tx_alh(txid, prev, inner)
    hdr = struct.pack(">QQQ", txid, 1000 + txid, 0) + bytes(32) + prev + struct.pack(">H", ver)
    hdr += struct.pack(">H", ne) if ver == 0 else struct.pack(">H", len(txmd_raw)) + txmd_raw + \
        struct.pack(">I", ne)
    return bytes(hdr + ents + alh), alh


def metadata_logs(orc):
    """Tx logs exercising the metadata parse of the reader: valid but
    non-canonical KV / tx metadata (Go re-serialises it before hashing),
    the same sealed over the raw bytes (an ALH mismatch in Go), and every
    ErrCorruptedData case of KVMetadata.unsafeReadFrom / TxMetadata.ReadFrom.
    -> list of (name, log bytes)"""
    exp = lambda v: b"\x01" + struct.pack(">Q", v)  # noqa: E731
    trunc = lambda v: b"\x00" + struct.pack(">Q", v)  # noqa: E731
    extra = lambda b: b"\x01" + struct.pack(">H", len(b)) + b  # noqa: E731
    key, hv = b"key-1", bytes(range(32))
    noncanon_kv = [(b"\x02\x00", b"\x00\x02"), (b"\x00\x00", b"\x00"), (exp(9) + b"\x00", b"\x00" + exp(9)),
                   (b"\x02" + exp(7) + b"\x00", b"\x00" + exp(7) + b"\x02"), (b"\x02\x02\x02", b"\x02")]
    noncanon_tx = [(extra(b"xyz") + trunc(4), trunc(4) + extra(b"xyz")),
                   (trunc(1) + trunc(2), trunc(2)), (extra(b"a") + extra(b"bc"), extra(b"bc"))]
    bad_kv = [b"\x03", b"\x01" + bytes(4), b"\x00\x07", bytes([0x01]) + bytes(8) + b"\x09"]
    bad_tx = [b"\x05", trunc(1)[:5], b"\x01\x00", extra(b"abc")[:4], b"\x01" + struct.pack(">H", 257)
              + bytes(257)]
    logs = []

    def chain(recs):
        out, prev = bytearray(), orc.sha256(b"")
        for k, (txmd_raw, txmd_hash, ents, seal_raw) in enumerate(recs):
            r, prev = md_record(orc, k + 1, prev, 1, txmd_raw, txmd_hash, ents, seal_raw)
            out += r
        return bytes(out)

    good = (b"", b"", [(b"\x00", b"\x00", key, hv)], False)
    for seal_raw in (False, True):
        recs = [good]
        for raw, canon in noncanon_kv:
            recs.append((b"", b"", [(b"", b"", b"k0", hv), (raw, canon, key, hv)], seal_raw))
        for raw, canon in noncanon_tx:
            recs.append((raw, canon, [(b"\x02", b"\x02", key, hv)], seal_raw))
        recs.append(good)
        logs.append(("noncanonical_sealed_%s" % ("raw" if seal_raw else "canonical"), chain(recs)))
    for k, md in enumerate(bad_kv):
        logs.append(("bad_kv_%d" % k, chain([good, (b"", b"", [(b"", b"", b"a", hv), (md, md, key, hv)],
                                                      True), good])))
    for k, md in enumerate(bad_tx):
        logs.append(("bad_tx_%d" % k, chain([good, (md, md, [], True), good])))
    return logs


def record_spans(raw, n=None):
    """(start, end) of the first n records of a structurally valid tx log
    (immustore.go:1812-1924 layout, parsed in Python), stopping at an id-0
    tail or the end of the buffer."""
    spans, p = [], 0
    while p + 8 <= len(raw) and (n is None or len(spans) < n):
        if struct.unpack_from(">Q", raw, p)[0] == 0:
            break
        ver, = struct.unpack_from(">H", raw, p + 88)
        if ver == 0:
            ne, = struct.unpack_from(">H", raw, p + 90)
            q = p + 92
        else:
            ml, = struct.unpack_from(">H", raw, p + 90)
            ne, = struct.unpack_from(">I", raw, p + 92 + ml)
            q = p + 96 + ml
        for _ in range(ne):
            m_, = struct.unpack_from(">H", raw, q)
            k_, = struct.unpack_from(">H", raw, q + 2 + m_)
            q += 4 + m_ + k_ + 44
        spans.append((p, q + 32))
        p = q + 32
    return spans


def clog_for(raw, spans, es=12):
    """The commit-log entries of those records (txOffsetAndSize,
    immustore.go:2569-2597: BE64 offset || BE32 size, + the stored Alh for the
    44-byte cLogEntrySizeV2, :122-123)."""
    out = bytearray()
    for s, e in spans:
        out += struct.pack(">QI", s, e - s)
        if es == 44:
            out += raw[e - 32:e]
    return bytes(out)
