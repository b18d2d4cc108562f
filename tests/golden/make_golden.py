#!/usr/bin/env python3
"""Generate the committed golden vectors under tests/golden/.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (`immustore_amd/`) imports
this file.  It is run once, in the build container where `/root/reference`
exists, and its JSON outputs are committed so that the GPU box (which has no
`/root/reference`) can check parity.

Two kinds of vectors are produced:

1. `immudb_fixtures.json` -- values parsed out of the Go-written on-disk stores
   shipped with the reference (`test/data_long_linear_proof`,
   `test/data_v1.1.0/{defaultdb,systemdb}`).  These are *data*: tx headers,
   entries (key, KV metadata bytes, value, hVal), the Alh stored by Go after
   every tx, the ahtree payload stream and the ahtree dLog digest stream.  They
   pin the SHA-256 boundary, the v0/v1 entry digests, htree, the tx header
   inner hash / Alh and the ahtree dLog bit-exactly against Go output.

2. `synthetic.json` -- wider cases computed by the small pure-Python
   restatement below (hashlib SHA-256).  The restatement is first checked
   against (1) (this script asserts it), so these vectors inherit the pin.

File formats followed (reference, read as text):
- appendable file header: 4-byte BE metadata length + metadata
  (embedded/appendable/singleapp/single_app.go:116-212)
- tx record: embedded/store/immustore.go:1812-1924 and tx.go:437-603
- ahtree pLog record: BE32 len + payload (embedded/ahtree/ahtree.go:266-279)
- ahtree dLog: 32-byte digests (ahtree.go:324-333)
- ahtree cLog entry: BE64 pLog offset + BE32 payload len (ahtree.go:341-345)
"""
import hashlib
import json
import os
import struct
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def sha(b):
    return hashlib.sha256(b).digest()


# ---------------------------------------------------------------- restatement
def htree_build(digests):
    """embedded/htree/htree.go:68-113 -> (levels, root)."""
    if not digests:
        return [], sha(b"")
    lv = [[sha(b"\x00" + d) for d in digests]]
    while len(lv[-1]) > 1:
        cur, nxt = lv[-1], []
        for i in range(0, len(cur) - 1, 2):
            nxt.append(sha(b"\x01" + cur[i] + cur[i + 1]))
        if len(cur) % 2 == 1:
            nxt.append(cur[-1])
        lv.append(nxt)
    return lv, lv[-1][0]


def bitlen(x):
    return x.bit_length()


def htree_inclusion_proof(levels, width, i):
    """embedded/htree/htree.go:121-164."""
    m, n, offset, terms = i, width, 0, []
    if width == 1:
        return terms
    while True:
        d = bitlen(n - 1)
        k = 1 << (d - 1)
        if m < k:
            l, r = offset + k, offset + n - 1
            n = k
        else:
            l, r = offset, offset + k - 1
            m, n = m - k, n - k
            offset += k
        layer = bitlen(r - l)
        index = l // (1 << layer)
        terms.insert(0, levels[layer][index])
        if n < 1 or (n == 1 and m == 0):
            return terms


def htree_verify(leaf, width, terms, digest, root):
    """embedded/htree/htree.go:166-195."""
    calc = sha(b"\x00" + digest)
    i, r = leaf, width - 1
    for t in terms:
        if i % 2 == 0 and i != r:
            calc = sha(b"\x01" + calc + t)
        else:
            calc = sha(b"\x01" + t + calc)
        i //= 2
        r //= 2
    return i == r and calc == root


def entry_digest(version, key, md, hval):
    """embedded/store/tx.go:690-731."""
    if version == 0:
        if md:
            raise ValueError("metadata unsupported")
        return sha(key + hval)
    return sha(struct.pack(">H", len(md)) + md + struct.pack(">H", len(key)) + key + hval)


def inner_hash(h):
    """embedded/store/tx.go:249-302."""
    b = struct.pack(">QH", h["ts"], h["version"])
    if h["version"] == 0:
        b += struct.pack(">H", h["nentries"])
    else:
        md = bytes.fromhex(h["md"])
        b += struct.pack(">H", len(md)) + md + struct.pack(">I", h["nentries"])
    b += bytes.fromhex(h["eh"]) + struct.pack(">Q", h["bltxid"]) + bytes.fromhex(h["blroot"])
    return sha(b)


def alh(h):
    """embedded/store/tx.go:307-319."""
    return sha(struct.pack(">Q", h["id"]) + bytes.fromhex(h["prevalh"]) + inner_hash(h))


def nodes_upto(n):
    """embedded/ahtree/ahtree.go:492-511 (closed form: n + sum popcount(i<n))."""
    o, l = n, 0
    while n >= (1 << l):
        o += (n >> (l + 1)) << l
        if (n >> l) % 2 == 1:
            o += n % (1 << l)
        l += 1
    return o


def nodes_until(n):
    return 0 if n == 1 else nodes_upto(n - 1)


class AHT:
    """In-memory restatement of embedded/ahtree/ahtree.go:246-373,460-771."""

    def __init__(self):
        self.dlog = []
        self.n = 0

    def node(self, k, l):
        return self.dlog[nodes_until(k) + l]

    def append(self, d):
        n = self.n + 1
        h = sha(b"\x00" + d)
        out = [h]
        w, l, k = n - 1, 0, n - 1
        while w > 0:
            if w % 2 == 1:
                h = sha(b"\x01" + self.node(k, l) + h)
                out.append(h)
            k &= ~(1 << l)
            w >>= 1
            l += 1
        self.dlog.extend(out)
        self.n = n
        return h

    def levels_at(self, n):
        return bin(n - 1).count("1")

    def root_at(self, n):
        return self.dlog[nodes_until(n) + self.levels_at(n)]

    def highest_node(self, i, d):
        l = sum(1 for r in range(d - 1, -1, -1) if (i - 1) & (1 << r))
        return self.node(i, l)

    def inclusion_proof(self, i, j, height=None):
        if height is None:
            height = bitlen(j - 1)
        proof = []
        for h in range(height - 1, -1, -1):
            if (j - 1) & (1 << h):
                k = (j - 1) >> h << h
                if i <= k:
                    proof.insert(0, self.highest_node(j, h))
                    return self.inclusion_proof(i, k, h) + proof
                proof.insert(0, self.node(k, h))
        return proof

    def consistency_proof(self, i, j, height=None):
        if height is None:
            height = bitlen(j - 1)
        proof = []
        for h in range(height - 1, -1, -1):
            if (j - 1) & (1 << h):
                k = (j - 1) >> h << h
                if i <= k:
                    proof.insert(0, self.highest_node(j, h))
                    if i < k:
                        proof = self.consistency_proof(i, k, h) + proof
                    if i == k:
                        proof.insert(0, self.highest_node(i, h))
                    return proof
                proof.insert(0, self.node(k, h))
                if i == j:
                    proof.insert(0, self.highest_node(i, h))
                    return proof
        return proof


def eval_inclusion(proof, i, j, leaf):
    """embedded/ahtree/verification.go:32-56."""
    i1, j1, c = i - 1, j - 1, leaf
    for h in proof:
        c = sha(b"\x01" + c + h) if (i1 % 2 == 0 and i1 != j1) else sha(b"\x01" + h + c)
        i1 >>= 1
        j1 >>= 1
    return c


def verify_inclusion(proof, i, j, leaf, root):
    if i > j or i == 0 or (i < j and len(proof) == 0):
        return False
    return eval_inclusion(proof, i, j, leaf) == root


def eval_consistency(proof, i, j):
    """embedded/ahtree/verification.go:72-109."""
    fn, sn = i - 1, j - 1
    while fn % 2 == 1:
        fn >>= 1
        sn >>= 1
    ci = cj = proof[0]
    for h in proof[1:]:
        if fn % 2 == 1 or fn == sn:
            ci = sha(b"\x01" + h + ci)
            cj = sha(b"\x01" + h + cj)
            while fn % 2 == 0 and fn != 0:
                fn >>= 1
                sn >>= 1
        else:
            cj = sha(b"\x01" + cj + h)
        fn >>= 1
        sn >>= 1
    return ci, cj


def verify_consistency(proof, i, j, iroot, jroot):
    if i > j or i == 0 or (i < j and len(proof) == 0):
        return False
    if i == j and len(proof) == 0:
        return iroot == jroot
    ci, cj = eval_consistency(proof, i, j)
    return iroot == ci and jroot == cj


def eval_last_inclusion(proof, i, leaf):
    """embedded/ahtree/verification.go:120-137."""
    r = leaf
    for h in proof:
        r = sha(b"\x01" + h + r)
    return r


# ---------------------------------------------------------------- fixtures
def read_appendable(path):
    b = open(path, "rb").read()
    ml = struct.unpack(">I", b[:4])[0]
    return b[4 + ml:]


def appendable_header(path):
    """The singleapp header bytes of a Go-written appendable file (BE32 len ||
    appendable.Metadata bytes, single_app.go:116-171) -- data, kept to pin
    the header writer."""
    b = open(path, "rb").read()
    ml = struct.unpack(">I", b[:4])[0]
    return b[:4 + ml]


def parse_txlog(raw):
    """tx record layout: embedded/store/immustore.go:1812-1924."""
    txs, p = [], 0
    while p + 8 <= len(raw):
        tid = struct.unpack(">Q", raw[p:p + 8])[0]
        if tid == 0:
            break
        h = {"id": tid}
        p += 8
        h["ts"], h["bltxid"] = struct.unpack(">QQ", raw[p:p + 16]); p += 16
        h["blroot"] = raw[p:p + 32].hex(); p += 32
        h["prevalh"] = raw[p:p + 32].hex(); p += 32
        h["version"] = struct.unpack(">H", raw[p:p + 2])[0]; p += 2
        if h["version"] == 0:
            h["md"] = ""
            h["nentries"] = struct.unpack(">H", raw[p:p + 2])[0]; p += 2
        else:
            mdl = struct.unpack(">H", raw[p:p + 2])[0]; p += 2
            h["md"] = raw[p:p + mdl].hex(); p += mdl
            h["nentries"] = struct.unpack(">I", raw[p:p + 4])[0]; p += 4
        ents = []
        for _ in range(h["nentries"]):
            mdl = struct.unpack(">H", raw[p:p + 2])[0]; p += 2
            md = raw[p:p + mdl]; p += mdl
            kl = struct.unpack(">H", raw[p:p + 2])[0]; p += 2
            key = raw[p:p + kl]; p += kl
            vlen, voff = struct.unpack(">IQ", raw[p:p + 12]); p += 12
            hval = raw[p:p + 32]; p += 32
            ents.append({"md": md.hex(), "key": key.hex(), "vlen": vlen, "voff": voff, "hval": hval.hex()})
        h["alh"] = raw[p:p + 32].hex(); p += 32
        txs.append({"header": h, "entries": ents})
    return txs


def fixture_store(root):
    txs = parse_txlog(read_appendable(os.path.join(root, "tx/00000000.tx")))
    vlog_path = os.path.join(root, "val_0/00000000.val")
    vlog = read_appendable(vlog_path) if os.path.exists(vlog_path) else b""
    prev = sha(b"")  # initial prevAlh = SHA256(nil), immustore.go:464
    aht = AHT()
    for tx in txs:
        h = tx["header"]
        assert bytes.fromhex(h["prevalh"]) == prev, "prevAlh chain"
        digs = []
        for e in tx["entries"]:
            off = e["voff"] & ((1 << 56) - 1)  # top byte = vLog id (immustore.go encodeOffset)
            v = vlog[off:off + e["vlen"]]
            if len(v) == e["vlen"] and sha(v).hex() == e["hval"]:
                e["value"] = v.hex()  # value present in the vLog: pins hVal = SHA256(value)
            digs.append(entry_digest(h["version"], bytes.fromhex(e["key"]), bytes.fromhex(e["md"]),
                                     bytes.fromhex(e["hval"])))
        _, eh = htree_build(digs)
        h["eh"] = eh.hex()  # Eh is not stored: it is derived, and Alh (stored) pins it
        assert alh(h).hex() == h["alh"], "Alh mismatch tx %d" % h["id"]
        if h["bltxid"] > 0:
            assert aht.root_at(h["bltxid"]).hex() == h["blroot"], "BlRoot mismatch"
        aht.append(bytes.fromhex(h["alh"]))
        prev = bytes.fromhex(h["alh"])
    dlog = read_appendable(os.path.join(root, "aht/tree/00000000.sha"))
    n_aht = len(dlog) // 32
    pl = read_appendable(os.path.join(root, "aht/data/00000000.dat"))
    payloads, p = [], 0
    while p + 4 <= len(pl):
        ln = struct.unpack(">I", pl[p:p + 4])[0]
        payloads.append(pl[p + 4:p + 4 + ln].hex())
        p += 4 + ln
    ours = b"".join(aht.dlog)
    assert ours[:len(dlog)] == dlog, "dLog mismatch"
    assert n_aht == nodes_upto(len(payloads))
    # the cLog: one 12-byte entry per append pointing at its pLog record
    clog = read_appendable(os.path.join(root, "aht/commit/00000000.di"))
    assert len(clog) == 12 * len(payloads), "cLog size"
    q = 0
    for k, pay in enumerate(payloads):
        poff, ln = struct.unpack(">QI", clog[12 * k:12 * k + 12])
        assert poff == q and ln == len(pay) // 2, "cLog entry %d" % k
        q += 4 + ln
    # raw tx-log records (data file of the reference's test store) for the
    # read-path validation tests, and dual / linear proofs built the way
    # ImmuStore.DualProofV2 / LinearProof build them (immustore.go:2356-2387,
    # :2471-2510) from this store's own headers and dLog
    raw = read_appendable(os.path.join(root, "tx/00000000.tx"))
    hdrs = [t["header"] for t in txs]
    dual, linear = [], []
    for s_ in range(1, len(hdrs) + 1):
        for t_ in range(s_, len(hdrs) + 1):
            sh, th = hdrs[s_ - 1], hdrs[t_ - 1]
            if sh["bltxid"] != s_ - 1 or th["bltxid"] != t_ - 1:
                continue
            case = {"src": s_, "tgt": t_, "incl": [], "cons": []}
            if s_ < t_:
                case["incl"] = [x.hex() for x in aht.inclusion_proof(s_, th["bltxid"])]
                case["cons"] = [x.hex() for x in aht.consistency_proof(max(1, sh["bltxid"]),
                                                                       th["bltxid"])]
            dual.append(case)
            terms = [sh["alh"]] + [inner_hash(hdrs[k - 1]).hex() for k in range(s_ + 1, t_ + 1)]
            c = bytes.fromhex(terms[0])
            for k in range(1, len(terms)):
                c = sha(struct.pack(">Q", s_ + k) + c + bytes.fromhex(terms[k]))
            assert c.hex() == th["alh"]
            if (t_ - s_) % 7 == 0 or t_ == len(hdrs):
                linear.append({"src": s_, "tgt": t_, "terms": terms})
    # DualProof (v1) exactly as ImmuStore.DualProof / LinearAdvanceProof build
    # them (immustore.go:2392-2463, :2513-2562)
    dual1 = []
    for s_ in range(1, len(hdrs) + 1):
        for t_ in range(s_, len(hdrs) + 1):
            sh, th = hdrs[s_ - 1], hdrs[t_ - 1]
            if sh["bltxid"] > th["bltxid"]:
                continue
            c = {"src": s_, "tgt": t_, "incl": [], "cons": [], "last": [], "tbl_alh": "00" * 32}
            if s_ < th["bltxid"]:
                c["incl"] = [x.hex() for x in aht.inclusion_proof(s_, th["bltxid"])]
            if sh["bltxid"] > 0:
                c["cons"] = [x.hex() for x in aht.consistency_proof(sh["bltxid"], th["bltxid"])]
            if th["bltxid"] > 0:
                c["tbl_alh"] = hdrs[th["bltxid"] - 1]["alh"]
                c["last"] = [x.hex() for x in aht.inclusion_proof(th["bltxid"], th["bltxid"])]
            ls = max(s_, th["bltxid"])
            c["lin_src"] = ls
            c["lin"] = [hdrs[ls - 1]["alh"]] + [inner_hash(hdrs[k - 1]).hex()
                                                 for k in range(ls + 1, t_ + 1)]
            a0, a1 = sh["bltxid"], min(s_, th["bltxid"])
            if a1 <= a0 + 1:
                c["lap"] = None
            else:
                lt = [hdrs[a0]["alh"]] + [inner_hash(hdrs[k]).hex() for k in range(a0 + 1, a1)]
                ips = [[x.hex() for x in aht.inclusion_proof(k, th["bltxid"])]
                       for k in range(a0 + 1, a1)]
                c["lap"] = {"terms": lt, "incl": ips}
            dual1.append(c)
    # the store's commit log (commit/00000000.txi): one entry per tx, BE64
    # offset || BE32 size of its record in the tx log (cLogEntrySizeV1,
    # immustore.go:122, 2569-2597) -- pinned against the records parsed above
    txi = read_appendable(os.path.join(root, "commit/00000000.txi"))
    assert len(txi) == 12 * len(txs), "cLog size"
    q = 0
    for k, tx in enumerate(txs):
        off, size = struct.unpack(">QI", txi[12 * k:12 * k + 12])
        n = 90 + (2 if tx["header"]["version"] == 0 else 2 + len(tx["header"]["md"]) // 2 + 4)
        n += sum(4 + len(e["md"]) // 2 + len(e["key"]) // 2 + 12 + 32 for e in tx["entries"]) + 32
        assert off == q and size == n, "cLog entry %d" % k
        q += n
    headers = {rel: appendable_header(os.path.join(root, rel)).hex()
               for rel in ("aht/data/00000000.dat", "aht/tree/00000000.sha",
                           "aht/commit/00000000.di")}
    return {"txs": txs, "txi": txi.hex(),
        "txi_header": appendable_header(os.path.join(root, "commit/00000000.txi")).hex(), "aht_payloads": payloads, "aht_dlog": dlog.hex(), "app_headers": headers,
        "aht_plog": pl.hex(), "aht_clog": clog.hex(), "n_values": sum(
        1 for t in txs for e in t["entries"] if "value" in e), "txlog": raw.hex(),
        "dual_v2": dual, "linear": linear, "dual_v1": dual1}


# ---------------------------------------------------------------- synthetic
def splitmix64(state):
    state = (state + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return state, z ^ (z >> 31)


def rand_bytes(seed, n):
    out, s = bytearray(), seed
    while len(out) < n:
        s, z = splitmix64(s)
        out += struct.pack("<Q", z)
    return bytes(out[:n])


def synthetic():
    res = {}
    # htree widths, digests = SHA256(BE64(i)) as in embedded/htree/htree_test.go:45-50
    ht = []
    for w in [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 33, 63, 64, 65, 127, 129, 255, 257, 1000,
              1023, 1024, 1025, 4097]:
        digs = [sha(struct.pack(">Q", i)) for i in range(w)]
        lv, root = htree_build(digs)
        flat = b"".join(b"".join(x) for x in lv)
        case = {"width": w, "root": root.hex(), "levels_sha256": sha(flat).hex(),
                "levels_len": len(flat) // 32}
        if 0 < w <= 1025:
            step = max(1, w // 17)
            pr = []
            for i in list(range(0, w, step)) + [w - 1]:
                terms = htree_inclusion_proof(lv, w, i)
                assert htree_verify(i, w, terms, digs[i], root)
                pr.append({"leaf": i, "terms": [t.hex() for t in terms]})
            case["proofs"] = pr
        ht.append(case)
    res["htree"] = ht
    # entry digests, v0 and v1, with / without KV metadata (tx.go:690-731)
    ents = []
    for idx in range(64):
        key = rand_bytes(1000 + idx, (idx * 7) % 70)
        value = rand_bytes(2000 + idx, (idx * 37) % 300)
        md = [b"", b"\x00", b"\x01" + struct.pack(">Q", 1700000000 + idx), b"\x02",
              b"\x00\x01" + struct.pack(">Q", idx) + b"\x02"][idx % 5]
        hv = sha(value)
        e = {"key": key.hex(), "value": value.hex(), "md": md.hex(), "hval": hv.hex(),
             "digest_v1": entry_digest(1, key, md, hv).hex()}
        if not md:
            e["digest_v0"] = entry_digest(0, key, md, hv).hex()
        ents.append(e)
    res["entries"] = ents
    # BASELINE C1 plumbing case: 1024 x 256 B values (seed 1), key = BE64(i), v1, no md
    vals = rand_bytes(1, 1024 * 256)
    digs = [entry_digest(1, struct.pack(">Q", i), b"", sha(vals[i * 256:(i + 1) * 256])) for i in range(1024)]
    lv, root = htree_build(digs)
    res["c1"] = {"n": 1024, "value_len": 256, "seed": 1, "eh": root.hex(),
                 "levels_sha256": sha(b"".join(b"".join(x) for x in lv)).hex()}
    # ahtree, payload {byte(i)} as in embedded/ahtree/ahtree_test.go:647-715
    aht = AHT()
    roots = []
    for i in range(1, 1101):
        aht.append(bytes([i & 0xFF]))
        roots.append(aht.root_at(i).hex())
    res["ahtree"] = {"n": 1100, "payload": "byte(i)", "roots": roots,
                     "dlog_sha256": sha(b"".join(aht.dlog)).hex(), "dlog_len": len(aht.dlog),
                     "nodes_upto_1_16": [nodes_upto(n) for n in range(1, 17)]}
    # all-pairs proofs for n <= 40
    pairs = []
    for j in range(1, 41):
        for i in range(1, j + 1):
            ip = aht.inclusion_proof(i, j)
            cp = aht.consistency_proof(i, j)
            leaf = sha(b"\x00" + bytes([i & 0xFF]))
            assert verify_inclusion(ip, i, j, leaf, aht.root_at(j))
            assert verify_consistency(cp, i, j, aht.root_at(i), aht.root_at(j))
            pairs.append({"i": i, "j": j, "iproof": [t.hex() for t in ip], "cproof": [t.hex() for t in cp]})
    res["ahtree_proofs"] = pairs
    # 32-byte payloads (Alh-like), BASELINE C3 shape at small n, seed 3
    aht2 = AHT()
    pay = rand_bytes(3, 32 * 777)
    for i in range(777):
        aht2.append(pay[i * 32:(i + 1) * 32])
    res["ahtree32"] = {"n": 777, "seed": 3, "dlog_sha256": sha(b"".join(aht2.dlog)).hex(),
                       "root": aht2.root_at(777).hex(), "dlog_len": len(aht2.dlog)}
    return res


SCHEMA_MESSAGES = ("TxMetadata", "TxHeader", "DualProofV2", "InclusionProof", "DualProof",
                   "LinearProof", "LinearAdvanceProof")


def schema_fields():
    """(name, number, type, label, type_name) of the proof messages, decoded
    from the reference's generated descriptor (pkg/api/schema/schema.pb.go,
    file_schema_proto_rawDesc: the serialised FileDescriptorProto of
    schema.proto).  Data only: the byte literal is parsed and decoded here,
    nothing of the Go file is kept but these tuples."""
    import re
    from google.protobuf import descriptor_pb2
    lines = open(os.path.join(REF, "pkg/api/schema/schema.pb.go")).read().split("\n")
    start = next(k for k, ln in enumerate(lines) if ln.startswith("var file_schema_proto_rawDesc = []byte{"))
    raw = bytearray()
    for ln in lines[start + 1:]:
        if ln.startswith("}"):
            break
        raw += bytes(int(x, 16) for x in re.findall(r"0x([0-9a-f]{2})", ln))
    fdp = descriptor_pb2.FileDescriptorProto.FromString(bytes(raw))
    out = {"package": fdp.package, "syntax": fdp.syntax, "messages": {}}
    for m in fdp.message_type:
        if m.name in SCHEMA_MESSAGES:
            out["messages"][m.name] = [[f.name, f.number, f.type, f.label, f.type_name]
                                       for f in m.field]
    assert set(out["messages"]) == set(SCHEMA_MESSAGES)
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference (build container only)")
    if "--schema-only" in sys.argv:  # refresh schema_fields.json alone
        with open(os.path.join(OUT, "schema_fields.json"), "w") as f:
            json.dump(schema_fields(), f, indent=1, sort_keys=True)
        print("ok")
        return
    fx = {}
    for name, rel in [("long_linear_proof", "test/data_long_linear_proof"),
                      ("v110_defaultdb", "test/data_v1.1.0/defaultdb"),
                      ("v110_systemdb", "test/data_v1.1.0/systemdb")]:
        fx[name] = fixture_store(os.path.join(REF, rel))
        print(name, "txs", len(fx[name]["txs"]), "dlog digests", len(fx[name]["aht_dlog"]) // 64,
              "values", fx[name]["n_values"])
    with open(os.path.join(OUT, "immudb_fixtures.json"), "w") as f:
        json.dump(fx, f, indent=0, sort_keys=True)
    with open(os.path.join(OUT, "schema_fields.json"), "w") as f:
        json.dump(schema_fields(), f, indent=1, sort_keys=True)
    syn = synthetic()
    with open(os.path.join(OUT, "synthetic.json"), "w") as f:
        json.dump(syn, f, indent=0, sort_keys=True)
    print("ok")


if __name__ == "__main__":
    main()
