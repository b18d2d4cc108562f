"""Pin the CPU oracle (oracle/liboracle.so) against the reference's golden data.

Go-written fixtures (tests/golden/immudb_fixtures.json, extracted by
tests/golden/make_golden.py from /root/reference/test/...):
- every stored value hashes to its stored hVal (a1, immustore.go:1620-1630)
- entry digests v0/v1 -> htree root Eh -> innerHash -> Alh equals the Alh Go
  stored after each tx (a2-a4, a7; tx.go:249-355, htree.go:68-113)
- appending the stored Alh stream to an ahtree reproduces Go's dLog byte for
  byte (a8-a9, ahtree.go:246-373) and BlRoot (ahtree.go:749-771)
- the pLog / cLog record streams of those appends equal Go's aht/data and
  aht/commit files (8(f) row 4, ahtree.go:266-282, 341-351)
Reference known-answer tables: nodesUpto(1..16) (ahtree_test.go:36-64), empty
root SHA256(nil) (htree_test.go:36-38).
"""
import hashlib
import struct

import numpy as np
import pytest


def H(b):
    return hashlib.sha256(b).digest()


def test_sha256_known_answers(orc):
    for shani in (False, True):
        if shani and not orc.has_shani():
            continue
        orc.use_shani(shani)
        assert orc.sha256(b"").hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
        rng = np.random.default_rng(7)
        for n in list(range(0, 200)) + [1023, 1024, 1025, 4096, 65536 + 17]:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert orc.sha256(b) == H(b), n
    orc.use_shani(True)


@pytest.mark.parametrize("store", ["long_linear_proof", "v110_defaultdb", "v110_systemdb"])
def test_fixture_alh_chain(orc, fixtures, store):
    fx = fixtures[store]
    prev = H(b"")
    aht = orc.AHtree()
    nvals = 0
    for tx in fx["txs"]:
        h = tx["header"]
        assert bytes.fromhex(h["prevalh"]) == prev
        digs = []
        for e in tx["entries"]:
            if "value" in e:
                assert orc.sha256(bytes.fromhex(e["value"])).hex() == e["hval"]
                nvals += 1
            st, d = orc.entry_digest(h["version"], bytes.fromhex(e["key"]), bytes.fromhex(e["md"]),
                                     bytes.fromhex(e["hval"]))
            assert st == 0
            digs.append(np.frombuffer(d, np.uint8))
        _, eh = orc.htree_build(np.stack(digs))
        st, inner = orc.tx_inner_hash(h["ts"], h["version"], bytes.fromhex(h["md"]), h["nentries"],
                                      eh, h["bltxid"], bytes.fromhex(h["blroot"]))
        assert st == 0
        alh = orc.tx_alh(h["id"], prev, inner)
        assert alh.hex() == h["alh"], "tx %d" % h["id"]
        if h["bltxid"]:
            st, r = aht.root_at(h["bltxid"])
            assert st == 0 and r.hex() == h["blroot"]
        aht.append(alh)
        prev = alh
    assert nvals == fx["n_values"]
    # the stored ahtree payload stream is exactly the Alh stream
    assert [x["header"]["alh"] for x in fx["txs"]][:len(fx["aht_payloads"])] == fx["aht_payloads"]
    dlog = bytes.fromhex(fx["aht_dlog"])
    assert aht.dlog_bytes()[:len(dlog)] == dlog
    # and the batch append path reproduces it too
    b = orc.AHtree()
    b.append_batch(np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]]))
    assert b.dlog_bytes() == dlog


@pytest.mark.parametrize("store", ["long_linear_proof", "v110_defaultdb", "v110_systemdb"])
@pytest.mark.parametrize("split", [0, 1, 7])
def test_fixture_appendable_streams(orc, fixtures, store, split):
    """pLog / cLog / dLog byte streams of the Go-written aht/{data,commit,tree}
    files, rebuilt by appending the stored payloads in two batches."""
    fx = fixtures[store]
    pays = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
    split = min(split, len(pays))
    t = orc.AHtree()
    p1, c1 = t.append_batch_logs(pays[:split], 0)
    p2, c2 = t.append_batch_logs(pays[split:], len(p1))
    assert p1 + p2 == bytes.fromhex(fx["aht_plog"])
    assert c1 + c2 == bytes.fromhex(fx["aht_clog"])
    assert t.dlog_bytes() == bytes.fromhex(fx["aht_dlog"])


def test_nodes_upto_table(orc, synthetic):
    # embedded/ahtree/ahtree_test.go:36-64
    expected = [1, 3, 5, 8, 10, 13, 16, 20, 22, 25, 28, 32, 35, 39, 43, 48]
    assert [orc.nodes_upto(n) for n in range(1, 17)] == expected
    assert synthetic["ahtree"]["nodes_upto_1_16"] == expected
    for n in range(1, 17):
        assert orc.nodes_until(n) + bin(n - 1).count("1") + 1 == orc.nodes_upto(n)


def test_htree_synthetic(orc, synthetic):
    for case in synthetic["htree"]:
        w = case["width"]
        digs = np.stack([np.frombuffer(H(struct.pack(">Q", i)), np.uint8) for i in range(w)]) if w else \
            np.zeros((0, 32), np.uint8)
        lv, root = orc.htree_build(digs)
        assert root.hex() == case["root"], w
        assert lv.shape[0] == case["levels_len"]
        assert H(lv.tobytes()).hex() == case["levels_sha256"]
        for pr in case.get("proofs", []):
            st, terms = orc.htree_inclusion_proof(lv, w, pr["leaf"])
            assert st == 0
            assert [t.tobytes().hex() for t in terms] == pr["terms"]
            assert orc.htree_verify_inclusion(pr["leaf"], w, terms, digs[pr["leaf"]], root)
            assert not orc.htree_verify_inclusion(pr["leaf"], w, terms, H(digs[pr["leaf"]].tobytes()), root)
            assert not orc.htree_verify_inclusion(pr["leaf"], w, terms, digs[pr["leaf"]], H(root))
            if w > 1:
                assert not orc.htree_verify_inclusion(pr["leaf"], w, terms[:0], digs[pr["leaf"]], root)


def test_htree_errors(orc):
    lv, root = orc.htree_build(np.zeros((0, 32), np.uint8))
    assert root == H(b"")
    lv, root = orc.htree_build(np.zeros((5, 32), np.uint8))
    st, _ = orc.htree_inclusion_proof(lv, 5, 5)
    assert st == 2  # ErrIllegalArguments (htree.go:122-124)


def test_entry_digests(orc, synthetic):
    for e in synthetic["entries"]:
        k, m, hv = bytes.fromhex(e["key"]), bytes.fromhex(e["md"]), bytes.fromhex(e["hval"])
        assert orc.sha256(bytes.fromhex(e["value"])) == hv
        st, d = orc.entry_digest(1, k, m, hv)
        assert st == 0 and d.hex() == e["digest_v1"]
        st, d = orc.entry_digest(0, k, m, hv)
        if m:
            assert st == 6  # ErrMetadataUnsupported (tx.go:691-693)
        else:
            assert st == 0 and d.hex() == e["digest_v0"]


def test_build_entries_csr_and_fixed(orc, synthetic):
    ents = synthetic["entries"]
    keys = [bytes.fromhex(e["key"]) for e in ents]
    mds = [bytes.fromhex(e["md"]) for e in ents]
    vals = [bytes.fromhex(e["value"]) for e in ents]
    st, hv, lv, root = orc.build_entries(1, keys, mds, vals)
    assert st == 0
    digs = np.stack([np.frombuffer(bytes.fromhex(e["digest_v1"]), np.uint8) for e in ents])
    assert root == orc.htree_build(digs)[1]
    # v0 with metadata present -> ErrMetadataUnsupported
    st, *_ = orc.build_entries(0, keys, mds, vals)
    assert st == 6
    # IsValueTruncated override (immustore.go:1624-1626)
    ov = [bytes.fromhex(e["hval"]) if i % 3 == 0 else None for i, e in enumerate(ents)]
    st2, hv2, _, root2 = orc.build_entries(1, keys, mds, [b"" if o else v for o, v in zip(ov, vals)], ov)
    assert st2 == 0 and root2 == root and (hv2 == hv).all()
    # C1 plumbing config: 1024 x 256 B, key = BE64(i), seed 1
    c1 = synthetic["c1"]
    vals = orc.fill_random(1024 * 256, 1).reshape(1024, 256)
    keys = np.frombuffer(b"".join(struct.pack(">Q", i) for i in range(1024)), np.uint8).reshape(1024, 8)
    for nt in (1, 3, 8):
        hv, lv, root = orc.build_entries_fixed(1, keys, vals, nthreads=nt)
        assert root.hex() == c1["eh"]
        assert H(lv.tobytes()).hex() == c1["levels_sha256"]


def test_ahtree_synthetic(orc, synthetic):
    a = synthetic["ahtree"]
    t = orc.AHtree()
    for i in range(1, a["n"] + 1):
        r = t.append(bytes([i & 0xFF]))
        assert r.hex() == a["roots"][i - 1]
    assert H(t.dlog_bytes()).hex() == a["dlog_sha256"]
    for i in (1, 17, 1100):
        st, r = t.root_at(i)
        assert st == 0 and r.hex() == a["roots"][i - 1]
    assert t.root_at(0)[0] == 2 and t.root_at(1101)[0] == 5
    assert orc.AHtree().root_at(1)[0] == 4
    for pr in synthetic["ahtree_proofs"]:
        i, j = pr["i"], pr["j"]
        st, ip = t.inclusion_proof(i, j)
        assert st == 0 and [x.tobytes().hex() for x in ip] == pr["iproof"]
        st, cp = t.consistency_proof(i, j)
        assert st == 0 and [x.tobytes().hex() for x in cp] == pr["cproof"]
        leaf = H(bytes([0, i & 0xFF]))
        jr = bytes.fromhex(a["roots"][j - 1])
        ir = bytes.fromhex(a["roots"][i - 1])
        assert orc.ahtree_verify_inclusion(ip, i, j, leaf, jr)
        assert orc.ahtree_verify_consistency(cp, i, j, ir, jr)
        assert orc.ahtree_verify_last_inclusion(ip, i, leaf,
                                                jr) == (i == j)
    assert t.inclusion_proof(2, 1)[0] == 2 and t.consistency_proof(2, 1)[0] == 2
    # verification.go edge cases (verification_test.go:26-32)
    z = H(b"")
    assert not orc.ahtree_verify_inclusion([], 1, 10, z, z)
    assert not orc.ahtree_verify_inclusion([], 10, 1, z, z)
    assert not orc.ahtree_verify_consistency([], 1, 10, z, z)
    assert not orc.ahtree_verify_consistency([], 10, 1, z, z)
    # C3-shaped 32-byte payloads
    a32 = synthetic["ahtree32"]
    t2 = orc.AHtree()
    t2.append_batch(orc.fill_random(32 * a32["n"], a32["seed"]).reshape(-1, 32))
    assert H(t2.dlog_bytes()).hex() == a32["dlog_sha256"]
    assert t2.root_at(a32["n"])[1].hex() == a32["root"]


def test_fill_random_matches_generator(orc):
    # splitmix64 stream identical to tests/golden/make_golden.py:rand_bytes
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "mg", os.path.join(os.path.dirname(__file__), "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    for seed in (1, 2, 3, 12345):
        for n in (1, 7, 8, 100, 4096):
            assert orc.fill_random(n, seed).tobytes() == mg.rand_bytes(seed, n)


def _values_case(seed, n=500):
    """Values, their stored hVals and expected lengths with the corruptions
    readValueAt rejects (immustore.go:3235): a flipped byte, a short read
    (vLen above the bytes returned), a long read, a wrong hVal; empty values."""
    import hashlib
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, n)
    lens[:20] = 0
    vals = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    hv = np.frombuffer(b"".join(hashlib.sha256(v).digest() for v in vals), np.uint8).reshape(n, 32).copy()
    vlen = lens.astype(np.uint64).copy()
    bad = np.zeros(n, bool)
    for i in rng.choice(n, min(60, n // 2), replace=False):
        kind = int(rng.integers(0, 4))
        if kind == 0 and len(vals[i]):
            b = bytearray(vals[i])
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            vals[i] = bytes(b)
        elif kind == 1 and len(vals[i]):
            vals[i] = vals[i][:-1]           # short read: n < len(b)
        elif kind == 2:
            vlen[i] += 1                       # stored length above the bytes read
        else:
            hv[i, int(rng.integers(0, 32))] ^= 0x80
        bad[i] = True
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(v) for v in vals], out=off[1:])
    return np.frombuffer(b"".join(vals) + b"\0", np.uint8)[:int(off[-1])].copy(), off, hv, vlen, bad


def test_verify_values_oracle_vs_hashlib(orc):
    for seed in (1, 2):
        vb, off, hv, vlen, bad = _values_case(seed)
        for nt in (1, 4):
            c, st = orc.verify_values(vb, off, hv, vlen, nthreads=nt)
            assert c == int(bad.sum())
            assert np.array_equal(st != 0, bad)
            assert set(np.unique(st)) <= {0, 14}
        # no lengths: only the digest decides (a long vLen alone passes)
        c2, st2 = orc.verify_values(vb, off, hv, None)
        assert np.all(st2[~bad] == 0) and c2 <= c


@pytest.mark.parametrize("n_start", [0, 1, 5, 64, 1000, 1023, 1024])
def test_ahtree_stream_equals_dlog(orc, n_start):
    """orc_ahtree_stream (peaks only, no dLog; the checker of the multi-rank
    C3 bench line) gives the digests append n writes (ahtree.go:287-322) and
    the peaks (ahtree.go:460-462) of the full-dLog restatement, from any
    starting size with the peaks handed over."""
    M = 3000
    raw = orc.fill_random(32 * M, 9).reshape(M, 32)
    t = orc.AHtree()
    t.append_batch(raw)
    dl = t.dlog
    pin = orc.ahtree_stream(9, 32, 0, n_start)[1] if n_start else None
    rng = np.random.default_rng(n_start)
    samples = sorted(set(int(x) for x in rng.integers(n_start + 1, M + 1, 300)) | {n_start + 1, M})
    res, pk = orc.ahtree_stream(9, 32, n_start, M, samples, peaks_in=pin)
    assert sorted(res) == samples
    for n, ds in res.items():
        base = orc.nodes_until(n)
        assert ds == [bytes(dl[base + c]) for c in range(1 + bin(n - 1).count("1"))], n
        assert ds[-1] == t.root_at(n)[1]
    for l in range(64):
        if (M >> l) & 1:
            assert bytes(pk[l]) == bytes(dl[orc.nodes_until((M >> l) << l) + l]), l


def test_ahtree_peaks_streamed_in_blocks(orc):
    """The peaks rebuilt block by block on several threads equal the dLog's."""
    M = 3000
    t = orc.AHtree()
    t.append_batch(orc.fill_random(32 * M, 9).reshape(M, 32))
    for n in (1, 2, 3, 1000, 2047, 2048, 3000):
        for bb in (0, 3, 20):
            pk = orc.ahtree_peaks_streamed(9, 32, n, threads=4, block_bits=bb)
            for l in range(64):
                if (n >> l) & 1:
                    assert bytes(pk[l]) == bytes(t.dlog[orc.nodes_until((n >> l) << l) + l]), (n, l)
    with pytest.raises(ValueError):
        orc.ahtree_stream(9, 31, 0, 4)  # payloads must be whole splitmix64 words


def test_ahtree_proof_batch_equals_single_calls(orc):
    """orc_ahtree_proof_batch (the checker of the device's batch proof
    generation at the reference suite's N = 1024) = one call per pair."""
    n = 200
    t = orc.AHtree(n)
    t.append_batch((np.arange(1, n + 1) & 0xFF).astype(np.uint8).reshape(n, 1))
    I, J = np.triu_indices(n, 0)
    I, J = I + 1, J + 1
    for kind, fn in ((0, t.inclusion_proof), (1, t.consistency_proof)):
        terms, nt, st = t.proof_batch(kind, I, J, cap=32)
        assert not st.any()
        for p in range(0, len(I), 7):
            _, o = fn(int(I[p]), int(J[p]))
            assert nt[p] == len(o) and terms[p, :nt[p]].tobytes() == o.tobytes()
        assert list(t.proof_batch(kind, [2, 1], [1, n + 1])[2]) == [2, 5]
        assert list(t.proof_batch(kind, [1], [n], cap=2)[2]) == [2]  # longer than cap
