"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden data.  Bit-exact everywhere (integer/byte work).

Run on the MI355X box:  python -m pytest tests -m gpu -x -q
"""
import hashlib
import os
import struct

import numpy as np
import pytest

from gpu_util import DevBuf

pytestmark = pytest.mark.gpu


def H(b):
    return hashlib.sha256(b).digest()


@pytest.fixture(scope="module")
def m():
    import torch  # noqa: F401  (load the HIP runtime the way the bench does)
    import immustore_amd as m
    if m.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return m


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


@pytest.fixture(params=["1", "2", "4"])
def lpl(request):
    old = os.environ.get("MH_LPL")
    os.environ["MH_LPL"] = request.param
    yield int(request.param)
    if old is None:
        del os.environ["MH_LPL"]
    else:
        os.environ["MH_LPL"] = old


# ------------------------------------------------------------------ SHA-256
def test_sha256_batch_any_alignment(m, ctx):
    from immustore_amd import _native as N
    rng = np.random.default_rng(11)
    lens = list(range(0, 140)) + [255, 256, 257, 1000, 1023, 1024, 1025, 4096, 5000]
    # random gaps make every start alignment mod 4 / mod 16 appear
    offs, pos = [], 0
    for L in lens:
        pos += int(rng.integers(0, 7))
        offs.append((pos, pos + L))
        pos += L
    buf = rng.integers(0, 256, pos + 3, dtype=np.uint8)
    # CSR needs contiguous ranges: build [start_i, end_i) as off[i], off[i+1] pairs by
    # hashing every range through its own 2-entry offset table
    d_buf = DevBuf.from_host(ctx, buf)
    for (a, b) in offs:
        off = np.array([a, b], np.uint64)
        d_off = DevBuf.from_host(ctx, off)
        d_out = DevBuf(ctx, 32)
        N.check(N.load().mh_dev_sha256_batch(ctx.handle, d_buf.ptr, d_off.ptr, 1, d_out.ptr))
        assert d_out.to_host().tobytes() == H(buf[a:b].tobytes()), (a, b)
    # and one big batch over contiguous ranges
    cuts = np.sort(rng.integers(0, pos, 500)).astype(np.uint64)
    cuts[0] = 0
    d_off = DevBuf.from_host(ctx, cuts)
    d_out = DevBuf(ctx, 32 * (len(cuts) - 1))
    N.check(N.load().mh_dev_sha256_batch(ctx.handle, d_buf.ptr, d_off.ptr, len(cuts) - 1, d_out.ptr))
    got = d_out.to_host().reshape(-1, 32)
    for i in range(len(cuts) - 1):
        assert got[i].tobytes() == H(buf[int(cuts[i]):int(cuts[i + 1])].tobytes())


def test_sha256_batch_ragged_length_classes(m, ctx):
    """Many ragged messages (the length-class sorted kernel, n > 256): every
    length 0..1100 several times over at random alignments, a spread up to
    4 KiB, and messages past the last length class (> 1023 blocks)."""
    from immustore_amd import _native as N
    rng = np.random.default_rng(12)
    lens = np.concatenate([np.tile(np.arange(0, 1101), 3), rng.integers(0, 4097, 6000),
                           [65472 - 9, 65472 - 8, 70000, 100000, 0, 0]])
    rng.shuffle(lens)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    for shift in (0, 1, 3):   # the whole batch starts at every alignment
        d_buf = DevBuf.from_host(ctx, buf)
        o = off + np.uint64(shift)
        d_off = DevBuf.from_host(ctx, o)
        d_out = DevBuf(ctx, 32 * len(lens))
        N.check(N.load().mh_dev_sha256_batch(ctx.handle, d_buf.ptr, d_off.ptr, len(lens), d_out.ptr))
        got = d_out.to_host().reshape(-1, 32)
        bb = buf.tobytes()
        for k in range(len(lens)):
            assert got[k].tobytes() == H(bb[int(o[k]):int(o[k + 1])]), (shift, k, int(lens[k]))


def test_csr_offsets_running_backwards(m, ctx):
    """Caller bugs never reach the device as wrapped-around lengths: host CSR
    offsets that run backwards are MH_ERR_ILLEGAL_ARGUMENTS; device CSR ones
    (checked nowhere on the host) hash the bad range as an empty message."""
    from immustore_amd import _native as N
    L = N.load()
    buf = np.arange(64, dtype=np.uint8)
    off = np.array([0, 10, 5, 20], np.uint64)
    d_buf, d_off, d_out = DevBuf.from_host(ctx, buf), DevBuf.from_host(ctx, off), DevBuf(ctx, 96)
    N.check(L.mh_dev_sha256_batch(ctx.handle, d_buf.ptr, d_off.ptr, 3, d_out.ptr))
    got = d_out.to_host().reshape(3, 32)
    assert got[0].tobytes() == H(buf[0:10].tobytes())
    assert got[1].tobytes() == H(b"")
    assert got[2].tobytes() == H(buf[5:20].tobytes())
    t = m.HTree(8, ctx)
    keys = np.frombuffer(b"abcdefgh", np.uint8).copy()
    ko = np.array([0, 4, 2, 8], np.uint64)   # entry 1 runs backwards
    vo = np.array([0, 1, 2, 3], np.uint64)
    vals = np.zeros(8, np.uint8)
    hv = np.zeros((3, 32), np.uint8)
    st = L.mh_htree_build_entries(t.handle, 1, 3, keys.ctypes.data, ko.ctypes.data, None, None,
                                  vals.ctypes.data, vo.ctypes.data, None, None, hv.ctypes.data)
    assert st == N.MH_ERR_ILLEGAL_ARGUMENTS
    t.close()


def test_entries_ragged_with_overrides_vs_oracle(m, ctx, orc):
    """General entry path with ragged keys / metadata / values and a share of
    IsValueTruncated overrides (their hVal taken from the caller)."""
    rng = np.random.default_rng(13)
    for n in (257, 3001):
        keys = [rng.integers(0, 256, int(rng.integers(1, 130)), dtype=np.uint8).tobytes()
                for _ in range(n)]
        mds = [rng.integers(0, 256, int(rng.integers(0, 12)), dtype=np.uint8).tobytes()
               for _ in range(n)]
        vals = [rng.integers(0, 256, int(rng.integers(0, 4097)), dtype=np.uint8).tobytes()
                for _ in range(n)]
        ov = [H(v) if rng.random() < 0.2 else None for v in vals]
        vals2 = [b"" if o is not None else v for o, v in zip(ov, vals)]
        eh, hv, lv = m.build_hash_tree(1, keys, vals2, mds, hval_overrides=ov, ctx=ctx)
        st, ohv, olv, oroot = orc.build_entries(1, keys, mds, vals)
        assert st == 0 and eh == oroot and np.array_equal(hv, ohv) and np.array_equal(lv, olv)



# ------------------------------------------------------------------ htree
def test_htree_build_with_golden(m, ctx, synthetic, lpl):
    for case in synthetic["htree"]:
        w = case["width"]
        digs = [H(struct.pack(">Q", i)) for i in range(w)]
        t = m.HTree(max(w, 1), ctx)
        t.build_with(digs)
        assert t.root().hex() == case["root"], w
        lv = t.levels()
        assert lv.shape[0] == case["levels_len"]
        assert H(lv.tobytes()).hex() == case["levels_sha256"], w
        for pr in case.get("proofs", []):
            p = t.inclusion_proof(pr["leaf"])
            assert [x.hex() for x in p.terms] == pr["terms"]
        t.close()


def test_htree_errors(m, ctx):
    # embedded/htree/htree_test.go:27-87
    t = m.HTree(0, ctx)
    with pytest.raises(m.ErrMaxWidthExceeded):
        t.build_with([H(b"")])
    t.build_with([])
    assert t.root() == H(b"")
    t = m.HTree(1000, ctx)
    digs = [H(struct.pack(">Q", i)) for i in range(1000)]
    t.build_with(digs)
    root = t.root()
    proofs = [t.inclusion_proof(i) for i in range(1000)]
    assert m.verify_inclusion_batch(proofs, digs, [root] * 1000).all()
    assert not m.verify_inclusion_batch(proofs, [H(d) for d in digs], [root] * 1000).any()
    assert not m.verify_inclusion_batch(proofs, digs, [H(root)] * 1000).any()
    stripped = [m.InclusionProof(p.leaf, p.width, []) for p in proofs]
    assert not m.verify_inclusion_batch(stripped, digs, [root] * 1000).any()
    assert not m.verify_inclusion(None, digs[0], root)
    t.build_with([])
    assert t.root() == H(b"")
    with pytest.raises(m.ErrMaxWidthExceeded):
        t.build_with([b"\0" * 32] * 1001)
    with pytest.raises(m.ErrIllegalArguments):
        t.inclusion_proof(1000)


def test_htree_random_widths_vs_oracle(m, ctx, orc, lpl):
    rng = np.random.default_rng(5)
    for w in [1, 2, 3, 4, 5, 6, 7, 8, 9, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025,
              4095, 4097, 65535, 65537, 262145, 1048577]:
        d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
        t = m.HTree(w, ctx)
        t.build_with(d)
        lv, root = orc.htree_build(d)
        assert t.root() == root, w
        assert np.array_equal(t.levels(), lv), w
        t.close()


# ------------------------------------------------------------ entries (fused)
def _fixed_inputs(orc, n, klen, vlen, seed):
    vals = orc.fill_random(n * vlen, seed).reshape(n, vlen) if vlen else np.zeros((n, 0), np.uint8)
    keys = orc.fill_random(n * klen, seed + 1000).reshape(n, klen) if klen else np.zeros((n, 0), np.uint8)
    return keys, vals


def _dev_build_fixed(m, ctx, version, keys, vals):
    from immustore_amd import _native as N
    n, klen = keys.shape
    vlen = vals.shape[1]
    dk = DevBuf.from_host(ctx, keys if keys.size else np.zeros(16, np.uint8))
    dv = DevBuf.from_host(ctx, vals if vals.size else np.zeros(16, np.uint8))
    dl = DevBuf(ctx, max(m.levels_len(n), 1) * 32)
    dh = DevBuf(ctx, max(n, 1) * 32)
    dr = DevBuf(ctx, 32)
    N.check(N.load().mh_dev_htree_build_entries_fixed(ctx.handle, version, n, dk.ptr, klen, dv.ptr,
                                                       vlen, dh.ptr, dl.ptr, dr.ptr))
    ctx.synchronize()
    return (dh.to_host().reshape(-1, 32)[:n], dl.to_host().reshape(-1, 32)[:m.levels_len(n)],
            dr.to_host().tobytes())


def test_c1_plumbing_config(m, ctx, orc, synthetic, lpl):
    # BASELINE configs[0]: 1024 x 256 B, key = BE64(i), v1, seed 1
    c1 = synthetic["c1"]
    vals = orc.fill_random(1024 * 256, 1).reshape(1024, 256)
    keys = np.frombuffer(b"".join(struct.pack(">Q", i) for i in range(1024)), np.uint8).reshape(1024, 8)
    hv, lv, root = _dev_build_fixed(m, ctx, 1, keys, vals)
    assert root.hex() == c1["eh"]
    assert H(lv.tobytes()).hex() == c1["levels_sha256"]
    for i in (0, 1, 511, 1023):
        assert hv[i].tobytes() == H(vals[i].tobytes())


@pytest.mark.parametrize("version,klen", [(1, 0), (1, 4), (1, 8), (1, 12), (1, 16), (0, 0), (0, 8),
                                          (0, 20)])
def test_entries_fixed_shapes(m, ctx, orc, lpl, version, klen):
    for vlen in (0, 16, 48, 64, 80, 112, 128, 192, 1024, 1040):
        for n in (1, 2, 3, 5, 63, 64, 65, 255, 257, 1000):
            keys, vals = _fixed_inputs(orc, n, klen, vlen, 7 + vlen + n)
            hv, lv, root = _dev_build_fixed(m, ctx, version, keys, vals)
            ohv, olv, oroot = orc.build_entries_fixed(version, keys, vals)
            assert root == oroot, (version, klen, vlen, n)
            assert np.array_equal(hv, ohv), (version, klen, vlen, n)
            assert np.array_equal(lv, olv), (version, klen, vlen, n)


def test_entries_fixed_odd_shapes_use_general_path(m, ctx, orc):
    # shapes outside the fused kernel's preconditions (unaligned stride,
    # long keys) go through the generic CSR kernels -- same answer
    for version, klen, vlen in [(1, 3, 17), (1, 33, 100), (0, 1, 1), (1, 64, 63), (0, 100, 5)]:
        for n in (1, 7, 300):
            keys, vals = _fixed_inputs(orc, n, klen, vlen, 99)
            hv, lv, root = _dev_build_fixed(m, ctx, version, keys, vals)
            ohv, olv, oroot = orc.build_entries_fixed(version, keys, vals)
            assert root == oroot and np.array_equal(lv, olv) and np.array_equal(hv, ohv)


def test_entries_csr_md_override(m, ctx, orc, synthetic):
    ents = synthetic["entries"]
    keys = [bytes.fromhex(e["key"]) for e in ents]
    mds = [bytes.fromhex(e["md"]) for e in ents]
    vals = [bytes.fromhex(e["value"]) for e in ents]
    eh, hv, lv = m.build_hash_tree(1, keys, vals, mds, ctx=ctx)
    digs = np.stack([np.frombuffer(bytes.fromhex(e["digest_v1"]), np.uint8) for e in ents])
    olv, oroot = orc.htree_build(digs)
    assert eh == oroot and np.array_equal(lv, olv)
    assert [h.tobytes().hex() for h in hv] == [e["hval"] for e in ents]
    with pytest.raises(m.ErrMetadataUnsupported):
        m.build_hash_tree(0, keys, vals, mds, ctx=ctx)
    # IsValueTruncated: override hVal, value absent (immustore.go:1624-1626)
    ov = [bytes.fromhex(e["hval"]) if i % 3 == 0 else None for i, e in enumerate(ents)]
    vals2 = [b"" if o else v for o, v in zip(ov, vals)]
    eh2, hv2, _ = m.build_hash_tree(1, keys, vals2, mds, hval_overrides=ov, ctx=ctx)
    assert eh2 == eh and np.array_equal(hv2, hv)
    # v0 without metadata
    nomd = [i for i, e in enumerate(ents) if not e["md"]]
    eh0, _, _ = m.build_hash_tree(0, [keys[i] for i in nomd], [vals[i] for i in nomd], ctx=ctx)
    d0 = np.stack([np.frombuffer(bytes.fromhex(ents[i]["digest_v0"]), np.uint8) for i in nomd])
    assert eh0 == orc.htree_build(d0)[1]


def test_entries_csr_random_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(3)
    for n in (1, 2, 17, 300, 2049):
        keys = [rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8).tobytes() for _ in range(n)]
        mds = [rng.integers(0, 256, int(rng.integers(0, 12)), dtype=np.uint8).tobytes() for _ in range(n)]
        vals = [rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8).tobytes() for _ in range(n)]
        eh, hv, lv = m.build_hash_tree(1, keys, vals, mds, ctx=ctx)
        st, ohv, olv, oroot = orc.build_entries(1, keys, mds, vals)
        assert st == 0 and eh == oroot and np.array_equal(hv, ohv) and np.array_equal(lv, olv)


def test_entries_long_metadata_vs_oracle(m, ctx, orc):
    """Metadata longer than immudb's attributes (> 12 bytes: the digest
    prefix then spans more than the first 4 message words, and more than one
    block for the longest) through the general path, next to short ones."""
    rng = np.random.default_rng(21)
    for n in (5, 300, 2000):
        keys = [rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes()
                for _ in range(n)]
        mds = [rng.integers(0, 256, int(rng.choice([0, 3, 11, 13, 17, 40, 61, 62, 70, 130])),
                            dtype=np.uint8).tobytes() for _ in range(n)]
        vals = [rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
                for _ in range(n)]
        eh, hv, lv = m.build_hash_tree(1, keys, vals, mds, ctx=ctx)
        st, ohv, olv, oroot = orc.build_entries(1, keys, mds, vals)
        assert st == 0 and eh == oroot and np.array_equal(hv, ohv) and np.array_equal(lv, olv)


def test_entries_max_sizes_vs_oracle(m, ctx, orc):
    """The reference's limits (options.go:37-39: MaxKeyLen 1024, MaxValueLen
    4096; KV metadata <= 11 bytes, kv_metadata.go) and the block boundaries of
    the digest message around them (v1: 4 + ml + kl + 32 bytes, v0: kl + 32):
    keys of 0..1024 bytes at every class edge, next to empty and 4096-byte
    values, v1 and v0, some IsValueTruncated."""
    rng = np.random.default_rng(77)
    kls = [0, 1, 7, 8, 19, 20, 23, 24, 55, 56, 63, 64, 87, 88, 119, 120, 500, 1000, 1015, 1016,
           1023, 1024]
    vls = [0, 1, 55, 56, 63, 64, 119, 120, 4031, 4032, 4095, 4096]
    keys, mds, vals = [], [], []
    for kl in kls:
        for vl in vls:
            keys.append(rng.integers(0, 256, kl, dtype=np.uint8).tobytes())
            mds.append(rng.integers(0, 256, int(rng.choice([0, 1, 9, 11])), dtype=np.uint8).tobytes())
            vals.append(rng.integers(0, 256, vl, dtype=np.uint8).tobytes())
    eh, hv, lv = m.build_hash_tree(1, keys, vals, mds, ctx=ctx)
    st, ohv, olv, oroot = orc.build_entries(1, keys, mds, vals)
    assert st == 0 and eh == oroot and np.array_equal(hv, ohv) and np.array_equal(lv, olv)
    eh, hv, lv = m.build_hash_tree(0, keys, vals, ctx=ctx)
    st, ohv, olv, oroot = orc.build_entries(0, keys, [b""] * len(keys), vals)
    assert st == 0 and eh == oroot and np.array_equal(lv, olv)
    ov = [H(v) if k % 3 == 0 else None for k, v in enumerate(vals)]
    vals2 = [b"" if o is not None else v for o, v in zip(ov, vals)]
    eh, hv, lv = m.build_hash_tree(1, keys, vals2, mds, hval_overrides=ov, ctx=ctx)
    st, ohv, olv, oroot = orc.build_entries(1, keys, mds, vals)
    assert st == 0 and eh == oroot and np.array_equal(hv, ohv)
    # 64 copies: past the 16384 entries where the length-class sort starts
    K, M, V = keys * 64, mds * 64, vals * 64
    eh, hv, lv = m.build_hash_tree(1, K, V, M, ctx=ctx)
    st, ohv, olv, oroot = orc.build_entries(1, K, M, V)
    assert st == 0 and eh == oroot and np.array_equal(hv, ohv) and np.array_equal(lv, olv)


def test_go_fixtures_alh_chain_on_gpu(m, ctx, orc, fixtures):
    """Eh computed on the GPU -> innerHash/Alh (oracle) == Alh stored by Go."""
    for name, fx in fixtures.items():
        prev = H(b"")
        for tx in fx["txs"]:
            h = tx["header"]
            ents = tx["entries"]
            keys = [bytes.fromhex(e["key"]) for e in ents]
            mds = [bytes.fromhex(e["md"]) for e in ents]
            # values where the vLog holds them, otherwise the stored hVal as override
            vals = [bytes.fromhex(e.get("value", "")) for e in ents]
            ov = [None if "value" in e else bytes.fromhex(e["hval"]) for e in ents]
            eh, hv, _ = m.build_hash_tree(h["version"], keys, vals, mds, hval_overrides=ov, ctx=ctx)
            assert [x.tobytes().hex() for x in hv] == [e["hval"] for e in ents]
            st, inner = orc.tx_inner_hash(h["ts"], h["version"], bytes.fromhex(h["md"]),
                                          h["nentries"], eh, h["bltxid"], bytes.fromhex(h["blroot"]))
            alh = orc.tx_alh(h["id"], prev, inner)
            assert alh.hex() == h["alh"], (name, h["id"])
            prev = alh


def test_c2_full_size_vs_oracle(m, ctx, orc):
    """BASELINE configs[1] at full size: 2^20 x 1 KiB, key = BE64(i), v1."""
    n, vlen = 1 << 20, 1024
    vals = orc.fill_random(n * vlen, 2).reshape(n, vlen)
    keys = np.frombuffer(np.arange(n, dtype=">u8").tobytes(), np.uint8).reshape(n, 8)
    hv, lv, root = _dev_build_fixed(m, ctx, 1, keys, vals)
    ohv, olv, oroot = orc.build_entries_fixed(1, keys, vals, nthreads=min(16, os.cpu_count() or 1))
    assert root == oroot
    assert np.array_equal(lv, olv)
    assert np.array_equal(hv, ohv)


def test_reduce_nodes_matches_sharded_build(m, ctx, orc):
    """Finding 3: subtree roots of power-of-two shards + top levels == full root."""
    from immustore_amd import _native as N
    rng = np.random.default_rng(8)
    for n, shard in [(1000, 128), (1 << 14, 1 << 11), (5000, 1024), (4097, 512)]:
        d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        roots = [orc.htree_build(d[i:i + shard])[1] for i in range(0, n, shard)]
        w = len(roots)
        dn = DevBuf.from_host(ctx, np.frombuffer(b"".join(roots), np.uint8))
        dl = DevBuf(ctx, m.levels_len(w) * 32)
        dr = DevBuf(ctx, 32)
        N.check(N.load().mh_dev_htree_reduce_nodes(ctx.handle, dn.ptr, w, dl.ptr, dr.ptr))
        assert dr.to_host().tobytes() == orc.htree_build(d)[1]


def test_reduce_nodes_levels_every_small_width(m, ctx, orc):
    """mh_dev_htree_reduce_nodes for every width 1..70 (the single-wave
    k_reduce_small up to 64, the level kernels above): every level above the
    row (htree.go:85-110 without the leaf step: pairs hashed, an odd last node
    promoted unchanged) and the root, against a host restatement over the
    oracle's SHA-256."""
    from immustore_amd import _native as N
    rng = np.random.default_rng(81)
    for w in list(range(1, 71)) + [127, 128, 129]:
        row = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(w)]
        want, lvl = list(row), list(row)
        while len(lvl) > 1:
            nxt = [orc.sha256(b"\x01" + lvl[i] + lvl[i + 1]) for i in range(0, len(lvl) - 1, 2)]
            if len(lvl) % 2:
                nxt.append(lvl[-1])
            want += nxt
            lvl = nxt
        dn = DevBuf.from_host(ctx, np.frombuffer(b"".join(row), np.uint8))
        dl = DevBuf(ctx, m.levels_len(w) * 32)
        dr = DevBuf(ctx, 32)
        N.check(N.load().mh_dev_htree_reduce_nodes(ctx.handle, dn.ptr, w, dl.ptr, dr.ptr))
        assert len(want) == m.levels_len(w)
        assert dl.to_host().tobytes() == b"".join(want), w
        assert dr.to_host().tobytes() == lvl[0], w


# ------------------------------------------------------------------ ahtree
def test_ahtree_golden_small(m, ctx, synthetic):
    a = synthetic["ahtree"]
    t = m.AHtree(ctx)
    for i in range(1, 301):
        n, r = t.append(bytes([i & 0xFF]))
        assert n == i and r.hex() == a["roots"][i - 1]
    # rest in one batch of 1-byte payloads
    p = np.array([[i & 0xFF] for i in range(301, a["n"] + 1)], np.uint8)
    roots = t.append_batch(p, with_roots=True)
    assert [x.tobytes().hex() for x in roots] == a["roots"][300:]
    assert H(t.dlog()).hex() == a["dlog_sha256"]
    for i in (1, 2, 17, 1024, 1100):
        assert t.root_at(i).hex() == a["roots"][i - 1]
    with pytest.raises(m.ErrIllegalArguments):
        t.root_at(0)
    with pytest.raises(m.ErrUnexistentData):
        t.root_at(1101)
    with pytest.raises(m.ErrEmptyTree):
        m.AHtree(ctx).root()
    with pytest.raises(m.ErrIllegalArguments):
        t.append(None)
    for pr in synthetic["ahtree_proofs"]:
        i, j = pr["i"], pr["j"]
        assert [x.hex() for x in t.inclusion_proof(i, j)] == pr["iproof"]
        assert [x.hex() for x in t.consistency_proof(i, j)] == pr["cproof"]
    with pytest.raises(m.ErrIllegalArguments):
        t.inclusion_proof(2, 1)
    with pytest.raises(m.ErrIllegalArguments):
        t.consistency_proof(2, 1)


def test_ahtree_go_fixture_dlogs(m, ctx, fixtures):
    for name, fx in fixtures.items():
        pay = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
        t = m.AHtree(ctx)
        t.append_batch(pay)
        assert t.dlog() == bytes.fromhex(fx["aht_dlog"]), name
        # one at a time as the store does (immustore.go:1939-1946)
        t2 = m.AHtree(ctx)
        for p in pay:
            t2.append(p.tobytes())
        assert t2.dlog() == bytes.fromhex(fx["aht_dlog"]), name


def test_ahtree_random_batches_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(21)
    t = m.AHtree(ctx)
    o = orc.AHtree()
    total = 0
    for bs in [1, 1, 2, 3, 7, 64, 1, 1000, 4096, 5, 33333, 1, 2]:
        p = rng.integers(0, 256, (bs, 32), dtype=np.uint8)
        roots = t.append_batch(p, with_roots=True)
        o.append_batch(p)
        total += bs
        assert t.size() == total
        assert t.dlog() == o.dlog_bytes()
        assert roots[-1].tobytes() == o.root_at(total)[1]
    # reset and re-append (ResetSize, ahtree.go:375-458)
    t.reset_size(total - 10)
    with pytest.raises(m.ErrCannotResetToLargerSize):
        t.reset_size(total + 1)
    o2 = orc.AHtree()
    # rebuild oracle to the same prefix then the same suffix
    t.append_batch(np.zeros((10, 32), np.uint8))
    assert t.root_at(total - 10) == o.root_at(total - 10)[1]
    # variable-size payloads (generic leaf path)
    t3 = m.AHtree(ctx)
    for ln in [0, 1, 31, 32, 33, 55, 56, 63, 64, 100, 1000]:
        pp = rng.integers(0, 256, (5, ln), dtype=np.uint8) if ln else np.zeros((5, 0), np.uint8)
        t3.append_batch(pp)
        for row in pp:
            o2.append(row.tobytes())
    assert t3.dlog() == o2.dlog_bytes()


def test_ahtree_large_recurrence(m, ctx, orc):
    """10^6 appends: sampled appends re-derived from the dLog's own nodes
    (ahtree.go:296-322) with the oracle's SHA-256, plus a 2^17 prefix vs oracle."""
    rng = np.random.default_rng(4)
    M = 10 ** 6
    pay = orc.fill_random(32 * M, 3).reshape(M, 32)
    t = m.AHtree(ctx)
    t.append_batch(pay[: 1 << 17])
    o = orc.AHtree(1 << 17)
    o.append_batch(pay[: 1 << 17])
    assert t.dlog() == o.dlog_bytes()
    t.append_batch(pay[1 << 17:])
    dl = np.frombuffer(t.dlog(), np.uint8).reshape(-1, 32)
    assert dl.shape[0] == orc.nodes_upto(M)

    def node(k, l):
        return dl[orc.nodes_until(k) + l].tobytes()

    for n in list(rng.integers(1, M + 1, 3000)) + [M, M - 1, 1 << 19, (1 << 19) + 1]:
        n = int(n)
        h = H(b"\x00" + pay[n - 1].tobytes())
        base = orc.nodes_until(n)
        assert dl[base].tobytes() == h
        w, k, l, cnt = n - 1, n - 1, 0, 1
        while w > 0:
            if w & 1:
                h = H(b"\x01" + node(k, l) + h)
                assert dl[base + cnt].tobytes() == h, (n, l)
                cnt += 1
            k &= ~(1 << l)
            w >>= 1
            l += 1


def test_ahtree_verify_batch_vs_oracle(m, ctx, orc):
    from immustore_amd import _native as N
    rng = np.random.default_rng(9)
    o = orc.AHtree()
    pay = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    o.append_batch(pay)
    inc, cons, last, exp_i, exp_c, exp_l = [], [], [], [], [], []
    for _ in range(600):
        j = int(rng.integers(1, 701))
        i = int(rng.integers(1, j + 1))
        _, ip = o.inclusion_proof(i, j)
        _, cp = o.consistency_proof(i, j)
        ip = [x.tobytes() for x in ip]
        cp = [x.tobytes() for x in cp]
        leaf = H(b"\x00" + pay[i - 1].tobytes())
        jr = o.root_at(j)[1]
        ir = o.root_at(i)[1]
        if rng.random() < 0.2 and ip:
            k = int(rng.integers(0, len(ip)))
            ip[k] = bytes([ip[k][0] ^ 1]) + ip[k][1:]
        if rng.random() < 0.2 and cp:
            k = int(rng.integers(0, len(cp)))
            cp[k] = bytes([cp[k][0] ^ 1]) + cp[k][1:]
        ii = i if rng.random() > 0.05 else 0
        inc.append((ip, ii, j, leaf, jr))
        exp_i.append(orc.ahtree_verify_inclusion(ip, ii, j, leaf, jr))
        cons.append((cp, i, j, ir, jr))
        exp_c.append(orc.ahtree_verify_consistency(cp, i, j, ir, jr))
        _, lp = o.inclusion_proof(i, j)
        lp = [x.tobytes() for x in lp]
        last.append((lp, i, j, leaf, ir))
        exp_l.append(orc.ahtree_verify_last_inclusion(lp, i, leaf, ir))
    assert list(m.ahtree_verify_batch(N.MH_AHT_INCLUSION, inc, ctx)[0]) == exp_i
    assert list(m.ahtree_verify_batch(N.MH_AHT_CONSISTENCY, cons, ctx)[0]) == exp_c
    assert list(m.ahtree_verify_batch(N.MH_AHT_LAST_INCLUSION, last, ctx)[0]) == exp_l
    assert any(exp_i) and not all(exp_i) and any(exp_c) and not all(exp_c) and any(exp_l)
    # verification_test.go:26-32 edge cases
    z = H(b"")
    assert not m.ahtree_verify_inclusion([], 1, 10, z, z, ctx)
    assert not m.ahtree_verify_inclusion([], 10, 1, z, z, ctx)
    assert not m.ahtree_verify_consistency([], 1, 10, z, z, ctx)
    assert not m.ahtree_verify_consistency([], 10, 1, z, z, ctx)
    assert m.ahtree_verify_consistency([], 5, 5, z, z, ctx)


def test_htree_verify_batch_c5_shape(m, ctx, orc):
    """BASELINE configs[4] shape at reduced count: depth-24 proofs over a
    2^24-leaf tree would need 512 MiB of levels on the host oracle; use a
    2^16-leaf tree (depth 16) and 20k proofs with 10 % tampered."""
    rng = np.random.default_rng(5)
    w = 1 << 16
    d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
    lv, root = orc.htree_build(d)
    P = 20000
    idx = rng.integers(0, w, P)
    proofs, digs, exp = [], [], []
    for i in idx:
        _, terms = orc.htree_inclusion_proof(lv, w, int(i))
        terms = [x.tobytes() for x in terms]
        dg = d[i].tobytes()
        if rng.random() < 0.1:
            k = int(rng.integers(0, len(terms)))
            terms[k] = bytes([terms[k][0] ^ 0x80]) + terms[k][1:]
        proofs.append(m.InclusionProof(int(i), w, terms))
        digs.append(dg)
        exp.append(orc.htree_verify_inclusion(int(i), w, terms, dg, root))
    got = m.verify_inclusion_batch(proofs, digs, [root] * P, ctx)
    assert list(got) == exp
    assert 0.85 < np.mean(exp) < 0.95


# ------------------------------------------------------------------ device proof generation
def test_htree_inclusion_proof_batch_vs_oracle(m, ctx, orc):
    """InclusionProof (htree.go:121-164) generated on the
    device for every leaf of several widths, equal to the oracle's proofs."""
    rng = np.random.default_rng(12)
    for w in [1, 2, 3, 5, 8, 17, 100, 1000, 1025, 4096, 5000]:
        d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
        t = m.HTree(max(w, 1), ctx)
        t.build_with(d)
        lv, _ = orc.htree_build(d)
        leaves = np.arange(w) if w <= 1025 else rng.integers(0, w, 700)
        terms, nt, st = t.inclusion_proof_batch(leaves)
        assert not st.any()
        for k, i in enumerate(leaves):
            _, ot = orc.htree_inclusion_proof(lv, w, int(i))
            assert nt[k] == len(ot) and terms[k, :nt[k]].tobytes() == ot.tobytes(), (w, i)
        _, _, st = t.inclusion_proof_batch([w])
        assert st[0] == m._native.MH_ERR_ILLEGAL_ARGUMENTS
        t.close()


def test_ahtree_proof_batch_vs_oracle(m, ctx, orc):
    """ahtree InclusionProof / ConsistencyProof (ahtree.go:525-651) on the
    device for all pairs j <= 70 and random pairs up to 10^5."""
    N_ = 100000
    pay = orc.fill_random(32 * N_, 21).reshape(N_, 32)
    t = m.AHtree(ctx)
    t.append_batch(pay)
    o = orc.AHtree(N_)
    o.append_batch(pay)
    rng = np.random.default_rng(13)
    pairs = [(i, j) for j in range(1, 71) for i in range(0, j + 1)]
    jj = rng.integers(1, N_ + 1, 3000)
    pairs += [(int(rng.integers(1, j + 1)), int(j)) for j in jj] + [(N_, N_), (1, N_)]
    I = np.array([p[0] for p in pairs], np.uint64)
    J = np.array([p[1] for p in pairs], np.uint64)
    for kind, fn in ((0, o.inclusion_proof), (1, o.consistency_proof)):
        terms, nt, st = t.proof_batch(kind, I, J)
        assert not st.any()
        for k, (i, j) in enumerate(pairs):
            if i == 0:
                continue  # the oracle's proof walk needs i >= 1
            _, ot = fn(i, j)
            assert nt[k] == len(ot) and terms[k, :nt[k]].tobytes() == ot.tobytes(), (kind, i, j)
    # argument checks (ahtree.go:534-540)
    _, _, st = t.proof_batch(0, [5, 1, 0], [4, N_ + 1, 0])
    assert list(st) == [2, 5, 5]
    t.close()


def _aht_verify_csr(m, ctx, kind, i, j, terms, nt, a, b):
    """mh_ahtree_verify_batch over device-generated proofs (terms[n, max, 32],
    nt[n]) as a CSR term list -> ok[n]."""
    from immustore_amd import _native as N
    mask = np.arange(terms.shape[1])[None, :] < nt[:, None]
    flat = np.ascontiguousarray(terms[mask]) if nt.sum() else np.zeros((1, 32), np.uint8)
    off = np.zeros(len(i) + 1, np.uint64)
    off[1:] = np.cumsum(nt.astype(np.uint64))
    ok = np.zeros(len(i), np.uint8)
    vi = np.ascontiguousarray(i, np.uint64)
    vj = np.ascontiguousarray(j, np.uint64)
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    N.check(N.load().mh_ahtree_verify_batch(ctx.handle, kind, len(i), vi.ctypes.data,
                                            vj.ctypes.data, off.ctypes.data, flat.ctypes.data,
                                            a.ctypes.data, b.ctypes.data, ok.ctypes.data, None))
    return ok.astype(bool)


def test_ahtree_reset_reference_sequence(m, ctx):
    """The reference's TestReset (embedded/ahtree/ahtree_test.go:759-850) on
    the device: 32 one-byte appends, ResetSize(0), 1024 appends of byte(i),
    ResetSize(N+1) -> ErrCannotResetToLargerSize, ResetSize(1024), ResetSize(512);
    then for every 1 <= i <= j <= 512 the inclusion and consistency proofs
    verify against RootAt, and VerifyLastInclusion(InclusionProof(i, 512), i,
    leaf_i, RootAt(i)) holds only for i == 512 (ahtree/verification.go)."""
    from immustore_amd import _native as N
    t = m.AHtree(ctx)
    for i in range(1, 33):
        t.append(bytes([i]))
    t.reset_size(0)
    assert t.size() == 0
    n = 1024
    for i in range(1, n + 1):
        t.append(bytes([i & 0xFF]))  # Go: byte(i)
    with pytest.raises(m.ErrCannotResetToLargerSize):
        t.reset_size(n + 1)
    t.reset_size(n)
    assert t.size() == n
    n = 512
    t.reset_size(n)
    assert t.size() == n
    leaf = np.stack([np.frombuffer(H(b"\x00" + bytes([i & 0xFF])), np.uint8) for i in range(n + 1)])
    root = np.stack([np.zeros(32, np.uint8)] +
                    [np.frombuffer(t.root_at(k), np.uint8) for k in range(1, n + 1)])
    I, J = np.triu_indices(n, 0)
    I = (I + 1).astype(np.uint64)
    J = (J + 1).astype(np.uint64)
    terms, nt, st = t.proof_batch(N.MH_AHT_INCLUSION, I, J, max_terms=32)
    assert (st == 0).all()
    assert _aht_verify_csr(m, ctx, N.MH_AHT_INCLUSION, I, J, terms, nt, leaf[I], root[J]).all()
    terms, nt, st = t.proof_batch(N.MH_AHT_CONSISTENCY, I, J, max_terms=32)
    assert (st == 0).all()
    assert _aht_verify_csr(m, ctx, N.MH_AHT_CONSISTENCY, I, J, terms, nt, root[I], root[J]).all()
    K = np.arange(1, n + 1, dtype=np.uint64)
    terms, nt, st = t.proof_batch(N.MH_AHT_INCLUSION, K, np.full(n, n, np.uint64), max_terms=32)
    assert (st == 0).all()
    ok = _aht_verify_csr(m, ctx, N.MH_AHT_LAST_INCLUSION, K, K, terms, nt, leaf[K], root[K])
    assert list(np.nonzero(ok)[0] + 1) == [n]


def test_ahtree_reference_suite_full_size(m, ctx, orc):
    """The reference's own ahtree suite at ITS size (N = 1024, payload
    {byte(i)}) on the device: TestIntegrity (ahtree_test.go:579-612) and
    TestInclusionAndConsistencyProofs (:647-715).  Every InclusionProof and
    ConsistencyProof for 1 <= i <= j <= 1024 (524,800 pairs each) generated by
    k_ahtree_proof is byte-equal to the oracle's (ahtree.go:525-651) and
    verifies on the device (k_ahtree_verify, ahtree/verification.go:21-109)
    against RootAt; VerifyLastInclusion(InclusionProof(i, N), i, leaf_i,
    RootAt(i)) holds only for i = N; InclusionProof(2, 1) / ConsistencyProof(2,
    1) are ErrIllegalArguments."""
    from immustore_amd import _native as N
    n = 1024
    pay = (np.arange(1, n + 1) & 0xFF).astype(np.uint8).reshape(n, 1)  # Go: []byte{byte(i)}
    t = m.AHtree(ctx)
    t.append_batch(pay)
    o = orc.AHtree(n)
    o.append_batch(pay)
    assert t.dlog() == o.dlog_bytes()
    leaf = np.stack([np.zeros(32, np.uint8)] + [np.frombuffer(H(b"\x00" + bytes([i & 0xFF])), np.uint8)
                                               for i in range(1, n + 1)])
    root = np.stack([np.zeros(32, np.uint8)] +
                    [np.frombuffer(t.root_at(k), np.uint8) for k in range(1, n + 1)])
    assert all(root[k].tobytes() == o.root_at(k)[1] for k in range(1, n + 1))
    I, J = np.triu_indices(n, 0)
    I = (I + 1).astype(np.uint64)
    J = (J + 1).astype(np.uint64)
    for kind, a in ((N.MH_AHT_INCLUSION, leaf[I]), (N.MH_AHT_CONSISTENCY, root[I])):
        terms, nt, st = t.proof_batch(kind, I, J, max_terms=32)
        assert (st == 0).all()
        ot, ont, ost = o.proof_batch(kind, I, J, cap=32)
        assert (ost == 0).all() and np.array_equal(nt, ont)
        mask = np.arange(32)[None, :] < nt[:, None]
        assert np.array_equal(terms[mask], ot[mask]), kind  # every proof byte-equal
        ok = _aht_verify_csr(m, ctx, kind, I, J, terms, nt, a, root[J])
        assert ok.all(), (kind, int((~ok).sum()))
        del terms, ot
    K = np.arange(1, n + 1, dtype=np.uint64)
    terms, nt, st = t.proof_batch(N.MH_AHT_INCLUSION, K, np.full(n, n, np.uint64), max_terms=32)
    assert (st == 0).all()
    ok = _aht_verify_csr(m, ctx, N.MH_AHT_LAST_INCLUSION, K, K, terms, nt, leaf[K], root[K])
    assert list(np.nonzero(ok)[0] + 1) == [n]
    for kind in (N.MH_AHT_INCLUSION, N.MH_AHT_CONSISTENCY):
        _, _, st = t.proof_batch(kind, [2], [1])
        assert list(st) == [N.MH_ERR_ILLEGAL_ARGUMENTS]
    t.close()


# ------------------------------------------ upper levels (k_entries_fixed + k_reduce)
@pytest.mark.parametrize("wgl", ["0", "2", "4", "8"])
def test_entries_fixed_wg_levels_vs_oracle(m, ctx, orc, lpl, wgl):
    """Every depth of the leaf workgroups' in-LDS subtrees (MH_WG_LEVELS) with
    the level reduction above them (htree.go:85-110): widths that cut
    workgroups and 512-node reduce blocks unevenly, and two different data
    sets built alternately into the SAME level / root buffers (a stale read
    of the previous build's nodes would show), all vs the oracle."""
    from immustore_amd import _native as N
    old = os.environ.get("MH_WG_LEVELS")
    os.environ["MH_WG_LEVELS"] = wgl
    try:
        for n in (257, 513, 1025, 4097, 33000, 131073, 262147, 1 << 19, (1 << 20) + 3):
            klen, vlen = 8, 64
            dl = DevBuf(ctx, m.levels_len(n) * 32)
            dr = DevBuf(ctx, 32)
            dh = DevBuf(ctx, n * 32)
            sets = []
            for seed in (31, 32):
                keys, vals = _fixed_inputs(orc, n, klen, vlen, seed + n)
                sets.append((keys, vals, DevBuf.from_host(ctx, keys), DevBuf.from_host(ctx, vals),
                             orc.build_entries_fixed(1, keys, vals, nthreads=8)))
            for k in (0, 1, 0, 1):
                keys, vals, dk, dv, (ohv, olv, oroot) = sets[k]
                N.check(N.load().mh_dev_htree_build_entries_fixed(
                    ctx.handle, 1, n, dk.ptr, klen, dv.ptr, vlen, dh.ptr, dl.ptr, dr.ptr))
                ctx.synchronize()
                assert dr.to_host().tobytes() == oroot, (n, wgl, k)
                assert np.array_equal(dl.to_host().reshape(-1, 32), olv), (n, wgl, k)
                assert np.array_equal(dh.to_host().reshape(-1, 32), ohv), (n, wgl, k)
    finally:
        if old is None:
            del os.environ["MH_WG_LEVELS"]
        else:
            os.environ["MH_WG_LEVELS"] = old


def test_entries_fixed_concurrent_streams(m, orc):
    """Three contexts on three streams building different trees at once
    (the bench's builds in flight): every root and level array matches the
    oracle."""
    import torch
    from immustore_amd import _native as N
    L = N.load()
    n, vlen = (1 << 18) + 77, 256
    streams = [torch.cuda.Stream() for _ in range(3)]
    ctxs = [m.Context(0, s.cuda_stream) for s in streams]
    try:
        jobs = []
        for k, c in enumerate(ctxs):
            keys, vals = _fixed_inputs(orc, n, 8, vlen, 600 + k)
            dk = torch.from_numpy(keys.reshape(-1).copy()).cuda()
            dv = torch.from_numpy(vals.reshape(-1).copy()).cuda()
            lv = torch.empty(m.levels_len(n) * 32, dtype=torch.uint8, device="cuda")
            rt = torch.empty(32, dtype=torch.uint8, device="cuda")
            jobs.append((c, keys, vals, dk, dv, lv, rt))
        torch.cuda.synchronize()
        for rep in range(4):
            for c, keys, vals, dk, dv, lv, rt in jobs:
                N.check(L.mh_dev_htree_build_entries_fixed(c.handle, 1, n, dk.data_ptr(), 8,
                                                           dv.data_ptr(), vlen, None,
                                                           lv.data_ptr(), rt.data_ptr()))
        torch.cuda.synchronize()
        for c, keys, vals, dk, dv, lv, rt in jobs:
            _, olv, oroot = orc.build_entries_fixed(1, keys, vals, nthreads=8)
            assert rt.cpu().numpy().tobytes() == oroot
            assert np.array_equal(lv.cpu().numpy().reshape(-1, 32), olv)
    finally:
        for c in ctxs:
            c.close()
