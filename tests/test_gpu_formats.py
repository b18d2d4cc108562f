"""GPU parity for SURVEY.md 8(f) row 4, the formats either side of the path:
- the ahtree appendable record streams (pLog / cLog / dLog, ahtree.go:266-351)
  written by the device next to the dLog, pinned by the Go-written
  aht/{data,commit,tree} files of the reference's test stores
  (tests/golden/immudb_fixtures.json) and the oracle (orc_ahtree_log_records);
- proofs as protobuf messages (InclusionProof, DualProofV2 with TxHeader /
  TxMetadata; pkg/api/schema/schema.proto, database_protoconv.go) generated and
  encoded on the device, against oracle/wire.py (C-oracle proofs serialised by
  the protobuf runtime).  Bit-exact.
"""
import ctypes as C

import numpy as np
import pytest

from gpu_util import DevBuf

pytestmark = pytest.mark.gpu


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


def expected_logs(pay, p_off0):
    """numpy restatement of the record streams for a fixed payload size."""
    mm, plen = pay.shape
    rec = 4 + plen
    plog = np.zeros((mm, rec), np.uint8)
    plog[:, :4] = np.frombuffer(np.uint32(plen).byteswap().tobytes(), np.uint8)
    plog[:, 4:] = pay
    clog = np.zeros((mm, 12), np.uint8)
    off = (p_off0 + np.arange(mm, dtype=np.uint64) * np.uint64(rec)).astype(">u8")
    clog[:, :8] = off.view(np.uint8).reshape(mm, 8)
    clog[:, 8:] = np.frombuffer(np.uint32(plen).byteswap().tobytes(), np.uint8)
    return plog.tobytes(), clog.tobytes()


@pytest.mark.parametrize("split", [0, 1, 5, 1000])
def test_go_fixture_appendables(m, ctx, fixtures, split):
    for name, fx in fixtures.items():
        pay = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
        k = min(split, len(pay))
        t = m.AHtree(ctx)
        p1, c1 = t.append_batch_logs(pay[:k], 0)
        p2, c2 = t.append_batch_logs(pay[k:], len(p1))
        assert p1 + p2 == bytes.fromhex(fx["aht_plog"]), name
        assert c1 + c2 == bytes.fromhex(fx["aht_clog"]), name
        assert t.dlog() == bytes.fromhex(fx["aht_dlog"]), name


def test_appendables_random_batches_vs_oracle(m, ctx, orc):
    rng = np.random.default_rng(44)
    t = m.AHtree(ctx)
    o = orc.AHtree()
    poff = 0
    for bs in [1, 255, 256, 257, 3, 4096, 70001, 2]:
        p = rng.integers(0, 256, (bs, 32), dtype=np.uint8)
        pl, cl = t.append_batch_logs(p, poff)
        opl, ocl = o.append_batch_logs(p, poff)
        assert pl == opl and cl == ocl, bs
        assert t.dlog() == o.dlog_bytes()
        poff += len(pl)
    # other payload sizes take the per-lane byte path
    for plen in [0, 1, 31, 33, 100]:
        p = rng.integers(0, 256, (300, plen), dtype=np.uint8)
        pl, cl = t.append_batch_logs(p, poff)
        opl, ocl = o.append_batch_logs(p, poff)
        assert pl == opl and cl == ocl, plen
        assert t.dlog() == o.dlog_bytes()
        poff += len(pl)


def test_appendables_large_offsets(m, ctx):
    """10^6 appends with a pLog offset above 2^32 (BE64 high word in use)."""
    from immustore_amd import _native as N
    M = 10 ** 6
    pay = np.random.default_rng(5).integers(0, 256, (M, 32), dtype=np.uint8)
    p0 = (1 << 32) + 12345 * 36
    t = m.AHtree(ctx)
    pl, cl = t.append_batch_logs(pay, p0)
    epl, ecl = expected_logs(pay, p0)
    assert pl == epl and cl == ecl
    # fused device call == separate append + records-only call
    L = N.load()
    dpay = DevBuf.from_host(ctx, pay)
    dl = DevBuf(ctx, orc_nodes_upto(M) * 32)
    dpl, dcl = DevBuf(ctx, M * 36), DevBuf(ctx, M * 12)
    N.check(L.mh_dev_ahtree_append_batch_logs(ctx.handle, C.c_void_p(dl.ptr), 0,
                                              C.c_void_p(dpay.ptr), M, 32, p0,
                                              C.c_void_p(dpl.ptr), C.c_void_p(dcl.ptr), None))
    ctx.synchronize()
    assert dpl.to_host().tobytes() == epl and dcl.to_host().tobytes() == ecl
    assert dl.to_host().tobytes() == t.dlog()


def orc_nodes_upto(n):
    from immustore_amd import _native as N
    return N.load().mh_ahtree_nodes_upto(n)


@pytest.mark.parametrize("shift", [0, 4, 1])
def test_records_only_alignment(m, ctx, shift):
    """mh_dev_ahtree_log_records at 16-, 4- and 1-byte aligned outputs (LDS
    staged dword stores vs the byte path) and with m not a multiple of 256."""
    from immustore_amd import _native as N
    L = N.load()
    M = 1000
    pay = np.random.default_rng(shift).integers(0, 256, (M, 32), dtype=np.uint8)
    dpay = DevBuf.from_host(ctx, pay)
    dpl, dcl = DevBuf(ctx, M * 36 + 32), DevBuf(ctx, M * 12 + 32)
    N.check(L.mh_dev_ahtree_log_records(ctx.handle, C.c_void_p(dpay.ptr), M, 32, 777,
                                        C.c_void_p(dpl.ptr + shift), C.c_void_p(dcl.ptr + shift)))
    ctx.synchronize()
    epl, ecl = expected_logs(pay, 777)
    assert dpl.to_host()[shift:shift + M * 36].tobytes() == epl
    assert dcl.to_host()[shift:shift + M * 12].tobytes() == ecl
    # NULL outputs and m = 0 are no-ops; offsets that overflow uint64 are rejected
    N.check(L.mh_dev_ahtree_log_records(ctx.handle, C.c_void_p(dpay.ptr), M, 32, 0, None, None))
    N.check(L.mh_dev_ahtree_log_records(ctx.handle, None, 0, 32, 0, C.c_void_p(dpl.ptr), None))
    assert L.mh_dev_ahtree_log_records(ctx.handle, C.c_void_p(dpay.ptr), M, 32, (1 << 64) - 100,
                                       C.c_void_p(dpl.ptr), None) == N.MH_ERR_ILLEGAL_ARGUMENTS


# ---------------------------------------------------------------- protobuf proofs
@pytest.fixture(scope="module")
def wire(orc):
    import wire
    return wire


@pytest.fixture(params=["wave", "staged"])
def writer(request, monkeypatch):
    """both protobuf record writers: wave-dense (trees below 2^32 nodes, the
    default) and staged (larger trees; forced with MH_PB_STAGED=1)."""
    if request.param == "staged":
        monkeypatch.setenv("MH_PB_STAGED", "1")
    else:
        monkeypatch.delenv("MH_PB_STAGED", raising=False)
    return request.param


def _rec_hdr(r, blob):
    return {"id": int(r["id"]), "ts": int(r["ts"]), "bltxid": int(r["bl_tx_id"]),
            "blroot": r["bl_root"].tobytes(), "prevalh": r["prev_alh"].tobytes(),
            "eh": r["eh"].tobytes(), "version": int(r["version"]), "nentries": int(r["nentries"]),
            "md": blob[int(r["md_off"]):int(r["md_off"]) + int(r["md_len"])]}


def test_dual_proof_v2_pb_fixture_stores(m, ctx, orc, wire, fixtures, writer):
    from tx_util import headers_from_fixture
    for name, fx in fixtures.items():
        pay = np.stack([np.frombuffer(bytes.fromhex(p), np.uint8) for p in fx["aht_payloads"]])
        t = m.AHtree(ctx)
        t.append_batch(pay)
        o = orc.AHtree()
        o.append_batch(pay)
        recs, blob, _ = headers_from_fixture(fx["txs"])
        cases = [(c["src"], c["tgt"]) for c in fx["dual_v2"]]
        # plus the Go error cases: newer source, broken linking
        cases += [(2, 1), (2, 2)]
        s = recs[[a - 1 for a, _ in cases]]
        g = recs[[b - 1 for _, b in cases]]
        g[-1]["bl_tx_id"] = 0 if g[-1]["id"] != 1 else 5  # linking error
        msgs, st = t.dual_proof_v2_pb_batch(s, g, blob)
        for k in range(len(cases)):
            est, eb = wire.dual_proof_v2_pb(_rec_hdr(s[k], blob), _rec_hdr(g[k], blob), o)
            assert st[k] == est and msgs[k] == eb, (name, cases[k])
        assert st[-2] == wire.MH_ERR_SOURCE_TX_NEWER and st[-1] == wire.MH_ERR_UNEXPECTED_LINKING


def _random_headers(rng, n_tx, with_md=True):
    from tx_util import TX_HEADER
    recs = np.zeros(n_tx, TX_HEADER)
    blob = bytearray()
    for k in range(n_tx):
        r = recs[k]
        r["id"] = k + 1
        r["bl_tx_id"] = k
        r["ts"] = int(rng.integers(-2**40, 2**40)) if k % 7 else 0
        for f in ("bl_root", "prev_alh", "eh"):
            r[f] = rng.integers(0, 256, 32, dtype=np.uint8)
        r["version"] = 1 if k % 5 else 0
        r["nentries"] = [0, 1, 127, 128, 300, 2**31 + 5, 2**32 - 1][k % 7]
        md = b""
        if with_md and r["version"] == 1 and k % 3:
            kind = k % 4
            if kind == 0:
                md = bytes([0]) + int(rng.integers(0, 2**63)).to_bytes(8, "big")
            elif kind == 1:
                ln = int(rng.integers(0, 257))
                md = bytes([1]) + ln.to_bytes(2, "big") + rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            elif kind == 2:
                md = bytes([0]) + bytes(8) + bytes([1, 0, 0])  # zero id, empty extra: empty message
            else:
                md = bytes([0]) + (200).to_bytes(8, "big") + bytes([1, 0, 3]) + b"abc"
        r["md_len"], r["md_off"] = len(md), len(blob)
        blob += md
    return recs, bytes(blob)


def test_dual_proof_v2_pb_random_vs_oracle(m, ctx, orc, wire, writer):
    rng = np.random.default_rng(91)
    N_TX = 70000
    pay = rng.integers(0, 256, (N_TX, 32), dtype=np.uint8)
    t = m.AHtree(ctx)
    t.append_batch(pay)
    o = orc.AHtree(N_TX)
    o.append_batch(pay)
    recs, blob = _random_headers(rng, N_TX + 10)
    tgt = rng.integers(1, N_TX + 2, 3000)
    src = np.array([int(rng.integers(1, x + 1)) for x in tgt])
    src[:5] = tgt[:5]            # same tx: headers only
    src[5:8] = tgt[5:8] + 1      # newer source
    src[8] = 0                   # id 0
    tgt[9] = N_TX + 5            # beyond the tree
    s = recs[np.maximum(src, 1) - 1].copy()
    s[8]["id"] = 0
    g = recs[tgt - 1]
    msgs, st = t.dual_proof_v2_pb_batch(s, g, blob)
    for k in range(len(tgt)):
        est, eb = wire.dual_proof_v2_pb(_rec_hdr(s[k], blob), _rec_hdr(g[k], blob), o)
        assert st[k] == est and msgs[k] == eb, (k, int(src[k]), int(tgt[k]))
    assert (st == 0).sum() > 2900


def test_htree_inclusion_proof_pb_vs_oracle(m, ctx, orc, wire, writer):
    rng = np.random.default_rng(17)
    for w in [1, 2, 3, 1000, (1 << 18) + 3]:
        d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
        h = m.HTree(w, ctx)
        h.build_with(d)
        lv, _ = orc.htree_build(d)
        leaves = np.concatenate([rng.integers(0, w, 500), [0, w - 1, w, w + 7]]).astype(np.uint64)
        msgs, st = h.inclusion_proof_pb_batch(leaves)
        for k, i in enumerate(leaves):
            est, eb = wire.htree_inclusion_proof_pb(lv, w, int(i))
            assert st[k] == est and msgs[k] == eb, (w, int(i))


def test_pb_device_phases_and_capacity(m, ctx, orc, wire, writer):
    """phase 1 (sizes/offsets) then phase 2 (write) through the device ABI; a
    too-small output marks exactly the messages past the capacity."""
    from immustore_amd import _native as N
    L = N.load()
    rng = np.random.default_rng(3)
    w = 4097
    d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
    h = m.HTree(w, ctx)
    h.build_with(d)
    lv_ptr = h.levels_device_ptr()
    n = 777
    leaves = rng.integers(0, w, n).astype(np.uint64)
    dleaf = DevBuf.from_host(ctx, leaves)
    doff = DevBuf(ctx, (n + 1) * 8)
    dst = DevBuf(ctx, n * 4)
    scr = DevBuf(ctx, L.mh_pb_scratch_size(n))
    N.check(L.mh_dev_htree_inclusion_proof_pb_batch(ctx.handle, 1, C.c_void_p(lv_ptr), w, n,
                                                    C.c_void_p(dleaf.ptr), None, 0,
                                                    C.c_void_p(doff.ptr), C.c_void_p(dst.ptr),
                                                    C.c_void_p(scr.ptr)))
    ctx.synchronize()
    off = doff.to_host(np.uint64)
    assert off[0] == 0 and np.all(np.diff(off.astype(np.int64)) > 0)
    cap = int(off[n // 2])
    dout = DevBuf(ctx, int(off[n]))
    N.check(L.mh_dev_htree_inclusion_proof_pb_batch(ctx.handle, 2, C.c_void_p(lv_ptr), w, n,
                                                    C.c_void_p(dleaf.ptr), C.c_void_p(dout.ptr),
                                                    cap, C.c_void_p(doff.ptr), C.c_void_p(dst.ptr),
                                                    C.c_void_p(scr.ptr)))
    ctx.synchronize()
    st = dst.to_host(np.int32)
    out = dout.to_host()
    lv, _ = orc.htree_build(d)
    for k in range(n):
        if off[k + 1] <= cap:
            assert st[k] == 0
            assert out[off[k]:off[k + 1]].tobytes() == wire.htree_inclusion_proof_pb(lv, w, int(leaves[k]))[1]
        else:
            assert st[k] == N.MH_ERR_BUFFER_TOO_SMALL
    # host API: a too-small buffer returns the sizes so the caller can retry
    offh = np.zeros(n + 1, np.uint64)
    sth = np.zeros(n, np.int32)
    small = np.zeros(16, np.uint8)
    r = L.mh_htree_inclusion_proof_pb_batch(h.handle, n, leaves.ctypes.data, small.ctypes.data, 16,
                                            offh.ctypes.data, sth.ctypes.data)
    assert r == N.MH_ERR_BUFFER_TOO_SMALL and np.array_equal(offh, off)
