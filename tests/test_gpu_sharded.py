"""Sharded (multi-GPU) paths of SURVEY.md 8(e) on ONE device: G ranks are run
one after another in this process, each with its own globally indexed dLog,
and the "all-gather" is a device copy.  The per-rank dLog ranges must equal a
single-device append of the whole batch byte for byte (and the oracle's).
The process-group wiring is covered by tests/test_distributed_cpu.py (gloo)
and exercised by bench_workloads.py under torch.distributed.run."""
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


@pytest.mark.parametrize("world,m_total", [(2, 1 << 12), (4, 1 << 16), (3, 3000), (8, 1 << 17),
                                           (4, 1000)])
def test_sharded_ahtree_append_matches_single(m, ctx, orc, world, m_total):
    from immustore_amd import _native as N
    from immustore_amd import sharding
    L = N.load()
    k = sharding.ahtree_shard_bits(world, m_total)
    S = 1 << k
    pay = orc.fill_random(32 * m_total, 17).reshape(m_total, 32)
    nd = m.nodes_upto(m_total)
    # single device reference
    ref = DevBuf(ctx, nd * 32)
    dp = DevBuf.from_host(ctx, pay)
    N.check(L.mh_dev_ahtree_append_batch(ctx.handle, ref.ptr, 0, dp.ptr, m_total, 32, None))
    ctx.synchronize()
    full = ref.to_host().tobytes()
    o = orc.AHtree(m_total)
    o.append_batch(pay)
    assert full == o.dlog_bytes()
    # ranks: phase 1 everywhere, then the exchange, then phase 3 everywhere
    dlogs, spans = [], []
    for r in range(world):
        d = DevBuf(ctx, nd * 32)
        n0, mm = min(r * S, m_total), min(S, max(m_total - r * S, 0))
        if mm:
            pr = DevBuf.from_host(ctx, pay[n0:n0 + mm])
            N.check(L.mh_dev_ahtree_append_local(ctx.handle, d.ptr, n0, pr.ptr, mm, 32, k))
            ctx.synchronize()
        dlogs.append(d)
        spans.append((n0, mm))
    roots = np.zeros((world, 32), np.uint8)
    for r, (n0, mm) in enumerate(spans):
        if mm == S:
            idx = L.mh_ahtree_node_index(n0 + S, k)
            roots[r] = np.frombuffer(dlogs[r].to_host().tobytes()[32 * idx:32 * idx + 32], np.uint8)
    groots = DevBuf.from_host(ctx, roots)
    complete = min(m_total // S, world)
    covered = 0
    for r, (n0, mm) in enumerate(spans):
        if not mm:
            continue
        N.check(L.mh_dev_ahtree_put_shard_roots(ctx.handle, dlogs[r].ptr, k, complete, groots.ptr))
        N.check(L.mh_dev_ahtree_append_spine(ctx.handle, dlogs[r].ptr, n0, mm, None))
        ctx.synchronize()
        lo, hi = L.mh_ahtree_node_index(n0 + 1, 0), m.nodes_upto(n0 + mm)
        got = dlogs[r].to_host().tobytes()[32 * lo:32 * hi]
        assert got == full[32 * lo:32 * hi], r
        covered += hi - lo
    assert covered == nd


def test_sharded_proof_verify_split(m, ctx, orc):
    """C5 split by index across G 'ranks': the concatenated result bitmaps equal
    one batch over all proofs."""
    rng = np.random.default_rng(6)
    w = 1 << 12
    d = rng.integers(0, 256, (w, 32), dtype=np.uint8)
    lv, root = orc.htree_build(d)
    P = 3000
    idx = rng.integers(0, w, P)
    proofs, digs = [], []
    for i in idx:
        _, terms = orc.htree_inclusion_proof(lv, w, int(i))
        terms = [x.tobytes() for x in terms]
        if rng.random() < 0.1:
            terms[0] = bytes([terms[0][0] ^ 1]) + terms[0][1:]
        proofs.append(m.InclusionProof(int(i), w, terms))
        digs.append(d[i].tobytes())
    whole = list(m.verify_inclusion_batch(proofs, digs, [root] * P, ctx))
    parts = []
    for r in range(4):
        lo, hi = r * P // 4, (r + 1) * P // 4
        parts += list(m.verify_inclusion_batch(proofs[lo:hi], digs[lo:hi], [root] * (hi - lo), ctx))
    assert parts == whole and 0.8 < np.mean(whole) < 0.95
