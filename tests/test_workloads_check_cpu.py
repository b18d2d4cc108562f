"""bench_workloads.py's multi-rank result checks on the
CPU: the C3 ranged append check (every rank: the oracle's peaks of its range
start streamed from the payload stream in blocks, its range streamed from
them, sampled digests and RootAt values compared) and the C5 bitmap check,
each verdict shared over gloo ranks the way the GPU ranks share it over RCCL.
The "device" results here are the oracle's full dLog / verdicts in host
memory; a corrupted rank must turn the verdict false on every rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c3_rank(rank, world, port, per_rank, bad_rank, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    import bench_workloads as bw
    import oracle as orc
    from immustore_amd.multi import ahtree_range_plan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seed, plen, total = 3, 32, world * per_rank
        _, b = ahtree_range_plan(0, total, world)
        G = len(b) - 1
        lo, hi = (b[rank], b[rank + 1]) if rank < G else (b[G], b[G])
        o = orc.AHtree(total)
        o.append_batch(orc.fill_random(total * plen, seed).reshape(total, plen))
        dl = o.dlog[orc.nodes_upto(lo):orc.nodes_upto(hi)].copy()  # the "device" range
        if rank == bad_rank:
            dl[5, 0] ^= 1
        roots = np.stack([np.frombuffer(o.root_at(n)[1], np.uint8) for n in range(lo + 1, hi + 1)]) \
            if hi > lo else np.zeros((0, 32), np.uint8)
        ok, root = True, b"\0" * 32
        if hi > lo:
            s = bw.aht_samples(lo, hi, np.random.default_rng(rank), edge=8, rand=32)
            ok, root = bw.c3_rank_check(orc, seed, plen, lo, hi, lambda i: dl[i], lambda i: roots[i],
                                        s, 2)
        ok_all, bad, rts = bw.share_verdict(dist, "gloo", torch.device("cpu"), ok,
                                            rank == bad_rank, root)
        q.put((rank, ok_all, bad, rts[G - 1], bytes(o.root_at(total)[1])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,per_rank,bad_rank", [(2, 1 << 10, -1), (2, 1 << 10, 1),
                                                     (8, 1 << 9, -1), (8, 1 << 9, 6),
                                                     (3, 333, -1)])
def test_c3_rank_check_gloo(world, per_rank, bad_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_c3_rank, args=(r, world, port, per_rank, bad_rank, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, ok, bad, root, want in res:
        assert ok == (bad_rank < 0), rank
        assert bad == ([] if bad_rank < 0 else [bad_rank])
        assert root == want  # RootAt(total) as the last range's check reports it


def _c5_rank(rank, world, port, bad_rank, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    import bench_workloads as bw
    import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D, P = 10, 3000
        W = 1 << D
        dig = orc.fill_random(W * 32, 5).reshape(W, 32)
        lv, root = orc.htree_build(dig)
        rng = np.random.default_rng(5 + rank)
        leaf = rng.integers(0, W, P, dtype=np.int64)
        offs = np.array([orc.level_offset(W, l) for l in range(D)], np.int64)
        terms = lv[offs[None, :] + ((leaf[:, None] >> np.arange(D)[None, :]) ^ 1)]
        tamper = rng.random(P) < 0.10
        digs = dig[np.where(tamper, (leaf + 1) % W, leaf)]
        _, ok_dev = orc.htree_verify_batch(leaf.astype(np.uint64), W, terms, digs, root)
        if rank == bad_rank:
            ok_dev = ok_dev.copy()
            ok_dev[int(np.nonzero(~tamper)[0][0])] = 0
        sample = np.unique(np.concatenate([np.arange(64), rng.integers(0, P, 256)]))
        ok, ns = bw.c5_rank_check(orc, leaf, W, terms[sample], digs[sample], root, ok_dev, tamper,
                                  sample)
        ok_all, bad, _ = bw.share_verdict(dist, "gloo", torch.device("cpu"), ok, rank == bad_rank)
        q.put((rank, ok_all, bad, ns))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad_rank", [(2, -1), (2, 0), (8, -1), (8, 3)])
def test_c5_rank_check_gloo(world, bad_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_c5_rank, args=(r, world, port, bad_rank, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, ok, bad, ns in res:
        assert ok == (bad_rank < 0), rank
        assert bad == ([] if bad_rank < 0 else [bad_rank]) and ns > 64


def test_aht_samples_cover_both_ends():
    sys.path.insert(0, ROOT)
    import bench_workloads as bw
    s = bw.aht_samples(100, 1000, np.random.default_rng(0), edge=8, rand=16)
    assert s[0] == 101 and s[-1] == 1000 and list(s[:8]) == list(range(101, 109))
    assert (np.diff(s.astype(np.int64)) > 0).all()
    s = bw.aht_samples(0, 3, np.random.default_rng(0))
    assert list(s) == [1, 2, 3]


def test_force_pg_relaunches_one_rank(tmp_path):
    """MH_DIST_FORCE_PG=1 without WORLD_SIZE: bench_workloads.py restarts
    itself as one torch.distributed.run rank (child process) -- here with a
    GPU-less host: the child reaches distributed_main under the launcher and
    fails there (no device), and the parent exits with the child's status."""
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(MH_DIST_FORCE_PG="1", MH_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench_workloads.py"), "--workload",
                        "wire"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0
    assert "in distributed_main" in r.stderr, r.stderr[-3000:]
    assert os.path.join("torch", "distributed", "run.py") in r.stderr, r.stderr[-3000:]
