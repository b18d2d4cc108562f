"""Multi-rank htree build on CPU (gloo): the sharding + all-gather logic of the
multi-GPU path (immustore_amd/sharding.py, used by bench.py --gpus N) with
the oracle doing the hashing.  The GPU version swaps the oracle for the HIP
kernels and gloo for RCCL; the exchange is the same 32 B per rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, seed, q):
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root_dir, os.path.join(root_dir, "oracle")]
    import torch.distributed as dist
    import oracle as orc
    from immustore_amd import sharding
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        digs = orc.fill_random(n * 32, seed).reshape(n, 32)
        lo, hi = sharding.shard_range(rank, world, n)
        if hi > lo:
            _, sub = orc.htree_build(digs[lo:hi])
        else:
            sub = b"\0" * 32
        r = torch.from_numpy(np.frombuffer(sub, np.uint8).copy())
        g = sharding.allgather_roots(r, world)
        g = sharding.nonempty_roots(g, world, n)
        roots = g.numpy().reshape(-1, 32)
        # top levels: pair the chunk roots with htree's rule (no leaf hashing)
        lvl = [bytes(x) for x in roots]
        while len(lvl) > 1:
            nxt = [orc.sha256(b"\x01" + lvl[i] + lvl[i + 1]) for i in range(0, len(lvl) - 1, 2)]
            if len(lvl) % 2:
                nxt.append(lvl[-1])
            lvl = nxt
        q.put((rank, lvl[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1 << 12), (2, 1000), (3, 1025), (4, 4097), (2, 1),
                                     (8, 1 << 13), (8, 5001)])
def test_sharded_build_equals_single_tree(world, n, orc):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 77, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    digs = orc.fill_random(n * 32, 77).reshape(n, 32)
    _, full = orc.htree_build(digs)
    assert all(r == full for r in res.values())


def test_shard_ranges_power_of_two():
    from immustore_amd.sharding import shard_range
    for world in (1, 2, 3, 4, 8):
        for n in (1, 7, 8, 1000, 1 << 20, (1 << 20) + 5):
            covered = 0
            for r in range(world):
                lo, hi = shard_range(r, world, n)
                assert lo == min(covered, n) or hi == lo
                size = hi - lo
                covered = max(covered, hi)
                if r < world - 1 and hi < n:
                    assert size and (size & (size - 1)) == 0
            assert covered == n


def _aht_model_rank(rank, world, k, pay, orc):
    """Pure-Python model of immustore_amd.sharding.ahtree_sharded_append's three
    phases for one rank (ahtree.go:246-322 split by range): returns the rank's
    dLog entries {index: digest} and its shard root."""
    import hashlib
    H = lambda b: hashlib.sha256(b).digest()  # noqa: E731
    S, m_total = 1 << k, len(pay)
    n0, m = rank * S, min(S, len(pay) - rank * S)
    d = {}
    nu = orc.nodes_until
    for n in range(n0 + 1, n0 + m + 1):                     # leaves
        d[nu(n)] = H(b"\x00" + pay[n - 1])
    for l in range(1, k + 1):                               # perfect, levels <= k
        for e in range(((n0 >> l) + 1) << l, n0 + m + 1, 1 << l):
            d[nu(e) + l] = H(b"\x01" + d[nu(e - (1 << (l - 1))) + l - 1] + d[nu(e) + l - 1])
    root = d[nu(n0 + S) + k] if m == S else b"\0" * 32
    return d, root, n0, m


def _aht_worker(rank, world, port, k, m_total, q):
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root_dir, os.path.join(root_dir, "oracle")]
    import hashlib
    import torch.distributed as dist
    import oracle as orc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        H = lambda b: hashlib.sha256(b).digest()  # noqa: E731
        raw = orc.fill_random(32 * m_total, 9)
        pay = [bytes(raw[32 * i:32 * i + 32]) for i in range(m_total)]
        d, root, n0, m = _aht_model_rank(rank, world, k, pay, orc)
        g = torch.empty(world * 32, dtype=torch.uint8)
        dist.all_gather_into_tensor(g, torch.frombuffer(bytearray(root), dtype=torch.uint8))
        roots = [bytes(g[32 * r:32 * r + 32].numpy()) for r in range(world)]
        nu, S = orc.nodes_until, 1 << k
        complete = min(m_total // S, world)
        for r in range(complete):                           # put_shard_roots
            d[nu((r + 1) * S) + k] = roots[r]
        for l in range(k + 1, 64):
            if (complete * S) >> l == 0:
                break
            for e in range(1 << l, complete * S + 1, 1 << l):
                d[nu(e) + l] = H(b"\x01" + d[nu(e - (1 << (l - 1))) + l - 1] + d[nu(e) + l - 1])
        for n in range(n0 + 1, n0 + m + 1):                 # spine (ahtree.go:296-322)
            h, w, kk, l, c = d[nu(n)], n - 1, n - 1, 0, 1
            while w > 0:
                if w & 1:
                    h = H(b"\x01" + d[nu(kk) + l] + h)
                    d[nu(n) + c] = h
                    c += 1
                kk &= ~(1 << l)
                w >>= 1
                l += 1
        lo, hi = (nu(n0 + 1) if m else 0), (orc.nodes_upto(n0 + m) if m else 0)
        q.put((rank, lo, b"".join(d[i] for i in range(lo, hi))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,m_total", [(2, 3, 16), (4, 2, 16), (3, 3, 20), (4, 4, 64)])
def test_sharded_ahtree_append_equals_single_tree(world, k, m_total, orc):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_aht_worker, args=(r, world, port, k, m_total, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (lo, b)) for r, lo, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t = orc.AHtree()
    raw = orc.fill_random(32 * m_total, 9).reshape(m_total, 32)
    t.append_batch(raw)
    full = t.dlog_bytes()
    covered = 0
    for r in range(world):
        lo, b = res[r]
        assert full[32 * lo:32 * lo + len(b)] == b, r
        covered += len(b)
    assert covered == len(full)


@pytest.mark.parametrize("n", [2, 4])
def test_bench_launcher_spawns_n_ranks(n):
    """`python bench.py --gpus N` without torchrun (WORLD_SIZE unset) must
    start N ranks itself -- never run one rank and report n_gpus 1
    (VERDICT r01 weak #6).  --launch-check brings up the gloo group only."""
    import json
    import subprocess
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root_dir, "bench.py"), "--gpus", str(n),
                        "--launch-check"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["process_group"]["world_size"] == n


def test_bench_rejects_mismatched_world():
    import subprocess
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root_dir, "bench.py"), "--gpus", "2",
                        "--launch-check"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0


def test_bench_cabi_mode_routing():
    """--api cabi is one process over N devices (mh_multi_*): it must refuse to
    run when fewer than N devices are visible -- before any clique is made --
    and under torch.distributed.run."""
    import subprocess
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bench = os.path.join(root_dir, "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, bench, "--api", "cabi", "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0
    assert "device(s) visible" in r.stderr, r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    env2 = dict(env, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, bench, "--api", "cabi", "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=240, env=env2)
    assert r.returncode != 0 and "one process" in r.stderr, r.stderr[-2000:]


def test_bench_cabi_txlog_routing():
    """--api cabi --config txlog (mh_multi_txlog_validate over N devices, VERDICT
    r04 next #4) refuses with fewer than N devices before touching any, and the
    torch.distributed mode refuses --config txlog."""
    import subprocess
    import sys
    root_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bench = os.path.join(root_dir, "bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, bench, "--api", "cabi", "--config", "txlog", "--gpus", "2",
                        "--steps", "1"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0 and "device(s) visible" in r.stderr, r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    r = subprocess.run([sys.executable, bench, "--config", "txlog", "--steps", "1"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0 and "--api cabi" in r.stderr, r.stderr[-2000:]
