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


@pytest.mark.parametrize("world,n", [(2, 1 << 12), (2, 1000), (3, 1025), (4, 4097), (2, 1)])
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
