"""bench.py's root check on the CPU: every multi-GPU bench
line rebuilds its tree with the oracle after the timed region and exits
non-zero on a mismatch.  Here the "device" results are the oracle's own
levels / roots held in CPU tensors, so the routing -- shard regeneration from
the splitmix64 stream at an entry offset, full vs sampled shard checks, the
128-byte per-rank records over gloo, the top levels over the shard roots and
the shared verdict -- runs on world-size-2 gloo without a GPU; a corrupted
shard must turn the verdict false on every rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _shard_levels(orc, bench, n, val, seed, key0, corrupt=False):
    keys, vals = bench.shard_block(orc, seed, key0, 0, n, val)
    if corrupt:
        vals = vals.copy()
        vals[0, 100 % val] ^= 1
    _, lv, root = orc.build_entries_fixed(1, keys, vals, nthreads=2)
    return torch.from_numpy(lv.reshape(-1).copy()), root


def test_shard_block_is_the_stream_at_an_offset(orc):
    b = _bench()
    n, val = 300, 64
    keys, vals = b.shard_block(orc, 9, 1000, 0, n, val)
    k2, v2 = b.shard_block(orc, 9, 1000, 137, 50, val)
    assert np.array_equal(v2, vals[137:187]) and np.array_equal(k2, keys[137:187])
    assert keys[5].tobytes() == (1005).to_bytes(8, "big")


def test_full_and_sampled_shard_roots_agree(orc, monkeypatch):
    b = _bench()
    n, val = 1 << 8, 64
    lv, root = _shard_levels(orc, b, n, val, 4, 256)
    r_full, ok, mode = b.oracle_shard_root(orc, n, val, 4, 256, lv, 2)
    assert ok and mode == "full" and r_full == root
    monkeypatch.setattr(b, "FULL_CHECK_BYTES", 0)
    monkeypatch.setattr(b, "CHECK_BLOCK_BITS", 4)
    r_s, ok, mode = b.oracle_shard_root(orc, n, val, 4, 256, lv, 2)
    assert ok and mode.startswith("sampled") and r_s == root
    # a wrong value byte in block 0 (always sampled) fails the block check
    bad, _ = _shard_levels(orc, b, n, val, 4, 256, corrupt=True)
    _, ok, _ = b.oracle_shard_root(orc, n, val, 4, 256, bad, 2)
    assert not ok


def test_global_expected_is_the_whole_tree(orc):
    b = _bench()
    n, val, G = 64, 32, 4
    parts = [b.shard_block(orc, 2 + r, r * n, 0, n, val) for r in range(G)]
    roots = [orc.build_entries_fixed(1, k, v)[2] for k, v in parts]
    keys = np.concatenate([k for k, _ in parts])
    vals = np.concatenate([v for _, v in parts])
    assert b.global_expected(orc, roots) == orc.build_entries_fixed(1, keys, vals)[2]
    assert b.global_expected(orc, roots[:1]) == roots[0]


def test_corrupt_hook_routing(monkeypatch):
    b = _bench()
    t = torch.zeros(256, dtype=torch.uint8)
    monkeypatch.delenv("MH_BENCH_CORRUPT", raising=False)
    assert not b.corrupt_hook(t, 0) and int(t.sum()) == 0
    monkeypatch.setenv("MH_BENCH_CORRUPT", "1")
    assert not b.corrupt_hook(t, 0) and int(t.sum()) == 0
    assert b.corrupt_hook(t, 1) and int(t[100]) == 1 and int(t.sum()) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, n, val, bad_rank, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import bench
    import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the "device" side: this shard's levels / subtree root, the global
        # root from the all-gathered subtree roots (as bench.py's step does)
        lv, sub = _shard_levels(orc, bench, n, val, 2 + rank, rank * n, corrupt=rank == bad_rank)
        g = torch.empty(world * 32, dtype=torch.uint8)
        dist.all_gather_into_tensor(g, torch.from_numpy(np.frombuffer(sub, np.uint8).copy()))
        glob = bench.reduce_nodes(orc, [bytes(x) for x in g.numpy().reshape(-1, 32)])
        t = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy())  # noqa: E731
        rc = bench.root_check_ranks(None, n, val, rank, world, dist, "gloo", torch.device("cpu"),
                                    lv, t(sub), t(glob), rank == bad_rank)
        q.put((rank, rc["ok"], rc["root"], rc["corrupted_shards"], rc["n"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad_rank", [(2, -1), (2, 1), (8, -1), (8, 5)])
def test_root_check_ranks_gloo(orc, world, bad_rank):
    """bench.py's post-timing root check over `world` gloo ranks -- 8 is the
    driver's largest --gpus: the same all-gather of 128-byte records, verdict
    and all-reduce it runs over RCCL on an 8-GPU node."""
    n, val = 1 << 9, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, n, val, bad_rank, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    b = _bench()
    parts = [b.shard_block(orc, 2 + r, r * n, 0, n, val) for r in range(world)]
    whole = orc.build_entries_fixed(1, np.concatenate([k for k, _ in parts]),
                                    np.concatenate([v for _, v in parts]))[2]
    for rank, ok, root, bad, ntot in res:
        assert ok == (bad_rank < 0), (rank, ok)   # every rank shares the verdict
        assert root == whole.hex() and ntot == world * n
        assert bad == ([] if bad_rank < 0 else [bad_rank])


def _rank_strong(rank, world, port, total, val, bad_rank, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import bench
    import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = total // world
        seed = bench.shard_seed(rank, n, val, True)
        lv, sub = _shard_levels(orc, bench, n, val, seed, rank * n, corrupt=rank == bad_rank)
        g = torch.empty(world * 32, dtype=torch.uint8)
        dist.all_gather_into_tensor(g, torch.from_numpy(np.frombuffer(sub, np.uint8).copy()))
        glob = bench.reduce_nodes(orc, [bytes(x) for x in g.numpy().reshape(-1, 32)])
        t = lambda b: torch.from_numpy(np.frombuffer(b, np.uint8).copy())  # noqa: E731
        rc = bench.root_check_ranks(None, n, val, rank, world, dist, "gloo", torch.device("cpu"),
                                    lv, t(sub), t(glob), rank == bad_rank, seed)
        q.put((rank, rc["ok"], rc["root"], glob.hex(), rc["n"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad_rank", [(2, -1), (8, -1), (8, 3)])
def test_strong_scaling_root_check_gloo(orc, world, bad_rank):
    """bench.py --scaling strong: ONE tree of `total` entries split over the
    ranks (each rank's values the N = 1 tree's stream at its entry offset,
    bench.shard_seed): the global root every rank assembles, and the root
    check's, equal the oracle's rebuild of the whole tree -- the same root at
    every world size; a corrupted rank fails the check on every rank."""
    total, val = 1 << 10, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_strong, args=(r, world, port, total, val, bad_rank, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    b = _bench()
    keys, vals = b.shard_block(orc, 2, 0, 0, total, val)  # the N = 1 tree
    whole = orc.build_entries_fixed(1, keys, vals)[2].hex()
    assert b.shard_seed(0, total, val, True) == 2
    for rank, ok, root, glob, ntot in res:
        assert ok == (bad_rank < 0), (rank, ok)
        assert root == whole and ntot == total
        assert (glob == whole) == (bad_rank < 0)
