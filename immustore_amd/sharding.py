"""Multi-GPU builds: power-of-two shards + one all-gather of 32-byte roots.

htree (C2/C4):

SURVEY.md 8(e) / finding 3: if the leaves are cut into contiguous chunks of
S = 2^k, reducing every chunk with htree's pairing rule and then reducing the
chunk roots with the same rule gives exactly htree.BuildWith's root
(embedded/htree/htree.go:85-110).  So every rank builds the subtree of its own
chunk (all its levels stay local and are per-level contiguous slices of the
global levels), the G x 32-byte chunk roots are all-gathered once over RCCL
(xGMI), and the top ceil(log2 G) levels are reduced on every rank
(replicated; identical inputs give identical roots).

The payload is 32 B per rank, so the exchange is latency bound (tens of us);
there is no other data-path collective.

ahtree batch append (C3 at scale): rank r appends
(r*S, (r+1)*S], S = 2^k.  Its leaves, the perfect nodes of levels <= k and
every spine node of level < k lie inside its own range; the nodes above level
k are built from the G shard roots (node((r+1)*S, k)), all-gathered once.
Each rank keeps a globally indexed dLog and ends with its own range
byte-identical to a single-device append (ahtree_sharded_append).

Proof verification (C5): proofs are independent -- split by index, no
collective besides gathering counts / bitmaps.
"""
from typing import Tuple


def shard_range(rank: int, world: int, n: int) -> Tuple[int, int]:
    """[lo, hi) of the leaves owned by `rank`: chunks of S = 2^k leaves, with
    S the smallest power of two such that world * S >= n; the last ranks may
    get a short or empty chunk (still exact by finding 3)."""
    if world < 1 or rank < 0 or rank >= world:
        raise ValueError("bad rank/world")
    s = 1
    while s * world < n:
        s <<= 1
    lo = min(rank * s, n)
    return lo, min(lo + s, n)


def allgather_roots(root, world: int):
    """All-gather one 32-byte root per rank (torch uint8 tensor of 32 on the
    rank's device: RCCL for cuda tensors, gloo for cpu tensors)."""
    import torch
    import torch.distributed as dist
    if root.is_cuda and dist.get_backend() == "gloo":
        # rehearsal of the multi-rank path with gloo (several ranks sharing
        # one GPU): stage the 32 bytes through the host
        out = torch.empty(world * 32, dtype=torch.uint8)
        dist.all_gather_into_tensor(out, root.contiguous().view(32).cpu())
        return out.to(root.device)
    out = torch.empty(world * 32, dtype=torch.uint8, device=root.device)
    dist.all_gather_into_tensor(out, root.contiguous().view(32))
    return out


def nonempty_roots(gathered, world: int, n: int):
    """Drop the roots of empty shards (ranks past the end of the leaves)."""
    used = sum(1 for r in range(world) if shard_range(r, world, n)[1] > shard_range(r, world, n)[0])
    return gathered[: used * 32]


def ahtree_shard_bits(world: int, m: int) -> int:
    """k such that S = 2^k appends per rank cover m appends (weak scaling passes
    m = world * S exactly)."""
    k = 0
    while (1 << k) * world < m:
        k += 1
    return k


def ahtree_sharded_append(ctx, dlog_ptr: int, payloads_ptr: int, rank: int, world: int,
                          shard_bits: int, m_total: int, allgather, plen: int = 32,
                          roots_out_ptr=None):
    """This rank's part of appending m_total payloads (global n0 = 0) to an
    empty tree; payloads_ptr holds only this rank's payloads.  `allgather(ptr)`
    must all-gather 32 bytes (device pointer) across ranks and return a device
    pointer to world*32 bytes in rank order.  Returns (n0, m) of this rank."""
    from . import _native as N
    L = N.load()
    S = 1 << shard_bits
    n0 = min(rank * S, m_total)
    m = min(S, m_total - n0)
    N.check(L.mh_dev_ahtree_append_local(ctx.handle, dlog_ptr, n0, payloads_ptr, m, plen,
                                         shard_bits))
    # shard root of this rank (any 32 B for a short / empty last shard: unused)
    idx = L.mh_ahtree_node_index(n0 + S, shard_bits) if m == S else 0
    gathered = allgather(dlog_ptr + idx * 32)
    complete = m_total // S
    N.check(L.mh_dev_ahtree_put_shard_roots(ctx.handle, dlog_ptr, shard_bits,
                                            min(complete, world), gathered))
    N.check(L.mh_dev_ahtree_append_spine(ctx.handle, dlog_ptr, n0, m, roots_out_ptr))
    return n0, m


def ahtree_range_sizes(n0: int, total: int, world: int) -> Tuple[int, int]:
    """(send_bytes, work_bytes) of one rank's ranged append (mh_ahtree_range_sizes)."""
    import ctypes as C
    from . import _native as N
    s, w = C.c_uint64(), C.c_uint64()
    N.check(N.load().mh_ahtree_range_sizes(n0, total, world, C.byref(s), C.byref(w)))
    return s.value, w.value


def ahtree_range_append(ctx, n0: int, peaks, total: int, world: int, rank: int, payloads_ptr: int,
                        plen: int, dlog_ptr: int, work_ptr: int, send_ptr: int, recv_ptr: int,
                        exchange, roots_out_ptr=None):
    """This rank's range of appending `total` payloads onto a tree of n0
    (peaks: host bytes of the old tree's popcount(n0) peaks, None for n0 = 0),
    keeping only its own dLog range (range `rank` of mh_ahtree_range_plan):
    local phase -> exchange() (the caller's all-gather of send_bytes per rank
    from send into recv, rank order; None when the plan has one range) ->
    piece tree + spines.  Every pointer is a device address on ctx's device;
    asynchronous on ctx's stream, the exchange ordered after the local phase
    by the caller (torch's collectives wait on the current stream)."""
    import numpy as np
    from . import _native as N
    from .merkle import _addr
    L = N.load()
    pk = np.frombuffer(peaks, np.uint8) if peaks else None
    N.check(L.mh_dev_ahtree_range_local(ctx.handle, n0, _addr(pk), total, world, rank,
                                        payloads_ptr, plen, dlog_ptr, work_ptr, send_ptr))
    if exchange is not None:
        exchange()
    N.check(L.mh_dev_ahtree_range_finish(ctx.handle, n0, _addr(pk), total, world, rank, recv_ptr,
                                         dlog_ptr, work_ptr, roots_out_ptr))
