"""Multi-GPU htree build: power-of-two leaf shards + one all-gather of roots.

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
