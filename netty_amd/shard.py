"""Multi-GPU sharding of a chunk batch.

Every Snappy/FastLZ/LZF chunk is self-contained (a copy offset never reaches outside its own
chunk: Snappy.java:647-649 bounds it by the bytes written in *this* chunk; FastLZ/LZF blocks are
independent), so a batch shards by contiguous chunk-index ranges with no data-path collective.
The only exchange is one all-gather of each rank's output byte count, from which every rank
learns where its compressed shard starts in the single logical output stream.  The timing
barrier and the max-over-ranks reduction ride on the same process group.

One process per GPU (torchrun); ``nccl`` is RCCL over xGMI on the GPU box, ``gloo`` on CPU tests.
"""
from __future__ import annotations

from typing import List, Tuple


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous chunk range [lo, hi) owned by `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return n_total * rank // world, n_total * (rank + 1) // world


def exchange_offsets(local_bytes: int, device=None, group=None) -> Tuple[int, int, List[int]]:
    """All-gather per-rank output sizes; returns (this rank's byte offset in the global stream,
    global total, per-rank sizes).  Single-process (no initialised group): (0, local, [local])."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return 0, int(local_bytes), [int(local_bytes)]
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    t = torch.tensor([int(local_bytes)], dtype=torch.int64, device=device)
    got = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(got, t, group=group)
    sizes = [int(x.item()) for x in got]
    return sum(sizes[:rank]), sum(sizes), sizes


def max_over_ranks(value: float, device=None, group=None) -> float:
    """The job's wall time is the slowest rank's (bench.py contract)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def all_true(flag: bool, device=None, group=None) -> bool:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())
