"""Trial sharding across GPUs (one process per GPU) and the histogram merge.

Trials are independent networks (launchNodes.ts:15-43 builds each network in
isolation), so the only multi-GPU data movement is one all-reduce (sum) of the
small uint64 outcome histogram over RCCL.  Philox counters are keyed by the
global trial id, so the merged histogram is bit-identical for any GPU count.
"""
from __future__ import annotations


def weak_range(step: int, rank: int, world: int, per_rank: int) -> tuple[int, int]:
    """Weak scaling: every rank runs `per_rank` trials per step; global ids
    [(step * world + rank) * per_rank, +per_rank)."""
    return (step * world + rank) * per_rank, per_rank


def strong_range(begin: int, total: int, rank: int, world: int) -> tuple[int, int]:
    """Strong scaling: split [begin, begin + total) into `world` contiguous,
    near-equal shards."""
    q, r = divmod(total, world)
    lo = begin + rank * q + min(rank, r)
    return lo, q + (1 if rank < r else 0)


def merge_histogram(hist, group=None):
    """Sum a histogram tensor over all ranks in place (RCCL on GPU, gloo on
    CPU).  int64 tensors; counts stay far below 2^63."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    return hist
