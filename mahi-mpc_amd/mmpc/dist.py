"""Batch sharding across ranks (one process per GPU, torch.distributed).

The path partitions into independent instances: rank r solves the instances with global
indices [r*B, (r+1)*B) generated from (seed, global index), so results do not depend on the number of
ranks and no collective is on the data path.  Only the timing/reporting reductions below use the
process group (RCCL on GPUs, gloo in the CPU tests)."""
from __future__ import annotations


def shard(batch_per_rank: int, rank: int) -> tuple[int, int]:
    """(first global instance index, count) of this rank (weak scaling: fixed work per rank)."""
    if batch_per_rank < 0 or rank < 0:
        raise ValueError("negative batch or rank")
    return rank * batch_per_rank, batch_per_rank


def shard_strong(total: int, rank: int, world: int) -> tuple[int, int]:
    """contiguous split of a fixed total: rank r gets [floor(r T / W), floor((r+1) T / W))."""
    lo = (rank * total) // world
    hi = ((rank + 1) * total) // world
    return lo, hi - lo


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64 if isinstance(value, float) else torch.int64, device=device)
    dist.all_reduce(t)
    return t.item()
