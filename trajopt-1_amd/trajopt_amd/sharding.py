"""Multi-GPU sharding of a batch of independent SQP problems.

Problems are independent: rank r of W solves the contiguous seed range
[r * B, (r + 1) * B) of its own GPU (weak scaling, B problems per GPU) and no
data crosses ranks.  The only collectives are the timing reductions of the
benchmark (max elapsed time, sum of SQP iterations), on a gloo group.
"""
from __future__ import annotations

from . import problems


def shard_first(rank: int, batch_per_rank: int) -> int:
    """First problem index (seed offset) of a rank's shard."""
    if rank < 0 or batch_per_rank <= 0:
        raise ValueError("rank must be >= 0 and batch_per_rank > 0")
    return rank * batch_per_rank


def rank_workload(config: str, batch_per_rank: int, rank: int, n_steps: int | None = None):
    """The synthetic workload a rank solves: problems shard_first(rank) + [0, B)."""
    return problems.make_workload(config, batch_per_rank, first_problem=shard_first(rank, batch_per_rank),
                                  n_steps=n_steps)


def reduce_step_stats(elapsed_s: float, sqp_iters: float, world: int):
    """(max elapsed over ranks, sum of SQP iterations over ranks).

    Uses the default torch.distributed process group when world > 1 (gloo in
    bench.py: two doubles per call, outside the timed region)."""
    if world <= 1:
        return float(elapsed_s), float(sqp_iters)
    import torch
    import torch.distributed as dist

    tmax = torch.tensor([float(elapsed_s)], dtype=torch.float64)
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tsum = torch.tensor([float(sqp_iters)], dtype=torch.float64)
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    return float(tmax[0]), float(tsum[0])
