"""Read-chunk sharding across GPUs.

Every rank holds a full replica of the index and maps its own pairs, so the
data path has no collective.  The only exchanges are the end-of-run reductions
below -- the analogue of the reference summing its per-thread
AlignmentStatistics (src/main.cpp:597-600) -- over torch.distributed (RCCL on
GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

STAT_FIELDS = ("n_reads", "sam_bytes", "sw_calls", "tried", "nam_rescue", "mate_rescue", "inconsistent")


def first_pair(rank: int, step: int, total_steps: int, pairs_per_step: int) -> int:
    """Index of the first synthetic pair rank `rank` maps in step `step`.
    Ranges of different (rank, step) never overlap."""
    return (rank * total_steps + step) * pairs_per_step


def _reduce(values, op, device):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op)
    return [float(x) for x in t.tolist()]


def reduce_run(elapsed_s: float, stats: dict, device="cpu") -> tuple[float, dict]:
    """Max wall time over ranks and the sum of every counter in `stats`."""
    import torch.distributed as dist
    (wall,) = _reduce([elapsed_s], dist.ReduceOp.MAX, device)
    keys = sorted(stats)
    summed = _reduce([float(stats[k]) for k in keys], dist.ReduceOp.SUM, device)
    return wall, {k: int(round(v)) for k, v in zip(keys, summed)}
