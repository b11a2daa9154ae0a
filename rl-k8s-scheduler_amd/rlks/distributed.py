"""Data-parallel plumbing: one process per GPU, torch.distributed (backend "nccl" = RCCL on ROCm).

The env lanes shard with no data-path collective: rank r owns global lanes
[r*N, (r+1)*N) — the Philox counters are keyed by the global lane id, so a lane's trajectory does
not depend on the world size.  The only exchanges are
  * one all-reduce (sum) of the flat fp32 gradient per SGD step; every rank scales its loss by
    1 / (rows_per_rank * world), so the sum is the gradient of the global-minibatch mean;
  * per iteration: the advantage moments [sum A, sum A^2, count], the SGD-step loss stats and the
    episode-return sums, so that standardisation, the KL-coefficient update and the reported
    episode_reward_mean equal the single-process values.
"""
from __future__ import annotations


def group():
    """the initialised default process group's torch.distributed module, or None"""
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def rank_world():
    d = group()
    return (d.get_rank(), d.get_world_size()) if d else (0, 1)


def lane_range(lanes_per_rank: int, rank: int):
    """global lane ids owned by `rank` (env_offset = first)"""
    return rank * lanes_per_rank, (rank + 1) * lanes_per_rank


def loss_scale(rows_per_rank: int, world: int) -> float:
    """1 / global minibatch rows: per-rank gradients then sum to the global mean"""
    return 1.0 / (rows_per_rank * world)


def allreduce_sum_(t):
    """in-place sum over ranks (no-op for a single process)"""
    d = group()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t)
    return t
