"""Data-parallel plumbing: one process per GPU, torch.distributed (backend "nccl" = RCCL on ROCm).

The env lanes shard with no data-path collective: rank r owns global lanes
[r*N, (r+1)*N) — the Philox counters are keyed by the global lane id, so a lane's trajectory does
not depend on the world size.  The only exchanges are
  * one all-reduce (sum) of the flat fp32 gradient per SGD step; every rank scales its loss by
    1 / (rows_per_rank * world), so the sum is the gradient of the global-minibatch mean.  With the
    split-fp16 step it is issued as two buckets (rlks_ppo_grad_step_part): W2 / b2 / W3 / b3 as soon
    as they are reduced, under the dH1 / dW1 kernel, then W1 / b1;
  * per iteration: the advantage moments [sum A, sum A^2, count], the SGD-step loss stats and the
    episode-return sums, so that standardisation, the KL-coefficient update and the reported
    episode_reward_mean equal the single-process values.
"""
from __future__ import annotations

import os


def group():
    """the initialised default process group's torch.distributed module, or None"""
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def forced():
    """RLKS_DDP_FORCE=1 with an initialised process group: a single rank still takes the multi-rank
    path (gradient -> all-reduce -> Adam, the overlapped two-bucket all-reduce, the per-iteration
    sums), with every collective really issued.  On one GPU this runs RCCL's all-reduce on hardware
    (a one-rank communicator) through the exact calls the 8-GPU run makes; the result equals the
    ordinary one-rank path bit for bit (tests/test_gpu_multirank.py)."""
    return os.environ.get("RLKS_DDP_FORCE") == "1" and group() is not None


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
    if d is not None and (d.get_world_size() > 1 or forced()):
        d.all_reduce(t)
    return t


def allreduce_sum_async(tensors):
    """start in-place sums over ranks of each tensor (contiguous views of one buffer are fine) and
    return their work handles; wait() on each orders the caller's stream after the collective
    (RCCL: the collective runs on its own stream, so it overlaps whatever the caller's stream does
    until then).  Single process: no-op, []."""
    d = group()
    if d is None or (d.get_world_size() == 1 and not forced()):
        return []
    return [d.all_reduce(t, async_op=True) for t in tensors]
