"""Data-parallel plumbing (one process per GPU, torch.distributed).

The env batch shards with no exchange at all: rank r owns global env ids
[r*N, (r+1)*N) (its Philox streams are keyed by those ids).  PPO adds the
only collectives on the hot path:
  * one broadcast of the flat parameter buffer at start (rank 0 -> all),
  * one all-reduce (sum, then 1/world) of the flat fp32 gradient per
    optimizer step -- 141,065 floats = 564 KB for the 2x256 net, a single
    bucket: on xGMI this is latency-bound, so it is never split,
  * one all-reduce of 3 episode-statistics scalars per logged update.
Backend "nccl" is RCCL on ROCm; every function also runs under gloo (CPU
tests, tests/test_dist_cpu.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def env_shard(rank: int, envs_per_rank: int) -> tuple[int, int]:
    """Global env-id range [lo, hi) owned by `rank`."""
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


def broadcast_params_(flat: torch.Tensor, group=None, src: int = 0) -> torch.Tensor:
    dist.broadcast(flat, src=src, group=group)
    return flat


def allreduce_mean_(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """In-place mean over ranks (sum all-reduce, then scale)."""
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.mul_(1.0 / world)
    return t


def allreduce_sum_(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def allreduce_max_(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t
