"""Data-parallel plumbing (one process per GPU, torch.distributed).

The env batch shards with no exchange at all: rank r owns global env ids
[r*N, (r+1)*N) (its Philox streams are keyed by those ids).  PPO adds the
only collectives on the hot path:
  * one broadcast of the flat parameter buffer at start (rank 0 -> all),
  * ONE sum all-reduce of the flat fp32 gradient per optimizer step --
    141,065 floats = 564 KB for the 2x256 net -- between the launch that
    finishes the deferred gradient reductions and clip+Adam, which takes
    the 1/world mean inside its norm and update (PPOTrainer._train_body,
    grad_buckets=1, the default).  At this size an xGMI ring is latency-
    bound, so the buffer is not split.  grad_buckets=2 keeps an older step
    whose per-kernel finishes let everything but the first layer start as
    an async bucket while the first-layer backward runs
    (BucketedAllReduce),
  * one all-reduce of 3 episode-statistics scalars per logged update.
Backend "nccl" is RCCL on ROCm; every function also runs under gloo (CPU
tests, tests/test_dist_cpu.py; two ranks sharing one GPU in the -m gpu
tests, where RCCL refuses two ranks per device).
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


def allreduce_flat_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """The per-optimizer-step gradient all-reduce: in-place sum over the
    group's ranks, enqueued on the current stream (RCCL: the stream waits
    for it, the host does not; capturable into a hipGraph).  Called even on
    a one-rank group (PPOConfig.force_dp_path) so the collective path runs."""
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def allreduce_max_(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


class BucketedAllReduce:
    """Mean all-reduce of one flat buffer in buckets started as they become
    ready (async collectives on the backend's stream; each waits for the
    work already queued on the current stream), then finished together."""

    def __init__(self, flat: torch.Tensor, world: int, group=None):
        self.flat, self.world, self.group = flat, world, group
        self.works = []
        self.done_ranges = []

    def start(self, lo: int, hi: int):
        if self.world > 1 and hi > lo:
            self.works.append(dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM,
                                              group=self.group, async_op=True))
            self.done_ranges.append((lo, hi))

    def finish(self):
        """Start whatever was not covered, wait for all, scale by 1/world."""
        if self.world <= 1:
            return self.flat
        gaps, pos = [], 0
        for lo, hi in sorted(self.done_ranges):
            if lo > pos:
                gaps.append((pos, lo))
            pos = max(pos, hi)
        if pos < self.flat.numel():
            gaps.append((pos, self.flat.numel()))
        for lo, hi in gaps:
            self.start(lo, hi)
        for w in self.works:
            w.wait()
        self.works.clear()
        self.done_ranges.clear()
        self.flat.mul_(1.0 / self.world)
        return self.flat
