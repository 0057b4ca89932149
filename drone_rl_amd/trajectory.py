"""Trajectory logging for GPU training: the data path of the reference's
TrajectoryTensorboardCallback (/root/reference/traj_tb.py:6-69).

The reference records env 0's position after every step
(``get_attr('pos')``, traj_tb.py:34), splits episodes at ``dones``
(traj_tb.py:38-44; the position appended on the done step is the auto-reset
start of the next episode and is dropped), keeps every
``record_interval``-th finished episode (traj_tb.py:47-48) and every
``block_size`` episodes emits the buffered trajectories as XY/XZ/YZ overlay
figures (traj_tb.py:51-69).

Here the per-step recording stays on the device: each step gathers the
positions of the tracked envs (``dr_gather_state``, k rows, no full-batch
copy) and their done flags into a preallocated buffer; ``flush()`` (once per
rollout, where the trainer synchronises anyway) moves them to the host and
does the episode bookkeeping.  ``on_block`` receives
``(block_index, start_episode, end_episode, [trajectories])``; the default
writes an ``.npz`` (and PNG overlays when matplotlib is importable; figure
rendering is otherwise out of scope).
"""
from __future__ import annotations

import os

import numpy as np
import torch


class TrajectoryRecorder:
    def __init__(self, batch, env_ids=(0,), record_interval: int = 25, block_size: int = 500,
                 capacity: int = 4096, out_dir: str | None = None, on_block=None):
        self.batch = batch
        dev = batch.device
        self.ids = torch.as_tensor(list(env_ids), dtype=torch.int32, device=dev)
        k = self.ids.numel()
        self.k = k
        self.record_interval, self.block_size = record_interval, block_size
        self.capacity = capacity
        self.pos = torch.empty(capacity, k, 3, dtype=torch.float64, device=dev)
        self.done = torch.empty(capacity, k, dtype=torch.uint8, device=dev)
        self.n = 0
        self.out_dir = out_dir
        self.on_block = on_block if on_block is not None else self._save_block
        self.current = [[] for _ in range(k)]      # open episode per tracked env
        self.episode_count = 0                      # finished episodes of env_ids[0]
        self.buffered = []
        self.blocks_emitted = 0

    def on_step(self, dones: torch.Tensor):
        """Call after each env step with that step's (N,) done flags."""
        if self.n == self.capacity:
            self.flush()
        self.batch.gather("pos", self.ids, out=self.pos[self.n])
        torch.index_select(dones, 0, self.ids.long(), out=self.done[self.n])
        self.n += 1

    def flush(self):
        """Move the recorded steps to the host and split them into episodes
        exactly as traj_tb.py does for env 0 (other tracked envs are split
        too; only env_ids[0] drives the interval / block counters)."""
        if self.n == 0:
            return
        pos = self.pos[:self.n].cpu().numpy()
        done = self.done[:self.n].cpu().numpy().astype(bool)
        self.n = 0
        for t in range(pos.shape[0]):
            for j in range(self.k):
                self.current[j].append(pos[t, j])
                if not done[t, j]:
                    continue
                traj = np.array(self.current[j][:-1])   # drop the reset position
                self.current[j] = []
                if j != 0:
                    continue
                self.episode_count += 1
                if self.episode_count % self.record_interval == 0:
                    self.buffered.append(traj)
                if self.episode_count % self.block_size == 0 and self.buffered:
                    blk = self.episode_count // self.block_size
                    self.on_block(blk, (blk - 1) * self.block_size + 1,
                                  blk * self.block_size, list(self.buffered))
                    self.blocks_emitted += 1
                    self.buffered.clear()

    def _save_block(self, blk, start_ep, end_ep, trajs):
        if self.out_dir is None:
            return
        os.makedirs(self.out_dir, exist_ok=True)
        base = os.path.join(self.out_dir, f"trajectories_block{blk}")
        np.savez(base + ".npz", *trajs, start_ep=start_ep, end_ep=end_ep,
                 record_interval=self.record_interval)
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except Exception:
            return
        for i, j, tag in ((0, 1, "Overlay_XY"), (0, 2, "Overlay_XZ"), (1, 2, "Overlay_YZ")):
            fig, ax = plt.subplots(figsize=(6, 6))
            for run_i, t in enumerate(trajs):
                if len(t):
                    ax.plot(t[:, i], t[:, j], label=f"ep {(run_i + 1) * self.record_interval}")
            ax.set_xlabel("XYZ"[i])
            ax.set_ylabel("XYZ"[j])
            ax.set_title(f"Trajectories {tag} (eps {start_ep}-{end_ep})")
            fig.savefig(f"{base}_{tag}.png")
            plt.close(fig)
