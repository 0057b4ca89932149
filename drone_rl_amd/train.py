"""Drop-in for the reference's train.py (/root/reference/train.py:1-70):
PPO on the quadrotor env, here GPU-resident over N batched envs.

  python -m drone_rl_amd.train                        # 65,536 envs, 2x256 MLP
  python -m drone_rl_amd.train --sb3-defaults --envs 1 # the reference's config
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m drone_rl_amd.train
  python -m drone_rl_amd.train --checkpoint dd.zip     # SB3 .zip in and out

Like the reference it resumes from a checkpoint when one exists
(train.py:10-31; ours also restores the env curriculum), trains for
--total-steps (train.py:11,63-68) and saves at the end (train.py:70).
Logs are JSON lines on stdout (SB3's logger keys: ep_rew_mean, ep_len_mean,
fps, loss terms) instead of TensorBoard.
"""
import argparse
import json
import os

import torch
import torch.distributed as dist

from .ppo import PPOConfig, PPOTrainer


def checkpoint_path(path: str, rank: int, world: int) -> str:
    """Per-rank checkpoint name that keeps the extension (dd.zip ->
    dd.rank0.zip), so the SB3 / torch format choice survives the suffix."""
    if world == 1:
        return path
    root, ext = os.path.splitext(path)
    return f"{root}.rank{rank}{ext}"


def resume_path(path: str, rank: int, world: int) -> str | None:
    """The per-rank file to resume from: checkpoint_path(), or a file under
    the name earlier versions wrote ('<checkpoint>.rank<r>', the extension
    before the suffix), which is then used with a warning; None if neither
    exists."""
    ck = checkpoint_path(path, rank, world)
    if os.path.exists(ck):
        return ck
    legacy = f"{path}.rank{rank}" if world > 1 else None
    if legacy and os.path.exists(legacy):
        import warnings
        warnings.warn(f"resuming from the legacy per-rank checkpoint name {legacy!r}; "
                      f"new checkpoints are written to {ck!r}")
        return legacy
    return None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--total-steps", type=float, default=2e6 * 64)
    ap.add_argument("--n-steps", type=int, default=32)
    ap.add_argument("--batch-size", type=int, default=65536)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--ent-coef", type=float, default=0.0,
                    help="entropy coefficient (SB3 default 0.0)")
    ap.add_argument("--net", type=int, nargs="+", default=[256, 256])
    ap.add_argument("--state-dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--variant", choices=["gym", "moving"], default="gym",
                    help="gym = DroneGymEnv; moving = the moving-target curriculum")
    ap.add_argument("--sb3-defaults", action="store_true",
                    help="SB3 PPO defaults of the reference (n_steps 2048, batch 64, 64x64)")
    ap.add_argument("--checkpoint", default="./dd_gpu.pt")
    ap.add_argument("--log-every", type=int, default=1)
    ap.add_argument("--initial-eps", type=float, default=0.0,
                    help="curriculum level every env starts at (reference: 0.0)")
    ap.add_argument("--eps-schedule", default="",
                    help="staged curriculum 'update:eps,update:eps,...' (all envs)")
    ap.add_argument("--traj-dir", default=None,
                    help="record env 0's trajectories like traj_tb.py (every 25th episode, "
                         "blocks of 500) into this directory (npz, PNG if matplotlib)")
    ap.add_argument("--grad-buckets", type=int, choices=[1, 2], default=1,
                    help="data parallel: 1 = one gradient all-reduce per optimizer step; "
                         "2 = an early bucket overlapped with the first-layer backward")
    ap.add_argument("--bootstrap-timeouts", action="store_true",
                    help="SB3 TimeLimit handling: bootstrap V(terminal obs) into the reward "
                         "of steps that end an episode at the 200-step limit without a "
                         "crash (off = the reference's semantics)")
    ap.add_argument("--reset-num-timesteps", action=argparse.BooleanOptionalAction,
                    default=True,
                    help="after a resume, train --total-steps more (SB3's default, the "
                         "reference's behaviour); --no-reset-num-timesteps trains up to "
                         "--total-steps in all")
    a = ap.parse_args(argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    common = dict(num_envs=a.envs, learning_rate=a.lr, ent_coef=a.ent_coef, seed=a.seed,
                  grad_buckets=a.grad_buckets,
                  state_dtype=a.state_dtype, variant=a.variant, initial_eps=a.initial_eps,
                  bootstrap_timeouts=a.bootstrap_timeouts,
                  eps_schedule=tuple((int(u), float(e)) for u, e in
                                     (kv.split(":") for kv in a.eps_schedule.split(",") if kv)))
    if a.sb3_defaults:
        cfg = PPOConfig.sb3_defaults(**common)
    else:
        cfg = PPOConfig(n_steps=a.n_steps, batch_size=a.batch_size, n_epochs=a.epochs,
                        net_arch=tuple(a.net), **common)
    tr = PPOTrainer(cfg, rank=rank, world_size=world)
    if a.traj_dir and rank == 0:
        from .trajectory import TrajectoryRecorder
        tr.trajectory = TrajectoryRecorder(tr.env, out_dir=a.traj_dir)
    ck = checkpoint_path(a.checkpoint, rank, world)
    src = resume_path(a.checkpoint, rank, world)
    # *.zip = stable-baselines3 PPO checkpoint (the reference's dd.zip,
    # train.py:10-31 / 70); anything else = this trainer's bit-exact resume file
    sb3 = a.checkpoint.endswith(".zip")
    total = int(a.total_steps)
    if src is not None:
        tr.load_sb3(src) if sb3 else tr.load(src)
        if rank == 0:
            print(json.dumps({"resumed": src, "num_timesteps": tr.num_timesteps}), flush=True)
        if a.reset_num_timesteps:
            # SB3 learn(reset_num_timesteps=True), the reference's call
            # (train.py:63-68): every run trains --total-steps more steps and
            # counts from 0 (the update counter, which keys the random
            # streams, keeps running)
            tr.num_timesteps = 0
    tr.learn(total, log_every=a.log_every, logger=lambda d: print(json.dumps(d), flush=True))
    tr.save_sb3(ck) if sb3 else tr.save(ck)
    tr.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
