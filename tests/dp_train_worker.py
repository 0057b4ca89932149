"""One rank of the configs[3] data-parallel check at its PER-RANK size
(launched by tests/test_dp_train_gpu.py; BASELINE.json configs[3]: 8 x 65,536
envs, PPO with one gradient all-reduce per optimizer step; reference learn
loop /root/reference/train.py:63-68).

Both ranks share the test box's one GPU, so the group is gloo (RCCL refuses
two ranks per device); the call sites are the ones RCCL runs on a multi-GPU
node.  Everything goes through PPOTrainer.train(), i.e. the data-parallel
optimizer step the trainer uses at world > 1 (deferred finish -> one sum
all-reduce of the flat gradient -> clip+Adam on its mean).

Phase A (configs[3] per rank: 65,536 envs, T = 32, 2x256, 65,536-row
minibatches, n_epochs 2 -> 64 optimizer steps and 64 all-reduces per
update): two learn_step()s; after each, the flat parameters and both Adam
moments must be BITWISE equal on the two ranks.

Phase B (the union-minibatch gradient): one rollout of T = 1 per rank, one
65,536-row minibatch per rank, one epoch, advantage normalisation off (SB3
normalises per minibatch, so with it on the DP gradient is by design the mean
of per-rank-normalised gradients).  After train() the flat gradient buffer
holds c * mean_r g_r (clip_grad_norm_ leaves the clipped gradient, as torch
does).  Rank 0 gathers both ranks' rows and checks every entry against the
f64 gradient of the UNION minibatch (131,072 rows, tests/ppo_f64.py) within
the per-entry fp32 reduction bound of tests/test_ppo_flagship_parity_gpu.py,
with one more rounding in the chain (the cross-rank add)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ppo_f64 import U, f64_reference, gamma  # noqa: E402

from drone_rl_amd.policy import _sb3_name  # noqa: E402
from drone_rl_amd.ppo import PPOConfig, PPOTrainer  # noqa: E402


def _equal_on_all_ranks(t: torch.Tensor) -> bool:
    mx, mn = t.clone(), t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    # MAX == MIN entrywise <=> every rank holds the same value (no NaN here)
    return bool(torch.equal(mx, mn))


def phase_a(rank, world, dev):
    cfg = PPOConfig(num_envs=65536, n_steps=32, batch_size=65536, n_epochs=2,
                    seed=3 + 11 * rank)          # different seeds: the broadcast equalises
    tr = PPOTrainer(cfg, device=dev, rank=rank, world_size=world)
    assert tr.dp_step and tr.dp_collective, "the DP optimizer step is not in use"
    assert not tr._train_graphable(), "gloo collectives cannot be graph-captured"
    for it in range(2):
        st = tr.learn_step()
        assert torch.isfinite(st).all(), st
        for name, t in (("params", tr.policy.flat.detach()), ("exp_avg", tr.opt.m),
                        ("exp_avg_sq", tr.opt.v)):
            assert _equal_on_all_ranks(t), f"iteration {it}: ranks' {name} differ"
        assert tr.opt.t == (it + 1) * 64
    es = tr.episode_stats()
    assert es["episodes"] > 0
    # the shards are disjoint envs: their states differ
    p = tr.env.get("pos")[:8].cpu()
    other = [torch.zeros_like(p) for _ in range(world)]
    dist.all_gather(other, p)
    assert not torch.equal(other[0], other[1])
    tr.close()
    if rank == 0:
        print("phase A ok: params and Adam moments bitwise equal after 2 updates "
              "(2 x 64 all-reduces)", flush=True)


def phase_b(rank, world, dev):
    M = 65536
    cfg = PPOConfig(num_envs=M, n_steps=1, batch_size=M, n_epochs=1, seed=21,
                    normalize_advantage=False)
    tr = PPOTrainer(cfg, device=dev, rank=rank, world_size=world)
    tr.collect_rollouts()
    sd0 = tr.policy.state_dict()
    rows = torch.cat([tr.obs[0].reshape(M, -1), tr.actions[0].reshape(M, 4), tr.aux], 1)
    allr = [torch.zeros_like(rows) for _ in range(world)]
    dist.all_gather(allr, rows.contiguous())
    tr.train()
    norm = tr.opt.grad_norm.item()
    c = min(1.0, cfg.max_grad_norm / (norm + 1e-6))
    g_dp = {_sb3_name(n, 2): tr.fused.gview(n).detach().double().cpu() / c
            for n, _, _ in tr.policy.layout}
    if rank == 0:
        u = torch.cat(allr, 0).to(dev)
        od = tr.obs.shape[2]
        g_ref, env = f64_reference(sd0, cfg.net_arch, u[:, :od], u[:, od:od + 4],
                                   u[:, od + 4], u[:, od + 5], u[:, od + 6], cfg.clip_range,
                                   cfg.vf_coef, False, device=dev)
        # the flagship test's chain (n = 2,048) + the cross-rank add + the
        # 1 / world scale (exact for world 2)
        G = gamma(2049)
        worst = 0.0
        for k in g_ref:
            ref = g_ref[k].cpu()
            tol = G * env[k].cpu() + 4 * U * ref.abs() + 1e-30
            r = ((g_dp[k].reshape(ref.shape) - ref).abs() / tol).max().item()
            worst = max(worst, r)
            assert r <= 1.0, f"{k}: DP gradient error {r:.3f} x its fp32 bound"
        print(f"phase B ok: all-reduced gradient vs the union f64 gradient, "
              f"worst {worst:.4f} of the per-entry bound", flush=True)
    tr.close()


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    phase_a(rank, world, dev)
    dist.barrier()
    phase_b(rank, world, dev)
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    main()
