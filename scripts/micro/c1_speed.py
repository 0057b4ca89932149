import sys, time, os
sys.path.insert(0, ".")
import torch
from drone_rl_amd.ppo import PPOConfig, PPOTrainer
for g in (False, True):
    tr = PPOTrainer(PPOConfig.sb3_defaults(seed=0))
    tr.rollout_graph = tr.train_graph = g
    tr.learn_step(); tr.learn_step(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        tr.learn_step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    t1 = time.perf_counter(); tr.collect_rollouts(); torch.cuda.synchronize(); tr_roll = time.perf_counter() - t1
    print(f"c1 graphs={g}: {dt*1e3:.1f} ms/update, {2048/dt:.0f} env-steps/s, rollout {tr_roll*1e3:.1f} ms", flush=True)
    tr.close()
