"""In-process A/B of PPO trainer variants (box clocks drift by more than the
effects measured): two PPOTrainers with the same config, updates timed
alternately, medians reported.  Variants are set by an attribute override:
  python scripts/micro/ppo_ab_inproc.py defer_finish=False defer_finish=True"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd.ppo import PPOConfig, PPOTrainer  # noqa: E402

specs = sys.argv[1:] or ["defer_finish=False", "defer_finish=True"]
trs = []
for sp in specs:
    tr = PPOTrainer(PPOConfig(seed=0))
    k, _, v = sp.partition("=")
    obj = tr
    *path, k = k.split(".")          # e.g. fused.overlap_wgrad=True
    for a in path:
        obj = getattr(obj, a)
    setattr(obj, k, eval(v))
    tr.learn_step()
    trs.append((sp, tr))
torch.cuda.synchronize()
times = {sp: [] for sp in specs}
for _ in range(5):
    for sp, tr in trs:
        t0 = time.perf_counter()
        tr.learn_step()
        torch.cuda.synchronize()
        times[sp].append(time.perf_counter() - t0)
for sp in specs:
    t = np.median(times[sp])
    print(f"{sp}: {1 / t:.4f} updates/s (median of {len(times[sp])}; {t * 1e3:.1f} ms)", flush=True)
