"""Host-buffer (PCIe-inclusive) rates of the drop-in surfaces, next to the
device-resident path:
  * DroneGymEnv (1 env): numpy action in, (obs, reward, done, info) out --
    the reference's per-step call (drone.py:266-268);
  * BatchedDroneVecEnv (N envs, SB3 VecEnv): numpy actions in, numpy obs /
    rewards / dones + N info dicts out (SB3 DummyVecEnv + VecMonitor
    semantics);
  * DroneBatch.step on device tensors (the trainer's path), for reference.
Usage: python scripts/host_path.py [--n 65536] [--steps 200]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drone_rl_amd import DroneBatch, DroneGymEnv, random_actions  # noqa: E402
from drone_rl_amd.vec_env import BatchedDroneVecEnv  # noqa: E402


def timed(fn, steps, warm=20):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    out = {}
    rng = np.random.default_rng(0)

    env = DroneGymEnv(seed=1)
    env.reset()
    act1 = rng.uniform(0, 7.3575, 4).astype(np.float32)

    def one():
        _, _, done, _ = env.step(act1)
        if done:
            env.reset()
    s = timed(one, 2000)
    out["gym_env_1"] = {"us_per_step": round(s * 1e6, 2), "env_steps_per_s": round(1 / s, 1)}

    ve1 = BatchedDroneVecEnv(1, seed=1)
    ve1.reset()
    s = timed(lambda: ve1.step(act1[None]), 2000)
    out["vecenv_1_host"] = {"us_per_step": round(s * 1e6, 2), "env_steps_per_s": round(1 / s, 1)}
    s = timed(lambda: ve1.get_attr("pos"), 2000)
    out["vecenv_1_get_attr_pos"] = {"us_per_call": round(s * 1e6, 2)}
    ve1.close()

    ve = BatchedDroneVecEnv(a.n, seed=1)
    ve.reset()
    acts = rng.uniform(0, 7.3575, (a.n, 4)).astype(np.float32)
    s = timed(lambda: ve.step(acts), a.steps)
    out[f"vecenv_{a.n}_host"] = {"ms_per_step": round(s * 1e3, 3),
                                 "env_steps_per_s": round(a.n / s, 1)}
    ve.close()

    b = DroneBatch(a.n, "gym", seed=1, auto_reset=True)
    b.reset()
    ad = random_actions(a.n, seed=3, step=0)
    s = timed(lambda: b.step(ad), a.steps * 10)
    out[f"batch_{a.n}_device_eager"] = {"us_per_step": round(s * 1e6, 2),
                                        "env_steps_per_s": round(a.n / s, 1)}
    b.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
