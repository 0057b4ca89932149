"""K-step rollout kernel (dr_rollout / dr_rollout_random) against K graph-
replayed dr_step launches: env-steps/s and algorithmic GB/s per launch.

  python scripts/micro/rollout_bench.py [--envs 65536] [--reps 20]
The kernel form follows dr_rollout's launch rule (DRONERL_ROLLOUT_WS=0/1 forces it)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import DroneBatch, random_actions  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, nargs="+", default=[65536, 1 << 22])
ap.add_argument("--ks", type=int, nargs="+", default=[8, 32, 128])
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--dtype", default="f64")
ap.add_argument("--act-sets", type=int, default=1,
                help="distinct (k,N,4) action buffers cycled over the launches")
a = ap.parse_args()
dev = torch.device("cuda", 0)
dt = torch.float64 if a.dtype == "f64" else torch.float32
sb = 8 if a.dtype == "f64" else 4
res = {"ws": os.environ.get("DRONERL_ROLLOUT_WS", "auto"),
       "dtype": a.dtype, "act_sets": a.act_sets}


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for n in a.envs:
    for k in a.ks:
        if k * n * 60 > 8e9:
            continue
        b = DroneBatch(n, "gym", dtype=dt, device=dev, seed=1)
        b.reset()
        obs = torch.empty(k, n, 15, device=dev)
        rew = torch.empty(k, n, device=dev)
        done = torch.empty(k, n, dtype=torch.uint8, device=dev)
        sets = torch.empty(a.act_sets, k, n, 4, device=dev)
        for r in range(a.act_sets):
            for t in range(k):
                random_actions(n, seed=7, step=r * k + t, out=sets[r, t])
        cyc = [0]

        def nxt():
            cyc[0] = (cyc[0] + 1) % a.act_sets
            return sets[cyc[0]]
        st = 15 * sb + 4 + (12 * sb + 4)         # state in + out once per launch
        us_gen = timed(lambda: b.rollout(k, None, seed=7, obs_out=obs, rew_out=rew,
                                         done_out=done), a.reps)
        us_rd = timed(lambda: b.rollout(k, nxt(), obs_out=obs, rew_out=rew, done_out=done),
                      a.reps)
        byt_gen = n * (k * 65 + st)
        byt_rd = n * (k * 81 + st)
        res[f"n{n}_k{k}"] = {
            "gen_us": round(us_gen, 2), "gen_env_steps_per_s": round(n * k / us_gen * 1e6, 1),
            "gen_GBs": round(byt_gen / us_gen / 1e3, 1),
            "read_us": round(us_rd, 2), "read_env_steps_per_s": round(n * k / us_rd * 1e6, 1),
            "read_GBs": round(byt_rd / us_rd / 1e3, 1),
            "mean_done_per_step": round(done.float().mean().item(), 4)}
        print(json.dumps({f"n{n}_k{k}": res[f"n{n}_k{k}"]}), flush=True)
        b.close()
print(json.dumps(res))
