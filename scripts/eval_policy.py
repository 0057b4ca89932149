"""Evaluate a trained policy (a PPOTrainer checkpoint) on N fresh gym envs at
a fixed curriculum level, the way the reference's test.py does
(model.predict(obs, deterministic=True): the Gaussian's mean clipped to the
action space) and with sampled actions (the training-time policy), for S
steps with DummyVecEnv auto-reset.  Prints one JSON line: mean return and
length of the episodes that ended, the fraction of steps inside the 5 cm
bonus radius, and the fraction of episodes that ended by crashing (before
the 200-step limit).

  python scripts/eval_policy.py CKPT --eps 1.0 [--envs 65536 --steps 400]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from drone_rl_amd import DroneBatch  # noqa: E402
from drone_rl_amd.env import MOTOR_MAX  # noqa: E402
from drone_rl_amd.policy import ActorCritic, PolicyInference  # noqa: E402


@torch.no_grad()
def evaluate(ckpt, eps, envs, steps, seed, deterministic):
    sd = torch.load(ckpt, map_location="cpu", weights_only=True)
    cfg = sd["config"]
    dev = torch.device("cuda", 0)
    pol = ActorCritic(15, 4, tuple(cfg["net_arch"]), dev, 0.0, 0)
    pol.flat.data.copy_(sd["flat"].to(dev))
    env = DroneBatch(envs, "gym", device=dev, seed=seed, env_id_offset=1 << 40, monitor=True)
    env.set("eps", torch.full((envs,), float(eps), dtype=torch.float64))
    obs = env.reset().clone()
    infer = PolicyInference(pol, envs)
    g = torch.Generator(device=dev).manual_seed(seed)
    std = pol.log_std.exp()
    ret_sum = len_sum = n_done = n_crash = 0.0
    in_bonus = 0.0
    ep_ret = torch.empty(envs, device=dev)
    ep_len = torch.empty(envs, dtype=torch.int32, device=dev)
    for _ in range(steps):
        mean, _ = infer(obs)
        a = mean if deterministic else mean + std * torch.randn(mean.shape, generator=g,
                                                                 device=dev)
        env.ep_ret, env.ep_len = ep_ret, ep_len
        o, r, d = env.step(a.clamp(0.0, MOTOR_MAX).contiguous())
        obs = o.clone()
        db = d.bool()
        in_bonus += float((r > 0).float().mean())      # +1 - 0.01 d > 0 only within 5 cm
        n_done += float(db.sum())
        ret_sum += float(ep_ret[db].sum())
        len_sum += float(ep_len[db].float().sum())
        n_crash += float((db & (ep_len < 200)).sum())
    env.close()
    n = max(n_done, 1.0)
    return {"deterministic": deterministic, "episodes": int(n_done),
            "ep_rew_mean": ret_sum / n, "ep_len_mean": len_sum / n,
            "crash_frac": n_crash / n, "bonus_step_frac": in_bonus / steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ckpt")
    ap.add_argument("--eps", type=float, default=1.0)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--seed", type=int, default=123)
    a = ap.parse_args()
    out = {"ckpt": os.path.basename(a.ckpt), "eps": a.eps, "envs": a.envs, "steps": a.steps}
    for det in (True, False):
        out["deterministic" if det else "sampled"] = evaluate(a.ckpt, a.eps, a.envs, a.steps,
                                                               a.seed, det)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
