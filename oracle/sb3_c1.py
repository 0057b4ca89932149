"""Config-1 CPU PPO anchor -- TEST INFRASTRUCTURE / BASELINE ONLY.

The reference's training path (/root/reference/train.py:33-43, 63-68) is
SB3 PPO("MlpPolicy") with its defaults over DummyVecEnv(1 x DroneGymEnv) +
VecMonitor.  SB3 is not installed, so this file restates that
loop on CPU (torch f32, numpy env = oracle/drone_np.GymDronePort, which is
pinned bit-exact to the reference's golden vectors) and runs it for 2e6
steps.  Its final ep_rew_mean is the "hover-to-target return" that the GPU
PPO (configs[2]) must reach (BASELINE.md CPU-baseline plan 4).
Parity unpinned w.r.t. SB3 itself (restated from its published algorithm,
SURVEY.md Appendix C): n_steps 2048, batch 64, 10 epochs, lr 3e-4,
gamma 0.99, gae_lambda 0.95, clip 0.2, ent 0, vf 0.5, max_grad_norm 0.5,
Adam eps 1e-5, 64x64 tanh, orthogonal init (sqrt 2 / 0.01 / 1), log_std 0,
actions clipped to [0, 7.3575] for the env only, no time-limit bootstrap
(the env returns info {}), ep_rew_mean over the last 100 episodes.

Usage: python -m oracle.sb3_c1 --steps 2000000 --seed 0 --out c1_seed0.json
"""
import argparse
import json
import time
from collections import deque

import numpy as np
import torch
from torch import nn

from oracle.drone_np import A_MAX, GymDronePort


class MlpPolicy(nn.Module):
    def __init__(self, obs_dim=15, act_dim=4, arch=(64, 64)):
        super().__init__()

        def mlp():
            layers, d = [], obs_dim
            for h in arch:
                lin = nn.Linear(d, h)
                nn.init.orthogonal_(lin.weight, gain=np.sqrt(2))
                nn.init.zeros_(lin.bias)
                layers += [lin, nn.Tanh()]
                d = h
            return nn.Sequential(*layers)

        self.pi, self.vf = mlp(), mlp()
        self.action_net = nn.Linear(arch[-1], act_dim)
        nn.init.orthogonal_(self.action_net.weight, gain=0.01)
        nn.init.zeros_(self.action_net.bias)
        self.value_net = nn.Linear(arch[-1], 1)
        nn.init.orthogonal_(self.value_net.weight, gain=1.0)
        nn.init.zeros_(self.value_net.bias)
        self.log_std = nn.Parameter(torch.zeros(act_dim))

    def dist_value(self, obs):
        mean = self.action_net(self.pi(obs))
        dist = torch.distributions.Normal(mean, torch.ones_like(mean) * self.log_std.exp())
        return dist, self.value_net(self.vf(obs)).flatten()


def run(steps=2_000_000, seed=0, n_steps=2048, batch=64, epochs=10, lr=3e-4, gamma=0.99,
        lam=0.95, clip=0.2, vf_coef=0.5, max_grad_norm=0.5, log_every=10, log=print):
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    env = GymDronePort(rng)
    pol = MlpPolicy()
    opt = torch.optim.Adam(pol.parameters(), lr=lr, eps=1e-5)
    obs = env.reset()
    last_start = True
    ep_ret, ep_len = 0.0, 0
    ep_buf = deque(maxlen=100)
    len_buf = deque(maxlen=100)
    hist = []
    t0 = time.perf_counter()
    done_steps = 0
    it = 0
    while done_steps < steps:
        O = np.zeros((n_steps, 15), np.float32)
        A = np.zeros((n_steps, 4), np.float32)
        R = np.zeros(n_steps, np.float32)
        S = np.zeros(n_steps, np.float32)
        V = np.zeros(n_steps, np.float32)
        LP = np.zeros(n_steps, np.float32)
        with torch.no_grad():
            for t in range(n_steps):
                dist, v = pol.dist_value(torch.from_numpy(obs)[None])
                a = dist.sample()
                O[t], A[t], S[t] = obs, a[0].numpy(), float(last_start)
                V[t], LP[t] = v.item(), dist.log_prob(a).sum(-1).item()
                obs, r, d, _ = env.step(np.clip(A[t], 0.0, A_MAX))
                ep_ret += np.float32(r)
                ep_len += 1
                R[t] = r
                if d:
                    ep_buf.append(float(ep_ret))
                    len_buf.append(ep_len)
                    ep_ret, ep_len = 0.0, 0
                    obs = env.reset()
                last_start = d
            _, last_v = pol.dist_value(torch.from_numpy(obs)[None])
        # GAE (RolloutBuffer.compute_returns_and_advantage)
        adv = np.zeros(n_steps, np.float32)
        g = 0.0
        for t in reversed(range(n_steps)):
            if t == n_steps - 1:
                nnt, nv = 1.0 - float(last_start), last_v.item()
            else:
                nnt, nv = 1.0 - S[t + 1], V[t + 1]
            delta = R[t] + gamma * nv * nnt - V[t]
            g = delta + gamma * lam * nnt * g
            adv[t] = g
        ret = adv + V
        Ot, At, LPt = torch.from_numpy(O), torch.from_numpy(A), torch.from_numpy(LP)
        ADt, RTt = torch.from_numpy(adv), torch.from_numpy(ret)
        for _ in range(epochs):
            perm = torch.from_numpy(rng.permutation(n_steps))
            for k in range(n_steps // batch):
                idx = perm[k * batch:(k + 1) * batch]
                dist, v = pol.dist_value(Ot[idx])
                lp = dist.log_prob(At[idx]).sum(-1)
                a = ADt[idx]
                a = (a - a.mean()) / (a.std() + 1e-8)
                ratio = torch.exp(lp - LPt[idx])
                pl = -torch.min(a * ratio, a * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
                vl = nn.functional.mse_loss(RTt[idx], v)
                loss = pl + vf_coef * vl
                opt.zero_grad()
                loss.backward()
                nn.utils.clip_grad_norm_(pol.parameters(), max_norm=max_grad_norm)
                opt.step()
        done_steps += n_steps
        it += 1
        if it % log_every == 0 or done_steps >= steps:
            row = {"timesteps": done_steps, "ep_rew_mean": float(np.mean(ep_buf)) if ep_buf else None,
                   "ep_len_mean": float(np.mean(len_buf)) if len_buf else None,
                   "eps": env.eps, "ep_num": env.ep_num,
                   "elapsed_s": round(time.perf_counter() - t0, 1)}
            hist.append(row)
            log(json.dumps(row))
    return {"seed": seed, "steps": done_steps, "final_ep_rew_mean": float(np.mean(ep_buf)),
            "final_ep_len_mean": float(np.mean(len_buf)), "final_eps": env.eps, "episodes": env.ep_num, "history": hist,
            "elapsed_s": round(time.perf_counter() - t0, 1)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2_000_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.set_num_threads(1)
    res = run(a.steps, a.seed, log=lambda s: print(s, flush=True))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "history"}))
