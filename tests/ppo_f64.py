"""SB3 PPO.train's minibatch loss, gradient and fp32 error envelope in f64
(SURVEY.md Appendix C restatement; SB3 is absent, so "parity unpinned" with
respect to SB3 itself).  Test infrastructure shared by the flagship-size
parity test and the data-parallel union-gradient check
(tests/test_ppo_flagship_parity_gpu.py, tests/dp_train_worker.py)."""
import numpy as np
import torch

U = 2.0 ** -24
# the network's tanh on the GPU (common.h tanh_rat): <= 6 ulp from the
# correctly rounded tanh, against torch's <= 1-2; its derivative factor
# 1 - h^2 then carries an absolute error <= 2 |h| 6 u |h| + u <= 13 u
TANH_ULP = 6


def gamma(n: int) -> float:
    """Higham's gamma_n = n u / (1 - n u) for n dependent fp32 roundings."""
    return n * U / (1 - n * U)


def f64_reference(sd, arch, obs, act, old_logp, adv, ret, clip, vf_coef, normalize,
                  device="cpu", with_act=False):
    """SB3 PPO.train's minibatch loss in f64 with its gradient (SB3 names)
    and the absolute-value envelope of every gradient entry.  with_act: also
    the activation envelope, the same backward with the tanh derivative
    factor |1 - h^2| replaced by 1 -- times 13 u it bounds, to first order,
    what the derivative factor's absolute error (TANH_ULP) adds to an entry,
    which the relative envelope misses where tanh saturates."""
    d = lambda x: torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x,  # noqa: E731
                                  dtype=torch.float64, device=device)
    W = {k: d(v).clone().requires_grad_(True) for k, v in sd.items()}
    x = d(obs)
    hs = {}
    outs = {}
    for net, head in (("policy_net", "action_net"), ("value_net", "value_net")):
        h = x
        lay = []
        for k in range(len(arch)):
            z = h @ W[f"mlp_extractor.{net}.{2 * k}.weight"].T + \
                W[f"mlp_extractor.{net}.{2 * k}.bias"]
            lay.append((h, z))
            h = torch.tanh(z)
            z.retain_grad()
        hs[net] = (lay, h)
        o = h @ W[f"{head}.weight"].T + W[f"{head}.bias"]
        o.retain_grad()
        outs[net] = o
    mean, value = outs["policy_net"], outs["value_net"].flatten()
    log_std = W["log_std"]
    a = d(act)
    z_std = (a - mean) / log_std.exp()
    lp_dim = -0.5 * z_std ** 2 - log_std - 0.5 * np.log(2 * np.pi)
    lp_dim.retain_grad()
    log_prob = lp_dim.sum(1)
    A = d(adv)
    if normalize:
        A = (A - A.mean()) / (A.std() + 1e-8)
    ratio = torch.exp(log_prob - d(old_logp))
    pol = -torch.min(A * ratio, A * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    vloss = torch.mean((d(ret) - value) ** 2)
    loss = pol + vf_coef * vloss                 # ent_coef = 0 (SB3 default)
    loss.backward()
    g = {k: v.grad.detach().clone() for k, v in W.items()}
    # envelope: the backward with |.| products (ent_coef = 0)
    env, env_act = {}, {}
    for net, head in (("policy_net", "action_net"), ("value_net", "value_net")):
        lay, htop = hs[net]
        dout = outs[net].grad.detach().abs()                 # (M, 4) or (M, 1)
        Wh = W[f"{head}.weight"].detach().abs()
        env[f"{head}.weight"] = dout.T @ htop.detach().abs()
        env[f"{head}.bias"] = dout.sum(0)
        env_act[f"{head}.weight"] = torch.zeros_like(env[f"{head}.weight"])
        env_act[f"{head}.bias"] = torch.zeros_like(env[f"{head}.bias"])
        dh = dout @ Wh                                       # |dL/dh| envelope
        dh_a = dh
        for k in reversed(range(len(arch))):
            h_in, z = lay[k]
            th = torch.tanh(z.detach())
            dz = dh * (1 - th ** 2).abs()
            env[f"mlp_extractor.{net}.{2 * k}.weight"] = dz.T @ h_in.detach().abs()
            env[f"mlp_extractor.{net}.{2 * k}.bias"] = dz.sum(0)
            if with_act:
                env_act[f"mlp_extractor.{net}.{2 * k}.weight"] = dh_a.T @ h_in.detach().abs()
                env_act[f"mlp_extractor.{net}.{2 * k}.bias"] = dh_a.sum(0)
            dh = dz @ W[f"mlp_extractor.{net}.{2 * k}.weight"].detach().abs()
            dh_a = dh_a @ W[f"mlp_extractor.{net}.{2 * k}.weight"].detach().abs()
    # log_std: d lp_dim / d log_std = z^2 - 1 per row and dimension
    env["log_std"] = (lp_dim.grad.detach() * (z_std.detach() ** 2 - 1)).abs().sum(0) + \
        (lp_dim.grad.detach()).abs().sum(0)
    if with_act:
        env_act["log_std"] = torch.zeros_like(env["log_std"])
        return g, env, env_act
    return g, env
