"""CPU restatement of stable-baselines3 PPO arithmetic -- TEST INFRASTRUCTURE.

stable-baselines3 is neither vendored in the reference nor installed here
(SURVEY.md 8c), so these functions restate its published algorithm
 and are "parity unpinned": they pin the HIP kernels,
nothing pins them except the known-answer tests in tests/test_oracle.py.
Reference call sites: /root/reference/train.py:36-43 (PPO defaults),
63-68 (learn).

  gae_numpy        RolloutBuffer.compute_returns_and_advantage (f32, NEP 50)
  ppo_loss_torch   PPO.train's loss expression on CPU, with autograd grads
                   w.r.t. (mean, log_std, values)
  clip_adam_torch  clip_grad_norm_(max_norm) + torch.optim.Adam step
  timeout_bootstrap_numpy  OnPolicyAlgorithm.collect_rollouts' TimeLimit
                   bootstrap (rewards[idx] += gamma * terminal_value)
"""
import numpy as np
import torch


def gae_numpy(rewards, values, episode_starts, last_values, dones, gamma, lam):
    """(T,N) f32 arrays; SB3's loop, same dtypes (python-float scalars)."""
    T = rewards.shape[0]
    adv = np.zeros_like(rewards, dtype=np.float32)
    last = 0
    for step in reversed(range(T)):
        if step == T - 1:
            nnt = 1.0 - dones.astype(np.float32)
            nv = last_values
        else:
            nnt = 1.0 - episode_starts[step + 1]
            nv = values[step + 1]
        delta = rewards[step] + gamma * nv * nnt - values[step]
        last = delta + gamma * lam * nnt * last
        adv[step] = last
    return adv, adv + values


def timeout_bootstrap_numpy(rewards, truncated, terminal_values, gamma):
    """SB3 OnPolicyAlgorithm.collect_rollouts: for every env whose step ended
    an episode by TimeLimit truncation (a terminal_observation and
    TimeLimit.truncated in its info), rewards[idx] += gamma * V(terminal obs).
    rewards (N,) f32, truncated (N,) bool, terminal_values (N,) f32; gamma a
    python float multiplied into the f32 value tensor, as SB3 does."""
    r = np.array(rewards, dtype=np.float32, copy=True)
    tv = (np.float32(gamma) * np.asarray(terminal_values, np.float32)).astype(np.float32)
    r[np.asarray(truncated, bool)] += tv[np.asarray(truncated, bool)]
    return r


def ppo_loss_torch(mean, log_std, values, actions, old_logp, adv, returns,
                   clip=0.2, ent_coef=0.0, vf_coef=0.5, normalize=True):
    """PPO.train's per-minibatch loss (f32 CPU) and its gradients."""
    mean = torch.as_tensor(mean, dtype=torch.float32).clone().requires_grad_(True)
    log_std = torch.as_tensor(log_std, dtype=torch.float32).clone().requires_grad_(True)
    values = torch.as_tensor(values, dtype=torch.float32).clone().requires_grad_(True)
    actions = torch.as_tensor(actions, dtype=torch.float32)
    old_logp = torch.as_tensor(old_logp, dtype=torch.float32)
    adv = torch.as_tensor(adv, dtype=torch.float32)
    returns = torch.as_tensor(returns, dtype=torch.float32)
    std = torch.ones_like(mean) * log_std.exp()
    dist = torch.distributions.Normal(mean, std)
    log_prob = dist.log_prob(actions).sum(dim=1)
    entropy = dist.entropy().sum(dim=1)
    if normalize and len(adv) > 1:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ratio = torch.exp(log_prob - old_logp)
    l1 = adv * ratio
    l2 = adv * torch.clamp(ratio, 1 - clip, 1 + clip)
    policy_loss = -torch.min(l1, l2).mean()
    clip_fraction = torch.mean((torch.abs(ratio - 1) > clip).float()).item()
    value_loss = torch.nn.functional.mse_loss(returns, values)
    entropy_loss = -torch.mean(entropy)
    loss = policy_loss + ent_coef * entropy_loss + vf_coef * value_loss
    with torch.no_grad():
        log_ratio = log_prob - old_logp
        approx_kl = torch.mean((torch.exp(log_ratio) - 1) - log_ratio).item()
    loss.backward()
    stats = dict(loss=loss.item(), policy_loss=policy_loss.item(),
                 value_loss=value_loss.item(), entropy_loss=entropy_loss.item(),
                 clip_fraction=clip_fraction, approx_kl=approx_kl)
    return stats, mean.grad.numpy(), log_std.grad.numpy(), values.grad.numpy()


def clip_adam_torch(params, grads, exp_avg, exp_avg_sq, step, lr=3e-4,
                    betas=(0.9, 0.999), eps=1e-5, max_norm=0.5):
    """One optimizer step as SB3 does it: clip_grad_norm_ then Adam."""
    p = torch.nn.Parameter(torch.as_tensor(params, dtype=torch.float32).clone())
    p.grad = torch.as_tensor(grads, dtype=torch.float32).clone()
    norm = torch.nn.utils.clip_grad_norm_([p], max_norm).item()
    opt = torch.optim.Adam([p], lr=lr, betas=betas, eps=eps, foreach=False)
    st = opt.state[p]
    st["step"] = torch.tensor(float(step - 1))
    st["exp_avg"] = torch.as_tensor(exp_avg, dtype=torch.float32).clone()
    st["exp_avg_sq"] = torch.as_tensor(exp_avg_sq, dtype=torch.float32).clone()
    opt.step()
    return (p.detach().numpy(), st["exp_avg"].numpy(), st["exp_avg_sq"].numpy(),
            p.grad.numpy(), norm)


def sb3_policy_modules(state, net_arch):
    """torch.nn modules shaped like SB3's MlpPolicy from an SB3-named
    state dict (see drone_rl_amd.policy._sb3_name)."""
    nn = torch.nn
    d = len(net_arch)
    pi, vf = [], []
    for k in range(d):
        for net, lst in (("policy_net", pi), ("value_net", vf)):
            w = state[f"mlp_extractor.{net}.{2 * k}.weight"]
            lin = nn.Linear(w.shape[1], w.shape[0])
            lin.weight.data.copy_(w)
            lin.bias.data.copy_(state[f"mlp_extractor.{net}.{2 * k}.bias"])
            lst += [lin, nn.Tanh()]
    act = nn.Linear(net_arch[-1], 4)
    act.weight.data.copy_(state["action_net.weight"])
    act.bias.data.copy_(state["action_net.bias"])
    val = nn.Linear(net_arch[-1], 1)
    val.weight.data.copy_(state["value_net.weight"])
    val.bias.data.copy_(state["value_net.bias"])
    log_std = nn.Parameter(state["log_std"].clone())
    return nn.Sequential(*pi), nn.Sequential(*vf), act, val, log_std


def sb3_train(state, net_arch, obs, actions, old_logp, adv, returns, perms, batch_size,
              lr=3e-4, clip=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
              normalize=True):
    """PPO.train() as SB3 runs it (CPU, f32), over a flat rollout and a given
    list of per-epoch permutations.  Returns the updated SB3-named state."""
    pi, vf, act, val, log_std = sb3_policy_modules(state, net_arch)
    params = list(pi.parameters()) + list(act.parameters()) + list(vf.parameters()) + \
        list(val.parameters()) + [log_std]
    opt = torch.optim.Adam(params, lr=lr, eps=1e-5)
    obs = torch.as_tensor(obs)
    actions = torch.as_tensor(actions)
    old_logp = torch.as_tensor(old_logp)
    adv_all = torch.as_tensor(adv)
    ret_all = torch.as_tensor(returns)
    for perm in perms:
        perm = torch.as_tensor(perm, dtype=torch.long)
        for k in range(len(perm) // batch_size):
            idx = perm[k * batch_size:(k + 1) * batch_size]
            x = obs[idx]
            mean = act(pi(x))
            values = val(vf(x)).flatten()
            dist = torch.distributions.Normal(mean, torch.ones_like(mean) * log_std.exp())
            log_prob = dist.log_prob(actions[idx]).sum(dim=1)
            entropy = dist.entropy().sum(dim=1)
            a = adv_all[idx]
            if normalize and len(a) > 1:
                a = (a - a.mean()) / (a.std() + 1e-8)
            ratio = torch.exp(log_prob - old_logp[idx])
            l1 = a * ratio
            l2 = a * torch.clamp(ratio, 1 - clip, 1 + clip)
            policy_loss = -torch.min(l1, l2).mean()
            value_loss = torch.nn.functional.mse_loss(ret_all[idx], values)
            entropy_loss = -torch.mean(entropy)
            loss = policy_loss + ent_coef * entropy_loss + vf_coef * value_loss
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(params, max_grad_norm)
            opt.step()
    d = len(net_arch)
    out = {}
    for k in range(d):
        out[f"mlp_extractor.policy_net.{2 * k}.weight"] = pi[2 * k].weight.detach()
        out[f"mlp_extractor.policy_net.{2 * k}.bias"] = pi[2 * k].bias.detach()
        out[f"mlp_extractor.value_net.{2 * k}.weight"] = vf[2 * k].weight.detach()
        out[f"mlp_extractor.value_net.{2 * k}.bias"] = vf[2 * k].bias.detach()
    out["action_net.weight"] = act.weight.detach()
    out["action_net.bias"] = act.bias.detach()
    out["value_net.weight"] = val.weight.detach()
    out["value_net.bias"] = val.bias.detach()
    out["log_std"] = log_std.detach()
    return out
