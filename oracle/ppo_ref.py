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
