"""PPO.train parity at the flagship size: 2x256 MLP, one 65,536-row
minibatch (configs[2]'s minibatch), against an f64 restatement of SB3's
PPO.train (SB3 itself is absent, so this is parity
with the restatement -- "parity unpinned" with respect to SB3).

Tolerances are derived, per parameter, from fp32 reduction-order error
bounds instead of a fraction of the largest update:

* Gradient.  Every gradient entry is a sum over rows of products of
  activations and back-propagated deltas, g_i = sum_r t_{r,i}.  Its fp32
  evaluation in any summation order satisfies |fl(g_i) - g_i| <=
  gamma_n * sum_r |t_{r,i}| (Higham, Accuracy and Stability of Numerical
  Algorithms, eq. 4.4, gamma_n = n u / (1 - n u), u = 2^-24), where n is the
  longest chain of dependent roundings.  On the GPU path that chain is the
  forward / backward dot products (K = 256 terms, twice), the split-K
  chunk of 65,536 / 64 = 1,024 rows accumulated in a GEMM, and the
  64-chunk sum: n = 256 + 256 + 1,024 + 64 (+ 448 for the elementwise loss,
  tanh and normalisation steps) = 2,048.  The envelope sum_r |t_{r,i}| is
  computed in f64 by running the backward with every product replaced by the
  product of absolute values (an upper bound for every partial sum, so the
  bound also covers errors in the per-row factors to first order).  The
  network's tanh is a rational approximation within 6 ulp (common.h
  tanh_rat; torch's is within 1-2): its relative error is one more rounding
  in the chain, and its derivative factor 1 - h^2 carries an absolute error
  <= 13 u, which where tanh saturates exceeds u |1 - h^2|; that term is
  bounded separately by 13 u times the envelope with |1 - h^2| replaced by
  1 (ppo_f64.f64_reference(with_act=True)).

* Update.  clip_grad_norm_ + the first Adam step (bias-corrected) map g to
  u_i = lr * c g_i / (c |g_i| + eps), c = min(1, max_norm / ||g||).  The
  gradient error propagates through d u_i / d g_i = lr c eps / (c |g_i| +
  eps)^2 and through the clip factor (d c / c <= ||dg|| / ||g||), plus the
  fp32 rounding of the update itself and of the parameter (one ulp).
"""
import pytest
import torch

from ppo_f64 import TANH_ULP, U, f64_reference, gamma

pytestmark = pytest.mark.gpu

GAMMA = gamma(2048 + 2 * 2 * TANH_ULP)     # + each tanh / derivative as TANH_ULP roundings


def test_train_one_minibatch_matches_f64_restatement_within_fp32_bounds():
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=65536, n_steps=1, batch_size=65536, n_epochs=1, seed=21)
    tr = PPOTrainer(cfg)
    tr.train_graph = False
    tr.collect_rollouts()
    sd0 = tr.policy.state_dict()
    M = 65536
    obs = tr.obs[0].reshape(M, -1).cpu().numpy()
    act = tr.actions[0].reshape(M, 4).cpu().numpy()
    aux = tr.aux.cpu().numpy()
    # the GPU minibatch gradient, exactly as train() forms it (the fused
    # clip + Adam kernel leaves the clipped gradient c * g in the buffer, as
    # torch's clip_grad_norm_ does; c from the norm the kernel reports)
    from drone_rl_amd.policy import _sb3_name
    tr.train()
    norm_gpu = tr.opt.grad_norm.item()
    c_gpu = min(1.0, cfg.max_grad_norm / (norm_gpu + 1e-6))
    g_gpu = {_sb3_name(name, 2): tr.fused.gview(name).detach().cpu().double() / c_gpu
             for name, _, _ in tr.policy.layout}
    sd1 = tr.policy.state_dict()
    g_ref, env, env_act = f64_reference(sd0, cfg.net_arch, obs, act, aux[:, 0], aux[:, 1],
                                        aux[:, 2], cfg.clip_range, cfg.vf_coef,
                                        cfg.normalize_advantage, with_act=True)
    # every entry's fp32 error bound: reduction order (GAMMA x envelope) + the
    # tanh derivative factor's absolute error ((2 TANH_ULP + 1) u x the
    # activation envelope)
    dgb = {k: GAMMA * env[k] + (2 * TANH_ULP + 1) * U * env_act[k] for k in env}
    # 1. gradient within the fp32 reduction-order bound, entrywise
    worst = 0.0
    for k in g_ref:
        # + the clip factor's own rounding and the division by it
        tol = dgb[k] + 4 * U * g_ref[k].abs() + 1e-30
        r = ((g_gpu[k].reshape(g_ref[k].shape) - g_ref[k]).abs() / tol).max().item()
        worst = max(worst, r)
        assert r <= 1.0, f"{k}: gradient error {r:.3f} x its fp32 bound"
    # 2. the clip + Adam update, with the gradient bound propagated
    gv = torch.cat([g_ref[k].flatten() for k in g_ref])
    ev = torch.cat([dgb[k].flatten() for k in g_ref])
    norm = gv.norm().item()
    c = min(1.0, cfg.max_grad_norm / (norm + 1e-6))
    # the norm the kernel used: within the propagated gradient bound plus its
    # own fp32 sum of squares over 141,065 entries
    assert abs(norm_gpu - norm) <= ev.norm().item() + 1e-5 * norm
    dc = c * (ev.norm().item() + 1e-5 * norm) / norm
    lr, eps = cfg.learning_rate, 1e-5
    for k in g_ref:
        g, dg = g_ref[k].flatten().abs(), dgb[k].flatten()
        upd_ref = lr * c * g_ref[k].flatten() / (c * g + eps)
        den = (c * (g - dg).clamp(min=0) + eps) ** 2
        bound = lr * (c * eps * dg + eps * g * dc) / den + 8 * U * upd_ref.abs()
        p0 = sd0[k].flatten().double()
        p1 = sd1[k].flatten().double()
        ulp = p1.abs() * U * 2 + 1e-45
        err = ((p0 - p1) - upd_ref).abs()
        r = (err / (bound + ulp)).max().item()
        worst = max(worst, r)
        assert r <= 1.0, f"{k}: update error {r:.3f} x its bound"
    print(f"worst error / bound: {worst:.4f}")
    tr.close()
