"""torch-facing wrappers of the PPO HIP kernels in libdronerl.so.

Each call enqueues work on the current HIP stream of the tensors' device and
returns device tensors; nothing here synchronises with the host.  Semantics
follow stable-baselines3 PPO (reference call sites
/root/reference/train.py:36-43, 63-68).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check, ptr


def _s(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _f32(t):
    assert t.dtype == torch.float32 and t.is_cuda and t.is_contiguous(), \
        "expected a contiguous f32 device tensor"
    return t


def gae(rewards, values, episode_starts, last_values, last_dones, gamma=0.99,
        gae_lambda=0.95, advantages=None, returns=None):
    """(T,N) rewards/values/episode_starts(u8), (N,) last_values/last_dones(u8)
    -> advantages, returns (T,N) f32 (RolloutBuffer.compute_returns_and_advantage)."""
    T, N = rewards.shape
    adv = torch.empty_like(rewards) if advantages is None else advantages
    ret = torch.empty_like(rewards) if returns is None else returns
    check(_lib.lib().dr_gae(T, N, ptr(_f32(rewards)), ptr(_f32(values)),
                            ptr(episode_starts.contiguous()), ptr(_f32(last_values)),
                            ptr(last_dones.contiguous()), float(gamma), float(gae_lambda),
                            ptr(adv), ptr(ret), _s(rewards)))
    return adv, ret


def policy_sample(mean, log_std, seed, counter, lo, hi, actions_raw=None,
                  actions_clipped=None, logp=None):
    """Diagonal-Gaussian sample a = mean + exp(log_std) z, its log-prob, and
    the clipped action passed to the env (SB3 collect_rollouts)."""
    n = mean.shape[0]
    check(_lib.lib().dr_policy_sample(n, ptr(_f32(mean)), ptr(_f32(log_std)),
                                      seed & (2**64 - 1), counter & (2**64 - 1),
                                      float(lo), float(hi), ptr(actions_raw),
                                      ptr(actions_clipped), ptr(logp), _s(mean)))
    return actions_raw, actions_clipped, logp


def policy_sample_dev(mean, log_std, seed, counter_base, counter_offset, lo, hi,
                      actions_raw=None, actions_clipped=None, logp=None):
    """policy_sample with counter = counter_base[0] + counter_offset, the
    base an int64 device tensor (read by the kernel: graph-capturable)."""
    n = mean.shape[0]
    assert counter_base.dtype == torch.int64 and counter_base.device == mean.device
    check(_lib.lib().dr_policy_sample_dev(n, ptr(_f32(mean)), ptr(_f32(log_std)),
                                          seed & (2**64 - 1), ptr(counter_base),
                                          counter_offset & (2**64 - 1), float(lo), float(hi),
                                          ptr(actions_raw), ptr(actions_clipped), ptr(logp),
                                          _s(mean)))
    return actions_raw, actions_clipped, logp


class Permuter:
    """Uniform random permutations of [0, n) (RolloutBuffer.get)."""

    def __init__(self, n: int, device):
        self.n = n
        nbytes = _lib.lib().dr_permutation_workspace_bytes(n)
        self.ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        self.out = torch.empty(n, dtype=torch.int32, device=device)

    def __call__(self, seed: int, counter: int, out=None):
        o = self.out if out is None else out
        check(_lib.lib().dr_permutation(self.n, seed & (2**64 - 1), counter & (2**64 - 1),
                                        ptr(o), ptr(self.ws), self.ws.numel(), _s(o)))
        return o

    def dev(self, seed: int, counter_base: torch.Tensor, counter_offset: int, out=None):
        """__call__ with counter = counter_base[0] + counter_offset, the base
        an int64 device tensor read by the kernel (graph-capturable)."""
        o = self.out if out is None else out
        assert counter_base.dtype == torch.int64 and counter_base.device == o.device
        check(_lib.lib().dr_permutation_dev(self.n, seed & (2**64 - 1), ptr(counter_base),
                                            counter_offset & (2**64 - 1), ptr(o), ptr(self.ws),
                                            self.ws.numel(), _s(o)))
        return o


def gather_rows(idx, src, out=None):
    """out[k] = src[idx[k]] for a 2-D f32 src (row width = src.shape[1])."""
    src2 = src.reshape(src.shape[0], -1)
    m, w = idx.shape[0], src2.shape[1]
    o = torch.empty(m, w, dtype=torch.float32, device=src.device) if out is None else out
    check(_lib.lib().dr_gather_rows(m, w, ptr(idx), ptr(_f32(src2)), ptr(o), _s(src)))
    return o


def tanh_backward_workspace_bytes(m: int, n: int) -> int:
    return int(_lib.lib().dr_tanh_backward_workspace_bytes(m, n))


def tanh_backward(grad_h, h, grad_z, bias_grad, workspace):
    """grad_z = grad_h * (1 - h^2); bias_grad = grad_z.sum(0) (one pass).
    grad_h / h / grad_z: contiguous (m, n) f32; bias_grad: contiguous (n,)."""
    m, n = h.shape
    for t in (grad_h, h, grad_z):
        assert t.is_contiguous() and t.dtype == torch.float32
    check(_lib.lib().dr_tanh_backward(m, n, ptr(grad_h), ptr(h), ptr(grad_z), ptr(bias_grad),
                                      ptr(workspace), workspace.numel() * workspace.element_size(),
                                      _s(h)))
    return grad_z


class PPOLoss:
    """Fused PPO minibatch loss and its gradient w.r.t. the policy head
    outputs (mean (m,4), log_std (4,), values (m,))."""

    STATS = ("loss", "policy_loss", "value_loss", "entropy_loss", "clip_fraction",
             "approx_kl", "adv_mean", "adv_std")

    def __init__(self, m: int, device, clip_range=0.2, ent_coef=0.0, vf_coef=0.5,
                 normalize_advantage=True):
        self.m = m
        self.clip, self.ent, self.vf = clip_range, ent_coef, vf_coef
        self.norm = int(bool(normalize_advantage))
        nbytes = _lib.lib().dr_ppo_loss_workspace_bytes(m)
        self.ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.grad_mean = torch.empty(m, 4, dtype=torch.float32, device=device)
        self.grad_values = torch.empty(m, dtype=torch.float32, device=device)
        self.grad_log_std = torch.empty(4, dtype=torch.float32, device=device)
        self.stats = torch.empty(8, dtype=torch.float32, device=device)

    def __call__(self, mean, log_std, values, actions, old_logp=None, advantages=None,
                 returns=None, aux=None):
        """Either old_logp / advantages / returns as three (m,) arrays, or
        aux = one contiguous (m,3) array of (old_logp, advantage, return)
        rows (read in place with stride 3)."""
        m = mean.shape[0]
        assert m == self.m
        if aux is not None:
            assert aux.shape == (m, 3)
            base = _f32(aux)
            p_lp, p_adv, p_ret = ptr(base), ptr(base) + 4, ptr(base) + 8
            stride = 3
        else:
            p_lp, p_adv, p_ret = ptr(_f32(old_logp)), ptr(_f32(advantages)), ptr(_f32(returns))
            stride = 1
        check(_lib.lib().dr_ppo_loss(
            m, ptr(_f32(mean)), ptr(_f32(log_std)), ptr(_f32(values)), ptr(_f32(actions)),
            p_lp, p_adv, p_ret, stride,
            float(self.clip), float(self.ent), float(self.vf), self.norm,
            ptr(self.grad_mean), ptr(self.grad_values), ptr(self.grad_log_std),
            ptr(self.stats), ptr(self.ws), self.ws.numel(), _s(mean)))
        return self.grad_mean, self.grad_log_std, self.grad_values, self.stats


class ClipAdam:
    """clip_grad_norm_(max_norm) + torch.optim.Adam over one flat f32 buffer."""

    def __init__(self, params: torch.Tensor, lr=3e-4, betas=(0.9, 0.999), eps=1e-5,
                 max_grad_norm=0.5):
        self.p = params
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.max_norm = max_grad_norm
        self.t = 0
        n = params.numel()
        self.ws = torch.empty(_lib.lib().dr_adam_workspace_bytes(n), dtype=torch.uint8,
                              device=params.device)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=params.device)

    def step_finish(self, grads: torch.Tensor, finish: "GradFinish", lr=None):
        """step() for a gradient whose last reductions were deferred
        (dr_grad_finish_clip_adam: the finish and the norm in one launch,
        then clip + Adam)."""
        self.t += 1
        L = _lib.lib()
        f = ctypes.byref(finish.desc)
        need = L.dr_grad_finish_workspace_bytes(f)
        if finish.ws is None or finish.ws.numel() < need:
            finish.ws = torch.empty(need, dtype=torch.uint8, device=self.p.device)
        check(L.dr_grad_finish_clip_adam(
            f, self.p.numel(), ptr(self.p), ptr(_f32(grads)), ptr(self.m), ptr(self.v),
            float(self.lr if lr is None else lr), float(self.b1), float(self.b2),
            float(self.eps), float(self.max_norm), self.t, ptr(self.grad_norm),
            ptr(finish.ws), finish.ws.numel(), _s(self.p)))
        return self.grad_norm

    def schedule(self, first_step: int, count: int, out: torch.Tensor | None = None):
        """(count, 2) f32 of Adam's step-dependent scalars for steps
        first_step .. first_step + count - 1 (dr_adam_schedule, host)."""
        L = _lib.lib()
        buf = (ctypes.c_float * (2 * count))()
        for j in range(count):
            check(L.dr_adam_schedule(float(self.lr), float(self.b1), float(self.b2),
                                     first_step + j, ctypes.byref(buf, 8 * j)))
        t = torch.frombuffer(bytearray(buf), dtype=torch.float32).view(count, 2)
        if out is None:
            return t
        out.copy_(t)
        return out

    def step_finish_sched(self, grads: torch.Tensor, finish: "GradFinish", sched: torch.Tensor):
        """step_finish with this step's scalars read on the device from
        `sched` (2 f32, from schedule()); advances nothing on the host (the
        caller owns the step count: graph replays)."""
        L = _lib.lib()
        f = ctypes.byref(finish.desc)
        need = L.dr_grad_finish_workspace_bytes(f)
        if finish.ws is None or finish.ws.numel() < need:
            finish.ws = torch.empty(need, dtype=torch.uint8, device=self.p.device)
        check(L.dr_grad_finish_clip_adam_sched(
            f, self.p.numel(), ptr(self.p), ptr(_f32(grads)), ptr(self.m), ptr(self.v),
            float(self.lr), float(self.b1), float(self.b2), float(self.eps),
            float(self.max_norm), ptr(sched), ptr(self.grad_norm), ptr(finish.ws),
            finish.ws.numel(), _s(self.p)))
        return self.grad_norm

    def step_sched(self, grads: torch.Tensor, sched: torch.Tensor, grad_scale: float = 1.0):
        """clip_grad_norm_ + Adam on grad_scale * grads (1 / world after a
        summing all-reduce) with this step's scalars read on the device
        from `sched` (dr_clip_adam_sched; graph-capturable, advances nothing
        on the host).  After dr_grad_finish_run at grad_scale 1 this is
        bitwise step_finish_sched."""
        check(_lib.lib().dr_clip_adam_sched(
            self.p.numel(), ptr(self.p), ptr(_f32(grads)), ptr(self.m), ptr(self.v),
            float(self.b1), float(self.b2), float(self.eps), float(self.max_norm),
            float(grad_scale), ptr(sched), ptr(self.grad_norm), ptr(self.ws), self.ws.numel(),
            _s(self.p)))
        return self.grad_norm

    def step(self, grads: torch.Tensor, lr=None):
        self.t += 1
        check(_lib.lib().dr_clip_adam(
            self.p.numel(), ptr(self.p), ptr(_f32(grads)), ptr(self.m), ptr(self.v),
            float(self.lr if lr is None else lr), float(self.b1), float(self.b2),
            float(self.eps), float(self.max_norm), self.t, ptr(self.grad_norm),
            ptr(self.ws), self.ws.numel(), _s(self.p)))
        return self.grad_norm


LINEAR_TANH_K = (4, 8, 12, 15, 16, 18, 24, 32)


def _rows(rows):
    if rows is None:
        return None
    assert rows.dtype == torch.int32 and rows.is_contiguous()
    return ptr(rows)


def linear_tanh(x, w, b, out, rows=None):
    """out = tanh(x w^T + b) for a narrow input x (., k), k in LINEAR_TANH_K;
    row r of the input is x[rows[r]] when rows (int32) is given."""
    k = x.shape[1]
    m = out.shape[0]
    n = w.shape[0]
    check(_lib.lib().dr_linear_tanh(m, k, n, ptr(_f32(x)), _rows(rows), ptr(_f32(w)),
                                    ptr(_f32(b)), ptr(out), _s(x)))
    return out


def linear_tanh2(x, w0, b0, h0, w1, b1, h1, rows=None):
    """linear_tanh for both MLPs (pi: w0/b0 -> h0, vf: w1/b1 -> h1) over the
    same input rows, one launch."""
    k = x.shape[1]
    m, n = h0.shape
    assert h1.shape == (m, n) and w0.shape == w1.shape == (n, k)
    check(_lib.lib().dr_linear_tanh2(m, k, n, ptr(_f32(x)), _rows(rows), ptr(_f32(w0)),
                                     ptr(_f32(b0)), ptr(h0), ptr(_f32(w1)), ptr(_f32(b1)),
                                     ptr(h1), _s(x)))
    return h0, h1


def linear_tanh2_x6(x, w0, b0, h0, w1, b1, h1, w256, img, ximg=None, rows=None):
    """linear_tanh2 (k 15, n 256) with the 256 x 256 layer's x6 weight images
    (both forms, from w256 (2, 256, 256)) into img and, with ximg, the
    observation image of dr_gemm_x6_bwd_first built in the same launch."""
    k = x.shape[1]
    m, n = h0.shape
    assert h1.shape == (m, n) and w0.shape == w1.shape == (n, k)
    assert w256.shape == (2, 256, 256) and w256.is_contiguous()
    check(_lib.lib().dr_linear_tanh2_x6(m, k, n, ptr(_f32(x)), _rows(rows), ptr(_f32(w0)),
                                        ptr(_f32(b0)), ptr(h0), ptr(_f32(w1)), ptr(_f32(b1)),
                                        ptr(h1), ptr(w256), ptr(img), ptr(ximg), _s(x)))
    return h0, h1


def gather_minibatch(idx, obs, actions, aux, obs_out, actions_out, aux_out, adv_part=None):
    """obs_out / actions_out / aux_out = rows idx of obs (., d) / actions
    (., 4) / aux (., 3), one launch; with adv_part (a HeadLossBackward's
    `adv_part`) also the advantage partials its normalisation needs."""
    m = idx.numel()
    assert idx.dtype == torch.int32 and idx.is_contiguous()
    assert obs_out.shape == (m, obs.shape[1]) and actions_out.shape == (m, 4)
    assert aux_out.shape == (m, 3) and actions.shape[1] == 4 and aux.shape[1] == 3
    check(_lib.lib().dr_gather_minibatch(m, ptr(idx), obs.shape[1], ptr(_f32(obs)),
                                         ptr(_f32(actions)), ptr(_f32(aux)), ptr(obs_out),
                                         ptr(actions_out), ptr(aux_out), ptr(adv_part),
                                         _s(obs)))


RECORD_FLOATS = 32      # DR_RECORD_FLOATS: one 128-B rollout record


def pack_rollout_records(obs, actions, logp, adv, ret, records):
    """records (n, 32) f32: rollout row r as one 128-B record (obs, action,
    old log-prob, advantage, return; dr_pack_rollout_records), for
    gather_records."""
    n, d = obs.shape
    assert actions.shape == (n, 4) and records.shape == (n, RECORD_FLOATS)
    assert logp.numel() == adv.numel() == ret.numel() == n and records.is_contiguous()
    check(_lib.lib().dr_pack_rollout_records(n, d, ptr(_f32(obs)), ptr(_f32(actions)),
                                             ptr(_f32(logp)), ptr(_f32(adv)), ptr(_f32(ret)),
                                             ptr(records), _s(obs)))


def gather_records(idx, records, obs_dim, obs_out, actions_out, aux_out, adv_part=None):
    """gather_minibatch's outputs (the same bytes) from the packed records:
    one cache line per gathered row."""
    m = idx.numel()
    assert idx.dtype == torch.int32 and idx.is_contiguous()
    assert records.shape[1] == RECORD_FLOATS and records.is_contiguous()
    assert obs_out.shape == (m, obs_dim) and actions_out.shape == (m, 4)
    assert aux_out.shape == (m, 3)
    check(_lib.lib().dr_gather_records(m, ptr(idx), obs_dim, ptr(records), ptr(obs_out),
                                       ptr(actions_out), ptr(aux_out), ptr(adv_part),
                                       _s(records)))


def policy_heads(h_pi, h_vf, w_act, b_act, w_val, b_val, mean, value, preact=False,
                 zb_pi=None, zb_vf=None):
    """mean (m,4) = h_pi w_act^T + b_act, value (m) = h_vf w_val^T + b_val;
    with preact the inputs are pre-activations and tanh(z + zb) is applied
    on load (zb_pi / zb_vf: the top layer's biases, when its GEMM left them
    out)."""
    m, hd = h_pi.shape
    check(_lib.lib().dr_policy_heads(m, hd, int(bool(preact)), ptr(_f32(h_pi)), ptr(_f32(h_vf)),
                                     ptr(zb_pi), ptr(zb_vf), ptr(_f32(w_act)),
                                     ptr(_f32(b_act)), ptr(_f32(w_val)), ptr(_f32(b_val)),
                                     ptr(mean), ptr(value), _s(h_pi)))
    return mean, value


class HeadLossBackward:
    """dr_ppo_head_loss_backward: heads + PPO loss + backward through the
    heads and the top tanh of both MLPs, one minibatch of m rows."""

    def __init__(self, m: int, hd: int, device, clip_range=0.2, ent_coef=0.0, vf_coef=0.5,
                 normalize_advantage=True):
        self.m, self.hd = m, hd
        self.clip, self.ent, self.vf = clip_range, ent_coef, vf_coef
        self.norm = int(bool(normalize_advantage))
        self.ws = torch.empty(_lib.lib().dr_ppo_head_workspace_bytes(m, hd), dtype=torch.uint8,
                              device=device)
        self.stats = torch.empty(8, dtype=torch.float32, device=device)

    @property
    def adv_part(self):
        """Where gather_minibatch writes the advantage partials (the head of
        the workspace) for a call with adv_ready=True."""
        return self.ws

    def __call__(self, h_pi, h_vf, w_act, b_act, w_val, b_val, log_std, actions, aux,
                 gz_pi, gz_vf, g_w_act, g_b_act, g_w_val, g_b_val, g_b_pi, g_b_vf, g_log_std,
                 rows=None, preact=False, adv_ready=False, stats_out=None, zb_pi=None,
                 zb_vf=None, defer=False):
        """actions (.,4) / aux (.,3) rows are read as [rows[r]] when rows
        (int32, m) is given, else the first m rows; with preact h_pi / h_vf
        are the top layer's pre-activations (tanh applied on load).  With
        adv_ready the advantage partials were written by gather_minibatch
        (adv_part=self.adv_part) for this minibatch; stats_out (8 f32)
        receives the stats instead of self.stats; zb_pi / zb_vf as
        policy_heads.  With defer the gradient / stats outputs are written
        later by ClipAdam.step_finish (GradFinish); defer=2 leaves the
        per-block rows unreduced for a finish with head_direct = 1."""
        assert h_pi.shape == (self.m, self.hd) and aux.shape[1] == 3
        assert rows is not None or aux.shape[0] == self.m
        stats = self.stats if stats_out is None else stats_out
        assert stats.numel() == 8 and stats.dtype == torch.float32 and stats.is_contiguous()
        norm = 2 if (self.norm and adv_ready) else self.norm
        check(_lib.lib().dr_ppo_head_loss_backward(
            self.m, self.hd, int(bool(preact)), ptr(_f32(h_pi)), ptr(_f32(h_vf)), ptr(zb_pi),
            ptr(zb_vf), ptr(_f32(w_act)),
            ptr(_f32(b_act)), ptr(_f32(w_val)), ptr(_f32(b_val)), ptr(_f32(log_std)),
            ptr(_f32(actions)), ptr(_f32(aux)), _rows(rows), float(self.clip), float(self.ent),
            float(self.vf), norm, ptr(gz_pi), ptr(gz_vf), ptr(g_w_act), ptr(g_b_act),
            ptr(g_w_val), ptr(g_b_val), ptr(g_b_pi), ptr(g_b_vf), ptr(g_log_std),
            ptr(stats), int(defer), ptr(self.ws), self.ws.numel(), _s(h_pi)))
        return stats


class FirstLayerBackward:
    """dr_first_layer_backward: grad_w (n,k), grad_b (n) of h = tanh(x W^T + b)
    from grad_h, without materialising grad_z."""

    def __init__(self, m: int, k: int, n: int, device):
        self.m, self.k, self.n = m, k, n
        self.ws = torch.empty(_lib.lib().dr_first_layer_backward_workspace_bytes(m, k, n),
                              dtype=torch.uint8, device=device)

    def __call__(self, grad_h, h, x, grad_w, grad_b, rows=None):
        assert grad_h.shape == (self.m, self.n) and x.shape[1] == self.k
        assert rows is not None or x.shape[0] == self.m
        check(_lib.lib().dr_first_layer_backward(
            self.m, self.k, self.n, ptr(_f32(grad_h)), ptr(_f32(h)), ptr(_f32(x)), _rows(rows),
            ptr(grad_w), ptr(grad_b), ptr(self.ws), self.ws.numel(), _s(h)))


class FirstLayerBackward2:
    """dr_first_layer_backward2: FirstLayerBackward for both MLPs over the
    same input in one launch (bitwise the same as two single calls)."""

    def __init__(self, m: int, k: int, n: int, device):
        self.m, self.k, self.n = m, k, n
        self.ws = torch.empty(_lib.lib().dr_first_layer_backward2_workspace_bytes(m, k, n),
                              dtype=torch.uint8, device=device)

    def __call__(self, x, grad_h0, h0, grad_w0, grad_b0, grad_h1, h1, grad_w1, grad_b1,
                 rows=None, defer=False):
        for g, h in ((grad_h0, h0), (grad_h1, h1)):
            assert g.shape == (self.m, self.n) and h.shape == (self.m, self.n)
        assert x.shape[1] == self.k and (rows is not None or x.shape[0] == self.m)
        check(_lib.lib().dr_first_layer_backward2(
            self.m, self.k, self.n, ptr(_f32(x)), _rows(rows), ptr(_f32(grad_h0)), ptr(_f32(h0)),
            ptr(grad_w0), ptr(grad_b0), ptr(_f32(grad_h1)), ptr(_f32(h1)), ptr(grad_w1),
            ptr(grad_b1), int(bool(defer)), ptr(self.ws), self.ws.numel(), _s(x)))


class GradFinish:
    """The deferred reductions of one fused minibatch step (the
    dr_grad_finish descriptor: head / first-layer partials, split-K chunks),
    consumed by ClipAdam.step_finish.  `desc` holds raw device pointers: the
    tensors it points into must stay alive (FusedTrainStep owns them)."""

    def __init__(self):
        self.desc = _lib.dr_grad_finish()
        self.ws = None

    def _workspace(self, device):
        need = _lib.lib().dr_grad_finish_workspace_bytes(ctypes.byref(self.desc))
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=device)
        return self.ws

    def run(self, device):
        """dr_grad_finish_run: every deferred partial reduced into the flat
        gradient (and the loss stats) on the current stream -- the
        data-parallel step's finish, ahead of the gradient all-reduce."""
        ws = self._workspace(device)
        check(_lib.lib().dr_grad_finish_run(ctypes.byref(self.desc), ptr(ws), ws.numel(),
                                            torch.cuda.current_stream(device).cuda_stream))
