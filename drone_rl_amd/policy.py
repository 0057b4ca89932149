"""Actor-critic MLP over ONE flat fp32 parameter buffer.

Mirrors stable-baselines3's default `MlpPolicy` for a Box action space
(called by the reference at /root/reference/train.py:36-43; SB3 is not
vendored): Flatten features, separate pi / vf MLPs with
Tanh, `action_net` Linear(h, 4) for the Gaussian mean, `value_net`
Linear(h, 1), a state-independent `log_std` (init 0), orthogonal init with
gains sqrt(2) (hidden), 0.01 (action), 1 (value) and zero biases.

Every parameter is a view into `self.flat`, so autograd accumulates all
gradients into one contiguous `flat.grad`: one RCCL all-reduce and one fused
clip+Adam kernel per optimizer step (drone_rl_amd/ppo_kernels.py).  The
GEMMs run through torch (hipBLASLt -> MFMA, fp32).  The layer order inside
`flat` is pi layers, action head, vf layers, value head, log_std.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.nn.functional as F


TUNED_GEMMS_CSV = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned",
                               "gemm_gfx950.csv")


def use_tuned_gemms(path: str = TUNED_GEMMS_CSV) -> bool:
    """Load the GEMM solutions measured for this trainer's shapes on MI355X.

    The fp32 GEMM shapes of a 65,536-row 2x256 minibatch (the batched
    top-layer forward of both MLPs, batched grad-input, batched split-K
    weight gradient; the single-net addmm) were timed by
    PyTorch's TunableOp over every hipBLASLt and rocBLAS solution on the box
    (scripts/tune_gemm.sh); the winners are committed in `tuned/`.  This
    turns TunableOp on in lookup-only mode (no tuning at run time; shapes
    not in the file keep the library heuristic).  The grad-input GEMM goes
    from 146 to 123 us, the weight gradient from 126 to 122 us, the batched
    forward takes 125 us (two heuristic addmm: 148 us).
    `DRONERL_TUNED_GEMMS=0` opts out; a caller that already enabled TunableOp
    (PYTORCH_TUNABLEOP_*) keeps its own settings.  Returns whether the file
    was loaded (False off-GPU or when its validators do not match)."""
    if os.environ.get("DRONERL_TUNED_GEMMS", "1") == "0" or not torch.cuda.is_available():
        return False
    import torch.cuda.tunable as tun
    if not tun.is_enabled():
        tun.enable(True)
        tun.tuning_enable(False)
    return bool(tun.read_file(path))


class _SplitKLinear(torch.autograd.Function):
    """y = x W^T + b whose backward forms dW = g^T x and db = sum(g) as a
    batched GEMM over C row chunks followed by a sum (split-K).  With
    M = 65,536 rows and a 256-wide layer the library's own dW GEMM is a
    (256 x 256, K = 65,536) problem that it tiles into ~70 workgroups on a
    256-CU chip (215 us); the chunked form fills the chip (77 us)."""

    @staticmethod
    def forward(ctx, x, w, b, chunks):
        ctx.save_for_backward(x, w)
        ctx.chunks = chunks
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        C = ctx.chunks
        M, N = g.shape
        gx = g @ w if ctx.needs_input_grad[0] else None
        gc = g.reshape(C, M // C, N)
        gw = torch.bmm(gc.transpose(1, 2), x.reshape(C, M // C, -1)).sum(0)
        gb = gc.sum(1).sum(0)
        return gx, gw, gb, None


def linear(x, w, b):
    """F.linear, with the split-K backward when x has many rows."""
    M = x.shape[0]
    if torch.is_grad_enabled() and M >= 8192 and M % 64 == 0:
        return _SplitKLinear.apply(x, w, b, 128 if w.shape[0] == 1 else 64)
    return F.linear(x, w, b)


class ActorCritic:
    def __init__(self, obs_dim: int = 15, act_dim: int = 4, net_arch=(256, 256),
                 device=None, log_std_init: float = 0.0, seed: int = 0):
        self.obs_dim, self.act_dim = obs_dim, act_dim
        self.net_arch = tuple(net_arch)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        # Parameters in SB3 registration order (also the init order, so a
        # seed gives SB3's draw sequence): (name, shape, init gain or None)
        self.layout = []
        dims = (obs_dim,) + self.net_arch
        for pre in ("pi", "vf"):
            for k in range(len(self.net_arch)):
                self.layout.append((f"{pre}{k}.w", (dims[k + 1], dims[k]), math.sqrt(2)))
                self.layout.append((f"{pre}{k}.b", (dims[k + 1],), None))
            if pre == "pi":
                self.layout.append(("action.w", (act_dim, dims[-1]), 0.01))
                self.layout.append(("action.b", (act_dim,), None))
            else:
                self.layout.append(("value.w", (1, dims[-1]), 1.0))
                self.layout.append(("value.b", (1,), None))
        self.layout.append(("log_std", (act_dim,), "log_std"))
        # Storage order in the flat buffer: the pi and vf tensors of each
        # hidden layer adjacent (pi{k}.w, vf{k}.w, pi{k}.b, vf{k}.b), so a
        # layer of both MLPs is one (2, out, in) view for batched GEMMs;
        # every tensor size is a multiple of 4 floats up to value.b, so each
        # weight stays 16-byte aligned.
        by_name = {name: (shape, gain) for name, shape, gain in self.layout}
        store = []
        for k in range(len(self.net_arch)):
            store += [f"pi{k}.w", f"vf{k}.w", f"pi{k}.b", f"vf{k}.b"]
        store += ["action.w", "action.b", "value.w", "value.b", "log_std"]
        self.offsets = {}
        off = 0
        for name in store:
            shape = by_name[name][0]
            n = int(np.prod(shape))
            self.offsets[name] = (off, off + n, shape)
            off += n
        self.num_params = off
        # the 256 x 256 layer's forward / input-gradient GEMMs on dr_gemm_x6
        # (fp32-accurate bf16 MFMA) where it applies;
        # DRONERL_GEMM_X6=0: the f32 library GEMMs
        self.gemm_x6 = os.environ.get("DRONERL_GEMM_X6", "1") != "0"
        # the layer's input gradient with the first layer's backward fused
        # into its epilogue (dr_gemm_x6_bwd_first, round 5) on the deferred-
        # finish path; DRONERL_X6_FL=0: dr_gemm_x6 + dr_first_layer_backward2
        self.gemm_x6_fl = os.environ.get("DRONERL_X6_FL", "1") != "0"
        # its per-block rows summed by the deferred finish (no grouping launch)
        self.gemm_x6_fl_direct = os.environ.get("DRONERL_X6_FL_DIRECT", "1") != "0"
        # the x6 operand images built by the first layer's forward launch
        # (dr_linear_tanh2_x6) instead of their own launches
        self.x6_fused_images = os.environ.get("DRONERL_X6_FUSED_IMAGES", "1") != "0"
        # the head kernel's per-block rows summed by the deferred finish too
        self.head_direct = os.environ.get("DRONERL_HEAD_DIRECT", "1") != "0"
        self._x6 = None
        self.flat = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.reset_parameters(seed, log_std_init)
        self.flat.requires_grad_(True)

    def reset_parameters(self, seed: int, log_std_init: float = 0.0):
        g = torch.Generator().manual_seed(seed)
        host = torch.zeros(self.num_params, dtype=torch.float32)
        for name, shape, gain in self.layout:
            a, b, _ = self.offsets[name]
            if gain == "log_std":
                host[a:b] = log_std_init
            elif gain is not None:
                w = torch.empty(shape)
                torch.nn.init.orthogonal_(w, gain=gain, generator=g)
                host[a:b] = w.reshape(-1)
        with torch.no_grad():
            self.flat.copy_(host.to(self.device))

    def p(self, name):
        a, b, shape = self.offsets[name]
        return self.flat[a:b].view(shape)

    def p2(self, k: int, kind: str, buf=None):
        """Layer k of both MLPs as one (2, ...) view of `buf` (default the
        parameters): kind "w" -> (2, out, in), "b" -> (2, out)."""
        buf = self.flat if buf is None else buf
        a, _, shape = self.offsets[f"pi{k}.{kind}"]
        _, b, _ = self.offsets[f"vf{k}.{kind}"]
        return buf[a:b].view((2,) + tuple(shape))

    @property
    def log_std(self):
        return self.p("log_std")

    def _mlp(self, x, pre):
        for k in range(len(self.net_arch)):
            x = torch.tanh(linear(x, self.p(f"{pre}{k}.w"), self.p(f"{pre}{k}.b")))
        return x

    def forward(self, obs):
        """obs (M, obs_dim) f32 -> (mean (M, act_dim), value (M,))."""
        mean = linear(self._mlp(obs, "pi"), self.p("action.w"), self.p("action.b"))
        value = linear(self._mlp(obs, "vf"), self.p("value.w"), self.p("value.b"))
        return mean, value.squeeze(-1)

    __call__ = forward

    @torch.no_grad()
    def predict(self, obs, deterministic: bool = True, generator=None):
        """SB3 ``BasePolicy.predict`` (test.py:13): the distribution's mode
        (or a sample) clipped to the action space [0, 7.3575].  Accepts one
        observation (obs_dim,) or a batch (N, obs_dim), numpy or tensor;
        returns the same kind it was given."""
        is_np = not isinstance(obs, torch.Tensor)
        x = torch.as_tensor(np.asarray(obs, np.float32) if is_np else obs,
                            dtype=torch.float32, device=self.device)
        single = x.dim() == 1
        x = x.reshape(-1, self.obs_dim)
        mean, _ = self.forward(x)
        if not deterministic:
            z = torch.randn(mean.shape, generator=generator, device=self.device)
            mean = mean + self.log_std.exp() * z
        a = mean.clamp(0.0, 3 * 1.0 * 9.81 / 4.0)
        a = a[0] if single else a
        return (a.cpu().numpy(), None) if is_np else (a, None)

    def state_dict(self):
        """SB3-style parameter names (policy.mlp_extractor.policy_net.0.weight
        etc.) mapped to CPU tensors."""
        out = {}
        for name, _, _ in self.layout:
            out[_sb3_name(name, len(self.net_arch))] = self.p(name).detach().cpu().clone()
        return out

    def load_state_dict(self, sd):
        with torch.no_grad():
            for name, _, _ in self.layout:
                self.p(name).copy_(torch.as_tensor(sd[_sb3_name(name, len(self.net_arch))]))


class X6Weights:
    """Both MLPs' 256 x 256 layer weights pre-split for dr_gemm_x6
    (DESIGN.md section 12): `fwd` for z = h W^T, `bwd` for grad_h = grad_z W.
    refresh() re-splits the current weights (one launch, graph-capturable);
    callers refresh whenever the weights may have changed."""

    def __init__(self, pol: "ActorCritic"):
        from . import _lib
        nb = _lib.lib().dr_gemm_x6_weights_bytes(2)
        self.pol = pol
        self.img = torch.empty(2 * nb, dtype=torch.uint8, device=pol.device)
        self.fwd, self.bwd = self.img[:nb], self.img[nb:]

    def refresh(self):
        from . import _lib
        w = self.pol.p2(1, "w")
        _lib.check(_lib.lib().dr_gemm_x6_split_weights(
            2, w.data_ptr(), 2, self.img.data_ptr(),
            torch.cuda.current_stream(w.device).cuda_stream))


def x6_weights(pol: "ActorCritic", m: int):
    """pol's X6Weights when dr_gemm_x6 covers its 256 x 256 layer at m rows
    (net_arch (256, 256), m a positive multiple of 128, pol.gemm_x6), else
    None (the library GEMMs run)."""
    if (not pol.gemm_x6 or pol.net_arch != (256, 256) or m < 128 or m % 128 or
            pol.device.type != "cuda"):
        return None
    if pol._x6 is None:
        pol._x6 = X6Weights(pol)
    return pol._x6


def gemm_x6(a, img, out):
    """out (2, m, 256) = a (2, m, 256) . Bt^T for the pre-split image img."""
    from . import _lib
    _lib.check(_lib.lib().dr_gemm_x6(2, a.shape[1], a.data_ptr(), img.data_ptr(), out.data_ptr(),
                                     torch.cuda.current_stream(a.device).cuda_stream))


def _sb3_name(name: str, depth: int) -> str:
    if name == "log_std":
        return "log_std"
    if name.startswith("action."):
        return "action_net." + ("weight" if name.endswith("w") else "bias")
    if name.startswith("value."):
        return "value_net." + ("weight" if name.endswith("w") else "bias")
    net = "policy_net" if name.startswith("pi") else "value_net"
    k = int(name[2:name.index(".")])
    # SB3 MlpExtractor: Sequential(Linear, Tanh, Linear, Tanh) -> indices 0, 2
    return f"mlp_extractor.{net}.{2 * k}." + ("weight" if name.endswith("w") else "bias")


class FusedTrainStep:
    """Forward + hand-written backward of the actor-critic for one minibatch,
    writing every parameter gradient straight into a flat buffer (no
    autograd graph, no per-view gradient accumulation kernels).

    Per hidden layer the backward is: the fused HIP `dr_tanh_backward`
    (grad_z = grad_h * (1 - h^2) and the bias gradient in one pass), a
    split-K weight gradient (batched GEMM over C row chunks, then one sum
    into the flat-gradient view) and, below the top layer, grad_h = grad_z W.
    GEMMs are fp32 (hipBLASLt, MFMA).  Numerically this is the same
    computation autograd performs (checked in tests/test_ppo_gpu.py against
    the SB3 restatement)."""

    def __init__(self, policy: ActorCritic, m: int, chunks: int = 64):
        from . import ppo_kernels as K
        self.K = K
        self.pol = policy
        self.m = m
        self.C = chunks if m % chunks == 0 else 1
        dev = policy.device
        wmax = max(policy.net_arch)
        f32 = dict(dtype=torch.float32, device=dev)
        self.grad = torch.zeros(policy.num_params, **f32)
        # flat storage, viewed per layer width so every view is contiguous
        self._g = torch.empty(m * wmax, **f32)
        self._gz = torch.empty(m * wmax, **f32)
        dims = (policy.obs_dim,) + policy.net_arch
        self._ws = torch.empty(self.C * wmax * max(dims), **f32)
        self.tanh_ws = torch.empty(
            max(K.tanh_backward_workspace_bytes(m, n) for n in policy.net_arch) // 4 + 1, **f32)
        # the fused input-gradient + first-layer kernel right after the head,
        # ahead of the weight gradient: it reads grad_z2 and h1 first, while
        # grad_z2 is fresh in the Infinity Cache (7.32 vs 7.27 updates/s
        # in-process, one box; DRONERL_FL_FIRST=0 for the other order)
        self.fl_first = os.environ.get("DRONERL_FL_FIRST", "1") != "0"
        # optional instrumentation: mark(name) is called on the host right
        # after each kernel of the fused step is enqueued (bench.py records a
        # HIP event there to time every kernel on the stream)
        self.mark = None

    def gview(self, name):
        a, b, shape = self.pol.offsets[name]
        return self.grad[a:b].view(shape)

    # ------------------------------------------------- fused minibatch step
    def fusable(self) -> bool:
        return fusable(self.pol)

    def _alloc_fused(self):
        if getattr(self, "_acts2", None) is not None:
            return
        pol, M = self.pol, self.m
        f32 = dict(dtype=torch.float32, device=pol.device)
        # both MLPs' activations of a layer in one (2, M, n) buffer, so the
        # layers above the first run as one batched GEMM for pi and vf
        self._acts2 = [torch.empty(2, M, n, **f32) for n in pol.net_arch]
        self._acts = {pre: [a[j] for a in self._acts2] for j, pre in enumerate(("pi", "vf"))}
        self._gz2 = [torch.empty(2, M, n, **f32) for n in pol.net_arch]
        self._g2 = torch.empty(2, M, max(pol.net_arch), **f32)
        self._ws2 = torch.empty(2 * self.C * max(pol.net_arch) ** 2, **f32) if self.C > 1 else None
        self._first = self.K.FirstLayerBackward2(M, pol.obs_dim, pol.net_arch[0], pol.device)

    def first_layer_end(self) -> int:
        """Flat offset where the first layer's parameters end (they come
        first in the interleaved layout)."""
        return self.pol.offsets["pi1.w"][0] if len(self.pol.net_arch) > 1 else \
            self.grad.numel()

    def _wgrad2(self, gz, x, out, defer=False):
        """out (2, N, K) = gz[j]^T x[j] for both MLPs in one batched split-K
        GEMM over 2C row chunks, then one fixed-order sum over the chunks
        (left to the deferred finish with defer)."""
        _, M, N = gz.shape
        Kd = x.shape[2]
        C = self.C
        if C == 1:
            torch.bmm(gz.transpose(1, 2), x, out=out)
            return
        ws = self._ws2[:2 * C * N * Kd].view(2 * C, N, Kd)
        rows = M // C
        if (x6_weights(self.pol, M) is not None and N == 256 and Kd == 256 and rows % 32 == 0
                and rows >= 32):
            from . import _lib
            _lib.check(_lib.lib().dr_gemm_x6_wgrad(
                2, M, C, gz.data_ptr(), x.data_ptr(), ws.data_ptr(),
                torch.cuda.current_stream(gz.device).cuda_stream))
        else:
            torch.bmm(gz.reshape(2 * C, rows, N).transpose(1, 2), x.reshape(2 * C, rows, Kd),
                      out=ws)
        if not defer:
            torch.sum(ws.view(2, C, N, Kd), dim=1, out=out)

    def can_defer(self) -> bool:
        """Whether step(defer_finish=True) covers every gradient entry (the
        2-hidden-layer actor-critic: head, first-layer and split-K chunk
        reductions are the whole flat gradient)."""
        return len(self.pol.net_arch) == 2

    @torch.no_grad()
    def step(self, obs, actions, aux, head, rows=None, on_ready=None, adv_ready=False,
             stats_out=None, defer_finish=False):
        """One PPO.train minibatch on the fused path: hidden forward
        (dr_linear_tanh2 for both first layers, one batched bias-free GEMM
        for both top layers -- addmm + tanh for any layer in between),
        dr_ppo_head_loss_backward (heads, loss, backward through the heads
        and top tanh, head / top-bias / log_std gradients), then for the
        layers above the first ONE batched split-K weight-gradient GEMM and
        ONE batched grad_h = grad_z W for pi and vf together (the flat
        layout keeps the two MLPs' tensors of a layer adjacent), tanh
        backward down the stack, and the first layer by
        dr_first_layer_backward (its grad_z is never stored).
        With `rows` (int32, m), obs / actions / aux are the whole rollout
        buffers and minibatch row r is their row rows[r] (no gather copies).
        `on_ready(lo, hi)` is called (depth >= 2) as soon as grad[lo:hi] --
        every parameter except the first layer's -- is final on the current
        stream, so a data-parallel caller can start that bucket's
        all-reduce while the first-layer backward still runs.
        `adv_ready` / `stats_out` are passed to the head (HeadLossBackward).
        With defer_finish (can_defer(), no on_ready) the last reductions of
        the head, the first layer and the split-K weight gradient are left
        for ONE launch inside ClipAdam.step_finish(grad, self.finish): the
        returned grad and stats are final only after that call.
        Returns (flat grad, stats (8))."""
        self._alloc_fused()
        pol, M = self.pol, (obs.shape[0] if rows is None else rows.numel())
        depth, top = len(pol.net_arch), len(pol.net_arch) - 1
        preact = depth >= 2                   # top tanh applied inside the head kernel
        if defer_finish and (not self.can_defer() or on_ready is not None):
            raise ValueError("defer_finish needs a 2-hidden-layer net and no on_ready")
        mark = self.mark or _no_mark
        self._first_rows = 0
        # the fused input-gradient GEMM + first-layer backward
        # (dr_gemm_x6_bwd_first): its observation image is built by the
        # first layer's forward launch
        fl = (defer_finish and rows is None and pol.gemm_x6_fl and pol.obs_dim == 15 and
              pol.net_arch == (256, 256) and x6_weights(pol, M) is not None)
        if fl:
            # the observation image is written for the minibatch's M rows
            # (by the first layer's launch or dr_gemm_x6_split_x) and read
            # for M rows by dr_gemm_x6_bwd_first: sized for M, which the
            # step's preallocated buffers fix at self.m (advisor r05)
            from . import _lib
            if M != self.m:
                raise ValueError(f"minibatch of {M} rows on a FusedTrainStep built for {self.m}")
            need = _lib.lib().dr_gemm_x6_x_bytes(M)
            if getattr(self, "_ximg", None) is None or self._ximg.numel() < need:
                self._ximg = torch.empty(need, dtype=torch.uint8, device=pol.device)
        fused_img = fl and pol.x6_fused_images
        hs = hidden_forward(pol, obs, self._acts, self._acts2, rows, top_preact=preact,
                            mark=self.mark, ximg=self._ximg if fused_img else None)
        gz = self._gz2[top]
        stats = head(hs["pi"][top], hs["vf"][top], pol.p("action.w"), pol.p("action.b"),
                     pol.p("value.w"), pol.p("value.b"), pol.log_std, actions, aux,
                     gz[0], gz[1], self.gview("action.w"),
                     self.gview("action.b"), self.gview("value.w"), self.gview("value.b"),
                     self.gview(f"pi{top}.b"), self.gview(f"vf{top}.b"),
                     self.gview("log_std"), rows, preact=preact, adv_ready=adv_ready,
                     stats_out=stats_out,
                     defer=(2 if pol.head_direct else 1) if defer_finish else 0,
                     **top_bias(pol, self._acts2))
        self._head_direct = bool(defer_finish and pol.head_direct)
        mark("ppo_head")
        if depth == 1:                        # the head kernel gave grad_z of layer 0
            if rows is not None:
                obs = obs.index_select(0, rows.long())
            for j, pre in enumerate(("pi", "vf")):
                self._wgrad(gz[j], obs, self.gview(f"{pre}0.w"))
            return self.grad, stats
        def fused_first(x):
            # grad_h1 never stored: the first layer's backward in the GEMM's
            # epilogue, its partials left in the first-layer workspace for the
            # deferred finish (dr_gemm_x6_bwd_first)
            from . import _lib
            xw = x6_weights(pol, M)
            st = torch.cuda.current_stream(pol.device).cuda_stream
            if not fused_img:
                xo = obs.to(torch.float32).contiguous()
                _lib.check(_lib.lib().dr_gemm_x6_split_x(M, 15, xo.data_ptr(),
                                                         self._ximg.data_ptr(), st))
                mark("split_x")
            direct = int(pol.gemm_x6_fl_direct)
            _lib.check(_lib.lib().dr_gemm_x6_bwd_first(
                2, M, 15, gz.data_ptr(), xw.bwd.data_ptr(), x.data_ptr(),
                self._ximg.data_ptr(), self._first.ws.data_ptr(), self._first.ws.numel(),
                direct, st))
            if direct:
                self._first_rows = _lib.lib().dr_gemm_x6_bwd_first_rows(M)
            mark("gemm_x6_bwd_first")

        for k in reversed(range(1, depth)):
            x = self._acts2[k - 1]
            n_in = x.shape[2]
            # fl_first: the fused kernel ahead of the weight gradient
            # (independent outputs: the same bytes either way)
            if k == 1 and fl and self.fl_first:
                fused_first(x)
            self._wgrad2(gz, x, pol.p2(k, "w", self.grad), defer=defer_finish)
            mark("gemm_x6_wgrad")
            if k == 1 and on_ready is not None:
                # all but the first layer's gradient is final from here on
                on_ready(self.first_layer_end(), self.grad.numel())
            g = self._g2.view(-1)[:2 * M * n_in].view(2, M, n_in)
            xw = x6_weights(pol, M) if k == 1 else None
            if k == 1 and fl:
                if not self.fl_first:
                    fused_first(x)
                continue
            if xw is not None:
                gemm_x6(gz, xw.bwd, g)       # images refreshed by hidden_forward
            else:
                torch.bmm(gz, pol.p2(k, "w"), out=g)
            mark("gemm_x6_bwd")
            if k == 1:
                # first layer of both MLPs: tanh backward + weight/bias
                # gradients fused, one launch
                self._first(obs, g[0], x[0], self.gview("pi0.w"), self.gview("pi0.b"),
                            g[1], x[1], self.gview("vf0.w"), self.gview("vf0.b"), rows,
                            defer=defer_finish)
                mark("first_layer_bwd")
            else:
                gz = self._gz2[k - 1]
                for j, pre in enumerate(("pi", "vf")):
                    self.K.tanh_backward(g[j], x[j], gz[j], self.gview(f"{pre}{k - 1}.b"),
                                         self.tanh_ws)
        if defer_finish:
            self._describe_finish(head, stats, M)
        return self.grad, stats

    def _describe_finish(self, head, stats, M):
        """Point self.finish (a GradFinish) at this step's deferred partials."""
        pol = self.pol
        if getattr(self, "finish", None) is None:
            self.finish = self.K.GradFinish()
        d = self.finish.desc
        gp = lambda name: self.gview(name).data_ptr()          # noqa: E731
        d.head_workspace, d.head_m, d.head_hd = head.ws.data_ptr(), head.m, head.hd
        d.log_std = pol.log_std.data_ptr()
        d.ent_coef, d.vf_coef = float(head.ent), float(head.vf)
        d.g_w_act, d.g_b_act = gp("action.w"), gp("action.b")
        d.g_w_val, d.g_b_val = gp("value.w"), gp("value.b")
        d.g_b_pi, d.g_b_vf, d.g_log_std = gp("pi1.b"), gp("vf1.b"), gp("log_std")
        d.stats = stats.data_ptr()
        d.first_workspace = self._first.ws.data_ptr()
        d.first_m, d.first_k, d.first_n = M, pol.obs_dim, pol.net_arch[0]
        d.first_rows = self._first_rows
        d.head_direct = int(self._head_direct)
        d.g_w0, d.g_b0, d.g_w1, d.g_b1 = gp("pi0.w"), gp("pi0.b"), gp("vf0.w"), gp("vf0.b")
        out = pol.p2(1, "w", self.grad)                        # (2, N, K), contiguous
        N, Kd = out.shape[1], out.shape[2]
        if self.C > 1:
            d.chunks, d.chunk_count = self._ws2.data_ptr(), self.C
        else:                        # the GEMM wrote the sums already: a 1-chunk pass
            d.chunks, d.chunk_count = out.data_ptr(), 1
        d.chunk_groups, d.chunk_size, d.chunk_dst = 2, N * Kd, out.data_ptr()

    @torch.no_grad()
    def forward(self, obs):
        pol = self.pol
        cache = {}
        outs = {}
        for pre, head in (("pi", "action"), ("vf", "value")):
            x, hs = obs, []
            for k in range(len(pol.net_arch)):
                h = torch.addmm(pol.p(f"{pre}{k}.b"), x, pol.p(f"{pre}{k}.w").t())
                torch.tanh_(h)
                hs.append(h)
                x = h
            outs[head] = torch.addmm(pol.p(f"{head}.b"), x, pol.p(f"{head}.w").t())
            cache[pre] = hs
        return outs["action"], outs["value"].squeeze(-1), cache

    def _wgrad(self, g, x, out):
        """out (N,K) = g^T x over M rows, split into C chunks."""
        M, N = g.shape
        Kd = x.shape[1]
        C = self.C
        ws = self._ws[:C * N * Kd].view(C, N, Kd)
        if C == 1:
            torch.mm(g.t(), x, out=out)
            return
        torch.bmm(g.reshape(C, M // C, N).transpose(1, 2), x.reshape(C, M // C, Kd),
                  out=ws)
        torch.sum(ws, dim=0, out=out)

    @torch.no_grad()
    def backward(self, obs, cache, g_mean, g_value, g_log_std):
        pol = self.pol
        M = obs.shape[0]
        for pre, head, gout in (("pi", "action", g_mean), ("vf", "value", g_value.view(M, 1))):
            hs = cache[pre]
            self._wgrad(gout, hs[-1], self.gview(f"{head}.w"))
            torch.sum(gout, dim=0, out=self.gview(f"{head}.b"))
            n = hs[-1].shape[1]
            g = self._g[:M * n].view(M, n)
            torch.mm(gout, pol.p(f"{head}.w"), out=g)
            for k in reversed(range(len(pol.net_arch))):
                h = hs[k]
                n = h.shape[1]
                gz = self._gz[:M * n].view(M, n)
                self.K.tanh_backward(g, h, gz, self.gview(f"{pre}{k}.b"), self.tanh_ws)
                x = hs[k - 1] if k > 0 else obs
                self._wgrad(gz, x, self.gview(f"{pre}{k}.w"))
                if k > 0:
                    g = self._g[:M * x.shape[1]].view(M, x.shape[1])
                    torch.mm(gz, pol.p(f"{pre}{k}.w"), out=g)
        self.gview("log_std").copy_(g_log_std)
        return self.grad


def fusable(pol: ActorCritic) -> bool:
    """The fused MLP kernels cover widths % 4 == 0 up to 256, the obs
    widths of dr_linear_tanh and the 4-d action head."""
    from .ppo_kernels import LINEAR_TANH_K
    return (all(n % 4 == 0 and n <= 256 for n in pol.net_arch) and
            pol.obs_dim in LINEAR_TANH_K and pol.act_dim == 4)


@torch.no_grad()
def hidden_forward(pol: ActorCritic, obs, acts, acts2=None, rows=None, top_preact=False,
                   mark=None, ximg=None):
    """Hidden activations of the pi and vf MLPs into preallocated buffers
    acts[pre][k] (M, net_arch[k]); with acts2 (the (2, M, n) buffers that
    acts views) each layer's tanh runs once over both MLPs; with rows the
    input rows are obs[rows].  With top_preact (and depth >= 2) the top
    layer is left as pre-activations z WITHOUT its bias: its only consumer,
    the head kernel, adds the bias and applies tanh on load (top_bias(pol)
    gives the pointers), so the (M, n) tanh pass is skipped and both MLPs'
    top GEMMs run as ONE batched GEMM (no bias epilogue; 125 us against
    2 x 74 us for two addmm at M = 65,536, MI355X-tuned solutions).
    On the x6 path the first layer's launch also re-splits the 256 x 256
    weights into their images (they may have changed since) and, with ximg,
    builds the fused input-gradient GEMM's observation image
    (dr_linear_tanh2_x6)."""
    from . import ppo_kernels as K
    mark = mark or _no_mark
    top = len(pol.net_arch) - 1
    xw = (x6_weights(pol, acts2[0].shape[1])
          if (top_preact and top == 1 and acts2 is not None and pol.obs_dim == 15 and
              pol.x6_fused_images) else None)
    if xw is not None:
        K.linear_tanh2_x6(obs, pol.p("pi0.w"), pol.p("pi0.b"), acts["pi"][0],
                          pol.p("vf0.w"), pol.p("vf0.b"), acts["vf"][0], pol.p2(1, "w"),
                          xw.img, ximg, rows)
    else:
        assert ximg is None
        K.linear_tanh2(obs, pol.p("pi0.w"), pol.p("pi0.b"), acts["pi"][0],
                       pol.p("vf0.w"), pol.p("vf0.b"), acts["vf"][0], rows)
    mark("linear_tanh")
    for k in range(1, len(pol.net_arch)):
        if top_preact and k == top and acts2 is not None:
            if k == 1 and xw is None:
                xw = x6_weights(pol, acts2[k - 1].shape[1])
                if xw is not None:
                    xw.refresh()             # the weights may have changed since
                    mark("split_weights")
            if xw is not None:
                gemm_x6(acts2[k - 1], xw.fwd, acts2[k])
                mark("gemm_x6_fwd")
            else:
                torch.bmm(acts2[k - 1], pol.p2(k, "w").transpose(1, 2), out=acts2[k])
            continue
        for pre in ("pi", "vf"):
            torch.addmm(pol.p(f"{pre}{k}.b"), acts[pre][k - 1], pol.p(f"{pre}{k}.w").t(),
                        out=acts[pre][k])
        if top_preact and k == len(pol.net_arch) - 1:
            continue
        if acts2 is not None:
            torch.tanh_(acts2[k])
        else:
            for pre in ("pi", "vf"):
                torch.tanh_(acts[pre][k])
    return acts


def _no_mark(name):
    pass


def top_bias(pol: ActorCritic, acts2) -> dict:
    """zb_pi / zb_vf kwargs for the head kernels after hidden_forward(...,
    acts2, top_preact=True): the top layer's biases (its batched GEMM left
    them out)."""
    if len(pol.net_arch) < 2 or acts2 is None:
        return {}
    top = len(pol.net_arch) - 1
    return {"zb_pi": pol.p(f"pi{top}.b"), "zb_vf": pol.p(f"vf{top}.b")}


class PolicyInference:
    """Rollout forward for a fixed batch of n observations on the fused
    kernels: returns (mean (n,4), value (n,)) in reused buffers.  Uses the
    same kernels as FusedTrainStep.step, so the rollout's log-probs and the
    first training epoch see identical network outputs."""

    def __init__(self, pol: ActorCritic, n: int):
        self.pol, self.n = pol, n
        f32 = dict(dtype=torch.float32, device=pol.device)
        self.acts2 = [torch.empty(2, n, w, **f32) for w in pol.net_arch]
        self.acts = {pre: [a[j] for a in self.acts2] for j, pre in enumerate(("pi", "vf"))}
        self.mean = torch.empty(n, pol.act_dim, **f32)
        self.value = torch.empty(n, **f32)

    @torch.no_grad()
    def __call__(self, obs):
        from . import ppo_kernels as K
        pol = self.pol
        preact = len(pol.net_arch) >= 2
        hs = hidden_forward(pol, obs, self.acts, self.acts2, top_preact=preact)
        K.policy_heads(hs["pi"][-1], hs["vf"][-1], pol.p("action.w"), pol.p("action.b"),
                       pol.p("value.w"), pol.p("value.b"), self.mean, self.value,
                       preact=preact, **top_bias(pol, self.acts2))
        return self.mean, self.value
