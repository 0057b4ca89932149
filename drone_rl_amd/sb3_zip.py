"""stable-baselines3 ``.zip`` checkpoints <-> the GPU trainer (SURVEY.md 8f
rank 2; reference call sites /root/reference/train.py:10-31 ``PPO.load``,
:70 ``model.save``; test.py:7 ``PPO.load('./dd.zip', env=env)``).

Layout written and read (SB3 ``save_util.save_to_zip_file``):

  data                    JSON of the algorithm's attributes; plain values
                          as JSON, objects as {":type:", ":serialized:"
                          base64 pickle}
  policy.pth              torch.save(policy.state_dict())
  policy.optimizer.pth    torch.save(Adam.state_dict()), params in SB3's
                          ``policy.parameters()`` order
  pytorch_variables.pth   torch.save({})
  _stable_baselines3_version, system_info.txt
  dronerl_env_state.npz   (extra; SB3 ignores non-.pth members) the per-env
                          curriculum (ep_num, eps) that SB3's zip does not
                          keep (drone.py:18,33)

Reading is SAFE by construction: only ``data``'s plain JSON values and the
``.pth`` members through ``torch.load(weights_only=True)`` are used; the
pickled entries of ``data`` are never unpickled.

Writing: the four pickled entries SB3 needs to rebuild the model are emitted
by a small opcode assembler (no SB3 / gymnasium import needed): a global
reference to ``stable_baselines3.common.policies.ActorCriticPolicy`` and two
``gymnasium.spaces.Box`` instances built from ``numpy.array`` / ``numpy.dtype``
calls (stable names across numpy 1.x / 2.x).  ``learning_rate`` and
``clip_range`` are stored as floats, which SB3's ``_setup_model`` turns into
schedules.  Target: SB3 2.x with gymnasium.  Parity unpinned: SB3 is not
installed here, so the round trip is checked against this module's own
reader and the opcodes against the standard library's pickle machinery
with stand-in classes (tests/test_sb3_zip.py).
"""
from __future__ import annotations

import base64
import io
import json
import platform
import struct
import zipfile

import numpy as np
import torch

from .policy import ActorCritic, _sb3_name

SB3_VERSION = "2.3.2"

# ----------------------------------------------------------------- naming


def sb3_param_order(depth: int):
    """SB3 ActorCriticPolicy.parameters() order: the policy's own parameter
    (log_std) first, then submodules in registration order: mlp_extractor
    (policy_net, value_net Sequentials), action_net, value_net."""
    names = ["log_std"]
    for net in ("policy_net", "value_net"):
        for k in range(depth):
            names += [f"mlp_extractor.{net}.{2 * k}.weight", f"mlp_extractor.{net}.{2 * k}.bias"]
    names += ["action_net.weight", "action_net.bias", "value_net.weight", "value_net.bias"]
    return names


# ------------------------------------------------------- pickle assembler
class _P:
    """Minimal protocol-2 pickle writer for globals, tuples, dicts, strings,
    floats, ints, bools and None (enough for SB3's data entries)."""

    def __init__(self):
        self.b = bytearray(b"\x80\x02")

    def glob(self, module, name):
        self.b += b"c" + module.encode() + b"\n" + name.encode() + b"\n"

    def obj(self, v):
        b = self.b
        if v is None:
            b += b"N"
        elif v is True:
            b += b"\x88"
        elif v is False:
            b += b"\x89"
        elif isinstance(v, int):
            b += b"J" + struct.pack("<i", v)
        elif isinstance(v, float):
            b += b"G" + struct.pack(">d", v)
        elif isinstance(v, str):
            e = v.encode()
            b += b"X" + struct.pack("<I", len(e)) + e
        elif isinstance(v, tuple):
            b += b"("
            for x in v:
                self.obj(x)
            b += b"t"
        elif isinstance(v, list):
            b += b"]("
            for x in v:
                self.obj(x)
            b += b"e"
        elif isinstance(v, dict):
            b += b"}("
            for k, x in v.items():
                self.obj(k)
                self.obj(x)
            b += b"u"
        elif callable(v):
            v(self)
        else:
            raise TypeError(type(v))

    def call(self, module, name, args):
        """module.name(*args) via REDUCE."""
        def emit(p):
            p.glob(module, name)
            p.obj(tuple(args))
            p.b += b"R"
        return emit

    def done(self):
        return bytes(self.b + b".")


def _np_array(values, dtype):
    return _P().call("numpy", "array", [list(map(float, values)), dtype])


def _box_pickle(low, high, dtype="float32"):
    """gymnasium.spaces.Box(low, high, dtype) as Box.__new__ + BUILD(state);
    Box.__setstate__ fills the repr fields, Space.__setstate__ the rest."""
    low = np.asarray(low, np.float64)
    high = np.asarray(high, np.float64)
    n = low.size
    state = {
        "dtype": _P().call("numpy", "dtype", [dtype]),
        "_shape": (n,),
        "low": _np_array(low, dtype),
        "high": _np_array(high, dtype),
        "bounded_below": _P().call("numpy", "array", [[bool(np.isfinite(x)) for x in low]]),
        "bounded_above": _P().call("numpy", "array", [[bool(np.isfinite(x)) for x in high]]),
        "_np_random": None,
    }
    p = _P()
    p.glob("gymnasium.spaces.box", "Box")
    p.b += b")\x81"             # EMPTY_TUPLE, NEWOBJ -> Box.__new__(Box)
    p.obj(state)
    p.b += b"b"                 # BUILD -> __setstate__(state)
    return p.done()


def _global_pickle(module, name):
    p = _P()
    p.glob(module, name)
    return p.done()


def _ser(type_str, payload: bytes):
    return {":type:": type_str, ":serialized:": base64.b64encode(payload).decode()}


# ---------------------------------------------------------------- writing
def save(trainer, path):
    """Write ``trainer`` (drone_rl_amd.ppo.PPOTrainer) as an SB3 PPO zip."""
    cfg = trainer.cfg
    pol = trainer.policy
    depth = len(pol.net_arch)
    sd = pol.state_dict()
    order = sb3_param_order(depth)
    policy_sd = {k: sd[k] for k in order}
    # Adam state in SB3's parameter order
    inv = {_sb3_name(n, depth): n for n, _, _ in pol.layout}
    m = trainer.opt.m.detach().cpu()
    v = trainer.opt.v.detach().cpu()
    state = {}
    for idx, k in enumerate(order):
        a, b, shape = pol.offsets[inv[k]]
        state[idx] = {"step": torch.tensor(float(trainer.opt.t)),
                      "exp_avg": m[a:b].view(shape).clone(),
                      "exp_avg_sq": v[a:b].view(shape).clone()}
    opt_sd = {"state": state if trainer.opt.t > 0 else {},
              "param_groups": [{"lr": float(cfg.learning_rate), "betas": (0.9, 0.999),
                                "eps": 1e-5, "weight_decay": 0, "amsgrad": False,
                                "maximize": False, "foreach": None, "capturable": False,
                                "differentiable": False, "fused": None,
                                "params": list(range(len(order)))}]}
    od = pol.obs_dim
    data = {
        "policy_class": _ser("<class 'abc.ABCMeta'>",
                             _global_pickle("stable_baselines3.common.policies",
                                            "ActorCriticPolicy")),
        "verbose": 1,
        "policy_kwargs": {"net_arch": list(cfg.net_arch),
                          "log_std_init": float(cfg.log_std_init)}
        if tuple(cfg.net_arch) != (64, 64) or cfg.log_std_init != 0.0 else {},
        "num_timesteps": int(trainer.num_timesteps),
        "_total_timesteps": int(trainer.num_timesteps),
        "_num_timesteps_at_start": 0,
        "seed": int(cfg.seed),
        "action_noise": None,
        "learning_rate": float(cfg.learning_rate),
        "tensorboard_log": None,
        "_episode_num": 0,
        "use_sde": False,
        "sde_sample_freq": -1,
        "_current_progress_remaining": 1.0,
        "_stats_window_size": 100,
        "_n_updates": int(trainer.num_updates * cfg.n_epochs),
        "observation_space": _ser("<class 'gymnasium.spaces.box.Box'>",
                                  _box_pickle([-np.inf] * od, [np.inf] * od)),
        "action_space": _ser("<class 'gymnasium.spaces.box.Box'>",
                             _box_pickle([0.0] * 4, [7.3575] * 4)),
        "n_envs": int(cfg.num_envs) * int(trainer.world),
        "n_steps": int(cfg.n_steps),
        "gamma": float(cfg.gamma),
        "gae_lambda": float(cfg.gae_lambda),
        "ent_coef": float(cfg.ent_coef),
        "vf_coef": float(cfg.vf_coef),
        "max_grad_norm": float(cfg.max_grad_norm),
        "batch_size": int(cfg.batch_size),
        "n_epochs": int(cfg.n_epochs),
        "clip_range": float(cfg.clip_range),
        "clip_range_vf": None,
        "normalize_advantage": bool(cfg.normalize_advantage),
        "target_kl": None,
    }
    env = {k: trainer.env.get(k).cpu().numpy() for k in ("ep_num", "eps")}

    def tbytes(obj):
        buf = io.BytesIO()
        torch.save(obj, buf)
        return buf.getvalue()

    with zipfile.ZipFile(path, "w", compression=zipfile.ZIP_DEFLATED) as z:
        z.writestr("data", json.dumps(data, indent=4))
        z.writestr("policy.pth", tbytes(policy_sd))
        z.writestr("policy.optimizer.pth", tbytes(opt_sd))
        z.writestr("pytorch_variables.pth", tbytes({}))
        z.writestr("_stable_baselines3_version", SB3_VERSION)
        z.writestr("system_info.txt",
                   f"- OS: {platform.platform()}\n- Python: {platform.python_version()}\n"
                   f"- Stable-Baselines3: {SB3_VERSION} (layout; written by drone_rl_amd)\n"
                   f"- PyTorch: {torch.__version__}\n- Numpy: {np.__version__}\n")
        buf = io.BytesIO()
        np.savez(buf, **env)
        z.writestr("dronerl_env_state.npz", buf.getvalue())


# ---------------------------------------------------------------- reading
def read(path):
    """Parse an SB3 PPO zip without unpickling anything.  Returns dict with
    ``data`` (plain JSON values only), ``policy`` (state dict), ``optimizer``
    (state dict or None) and ``env`` (curriculum arrays or None)."""
    out = {"data": {}, "policy": None, "optimizer": None, "env": None}
    with zipfile.ZipFile(path) as z:
        names = z.namelist()
        if "data" in names:
            raw = json.loads(z.read("data").decode())
            out["data"] = {k: v for k, v in raw.items()
                           if not (isinstance(v, dict) and ":serialized:" in v)}
        for member, key in (("policy.pth", "policy"), ("policy.optimizer.pth", "optimizer")):
            if member in names:
                out[key] = torch.load(io.BytesIO(z.read(member)), map_location="cpu",
                                      weights_only=True)
        if "dronerl_env_state.npz" in names:
            with np.load(io.BytesIO(z.read("dronerl_env_state.npz"))) as f:
                out["env"] = {k: f[k] for k in f.files}
    if out["policy"] is None:
        raise ValueError(f"{path}: no policy.pth member (not an SB3 checkpoint)")
    return out


def infer_net_arch(policy_sd):
    """Hidden sizes of the pi MLP from an SB3 policy state dict."""
    arch, k = [], 0
    while f"mlp_extractor.policy_net.{2 * k}.weight" in policy_sd:
        arch.append(int(policy_sd[f"mlp_extractor.policy_net.{2 * k}.weight"].shape[0]))
        k += 1
    return tuple(arch)


def load_into(trainer, path, load_env_state=True):
    """Resume ``trainer`` from an SB3 zip: parameters, Adam moments/step
    (when present and shaped like ours), timestep counter and, if the zip
    was written by ``save``, the per-env curriculum."""
    ck = read(path)
    pol = trainer.policy
    depth = len(pol.net_arch)
    if infer_net_arch(ck["policy"]) != tuple(pol.net_arch):
        raise ValueError(f"net_arch mismatch: checkpoint {infer_net_arch(ck['policy'])} "
                         f"vs trainer {tuple(pol.net_arch)}")
    pol.load_state_dict(ck["policy"])
    opt = ck["optimizer"]
    if opt and opt.get("state"):
        inv = {_sb3_name(n, depth): n for n, _, _ in pol.layout}
        order = sb3_param_order(depth)
        with torch.no_grad():
            step = 0
            for idx, k in enumerate(order):
                st = opt["state"].get(idx)
                if st is None:
                    continue
                a, b, _ = pol.offsets[inv[k]]
                trainer.opt.m[a:b].copy_(st["exp_avg"].reshape(-1).to(trainer.opt.m.device))
                trainer.opt.v[a:b].copy_(st["exp_avg_sq"].reshape(-1).to(trainer.opt.v.device))
                step = int(float(st["step"]))
            trainer.opt.t = step
    trainer.num_timesteps = int(ck["data"].get("num_timesteps", 0))
    # SB3 counts optimizer passes (_n_updates = iterations x n_epochs); the
    # trainer's iteration count keys the policy-noise and permutation Philox
    # streams and the eps_schedule, so a resumed run continues them instead
    # of replaying the first iterations' streams and curriculum steps
    trainer.num_updates = int(ck["data"].get("_n_updates", 0)) // max(trainer.cfg.n_epochs, 1)
    if load_env_state and ck["env"] is not None and \
            len(ck["env"]["ep_num"]) == trainer.env.num_envs:
        trainer.env.set("ep_num", ck["env"]["ep_num"])
        trainer.env.set("eps", ck["env"]["eps"])
    return ck


def load_policy(path, device=None):
    """An ActorCritic from an SB3 PPO zip, for inference (test.py:7-13:
    ``PPO.load('./dd.zip')`` then ``predict(obs, deterministic=True)``)."""
    ck = read(path)
    sd = ck["policy"]
    arch = infer_net_arch(sd)
    obs_dim = int(sd["mlp_extractor.policy_net.0.weight"].shape[1])
    act_dim = int(sd["action_net.weight"].shape[0])
    pol = ActorCritic(obs_dim, act_dim, arch, device)
    pol.load_state_dict(sd)
    return pol
