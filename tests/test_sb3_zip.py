"""SB3 .zip checkpoint interop (drone_rl_amd/sb3_zip.py), CPU only.

stable-baselines3 is not installed: parity with SB3 itself is
unpinned.  Checked here: the member layout, that the reader never needs to
unpickle, the save -> read -> load round trip of parameters / Adam state /
curriculum, SB3's parameter order for the optimizer state, and that the
hand-assembled pickles of `data` decode with the standard pickle machinery
into the intended calls (stand-in classes registered for the test only)."""
import json
import pickle
import pickletools
import sys
import types
import zipfile
from dataclasses import dataclass

import base64
import numpy as np
import pytest
import torch

from drone_rl_amd import sb3_zip
from drone_rl_amd.policy import ActorCritic


@dataclass
class _Cfg:
    num_envs: int = 8
    n_steps: int = 16
    batch_size: int = 64
    n_epochs: int = 10
    learning_rate: float = 3e-4
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_range: float = 0.2
    ent_coef: float = 0.0
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    normalize_advantage: bool = True
    net_arch: tuple = (64, 64)
    log_std_init: float = 0.0
    seed: int = 3


class _Opt:
    def __init__(self, n, t):
        g = torch.Generator().manual_seed(t)
        self.m = torch.randn(n, generator=g)
        self.v = torch.rand(n, generator=g)
        self.t = t


class _Env:
    def __init__(self, n):
        self.num_envs = n
        self.f = {"ep_num": torch.arange(n, dtype=torch.int32) * 7,
                  "eps": torch.linspace(0, 0.7, n, dtype=torch.float64)}

    def get(self, k):
        return self.f[k]

    def set(self, k, v):
        self.f[k] = torch.as_tensor(v)


class _Trainer:
    def __init__(self, seed, t):
        self.cfg = _Cfg()
        self.policy = ActorCritic(15, 4, self.cfg.net_arch, "cpu", seed=seed)
        self.opt = _Opt(self.policy.num_params, t)
        self.env = _Env(self.cfg.num_envs)
        self.num_timesteps, self.num_updates, self.world = 12345, 7, 1


def test_roundtrip(tmp_path):
    a = _Trainer(seed=1, t=5)
    path = tmp_path / "dd.zip"
    sb3_zip.save(a, path)
    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        data = json.loads(z.read("data"))
    assert {"data", "policy.pth", "policy.optimizer.pth", "pytorch_variables.pth",
            "_stable_baselines3_version", "system_info.txt"} <= names
    assert data["n_steps"] == 16 and data["learning_rate"] == 3e-4 and data["clip_range"] == 0.2
    assert data["policy_kwargs"] == {}
    ck = sb3_zip.read(path)
    assert "observation_space" not in ck["data"]            # pickled entries skipped
    order = sb3_zip.sb3_param_order(2)
    assert list(ck["policy"].keys()) == order
    assert ck["optimizer"]["param_groups"][0]["params"] == list(range(len(order)))
    st0 = ck["optimizer"]["state"][0]                        # log_std first
    assert st0["exp_avg"].shape == (4,) and float(st0["step"]) == 5.0
    b = _Trainer(seed=2, t=0)
    assert not torch.equal(a.policy.flat, b.policy.flat)
    sb3_zip.load_into(b, path)
    assert torch.equal(a.policy.flat, b.policy.flat)
    assert torch.equal(a.opt.m, b.opt.m) and torch.equal(a.opt.v, b.opt.v) and b.opt.t == 5
    assert b.num_timesteps == 12345
    assert torch.equal(torch.as_tensor(b.env.get("eps")), a.env.get("eps"))
    pol = sb3_zip.load_policy(path)
    obs = np.random.default_rng(0).normal(size=(5, 15)).astype(np.float32)
    act, _ = pol.predict(obs)
    mean, _ = a.policy.forward(torch.from_numpy(obs))
    np.testing.assert_allclose(act, mean.clamp(0, 7.3575).detach().numpy(), rtol=1e-6)
    assert pol.predict(obs[0])[0].shape == (4,)


def test_net_arch_mismatch_rejected(tmp_path):
    a = _Trainer(seed=1, t=1)
    sb3_zip.save(a, tmp_path / "a.zip")
    b = _Trainer(seed=1, t=1)
    b.policy = ActorCritic(15, 4, (256, 256), "cpu")
    with pytest.raises(ValueError, match="net_arch"):
        sb3_zip.load_into(b, tmp_path / "a.zip")


def test_data_pickles_decode(tmp_path, monkeypatch):
    """The assembled opcodes are valid pickles that rebuild
    ActorCriticPolicy (by reference) and gymnasium Box instances."""
    class Box:
        def __setstate__(self, state):
            self.state = state

    class ActorCriticPolicy:
        pass

    for name, attrs in (("gymnasium", {}), ("gymnasium.spaces", {}),
                        ("gymnasium.spaces.box", {"Box": Box}),
                        ("stable_baselines3", {}), ("stable_baselines3.common", {}),
                        ("stable_baselines3.common.policies",
                         {"ActorCriticPolicy": ActorCriticPolicy})):
        mod = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(mod, k, v)
        monkeypatch.setitem(sys.modules, name, mod)
    Box.__module__, ActorCriticPolicy.__module__ = "gymnasium.spaces.box", \
        "stable_baselines3.common.policies"
    a = _Trainer(seed=1, t=1)
    sb3_zip.save(a, tmp_path / "a.zip")
    with zipfile.ZipFile(tmp_path / "a.zip") as z:
        data = json.loads(z.read("data"))
    raw = {k: base64.b64decode(data[k][":serialized:"])
           for k in ("policy_class", "observation_space", "action_space")}
    for v in raw.values():
        pickletools.dis(v, out=open("/dev/null", "w"))
    assert pickle.loads(raw["policy_class"]) is ActorCriticPolicy
    obs = pickle.loads(raw["observation_space"])
    act = pickle.loads(raw["action_space"])
    assert isinstance(obs, Box) and obs.state["_shape"] == (15,)
    assert obs.state["low"].dtype == np.float32 and np.isneginf(obs.state["low"]).all()
    assert obs.state["dtype"] == np.dtype("float32") and not obs.state["bounded_below"].any()
    np.testing.assert_array_equal(act.state["high"], np.full(4, 7.3575, np.float32))
    assert act.state["bounded_above"].all() and act.state["_np_random"] is None
