"""Vector-env facades over the GPU batch: SB3 `VecEnv` and gymnasium-style.

The reference trains through
    DummyVecEnv([lambda: DroneGymEnv()]) -> VecMonitor     (train.py:33-35)
and its callback reads `training_env.get_attr('pos')[0]` and
`locals["dones"][0]` (traj_tb.py:34,38).  `BatchedDroneVecEnv` is a drop-in
for that whole stack: the SB3 `VecEnv` surface (reset / step_async /
step_wait / get_attr / set_attr / env_method / seed / env_is_wrapped /
close), DummyVecEnv's same-step auto-reset with
`infos[i]["terminal_observation"]` and `"TimeLimit.truncated": False` (the
reference env goes through shimmy's GymV21 compat, which reports the
200-step limit as termination), and VecMonitor's
`infos[i]["episode"] = {"r", "l", "t"}` with f32 running returns.

Throughput does not come from here -- SB3 builds one info dict per env per
step in Python; at scale use DroneBatch.step (device tensors) or
drone_rl_amd.ppo.  Neither gym nor SB3 needs to be installed: when
stable_baselines3 is importable the class derives from its VecEnv so
`isinstance` checks inside SB3 pass.
"""
from __future__ import annotations

import itertools
import time

import numpy as np
import torch

from .env import (ARM_LENGTH, DT, G, INERTIA, K_YAW, MASS, MOTOR_MAX, DroneBatch,
                  make_box)

try:  # optional: let SB3's isinstance(env, VecEnv) checks pass
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except Exception:  # noqa: BLE001 - SB3 absent (this image)
    _VecEnvBase = object

_STATE = ("pos", "vel", "euler", "omega", "target")
_SCALAR = {"current_step": int, "ep_num": int, "eps": float}


_INFO_TEMPLATE = {"TimeLimit.truncated": False}


class BatchedDroneVecEnv(_VecEnvBase):
    """N DroneGymEnv envs on one GPU behind the SB3 VecEnv API."""

    def __init__(self, num_envs: int = 1, variant: str = "gym",
                 dtype: torch.dtype = torch.float64, device=None, seed: int | None = None,
                 monitor: bool = True, rng: str = "philox", env_id_offset: int = 0):
        if seed is None:
            seed = int(np.random.randint(0, 2**31 - 1))
        self.batch = DroneBatch(num_envs, variant, dtype=dtype, device=device, seed=seed,
                                auto_reset=(variant != "vectorized"), rng=rng,
                                env_id_offset=env_id_offset, keep_terminal_obs=True,
                                monitor=True)
        self._monitor = monitor
        od = self.batch.obs_dim
        obs_space = make_box(-np.inf, np.inf, (od,), np.float32)
        act_space = make_box(0, MOTOR_MAX, (4,), np.float32)
        if _VecEnvBase is not object:
            super().__init__(num_envs, obs_space, act_space)
        else:
            self.num_envs = num_envs
            self.observation_space = obs_space
            self.action_space = act_space
        self.render_mode = None
        self._actions = None
        self._t_start = time.time()
        self._consts = {"mass": MASS, "g": G, "dt": DT, "I": np.array(INERTIA),
                        "arm_length": ARM_LENGTH, "k_yaw": K_YAW,
                        "max_steps": self.batch.max_steps,
                        "observation_space": obs_space, "action_space": act_space}

    # ------------------------------------------------------------- stepping
    def reset(self):
        return self.batch.reset_host().copy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        # one launch + one sync: the kernel reads the actions from and writes
        # obs / rewards / dones / terminal rows to pinned host memory
        o = self.batch.step_host(self._actions)
        obs_np = o["obs"].copy()
        rew_np = o["rew"].copy()
        done_np = o["done"].astype(bool)
        # one dict per env (SB3 semantics); copying a template is the
        # cheapest way to build N of them in CPython
        infos = list(map(dict.copy, itertools.repeat(_INFO_TEMPLATE, self.num_envs)))
        idx = np.nonzero(done_np)[0]
        if len(idx):
            if self.batch.auto_reset:
                term = o["term"][idx]
            else:
                term = obs_np[idx]
            if self._monitor:
                ret = o["ep_ret"][idx]
                ln = o["ep_len"][idx]
                t = round(time.time() - self._t_start, 6)
            for j, i in enumerate(idx):
                if self.batch.auto_reset:
                    infos[i]["terminal_observation"] = term[j]
                if self._monitor:
                    infos[i]["episode"] = {"r": np.float32(ret[j]), "l": int(ln[j]), "t": t}
        return obs_np, rew_np, done_np, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    # ------------------------------------------------------------ attributes
    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    def get_attr(self, attr_name, indices=None):
        idx = self._indices(indices)
        if attr_name in _STATE:
            v = self.batch.get_host(attr_name)
            return [v[i].copy() for i in idx]
        if attr_name in _SCALAR:
            v = self.batch.get_host(attr_name)
            return [_SCALAR[attr_name](v[i]) for i in idx]
        if attr_name in self._consts:
            return [self._consts[attr_name] for _ in idx]
        raise AttributeError(f"DroneGymEnv has no attribute {attr_name!r}")

    def set_attr(self, attr_name, value, indices=None):
        idx = self._indices(indices)
        if attr_name not in _STATE and attr_name not in _SCALAR:
            raise AttributeError(f"cannot set {attr_name!r} on the GPU env")
        cur = self.batch.get(attr_name).cpu().numpy().copy()
        for i in idx:
            cur[i] = value
        self.batch.set(attr_name, cur)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = self._indices(indices)
        if method_name == "reset":
            mask = torch.zeros(self.num_envs, dtype=torch.uint8)
            mask[idx] = 1
            obs = self.batch.reset_masked(mask).cpu().numpy()
            return [obs[i].copy() for i in idx]
        if method_name in ("get_wrapper_attr", "getattr"):
            return self.get_attr(method_args[0], idx)
        if method_name == "render":
            return [None for _ in idx]
        raise AttributeError(f"unsupported env_method {method_name!r}")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def seed(self, seed: int | None = None):
        if seed is None:
            seed = int(np.random.randint(0, 2**31 - 1))
        self.batch.seed(seed)
        return [seed + i for i in range(self.num_envs)]

    def get_images(self):
        raise NotImplementedError("rendering is out of scope (SURVEY.md 2 #11)")

    def render(self, mode: str | None = None):
        return None

    def close(self):
        self.batch.close()


class DroneVectorEnv:
    """gymnasium-1.x-style vector facade (same-step autoreset).

    reset(seed=None, options=None) -> (obs (N,15) f32, infos dict)
    step(actions) -> (obs, rewards f32, terminated bool, truncated bool, infos)

    terminated/truncated follow the reference as shimmy converts it: the
    old-API `done` (crash OR 200-step limit, drone.py:154-157) is reported as
    `terminated`, `truncated` is all False.  With `split_time_limit=True`,
    an episode that ended at the step limit without a crash is reported as
    truncated instead (crash judged on the f32 terminal obs).  For done envs
    infos carries "final_obs" / "final_info" / "_final_obs" masks, and
    "episode" {"r","l"} arrays like gymnasium's RecordEpisodeStatistics.
    `as_tensors=True` returns device tensors instead of numpy arrays.
    """

    metadata = {"autoreset_mode": "SameStep"}

    def __init__(self, num_envs: int, device=None, seed: int = 0,
                 dtype: torch.dtype = torch.float64, split_time_limit: bool = False,
                 as_tensors: bool = False):
        self.batch = DroneBatch(num_envs, "gym", dtype=dtype, device=device, seed=seed,
                                auto_reset=True, keep_terminal_obs=True, monitor=True)
        self.num_envs = num_envs
        self.single_observation_space = make_box(-np.inf, np.inf, (15,), np.float32)
        self.single_action_space = make_box(0, MOTOR_MAX, (4,), np.float32)
        self.observation_space = make_box(-np.inf, np.inf, (num_envs, 15), np.float32)
        self.action_space = make_box(0, MOTOR_MAX, (num_envs, 4), np.float32)
        self.split_time_limit = split_time_limit
        self.as_tensors = as_tensors

    def _out(self, t):
        return t if self.as_tensors else t.cpu().numpy().copy()

    def reset(self, seed: int | None = None, options=None):
        if seed is not None:
            self.batch.seed(seed)
        return self._out(self.batch.reset()), {}

    def step(self, actions):
        a = actions if torch.is_tensor(actions) else torch.as_tensor(
            np.asarray(actions, dtype=np.float32))
        obs, rew, done = self.batch.step(a.to(self.batch.device))
        d = done.bool()
        infos = {}
        if self.split_time_limit:
            t = self.batch.term_obs
            crash = (t[:, 2] < 0) | (torch.linalg.vector_norm(t[:, :3], dim=1) > 50)
            trunc = d & (self.batch.ep_len >= self.batch.max_steps) & ~crash
            term = d & ~trunc
        else:
            term, trunc = d, torch.zeros_like(d)
        if bool(d.any()):
            infos["final_obs"] = self._out(torch.where(d[:, None], self.batch.term_obs, 0))
            infos["_final_obs"] = self._out(d)
            infos["episode"] = {"r": self._out(torch.where(d, self.batch.ep_ret, 0)),
                                "l": self._out(torch.where(d, self.batch.ep_len, 0))}
            infos["_episode"] = self._out(d)
        return self._out(obs), self._out(rew), self._out(term), self._out(trunc), infos

    def close(self):
        self.batch.close()
