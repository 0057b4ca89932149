"""GPU-resident batch of quadrotor envs over libdronerl.so.

`DroneBatch` is the zero-copy torch path (every buffer is a device tensor,
all work is enqueued on the current HIP stream); `DroneGymEnv` mirrors the
reference's single-env gym class (/root/reference/drone.py:254-274) on top of
a one-env batch.  The SB3 / gymnasium vector facades live in vec_env.py.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

# Physical constants of the reference (drone.py:14-43, 263); exposed as
# attributes because callers read them (e.g. env.mass, env.g: drone.py:263,292).
DT = 0.02
MASS = 1.0
G = 9.81
INERTIA = (0.005, 0.005, 0.01)
ARM_LENGTH = 0.5
K_YAW = 0.01
MAX_STEPS = 200
MOTOR_MAX = 3 * MASS * G / 4.0          # 7.3575, action_space.high
OBS_DIM = {"gym": 15, "vectorized": 12, "moving": 18}
# reset uniforms per env and reset for rng="host" 
RESET_UNIFORMS = {"gym": 5, "vectorized": 5, "moving": 14}
_VARIANT_ID = {"gym": _lib.DR_VARIANT_GYM, "vectorized": _lib.DR_VARIANT_VECTORIZED,
               "moving": _lib.DR_VARIANT_MOVING}

_VEC_FIELDS = ("pos", "vel", "euler", "omega", "target")


def _stream(device):
    return torch.cuda.current_stream(device).cuda_stream


class DroneBatch:
    """N independent quadrotor envs in HBM (struct of arrays).

    variant    "gym" (DroneGymEnv, drone.py), "vectorized"
               (VectorizedDroneEnv, vectorized_drone.py) or "moving" (the
               moving-target curriculum of BASELINE configs[4]; 18-d obs)
    dtype      torch.float64 (reference precision) or torch.float32 state
    rng        "philox" (counter-based, seeded) or "host" (caller supplies
               the reset uniforms: numpy-MT19937 replay for parity tests)
    auto_reset DummyVecEnv semantics: a done env is reset inside the step
               and obs holds the reset observation.
    """

    def __init__(self, num_envs: int, variant: str = "gym",
                 dtype: torch.dtype = torch.float64, device=None, seed: int = 0,
                 auto_reset: bool = True, rng: str = "philox",
                 env_id_offset: int = 0, max_steps: int | None = None,
                 keep_terminal_obs: bool = False, monitor: bool = False):
        if variant not in OBS_DIM:
            raise ValueError(f"unknown variant {variant!r}")
        if dtype not in (torch.float64, torch.float32):
            raise ValueError("dtype must be torch.float64 or torch.float32")
        if rng not in ("philox", "host"):
            raise ValueError("rng must be 'philox' or 'host'")
        if not torch.cuda.is_available():
            raise RuntimeError("DroneBatch needs a HIP device (no CPU fallback)")
        self.L = _lib.lib()
        self.device = torch.device("cuda", torch.cuda.current_device()) \
            if device is None else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.variant = variant
        self.dtype = dtype
        self.obs_dim = OBS_DIM[variant]
        self.auto_reset = bool(auto_reset) and variant != "vectorized"
        self.monitor = monitor
        self.seed_value = int(seed)
        self.env_id_offset = int(env_id_offset)
        cfg = _lib.dr_config(
            num_envs=self.num_envs,
            variant=_VARIANT_ID[variant],
            state_dtype=_lib.DR_STATE_F64 if dtype == torch.float64 else _lib.DR_STATE_F32,
            rng_mode=_lib.DR_RNG_PHILOX if rng == "philox" else _lib.DR_RNG_HOST_UNIFORMS,
            auto_reset=int(self.auto_reset), device=self.device.index,
            max_steps=int(max_steps or 0), seed=self.seed_value & (2**64 - 1),
            env_id_offset=self.env_id_offset, dt=DT)
        h = ctypes.c_void_p()
        check(self.L.dr_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.handle = h
        self.max_steps = int(max_steps or (1000 if variant == "vectorized" else MAX_STEPS))
        n, od, dev = self.num_envs, self.obs_dim, self.device
        self.obs = torch.zeros(n, od, dtype=torch.float32, device=dev)
        self.rew = torch.zeros(n, dtype=torch.float32, device=dev)
        self.done = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.term_obs = torch.zeros(n, od, dtype=torch.float32, device=dev) \
            if keep_terminal_obs else None
        self.ep_ret = torch.zeros(n, dtype=torch.float32, device=dev) if monitor else None
        self.ep_len = torch.zeros(n, dtype=torch.int32, device=dev) if monitor else None
        self._uniforms = None

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.L.dr_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- core API ----------------------------------------------------------
    def reset(self, obs_out: torch.Tensor | None = None) -> torch.Tensor:
        out = self.obs if obs_out is None else obs_out
        self._check_out(out, (self.num_envs, self.obs_dim), torch.float32)
        check(self.L.dr_reset(self.handle, ptr(out), _stream(self.device)), self.handle)
        return out

    def reset_masked(self, mask: torch.Tensor, obs_out: torch.Tensor | None = None):
        out = self.obs if obs_out is None else obs_out
        mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        check(self.L.dr_reset_masked(self.handle, ptr(mask), ptr(out),
                                     _stream(self.device)), self.handle)
        return out

    def step(self, actions: torch.Tensor, obs_out=None, rew_out=None, done_out=None,
             trunc_out=None):
        """Advance every env one step.  `actions` (N,4) f32 on the device.
        Returns (obs, rew, done) device tensors (the batch's own buffers unless
        *_out are given: copy them before the next step if you keep them).
        `trunc_out` (N,) u8, monitor=True only: 1 where the episode ended at
        the step limit without a crash (dr_step_monitored_trunc)."""
        obs = self.obs if obs_out is None else obs_out
        rew = self.rew if rew_out is None else rew_out
        done = self.done if done_out is None else done_out
        a = actions
        if a.dtype != torch.float32 or a.device != self.device or not a.is_contiguous() \
                or a.data_ptr() % 16:
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        if a.shape != (self.num_envs, 4):
            raise ValueError(f"actions must be ({self.num_envs}, 4), got {tuple(a.shape)}")
        self._check_out(obs, (self.num_envs, self.obs_dim), torch.float32)
        self._check_out(rew, (self.num_envs,), torch.float32)
        self._check_out(done, (self.num_envs,), torch.uint8)
        s = _stream(self.device)
        if trunc_out is not None:
            if not self.monitor:
                raise ValueError("trunc_out needs a monitor=True batch")
            self._check_out(trunc_out, (self.num_envs,), torch.uint8)
            check(self.L.dr_step_monitored_trunc(self.handle, ptr(a), ptr(obs), ptr(rew),
                                                 ptr(done), ptr(self.term_obs), ptr(self.ep_ret),
                                                 ptr(self.ep_len), ptr(trunc_out), s),
                  self.handle)
        elif self.monitor:
            check(self.L.dr_step_monitored(self.handle, ptr(a), ptr(obs), ptr(rew), ptr(done),
                                           ptr(self.term_obs), ptr(self.ep_ret),
                                           ptr(self.ep_len), s), self.handle)
        else:
            check(self.L.dr_step(self.handle, ptr(a), ptr(obs), ptr(rew), ptr(done),
                                 ptr(self.term_obs), s), self.handle)
        return obs, rew, done

    def rollout(self, k: int, actions: torch.Tensor | None = None, *, seed: int = 0,
                step0: int = 0, lo: float = 0.0, hi: float = MOTOR_MAX,
                actions_out: torch.Tensor | None = None,
                obs_out=None, rew_out=None, done_out=None):
        """k steps in one launch (dr_rollout): outputs identical to k calls of
        step().  `actions` (k,N,4) f32 on the device, or None for the
        in-kernel random policy (step t draws random_actions(N, seed, step0+t,
        env_id_offset, lo, hi); `actions_out` (k,N,4) receives them if given).
        Returns (obs (k,N,obs_dim), rew (k,N), done (k,N)); no terminal obs or
        VecMonitor counters (use step() for those).  Refused on a monitor=True
        batch: the launch does not advance the running episode return /
        length, so a later step() would report wrong episodes."""
        if self.monitor:
            raise ValueError("rollout() on a monitor=True batch would leave the VecMonitor "
                             "episode counters stale; use step() or a monitor=False batch")
        k = int(k)
        n, od, dev = self.num_envs, self.obs_dim, self.device
        obs = torch.empty(k, n, od, dtype=torch.float32, device=dev) if obs_out is None else obs_out
        rew = torch.empty(k, n, dtype=torch.float32, device=dev) if rew_out is None else rew_out
        done = torch.empty(k, n, dtype=torch.uint8, device=dev) if done_out is None else done_out
        self._check_out(obs, (k, n, od), torch.float32)
        self._check_out(rew, (k, n), torch.float32)
        self._check_out(done, (k, n), torch.uint8)
        s = _stream(dev)
        if actions is None:
            if actions_out is not None:
                self._check_out(actions_out, (k, n, 4), torch.float32)
            check(self.L.dr_rollout_random(self.handle, k, seed & (2**64 - 1), step0, lo, hi,
                                           ptr(actions_out), ptr(obs), ptr(rew), ptr(done), s),
                  self.handle)
        else:
            a = actions
            if a.dtype != torch.float32 or a.device != dev or not a.is_contiguous() \
                    or a.data_ptr() % 16:
                a = a.to(device=dev, dtype=torch.float32).contiguous()
            if a.shape != (k, n, 4):
                raise ValueError(f"actions must be ({k}, {n}, 4), got {tuple(a.shape)}")
            check(self.L.dr_rollout(self.handle, k, ptr(a), ptr(obs), ptr(rew), ptr(done), s),
                  self.handle)
        return obs, rew, done

    # -- host-buffer I/O (the drop-in surfaces) ------------------------------
    def _host_buffers(self):
        """Pinned host buffers the kernels read / write directly (zero-copy
        over PCIe): a host-buffer step is one launch and one stream sync, no
        separate H2D / D2H copies."""
        hb = getattr(self, "_hb", None)
        if hb is None:
            n, od = self.num_envs, self.obs_dim
            pin = dict(device="cpu", pin_memory=True)
            f32 = dict(dtype=torch.float32, **pin)
            hb = {"act": torch.zeros(n, 4, **f32), "obs": torch.zeros(n, od, **f32),
                  "rew": torch.zeros(n, **f32),
                  "done": torch.zeros(n, dtype=torch.uint8, **pin),
                  "term": torch.zeros(n, od, **f32) if self.term_obs is not None else None,
                  "ep_ret": torch.zeros(n, **f32) if self.monitor else None,
                  "ep_len": torch.zeros(n, dtype=torch.int32, **pin) if self.monitor else None}
            hb["np"] = {k: (v.numpy() if v is not None else None) for k, v in hb.items()}
            self._hb = hb
        return hb

    def reset_host(self) -> np.ndarray:
        """reset() into a pinned host buffer; returns a numpy view of it
        (overwritten by the next host-buffer call: copy to keep)."""
        hb = self._host_buffers()
        check(self.L.dr_reset(self.handle, ptr(hb["obs"]), _stream(self.device)), self.handle)
        torch.cuda.current_stream(self.device).synchronize()
        return hb["np"]["obs"]

    def step_host(self, actions):
        """step() with host buffers: `actions` any (N,4)-shaped array-like;
        the kernel reads them from, and writes obs / rew / done (and, when
        kept, the terminal obs and VecMonitor outputs of done rows) to, pinned
        host memory.  Returns the numpy views {"obs", "rew", "done", "term",
        "ep_ret", "ep_len"}, valid until the next host-buffer call."""
        hb = self._host_buffers()
        a = np.asarray(actions, dtype=np.float32)
        if a.size != self.num_envs * 4:
            raise ValueError(f"actions must be ({self.num_envs}, 4), got {a.shape}")
        np.copyto(hb["np"]["act"], a.reshape(self.num_envs, 4))
        s = _stream(self.device)
        if self.monitor:
            check(self.L.dr_step_monitored(self.handle, ptr(hb["act"]), ptr(hb["obs"]),
                                           ptr(hb["rew"]), ptr(hb["done"]), ptr(hb["term"]),
                                           ptr(hb["ep_ret"]), ptr(hb["ep_len"]), s),
                  self.handle)
        else:
            check(self.L.dr_step(self.handle, ptr(hb["act"]), ptr(hb["obs"]), ptr(hb["rew"]),
                                 ptr(hb["done"]), ptr(hb["term"]), s), self.handle)
        torch.cuda.current_stream(self.device).synchronize()
        return hb["np"]

    # -- state access ------------------------------------------------------
    def _field_out(self, field: str, **where) -> torch.Tensor:
        n = self.num_envs
        if field in _VEC_FIELDS:
            return torch.empty(n, 3, dtype=torch.float64, **where)
        if field == "eps":
            return torch.empty(n, dtype=torch.float64, **where)
        if field == "ep_return":
            return torch.empty(n, dtype=torch.float32, **where)
        if field == "motion":
            return torch.empty(n, 9, dtype=torch.float32, **where)
        return torch.empty(n, dtype=torch.int32, **where)

    def get(self, field: str) -> torch.Tensor:
        fid = _lib.FIELDS[field]
        out = self._field_out(field, device=self.device)
        check(self.L.dr_get_state(self.handle, fid, ptr(out), _stream(self.device)), self.handle)
        return out

    def get_host(self, field: str) -> np.ndarray:
        """get(field) as a fresh numpy array: the field kernel writes into a
        pinned host buffer (one launch + one sync, no D2H copy)."""
        fid = _lib.FIELDS[field]
        bufs = self.__dict__.setdefault("_field_host", {})
        out = bufs.get(field)
        if out is None:
            out = bufs[field] = self._field_out(field, device="cpu", pin_memory=True)
        check(self.L.dr_get_state(self.handle, fid, ptr(out), _stream(self.device)), self.handle)
        torch.cuda.current_stream(self.device).synchronize()
        return out.numpy().copy()

    def gather(self, field: str, env_ids: torch.Tensor, out: torch.Tensor | None = None):
        """`get(field)` for the envs in env_ids (int32 device tensor), into
        `out` if given (k,3) f64 / (k,) / (k,9) f32 for "motion"."""
        fid = _lib.FIELDS[field]
        k = env_ids.numel()
        if out is None:
            if field in _VEC_FIELDS:
                out = torch.empty(k, 3, dtype=torch.float64, device=self.device)
            elif field == "eps":
                out = torch.empty(k, dtype=torch.float64, device=self.device)
            elif field == "ep_return":
                out = torch.empty(k, dtype=torch.float32, device=self.device)
            elif field == "motion":
                out = torch.empty(k, 9, dtype=torch.float32, device=self.device)
            else:
                out = torch.empty(k, dtype=torch.int32, device=self.device)
        ids = env_ids.to(device=self.device, dtype=torch.int32).contiguous()
        check(self.L.dr_gather_state(self.handle, fid, ptr(ids), k, ptr(out),
                                     _stream(self.device)), self.handle)
        return out

    def set(self, field: str, value) -> None:
        fid = _lib.FIELDS[field]
        if field in _VEC_FIELDS:
            dt, shape = torch.float64, (self.num_envs, 3)
        elif field == "eps":
            dt, shape = torch.float64, (self.num_envs,)
        elif field == "ep_return":
            dt, shape = torch.float32, (self.num_envs,)
        elif field == "motion":
            dt, shape = torch.float32, (self.num_envs, 9)
        else:
            dt, shape = torch.int32, (self.num_envs,)
        v = torch.as_tensor(value, dtype=dt).to(self.device).reshape(shape).contiguous()
        check(self.L.dr_set_state(self.handle, fid, ptr(v), _stream(self.device)), self.handle)
        torch.cuda.current_stream(self.device).synchronize()   # v may be freed

    def seed(self, seed: int) -> None:
        """New Philox key for every later reset (order-free per env)."""
        self.seed_value = int(seed)
        check(self.L.dr_set_seed(self.handle, self.seed_value & (2**64 - 1)), self.handle)

    def set_reset_uniforms(self, u) -> None:
        """rng='host': (N,5) f64 uniforms ((N,14) for "moving") consumed by
        the next resets."""
        t = torch.as_tensor(u, dtype=torch.float64).to(self.device).reshape(
            self.num_envs, RESET_UNIFORMS[self.variant]).contiguous()
        self._uniforms = t          # keep alive while kernels may read it
        check(self.L.dr_set_reset_uniforms(self.handle, ptr(t)), self.handle)

    @staticmethod
    def _check_out(t, shape, dtype):
        if t.dtype != dtype or tuple(t.shape) != shape or not t.is_contiguous():
            raise ValueError(f"output buffer must be contiguous {dtype} {shape}")


def random_actions(n: int, seed: int, step: int, env_id_offset: int = 0,
                   lo: float = 0.0, hi: float = MOTOR_MAX, out=None, device=None):
    """Synthetic random policy: (n,4) f32 i.i.d. U[lo,hi) (Philox)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    if out is None:
        out = torch.empty(n, 4, dtype=torch.float32, device=dev)
    check(_lib.lib().dr_random_actions(n, seed & (2**64 - 1), env_id_offset, step, lo, hi,
                                       ptr(out), _stream(out.device)))
    return out


class _Box:
    """Minimal gym.spaces.Box stand-in (gym/gymnasium are optional)."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)
        self._rng = np.random.default_rng()

    def sample(self):
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return self._rng.uniform(lo, hi).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def make_box(low, high, shape, dtype=np.float32):
    """gymnasium.spaces.Box if importable, then gym's, else a stand-in."""
    for mod in ("gymnasium", "gym"):
        try:
            spaces = __import__(mod + ".spaces", fromlist=["Box"])
            return spaces.Box(low=low, high=high, shape=shape, dtype=dtype)
        except Exception:
            continue
    return _Box(low, high, shape, dtype)


class DroneGymEnv:
    """Single-env drop-in for the reference's DroneGymEnv (drone.py:254-274),
    backed by a one-env GPU batch with raw (non-auto-reset) semantics:
    reset() -> obs (15,) f32; step(a) -> (obs, reward float, done bool, {})."""

    metadata = {"render_modes": []}

    def __init__(self, dt: float = DT, device=None, seed: int | None = None,
                 dtype: torch.dtype = torch.float64):
        if dt != DT:
            raise ValueError("only the reference dt=0.02 is supported")
        seed = int(np.random.randint(0, 2**31 - 1)) if seed is None else seed
        self._b = DroneBatch(1, "gym", dtype=dtype, device=device, seed=seed,
                             auto_reset=False)
        self.mass, self.g, self.dt = MASS, G, DT
        self.I = np.array(INERTIA)
        self.arm_length, self.k_yaw, self.max_steps = ARM_LENGTH, K_YAW, MAX_STEPS
        self.observation_space = make_box(-np.inf, np.inf, (15,), np.float32)
        self.action_space = make_box(0, MOTOR_MAX, (4,), np.float32)

    def reset(self):
        return self._b.reset_host()[0].copy()

    def step(self, action):
        # one launch + one sync: the kernel reads the action from and writes
        # its outputs to pinned host memory (DroneBatch.step_host)
        o = self._b.step_host(np.asarray(action, np.float32).reshape(1, 4))
        return (o["obs"][0].copy(), float(o["rew"][0]), bool(o["done"][0]), {})

    def _vec(self, f):
        return self._b.get_host(f)[0]

    pos = property(lambda self: self._vec("pos"))
    vel = property(lambda self: self._vec("vel"))
    euler = property(lambda self: self._vec("euler"))
    omega = property(lambda self: self._vec("omega"))
    target = property(lambda self: self._vec("target"))
    current_step = property(lambda self: int(self._b.get_host("current_step")[0]))
    ep_num = property(lambda self: int(self._b.get_host("ep_num")[0]))
    eps = property(lambda self: float(self._b.get_host("eps")[0]))

    # ---- recording (drone.py:189-248; test.py:9-21) -------------------------
    def _recorder(self):
        if getattr(self, "_rec", None) is None:
            from .render import DroneRecorder
            self._rec = DroneRecorder()
        return self._rec

    def start_record(self, filename="drone_run.mp4", dpi=200, fps=20, bitrate=-1):
        """Start a GIF (PillowWriter) of the frames render() draws."""
        self._recorder().start_record(filename, dpi=dpi, fps=fps, bitrate=bitrate)

    def stop_record(self):
        """Finish and save the recording."""
        self._recorder().stop_record()

    def render(self, mode="human", close=False, ax=None):
        """DroneGymEnv.render(mode="human", close=False) (drone.py:273-274):
        draw the drone (motors, arms, centre) and the target in 3-D from the
        device state; grabs a frame when recording.  `mode` and `close` are
        accepted as the reference accepts them (it ignores both); `ax` is this
        build's optional target axes.  Returns the (4, 3) motor positions."""
        return self._recorder().render(self.pos, self.euler, self.target, self.arm_length, ax)

    def close(self):
        if getattr(self, "_rec", None) is not None:
            self._rec.close()
        self._b.close()
