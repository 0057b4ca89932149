"""Generate the golden parity fixtures from the reference implementation.

RUNS ONLY IN THE BUILD CONTAINER (it imports /root/reference, which never
travels to the GPU box).  It writes plain data (.npz: inputs and the
reference's outputs) next to this file; no reference source is copied.

The reference imports `gym` (drone.py:2-3, vectorized_drone.py:2-3), which is
not installed here, so a minimal stand-in providing `gym.Env` and
`gym.spaces.Box` is placed in sys.modules first.
`vectorized_drone` is imported before `drone` because its
`matplotlib.use('TkAgg')` (vectorized_drone.py:5) must run before pyplot loads.

Fixtures (all compressed npz):
  gym_step.npz   one-step DroneGymEnv transitions (drone.py:81-159), sampled
                 along trajectories of several policies plus synthetic edge
                 states (near-gimbal, huge unwrapped angles, crash / distance
                 thresholds, the step-199 time limit).
  gym_reset.npz  DroneEnv.reset draws and curriculum (drone.py:48-75).
  gym_traj.npz   16 envs stepped DummyVecEnv-style (serial, auto-reset on
                 done, one shared np.random stream) with the uniforms each
                 reset consumed, for multi-step replay through the GPU.
  gym_drift.npz  200-step open-loop trajectories (drift characterisation).
  vec_step.npz   VectorizedDroneEnv one-step batches (vectorized_drone.py:135-216).
  vec_traj.npz   VectorizedDroneEnv 300-step trajectory, B=32.

Usage:  python tests/golden/make_golden.py [/root/reference]
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
A_MAX = np.float32(3 * 1.0 * 9.81 / 4.0)


def _install_gym_stub():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Env:
        def __init__(self):
            pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    gym.Env = Env
    spaces.Box = Box
    gym.spaces = spaces
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces


def _import_reference():
    _install_gym_stub()
    sys.path.insert(0, REF)
    import vectorized_drone  # noqa: E402  (must precede drone / pyplot)
    import drone  # noqa: E402
    return drone, vectorized_drone


class DrawLog:
    """Records every np.random.rand() draw (the reference's only RNG use)."""

    def __init__(self):
        self.orig = np.random.rand
        self.log = []

    def __enter__(self):
        def rec(*a):
            v = self.orig(*a)
            self.log.append(float(v))
            return v
        np.random.rand = rec
        return self

    def __exit__(self, *exc):
        np.random.rand = self.orig


def _snap(env):
    return dict(pos=env.pos.copy(), vel=env.vel.copy(), euler=env.euler.copy(),
                omega=env.omega.copy(), target=env.target.copy(),
                step=env.current_step)


def _set(env, s):
    env.pos = np.array(s["pos"], dtype=np.float64)
    env.vel = np.array(s["vel"], dtype=np.float64)
    env.euler = np.array(s["euler"], dtype=np.float64)
    env.omega = np.array(s["omega"], dtype=np.float64)
    env.target = np.array(s["target"], dtype=np.float64)
    env.current_step = int(s["step"])


# --------------------------------------------------------------------------
# gym variant, one-step transitions
# --------------------------------------------------------------------------
def gen_gym_step(drone, rng):
    env = drone.DroneGymEnv()
    rows = {k: [] for k in ["pos", "vel", "euler", "omega", "target", "step",
                            "action", "o_obs", "o_rew", "o_done", "o_pos",
                            "o_vel", "o_euler", "o_omega", "o_step", "kind"]}

    def record(action, kind):
        s = _snap(env)
        obs, rew, done, info = env.step(action)
        assert info == {}
        for k in ["pos", "vel", "euler", "omega", "target", "step"]:
            rows[k].append(s[k])
        rows["action"].append(action.copy())
        rows["o_obs"].append(obs)
        rows["o_rew"].append(float(rew))
        rows["o_done"].append(bool(done))
        rows["o_pos"].append(env.pos.copy())
        rows["o_vel"].append(env.vel.copy())
        rows["o_euler"].append(env.euler.copy())
        rows["o_omega"].append(env.omega.copy())
        rows["o_step"].append(env.current_step)
        rows["kind"].append(kind)
        return done

    hover = np.float32(9.81 / 4.0)
    # (0) uniform random policy U[0, a_max)^4 (what SB3 clipping produces)
    np.random.seed(0)
    env.reset()
    for _ in range(4000):
        a = rng.uniform(0, A_MAX, 4).astype(np.float32)
        if record(a, 0):
            env.reset()
    # (1) near-hover with noise: long episodes, time-limit terminations
    np.random.seed(1)
    env.reset()
    for _ in range(2600):
        a = np.clip(hover + rng.normal(0, 0.05, 4), 0, A_MAX).astype(np.float32)
        if record(a, 1):
            env.reset()
    # (2) spinners: differential thrust -> large, unwrapped Euler angles
    np.random.seed(2)
    env.reset()
    spin = [np.array([3.0, 2.0, 3.0, 2.0], np.float32),
            np.array([2.0, 3.5, 2.5, 1.8], np.float32),
            np.array([4.0, 1.0, 1.2, 3.9], np.float32)]
    for i in range(1800):
        a = (spin[(i // 200) % 3] + rng.normal(0, 0.2, 4)).astype(np.float32)
        a = np.clip(a, 0, A_MAX).astype(np.float32)
        if record(a, 2):
            env.reset()
    # (3) synthetic edge states
    for i in range(1600):
        s = dict(pos=rng.uniform(-2, 2, 3), vel=rng.normal(0, 2, 3),
                 euler=rng.normal(0, 1, 3), omega=rng.normal(0, 5, 3),
                 target=rng.uniform(-1, 1, 3) + np.array([0, 0, 1.0]),
                 step=int(rng.integers(0, 200)))
        sub = i % 8
        if sub == 0:    # near gimbal lock |cos(theta)| < 1e-3
            s["euler"][1] = np.pi / 2 * rng.choice([-1, 1]) + rng.uniform(-1e-3, 1e-3)
        elif sub == 1:  # huge unwrapped angles
            s["euler"] = rng.uniform(-1.3e4, 1.3e4, 3)
            s["omega"] = rng.normal(0, 60, 3)
        elif sub == 2:  # crash boundary z ~ 0
            s["pos"][2] = rng.uniform(0.0, 0.02)
            s["vel"][2] = rng.normal(-0.5, 0.5)
        elif sub == 3:  # distance boundary ||p|| ~ 50
            d = rng.normal(size=3)
            d[2] = abs(d[2])
            s["pos"] = d / np.linalg.norm(d) * rng.uniform(49.9, 50.1)
        elif sub == 4:  # time limit
            s["step"] = 199
        elif sub == 5:  # at the target (bonus radius 0.05)
            s["pos"] = s["target"] + rng.normal(0, 0.03, 3)
            s["vel"] = rng.normal(0, 0.2, 3)
        elif sub == 6:  # far away, fast
            s["pos"] = rng.uniform(-40, 40, 3)
            s["vel"] = rng.normal(0, 20, 3)
        _set(env, s)
        a = rng.uniform(0, A_MAX, 4).astype(np.float32)
        if sub == 7:    # exact action extremes
            a = rng.choice(np.array([0.0, A_MAX], np.float32), 4)
        record(a, 3)

    out = {}
    for k, v in rows.items():
        arr = np.array(v)
        if k in ("step", "o_step", "kind"):
            arr = arr.astype(np.int32)
        out[k] = arr
    out["action"] = out["action"].astype(np.float32)
    out["o_obs"] = out["o_obs"].astype(np.float32)
    return out


# --------------------------------------------------------------------------
# gym variant, reset draws + curriculum
# --------------------------------------------------------------------------
def gen_gym_reset(drone, rng):
    env = drone.DroneGymEnv()
    ep_in, eps_in, us, o = [], [], [], {k: [] for k in
                                        ["pos", "target", "eps", "ep_num", "obs"]}
    cases = []
    for ep in [0, 1, 2, 3, 100, 1997, 1998, 1999, 2000, 3998, 3999, 5999,
               19999, 39999, 123456, 199999]:
        cases.append(ep)
    cases += list(rng.integers(0, 10**6, 200))
    for k, ep in enumerate(cases):
        eps = float(rng.choice([0.0, 0.1, 0.2, 0.30000000000000004, 1.5, 9.9]))
        if k % 3 == 0:  # eps reached by repeated f64 addition (drone.py:70)
            eps = 0.0
            for _ in range(int(ep) // 2000):
                eps += 0.1
        env.ep_num, env.eps = int(ep), eps
        with DrawLog() as dl:
            obs = env.reset()
        assert len(dl.log) == 5
        ep_in.append(int(ep))
        eps_in.append(eps)
        us.append(dl.log)
        o["pos"].append(env.pos.copy())
        o["target"].append(env.target.copy())
        o["eps"].append(env.eps)
        o["ep_num"].append(env.ep_num)
        o["obs"].append(obs)
    return dict(ep_num=np.array(ep_in, np.int64), eps=np.array(eps_in),
                u=np.array(us), o_pos=np.array(o["pos"]),
                o_target=np.array(o["target"]), o_eps=np.array(o["eps"]),
                o_ep_num=np.array(o["ep_num"], np.int64),
                o_obs=np.array(o["obs"], np.float32))


# --------------------------------------------------------------------------
# gym variant, DummyVecEnv-style multi-env trajectory with auto-reset
# --------------------------------------------------------------------------
def gen_gym_traj(drone, rng, n_envs=16, n_steps=256):
    np.random.seed(1234)
    with DrawLog() as dl:
        envs = [drone.DroneGymEnv() for _ in range(n_envs)]   # ctor: 1 reset each
        ctor_u = np.array(dl.log).reshape(n_envs, 5)
        dl.log.clear()
        obs0 = np.stack([e.reset() for e in envs])             # VecEnv.reset
        reset_u = np.array(dl.log).reshape(n_envs, 5)
        dl.log.clear()
        st = {k: np.stack([getattr(e, k) for e in envs]) for k in
              ["pos", "vel", "euler", "omega", "target"]}
        st["step"] = np.array([e.current_step for e in envs], np.int32)
        st["ep_num"] = np.array([e.ep_num for e in envs], np.int64)
        st["eps"] = np.array([e.eps for e in envs])
        acts = rng.uniform(0, A_MAX, (n_steps, n_envs, 4)).astype(np.float32)
        # a few envs fly near-hover so that the 200-step limit is reached
        hover = np.float32(9.81 / 4.0)
        acts[:, :3] = np.clip(hover + rng.normal(0, 0.02, (n_steps, 3, 4)), 0,
                              A_MAX).astype(np.float32)
        obs = np.zeros((n_steps, n_envs, 15), np.float32)
        term = np.full((n_steps, n_envs, 15), np.nan, np.float32)
        rew = np.zeros((n_steps, n_envs))
        done = np.zeros((n_steps, n_envs), bool)
        ru = np.full((n_steps, n_envs, 5), np.nan)
        # full f64 pre-step state, so a replay can re-synchronise every step
        pre = {k: np.zeros((n_steps, n_envs, 3)) for k in
               ["pos", "vel", "euler", "omega", "target"]}
        pre_step = np.zeros((n_steps, n_envs), np.int32)
        for t in range(n_steps):
            for i, e in enumerate(envs):
                for k in pre:
                    pre[k][t, i] = getattr(e, k)
                pre_step[t, i] = e.current_step
                o, r, d, _ = e.step(acts[t, i])
                rew[t, i], done[t, i] = r, d
                if d:
                    term[t, i] = o
                    dl.log.clear()
                    o = e.reset()
                    ru[t, i] = dl.log
                    dl.log.clear()
                obs[t, i] = o
        final_ep = np.array([e.ep_num for e in envs], np.int64)
        final_eps = np.array([e.eps for e in envs])
    return dict(ctor_u=ctor_u, reset_u=reset_u, obs0=obs0, actions=acts,
                obs=obs, term_obs=term, reward=rew, done=done, reset_uniforms=ru,
                final_ep_num=final_ep, final_eps=final_eps, pre_step=pre_step,
                **{"pre_" + k: v for k, v in pre.items()},
                **{"s0_" + k: v for k, v in st.items()})


def gen_gym_drift(drone):
    np.random.seed(7)
    seqs = []
    hover = np.float32(9.81 / 4.0)
    base = [np.full(4, hover, np.float32), np.full(4, hover * 2, np.float32),
            np.array([2.5, 2.4, 2.5, 2.4], np.float32),
            np.array([2.46, 2.45, 2.44, 2.45], np.float32)]
    obs = np.zeros((len(base), 200, 15), np.float32)
    rew = np.zeros((len(base), 200))
    done = np.zeros((len(base), 200), bool)
    s0 = []
    for k, a in enumerate(base):
        env = drone.DroneGymEnv()
        env.reset()
        s0.append(_snap(env))
        for t in range(200):
            o, r, d, _ = env.step(a)
            obs[k, t], rew[k, t], done[k, t] = o, r, d
        seqs.append(a)
    return dict(actions=np.array(seqs), obs=obs, reward=rew, done=done,
                s0_pos=np.array([s["pos"] for s in s0]),
                s0_target=np.array([s["target"] for s in s0]))


# --------------------------------------------------------------------------
# vectorized variant
# --------------------------------------------------------------------------
def gen_vec_step(vd, rng, B=64, n_batches=40):
    env = vd.VectorizedDroneEnv(batch_size=B)
    keys = ["pos", "vel", "euler", "omega"]
    rows = {k: [] for k in keys + ["step", "action", "o_obs", "o_rew", "o_done",
                                   "o_pos", "o_vel", "o_euler", "o_omega"]}
    env.reset()
    for b in range(n_batches):
        if b % 10 == 9:   # synthetic states incl. huge angles / gimbal / limit
            env.pos = rng.uniform(-3, 3, (B, 3))
            env.pos[: B // 4, 2] = rng.uniform(0, 0.02, B // 4)
            env.vel = rng.normal(0, 2, (B, 3))
            env.euler = rng.normal(0, 1, (B, 3))
            env.euler[B // 4: B // 2] = rng.uniform(-1e4, 1e4, (B // 4, 3))
            env.euler[B // 2: B // 2 + 8, 1] = np.pi / 2 + rng.uniform(-1e-3, 1e-3, 8)
            env.omega = rng.normal(0, 5, (B, 3))
            env.current_step = 999 if b == 19 else int(rng.integers(0, 999))
        s = {k: getattr(env, k).copy() for k in keys}
        step = env.current_step
        a = rng.uniform(0, A_MAX, (B, 4)).astype(np.float32)
        if b % 4 == 1:
            a = np.clip(np.float32(9.81 / 4.0) + rng.normal(0, 0.3, (B, 4)),
                        0, A_MAX).astype(np.float32)
        obs, rew, done, _ = env.step(a)
        for k in keys:
            rows[k].append(s[k])
            rows["o_" + k].append(getattr(env, k).copy())
        rows["step"].append(np.full(B, step, np.int32))
        rows["action"].append(a)
        rows["o_obs"].append(obs)
        rows["o_rew"].append(rew)
        rows["o_done"].append(done)
        if b % 10 == 8:
            env.reset()
    out = {k: np.concatenate(v) for k, v in rows.items()}
    out["batch"] = np.int32(B)
    return out


def gen_vec_traj(vd, rng, B=32, T=300):
    env = vd.VectorizedDroneEnv(batch_size=B)
    obs0 = env.reset()
    acts = rng.uniform(0, A_MAX, (T, B, 4)).astype(np.float32)
    acts[:, : B // 2] = np.clip(np.float32(9.81 / 4.0 * 1.02) +
                                rng.normal(0, 0.01, (T, B // 2, 4)), 0,
                                A_MAX).astype(np.float32)
    obs = np.zeros((T, B, 12), np.float32)
    rew = np.zeros((T, B))
    done = np.zeros((T, B), bool)
    for t in range(T):
        obs[t], rew[t], done[t], _ = env.step(acts[t])
    return dict(obs0=obs0, actions=acts, obs=obs, reward=rew, done=done)


def main():
    drone, vd = _import_reference()
    rng = np.random.default_rng(20250620)
    meta = dict(numpy_version=np.__version__)
    outs = {
        "gym_step.npz": gen_gym_step(drone, rng),
        "gym_reset.npz": gen_gym_reset(drone, rng),
        "gym_traj.npz": gen_gym_traj(drone, rng),
        "gym_drift.npz": gen_gym_drift(drone),
        "vec_step.npz": gen_vec_step(vd, rng),
        "vec_traj.npz": gen_vec_traj(vd, rng),
    }
    for name, d in outs.items():
        d = dict(d)
        d["numpy_version"] = np.array(meta["numpy_version"])
        path = os.path.join(HERE, name)
        np.savez_compressed(path, **d)
        print(f"{name}: {os.path.getsize(path) / 1024:.0f} KiB",
              {k: v.shape for k, v in d.items() if hasattr(v, 'shape')})


if __name__ == "__main__":
    main()
