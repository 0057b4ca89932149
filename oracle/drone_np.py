"""NumPy restatement of the reference env -- TEST INFRASTRUCTURE ONLY.

* `GymDronePort`: one env with the reference's per-step numpy cost profile
  (3-vectors, a 3x3 matmul for the Euler rates, np.linalg.norm), used as the
  per-env worker of the CPU baseline (a SubprocVecEnv-equivalent process pool,
  bench.py) -- the reference's own CPU path is DummyVecEnv over DroneGymEnv
  (/root/reference/train.py:33-35, drone.py:81-159).
* `gym_step_batched`: the same step over (n,3) arrays (numpy-batched form,
  in the style of /root/reference/vectorized_drone.py:135-216).

Both follow SURVEY.md Appendix A op for op (f32 thrust/torque sums, f32 yaw
torque under NEP 50, R from the old Euler angles, semi-implicit v->p, Euler
rates and omega from the old omega).  Pinned by tests/test_oracle.py.
"""
import numpy as np

DT = 0.02
G = 9.81
MASS = 1.0
INERTIA = np.array([0.005, 0.005, 0.01])
ARM = 0.5
K_YAW = 0.01
MAX_STEPS = 200
A_MAX = 3 * MASS * G / 4.0
_FACTOR = ARM / np.sqrt(2)


class GymDronePort:
    """Single DroneGymEnv-equivalent env (drone.py:13-159) on numpy f64."""

    def __init__(self, rng=None):
        self.rng = rng if rng is not None else np.random.default_rng()
        self.ep_num = 0
        self.eps = 0.0
        self.reset()

    def _draw(self):
        return float(self.rng.random())

    def reset(self, u=None):
        """drone.py:48-75; `u` = the 5 uniforms in draw order (optional)."""
        u = [self._draw() for _ in range(5)] if u is None else list(u)
        self.pos = np.array([u[0] - 0.5, u[1] - 0.5, 1.0])
        self.vel = np.zeros(3)
        self.euler = np.zeros(3)
        self.omega = np.zeros(3)
        self.ep_num += 1
        self.current_step = 0
        if self.ep_num % 2000 == 0:
            self.eps += 0.1
        self.target = np.array([self.eps * u[2], self.eps * u[3],
                                self.eps * u[4] + 1.0 + 0])
        return self.obs()

    def obs(self):
        return np.concatenate([self.pos, self.vel, self.euler, self.omega,
                               self.target - self.pos]).astype(np.float32)

    def step(self, action):
        f = np.asarray(action, dtype=np.float32)
        thrust = f[0] + f[1] + f[2] + f[3]
        tau = (_FACTOR * (f[0] + f[1] - f[2] - f[3]),
               _FACTOR * (-f[0] + f[1] + f[2] - f[3]),
               K_YAW * (f[0] - f[1] + f[2] - f[3]))
        ph, th, ps = self.euler
        cph, sph, cth, sth = np.cos(ph), np.sin(ph), np.cos(th), np.sin(th)
        cps, sps = np.cos(ps), np.sin(ps)
        zcol = np.array([cps * sth * cph + sps * sph,
                         sps * sth * cph - cps * sph,
                         cth * cph])
        accel = np.array([0.0, 0.0, -G]) + zcol * np.float64(thrust) / MASS
        self.vel += accel * DT
        self.pos += self.vel * DT
        tth = np.tan(th)
        W = np.array([[1.0, sph * tth, cph * tth],
                      [0.0, cph, -sph],
                      [0.0, sph / cth, cph / cth]])
        w = self.omega
        I = INERTIA
        wdot = np.array([(tau[0] - (I[1] - I[2]) * w[1] * w[2]) / I[0],
                         (tau[1] - (I[2] - I[0]) * w[0] * w[2]) / I[1],
                         (tau[2] - (I[0] - I[1]) * w[0] * w[1]) / I[2]])
        self.euler += (W @ w) * DT
        self.omega += wdot * DT
        d = np.linalg.norm(self.pos - self.target)
        reward = 0.01 * -d + (1.0 if d < 0.05 else 0.0)
        done = bool(self.pos[2] < 0 or np.linalg.norm(self.pos) > 50)
        self.current_step += 1
        if self.current_step >= MAX_STEPS:
            done = True
        return self.obs(), float(reward), done, {}


def gym_step_batched(s, action):
    """Batched DroneEnv.step on a dict of (n,3) f64 arrays (mutated) and (n,)
    i32 'step'.  Returns obs (n,15) f32, reward (n,) f64, done (n,) bool."""
    a = np.asarray(action, dtype=np.float32)
    a0, a1, a2, a3 = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
    thrust = ((a0 + a1) + a2) + a3                      # f32
    tau_phi = _FACTOR * (((a0 + a1) - a2) - a3)         # f64
    tau_th = _FACTOR * (((-a0 + a1) + a2) - a3)
    tau_psi = np.float32(K_YAW) * (((a0 - a1) + a2) - a3)  # f32
    e = s["euler"]
    cph, sph = np.cos(e[:, 0]), np.sin(e[:, 0])
    cth, sth = np.cos(e[:, 1]), np.sin(e[:, 1])
    cps, sps = np.cos(e[:, 2]), np.sin(e[:, 2])
    T = thrust.astype(np.float64)
    acc = np.stack([0.0 + (cps * sth * cph + sps * sph) * T / MASS,
                    0.0 + (sps * sth * cph - cps * sph) * T / MASS,
                    -G + (cth * cph) * T / MASS], axis=1)
    s["vel"] += acc * DT
    s["pos"] += s["vel"] * DT
    w = s["omega"].copy()
    tth = np.tan(e[:, 1])
    ed = np.stack([w[:, 0] + (sph * tth) * w[:, 1] + (cph * tth) * w[:, 2],
                   0.0 * w[:, 0] + cph * w[:, 1] + (-sph) * w[:, 2],
                   0.0 * w[:, 0] + (sph / cth) * w[:, 1] + (cph / cth) * w[:, 2]],
                  axis=1)
    s["euler"] += ed * DT
    I = INERTIA
    wd = np.stack([(tau_phi - (I[1] - I[2]) * w[:, 1] * w[:, 2]) / I[0],
                   (tau_th - (I[2] - I[0]) * w[:, 0] * w[:, 2]) / I[1],
                   (tau_psi.astype(np.float64) - (I[0] - I[1]) * w[:, 0] * w[:, 1]) / I[2]],
                  axis=1)
    s["omega"] += wd * DT
    dv = s["pos"] - s["target"]
    d = np.sqrt((dv[:, 0] * dv[:, 0] + dv[:, 1] * dv[:, 1]) + dv[:, 2] * dv[:, 2])
    rew = 0.01 * -d + np.where(d < 0.05, 1.0, 0.0)
    p = s["pos"]
    pn = np.sqrt((p[:, 0] * p[:, 0] + p[:, 1] * p[:, 1]) + p[:, 2] * p[:, 2])
    s["step"] = s["step"] + 1
    done = (p[:, 2] < 0) | (pn > 50) | (s["step"] >= MAX_STEPS)
    obs = np.concatenate([s["pos"], s["vel"], s["euler"], s["omega"],
                          s["target"] - s["pos"]], axis=1).astype(np.float32)
    return obs, rew, done
