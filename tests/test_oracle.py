"""Pin the CPU oracle to the reference's golden vectors (CPU only).

The golden fixtures were produced by the reference itself
(tests/golden/make_golden.py imports /root/reference/drone.py and
vectorized_drone.py).  Two restatements are checked:
  oracle/drone_np.py  GymDronePort -- must be BIT-EXACT (same numpy paths)
  oracle/drone_ref.c  C restatement -- done/step exact, floats <= 1e-12 rel
                      (numpy routes `W @ omega` and np.linalg.norm through
                      OpenBLAS, whose FMA/ordering moves the last ulp).
"""
import numpy as np
import pytest

from oracle import cref, drone_np

REL = 1e-12


def _rel(a, b):
    return np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))


def _state(g, idx=slice(None)):
    s = {k: np.ascontiguousarray(g[k][idx], np.float64)
         for k in ("pos", "vel", "euler", "omega", "target")}
    s["step"] = np.ascontiguousarray(g["step"][idx], np.int32)
    return s


def test_golden_coverage(golden):
    g = golden("gym_step.npz")
    n = len(g["action"])
    assert n >= 10000
    assert g["o_done"].sum() > 500                       # crash + limit cases
    assert (g["step"] == 199).sum() > 100                # time limit
    assert (np.abs(g["euler"]).max(1) > 100).sum() > 100  # huge angles
    assert (np.abs(np.cos(g["euler"][:, 1])) < 1e-3).sum() > 50  # near gimbal
    assert (g["o_rew"] > 0).sum() > 10                   # target bonus
    assert str(g["numpy_version"]).startswith("2.")


def test_c_oracle_gym_step(golden):
    g = golden("gym_step.npz")
    s = _state(g)
    obs, rew, done = cref.gym_step(s, g["action"])
    np.testing.assert_array_equal(done, g["o_done"])
    np.testing.assert_array_equal(s["step"], g["o_step"])
    for k in ("pos", "vel", "euler", "omega"):
        assert _rel(s[k], g["o_" + k]) <= REL, k
    assert _rel(rew, g["o_rew"]) <= REL
    # obs is the f32 cast of the f64 state: exact unless an f64 ulp straddles
    # an f32 rounding boundary
    assert (obs != g["o_obs"]).mean() < 1e-4
    assert _rel(obs.astype(np.float64), g["o_obs"].astype(np.float64)) <= 1e-6


def test_numpy_port_bitexact(golden):
    g = golden("gym_step.npz")
    env = drone_np.GymDronePort(np.random.default_rng(0))
    for i in range(0, len(g["action"]), 3):
        env.pos, env.vel = g["pos"][i].copy(), g["vel"][i].copy()
        env.euler, env.omega = g["euler"][i].copy(), g["omega"][i].copy()
        env.target, env.current_step = g["target"][i].copy(), int(g["step"][i])
        obs, r, d, info = env.step(g["action"][i])
        assert info == {}
        assert d == bool(g["o_done"][i])
        assert r == g["o_rew"][i]
        np.testing.assert_array_equal(obs, g["o_obs"][i])
        np.testing.assert_array_equal(env.euler, g["o_euler"][i])
        np.testing.assert_array_equal(env.omega, g["o_omega"][i])


def test_numpy_batched_step(golden):
    g = golden("gym_step.npz")
    s = _state(g)
    obs, rew, done = drone_np.gym_step_batched(s, g["action"])
    np.testing.assert_array_equal(done, g["o_done"])
    for k in ("pos", "vel", "euler", "omega"):
        assert _rel(s[k], g["o_" + k]) <= REL, k
    assert _rel(rew, g["o_rew"]) <= REL


def test_c_oracle_reset(golden):
    g = golden("gym_reset.npz")
    n = len(g["u"])
    s = {k: np.zeros((n, 3)) for k in ("pos", "vel", "euler", "omega", "target")}
    s["step"] = np.full(n, 7, np.int32)
    s["ep_num"] = g["ep_num"].astype(np.int64).copy()
    s["eps"] = g["eps"].copy()
    obs = cref.gym_reset(s, g["u"])
    np.testing.assert_array_equal(s["pos"], g["o_pos"])
    np.testing.assert_array_equal(s["target"], g["o_target"])
    np.testing.assert_array_equal(s["eps"], g["o_eps"])
    np.testing.assert_array_equal(s["ep_num"], g["o_ep_num"])
    np.testing.assert_array_equal(obs, g["o_obs"])
    assert (s["step"] == 0).all()
    # the curriculum bump happened exactly where ep_num became a multiple of 2000
    bumped = g["o_eps"] != g["eps"]
    np.testing.assert_array_equal(bumped, (g["ep_num"] + 1) % 2000 == 0)


def test_numpy_port_traj_replay(golden):
    """DummyVecEnv-style 16-env, 256-step trajectory replayed through the
    single-env port with the recorded uniforms: bit-exact."""
    g = golden("gym_traj.npz")
    n = g["obs0"].shape[0]
    envs = []
    for i in range(n):
        e = drone_np.GymDronePort(np.random.default_rng(0))
        e.ep_num = 0
        e.eps = 0.0
        e.reset(g["ctor_u"][i])
        np.testing.assert_array_equal(e.reset(g["reset_u"][i]), g["obs0"][i])
        envs.append(e)
    for t in range(g["actions"].shape[0]):
        for i, e in enumerate(envs):
            o, r, d, _ = e.step(g["actions"][t, i])
            assert d == g["done"][t, i] and r == g["reward"][t, i]
            if d:
                np.testing.assert_array_equal(o, g["term_obs"][t, i])
                o = e.reset(g["reset_uniforms"][t, i])
            np.testing.assert_array_equal(o, g["obs"][t, i])
    np.testing.assert_array_equal([e.ep_num for e in envs], g["final_ep_num"])


def test_c_oracle_vec_step(golden):
    g = golden("vec_step.npz")
    B = int(g["batch"])
    nb = len(g["action"]) // B
    for b in range(nb):
        sl = slice(b * B, (b + 1) * B)
        s = {k: np.ascontiguousarray(g[k][sl], np.float64)
             for k in ("pos", "vel", "euler", "omega")}
        step0 = int(g["step"][sl][0])
        obs, rew, done, st = cref.vec_step(s, g["action"][sl], step0)
        assert st == step0 + 1
        np.testing.assert_array_equal(done, g["o_done"][sl])
        for k in ("pos", "vel", "euler", "omega"):
            assert _rel(s[k], g["o_" + k][sl]) <= REL, (b, k)
        assert _rel(rew, g["o_rew"][sl]) <= REL
        assert _rel(obs.astype(np.float64), g["o_obs"][sl].astype(np.float64)) <= 1e-6
    assert g["o_done"][g["step"] == 999].all()   # shared 1000-step limit


def test_c_oracle_vec_traj(golden):
    g = golden("vec_traj.npz")
    T, B, _ = g["actions"].shape
    s = {"pos": np.tile([0.1, 0.1, 0.1], (B, 1)).astype(np.float64),
         "vel": np.zeros((B, 3)), "euler": np.zeros((B, 3)), "omega": np.zeros((B, 3))}
    step = 0
    # Un-reset tumbling drones (|euler| reaches ~1e5 rad) amplify last-ulp
    # differences chaotically, so float state is compared over the first 30
    # steps only (divergence starts near step 32); done must match on every step.
    for t in range(T):
        obs, rew, done, step = cref.vec_step(s, g["actions"][t], step)
        np.testing.assert_array_equal(done, g["done"][t])
        if t < 30:
            assert _rel(rew, g["reward"][t]) <= 1e-9
            assert _rel(obs.astype(np.float64), g["obs"][t].astype(np.float64)) <= 1e-6


# ---------------------------------------------------------------- Philox / GAE
def test_philox_known_answers():
    # Random123 philox4x32_10 known-answer vectors.
    kat = [([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
           ([0xffffffff] * 4, [0xffffffff] * 2,
            [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
           ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
            [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1])]
    for c, k, want in kat:
        np.testing.assert_array_equal(cref.philox(c, k), np.array(want, np.uint32))


def test_gae_known_answers():
    rng = np.random.default_rng(3)
    T, N = 17, 9
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    starts = (rng.random((T, N)) < 0.2).astype(np.uint8)
    lv = rng.normal(size=N).astype(np.float32)
    ld = (rng.random(N) < 0.3).astype(np.uint8)
    # lambda = 1, gamma = 1: advantage + value = reward-to-go within episodes
    adv, ret = cref.gae(r, v, starts, lv, ld, 1.0, 1.0)
    for n in range(N):
        acc = 0.0 if ld[n] else float(lv[n])
        for t in reversed(range(T)):
            if t < T - 1 and starts[t + 1, n]:
                acc = 0.0
            acc = float(r[t, n]) + acc
            assert abs(ret[t, n] - acc) <= 1e-4 * max(1.0, abs(acc))
    # lambda = 0: advantage = one-step TD error
    adv0, _ = cref.gae(r, v, starts, lv, ld, 0.99, 0.0)
    nv = np.concatenate([v[1:], lv[None]], 0)
    nnt = 1.0 - np.concatenate([starts[1:], ld[None]], 0).astype(np.float32)
    td = (r + (np.float32(0.99) * nv) * nnt) - v
    np.testing.assert_array_equal(adv0, td)


def test_gae_matches_sb3_numpy_restatement():
    from oracle import ppo_ref
    rng = np.random.default_rng(5)
    T, N = 32, 50
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    starts = (rng.random((T, N)) < 0.1).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    ld = rng.random(N) < 0.1
    a1, r1 = cref.gae(r, v, starts.astype(np.uint8), lv, ld.astype(np.uint8), 0.99, 0.95)
    a2, r2 = ppo_ref.gae_numpy(r, v, starts, lv, ld, 0.99, 0.95)
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(r1, r2)


def test_c_oracle_moving_reduces_to_gym(golden):
    """The moving-target restatement with zero motion
    amplitude IS the gym env: same state, reward, done and obs[:15] on the
    reference's golden step vectors, zero target velocity; and its reset
    with u[:5] = the gym draws reproduces the golden reset."""
    g = golden("gym_step.npz")
    ref_obs, _, _ = cref.gym_step({k: np.array(v) for k, v in _state(g).items()}, g["action"])
    s = {k: np.array(v) for k, v in _state(g).items()}
    n = len(g["action"])
    rng = np.random.default_rng(0)
    s["motion"] = np.concatenate([np.zeros((n, 3)), rng.uniform(0.5, 2, (n, 3)),
                                  rng.uniform(0, 6.3, (n, 3))], 1).astype(np.float32)
    obs, rew, done = cref.moving_step(s, g["action"])
    np.testing.assert_array_equal(done, g["o_done"])
    assert _rel(s["pos"], g["o_pos"]) <= REL and _rel(rew, g["o_rew"]) <= REL
    assert (obs[:, 15:] == 0).all()
    np.testing.assert_array_equal(obs[:, :15], ref_obs)

    r = golden("gym_reset.npz")
    m = len(r["u"])
    s = {k: np.zeros((m, 3)) for k in ("pos", "vel", "euler", "omega", "target")}
    s["step"] = np.full(m, 7, np.int32)
    s["ep_num"] = r["ep_num"].astype(np.int64).copy()
    s["eps"] = r["eps"].copy()
    u = np.concatenate([r["u"], rng.uniform(0, 1, (m, 9))], 1)
    obs = cref.moving_reset(s, u)
    np.testing.assert_array_equal(s["target"], r["o_target"])
    np.testing.assert_array_equal(obs[:, :12], r["o_obs"][:, :12])
    # obs target-pos at s=0 uses the moved target: c + a sin(ph)
    want = s["target"] + (s["motion"][:, :3] * np.sin(s["motion"][:, 6:])).astype(np.float32)
    assert _rel(obs[:, 12:15].astype(np.float64), want - s["pos"]) < 1e-6
    assert _rel(s["motion"][:, :3].astype(np.float64), s["eps"][:, None] * u[:, 5:8]) < 1e-6
