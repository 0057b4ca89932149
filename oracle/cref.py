"""ctypes access to oracle/build/liboracle.so (test infrastructure only)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("ORACLE_LIB", os.path.join(_HERE, "build", "liboracle.so"))
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def gym_step(state, action):
    """One DroneEnv.step for n envs.  state: dict of (n,3) f64 pos/vel/euler/
    omega/target and (n,) i32 step; mutated in place.  Returns obs, reward,
    done."""
    n = len(action)
    action = np.ascontiguousarray(action, np.float32)
    for k in ("pos", "vel", "euler", "omega"):
        assert state[k].dtype == np.float64 and state[k].flags.c_contiguous
    state["step"] = np.ascontiguousarray(state["step"], np.int32)
    tgt = np.ascontiguousarray(state["target"], np.float64)
    obs = np.zeros((n, 15), np.float32)
    rew = np.zeros(n)
    done = np.zeros(n, np.uint8)
    lib().oracle_gym_step(ctypes.c_int64(n), _p(state["pos"]), _p(state["vel"]),
                          _p(state["euler"]), _p(state["omega"]), _p(tgt),
                          _p(state["step"]), _p(action), _p(obs), _p(rew), _p(done))
    return obs, rew, done.astype(bool)


def gym_reset(state, u):
    """DroneEnv.reset for n envs given the (n,5) uniforms; state also needs
    (n,) i64 ep_num and (n,) f64 eps.  Returns obs."""
    n = len(u)
    u = np.ascontiguousarray(u, np.float64)
    state["ep_num"] = np.ascontiguousarray(state["ep_num"], np.int64)
    state["step"] = np.ascontiguousarray(state["step"], np.int32)
    obs = np.zeros((n, 15), np.float32)
    lib().oracle_gym_reset(ctypes.c_int64(n), _p(state["pos"]), _p(state["vel"]),
                           _p(state["euler"]), _p(state["omega"]), _p(state["target"]),
                           _p(state["step"]), _p(state["ep_num"]), _p(state["eps"]),
                           _p(u), _p(obs))
    return obs


def moving_step(state, action):
    """One step of the moving-target variant (drone_ref.c oracle_moving_step).
    state: gym_step's dict with "target" = the reset centre (n,3) f64 and
    "motion" (n,9) f32; mutated in place.  Returns obs (n,18), reward, done."""
    n = len(action)
    action = np.ascontiguousarray(action, np.float32)
    for k in ("pos", "vel", "euler", "omega"):
        assert state[k].dtype == np.float64 and state[k].flags.c_contiguous
    state["step"] = np.ascontiguousarray(state["step"], np.int32)
    cen = np.ascontiguousarray(state["target"], np.float64)
    mot = np.ascontiguousarray(state["motion"], np.float32)
    obs = np.zeros((n, 18), np.float32)
    rew = np.zeros(n)
    done = np.zeros(n, np.uint8)
    lib().oracle_moving_step(ctypes.c_int64(n), _p(state["pos"]), _p(state["vel"]),
                             _p(state["euler"]), _p(state["omega"]), _p(cen), _p(mot),
                             _p(state["step"]), _p(action), _p(obs), _p(rew), _p(done))
    return obs, rew, done.astype(bool)


def moving_reset(state, u):
    """Moving-variant reset given (n,14) uniforms; fills state["motion"]."""
    n = len(u)
    u = np.ascontiguousarray(u, np.float64)
    state["ep_num"] = np.ascontiguousarray(state["ep_num"], np.int64)
    state["step"] = np.ascontiguousarray(state["step"], np.int32)
    state["motion"] = np.zeros((n, 9), np.float32)
    obs = np.zeros((n, 18), np.float32)
    lib().oracle_moving_reset(ctypes.c_int64(n), _p(state["pos"]), _p(state["vel"]),
                              _p(state["euler"]), _p(state["omega"]), _p(state["target"]),
                              _p(state["motion"]), _p(state["step"]), _p(state["ep_num"]),
                              _p(state["eps"]), _p(u), _p(obs))
    return obs


def vec_step(state, action, shared_step):
    """VectorizedDroneEnv.step; returns obs, reward, done, new shared step."""
    n = len(action)
    action = np.ascontiguousarray(action, np.float32)
    st = np.array([shared_step], np.int32)
    obs = np.zeros((n, 12), np.float32)
    rew = np.zeros(n)
    done = np.zeros(n, np.uint8)
    lib().oracle_vec_step(ctypes.c_int64(n), _p(state["pos"]), _p(state["vel"]),
                          _p(state["euler"]), _p(state["omega"]), _p(st), _p(action),
                          _p(obs), _p(rew), _p(done))
    return obs, rew, done.astype(bool), int(st[0])


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def gae(rew, val, starts, last_val, last_done, gamma, lam):
    T, N = rew.shape
    rew = np.ascontiguousarray(rew, np.float32)
    val = np.ascontiguousarray(val, np.float32)
    starts = np.ascontiguousarray(starts, np.uint8)
    last_val = np.ascontiguousarray(last_val, np.float32)
    last_done = np.ascontiguousarray(last_done, np.uint8)
    adv = np.zeros((T, N), np.float32)
    ret = np.zeros((T, N), np.float32)
    lib().oracle_gae_f32(ctypes.c_int64(T), ctypes.c_int64(N), _p(rew), _p(val), _p(starts),
                         _p(last_val), _p(last_done), ctypes.c_double(gamma),
                         ctypes.c_double(lam), _p(adv), _p(ret))
    return adv, ret


def philox_np(ctr, key):
    """Philox4x32-10 over rows of counters: ctr (n,4) uint32, key (2,) ->
    (n,4) uint32; the vectorised form of `philox` (numpy, for large test
    vectors), following drone_rl_amd/csrc/common.h philox4x32_10."""
    c = np.array(ctr, np.uint64).reshape(-1, 4) & 0xffffffff
    k0, k1 = np.uint64(key[0] & 0xffffffff), np.uint64(key[1] & 0xffffffff)
    m0, m1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    w0, w1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
    mask, sh = np.uint64(0xffffffff), np.uint64(32)
    x, y, z, w = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
    for _ in range(10):
        p0, p1 = m0 * x, m1 * z
        x, y, z, w = ((p1 >> sh) ^ y ^ k0) & mask, p1 & mask, ((p0 >> sh) ^ w ^ k1) & mask, \
            p0 & mask
        k0, k1 = (k0 + w0) & mask, (k1 + w1) & mask
    return np.stack([x, y, z, w], 1).astype(np.uint32)


def permutation_np(n, seed, counter):
    """dr_permutation's result restated: the stable argsort of the 64-bit
    Philox keys (r.x << 32 | r.y) of counters (i, counter, TAG_PERM)."""
    i = np.arange(n, dtype=np.uint64)
    ctr = np.stack([i & np.uint64(0xffffffff), i >> np.uint64(32),
                    np.full(n, counter & 0xffffffff, np.uint64),
                    np.full(n, 0x50000000 ^ (counter >> 32), np.uint64)], 1)
    r = philox_np(ctr, [seed & 0xffffffff, seed >> 32]).astype(np.uint64)
    keys = (r[:, 0] << np.uint64(32)) | r[:, 1]
    return np.argsort(keys, kind="stable").astype(np.int32)
