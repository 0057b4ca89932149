"""Edge cases of the HIP env through the C ABI: ragged batch sizes (partial
blocks / waves), unaligned output rows, NaN state semantics, argument
errors, sharded == unsharded (the DP env partition), vectorized f32."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import cref

pytestmark = pytest.mark.gpu
VEC = ("pos", "vel", "euler", "omega", "target")


def _close(a, b, tol=1e-5):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b) / np.maximum(np.abs(b), 1.0)
    assert err.max() <= tol, err.max()


@pytest.mark.parametrize("rpw", ["64", "32"])
@pytest.mark.parametrize("n", [1, 31, 33, 63, 64, 65, 255, 257, 1000])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_ragged_sizes_match_oracle(golden, n, dtype, rpw, monkeypatch):
    """Also with half-populated waves (32 envs per wave, the layout chosen
    for 384k-3M envs), forced here by DRONERL_ROWS_PER_WAVE."""
    monkeypatch.setenv("DRONERL_ROWS_PER_WAVE", rpw)
    from drone_rl_amd import DroneBatch
    g = golden("gym_step.npz")
    idx = np.arange(n) * 7 % len(g["action"])
    b = DroneBatch(n, "gym", dtype=dtype, rng="host", auto_reset=False)
    s = {}
    for k in VEC:
        v = g[k][idx]
        if dtype == torch.float32:
            v = v.astype(np.float32).astype(np.float64)
        s[k] = np.ascontiguousarray(v)
        b.set(k, v)
    s["step"] = g["step"][idx].astype(np.int32)
    b.set("current_step", s["step"])
    obs, rew, done = b.step(torch.from_numpy(g["action"][idx]).cuda())
    ro, rr, rd = cref.gym_step(s, g["action"][idx])
    d = done.cpu().numpy().astype(bool)
    keep = d == rd
    assert (~keep).sum() <= (0 if dtype == torch.float64 else 1)
    _close(obs.cpu().numpy()[keep], ro[keep])
    np.testing.assert_allclose(rew.cpu().numpy(), rr, atol=2e-5)


def test_unaligned_obs_rows_match_aligned(golden):
    """obs_out at a 60-B offset (not 16-B aligned) takes the scalar store
    path; results must equal the aligned float4 path."""
    from drone_rl_amd import DroneBatch, random_actions
    n = 1000
    a = DroneBatch(n, "gym", seed=5)
    b = DroneBatch(n, "gym", seed=5)
    a.reset()
    b.reset()
    buf = torch.zeros(n + 1, 15, device="cuda")
    out = buf[1:]
    assert out.data_ptr() % 16 != 0 and out.is_contiguous()
    for t in range(40):
        act = random_actions(n, seed=1, step=t)
        oa, _, _ = a.step(act)
        ob, _, _ = b.step(act, obs_out=out)
        assert torch.equal(oa, ob)


def test_nan_state_ends_only_at_time_limit():
    """drone.py:154 compares NaN positions -> False: a NaN env is not done
    until the 200-step limit (and its obs stay NaN)."""
    from drone_rl_amd import DroneBatch
    b = DroneBatch(2, "gym", auto_reset=False)
    b.set("pos", np.array([[np.nan, 0.0, 1.0], [0.0, 0.0, np.nan]]))
    b.set("current_step", np.array([10, 198], np.int32))
    a = torch.full((2, 4), 2.0, device="cuda")
    obs, rew, done = b.step(a)
    assert done.cpu().tolist() == [0, 0]
    assert torch.isnan(obs[0, 0]) and torch.isnan(rew).all()
    obs, rew, done = b.step(a)
    assert done.cpu().tolist() == [0, 1]


def test_abi_argument_errors():
    from drone_rl_amd import DroneBatch, _lib
    L = _lib.lib()
    b = DroneBatch(64, "gym")
    act = torch.zeros(65 * 4 + 1, device="cuda")
    obs = torch.zeros(64, 15, device="cuda")
    rew = torch.zeros(64, device="cuda")
    done = torch.zeros(64, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    rc = L.dr_step(b.handle, act.data_ptr() + 4, obs.data_ptr(), rew.data_ptr(),
                   done.data_ptr(), None, st)
    assert rc == _lib.DR_ERR_INVALID and "aligned" in _lib.last_error(b.handle)
    rc = L.dr_step(b.handle, act.data_ptr(), None, rew.data_ptr(), done.data_ptr(), None, st)
    assert rc == _lib.DR_ERR_INVALID
    assert L.dr_get_state(b.handle, 99, obs.data_ptr(), st) == _lib.DR_ERR_INVALID
    assert L.dr_set_reset_uniforms(b.handle, obs.data_ptr()) == _lib.DR_ERR_INVALID  # philox
    cfg = _lib.dr_config(num_envs=8, variant=0, state_dtype=0, rng_mode=1, auto_reset=1)
    h = ctypes.c_void_p()
    assert L.dr_create(ctypes.byref(cfg), ctypes.byref(h)) == 0
    # host-uniform mode without uniforms: reset refuses instead of reading NULL
    assert L.dr_reset(h, obs.data_ptr(), st) == _lib.DR_ERR_INVALID
    assert L.dr_destroy(h) == 0
    with pytest.raises(ValueError):
        b.step(torch.zeros(63, 4, device="cuda"))


@pytest.mark.parametrize("variant,dtype,form", [
    ("gym", "f64", ("32", "0")), ("gym", "f64", ("64", "1")), ("gym", "f64", ("32", "1")),
    ("moving", "f64", ("64", "1")), ("gym", "f32", ("32", "1"))])
def test_launch_forms_equal_default_form(variant, dtype, form, monkeypatch):
    """Every launch form (32 envs per wave, nontemporal state loads; chosen
    by batch size in dr_create) computes exactly what the 64-envs-per-wave
    plain-load form does, over 60 steps with auto-resets, terminal obs and
    monitor outputs."""
    from drone_rl_amd import DroneBatch, random_actions
    n = 4099
    out = []
    for rpw, ntl in (("64", "0"), form):
        monkeypatch.setenv("DRONERL_ROWS_PER_WAVE", rpw)
        monkeypatch.setenv("DRONERL_NT_LOADS", ntl)
        b = DroneBatch(n, variant, seed=21, keep_terminal_obs=True, monitor=True,
                       dtype=torch.float64 if dtype == "f64" else torch.float32)
        if variant == "moving":     # moving targets (eps > 0: nonzero amplitudes)
            b.set("eps", torch.full((n,), 0.3, dtype=torch.float64))
        b.reset()
        acc = []
        for t in range(60):
            o, r, d = b.step(random_actions(n, seed=4, step=t))
            acc += [o.clone(), r.clone(), d.clone(), b.term_obs.clone(), b.ep_ret.clone()]
        out.append(acc + [b.get("pos"), b.get("ep_num")])
    assert all(torch.equal(x, y) for x, y in zip(*out))


def test_sharded_equals_unsharded():
    """Two shards with env_id_offset 0 and N evolve exactly like the two
    halves of one 2N batch: resets are keyed by the GLOBAL env id, which is
    what makes the data-parallel partition free of communication."""
    from drone_rl_amd import DroneBatch, random_actions
    n = 3000
    full = DroneBatch(2 * n, "gym", seed=9)
    s0 = DroneBatch(n, "gym", seed=9, env_id_offset=0)
    s1 = DroneBatch(n, "gym", seed=9, env_id_offset=n)
    o = full.reset().clone()
    assert torch.equal(o[:n], s0.reset()) and torch.equal(o[n:], s1.reset())
    for t in range(80):
        act = random_actions(2 * n, seed=2, step=t)
        of, rf, df = full.step(act)
        o0, r0, d0 = s0.step(act[:n].contiguous())
        o1, r1, d1 = s1.step(act[n:].contiguous())
        assert torch.equal(of[:n], o0) and torch.equal(of[n:], o1)
        assert torch.equal(df[:n], d0) and torch.equal(df[n:], d1)
    assert torch.equal(full.get("ep_num")[:n], s0.get("ep_num"))


def test_vectorized_f32_and_shared_limit():
    from drone_rl_amd import DroneBatch
    b = DroneBatch(100, "vectorized", dtype=torch.float32)
    obs = b.reset()
    assert obs.shape == (100, 12) and torch.allclose(obs[:, :3], torch.full((100, 3), 0.1,
                                                                            device="cuda"))
    a = torch.full((100, 4), 9.81 / 4, device="cuda")
    for t in range(999):
        _, _, d = b.step(a)
    assert not d.any()
    _, _, d = b.step(a)                 # step 1000: everyone done
    assert d.all()
    _, _, d = b.step(a)                 # no auto-reset: stays done
    assert d.all()


def test_philox_reset_targets_with_curriculum():
    """Philox resets with eps > 0 use block 1 for the target z draw (block 1
    is skipped only while eps == 0, where 0 * u is exactly 0); check the
    reset targets of both regimes against the CPU Philox."""
    from oracle import cref as _c
    from drone_rl_amd import DroneBatch
    n, seed = 512, 31
    b = DroneBatch(n, "gym", seed=seed)
    eps = np.where(np.arange(n) % 2 == 0, 0.0, 0.7)
    b.set("eps", eps)
    b.set("current_step", np.full(n, 199, np.int32))      # all time out now
    ep0 = b.get("ep_num").cpu().numpy()
    b.step(torch.full((n, 4), 2.4525, device="cuda"))
    tgt = b.get("target").cpu().numpy()
    pos = b.get("pos").cpu().numpy()
    for i in range(0, n, 9):
        ep_new = int(ep0[i]) + 1
        w0 = _c.philox([ep_new, i, 0, 0x52000000], [seed, 0]).astype(np.float64) / 2 ** 32
        w1 = _c.philox([ep_new, i, 0, 0x52000001], [seed, 0]).astype(np.float64) / 2 ** 32
        np.testing.assert_array_equal(pos[i], [w0[0] - 0.5, w0[1] - 0.5, 1.0])
        want = [eps[i] * w0[2], eps[i] * w0[3], eps[i] * w1[0] + 1.0 + 0.0]
        np.testing.assert_array_equal(tgt[i], want)
