"""dr_rollout / dr_rollout_random: K env steps in one launch.

The contract (include/dronerl.h) is that the outputs are identical, bit for
bit, to K dr_step calls on the same actions -- so every parity property of
the single-step kernel (golden vectors, oracle, Philox reset draws; see
test_env_gpu.py) carries over.  Checked here: per-step obs / rew / done and
the final state of every field, across auto-resets, the 200-step time limit
(shortened), the curriculum bump inside a launch (ep_num 1999 -> 2000 with
the eps != 0 Philox block), ragged batch sizes, f64 / f32 state and all
three variants; the in-kernel random policy against dr_random_actions; and
one step through the rollout path against the CPU oracle."""
import numpy as np
import pytest
import torch

from drone_rl_amd import _lib
from oracle import cref

pytestmark = pytest.mark.gpu

VEC = ("pos", "vel", "euler", "omega", "target")


def _pair(n, variant, dtype, **kw):
    from drone_rl_amd import DroneBatch
    a = DroneBatch(n, variant, dtype=dtype, seed=4242, env_id_offset=3 * n, **kw)
    b = DroneBatch(n, variant, dtype=dtype, seed=4242, env_id_offset=3 * n, **kw)
    for x in (a, b):
        x.reset()
        if variant != "vectorized":
            # every 7th env is one episode before the curriculum bump
            # (drone.py:68-70) and some already at eps > 0, so resets inside
            # the launch take the bump path and the eps != 0 Philox block
            ep = x.get("ep_num").cpu()
            ep[::7] = 1999
            x.set("ep_num", ep)
            eps = x.get("eps").cpu()
            eps[1::5] = 0.5
            x.set("eps", eps)
    return a, b


def _fields(b):
    out = {k: b.get(k) for k in VEC + ("current_step",)}
    if b.variant != "vectorized":
        out["ep_num"] = b.get("ep_num")
        out["eps"] = b.get("eps")
    if b.variant == "moving":
        out["motion"] = b.get("motion")
    return out


@pytest.mark.parametrize("variant,dtype,n,max_steps", [
    ("gym", torch.float64, 65536, 40),
    ("gym", torch.float32, 4097, None),
    ("gym", torch.float64, 1000, 25),
    ("moving", torch.float64, 5003, 30),
    ("vectorized", torch.float64, 777, None),
    # the large-batch launch forms of the step kernel (32 rows per wave,
    # nontemporal loads) against the rollout kernel's 64 rows per wave
    ("gym", torch.float64, 1 << 20, None),
    ("moving", torch.float64, 1 << 20, None),
])
def test_rollout_is_bitwise_k_steps(variant, dtype, n, max_steps):
    from drone_rl_amd import random_actions
    K1, K2 = 29, 35
    K = K1 + K2
    a, b = _pair(n, variant, dtype, max_steps=max_steps)
    acts = torch.empty(K, n, 4, device="cuda")
    for t in range(K):
        random_actions(n, seed=11, step=t, env_id_offset=3 * n, out=acts[t])
    # two launches back to back: the state carried across launch boundaries
    o1, r1, d1 = a.rollout(K1, acts[:K1])
    o2, r2, d2 = a.rollout(K2, acts[K1:])
    obs = torch.cat([o1, o2])
    rew = torch.cat([r1, r2])
    done = torch.cat([d1, d2])
    for t in range(K):
        so, sr, sd = b.step(acts[t])
        assert torch.equal(obs[t], so), (t, "obs")
        assert torch.equal(rew[t], sr), (t, "rew")
        assert torch.equal(done[t], sd), (t, "done")
    fa, fb = _fields(a), _fields(b)
    for k in fa:
        assert torch.equal(fa[k], fb[k]), k
    if variant != "vectorized":
        nd = int(done.sum())
        assert nd > n // 4, nd                  # resets happened in the launch
        if max_steps:
            assert int(fa["current_step"].max()) < max_steps
        # the curriculum bump (eps 0 -> 0.1) happened inside a launch
        assert bool((fa["eps"][::7] == 0.1).any())


def test_rollout_random_policy_matches_random_actions():
    from drone_rl_amd import random_actions
    n, K = 65536 + 64, 24
    a, b = _pair(n, "gym", torch.float64)
    got_a = torch.empty(K, n, 4, device="cuda")
    obs, rew, done = a.rollout(K, None, seed=77, step0=1000, actions_out=got_a)
    acts = torch.empty(K, n, 4, device="cuda")
    for t in range(K):
        random_actions(n, seed=77, step=1000 + t, env_id_offset=3 * n, out=acts[t])
    assert torch.equal(got_a, acts)
    o2, r2, d2 = b.rollout(K, acts)
    assert torch.equal(obs, o2) and torch.equal(rew, r2) and torch.equal(done, d2)
    # without the action copy: same outputs
    c, _ = _pair(n, "gym", torch.float64)
    o3, r3, d3 = c.rollout(K, None, seed=77, step0=1000)
    assert torch.equal(obs, o3) and torch.equal(rew, r3) and torch.equal(done, d3)


def test_rollout_last_step_vs_oracle():
    """65,536 f64 envs: 15 rollout steps, then one more rollout step checked
    on a subset against the CPU oracle (cref.gym_step, pinned to the
    reference's golden vectors) from the state the rollout left."""
    from drone_rl_amd import DroneBatch, random_actions
    n = 65536
    b = DroneBatch(n, "gym", dtype=torch.float64, seed=5)
    b.reset()
    b.rollout(15, None, seed=3, step0=0)
    idx = torch.from_numpy(np.random.default_rng(1).choice(n, 4096, replace=False)).cuda()
    s = {k: b.get(k)[idx].cpu().numpy().astype(np.float64) for k in VEC}
    s["step"] = b.get("current_step")[idx].cpu().numpy().astype(np.int32)
    a = random_actions(n, seed=3, step=15)
    obs, rew, done = b.rollout(1, a.reshape(1, n, 4))
    ro, rr, rd = cref.gym_step(s, a[idx].cpu().numpy())
    d = done[0, idx].cpu().numpy().astype(bool)
    assert (d == rd).all()
    o = obs[0, idx].cpu().numpy().astype(np.float64)[~d]
    err = np.abs(o - ro[~d]) / np.maximum(np.abs(ro[~d]), 1.0)
    assert err.max() <= 1e-5
    np.testing.assert_allclose(rew[0, idx].cpu().numpy(), rr, rtol=0, atol=2e-5)


def test_rollout_bad_arguments():
    from drone_rl_amd import DroneBatch
    L = _lib.lib()
    b = DroneBatch(256, "gym", dtype=torch.float64)
    o = torch.empty(4, 256, 15, device="cuda")
    r = torch.empty(4, 256, device="cuda")
    d = torch.empty(4, 256, dtype=torch.uint8, device="cuda")
    acts = torch.zeros(4 * 256 * 4 + 1, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert L.dr_rollout(b.handle, -1, acts.data_ptr(), o.data_ptr(), r.data_ptr(),
                        d.data_ptr(), s) == _lib.DR_ERR_INVALID
    assert L.dr_rollout(b.handle, 4, None, o.data_ptr(), r.data_ptr(), d.data_ptr(),
                        s) == _lib.DR_ERR_INVALID
    assert L.dr_rollout(b.handle, 4, acts.data_ptr() + 4, o.data_ptr(), r.data_ptr(),
                        d.data_ptr(), s) == _lib.DR_ERR_INVALID
    assert L.dr_rollout(b.handle, 0, acts.data_ptr(), o.data_ptr(), r.data_ptr(),
                        d.data_ptr(), s) == _lib.DR_OK
    h = DroneBatch(256, "gym", dtype=torch.float64, rng="host")
    assert L.dr_rollout(h.handle, 4, acts.data_ptr(), o.data_ptr(), r.data_ptr(),
                        d.data_ptr(), s) == _lib.DR_ERR_UNSUPPORTED
    with pytest.raises(ValueError):
        b.rollout(3, torch.zeros(4, 256, 4, device="cuda"))


def test_rollout_timed_same_outputs_and_packet_events():
    """dr_rollout_timed (the bench's timed launch): the outputs of dr_rollout,
    bit for bit, and its two events (bound to the dispatch packet by
    hipExtLaunchKernel, either may be null) bracket the kernel: a positive
    elapsed time, no longer than the host wall around launch + sync."""
    import time

    from drone_rl_amd import random_actions
    L = _lib.lib()
    n, K = 65536, 20
    a, b = _pair(n, "gym", torch.float64)
    acts = torch.empty(K, n, 4, device="cuda")
    for t in range(K):
        random_actions(n, seed=9, step=t, env_id_offset=3 * n, out=acts[t])
    o1, r1, d1 = a.rollout(K, acts)
    o2 = torch.empty_like(o1)
    r2 = torch.empty_like(r1)
    d2 = torch.empty_like(d1)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    e1.record(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    assert L.dr_rollout_timed(b.handle, K, acts.data_ptr(), o2.data_ptr(), r2.data_ptr(),
                              d2.data_ptr(), s.cuda_stream, e0.cuda_event,
                              e1.cuda_event) == _lib.DR_OK
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3
    assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2)
    ms = e0.elapsed_time(e1)
    assert 0.0 < ms <= wall_ms, (ms, wall_ms)
    fa, fb = _fields(a), _fields(b)
    for k in fa:
        assert torch.equal(fa[k], fb[k]), k
    # null events: a plain launch; the outputs again those of dr_rollout
    assert L.dr_rollout_timed(b.handle, K, acts.data_ptr(), o2.data_ptr(), r2.data_ptr(),
                              d2.data_ptr(), s.cuda_stream, None, None) == _lib.DR_OK
    o3, r3, d3 = a.rollout(K, acts)
    torch.cuda.synchronize()
    assert torch.equal(o3, o2) and torch.equal(r3, r2) and torch.equal(d3, d2)


@pytest.mark.parametrize("ws,variant,n", [
    ("1", "gym", 131072 + 320),     # split-physics form at two blocks per CU, ragged
    ("1", "moving", 70000),         # warp-specialised moving variant above one block per CU
    ("0", "gym", 65536),            # the one-role kernel where the default is warp-specialised
])
def test_rollout_forms_outside_their_default(ws, variant, n):
    """Both kernel forms of dr_rollout stay bitwise equal to K dr_step launches
    in the regimes the size rule does not pick them for (DRONERL_ROLLOUT_WS
    forces a form; it is read once per process, hence the subprocess)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DRONERL_ROLLOUT_WS=ws, PYTHONPATH=root)
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "rollout_form_worker.py"),
                        variant, str(n), "37"], env=env, capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ok" in r.stdout
