"""GPU parity of the moving-target curriculum variant (BASELINE configs[4],
DESIGN.md section 11) against oracle/drone_ref.c (oracle_moving_step /
oracle_moving_reset).

The variant is this build's specification (the reference has no moving
target): parity is pinned (a) to the gym variant, which it must reproduce
bit for bit when the motion amplitude is zero (eps = 0, the first 2000
episodes), and through it to the reference's golden vectors; (b) to the C
restatement of the motion law on random states.  Bar as for the gym env:
done exact (f64), floats within 1e-5 * max(|ref|, 1).
"""
import numpy as np
import pytest
import torch

from oracle import cref

pytestmark = pytest.mark.gpu
VEC = ("pos", "vel", "euler", "omega", "target")


def _close(a, b, tol=1e-5, what=""):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b) / np.maximum(np.abs(b), 1.0)
    assert err.max() <= tol, f"{what}: {err.max():.3e}"


def _batch(n, **kw):
    from drone_rl_amd import DroneBatch
    return DroneBatch(n, **kw)


def test_zero_amplitude_is_the_gym_env():
    """eps = 0 -> a = 0: the target is the gym target, the extra obs are
    zero and every obs/reward/done/reset equals the gym variant's bitwise
    (the first five reset draws are the gym draws)."""
    from drone_rl_amd import random_actions
    n = 5000
    g = _batch(n, variant="gym", seed=11, keep_terminal_obs=True)
    m = _batch(n, variant="moving", seed=11, keep_terminal_obs=True)
    og, om = g.reset(), m.reset()
    assert om.shape == (n, 18)
    assert torch.equal(om[:, :15], og) and not om[:, 15:].any()
    resets = 0
    for t in range(120):
        a = random_actions(n, seed=3, step=t)
        og, rg, dg = g.step(a)
        om, rm, dm = m.step(a)
        assert torch.equal(om[:, :15], og) and torch.equal(rm, rg) and torch.equal(dm, dg)
        assert torch.equal(m.term_obs[:, :15], g.term_obs)
        resets += int(dg.sum())
    assert resets > n // 2
    assert torch.equal(m.get("ep_num"), g.get("ep_num"))


def _random_state(n, rng, eps):
    s = {"pos": rng.uniform(-0.5, 0.5, (n, 3)) + [0, 0, 1.5],
         "vel": rng.normal(0, 0.5, (n, 3)), "euler": rng.normal(0, 0.2, (n, 3)),
         "omega": rng.normal(0, 0.5, (n, 3)), "target": rng.uniform(-1, 1, (n, 3)) + [0, 0, 1],
         "step": rng.integers(0, 190, n).astype(np.int32)}
    s["motion"] = np.concatenate([eps * rng.uniform(0, 1, (n, 3)),
                                  0.5 + 1.5 * rng.uniform(0, 1, (n, 3)),
                                  2 * np.pi * rng.uniform(0, 1, (n, 3))], 1).astype(np.float32)
    return s


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_moving_steps_vs_oracle(dtype):
    """30 steps from random (tumbling) states with random motion, no
    auto-reset; the GPU state is re-synced to the oracle's after every step
    (the dynamics are chaotic: libm ulps grow by ~2x per step there)."""
    from drone_rl_amd import random_actions
    n = 4099
    rng = np.random.default_rng(0)
    s = _random_state(n, rng, eps=1.5)
    if dtype == torch.float32:
        for k in VEC:
            s[k] = s[k].astype(np.float32).astype(np.float64)
    b = _batch(n, variant="moving", dtype=dtype, rng="host", auto_reset=False)
    for k in VEC:
        b.set(k, s[k])
    b.set("current_step", s["step"])
    b.set("motion", s["motion"])
    np.testing.assert_array_equal(b.get("motion").cpu().numpy(), s["motion"])
    for t in range(30):
        a = random_actions(n, seed=5, step=t)
        obs, rew, done = b.step(a)
        ro, rr, rd = cref.moving_step(s, a.cpu().numpy())
        d = done.cpu().numpy().astype(bool)
        keep = d == rd
        assert (~keep).sum() <= (0 if dtype == torch.float64 else 2)
        _close(obs.cpu().numpy()[keep], ro[keep], 1e-5, f"obs t={t}")
        np.testing.assert_allclose(rew.cpu().numpy(), rr, rtol=0, atol=2e-5)
        if dtype == torch.float32:
            for k in VEC:
                s[k] = s[k].astype(np.float32).astype(np.float64)
        for k in VEC[:4]:
            b.set(k, s[k])
    np.testing.assert_array_equal(b.get("current_step").cpu().numpy(), s["step"])


def test_moving_reset_and_autoreset_vs_oracle():
    """Host-uniform resets (14 draws per env) and the same-step auto-reset:
    reset obs, terminal obs, centre, motion and curriculum vs the oracle."""
    n = 3000
    rng = np.random.default_rng(1)
    b = _batch(n, variant="moving", rng="host", keep_terminal_obs=True)
    u = rng.uniform(0, 1, (n, 14))
    b.set("eps", np.full(n, 0.7))
    b.set_reset_uniforms(u)
    obs = b.reset().cpu().numpy()
    s = {k: np.zeros((n, 3)) for k in VEC}
    s["step"] = np.zeros(n, np.int32)
    s["ep_num"] = b.get("ep_num").cpu().numpy().astype(np.int64) - 1
    s["eps"] = np.full(n, 0.7)
    ro = cref.moving_reset(s, u)
    _close(obs, ro, what="reset obs")
    np.testing.assert_array_equal(b.get("motion").cpu().numpy(), s["motion"])
    np.testing.assert_array_equal(b.get("target").cpu().numpy(), s["target"])
    # drive every env to its 200-step limit: all auto-reset in one step
    b.set("current_step", np.full(n, 199, np.int32))
    s["step"][:] = 199
    u2 = rng.uniform(0, 1, (n, 14))
    b.set_reset_uniforms(u2)
    a = torch.full((n, 4), 2.4525, device="cuda")
    obs, rew, done = b.step(a)
    term, rr, rd = cref.moving_step(s, a.cpu().numpy())
    assert rd.all() and done.cpu().numpy().all()
    _close(b.term_obs.cpu().numpy(), term, what="terminal obs")
    np.testing.assert_allclose(rew.cpu().numpy(), rr, rtol=0, atol=2e-5)
    ro = cref.moving_reset(s, u2)
    _close(obs.cpu().numpy(), ro, what="auto-reset obs")
    np.testing.assert_array_equal(b.get("motion").cpu().numpy(), s["motion"])
    assert (b.get("current_step").cpu().numpy() == 0).all()


def test_moving_philox_reset_draws():
    """Philox reset: 4 blocks, the first 5 words are the gym draws."""
    n, seed = 512, 77
    b = _batch(n, variant="moving", seed=seed)
    b.set("eps", np.full(n, 1.0))
    b.reset()
    mot = b.get("motion").cpu().numpy()
    cen = b.get("target").cpu().numpy()
    for i in range(0, n, 37):
        w = np.concatenate([cref.philox([2, i, 0, 0x52000000 | k], [seed, 0]) for k in range(4)])
        u = w.astype(np.float64) / 4294967296.0
        np.testing.assert_array_equal(cen[i], [u[2], u[3], u[4] + 1.0])
        want = np.concatenate([u[5:8], 0.5 + 1.5 * u[8:11], 6.283185307179586 * u[11:14]])
        np.testing.assert_array_equal(mot[i], want.astype(np.float32))


def test_moving_ppo_update_runs():
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    tr = PPOTrainer(PPOConfig(num_envs=2048, n_steps=16, batch_size=4096, n_epochs=2,
                              net_arch=(64, 64), seed=5, variant="moving"))
    assert tr.obs.shape[-1] == 18
    for _ in range(2):
        assert torch.isfinite(tr.learn_step()).all()
    assert "motion" in tr.state_dict()["env"]
    tr.close()


@pytest.mark.parametrize("n", [131072, 1048576])
def test_configs4_per_gpu_size_subset_parity(n):
    """configs[4] at its per-GPU slice (8 x 131,072 = 1M envs over a node)
    and its whole 1,048,576-env size on one GPU, with moving targets
    (eps = 0.5): 20 random-policy steps with Philox auto-reset, then one
    step checked on a 16k-env subset against oracle_moving_step, the reset
    of every done subset env (all 14 Philox draws) against oracle_moving_reset,
    and bitwise determinism of the whole batch."""
    from drone_rl_amd import random_actions
    seed = 4321

    def run(steps):
        b = _batch(n, variant="moving", seed=seed, keep_terminal_obs=True)
        b.set("eps", np.full(n, 0.5))
        b.reset()
        out = None
        for t in range(steps):
            out = b.step(random_actions(n, seed=9, step=t))
        return b, out

    b, _ = run(20)
    idx = torch.from_numpy(np.sort(np.random.default_rng(2).choice(n, 16384,
                                                                    replace=False))).cuda()
    pre = {k: b.get(k)[idx].cpu().numpy().astype(np.float64).copy() for k in VEC}
    pre["step"] = b.get("current_step")[idx].cpu().numpy().astype(np.int32)
    pre["motion"] = b.get("motion")[idx].cpu().numpy()
    ep_pre = b.get("ep_num")[idx].cpu().numpy()
    assert (np.abs(pre["motion"][:, :3]) > 0).any(), "moving targets expected"
    a = random_actions(n, seed=9, step=20)
    obs, rew, done = b.step(a)
    torch.cuda.synchronize()
    s = {k: v.copy() for k, v in pre.items()}
    ro, rr, rd = cref.moving_step(s, a[idx].cpu().numpy())
    d = done[idx].cpu().numpy().astype(bool)
    assert (d == rd).all()
    assert d.any() and (~d).any()
    _close(b.term_obs[idx].cpu().numpy()[d], ro[d], what="terminal obs")
    _close(obs[idx].cpu().numpy()[~d], ro[~d], what="obs")
    np.testing.assert_allclose(rew[idx].cpu().numpy(), rr, rtol=0, atol=2e-5)
    # resets of the done subset envs: Philox(seed, env id, new ep_num), 4 blocks
    di = idx.cpu().numpy()[d][:512]
    ep = ep_pre[d][:512].astype(np.int64)
    u = np.stack([np.concatenate([cref.philox([int(e) + 1, int(i) & 0xffffffff, int(i) >> 32,
                                               0x52000000 | k], [seed, 0]) for k in range(4)])
                  for i, e in zip(di, ep)]).astype(np.float64)[:, :14] / 4294967296.0
    m = len(di)
    rs = {k: np.zeros((m, 3)) for k in VEC}
    rs.update(step=np.zeros(m, np.int32), ep_num=ep.copy(), eps=np.full(m, 0.5))
    want = cref.moving_reset(rs, u)
    sel = torch.from_numpy(di).cuda()
    _close(obs[sel].cpu().numpy(), want, what="reset obs")
    np.testing.assert_array_equal(b.get("motion")[sel].cpu().numpy(), rs["motion"])
    np.testing.assert_array_equal(b.get("target")[sel].cpu().numpy(), rs["target"])
    np.testing.assert_array_equal(b.get("ep_num")[sel].cpu().numpy(), ep + 1)
    # determinism: an independent batch with the same seed, bit for bit
    o1, r1, d1 = obs.clone(), rew.clone(), done.clone()
    b.close()
    b2, (o2, r2, d2) = run(21)
    assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2)
    b2.close()
