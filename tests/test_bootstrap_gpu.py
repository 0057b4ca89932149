"""PPOConfig.bootstrap_timeouts (opt-in; the reference's semantics are off):
SB3's TimeLimit bootstrap in collect_rollouts -- rewards[idx] += gamma *
V(terminal obs) where an episode hit the 200-step limit (drone.py:155-157)
without crashing (drone.py:154) -- against the CPU restatement
oracle/ppo_ref.py:timeout_bootstrap_numpy (parity unpinned: SB3 is absent).

Two deterministic policies (log_std -30, so every sample is the mean): the
hover thrust (mass * g / 4 per motor) keeps the drone aloft until the step
limit, so every episode is truncated; zero thrust falls and crashes near
step 22, so no step is."""
import numpy as np
import pytest
import torch

from oracle.ppo_ref import timeout_bootstrap_numpy

pytestmark = pytest.mark.gpu

HOVER = 1.0 * 9.81 / 4.0


class _Tap:
    """TrajectoryRecorder stand-in: snapshots the env's terminal obs, VecMonitor
    episode lengths and truncation flags after every rollout step."""

    def __init__(self, tr):
        self.tr, self.rows, self.t = tr, [], 0

    def on_step(self, dones):
        t = self.t
        term = self.tr.env.term_obs
        self.rows.append((term.clone() if term is not None else None,
                          self.tr.ep_len[t].clone(),
                          self.tr.trunc[t].clone() if self.tr.trunc is not None else None))
        self.t += 1

    def flush(self):
        pass


def _rollout(thrust, bootstrap):
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=1024, n_steps=256, batch_size=8192, n_epochs=1, seed=4,
                    bootstrap_timeouts=bootstrap)
    tr = PPOTrainer(cfg)
    with torch.no_grad():
        tr.policy.p("action.w").zero_()
        tr.policy.p("action.b").fill_(thrust)
        tr.policy.p("log_std").fill_(-30.0)
    tap = _Tap(tr)
    tr.trajectory = tap
    tr.collect_rollouts()
    torch.cuda.synchronize()
    out = dict(rew=tr.rewards.cpu().numpy(), done=tr.dones[1:].cpu().numpy().astype(bool),
               rows=tap.rows, policy=tr.policy, tr=tr)
    return out


def test_timeout_bootstrap_matches_sb3_restatement():
    off = _rollout(HOVER, False)
    on = _rollout(HOVER, True)
    # same trajectories (the bootstrap only touches the stored rewards)
    assert np.array_equal(off["done"], on["done"])
    n_trunc = 0
    for t, (term, ep_len, trunc) in enumerate(on["rows"]):
        done = on["done"][t]
        tr_np = trunc.cpu().numpy().astype(bool)
        # the hover policy never crashes: truncated == done, at the limit
        assert np.array_equal(tr_np, done), t
        assert (ep_len.cpu().numpy()[done] == 200).all(), t
        n_trunc += int(tr_np.sum())
        if tr_np.any():
            with torch.no_grad():
                _, v = on["policy"].forward(term)          # torch fp32 reference forward
            exp = timeout_bootstrap_numpy(off["rew"][t], tr_np, v.cpu().numpy(), 0.99)
            got = on["rew"][t]
            assert np.array_equal(got[~tr_np], off["rew"][t][~tr_np]), t
            # the GPU value head (x6 GEMMs) vs the torch fp32 forward
            np.testing.assert_allclose(got[tr_np], exp[tr_np], rtol=1e-5, atol=1e-5)
        else:
            assert np.array_equal(on["rew"][t], off["rew"][t]), t
    assert n_trunc >= 1024        # every env reaches the limit once in 256 steps
    for r in (off, on):
        r["tr"].close()


def test_crashes_are_not_bootstrapped():
    off = _rollout(0.0, False)
    on = _rollout(0.0, True)
    assert on["done"].any()
    for t, (_, ep_len, trunc) in enumerate(on["rows"]):
        assert not trunc.any(), t
        d = on["done"][t]
        assert (ep_len.cpu().numpy()[d] < 200).all()
    assert np.array_equal(on["rew"], off["rew"])
    for r in (off, on):
        r["tr"].close()


def test_timeout_bootstrap_rollout_graph_is_bitwise_eager():
    """The default rollout path captures the T-step loop -- the extra value
    forward of the terminal obs and the masked reward add included -- into a
    hipGraph (no trajectory tap here).  Three collect_rollouts() calls on the
    graph path (eager warm-up, capture + replay, replay) give bitwise the
    rewards, values and dones of the same three calls run eagerly."""
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    res = []
    for graph in (True, False):
        cfg = PPOConfig(num_envs=1024, n_steps=256, batch_size=8192, n_epochs=1, seed=4,
                        bootstrap_timeouts=True)
        tr = PPOTrainer(cfg)
        tr.rollout_graph = graph
        with torch.no_grad():
            tr.policy.p("action.w").zero_()
            tr.policy.p("action.b").fill_(HOVER)
            tr.policy.p("log_std").fill_(-30.0)
        out = []
        for _ in range(3):
            tr.collect_rollouts()
            torch.cuda.synchronize()
            out.append((tr.rewards.clone(), tr.values.clone(), tr.dones.clone()))
        if graph:
            assert tr._rgraph is not None, "the rollout graph was not captured"
        res.append(out)
    n_trunc = 0
    for (rg, vg, dg), (re, ve, de) in zip(*res):
        assert torch.equal(rg, re) and torch.equal(vg, ve) and torch.equal(dg, de)
        n_trunc += int(dg.sum())
    assert n_trunc > 0          # the hover policy reaches the step limit
