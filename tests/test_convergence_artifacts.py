"""The convergence claim (configs[2] must reach at least the
return the SB3-default CPU PPO reaches on configs[0] at 2e6 steps), compared
at matched curriculum levels (the anchor ends at eps 4.8), checked on
committed artefacts (CPU only; every log is a builder run):

  tests/golden/c1_anchor.json          oracle/sb3_c1.py, 3 seeds, 2e6 steps (with
                                       episode lengths since round 3)
  profiles/r01_ppo_c3_converge.jsonl   GPU PPO, 65,536 envs, 2x256 (train.py), eps 0
  profiles/r02_ppo_c3_eps*.jsonl       the same from scratch at a FIXED eps 0.5 / 1 / 2 /
                                       4.8 (c3_matched.sh), and at eps 0 on the x6 GEMMs
  profiles/r03_ppo_c3_staged_ent01_*   the same with a staged curriculum (eps 0 -> 1.0,
                                       and a run to 4.8) and entropy coefficient 0.01,
                                       plus a deterministic evaluation of each trained
                                       policy (scripts/c3_staged.sh, eval_policy.py)
  profiles/r01_ppo_c1_gpu.jsonl        GPU PPO with SB3 defaults on 1 env

Every "learned" claim requires episodes longer than a uniform-random
policy's 32 steps (all of them end by crashing): the reward
(-0.01 * distance per step, +1 inside 5 cm, drone.py:142-148) is
larger for a policy that crashes at once than for one that flies without
reaching the bonus, and both the anchor and PPO from scratch at a fixed eps
above 0 settle on crashing early (ep_len 17-23).
"""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _jsonl(name):
    return [json.loads(l) for l in open(os.path.join(ROOT, "profiles", name)) if l.startswith("{")]


def _anchor():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "c1_anchor.json")))


def _anchor_at(a, eps):
    """Per seed: the anchor's mean ep_rew_mean over its history entries at
    curriculum level eps (drone.py:68-73 raises eps by 0.1 every 2000
    episodes, so each level covers ~2 logged points of the 1-env run)."""
    out = []
    for s in a["seeds"]:
        h = [x["ep_rew_mean"] for x in s["history"] if abs(x["eps"] - eps) < 0.05]
        if h:
            out.append(float(np.mean(h)))
    return out


# configs[2] GPU runs at a fixed curriculum level (every env starts at eps;
# the per-env 2000-episode bump never fires in these runs), scripts/c3_matched.sh
C3_AT_EPS = {0.0: ["r01_ppo_c3_converge.jsonl", "r02_ppo_c3_eps0_x6_s0.jsonl",
                   "r02_ppo_c3_eps0_x6_s1.jsonl", "r02_ppo_c3_eps0_x6_s2.jsonl",
                   # round 5's kernels (fused first-layer backward, direct finishes)
                   "r05_ppo_c3_eps0_s0.jsonl", "r05_ppo_c3_eps0_s0_final.jsonl"],
             0.5: ["r02_ppo_c3_eps0.5_s0.jsonl", "r02_ppo_c3_eps0.5_s1.jsonl",
                   "r02_ppo_c3_eps0.5_s2.jsonl"],
             1.0: ["r02_ppo_c3_eps1.0_s0.jsonl", "r02_ppo_c3_eps1.0_s1.jsonl",
                   "r02_ppo_c3_eps1.0_s2.jsonl"],
             2.0: ["r02_ppo_c3_eps2.0_s0.jsonl", "r02_ppo_c3_eps2.0_s1.jsonl",
                   "r02_ppo_c3_eps2.0_s2.jsonl"],
             4.8: ["r02_ppo_c3_eps4.8_s0.jsonl", "r02_ppo_c3_eps4.8_s1.jsonl",
                   "r02_ppo_c3_eps4.8_s2.jsonl"]}


RANDOM_POLICY_EP_LEN = 32.0        # SURVEY.md 6 (uniform random actions, eps 0)


def _final(rows, key, n=5):
    return float(np.mean([r[key] for r in rows[-n:]]))


def _anchor_len_at(a, eps):
    out = []
    for s in a["seeds"]:
        h = [x["ep_len_mean"] for x in s["history"] if abs(x["eps"] - eps) < 0.05]
        if h:
            out.append(float(np.mean(h)))
    return out


def test_anchor_and_fixed_eps_runs_crash_early_no_learning_claim():
    """At a fixed eps > 0, from scratch, neither the configs[0] anchor nor the
    configs[2] trainer learns to fly: both end episodes by crashing sooner
    than a random policy would (the reward favours it).  Their returns are
    compared like for like at each curriculum level -- the GPU run's is no
    worse than the best anchor seed's -- but this is NOT a learning claim
    (the learned claims below all require ep_len > 32)."""
    a = _anchor()
    for eps, logs in C3_AT_EPS.items():
        if eps == 0.0:
            continue
        anchor = _anchor_at(a, eps)
        assert len(anchor) == 3, eps
        assert max(_anchor_len_at(a, eps)) < RANDOM_POLICY_EP_LEN, eps
        for name in logs:
            rows = [r for r in _jsonl(name) if "update" in r]
            assert _final(rows, "ep_len_mean") < RANDOM_POLICY_EP_LEN, (eps, name)
            assert _final(rows, "ep_rew_mean") >= max(anchor), (eps, name, anchor)


# configs[2] with the staged curriculum (eps 0 -> 1.0 by +0.05 every 20
# updates from update 300) and ent_coef 0.01, three seeds
STAGED = ["r03_ppo_c3_staged_ent01_s0", "r03_ppo_c3_staged_ent01_s1",
          "r03_ppo_c3_staged_ent01_s2",
          # round 5's kernels (fused first-layer backward, direct finishes)
          "r05_ppo_c3_staged_ent01_s0", "r05_ppo_c3_staged_ent01_s1",
          # round 6's kernels (16x16x32 x6 GEMMs, record gather)
          "r06_ppo_c3_staged_ent01_s0", "r06_ppo_c3_staged_ent01_s1"]


def _eval(name):
    return json.load(open(os.path.join(ROOT, "profiles", name + "_eval.json")))


def _assert_flies_to_target(rows, eps, ev=None, anchor_per_step=None):
    """The learned hover-to-target claim at curriculum level eps: the last
    logged updates at that level have episodes that run to the step limit
    (> 150 steps, far above a random policy's 32) with a return above 100
    (most steps inside the 5 cm bonus radius), and -- given the evaluation
    file -- so does the trained policy on fresh envs, deterministically and
    sampled."""
    at = [r for r in rows if abs(r["eps_mean"] - eps) < 1e-6]
    assert len(at) >= 10, "too few logged updates at this curriculum level"
    ret, length = _final(at, "ep_rew_mean"), _final(at, "ep_len_mean")
    assert length > RANDOM_POLICY_EP_LEN and length > 150, length
    assert ret > 100, ret
    if anchor_per_step is not None:
        assert ret / length > anchor_per_step
    if ev is not None:
        assert abs(ev["eps"] - eps) < 1e-9
        for mode in ("deterministic", "sampled"):
            e = ev[mode]
            assert e["ep_len_mean"] > 150 and e["crash_frac"] < 0.05, (mode, e)
            assert e["bonus_step_frac"] > 0.5 and e["ep_rew_mean"] > 100, (mode, e)


def test_c3_staged_curriculum_flies_to_the_target_at_eps1():
    """Hover-to-target beyond eps 0: at eps 1.0 (targets up to (1, 1, 2) m from
    the (+-0.5, +-0.5, 1) start) every seed's episodes run to the step limit
    and most steps are inside the 5 cm bonus radius -- in training (sampled
    actions) and in a deterministic evaluation on 65,536 fresh envs (test.py's
    predict(deterministic=True)).  Its return and per-step reward beat the
    anchor's at the same eps (-0.27 .. -0.30 over ~23-step episodes)."""
    a = _anchor()
    anchor_per_step = max(r / l for r, l in zip(_anchor_at(a, 1.0), _anchor_len_at(a, 1.0)))
    for name in STAGED:
        rows = [r for r in _jsonl(name + ".jsonl") if "update" in r]
        _assert_flies_to_target(rows, 1.0, _eval(name), anchor_per_step)


def test_c3_staged_to_eps48_beats_the_anchor_end_point():
    """The anchor's own end point (eps 4.8 at 2e6 steps, return -0.81 with
    17-18-step episodes): the staged configs[2] run carried on to eps 4.8
    (+0.1 every 10 updates) flies to the target there, deterministically."""
    a = _anchor()
    rows = [r for r in _jsonl("r03_ppo_c3_staged_ent01_to48_s0.jsonl") if "update" in r]
    per_step = max(s["final_ep_rew_mean"] / s["final_ep_len_mean"] for s in a["seeds"])
    _assert_flies_to_target(rows, 4.8, _eval("r03_ppo_c3_staged_ent01_to48_s0"), per_step)
    assert _final([r for r in rows if abs(r["eps_mean"] - 4.8) < 1e-6], "ep_rew_mean") > \
        a["mean_final_return"] + 100


def test_learned_claims_fail_on_an_early_crash_policy():
    """The guard itself: logs of policies that crash early are rejected by
    the learned-claim check whatever their return -- the r02 fixed-eps runs
    at eps 1.0, and a synthetic log with a high return over 17-step
    episodes."""
    import pytest
    for name in C3_AT_EPS[1.0]:
        rows = [dict(r, eps_mean=1.0) for r in _jsonl(name) if "update" in r]
        with pytest.raises(AssertionError):
            _assert_flies_to_target(rows, 1.0)
    crash = [{"update": u, "ep_rew_mean": 150.0, "ep_len_mean": 17.0, "eps_mean": 1.0}
             for u in range(20)]
    with pytest.raises(AssertionError):
        _assert_flies_to_target(crash, 1.0)


def test_c3_at_eps0_learns_to_hover():
    """At eps 0 (target fixed at (0,0,1)) the configs[2] trainer learns the
    hover-to-target policy: episodes run to the 200-step limit mostly and the
    +1 bonus within 5 cm dominates the return."""
    for name in C3_AT_EPS[0.0]:
        rows = [r for r in _jsonl(name) if "update" in r]
        final = np.mean([r["ep_rew_mean"] for r in rows[-5:]])
        assert final > 100 and rows[-1]["ep_len_mean"] > 150, name
        assert _final(rows, "ep_len_mean") > RANDOM_POLICY_EP_LEN, name


def test_c1_on_gpu_tracks_the_cpu_restatement():
    """Same algorithm and config on both sides: the GPU trainer's learning
    curve on configs[0] stays inside the CPU seeds' band (+-0.15)."""
    a = _anchor()
    gpu = {r["timesteps"]: r["ep_rew_mean"] for r in _jsonl("r01_ppo_c1_gpu.jsonl")
           if "update" in r}
    for ts in (409600, 1024000, 1638400):
        g = min(gpu, key=lambda t: abs(t - ts))
        cpu = [min(s["history"], key=lambda h: abs(h["timesteps"] - ts))["ep_rew_mean"]
               for s in a["seeds"]]
        assert min(cpu) - 0.15 <= gpu[g] <= max(cpu) + 0.15, (ts, gpu[g], cpu)


def test_moving_curriculum_at_configs4_per_gpu_size():
    """configs[4]'s per-GPU slice (131,072 moving-target envs, 2x256, the
    staged schedule 350:0.05 ... 750:0.4; profiles/r02_ppo_moving_131072.jsonl):
    at eps 0 the trainer learns to hover (the variant is the gym env there),
    and once the target moves the episodes stay long (the drone keeps flying
    and following) while the 5 cm bonus gets rarer."""
    rows = [r for r in _jsonl("r02_ppo_moving_131072.jsonl") if "update" in r]
    at = {r["update"]: r for r in rows}
    assert at[330]["ep_rew_mean"] > 100 and at[330]["ep_len_mean"] > 150
    moving = [r for r in rows if r["update"] >= 450]
    assert len(moving) >= 30
    assert min(r["ep_len_mean"] for r in moving) > 150
