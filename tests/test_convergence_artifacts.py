"""The convergence claim (configs[2] must reach at least the
return the SB3-default CPU PPO reaches on configs[0] at 2e6 steps), compared
at matched curriculum levels (the anchor ends at eps 4.8), checked on
committed artefacts (CPU only; every log is a builder run):

  tests/golden/c1_anchor.json          oracle/sb3_c1.py, 3 seeds, 2e6 steps
  profiles/r01_ppo_c3_converge.jsonl   GPU PPO, 65,536 envs, 2x256 (train.py), eps 0
  profiles/r02_ppo_c3_eps*.jsonl       the same at eps 0.5 / 1 / 2 / 4.8 (c3_matched.sh),
                                       and at eps 0 on the x6 GEMMs (r02_ppo_c3_eps0_x6_s0..2)
  profiles/r01_ppo_c1_gpu.jsonl        GPU PPO with SB3 defaults on 1 env
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
                   "r02_ppo_c3_eps0_x6_s1.jsonl", "r02_ppo_c3_eps0_x6_s2.jsonl"],
             0.5: ["r02_ppo_c3_eps0.5_s0.jsonl", "r02_ppo_c3_eps0.5_s1.jsonl",
                   "r02_ppo_c3_eps0.5_s2.jsonl"],
             1.0: ["r02_ppo_c3_eps1.0_s0.jsonl", "r02_ppo_c3_eps1.0_s1.jsonl",
                   "r02_ppo_c3_eps1.0_s2.jsonl"],
             2.0: ["r02_ppo_c3_eps2.0_s0.jsonl", "r02_ppo_c3_eps2.0_s1.jsonl",
                   "r02_ppo_c3_eps2.0_s2.jsonl"],
             4.8: ["r02_ppo_c3_eps4.8_s0.jsonl", "r02_ppo_c3_eps4.8_s1.jsonl",
                   "r02_ppo_c3_eps4.8_s2.jsonl"]}


def test_c3_at_matched_curriculum_level_beats_the_c1_anchor():
    """Like for like: at each curriculum level the configs[0] anchor (SB3
    defaults, 1 env, CPU) passes through -- eps 0 at the start, 4.8 at 2e6
    steps -- the configs[2] GPU trainer run at that same level ends at a
    return no worse than the best anchor seed at it."""
    a = _anchor()
    for eps, logs in C3_AT_EPS.items():
        anchor = _anchor_at(a, eps)
        assert len(anchor) == 3, eps
        for name in logs:
            rows = [r for r in _jsonl(name) if "update" in r]
            final = float(np.mean([r["ep_rew_mean"] for r in rows[-5:]]))
            assert final >= max(anchor), (eps, name, final, anchor)
    # the anchor's own end point (eps 4.8, 2e6 steps) against the C3 run at 4.8
    rows = [r for r in _jsonl(C3_AT_EPS[4.8][0]) if "update" in r]
    assert np.mean([r["ep_rew_mean"] for r in rows[-5:]]) >= a["mean_final_return"]


def test_c3_at_eps0_learns_to_hover():
    """At eps 0 (target fixed at (0,0,1)) the configs[2] trainer learns the
    hover-to-target policy: episodes run to the 200-step limit mostly and the
    +1 bonus within 5 cm dominates the return."""
    for name in C3_AT_EPS[0.0]:
        rows = [r for r in _jsonl(name) if "update" in r]
        final = np.mean([r["ep_rew_mean"] for r in rows[-5:]])
        assert final > 100 and rows[-1]["ep_len_mean"] > 150, name


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
