"""Assemble tests/golden/c1_anchor.json from the three seed runs of
oracle/sb3_c1.py (TEST INFRASTRUCTURE: the CPU restatement of SB3-default PPO
on configs[0], SURVEY.md 8c's anchor).

  for s in 0 1 2; do python -m oracle.sb3_c1 --steps 2000000 --seed $s \\
      --out /tmp/anchor/seed$s.json; done
  python -m oracle.make_c1_anchor /tmp/anchor/seed{0,1,2}.json

Per history row it keeps timesteps, ep_rew_mean, ep_len_mean (mean length of
the last 100 episodes; added in round 3) and eps."""
import json
import os
import sys

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                   "golden", "c1_anchor.json")


def main(paths):
    seeds = []
    for p in paths:
        r = json.load(open(p))
        seeds.append({"seed": r["seed"], "steps": r["steps"],
                      "final_ep_rew_mean": r["final_ep_rew_mean"],
                      "final_ep_len_mean": r["final_ep_len_mean"], "final_eps": r["final_eps"],
                      "episodes": r["episodes"], "elapsed_s": r["elapsed_s"],
                      "history": [{"timesteps": h["timesteps"], "ep_rew_mean": h["ep_rew_mean"],
                                   "ep_len_mean": h["ep_len_mean"], "eps": h["eps"]}
                                  for h in r["history"]]})
    finals = [s["final_ep_rew_mean"] for s in seeds]
    out = {"description": "Config-1 anchor (SURVEY.md 8c 'hover-to-target return'): CPU PPO "
                          "with SB3 defaults (oracle/sb3_c1.py) on 1 DroneGymEnv-equivalent env "
                          "for 2e6 steps, 3 seeds, torch set_num_threads(1), build container "
                          "CPU. final_ep_rew_mean / final_ep_len_mean = mean return / length "
                          "of the last 100 episodes.",
           "generator": "python -m oracle.sb3_c1 --steps 2000000 --seed {0,1,2} --out ...; "
                        "python -m oracle.make_c1_anchor ...",
           "seeds": seeds, "anchor_return": max(finals),
           "mean_final_return": float(np.mean(finals))}
    json.dump(out, open(OUT, "w"))
    print(json.dumps({k: v for k, v in out.items() if k != "seeds"}))


if __name__ == "__main__":
    main(sys.argv[1:])
