"""Copy the judged artefacts of scripts/final_artifacts.sh's GPU sessions from
gpurun_out/ to profiles/ (runs here, on the CPU):

  profiles/<round>_gpu_suite_final.log    pytest -m gpu (prof session)
  profiles/<round>_kernel_stats.csv       rocprofv3 --kernel-trace --stats of
                                          K = 32 headline launches + 2 PPO
                                          updates (bench.py reads it)
  profiles/<round>_rollout_grid_stats.json  the rollout kernel split by grid
  profiles/<round>_pmc_rollout.json       the K-step rollout kernel's PMC
  profiles/<round>_pmc_{x6,fl,head}.json  the x6 GEMMs' / fused input-gradient
                                          / head kernels' PMC
  profiles/<round>_gather_pmc.json        the minibatch record gather's PMC
  profiles/traffic.json                   the headline kernel's HBM bytes per
                                          launch (scripts/traffic_update.py)
  profiles/<round>_bench_*.json           the bench lines (bench session)
Then stamp them: python scripts/provenance.py record <the files listed>.

Usage: python scripts/make_profiles.py r06
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r06"
    out = os.path.join(ROOT, "profiles")
    src = os.path.join(ROOT, "gpurun_out")
    fin = os.path.join(src, "fin")
    pairs = [
        (os.path.join(fin, "pytest_gpu.log"), f"{rnd}_gpu_suite_final.log"),
        (os.path.join(fin, "ks", "run_kernel_stats.csv"), f"{rnd}_kernel_stats.csv"),
        (os.path.join(fin, "rollout_grid_stats.json"), f"{rnd}_rollout_grid_stats.json"),
        (os.path.join(src, "pmc_rollout", "summary.json"), f"{rnd}_pmc_rollout.json"),
        (os.path.join(src, "pmc_gx6", "summary.json"), f"{rnd}_pmc_x6.json"),
        (os.path.join(src, "pmc_fl", "summary.json"), f"{rnd}_pmc_fl.json"),
        (os.path.join(src, "pmc_head", "summary.json"), f"{rnd}_pmc_head.json"),
        (os.path.join(src, "pmc_gather", "summary.json"), f"{rnd}_gather_pmc.json"),
    ]
    for b in ("default", "steps20_a", "steps20_b", "extra"):
        pairs.append((os.path.join(fin, f"bench_{b}.json"), f"{rnd}_bench_{b}.json"))
    done = []
    for s, d in pairs:
        if os.path.exists(s) and os.path.getsize(s) > 0:
            dst = os.path.join(out, d)
            keep = {}
            if d.endswith(".json") and os.path.exists(dst):
                # blocks added to a committed summary by hand (an A/B record
                # beside the counters) survive a re-copy of the counters
                try:
                    old, new = json.load(open(dst)), json.load(open(s))
                    if isinstance(old, dict) and isinstance(new, dict):
                        keep = {k: v for k, v in old.items() if k not in new and k.endswith("_ab")}
                except ValueError:
                    keep = {}
            shutil.copy(s, dst)
            if keep:
                merged = json.load(open(dst))
                merged.update(keep)
                json.dump(merged, open(dst, "w"), indent=1)
            done.append(os.path.join("profiles", d))
    rt = os.path.join(src, "pmc_rollout_traffic")            # scripts/rollout_traffic.sh
    if os.path.isdir(rt):
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "traffic_update.py"), rt],
                       check=True)
        done.append("profiles/traffic.json")
    print(" ".join(done))


if __name__ == "__main__":
    main()
