"""Copy the judged artefacts of a GPU session from gpurun_out/ to profiles/.

  profiles/<round>_kernel_stats.csv     rocprofv3 --kernel-trace --stats of
                                        `python bench.py --no-cpu-baseline`
  profiles/<round>_pmc_<tag>.json       per-dispatch counter averages
  profiles/traffic.json                 HBM bytes per env_step launch, read
                                        by bench.py for roofline.traffic
  profiles/<round>_bench[_extra].json   the bench.py JSON lines of the session
  profiles/<round>_pmc_rollout.json     the K-step rollout kernel's PMC summary
  profiles/<round>_pmc_x6.json          the x6 GEMM's PMC summary
  (+ the headline rollout kernel's traffic into traffic.json, traffic_update.py)
Usage: python scripts/make_profiles.py r01
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
out = os.path.join(ROOT, "profiles")
os.makedirs(out, exist_ok=True)
src = os.path.join(ROOT, "gpurun_out")
ks = os.path.join(src, "prof", "run_kernel_stats.csv")
if os.path.exists(ks):
    shutil.copy(ks, os.path.join(out, f"{rnd}_kernel_stats.csv"))
for name in ("bench.json", "bench_extra.json", "bench_steps20.json"):   # the bench lines
    if os.path.exists(os.path.join(src, name)):
        shutil.copy(os.path.join(src, name), os.path.join(out, f"{rnd}_{name}"))
traffic = {}
tpath = os.path.join(out, "traffic.json")
if os.path.exists(tpath):
    traffic = json.load(open(tpath))
for tag, key, n in (("n65536", "f64_65536", 65536), ("n4m", "f64_4194304", 4194304)):
    d = os.path.join(src, f"pmc_{tag}")
    if not os.path.isdir(d):
        continue
    js = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), d,
                         "env_step_kernel<double"], capture_output=True, text=True,
                        check=True).stdout
    m = json.loads(js)
    json.dump(m, open(os.path.join(out, f"{rnd}_pmc_{tag}.json"), "w"), indent=1, sort_keys=True)
    if "fetch_bytes_x2" in m and "write_bytes" in m:
        hbm = m["fetch_bytes_x2"] + m["write_bytes"]
        traffic[key] = {"hbm_bytes_per_launch": round(hbm),
                        "read_bytes": round(m["fetch_bytes_x2"]),
                        "write_bytes": round(m["write_bytes"]),
                        "algorithmic_bytes_per_launch": 305 * n,
                        "source": f"profiles/{rnd}_pmc_{tag}.json (FETCH_SIZE x2 gfx950 "
                                  "correction + WRITE_SIZE, KiB -> B)"}
rs = os.path.join(src, "pmc_rollout", "summary.json")     # scripts/micro/rollout_pmc.sh
if os.path.exists(rs):
    shutil.copy(rs, os.path.join(out, f"{rnd}_pmc_rollout.json"))
gx = os.path.join(src, "pmc_gx6", "summary.json")         # scripts/micro/gemm_x6_pmc.sh
if os.path.exists(gx):
    shutil.copy(gx, os.path.join(out, f"{rnd}_pmc_x6.json"))
json.dump(traffic, open(tpath, "w"), indent=1, sort_keys=True)
rt = os.path.join(src, "pmc_rollout_traffic")            # scripts/rollout_traffic.sh
if os.path.isdir(rt):
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "traffic_update.py"), rt],
                   check=True)
print(json.dumps(traffic, indent=1))
