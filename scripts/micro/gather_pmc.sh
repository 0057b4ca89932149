#!/bin/bash
# PMC passes over scripts/micro/gather_pmc.py 1 (one eager configs[2] PPO
# iteration, 1 epoch = 32 minibatch gathers of 65,536 rows), one counter
# group per run, plus a --kernel-trace --stats pass; summary of the
# gather_records_kernel dispatches into gpurun_out/pmc_gather/summary.json.
cd "$(dirname "$0")/../.."
OUT=$PWD/gpurun_out/pmc_gather
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$PWD/scripts/micro/gather_pmc.py" 1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks" -o run \
    -- python3 "$PWD/scripts/micro/gather_pmc.py" 1 > "$OUT/ks.log" 2>&1
rc=$?; echo "kernel trace rc=$rc"
if [ $rc -ne 0 ]; then tail -5 "$OUT/ks.log"; exit $rc; fi
rm -f "$OUT"/ks/*kernel_trace.csv
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
K = "gather_records_kernel"
acc = collections.defaultdict(list)
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if K in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
us = None
for r in csv.DictReader(open(out + "/ks/run_kernel_stats.csv")):
    if K in r["Name"]:
        us = float(r["AverageNs"]) / 1e3
rows, rec = 65536, 128
res = {"workload": "scripts/micro/gather_pmc.py 1: one eager configs[2] PPO iteration (65,536 envs, "
                   "T = 32, 2x256, 1 epoch = 32 minibatches of 65,536 rows); rocprofv3 --pmc passes "
                   "and a --kernel-trace --stats pass (scripts/micro/gather_pmc.sh), per-dispatch "
                   "averages over the gather_records_kernel dispatches",
       "counters_per_dispatch": {("%s_KiB" % k if k in ("FETCH_SIZE", "WRITE_SIZE") else k):
                                 round(v, 1) for k, v in sorted(m.items())},
       "dispatches": max((len(v) for v in acc.values()), default=0),
       "kernel_us_mean": round(us, 2) if us else None,
       "algorithmic_bytes": {"read": rows * (rec + 4),
                             "write": rows * (60 + 16 + 12),
                             "basis": "per minibatch row one 128-B rollout record (obs, action, "
                                      "old log-prob, advantage, return) read at a random rollout "
                                      "row + the 4-B row index; 60 B obs + 16 B action + 12 B aux "
                                      "written contiguously"}}
if "FETCH_SIZE" in m:
    res["fetch_bytes_x2"] = round(m["FETCH_SIZE"] * 2048)
if "WRITE_SIZE" in m:
    res["write_bytes"] = round(m["WRITE_SIZE"] * 1024)
if "TCP_TCC_READ_REQ_sum" in m:
    res["tcc_read_req_per_row"] = round(m["TCP_TCC_READ_REQ_sum"] / rows, 2)
if us and "fetch_bytes_x2" in res and "write_bytes" in res:
    mv = res["fetch_bytes_x2"] + res["write_bytes"]
    alg = res["algorithmic_bytes"]["read"] + res["algorithmic_bytes"]["write"]
    res["moved_bytes"] = mv
    res["moved_tb_s"] = round(mv / us / 1e6, 2)
    res["algorithmic_frac_of_8tb_s"] = round(alg / us / 1e6 / 8.0, 3)
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "workload"}))
PY
