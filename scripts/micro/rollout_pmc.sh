#!/bin/bash
# PMC passes over scripts/micro/rollout_bench.py at 65,536 envs, K = 32
# (one counter group per run): VALU instruction count and issue occupancy
# of the rollout kernel (env_rollout_ws_kernel: half its waves are memory
# waves, so the per-physics-wave figures divide by SQ_WAVES / 2 and count
# the memory waves' few VALU too -- upper bounds; env_rollout_kernel with
# DRONERL_ROLLOUT_WS=0).
cd "$(dirname "$0")/../.."
OUT=$PWD/gpurun_out/pmc_rollout
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$PWD/scripts/micro/rollout_bench.py" --envs 65536 --ks 32 --reps 5 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, json, re, sys, collections
out = sys.argv[1]
res = {"workload": "scripts/micro/rollout_bench.py --envs 65536 --ks 32 --reps 5 (f64 gym, "
                   "one action set), rocprofv3 --pmc, two passes (scripts/micro/rollout_pmc.sh)"}
for tag in ("false", "true"):   # actions from HBM / in-kernel random policy
    acc = collections.defaultdict(list)
    ws = ""
    pat = re.compile(r"env_rollout(_ws|_ab)?_kernel<double, (0, )?(64, )?" + tag + ">")
    for f in glob.glob(out + "/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            mt = pat.search(r["Kernel_Name"])
            if mt:
                ws = ws or mt.group(1) or ""
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    w, K = m["SQ_WAVES"], 32
    # physics waves: half of the warp-specialised kernel's, two thirds of the
    # split kernel's (translation + rotation)
    pw = w / 2 if ws == "_ws" else (2 * w / 3 if ws == "_ab" else w)
    res["random_policy_in_kernel" if tag == "true" else "actions_from_hbm"] = {
        "kernel": "env_rollout%s_kernel" % ws,
        "counters_per_launch": {k: round(v, 1) for k, v in sorted(m.items())},
        "valu_insts_per_wave_step": round(m["SQ_INSTS_VALU"] / pw / K, 1),
        "salu_insts_per_wave_step": round(m["SQ_INSTS_SALU"] / pw / K, 1),
        "valu_active_frac_of_wave_cycles": round(m["SQ_ACTIVE_INST_VALU"] /
                                                 (m["SQ_WAVE_CYCLES"] * pw / w), 3),
        "any_active_frac": round(m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3),
        "wait_any_frac": round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3),
        "wait_inst_any_frac": round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3),
        "quad_cycles_per_valu_inst": round(m["SQ_ACTIVE_INST_VALU"] / m["SQ_INSTS_VALU"], 3),
        "fetch_bytes_x2": round(m["FETCH_SIZE"] * 1024 * 2)}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "counters_per_launch"}
                  for k, v in res.items() if k != "workload"}, indent=1))
PY
