#!/bin/bash
# PMC passes over scripts/micro/gemm_x6_bench.py (one counter group per run);
# with FL=1 over scripts/micro/fl_bench.py instead (the fused input-gradient
# GEMM + first-layer backward, round 5), into gpurun_out/pmc_fl; with HEAD=1
# over scripts/micro/head_bench.py (ppo_head_kernel), into gpurun_out/pmc_head.
cd "$(dirname "$0")/../.."
if [ "${HEAD:-0}" = 1 ]; then
  OUT=$PWD/gpurun_out/pmc_head; PROG="$PWD/scripts/micro/head_bench.py"; export REPS=10
  export PMC_WORKLOAD="scripts/micro/head_bench.py (REPS=10; ppo_head_kernel, 65,536-row minibatch, the trainer's contiguous actions / aux rows), rocprofv3 --pmc, four passes (HEAD=1 scripts/micro/gemm_x6_pmc.sh)"
elif [ "${FL:-0}" = 1 ]; then
  OUT=$PWD/gpurun_out/pmc_fl; PROG="$PWD/scripts/micro/fl_bench.py"; export REPS=10
  export PMC_WORKLOAD="scripts/micro/fl_bench.py (REPS=10; the fused input-gradient GEMM + first-layer backward beside the forward), rocprofv3 --pmc, four passes (FL=1 scripts/micro/gemm_x6_pmc.sh)"
else
  OUT=$PWD/gpurun_out/pmc_gx6; PROG="$PWD/scripts/micro/gemm_x6_bench.py --reps 10"
fi
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 $PROG "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, json, re, sys, collections
out = sys.argv[1]
import os
res = {"workload": os.environ.get("PMC_WORKLOAD",
                                  "scripts/micro/gemm_x6_bench.py --reps 10 (both nets, 65,536 rows: "
                                  "the forward and input-gradient forms of dr_gemm_x6 and the 64-chunk "
                                  "weight gradient; cold inputs), rocprofv3 --pmc, four passes "
                                  "(scripts/micro/gemm_x6_pmc.sh); per-dispatch averages per kernel")}
for key, pat in (("gemm_x6_ws16_kernel", r"gemm_x6_ws16_kernel"),
                 ("gemm_x6_wgrad16_kernel", r"gemm_x6_wgrad16_kernel"),
                 ("gemm_x6_fl16_kernel", r"gemm_x6_fl16_kernel"),
                 ("ppo_head_kernel", r"ppo_head_kernel")):
    acc = collections.defaultdict(list)
    for f in glob.glob(out + "/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if re.search(pat, r["Kernel_Name"]):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not acc:
        continue
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    d = {"counters_per_dispatch": {k: round(v, 1) for k, v in sorted(m.items())},
         "dispatches": max((len(v) for v in acc.values()), default=0)}
    w = m.get("SQ_WAVE_CYCLES")
    if w:
        d["wait_any_frac"] = round(m["SQ_WAIT_ANY"] / w, 3)
        d["wait_inst_any_frac"] = round(m["SQ_WAIT_INST_ANY"] / w, 3)
        d["active_inst_any_frac"] = round(m["SQ_ACTIVE_INST_ANY"] / w, 3)
        if "SQ_WAIT_INST_LDS" in m:
            d["wait_inst_lds_frac"] = round(m["SQ_WAIT_INST_LDS"] / w, 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # MFMA busy cycles are summed over all SIMDs (cycles); GUI_ACTIVE over the 8 XCDs
        per_simd = m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0
        d["mfma_busy_frac"] = round(per_simd / (m["GRBM_GUI_ACTIVE"] / 8.0), 3)
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        # KiB; FETCH_SIZE x 2 on gfx950 (MI355X_MICROARCH.md, HBM / rocprofv3)
        d["hbm_bytes_per_dispatch"] = round(m["FETCH_SIZE"] * 2048 + m["WRITE_SIZE"] * 1024)
    if "SQ_ACTIVE_INST_VALU" in m and "GRBM_GUI_ACTIVE" in m:
        # VALU issue cycles summed over the 1,024 SIMDs, against the busy clock
        d["active_inst_valu_per_simd_over_gui_active"] = round(
            m["SQ_ACTIVE_INST_VALU"] / 1024.0 / (m["GRBM_GUI_ACTIVE"] / 8.0), 3)
        if w:
            d["valu_active_frac_of_wave_cycles"] = round(m["SQ_ACTIVE_INST_VALU"] / w, 3)
    if "SQ_LDS_BANK_CONFLICT" in m:
        d["lds_bank_conflict_cycles"] = m["SQ_LDS_BANK_CONFLICT"]
    res[key] = d
    print(key, json.dumps({k: v for k, v in d.items() if k != "counters_per_dispatch"}))
json.dump(res, open(out + "/summary.json", "w"), indent=1)
PY
