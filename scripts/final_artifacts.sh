#!/bin/bash
# The round's judged artefacts (scripts/collect_round.py copies them into
# profiles/<round>_*), in three GPU sessions, each well inside gpurun's limit:
#   bash scripts/final_artifacts.sh prof    GPU tests, smoke, a rocprofv3 kernel
#                                           trace of K = 32 headline launches +
#                                           2 PPO updates (kernel stats, the
#                                           rollout kernel split by grid)
#   bash scripts/final_artifacts.sh pmc     the rollout / x6 / fused / head /
#                                           gather PMC passes and the rollout
#                                           HBM traffic passes
#   bash scripts/final_artifacts.sh bench   the bench lines (after
#                                           scripts/provenance.py record)
# Each GPU step has its own time limit; a crash / abort / timeout ends it.
cd "$(dirname "$0")/.."
OUT=gpurun_out/fin
mkdir -p $OUT
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
}
export TMPDIR=/tmp
case "${1:-prof}" in
prof)
  step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  rm -rf "$PWD/$OUT/ks"
  step kstats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/ks" -o run \
      -- python3 "$PWD/bench.py" --steps 640 --warmup 64 --ppo-updates 2 --no-cpu-baseline
  step gridstats 60 python3 scripts/kernel_grid_stats.py "$OUT/ks/run_kernel_trace.csv" \
      "$OUT/rollout_grid_stats.json" env_rollout
  rm -f "$OUT"/ks/*kernel_trace.csv
  ;;
pmc)
  step pmc_rollout 300 bash scripts/micro/rollout_pmc.sh
  step rollout_traffic 500 bash scripts/rollout_traffic.sh
  step pmc_x6 300 bash scripts/micro/gemm_x6_pmc.sh
  step pmc_fl 300 env FL=1 bash scripts/micro/gemm_x6_pmc.sh
  step pmc_head 300 env HEAD=1 bash scripts/micro/gemm_x6_pmc.sh
  step pmc_gather 300 bash scripts/micro/gather_pmc.sh
  ;;
bench)
  for b in default:"" steps20_a:"--steps 20 --warmup 5" steps20_b:"--steps 20 --warmup 5" \
           extra:"--no-cpu-baseline --extra"; do
    step bench_${b%%:*} 400 python bench.py ${b#*:}
    grep '^{' $OUT/bench_${b%%:*}.log | tail -1 > $OUT/bench_${b%%:*}.json
  done
  ;;
esac
echo "== done"
