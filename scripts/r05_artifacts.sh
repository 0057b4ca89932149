#!/bin/bash
# Round 5's judged artefacts, session 1 (the profiles bench.py reads):
#   GPU tests and smoke; a rocprofv3 kernel trace of K = 32 headline launches
#   plus 2 PPO updates (kernel stats + the rollout kernel split by grid); the
#   rollout PMC passes; the rollout HBM traffic passes; the x6 GEMMs' and the
#   fused first-layer kernel's PMC passes.
# Session 2 (after scripts/provenance.py record): the bench lines.
#   bash scripts/r05_artifacts.sh prof | bench
# Each GPU step has its own time limit; a crash / abort / timeout ends it.
cd "$(dirname "$0")/.."
OUT=gpurun_out/r5fin
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
if [ "${1:-prof}" = prof ]; then
  step pytest_gpu 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  rm -rf "$PWD/$OUT/ks"
  step kstats 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/ks" -o run \
      -- python3 "$PWD/bench.py" --steps 640 --warmup 64 --ppo-updates 2 --no-cpu-baseline
  step gridstats 60 python3 scripts/kernel_grid_stats.py "$OUT/ks/run_kernel_trace.csv" \
      "$OUT/rollout_grid_stats.json" env_rollout
  rm -f "$OUT"/ks/*kernel_trace.csv
  step pmc_rollout 300 bash scripts/micro/rollout_pmc.sh
  step rollout_traffic 500 bash scripts/rollout_traffic.sh
  step pmc_x6 300 bash scripts/micro/gemm_x6_pmc.sh
  step pmc_fl 300 env FL=1 bash scripts/micro/gemm_x6_pmc.sh
fi
if [ "${1:-prof}" = bench ]; then
  step bench 400 python bench.py
  grep '^{' $OUT/bench.log > $OUT/bench.json
  step bench_steps20_a 300 python bench.py --steps 20 --warmup 5
  grep '^{' $OUT/bench_steps20_a.log > $OUT/bench_steps20_a.json
  step bench_steps20_b 300 python bench.py --steps 20 --warmup 5
  grep '^{' $OUT/bench_steps20_b.log > $OUT/bench_steps20_b.json
  step bench_extra 400 python bench.py --no-cpu-baseline --extra
  grep '^{' $OUT/bench_extra.log | tail -1 > $OUT/bench_extra.json
fi
echo "== done"
