#!/bin/bash
# Everything the round's judged artefacts come from, in two GPU sessions
# (each well inside gpurun's 20-minute limit):
#   bash scripts/round_artifacts.sh main   GPU tests, smoke, the default bench
#                                          line, the --extra bench, a rocprofv3
#                                          kernel trace of the default bench
#   bash scripts/round_artifacts.sh pmc    the PMC passes for the env kernel
# Each GPU step has its own time limit; a crash/abort/timeout ends the script.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal rc=$rc in $name: stopping"; exit $rc
  fi
  return 0
}
WHAT=${1:-main}
if [ "$WHAT" = main ]; then
  step pytest_gpu 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  step bench 300 python bench.py
  grep '^{' $OUT/bench.log > $OUT/bench.json || true
  step bench_steps20 300 python bench.py --steps 20 --warmup 5
  grep '^{' $OUT/bench_steps20.log > $OUT/bench_steps20.json || true
  step bench_extra 300 python bench.py --no-cpu-baseline --extra
  grep '^{' $OUT/bench_extra.log > $OUT/bench_extra.json || true
  export TMPDIR=/tmp
  rm -rf "$PWD/$OUT/prof"
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$OUT/prof" -o run -- python3 "$PWD/bench.py" --no-cpu-baseline --no-companion
  rm -f "$PWD/$OUT"/prof/*kernel_trace.csv   # per-dispatch rows: large, not judged
fi
if [ "$WHAT" = pmc ]; then
  step pmc_n65536 400 bash scripts/pmc.sh n65536 --steps 50 --ppo-updates 0
  step pmc_n4m 400 bash scripts/pmc.sh n4m --envs 4194304 --steps 20 --warmup 5 --ppo-updates 0
  step pmc_rollout 300 bash scripts/micro/rollout_pmc.sh
  step rollout_traffic 400 bash scripts/rollout_traffic.sh
  step pmc_x6 300 bash scripts/micro/gemm_x6_pmc.sh
fi
echo "== done"
