#!/bin/bash
# One GPU-box session: tests, smoke, bench, rocprof kernel trace.
# Each GPU step has its own time limit; a crash/abort/timeout (exit >= 124 or
# a signal) ends the script, a plain test failure (exit 1) does not.
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal rc=$rc in $name: stopping"; exit $rc
  fi
  return 0
}
WHAT=${1:-all}
if [[ $WHAT == all || $WHAT == test ]]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
  step bench 600 python bench.py --extra
  cat $OUT/bench.log | grep '^{' > $OUT/bench.json || true
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$OUT/prof" -o run -- python3 "$PWD/bench.py" --no-cpu-baseline --no-companion
fi
echo "== done"
