#!/bin/bash
# In-process A/B of libdronerl.so builds (scripts/micro/ab.py) at three sizes.
# Usage: bash scripts/micro/ab_run.sh lib1.so lib2.so ...
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
i=0
for spec in "65536 200 25" "131072 200 25" "4194304 50 9"; do
  read n k reps <<< "$spec"
  i=$((i+1))
  timeout -k 10 300 python scripts/micro/ab.py "$@" --n $n --k $k --reps $reps > gpurun_out/ab$i.log 2>&1 || exit $?
  echo "n=$n $(grep '^{' gpurun_out/ab$i.log)"
done
