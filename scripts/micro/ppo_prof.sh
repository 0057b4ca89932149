#!/bin/bash
# rocprofv3 kernel stats of the PPO part of bench.py for one or more library
# builds (DRONERL_LIB), top kernels by total time, per-call average in us.
# Usage: bash scripts/micro/ppo_prof.sh [lib.so ...]   (default: the product)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
libs=("$@"); [ ${#libs[@]} -eq 0 ] && libs=("$PWD/drone_rl_amd/libdronerl.so")
i=0
for lib in "${libs[@]}"; do
  i=$((i+1)); D=$PWD/gpurun_out/pprof$i; rm -rf $D
  DRONERL_LIB=$(realpath $lib) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run \
    -- python3 $PWD/bench.py --no-cpu-baseline --no-companion --steps 50 --warmup 10 --ppo-updates 3 > $D.log 2>&1 || exit $?
  rm -f $D/*kernel_trace.csv
  echo "== $lib: $(grep -o '"updates_per_s": [0-9.]*' $D.log)"
  python3 - "$D/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.2f} us {float(r['Percentage']):6.2f}%")
PY
done
