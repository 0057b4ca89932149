#!/bin/bash
# Round 5: the rollout kernel A/B (lib_base = the kernels before the change,
# the working tree's libdronerl.so after), alternating on one box, after the
# whole GPU suite on the working tree.  Usage: r5_rollout_ab.sh TAG [nosuite]
cd "$(dirname "$0")/../.."
T=${1:-r5c}; O=gpurun_out/$T; mkdir -p $O
B=$PWD/scripts/micro/build/lib_${BASE:-base}.so
export PYTHONPATH=$PWD
if [ "$2" != "nosuite" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
  tail -2 $O/suite.log
fi
for i in 1 2 3; do
  timeout -k 10 120 env DRONERL_LIB=$B python scripts/micro/rollout_bench.py --envs 65536 --ks 20 32 --act-sets 8 > $O/ro_base_$i.json 2>$O/ro_base_$i.err || exit 1
  timeout -k 10 120 python scripts/micro/rollout_bench.py --envs 65536 --ks 20 32 --act-sets 8 > $O/ro_new_$i.json 2>$O/ro_new_$i.err || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --no-companion > $O/bench20.json 2> $O/bench20.err || exit 1
echo done
