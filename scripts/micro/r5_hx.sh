#!/bin/bash
# Round 5: ppo_head_kernel variants (scripts/micro/build_variant.sh) timed
# alternately on one box by scripts/micro/head_bench.py, then the head's
# parity tests on the variant named by $2 (DRONERL_LIB).
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5hx}; mkdir -p $O
shift
export PYTHONPATH=$PWD
for i in 1 2 3; do
  for v in "$@"; do
    timeout -k 10 120 env DRONERL_LIB=$PWD/scripts/micro/build/lib_$v.so python scripts/micro/head_bench.py >> $O/h_$v.json 2>$O/h_$v.err || exit 1
  done
done
for v in "$@"; do echo "$v: $(cat $O/h_$v.json | tr '\n' ' ')"; done
timeout -k 10 300 env DRONERL_LIB=$PWD/scripts/micro/build/lib_$2.so python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ppo_kernels_gpu.py -k "fused_step or deferred_finish or gather_minibatch_equals" > $O/tests_$2.log 2>&1
rc=$?; tail -3 $O/tests_$2.log; exit $rc
