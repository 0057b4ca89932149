#!/bin/bash
# Round 5: the PPO row loss with reciprocal products (DR_LOSS_RCP=1): head
# kernel timing (head_bench.py, alternating with the baseline build), then
# the PPO kernel / trainer parity tests on the variant library.
cd "$(dirname "$0")/../.."
O=gpurun_out/r5rcp; mkdir -p $O
export PYTHONPATH=$PWD
for i in 1 2 3; do
  for v in hbase hrcp; do
    timeout -k 10 120 env DRONERL_LIB=$PWD/scripts/micro/build/lib_$v.so python scripts/micro/head_bench.py >> $O/h_$v.json 2>$O/h_$v.err || exit 1
  done
done
for v in hbase hrcp; do echo "$v: $(cat $O/h_$v.json | tr '\n' ' ')"; done
timeout -k 10 600 env DRONERL_LIB=$PWD/scripts/micro/build/lib_hrcp.so python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ppo_kernels_gpu.py tests/test_ppo_flagship_parity_gpu.py "tests/test_ppo_gpu.py::test_rollout_and_first_epoch_share_one_gemm_path" > $O/tests_hrcp.log 2>&1
rc=$?; tail -3 $O/tests_hrcp.log; exit $rc
