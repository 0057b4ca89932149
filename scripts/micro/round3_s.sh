#!/bin/bash
# overlapped minibatch gather: parity test, then in-process A/B (both orders)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_ppo_gpu.py -k "overlapped or graphs_follow" > gpurun_out/s_test.log 2>&1 &&
timeout -k 10 300 python -u scripts/micro/ppo_ab_inproc.py overlap_gather=False overlap_gather=True \
  > gpurun_out/s_ab1.log 2>&1 &&
timeout -k 10 300 python -u scripts/micro/ppo_ab_inproc.py overlap_gather=True overlap_gather=False \
  > gpurun_out/s_ab2.log 2>&1
rc=$?
tail -5 gpurun_out/s_test.log; cat gpurun_out/s_ab*.log
exit $rc
