#!/bin/bash
# round3_v (two physics waves per SIMD) + the launch-path host walls
ulimit -c 0
mkdir -p gpurun_out
bash scripts/micro/round3_v.sh || exit $?
timeout -k 10 300 python scripts/micro/launch_paths.py > gpurun_out/w_paths.log 2>&1; rc=$?
cat gpurun_out/w_paths.log; exit $rc
