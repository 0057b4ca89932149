#!/bin/bash
# split rollout kernel: reset draw-ahead group DR_WS_RA = 4 / 16 vs 8
# (bitwise by construction: the same Philox words, drawn at other steps)
ulimit -c 0
mkdir -p gpurun_out
DRONERL_LIB=$PWD/scripts/micro/build/ra16/libdronerl.so timeout -k 10 300 python -u -m pytest -x -q \
  --timeout 200 --timeout-method thread tests/test_rollout_gpu.py > gpurun_out/ai_test.log 2>&1; rc=$?
tail -2 gpurun_out/ai_test.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in 8 4 16; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $v != 8 ] && L=$PWD/scripts/micro/build/ra$v/libdronerl.so
  DRONERL_LIB=$L timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/ai_rb$v.log 2>&1 || exit 1
  echo "RA $v: $(tail -1 gpurun_out/ai_rb$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["read_us"] for k, v in d.items() if k.startswith("n")})')"
done; done
