#!/bin/bash
# split rollout kernel: ep_num / eps held in registers through the launch
# (DR_AB_EPREG=1) vs a global store per reset; parity tests, then timings
ulimit -c 0
mkdir -p gpurun_out
M=$PWD/scripts/micro/build/epr/libdronerl.so
DRONERL_LIB=$M timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_rollout_gpu.py > gpurun_out/ah_test.log 2>&1; rc=$?
tail -2 gpurun_out/ah_test.log; [ $rc -eq 0 ] || exit $rc
DRONERL_LIB=$M DRONERL_ROLLOUT_AB=1 DRONERL_ROLLOUT_WS=1 PYTHONPATH=$PWD timeout -k 10 120 python tests/rollout_form_worker.py gym 131392 37 || exit 1
for rep in 1 2 3; do for v in epr base; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $v == epr ] && L=$M
  DRONERL_LIB=$L timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/ah_rb$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/ah_rb$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["read_us"] for k, v in d.items() if k.startswith("n")})')"
done; done
