#!/bin/bash
# split rollout kernel with the yaw sincos moved to the translation wave vs
# the previous split (all three sincos on the rotation wave): parity tests,
# then rollout-kernel and headline timings alternating
ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_rollout_gpu.py > gpurun_out/ae_test.log 2>&1; rc=$?
tail -2 gpurun_out/ae_test.log; [ $rc -eq 0 ] || exit $rc
DRONERL_ROLLOUT_AB=1 DRONERL_ROLLOUT_WS=1 PYTHONPATH=$PWD timeout -k 10 120 python tests/rollout_form_worker.py gym 131392 37 || exit 1
for rep in 1 2 3; do for v in new old; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $v == old ] && L=$PWD/scripts/micro/build/abold/libdronerl.so
  DRONERL_LIB=$L timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/ae_rb$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/ae_rb$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["read_us"] for k, v in d.items() if k.startswith("n")})')"
  DRONERL_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion --ppo-updates 0 --rollout-k 0 \
    > gpurun_out/ae_b$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/ae_b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v headline', d['value'], d['roofline']['avg_launch_us'])"
done; done
