#!/bin/bash
# gather_minibatch with several rows per thread: tests, then the PPO bench leg
ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_ppo_kernels_gpu.py tests/test_ppo_gpu.py > gpurun_out/u_test.log 2>&1; rc=$?
tail -3 gpurun_out/u_test.log; [ $rc -eq 0 ] || exit $rc
for lib in new old new old; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $lib == old ] && L=$PWD/scripts/micro/build/gold/libdronerl.so
  DRONERL_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --rollout-k 0 --no-companion --ppo-updates 5 > gpurun_out/u_$lib.log 2>&1 || exit $?
  grep '^{' gpurun_out/u_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print('$lib', p['updates_per_s'], {k: v['us'] for k, v in p['roofline']['kernels_per_minibatch'].items() if 'gather' in k})"
done
