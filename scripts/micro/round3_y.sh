#!/bin/bash
# rational tanh (DR_TANH_RAT=1) A/B: the PPO GPU tests on the variant, the
# kernel times (rocprofv3), then PPO updates/s of both builds, alternating
ulimit -c 0
mkdir -p gpurun_out
R=$PWD/scripts/micro/build/rat/libdronerl.so
DRONERL_LIB=$R timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_ppo_kernels_gpu.py tests/test_gemm_x6_gpu.py tests/test_ppo_flagship_parity_gpu.py \
  tests/test_ppo_gpu.py > gpurun_out/y_test.log 2>&1; rc=$?
tail -3 gpurun_out/y_test.log; [ $rc -eq 0 ] || exit $rc
KERN="linear_tanh ppo_head" bash scripts/micro/ab_ppo_kern.sh run base rat || exit $?
for lib in new old new old; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $lib == new ] && L=$R
  DRONERL_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --rollout-k 0 --no-companion --ppo-updates 8 > gpurun_out/y_$lib.log 2>&1 || exit $?
  grep '^{' gpurun_out/y_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print('$lib', p['updates_per_s'], {k: v['us'] for k, v in p['roofline']['kernels_per_minibatch'].items()})"
done
