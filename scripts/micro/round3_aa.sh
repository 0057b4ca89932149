#!/bin/bash
# ws rollout action look-ahead D (DR_WS_AHEAD) A/B: the rollout parity tests
# on each variant, then the default headline (1,000 steps) alternating
ulimit -c 0
mkdir -p gpurun_out
for d in 4 6; do
  DRONERL_LIB=$PWD/scripts/micro/build/ah$d/libdronerl.so timeout -k 10 300 python -u -m pytest -x -q \
    --timeout 200 --timeout-method thread tests/test_rollout_gpu.py > gpurun_out/aa_t$d.log 2>&1 || { tail -20 gpurun_out/aa_t$d.log; exit 1; }
  echo "D=$d tests: $(tail -1 gpurun_out/aa_t$d.log)"
done
for rep in 1 2; do for d in 2 4 6; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $d != 2 ] && L=$PWD/scripts/micro/build/ah$d/libdronerl.so
  DRONERL_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion --ppo-updates 0 \
    > gpurun_out/aa_b$d.log 2>&1 || exit 1
  grep '^{' gpurun_out/aa_b$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['rollout_kernel']; print('D=$d', d['value'], d['roofline']['avg_launch_us'], r['actions_from_hbm']['avg_launch_us'], r['random_policy_in_kernel']['avg_launch_us'])"
done; done
