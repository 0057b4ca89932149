#!/bin/bash
# split-physics rollout kernel as the read-path default: the rollout tests
# (default selection), then the headline alternating (off / default) x 3
ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_rollout_gpu.py > gpurun_out/ad_test.log 2>&1; rc=$?
tail -2 gpurun_out/ad_test.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for ab in 0 d; do
  E=""; [ $ab == 0 ] && E="DRONERL_ROLLOUT_AB=0"
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion --ppo-updates 0 \
    > gpurun_out/ad_b$ab.log 2>&1 || exit 1
  grep '^{' gpurun_out/ad_b$ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ab $ab headline', d['value'], d['roofline']['avg_launch_us'], d['rollout_kernel']['actions_from_hbm']['avg_launch_us'], d['rollout_kernel']['random_policy_in_kernel']['avg_launch_us'])"
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion --ppo-updates 0 --steps 20 --warmup 5 \
    > gpurun_out/ad_c$ab.log 2>&1 || exit 1
  grep '^{' gpurun_out/ad_c$ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ab $ab steps20', d['value'], d['roofline']['avg_launch_us'], d['roofline']['avg_launch_us_packet'])"
done; done
