#!/bin/bash
# split-physics rollout kernel (DRONERL_ROLLOUT_AB=1): the rollout parity
# tests with it forced, then rollout-kernel and headline timings, A/B
ulimit -c 0
mkdir -p gpurun_out
DRONERL_ROLLOUT_AB=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_rollout_gpu.py > gpurun_out/ac_test.log 2>&1; rc=$?
tail -3 gpurun_out/ac_test.log; [ $rc -eq 0 ] || exit $rc
DRONERL_ROLLOUT_AB=1 DRONERL_ROLLOUT_WS=1 PYTHONPATH=$PWD timeout -k 10 120 python tests/rollout_form_worker.py gym 131392 37 || exit 1
for rep in 1 2; do for ab in 0 1; do
  DRONERL_ROLLOUT_AB=$ab timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/ac_rb$ab.log 2>&1 || exit 1
  echo "ab $ab: $(tail -1 gpurun_out/ac_rb$ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["read_us"], v["gen_us"]) for k, v in d.items() if k.startswith("n")})')"
done; done
for ab in 0 1; do
  DRONERL_ROLLOUT_AB=$ab timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion --ppo-updates 0 \
    > gpurun_out/ac_b$ab.log 2>&1 || exit 1
  grep '^{' gpurun_out/ac_b$ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ab $ab headline', d['value'], d['roofline']['avg_launch_us'])"
  DRONERL_ROLLOUT_AB=$ab timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion --ppo-updates 0 --steps 20 --warmup 5 \
    > gpurun_out/ac_c$ab.log 2>&1 || exit 1
  grep '^{' gpurun_out/ac_c$ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ab $ab steps20', d['value'], d['roofline']['avg_launch_us'], d['roofline']['avg_launch_us_packet'])"
done
