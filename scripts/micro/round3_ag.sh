#!/bin/bash
# split rollout kernel: issue priority for the translation (1) or rotation
# (2) waves vs none; rollout-kernel timings alternating (bitwise by
# construction: s_setprio changes no arithmetic)
ulimit -c 0
mkdir -p gpurun_out
for rep in 1 2 3; do for v in 0 1 2; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $v != 0 ] && L=$PWD/scripts/micro/build/pr$v/libdronerl.so
  DRONERL_LIB=$L timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/ag_rb$v.log 2>&1 || exit 1
  echo "prio $v: $(tail -1 gpurun_out/ag_rb$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["read_us"] for k, v in d.items() if k.startswith("n")})')"
done; done
