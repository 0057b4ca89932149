#!/bin/bash
# ws rollout: the product, DR_WS_ABL=1 (no stores) and DR_WS_ABL=6 (no
# per-step barrier, physics waves alone) at 65,536 envs, K = 32
ulimit -c 0
mkdir -p gpurun_out
for rep in 1 2; do for a in 0 1 6; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $a != 0 ] && L=$PWD/scripts/micro/build/ws$a/libdronerl.so
  DRONERL_LIB=$L timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 --ks 32 --reps 16 --act-sets 8 > gpurun_out/ab_ws$a.log 2>&1 || exit 1
  echo "ws $a: $(tail -1 gpurun_out/ab_ws$a.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["read_us"], v["gen_us"]) for k, v in d.items() if k.startswith("n")})')"
done; done
