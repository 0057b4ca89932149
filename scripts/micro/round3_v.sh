#!/bin/bash
# Two physics waves per SIMD on the warp-specialised rollout kernel: the
# product kernel, DR_WS_ABL=1 (memory waves store nothing: physics alone) and
# DR_WS_ABL=2 (no physics: the store stream alone), forced onto the ws kernel
# at 65,536 envs (one physics wave per SIMD) and 131,072 (two).
#   build here: VARIANTS="1 2" bash scripts/micro/ws_ablate.sh build
ulimit -c 0
mkdir -p gpurun_out
for rep in 1 2; do for a in 0 1 2; do
  L=$PWD/drone_rl_amd/libdronerl.so; [ $a != 0 ] && L=$PWD/scripts/micro/build/ws$a/libdronerl.so
  DRONERL_ROLLOUT_WS=1 DRONERL_LIB=$L timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 131072 --ks 32 --reps 16 --act-sets 8 > gpurun_out/v_ws$a.log 2>&1 || exit 1
  echo "ws $a: $(tail -1 gpurun_out/v_ws$a.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["read_us"], v["gen_us"]) for k, v in d.items() if k.startswith("n")})')"
done; done
