#!/bin/bash
# TunableOp experiment: tune the PPO GEMM shapes (hipBLASLt + rocBLAS
# solutions, timed on the box), then re-run the PPO bench on the tuned file.
cd "$(dirname "$0")/.."
OUT=gpurun_out/tune
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --steps 20 --warmup 5 --ppo-updates 3"
timeout -k 10 300 $B > $OUT/base.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop.csv \
  timeout -k 10 600 $B > $OUT/tuning.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 \
PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop.csv \
  timeout -k 10 300 $B > $OUT/tuned.log 2>&1 || exit $?
ls $OUT
for f in base tuning tuned; do grep -o '"updates_per_s": [0-9.]*' $OUT/$f.log; done
