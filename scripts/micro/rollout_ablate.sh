#!/bin/bash
# Diagnostic builds of libdronerl.so (DR_ABLATE variants; results wrong by
# construction) timed on the K = 32 rollout kernel at 65,536 envs:
#   build: hipcc the variants here (CPU);  run: time each on the GPU box.
cd "$(dirname "$0")/../.."
OUT=scripts/micro/build
V="${VARIANTS:-0 1 6 7 8}"
if [ "$1" == "build" ]; then
  mkdir -p $OUT
  for a in $V; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
      -Iinclude -DDR_ABLATE=$a -shared -o $OUT/libdronerl_ablate$a.so \
      drone_rl_amd/csrc/env_kernels.hip drone_rl_amd/csrc/ppo_kernels.hip drone_rl_amd/csrc/gemm_x6.hip || exit 1
  done
  exit 0
fi
mkdir -p gpurun_out
for a in $V; do
  DRONERL_LIB=$PWD/$OUT/libdronerl_ablate$a.so timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 131072 --ks 32 --reps 20 > gpurun_out/rabl$a.log 2>&1 || exit 1
  echo "ablate $a: $(tail -1 gpurun_out/rabl$a.log)"
done
