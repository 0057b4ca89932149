#!/bin/bash
# Host-code sanitizer builds (CPU only; never shipped to the GPU box -- this
# directory is in .gpurunignore):
#   build/asan/liboracle.so    oracle/*.c with gcc -fsanitize=address,undefined
#   build/asan/libdronerl.so   the product's host code (ABI argument
#                              validation, handle bookkeeping) with clang's
#                              ASan+UBSan on the host side only (-Xarch_host;
#                              the gfx950 device code is built as usual)
# Usage: bash tests/sanitize/build.sh [oracle|product|all]
set -e
cd "$(dirname "$0")/../.."
OUT=build/asan
mkdir -p $OUT
what=${1:-all}
if [ $what = oracle ] || [ $what = all ]; then
  gcc -O1 -g -fPIC -ffp-contract=off -fno-fast-math -fno-omit-frame-pointer \
      -fsanitize=address,undefined -fno-sanitize-recover=undefined \
      -shared -o $OUT/liboracle.so oracle/drone_ref.c oracle/ppo_ref.c -lm
fi
if [ $what = product ] || [ $what = all ]; then
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
      -fno-fast-math -Iinclude -fno-omit-frame-pointer \
      -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
      -shared -o $OUT/libdronerl.so drone_rl_amd/csrc/env_kernels.hip drone_rl_amd/csrc/ppo_kernels.hip \
      drone_rl_amd/csrc/gemm_x6.hip
fi
