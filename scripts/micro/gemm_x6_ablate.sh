#!/bin/bash
# Build variants of libdronerl.so with extra compile flags for gemm_x6.hip
# (scripts/micro/build/<name>/) and time each with gemm_x6_bench.py in one
# GPU session.  DR_X6_ABL variants are wrong by construction (times only).
#   bash scripts/micro/gemm_x6_ablate.sh build   (here)
#   bash scripts/micro/gemm_x6_ablate.sh         (on the GPU box)
cd "$(dirname "$0")/../.."
B=scripts/micro/build
declare -A V=(
  [base]=""
  [acc1]="-DDR_X6_ACC1=1"
  [acc1_early]="-DDR_X6_ACC1=1 -DDR_X6_EARLY=1"
  [noslp]="-fno-slp-vectorize"
)
if [ "$1" = build ]; then
  for v in "${!V[@]}"; do
    rm -rf $B/$v && mkdir -p $B/$v
    make -C drone_rl_amd/csrc OBJDIR=$PWD/$B/$v/obj OUT=$PWD/$B/$v/libdronerl.so \
         KFLAGS="${V[$v]}" -j8 > /dev/null 2>&1 || { echo "build $v failed"; exit 1; }
    rm -rf $B/$v/obj
  done
  exit 0
fi
for rep in 1 2; do
  for v in base acc1 acc1_early noslp; do
    echo "== $v"
    DRONERL_LIB=$PWD/$B/$v/libdronerl.so timeout -k 10 60 python scripts/micro/gemm_x6_bench.py \
        | grep -E '"us_x6"|"rel_err_x6"' || exit 1
  done
done
