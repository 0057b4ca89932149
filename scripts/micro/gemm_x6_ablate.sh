#!/bin/bash
# Build variants of libdronerl.so with extra compile flags for gemm_x6.hip
# (scripts/micro/build/<name>/) and time each with gemm_x6_bench.py in one
# GPU session.  DR_X6_ABL variants are wrong by construction (times only).
#   bash scripts/micro/gemm_x6_ablate.sh build   (here)
#   bash scripts/micro/gemm_x6_ablate.sh         (on the GPU box)
# VARIANTS="base cond" selects a subset (default: all below).
cd "$(dirname "$0")/../.."
B=scripts/micro/build
declare -A V=(
  [base]=""
  [cond]="-DDR_X6_CONDREAD=1"
  [f1early]="-DDR_X6_F1EARLY=1"
  [stagger]="-DDR_X6_STAGGER=1"
  [prio2]="-DDR_X6_PRIO=2"
)
SEL="${VARIANTS:-base cond f1early}"
if [ "$1" = build ]; then
  for v in $SEL; do
    rm -rf $B/$v && mkdir -p $B/$v
    make -C drone_rl_amd/csrc OBJDIR=$PWD/$B/$v/obj OUT=$PWD/$B/$v/libdronerl.so \
         KFLAGS="${V[$v]}" -j8 > /dev/null 2>&1 || { echo "build $v failed"; exit 1; }
    rm -rf $B/$v/obj
  done
  exit 0
fi
for rep in 1 2; do
  for v in $SEL; do
    echo "== $v"
    DRONERL_LIB=$PWD/$B/$v/libdronerl.so timeout -k 10 60 python scripts/micro/gemm_x6_bench.py \
        | grep -E '"us_x6"|"rel_err_x6"' || exit 1
  done
done
