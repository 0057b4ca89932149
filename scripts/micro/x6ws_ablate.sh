#!/bin/bash
# WS GEMM ablations (DR_WS_ABL, wrong by construction: times only).
#   bash scripts/micro/x6ws_ablate.sh build   (here)
#   bash scripts/micro/x6ws_ablate.sh         (on the GPU box)
cd "$(dirname "$0")/../.."
B=scripts/micro/build
SEL="${VARIANTS:-base a1 a2 a3 a4 a5}"
declare -A V=([base]="" [a1]="-DDR_WS_ABL=1" [a2]="-DDR_WS_ABL=2" [a3]="-DDR_WS_ABL=3" [a4]="-DDR_WS_ABL=4" [a5]="-DDR_WS_ABL=5" [a6]="-DDR_WS_ABL=6" [a7]="-DDR_WS_ABL=7" [stamps]="-DDR_WS_STAMPS=1" [sa1]="-DDR_WS_STAMPS=1 -DDR_WS_ABL=1" [sa2]="-DDR_WS_STAMPS=1 -DDR_WS_ABL=2" [sa3]="-DDR_WS_STAMPS=1 -DDR_WS_ABL=3" [sa4]="-DDR_WS_STAMPS=1 -DDR_WS_ABL=4" [nf2]="-DWS_NF=2" [csplit]="-DDR_WS_CSPLIT=1" [snf2]="-DDR_WS_STAMPS=1 -DWS_NF=2")
if [ "$1" = build ]; then
  for v in $SEL; do
    rm -rf $B/$v && mkdir -p $B/$v
    make -C drone_rl_amd/csrc OBJDIR=$PWD/$B/$v/obj OUT=$PWD/$B/$v/libdronerl.so \
         KFLAGS="${V[$v]}" -j8 > /dev/null 2>&1 || { echo "build $v failed"; exit 1; }
    rm -rf $B/$v/obj
  done
  exit 0
fi
if [ "$1" = stamps ]; then
  for v in $SEL; do
    echo "== $v"
    timeout -k 10 60 python scripts/micro/ws_stamps.py $PWD/$B/$v/libdronerl.so | grep -E "^mfma|^row" || exit 1
  done
  exit 0
fi
for rep in 1 2; do
  for v in $SEL; do
    echo "== $v"
    DRONERL_LIB=$PWD/$B/$v/libdronerl.so timeout -k 10 60 python scripts/micro/gemm_x6_bench.py \
        | grep -E '"us_x6"' || exit 1
  done
done
