#!/bin/bash
# Warp-specialised rollout kernel: diagnostic builds (DR_WS_ABL, wrong by
# construction) timed against the product kernel at 65,536 envs.
#   build: bash scripts/micro/ws_ablate.sh build (here);  run: on the GPU box
cd "$(dirname "$0")/../.."
OUT=scripts/micro/build
V="${VARIANTS:-0 1 2}"
# variant a: DR_WS_ABL=a; "prio": DR_WS_PRIO=1; "ra16" / "ra4": DR_WS_RA
flags() { case $1 in prio) echo "-DDR_WS_PRIO=1";; ra16) echo "-DDR_WS_RA=16";;
          5) echo "-DDR_WS_ABL=5 -DDR_ABLATE=5";; mwr0) echo "-DDR_WS_MWR=0";;
          ra4) echo "-DDR_WS_RA=4";; *) echo "-DDR_WS_ABL=$1";; esac; }
if [ "$1" == "build" ]; then
  for a in $V; do
    mkdir -p $OUT/ws$a
    make -C drone_rl_amd/csrc OBJDIR=$PWD/$OUT/ws$a/obj OUT=$PWD/$OUT/ws$a/libdronerl.so \
         KFLAGS="$(flags $a)" -j8 > /dev/null 2>&1 || { echo "build $a failed"; exit 1; }
    rm -rf $OUT/ws$a/obj
  done
  exit 0
fi
mkdir -p gpurun_out
for rep in 1 2; do for a in $V; do
  DRONERL_LIB=$PWD/$OUT/ws$a/libdronerl.so timeout -k 10 120 python scripts/micro/rollout_bench.py \
    --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/wsabl$a.log 2>&1 || exit 1
  echo "ws $a: $(tail -1 gpurun_out/wsabl$a.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["read_us"], v["gen_us"]) for k, v in d.items() if k.startswith("n")})')"
done; done
