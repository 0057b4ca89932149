#!/bin/bash
# In-process A/B of waves per workgroup of the step kernel (DR_ENV_WPB 4
# vs 8) at 65,536 and 131,072 envs.  build here, then run on the GPU box.
cd "$(dirname "$0")/../.."
B=scripts/micro/build
NAMES=(wpb4 wpb8)
declare -A V=([wpb4]="-DDR_ENV_WPB=4" [wpb8]="-DDR_ENV_WPB=8")
if [ "$1" = build ]; then
  for v in "${NAMES[@]}"; do
    rm -rf $B/env_$v && mkdir -p $B/env_$v
    make -C drone_rl_amd/csrc OBJDIR=$PWD/$B/env_$v/obj OUT=$PWD/$B/env_$v/lib_$v.so \
         KFLAGS="${V[$v]}" -j8 > /dev/null 2>&1 || { echo "build $v failed"; exit 1; }
    rm -rf $B/env_$v/obj
  done
  exit 0
fi
libs=""
for v in "${NAMES[@]}"; do libs="$libs $B/env_$v/lib_$v.so"; done
timeout -k 10 300 python scripts/micro/ab.py $libs --n 65536 --k 200 --reps 25 || exit $?
timeout -k 10 300 python scripts/micro/ab.py $libs --n 131072 --k 200 --reps 15 || exit $?
