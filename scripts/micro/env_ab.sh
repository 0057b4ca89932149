#!/bin/bash
# Build env-step variants (scripts/micro/build/env_<name>/) and A/B them in
# one process with scripts/micro/ab.py at 65,536 and 4M envs.
#   bash scripts/micro/env_ab.sh build     (here)     bash scripts/micro/env_ab.sh   (GPU box)
cd "$(dirname "$0")/../.."
B=scripts/micro/build
NAMES=(base obs2 noreset nophilox)
declare -A V=(
  [base]=""
  [obs2]="-DDR_OBS_ONCE=0"
  [noreset]="-DDR_ABLATE=2"
  [nophilox]="-DDR_ABLATE=5"
)
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
timeout -k 10 300 python scripts/micro/ab.py $libs --n 4194304 --k 40 --reps 7 || exit $?
