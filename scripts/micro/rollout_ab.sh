#!/bin/bash
# A/B of rollout-kernel build variants (DR_RO_* knobs in env_kernels.hip):
#   build: hipcc each variant into scripts/micro/build/libdronerl_ro_<tag>.so
#   run:   on the GPU box, the rollout parity tests and the K = 32 timing
#          (65,536 and 131,072 envs) per variant, through DRONERL_LIB
cd "$(dirname "$0")/../.."
OUT=scripts/micro/build
declare -A FLAGS=( [base]="" [pipe]="-DDR_RO_PIPE=1" [vm13]="-DDR_RO_PIPE=1 -DDR_RO_VM13=1"
                   [presc]="-DDR_RO_PIPE=1 -DDR_RO_PRESC=1" [presc0]="-DDR_RO_PRESC=1" )
TAGS="${TAGS:-base pipe presc}"
if [ "$1" == "build" ]; then
  mkdir -p $OUT
  for t in $TAGS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
      -fno-fast-math -Iinclude ${FLAGS[$t]} -shared -o $OUT/libdronerl_ro_$t.so \
      drone_rl_amd/csrc/env_kernels.hip drone_rl_amd/csrc/ppo_kernels.hip \
      drone_rl_amd/csrc/gemm_x6.hip || exit 1
  done
  exit 0
fi
mkdir -p gpurun_out
for t in $TAGS; do
  export DRONERL_LIB=$PWD/$OUT/libdronerl_ro_$t.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_rollout_gpu.py > gpurun_out/ro_t_$t.log 2>&1 || { tail -20 gpurun_out/ro_t_$t.log; exit 1; }
  echo "$t tests: $(tail -1 gpurun_out/ro_t_$t.log)"
done
for rep in 1 2; do
for t in $TAGS; do
  export DRONERL_LIB=$PWD/$OUT/libdronerl_ro_$t.so
  timeout -k 10 120 python scripts/micro/rollout_bench.py --envs 65536 131072 --ks 32 --reps 20 \
    > gpurun_out/ro_b_$t.log 2>&1 || exit 1
  echo "$t: $(tail -1 gpurun_out/ro_b_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (v['read_us'], v['gen_us']) for k, v in d.items() if k.startswith('n')})")"
done
done
