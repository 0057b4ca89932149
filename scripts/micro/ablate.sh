#!/bin/bash
# Build diagnostic variants of libdronerl.so (DR_ABLATE=1..4) next to this
# script and time each with bench.py through DRONERL_LIB.  Diagnostic only:
# the variants are numerically wrong by construction.
cd "$(dirname "$0")/../.."
OUT=scripts/micro/build
mkdir -p $OUT
if [ "$1" == "build" ]; then
  for a in 0 1 2 3 4; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
      -Iinclude -DDR_ABLATE=$a -shared -o $OUT/libdronerl_ablate$a.so \
      drone_rl_amd/csrc/env_kernels.hip drone_rl_amd/csrc/ppo_kernels.hip || exit 1
  done
  exit 0
fi
for a in 0 1 2 3 4; do
  DRONERL_LIB=$PWD/$OUT/libdronerl_ablate$a.so timeout -k 10 120 python bench.py \
    --no-cpu-baseline --ppo-updates 0 --extra > gpurun_out/ablate$a.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ablate$a.log') if l.startswith('{')][0])
print('ablate $a', d['roofline']['avg_launch_us'], {k: v['avg_launch_us'] for k, v in d['extra'].items() if k.startswith('lane')})"
done
