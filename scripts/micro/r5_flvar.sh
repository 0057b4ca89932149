#!/bin/bash
# Round 5: variants of the fused input-gradient GEMM + first-layer backward
# (scripts/micro/build_variant.sh), timed alternately on one box.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5flv}; mkdir -p $O
shift
export PYTHONPATH=$PWD
for i in 1 2; do
  for v in "$@"; do
    timeout -k 10 120 env DRONERL_LIB=$PWD/scripts/micro/build/lib_$v.so python scripts/micro/fl_bench.py >> $O/fl_$v.json 2>$O/fl_$v.err || exit 1
  done
done
for v in "$@"; do echo "$v: $(cat $O/fl_$v.json | tr '\n' ' ')"; done
