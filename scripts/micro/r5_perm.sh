#!/bin/bash
# Round 5: dr_permutation bucket-size variants (DR_PERM_MEAN), alternating.
cd "$(dirname "$0")/../.."
O=gpurun_out/r5perm; mkdir -p $O
export PYTHONPATH=$PWD
for i in 1 2 3; do
  for v in "$@"; do
    timeout -k 10 120 env DRONERL_LIB=$PWD/scripts/micro/build/lib_$v.so python scripts/micro/perm_bench.py >> $O/p_$v.json 2>$O/p_$v.err || exit 1
  done
done
for v in "$@"; do echo "$v: $(cat $O/p_$v.json | tr '\n' ' ')"; done
