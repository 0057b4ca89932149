#!/bin/bash
# Round 5: policy_heads in 4-row tiles: bitwise
# digests and update rates of the base and new library, alternating.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5ph4}; mkdir -p $O
export PYTHONPATH=$PWD
B=$PWD/scripts/micro/build
for i in 1 2 3; do
  for v in base ph4; do
    timeout -k 10 200 env DRONERL_LIB=$B/lib_$v.so python scripts/micro/ppo_digest.py >> $O/dig_$v.json 2>$O/dig_$v.err || exit 1
  done
done
for v in base ph4; do echo "$v: $(cat $O/dig_$v.json | tr '\n' ' ')"; done
