#!/bin/bash
# Round 5: the finish's 64-chunk sum with four times the threads: bitwise
# digests and update rates of the base and new library, alternating.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5c64}; mkdir -p $O
export PYTHONPATH=$PWD
B=$PWD/scripts/micro/build
for i in 1 2 3; do
  for v in base c64; do
    timeout -k 10 200 env DRONERL_LIB=$B/lib_$v.so python scripts/micro/ppo_digest.py >> $O/dig_$v.json 2>$O/dig_$v.err || exit 1
  done
done
for v in base c64; do echo "$v: $(cat $O/dig_$v.json | tr '\n' ' ')"; done
