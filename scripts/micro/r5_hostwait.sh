#!/bin/bash
# Round 5: host-side launch + synchronize cost under runtime settings
cd "$(dirname "$0")/../.."
O=gpurun_out/r5d; mkdir -p $O
export PYTHONPATH=$PWD
run() { tag=$1; shift; timeout -k 10 120 env "$@" python scripts/micro/host_wait.py > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }; cat $O/$tag.json; }
run default A=1
run nointr HSA_ENABLE_INTERRUPT=0
run nodd AMD_DIRECT_DISPATCH=0
run default2 A=1
run nointr2 HSA_ENABLE_INTERRUPT=0
timeout -k 10 120 python scripts/micro/host_wait.py --spin > $O/spin.json 2>$O/spin.err && cat $O/spin.json
timeout -k 10 120 env HSA_ENABLE_INTERRUPT=0 python scripts/micro/host_wait.py --spin > $O/nointr_spin.json 2>$O/nointr_spin.err && cat $O/nointr_spin.json
