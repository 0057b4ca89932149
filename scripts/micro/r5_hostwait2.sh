#!/bin/bash
cd "$(dirname "$0")/../.."
O=gpurun_out/r5e; mkdir -p $O
export PYTHONPATH=$PWD
for i in 1 2; do
timeout -k 10 180 python scripts/micro/host_wait.py --trials 100 > $O/a$i.json 2> $O/a$i.err || { tail -5 $O/a$i.err; exit 1; }; cat $O/a$i.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --no-companion --rollout-k 0 > $O/bench20.json 2> $O/bench20.err && python -c "
import json;d=json.load(open('$O/bench20.json'));r=d['roofline'];print(d['ms_per_step']*20e3, r['avg_launch_us'], r.get('avg_launch_us_packet'))"
