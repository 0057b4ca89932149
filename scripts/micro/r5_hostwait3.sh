#!/bin/bash
cd "$(dirname "$0")/../.."
O=gpurun_out/r5f; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 180 python scripts/micro/host_wait.py --trials 50 > $O/a1.json 2> $O/a1.err || { tail -5 $O/a1.err; exit 1; }; cat $O/a1.json
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --no-companion --rollout-k 0 > $O/bench20_$i.json 2> $O/bench20_$i.err || exit 1
python -c "
import json;d=json.load(open('$O/bench20_$i.json'));r=d['roofline'];print(d['value'], d['ms_per_step']*20e3, r['avg_launch_us'], r.get('avg_launch_us_packet'), r['frac_wall'])"
done
