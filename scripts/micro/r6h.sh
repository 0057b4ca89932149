# round 6: fl16 with its split pieces and memory instructions spread between
# its MFMAs (flnew) vs HEAD (flold): bytes and time, alternating, one box
set -o pipefail
for i in 1 2 3; do for v in flold flnew; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/fl_bench.py || exit 1; done; done
for v in flold flnew; do
DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion --rollout-k 0 > gpurun_out/r6h_bench_$v.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/r6h_bench_$v.json'));p=d['ppo'];print('$v',p['updates_per_s'],{k:v.get('isolated_us',v['prefix_split_us']) for k,v in p['roofline']['kernels_per_minibatch'].items()})"
done
