set -o pipefail
mkdir -p gpurun_out/r6c
for v in m32 m16; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 0.5 >> gpurun_out/r6c/sha.jsonl || exit 1; done
cat gpurun_out/r6c/sha.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6c/bench.json 2> gpurun_out/r6c/bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r6c/bench.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['frac_wall'],r.get('walls'),d['ppo']['updates_per_s'],d['ppo']['roofline']['dominant_kernel'],d['ppo']['roofline']['kernels_per_minibatch']['gather_minibatch'])"
