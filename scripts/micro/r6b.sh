set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6b/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6b/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r6b/gpu_tests.log
for v in m32 m16; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 0.5 >> gpurun_out/r6b/sha.jsonl || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6b/bench.json 2> gpurun_out/r6b/bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r6b/bench.json'));print(d['value'],d['roofline']['avg_launch_us'],d['roofline'].get('walls'),d['ppo']['updates_per_s'],d['ppo']['roofline']['dominant_kernel'])"
