# round 6: the 16x16x32-only library -- new x6 digests, the GPU suite, a bench
set -o pipefail
mkdir -p gpurun_out/r6e
for a in "384 1" "65536 64"; do PYTHONPATH=$PWD timeout -k 10 120 python tests/x6_forms_worker.py $a || exit 1; done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6e/gpu_tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|FAILED|Error" gpurun_out/r6e/gpu_tests.log | tail -15
grep -q "Memory access fault\|core dumped" gpurun_out/r6e/gpu_tests.log && exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6e/bench.json 2> gpurun_out/r6e/bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r6e/bench.json'));r=d['roofline'];p=d['ppo'];print(d['value'],r['avg_launch_us'],r['frac'],r['frac_wall'],p['updates_per_s'],{k:v.get('isolated_us',v['prefix_split_us']) for k,v in p['roofline']['kernels_per_minibatch'].items()})"
