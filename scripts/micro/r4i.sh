# full GPU suite, x6 micro-benchmark + stamps, the driver's bench form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r4i_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 gpurun_out/r4i_suite.log; grep -E "FAILED|Error" gpurun_out/r4i_suite.log | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python scripts/micro/gemm_x6_bench.py 2>&1 | grep -E "us_x6|rel_err" && \
  VARIANTS="stamps" timeout -k 10 120 bash scripts/micro/x6ws_ablate.sh stamps && \
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r4i_bench.json 2> gpurun_out/r4i_bench.err && \
  python3 -c "
import json; d=json.loads(open('gpurun_out/r4i_bench.json').read().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'packet', d['roofline']['avg_launch_us_packet'], 'ev', d['roofline']['avg_launch_us'])
print('ppo', d['ppo']['updates_per_s'], {k: v['us'] for k, v in d['ppo']['roofline']['kernels_per_minibatch'].items()})
print('comp_rollout', json.dumps(d.get('companion_rollout')))
"
