ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cs in 1 0 1 0; do
DRONERL_X6_CS=$cs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --no-companion --ppo-updates 5 > gpurun_out/bx_$cs.log 2>&1 || exit $?
grep '^{' gpurun_out/bx_$cs.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print('cs=$cs', p['updates_per_s'], {k: v['us'] for k, v in p['roofline']['kernels_per_minibatch'].items() if 'gemm' in k})"
done
