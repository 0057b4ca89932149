ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/t_x6.log 2>&1; rc=$?; tail -3 gpurun_out/t_x6.log; [ $rc -eq 0 ] || exit $rc
for w in 1 0 1 0; do
DRONERL_X6_WCS=$w timeout -k 10 60 python scripts/micro/gemm_x6_bench.py > gpurun_out/x6w_$w.log 2>&1 || exit $?
echo "wcs=$w $(grep -E 'wgrad' gpurun_out/x6w_$w.log | tr -d '\n ')"
done
for w in 1 0 1 0; do
DRONERL_X6_WCS=$w timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --no-companion --ppo-updates 5 > gpurun_out/bw_$w.log 2>&1 || exit $?
grep '^{' gpurun_out/bw_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print('wcs=$w', p['updates_per_s'], {k: v['us'] for k, v in p['roofline']['kernels_per_minibatch'].items() if 'gemm' in k})"
done
