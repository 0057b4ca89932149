ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/t_x6.log 2>&1; rc=$?; tail -3 gpurun_out/t_x6.log; [ $rc -eq 0 ] || exit $rc
for pp in 1 0 1 0; do
DRONERL_X6_PP=$pp timeout -k 10 60 python scripts/micro/gemm_x6_bench.py > gpurun_out/x6b_$pp.log 2>&1 || exit $?
echo "pp=$pp $(grep -E '"us_x6"' gpurun_out/x6b_$pp.log | tr -d '\n ')"
done
for pp in 1 0; do
DRONERL_X6_PP=$pp timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --no-companion --ppo-updates 5 > gpurun_out/bx_$pp.log 2>&1 || exit $?
grep '^{' gpurun_out/bx_$pp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print('pp=$pp', p['updates_per_s'], {k: v['us'] for k, v in p['roofline']['kernels_per_minibatch'].items()})"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ppo_gpu.py tests/test_ppo_flagship_parity_gpu.py > gpurun_out/t_ppo.log 2>&1; rc=$?; tail -3 gpurun_out/t_ppo.log; exit $rc
