ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/t_x6.log 2>&1; rc=$?; tail -6 gpurun_out/t_x6.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
DRONERL_X6_L1=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --no-companion --ppo-updates 5 > gpurun_out/bl1_$v.log 2>&1 || exit $?
grep '^{' gpurun_out/bl1_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print('L1=$v', p['updates_per_s'], {k: v['us'] for k, v in p['roofline']['kernels_per_minibatch'].items()})"
done
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1; rc=$?; tail -4 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
bash scripts/micro/rollout_ablate.sh run
