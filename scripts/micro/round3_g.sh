ulimit -c 0
mkdir -p gpurun_out
# x6 GEMM parity with the new default build, then the A/B micro and PPO
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_x6_gpu.py > gpurun_out/t_x6.log 2>&1; rc=$?; tail -3 gpurun_out/t_x6.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="base cond f1early" timeout -k 10 400 bash scripts/micro/gemm_x6_ablate.sh > gpurun_out/x6ab.log 2>&1; rc=$?; cat gpurun_out/x6ab.log | grep -E "==|us_x6"; [ $rc -eq 0 ] || exit $rc
for v in base cond base cond; do
DRONERL_LIB=$PWD/scripts/micro/build/$v/libdronerl.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --no-companion --ppo-updates 5 > gpurun_out/bx_$v.log 2>&1 || exit $?
grep '^{' gpurun_out/bx_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print('$v', p['updates_per_s'], {k: v['us'] for k, v in p['roofline']['kernels_per_minibatch'].items()})"
done
