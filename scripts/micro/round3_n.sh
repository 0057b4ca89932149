ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rollout_gpu.py tests/test_moving_gpu.py > gpurun_out/t_ro.log 2>&1; rc=$?; tail -3 gpurun_out/t_ro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --extra --ppo-updates 0 > gpurun_out/bench_extra2.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_extra2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']); print({k: v for k, v in d['extra'].items() if 'rollout' in k})"
