ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_rollout_gpu.py tests/test_abi.py > gpurun_out/t_ro.log 2>&1; rc=$?; tail -3 gpurun_out/t_ro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/micro/launch_paths.py > gpurun_out/launch_paths.log 2>&1 || exit $?
cat gpurun_out/launch_paths.log | grep -v amdgpu.ids
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b20_$i.log 2>&1 || exit $?
grep '^{' gpurun_out/b20_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'] if 'avg_launch_us' in d['roofline'] else d['roofline'], d['ppo']['updates_per_s'])"
done
