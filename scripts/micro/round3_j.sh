ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rollout_gpu.py > gpurun_out/t_ro.log 2>&1; rc=$?; tail -3 gpurun_out/t_ro.log; [ $rc -eq 0 ] || exit $rc
for ws in 1 0; do
DRONERL_ROLLOUT_WS=$ws timeout -k 10 120 python scripts/micro/rollout_bench.py --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/rb_ws$ws.log 2>&1 || exit $?
echo "ws=$ws $(tail -1 gpurun_out/rb_ws$ws.log)"
done
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b20_$i.log 2>&1 || exit $?
grep '^{' gpurun_out/b20_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; ro=d['rollout_kernel']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r.get('avg_launch_us_packet'), r['frac'], ro['actions_from_hbm']['avg_launch_us'], ro['random_policy_in_kernel']['avg_launch_us'], d['ppo']['updates_per_s'])"
done
