ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_bootstrap_gpu.py tests/test_ppo_gpu.py::test_rollout_and_first_epoch_share_one_gemm_path tests/test_render.py::test_gym_render_keeps_the_reference_signature > gpurun_out/t_new.log 2>&1; rc=$?; tail -12 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
for r in 64 32; do
DRONERL_ROLLOUT_RPW=$r timeout -k 10 200 python scripts/micro/rollout_bench.py --envs 65536 131072 --ks 32 --reps 20 > gpurun_out/rb_$r.log 2>&1 || exit $?
tail -3 gpurun_out/rb_$r.log
done
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --no-companion --ppo-updates 0 > gpurun_out/bench20_$i.log 2>&1 || exit $?
grep '^{' gpurun_out/bench20_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['traffic'])"
done
