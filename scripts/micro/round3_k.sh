ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rollout_gpu.py > gpurun_out/t_ro.log 2>&1; rc=$?; tail -3 gpurun_out/t_ro.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in pre1 pre0; do
DRONERL_LIB=$PWD/scripts/micro/build/$v/libdronerl.so timeout -k 10 120 python scripts/micro/rollout_bench.py --envs 65536 --ks 20 32 --reps 16 --act-sets 8 > gpurun_out/rb_$v.log 2>&1 || exit $?
echo "$v: $(tail -1 gpurun_out/rb_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["read_us"], v["gen_us"]) for k, v in d.items() if k.startswith("n")})')"
done; done
