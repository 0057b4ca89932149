# round 3, first GPU session: the new DP tests, the whole GPU suite, the
# default bench line and the driver's --steps 20 form
ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dp_train_gpu.py > gpurun_out/t_dp.log 2>&1; rc=$?; tail -15 gpurun_out/t_dp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1; rc=$?; tail -4 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log > gpurun_out/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20.log 2>&1 || exit $?
grep '^{' gpurun_out/bench20.log > gpurun_out/bench20.json
python - <<'PY'
import json
for f in ("bench", "bench20"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"],
          "single", d["single_step"]["env_steps_per_s"], d["single_step"]["roofline"]["frac"],
          "ppo", d.get("ppo", {}).get("updates_per_s"))
print(json.dumps(d.get("ppo", {}).get("roofline"), indent=1))
PY
