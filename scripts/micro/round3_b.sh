# round 3: bench (default + the driver's --steps 20), rollout-headline PMC
# traffic, rocprofv3 kernel stats of the default bench
ulimit -c 0
mkdir -p gpurun_out
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
          "ppo", d.get("ppo", {}).get("updates_per_s"), d.get("ppo", {}).get("roofline", {}).get("kernel_timing"))
    print({k: v["us"] for k, v in d["ppo"]["roofline"]["kernels_per_minibatch"].items()})
PY
bash scripts/rollout_traffic.sh || exit $?
export TMPDIR=/tmp
rm -rf "$PWD/gpurun_out/prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python3 "$PWD/bench.py" --no-cpu-baseline --no-companion > gpurun_out/rocprof.log 2>&1 || exit $?
rm -f "$PWD"/gpurun_out/prof/*kernel_trace.csv
find gpurun_out/prof -name "*stats*"
