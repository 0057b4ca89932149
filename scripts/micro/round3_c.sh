ulimit -c 0
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --no-companion > gpurun_out/bench20_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("bench20_1", "bench20_2", "bench"):
    d = json.loads([l for l in open(f"gpurun_out/{f}.log") if l.startswith("{")][0])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"], d["roofline"]["traffic"],
          "single", d["single_step"]["env_steps_per_s"], d["single_step"]["roofline"]["frac"],
          "ppo", d.get("ppo", {}).get("updates_per_s"))
    print({k: v["us"] for k, v in d["ppo"]["roofline"]["kernels_per_minibatch"].items()})
print(json.dumps(d["ppo"]["roofline"], indent=0)[:1500])
PY
