ulimit -c 0
for r in 1 2 3; do
for g in "" "--no-graph"; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion --ppo-updates 0 $g > gpurun_out/b.log 2>&1 || exit $?
grep '^{' gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$g', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done; done
