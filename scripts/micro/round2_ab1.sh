ulimit -c 0
B=scripts/micro/build
timeout -k 10 200 python scripts/micro/ab.py $B/libdr_a0.so $B/libdr_a1.so $B/libdr_a3.so $B/libdr_a4.so $B/libdr_a6.so --n 65536 --k 200 --reps 25 > gpurun_out/ab_ablate2.log 2>&1 || exit $?
grep '^{' gpurun_out/ab_ablate2.log
timeout -k 10 300 python bench.py --no-companion --ppo-updates 5 > gpurun_out/bench_tg.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_tg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_us'], d['ppo']['updates_per_s'], d['cpu_baseline']['cores'], d['cpu_baseline']['affinity_cpus'], d['cpu_baseline']['cores_limited_by'], d['cpu_baseline']['value'])"
