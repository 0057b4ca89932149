ulimit -c 0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1; rc=$?; tail -4 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log > gpurun_out/bench.json
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['companion']['avg_launch_us'], d['ppo']['updates_per_s'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20.log 2>&1 || exit $?
grep '^{' gpurun_out/bench20.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('steps20', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
