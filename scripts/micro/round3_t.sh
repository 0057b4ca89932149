#!/bin/bash
# final tree: full GPU suite, smoke, default bench line
ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/t_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/t_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/t_bench.log 2>&1; rc=$?
grep '^{' gpurun_out/t_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['ppo']['updates_per_s'])"
exit $rc
