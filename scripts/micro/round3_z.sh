#!/bin/bash
# the tree with the rational tanh: full GPU suite + smoke, then the
# first-layer backward block-count A/B (kernel times, PPO updates/s)
ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/z_all.log 2>&1; rc=$?; tail -3 gpurun_out/z_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/z_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/z_smoke.log; [ $rc -eq 0 ] || exit $rc
KERN="first_layer_bwd" bash scripts/micro/ab_ppo_kern.sh run base fl256 fl384 base fl256 || exit $?
