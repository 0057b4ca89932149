#!/bin/bash
# Round 5: the next minibatch's gather inside the deferred-finish launch.
# The whole GPU suite, then an in-process PPO A/B (fused gather on / off).
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5fg}; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 || { echo suite failed; tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 500 python -u scripts/micro/ppo_ab_inproc.py fused_gather=True fused_gather=False > $O/ppo_ab.txt 2>$O/ppo_ab.err || exit 1
cat $O/ppo_ab.txt
echo done
