#!/bin/bash
# Round 5: the head kernel's rows summed by the deferred finish (head_direct).
# The PPO kernel tests, the whole GPU suite, an in-process PPO A/B.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5hd}; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 || { echo suite failed; tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 500 python -u scripts/micro/ppo_ab_inproc.py policy.head_direct=True policy.head_direct=False policy.head_direct=True policy.head_direct=False > $O/ppo_ab.txt 2>$O/ppo_ab.err || exit 1
cat $O/ppo_ab.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ppo-updates 2 > $O/bench.log 2>&1 || exit 1
echo done
