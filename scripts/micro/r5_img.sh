#!/bin/bash
# Round 5: the x6 operand images built by the first layer's forward launch
# (dr_linear_tanh2_x6).  Its tests, the whole GPU suite, an in-process PPO
# A/B, a kernel trace.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5img}; mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_x6_fl_gpu.py > $O/test_fl.log 2>&1 || { echo fl tests failed; tail -30 $O/test_fl.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 || { echo suite failed; tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 500 python -u scripts/micro/ppo_ab_inproc.py policy.x6_fused_images=True policy.x6_fused_images=False > $O/ppo_ab.txt 2>$O/ppo_ab.err || exit 1
cat $O/ppo_ab.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ppo-updates 2 > $O/bench.log 2>&1 || exit 1
echo done
