#!/bin/bash
# Round 5: (1) the x6 forward in the streamed-l-plane form (gemm_x6_fl_kernel
# <true>, DR_X6_STREAM_L=1) against the weight-stationary kernel: output
# digests and alternating timings; (2) the operand images built by the first
# layer's forward launch: tests, the GPU suite, in-process PPO A/B, a trace.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r5xs}; mkdir -p $O
export PYTHONPATH=$PWD
B=$PWD/scripts/micro/build
for m in "384 1" "65536 64"; do
  for v in base streaml; do
    timeout -k 10 120 env DRONERL_LIB=$B/lib_$v.so python tests/x6_forms_worker.py $m > $O/dig_${v}_${m// /_}.txt 2>&1 || exit 1
  done
done
for i in 1 2 3; do
  for v in base streaml; do
    timeout -k 10 120 env DRONERL_LIB=$B/lib_$v.so python scripts/micro/gemm_x6_bench.py > $O/ab_${v}_$i.json 2>$O/ab_${v}_$i.err || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_x6_fl_gpu.py > $O/test_fl.log 2>&1 || { echo fl tests failed; tail -30 $O/test_fl.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 || { echo suite failed; tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 500 python -u scripts/micro/ppo_ab_inproc.py policy.x6_fused_images=True policy.x6_fused_images=False > $O/ppo_ab.txt 2>$O/ppo_ab.err || exit 1
cat $O/ppo_ab.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --ppo-updates 2 > $O/bench.log 2>&1 || exit 1
echo done
