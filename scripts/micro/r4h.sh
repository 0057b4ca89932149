# full GPU suite, then the x6 micro-benchmark and the WS stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r4h_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/r4h_suite.log; grep -E "FAILED|Error" gpurun_out/r4h_suite.log | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python scripts/micro/gemm_x6_bench.py 2>&1 | grep -E "us_x6|rel_err" && \
  VARIANTS="stamps" bash scripts/micro/x6ws_ablate.sh stamps
