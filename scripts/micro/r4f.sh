set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_x6_gpu.py -m gpu > gpurun_out/r4f_test.log 2>&1; rc=$?
echo "test rc=$rc"; tail -3 gpurun_out/r4f_test.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 120 python scripts/micro/gemm_x6_bench.py 2>&1 | grep -E "us_x6|rel_err" && \
  VARIANTS="stamps" bash scripts/micro/x6ws_ablate.sh stamps
