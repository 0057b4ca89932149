#!/bin/bash
# Round 5: the forward GEMM with column tile 1's weights loaded behind row
# step 0 (WS_W_LATE=1) against the product form, alternating (fl_bench.py),
# then the x6 GPU tests on the variant.
cd "$(dirname "$0")/../.."
bash scripts/micro/r5_flvar.sh r5wl gbase gwl gbase gwl || exit $?
timeout -k 10 300 env DRONERL_LIB=$PWD/scripts/micro/build/lib_gwl.so python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_x6_gpu.py tests/test_gemm_x6_fl_gpu.py > gpurun_out/r5wl/tests_gwl.log 2>&1
rc=$?; tail -2 gpurun_out/r5wl/tests_gwl.log; exit $rc
