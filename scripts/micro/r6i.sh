# round 6: fl16's D2 epilogue VALU spread over the MFMA slots of k32 steps
# 4 / 6 (d2new), + the forward's plane stores / staging DMA deferred into
# the next step's MFMA slots (wsdef), vs HEAD (d2old): bytes and time,
# alternating, one box; then the x6 parity tests on wsdef
set -o pipefail
for i in 1 2 3; do for v in d2old d2new wsdef; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/fl_bench.py || exit 1; done; done
for i in 1 2; do for v in d2old wsdef; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 1 || exit 1; done; done
DRONERL_LIB=scripts/micro/build/lib_wsdef.so timeout -k 10 300 python -u -m pytest tests/test_gemm_x6_fl_gpu.py tests/test_gemm_x6_gpu.py tests/test_ppo_flagship_parity_gpu.py -q --timeout 200 --timeout-method thread 2>&1 | tail -3
