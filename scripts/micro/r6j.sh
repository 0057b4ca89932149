# round 6: the committed candidate (cur: ws16 deferred plane stores / DMA,
# fl16 as HEAD) vs HEAD (d2old): fl / ws16 time, alternating; parity tests
set -o pipefail
for i in 1 2; do for v in d2old cur; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/fl_bench.py || exit 1; done; done
for i in 1 2; do for v in d2old cur; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 1 || exit 1; done; done
timeout -k 10 400 python -u -m pytest tests/test_gemm_x6_fl_gpu.py tests/test_gemm_x6_gpu.py tests/test_ppo_flagship_parity_gpu.py -q --timeout 200 --timeout-method thread 2>&1 | tail -3
