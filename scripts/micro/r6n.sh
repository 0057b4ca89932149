# round 6: iglp_opt(0) on the weight-gradient GEMM, alone and with the SIMD's
# two waves splitting at different points (wg1sj1 / wg1sj2), and two
# sched_group_barrier pipelines (wg5: a transposed read every 2 MFMAs;
# wg3sj2), alternating on one box against HEAD (wg0)
set -o pipefail
for i in 1 2 3; do for v in wg0 wg1 wg1sj1 wg1sj2 wg3 wg5 wg3sj2; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/wgrad_ab.py || exit 1; done; done
