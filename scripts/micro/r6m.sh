# round 6: the weight-gradient x6 GEMM's schedule, alternating on one box
# (wgrad_ab.py, the trainer's shape): wg0 = HEAD; wg1 / wg2 = iglp_opt(0 / 1);
# wg3 = a sched_group_barrier pipeline; wsj1 / wsj2 = the two waves of a SIMD
# splitting the next stage at different points of the stage (j 1 / 3, 0 / 2)
set -o pipefail
for i in 1 2 3; do for v in wg0 wg1 wg2 wg3 wsj1 wsj2; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/wgrad_ab.py || exit 1; done; done
