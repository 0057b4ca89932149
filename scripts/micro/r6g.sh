# round 6: the forward GEMM's split VALU interleaved with its MFMAs and its
# memory instructions spread between them: bytes and time, alternating
# processes, one box
set -o pipefail
for i in 1 2 3; do for v in sa0m0 sa1m0 sa1m1; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 1 || exit 1; done; done
