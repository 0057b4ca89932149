set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -4 gpurun_out/t.log
[ $rc -le 1 ] || exit $rc
B=scripts/micro/build
timeout -k 10 300 python scripts/micro/ab.py $B/libold.so $B/liblibtrig.so $B/libnew.so --n 65536 --reps 25 > gpurun_out/ab1.log 2>&1 || exit $?
cat gpurun_out/ab1.log | grep '^{'
timeout -k 10 300 python scripts/micro/ab.py $B/libold.so $B/liblibtrig.so $B/libnew.so --n 4194304 --k 50 --reps 9 > gpurun_out/ab2.log 2>&1 || exit $?
cat gpurun_out/ab2.log | grep '^{'
