ulimit -c 0
B=scripts/micro/build
timeout -k 10 200 python scripts/micro/ab.py $B/libdr_a0.so $B/libdr_a2.so $B/libdr_a5.so $B/libdr_hoist.so --n 65536 --k 200 --reps 25 > gpurun_out/ab_ablate.log 2>&1 || exit $?
grep '^{' gpurun_out/ab_ablate.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ppo_kernels_gpu.py -k permutation > gpurun_out/t_perm.log 2>&1; rc=$?; tail -15 gpurun_out/t_perm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1; rc=$?; tail -15 gpurun_out/t_all.log; exit $rc
