ulimit -c 0
B=scripts/micro/build
timeout -k 10 200 python scripts/micro/ab.py $B/libdr_a0.so $B/libdr_new.so $B/libdr_pre.so --n 65536 --k 200 --reps 25 > gpurun_out/ab_pre.log 2>&1 || exit $?
grep '^{' gpurun_out/ab_pre.log
timeout -k 10 200 python scripts/micro/ab.py $B/libdr_a0.so $B/libdr_new.so $B/libdr_pre.so --n 4194304 --k 50 --reps 9 > gpurun_out/ab_pre4m.log 2>&1 || exit $?
grep '^{' gpurun_out/ab_pre4m.log
timeout -k 10 200 python scripts/micro/ab.py $B/libdr_a0.so $B/libdr_pre.so --n 131072 --k 100 --reps 15 --variant 2 > gpurun_out/ab_pre_mov.log 2>&1 || exit $?
grep '^{' gpurun_out/ab_pre_mov.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_env_gpu.py tests/test_env_edge_gpu.py tests/test_moving_gpu.py tests/test_vecenv_dp_gpu.py tests/test_c_abi.py > gpurun_out/t_env.log 2>&1; rc=$?; tail -5 gpurun_out/t_env.log; exit $rc
