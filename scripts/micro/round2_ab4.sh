ulimit -c 0
B=scripts/micro/build
timeout -k 10 200 python scripts/micro/ab.py $B/libdr_a0.so $B/libdr_new.so $B/libdr_new2.so $B/libdr_early.so --n 65536 --k 200 --reps 25 > gpurun_out/ab_e.log 2>&1 || exit $?
grep '^{' gpurun_out/ab_e.log
timeout -k 10 200 python scripts/micro/ab.py $B/libdr_a0.so $B/libdr_new2.so $B/libdr_early.so --n 4194304 --k 50 --reps 9 > gpurun_out/ab_e4m.log 2>&1 || exit $?
grep '^{' gpurun_out/ab_e4m.log
