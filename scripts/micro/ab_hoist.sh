# In-process A/B of the reset-path variants (see scripts/micro/ab.py)
B=scripts/micro/build
mkdir -p gpurun_out
timeout -k 10 300 python scripts/micro/ab.py $B/lib_old.so $B/lib_hu.so $B/lib_hupf.so $B/lib_hupfh.so --n 65536 --k 200 --reps 25 > gpurun_out/abh1.log 2>&1 &&
timeout -k 10 300 python scripts/micro/ab.py $B/lib_old.so $B/lib_hu.so $B/lib_hupf.so $B/lib_hupfh.so --n 131072 --k 200 --reps 25 > gpurun_out/abh3.log 2>&1 &&
timeout -k 10 300 python scripts/micro/ab.py $B/lib_old.so $B/lib_hu.so $B/lib_hupf.so $B/lib_hupfh.so --n 4194304 --k 30 --reps 9 > gpurun_out/abh2.log 2>&1 &&
grep -h '^{' gpurun_out/abh1.log gpurun_out/abh3.log gpurun_out/abh2.log
