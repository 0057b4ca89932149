# Launch-form sweep of env_step_kernel: rows per wave (64/32) x nontemporal
# state loads (0/1), forced through DRONERL_ROWS_PER_WAVE / DRONERL_NT_LOADS,
# one in-process A/B per size (scripts/micro/ab.py).
B=scripts/micro/build/lib_sw.so
mkdir -p gpurun_out
for spec in "65536 200 21" "131072 200 21" "262144 200 15" "524288 100 11" "1048576 100 11" "2097152 50 9" "4194304 30 9"; do
  read n k reps <<< "$spec"
  timeout -k 10 300 python scripts/micro/ab.py $B:DRONERL_ROWS_PER_WAVE=64,DRONERL_NT_LOADS=0 $B:DRONERL_ROWS_PER_WAVE=64,DRONERL_NT_LOADS=1 $B:DRONERL_ROWS_PER_WAVE=32,DRONERL_NT_LOADS=0 $B:DRONERL_ROWS_PER_WAVE=32,DRONERL_NT_LOADS=1 --n $n --k $k --reps $reps > gpurun_out/absw.log 2>&1 || exit $?
  echo "n=$n $(grep '^{' gpurun_out/absw.log | sed 's/lib_sw.so:DRONERL_ROWS_PER_WAVE=//g; s/,DRONERL_NT_LOADS=/ ntl/g')"
done
