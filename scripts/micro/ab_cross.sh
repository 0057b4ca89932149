B=scripts/micro/build/libnew.so
for spec in "262144 200 15" "524288 100 11" "1048576 100 11" "2097152 50 9"; do
  read n k reps <<< "$spec"
  timeout -k 10 300 python scripts/micro/ab.py $B:DRONERL_ROWS_PER_WAVE=64 $B:DRONERL_ROWS_PER_WAVE=32 --n $n --k $k --reps $reps > gpurun_out/abx.log 2>&1 || exit $?
  echo "n=$n $(grep '^{' gpurun_out/abx.log)"
done
