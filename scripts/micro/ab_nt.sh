# In-process A/B: nontemporal state loads (DR_NT_LOADS) on top of nontemporal
# stores, with 64 / 32 rows per wave, at the large sizes
B=scripts/micro/build
mkdir -p gpurun_out
for spec in "524288 100 11" "1048576 100 11" "2097152 50 9" "4194304 30 9"; do
  read n k reps <<< "$spec"
  timeout -k 10 300 python scripts/micro/ab.py $B/lib_nt.so:DRONERL_ROWS_PER_WAVE=64 $B/lib_ntl.so:DRONERL_ROWS_PER_WAVE=64 $B/lib_nt.so:DRONERL_ROWS_PER_WAVE=32 $B/lib_ntl.so:DRONERL_ROWS_PER_WAVE=32 --n $n --k $k --reps $reps > gpurun_out/abn.log 2>&1 || exit $?
  echo "n=$n $(grep '^{' gpurun_out/abn.log)"
done
