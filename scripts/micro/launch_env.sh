# Launch-path diagnostics of the 65,536-env step (GPU box):
#  1. the step split over S shards on S streams (scripts/micro/streams.py);
#  2. the env-only bench with kernel arguments forced into device memory or
#     not (HIP_FORCE_DEV_KERNARG), alternated to average out box drift.
mkdir -p gpurun_out
timeout -k 10 200 python scripts/micro/streams.py > gpurun_out/streams.log 2>&1 || exit $?
grep 'S=' gpurun_out/streams.log
for v in 1 0 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python bench.py --no-cpu-baseline --ppo-updates 0 \
    --steps 2000 > gpurun_out/karg_$v.log 2>&1 || exit $?
  echo "DEV_KERNARG=$v $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/karg_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/karg_$v.log)"
done
