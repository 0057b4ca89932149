# In-process A/B: waves per workgroup of env_step_kernel (DR_ENV_WPB 1 / 2 / 4).
# Build on the CPU first:   bash scripts/micro/ab_wpb.sh build
# then on the GPU box:      bash scripts/micro/ab_wpb.sh
# Round 1 result (f64, gym): equal within noise at 65,536 / 131,072 envs,
# 4 waves best at 4M (234 us vs 239 / 249 us) -- 4 is kept.
B=scripts/micro/build
C=drone_rl_amd/csrc
if [ "$1" = build ]; then
  mkdir -p $B
  for w in 1 2 4; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
      -fno-fast-math -Iinclude -DDR_ENV_WPB=$w -c $C/env_kernels.hip -o $B/env_w$w.o &&
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $B/lib_w$w.so \
      $B/env_w$w.o $C/build/ppo_kernels.o || exit 1
  done
  exit 0
fi
mkdir -p gpurun_out
for spec in "65536 200 15" "131072 200 15" "4194304 30 9"; do
  read n k reps <<< "$spec"
  timeout -k 10 300 python scripts/micro/ab.py $B/lib_w4.so $B/lib_w2.so $B/lib_w1.so \
    --n $n --k $k --reps $reps > gpurun_out/abw.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/abw.log)"
done
