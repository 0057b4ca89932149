# Kernel-level A/B of PPO kernel build variants (rocprofv3 kernel trace of a
# short PPO bench per variant, average duration of the matching kernels).
# Build on the CPU:  bash scripts/micro/ab_ppo_kern.sh build NAME "-DFLAG=V ..." ...
# Run on the box:    KERN="first_layer_bwd ppo_head" bash scripts/micro/ab_ppo_kern.sh run base NAME ...
B=scripts/micro/build
C=drone_rl_amd/csrc
if [ "$1" = build ]; then
  shift
  mkdir -p $B
  while [ $# -ge 2 ]; do
    name=$1 flags=$2; shift 2
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
      -fno-fast-math -Iinclude $flags -c $C/ppo_kernels.hip -o $B/ppo_$name.o &&
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $B/lib_$name.so \
      $C/build/env_kernels.o $C/build/gemm_x6.o $B/ppo_$name.o || exit 1
    rm -f $B/ppo_$name.o
  done
  exit 0
fi
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then unset DRONERL_LIB; else export DRONERL_LIB="$GRAFT_REPO_ROOT/$B/lib_$v.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kp_$v -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --ppo-updates 2 > gpurun_out/kp_$v.log 2>&1 || exit $?
  for k in ${KERN:-first_layer_bwd ppo_head}; do
    echo "$v $k: $(python3 scripts/micro/dbstats.py gpurun_out/kp_$v/run_results.db $k | head -2 | tr '\n' ' ')"
  done
  grep -o '"updates_per_s": [0-9.]*' gpurun_out/kp_$v.log | head -1
  rm -rf gpurun_out/kp_$v   # the SQLite traces (tens of MB) stay on the box
done
