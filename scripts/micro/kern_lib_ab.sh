# rocprofv3 kernel-trace of a short PPO bench for each library variant
# (args: .so names under scripts/micro/build, "base" = product library);
# prints the average duration of kernels matching $KERN (default linear_tanh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
K=${KERN:-linear_tanh}
for v in "$@"; do
  if [ "$v" = base ]; then unset DRONERL_LIB; else export DRONERL_LIB="$GRAFT_REPO_ROOT/scripts/micro/build/$v"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kl_$v -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --ppo-updates 1 > gpurun_out/kl_$v.log 2>&1 || exit $?
  echo "$v: $(python3 scripts/micro/dbstats.py gpurun_out/kl_$v/run_results.db $K | head -3)"
done
