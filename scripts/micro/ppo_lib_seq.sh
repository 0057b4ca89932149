# Sequential A/B of PPO library variants in one box session (ABAB...):
# bench.py PPO-only runs; args: variant .so names under scripts/micro/build
# ("base" = the product library).  Prints updates/s per run.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset DRONERL_LIB; else export DRONERL_LIB="$GRAFT_REPO_ROOT/scripts/micro/build/$v"; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 5 \
        --ppo-updates 4 > gpurun_out/seq_$v.log 2>&1 || exit $?
    echo "$rep $v $(grep -o '"updates_per_s": [0-9.]*' gpurun_out/seq_$v.log)"
  done
done
