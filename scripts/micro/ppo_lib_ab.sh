# rocprofv3 kernel stats of 2 PPO updates (bench.py) with the product library
# and with an A/B variant library (arg 1: path under scripts/micro/build)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab0 -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --ppo-updates 2 > gpurun_out/ab0.log 2>&1 &&
DRONERL_LIB=$GRAFT_REPO_ROOT/scripts/micro/build/$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab1 -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --ppo-updates 2 > gpurun_out/ab1.log 2>&1 &&
grep -h '"ppo"' gpurun_out/ab0.log gpurun_out/ab1.log | python3 -c "import sys,json; [print(json.loads(l)['ppo']['updates_per_s']) for l in sys.stdin]"
