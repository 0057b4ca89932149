# rocprofv3 kernel stats of 2 PPO updates (bench.py) with the product library
# and with DR_PPO_NT=1 (nontemporal activation / grad_z stores)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pnt0 -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --ppo-updates 2 > gpurun_out/pnt0.log 2>&1 &&
DRONERL_LIB=$GRAFT_REPO_ROOT/scripts/micro/build/lib_ppont.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pnt1 -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --ppo-updates 2 > gpurun_out/pnt1.log 2>&1 &&
grep -h '"ppo"' gpurun_out/pnt0.log gpurun_out/pnt1.log | python3 -c "import sys,json; [print(json.loads(l)['ppo']['updates_per_s']) for l in sys.stdin]"
