ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 400 bash scripts/micro/rollout_pmc.sh > gpurun_out/pmc_rollout.log 2>&1; rc=$?; tail -40 gpurun_out/pmc_rollout.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash scripts/rollout_traffic.sh > gpurun_out/rollout_traffic.log 2>&1; rc=$?; tail -8 gpurun_out/rollout_traffic.log; exit $rc
