ulimit -c 0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_rollout_gpu.py tests/test_env_gpu.py > gpurun_out/t_ro.log 2>&1; rc=$?; tail -3 gpurun_out/t_ro.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="0 mwr0" timeout -k 10 400 bash scripts/micro/ws_ablate.sh
