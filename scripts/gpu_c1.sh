mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -4 gpurun_out/t.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -m drone_rl_amd.train --sb3-defaults --envs 1 --total-steps 2e6 --log-every 10 --checkpoint gpurun_out/c1_gpu.zip > gpurun_out/c1_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/c1_gpu.log; exit $rc
