# round 6: the weight-gradient GEMM with iglp_opt(0) (wgnew) against HEAD
# (wg0) in the trainer: PPO updates/s from bench.py, alternating; then the
# x6 GEMM and flagship parity tests on the new in-tree library
set -o pipefail
mkdir -p gpurun_out/r6o
for i in 1 2 3; do for v in wg0 wgnew; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion > gpurun_out/r6o/b_${v}_$i.log 2>&1 || exit 1; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ppo']['updates_per_s'], d['ppo']['roofline']['kernels_per_minibatch']['gemm_x6_wgrad'].get('isolated_us'))" gpurun_out/r6o/b_${v}_$i.log $v; done; done
timeout -k 10 400 python -u -m pytest tests/test_gemm_x6_gpu.py tests/test_gemm_x6_fl_gpu.py tests/test_ppo_flagship_parity_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -3
