# round 6: ppo_head_kernel's LDS-DMA row pipeline, alternating on one box
# (head_bench.py: the trainer's contiguous actions / aux rows): cur = HEAD
# build; p0 = this tree without the pipeline; p1 = pipeline (137 VGPRs, 3
# waves / SIMD); p1b = p1 on 768 blocks; p1w = p1 capped at 128 VGPRs (8
# spilled); p1rsw = p1w + the reduce-scatter dots; then the PPO kernel and
# flagship parity tests on p1 and p1w
set -o pipefail
for i in 1 2 3; do for v in cur p0 p1 p1b p1w p1rsw; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/head_bench.py || exit 1; done; done
for v in p1 p1w; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_ppo_kernels_gpu.py tests/test_ppo_flagship_parity_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -3 || exit 1; done
