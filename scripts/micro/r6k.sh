# round 6: where a block's waves run (wave_simd_probe), then ppo_head_kernel
# variants, alternating on one box: h0 = HEAD; h1 = the tile's dots by one
# reduce-scatter (133 VGPRs, 3 waves / SIMD); h1w = h1 capped at 128 VGPRs
# (4 waves, spills); h0r1 / h0r2 = HEAD with the policy / value wave pairs
# swapped on odd blocks / on blocks 256-511, 768-1023; then the PPO kernel
# tests on h1w
set -o pipefail
timeout -k 10 60 scripts/micro/build/wave_simd_probe || exit 1
for i in 1 2 3; do for v in h0 h1 h1w h0r1 h0r2; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/head_bench.py || exit 1; done; done
DRONERL_LIB=scripts/micro/build/lib_h1w.so timeout -k 10 400 python -u -m pytest tests/test_ppo_kernels_gpu.py tests/test_ppo_flagship_parity_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -3
