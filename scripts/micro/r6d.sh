# round 6: the X6_MFMA16 build (16x16x32 forward + fused input-gradient
# GEMMs) -- parity subset on its library, kernel times, PPO A/B vs the
# 32x32x16 build (alternating processes, one box)
set -o pipefail
mkdir -p gpurun_out/r6d
export DRONERL_LIB=scripts/micro/build/lib_m16.so
timeout -k 10 600 python -u -m pytest tests/test_gemm_x6_gpu.py tests/test_gemm_x6_fl_gpu.py tests/test_ppo_flagship_parity_gpu.py tests/test_trainer_knobs_gpu.py tests/test_ppo_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r6d/m16_tests.log 2>&1
echo "m16 tests rc=$?"; tail -15 gpurun_out/r6d/m16_tests.log
grep -q "Fatal\|Memory access fault\|core dumped" gpurun_out/r6d/m16_tests.log && exit 1
for v in m32 m16; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/gemm_x6_bench.py --reps 100 > gpurun_out/r6d/x6_$v.json || exit 1; tail -1 gpurun_out/r6d/x6_$v.json; DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/fl_bench.py > gpurun_out/r6d/fl_$v.json || exit 1; cat gpurun_out/r6d/fl_$v.json; done
for i in 1 2; do for v in m32 m16; do
DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion --rollout-k 0 > gpurun_out/r6d/bench_${v}_$i.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/r6d/bench_${v}_$i.json'));p=d['ppo'];print('$v',p['updates_per_s'],{k:v.get('isolated_us',v['prefix_split_us']) for k,v in p['roofline']['kernels_per_minibatch'].items()})"
done; done
