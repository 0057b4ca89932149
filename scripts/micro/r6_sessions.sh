#!/bin/bash
# Round 6's GPU A/B sessions, one case per session (run through gpurun from the
# repo root, e.g. `bash scripts/micro/r6_sessions.sh g > gpurun_out/r6g.log 2>&1`).
# Library variants are built beforehand with scripts/micro/build_variant.sh
# into scripts/micro/build/lib_<tag>.so; the results are in profiles/r06_*.
set -o pipefail
case "$1" in
b)
  mkdir -p gpurun_out/r6b
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6b/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6b/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/r6b/gpu_tests.log
  for v in m32 m16; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 0.5 >> gpurun_out/r6b/sha.jsonl || exit 1; done
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6b/bench.json 2> gpurun_out/r6b/bench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6b/bench.json'));print(d['value'],d['roofline']['avg_launch_us'],d['roofline'].get('walls'),d['ppo']['updates_per_s'],d['ppo']['roofline']['dominant_kernel'])"
  ;;
c)
  mkdir -p gpurun_out/r6c
  for v in m32 m16; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 0.5 >> gpurun_out/r6c/sha.jsonl || exit 1; done
  cat gpurun_out/r6c/sha.jsonl
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6c/bench.json 2> gpurun_out/r6c/bench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6c/bench.json'));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r['frac_wall'],r.get('walls'),d['ppo']['updates_per_s'],d['ppo']['roofline']['dominant_kernel'],d['ppo']['roofline']['kernels_per_minibatch']['gather_minibatch'])"
  ;;
d)
  # round 6: the X6_MFMA16 build (16x16x32 forward + fused input-gradient
  # GEMMs) -- parity subset on its library, kernel times, PPO A/B vs the
  # 32x32x16 build (alternating processes, one box)
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
  ;;
e)
  # round 6: the 16x16x32-only library -- new x6 digests, the GPU suite, a bench
  mkdir -p gpurun_out/r6e
  for a in "384 1" "65536 64"; do PYTHONPATH=$PWD timeout -k 10 120 python tests/x6_forms_worker.py $a || exit 1; done
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6e/gpu_tests.log 2>&1
  echo "tests rc=$?"; grep -E "passed|failed|FAILED|Error" gpurun_out/r6e/gpu_tests.log | tail -15
  grep -q "Memory access fault\|core dumped" gpurun_out/r6e/gpu_tests.log && exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6e/bench.json 2> gpurun_out/r6e/bench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6e/bench.json'));r=d['roofline'];p=d['ppo'];print(d['value'],r['avg_launch_us'],r['frac'],r['frac_wall'],p['updates_per_s'],{k:v.get('isolated_us',v['prefix_split_us']) for k,v in p['roofline']['kernels_per_minibatch'].items()})"
  ;;
f)
  # round 6: PMC passes over the 16x16x32 x6 kernels and the head kernel
  bash scripts/micro/gemm_x6_pmc.sh > gpurun_out/r6f_gx6.log 2>&1; echo "gx6 rc=$?"; tail -4 gpurun_out/r6f_gx6.log
  FL=1 bash scripts/micro/gemm_x6_pmc.sh > gpurun_out/r6f_fl.log 2>&1; echo "fl rc=$?"; tail -3 gpurun_out/r6f_fl.log
  HEAD=1 bash scripts/micro/gemm_x6_pmc.sh > gpurun_out/r6f_head.log 2>&1; echo "head rc=$?"; tail -3 gpurun_out/r6f_head.log
  ;;
g)
  # round 6: the forward GEMM's split VALU interleaved with its MFMAs and its
  # memory instructions spread between them: bytes and time, alternating
  # processes, one box
  for i in 1 2 3; do for v in sa0m0 sa1m0 sa1m1; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 1 || exit 1; done; done
  ;;
h)
  # round 6: fl16 with its split pieces and memory instructions spread between
  # its MFMAs (flnew) vs HEAD (flold): bytes and time, alternating, one box
  for i in 1 2 3; do for v in flold flnew; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/fl_bench.py || exit 1; done; done
  for v in flold flnew; do
  DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion --rollout-k 0 > gpurun_out/r6h_bench_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r6h_bench_$v.json'));p=d['ppo'];print('$v',p['updates_per_s'],{k:v.get('isolated_us',v['prefix_split_us']) for k,v in p['roofline']['kernels_per_minibatch'].items()})"
  done
  ;;
i)
  # round 6: fl16's D2 epilogue VALU spread over the MFMA slots of k32 steps
  # 4 / 6 (d2new), + the forward's plane stores / staging DMA deferred into
  # the next step's MFMA slots (wsdef), vs HEAD (d2old): bytes and time,
  # alternating, one box; then the x6 parity tests on wsdef
  for i in 1 2 3; do for v in d2old d2new wsdef; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/fl_bench.py || exit 1; done; done
  for i in 1 2; do for v in d2old wsdef; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 1 || exit 1; done; done
  DRONERL_LIB=scripts/micro/build/lib_wsdef.so timeout -k 10 300 python -u -m pytest tests/test_gemm_x6_fl_gpu.py tests/test_gemm_x6_gpu.py tests/test_ppo_flagship_parity_gpu.py -q --timeout 200 --timeout-method thread 2>&1 | tail -3
  ;;
j)
  # round 6: the committed candidate (cur: ws16 deferred plane stores / DMA,
  # fl16 as HEAD) vs HEAD (d2old): fl / ws16 time, alternating; parity tests
  for i in 1 2; do for v in d2old cur; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/fl_bench.py || exit 1; done; done
  for i in 1 2; do for v in d2old cur; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/x6_shape_ab.py --warm-s 1 || exit 1; done; done
  timeout -k 10 400 python -u -m pytest tests/test_gemm_x6_fl_gpu.py tests/test_gemm_x6_gpu.py tests/test_ppo_flagship_parity_gpu.py -q --timeout 200 --timeout-method thread 2>&1 | tail -3
  ;;
k)
  # round 6: where a block's waves run (wave_simd_probe), then ppo_head_kernel
  # variants, alternating on one box: h0 = HEAD; h1 = the tile's dots by one
  # reduce-scatter (133 VGPRs, 3 waves / SIMD); h1w = h1 capped at 128 VGPRs
  # (4 waves, spills); h0r1 / h0r2 = HEAD with the policy / value wave pairs
  # swapped on odd blocks / on blocks 256-511, 768-1023; then the PPO kernel
  # tests on h1w
  timeout -k 10 60 scripts/micro/build/wave_simd_probe || exit 1
  for i in 1 2 3; do for v in h0 h1 h1w h0r1 h0r2; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/head_bench.py || exit 1; done; done
  DRONERL_LIB=scripts/micro/build/lib_h1w.so timeout -k 10 400 python -u -m pytest tests/test_ppo_kernels_gpu.py tests/test_ppo_flagship_parity_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -3
  ;;
l)
  # round 6: ppo_head_kernel's LDS-DMA row pipeline, alternating on one box
  # (head_bench.py: the trainer's contiguous actions / aux rows): cur = HEAD
  # build; p0 = this tree without the pipeline; p1 = pipeline (137 VGPRs, 3
  # waves / SIMD); p1b = p1 on 768 blocks; p1w = p1 capped at 128 VGPRs (8
  # spilled); p1rsw = p1w + the reduce-scatter dots; then the PPO kernel and
  # flagship parity tests on p1 and p1w
  for i in 1 2 3; do for v in cur p0 p1 p1b p1w p1rsw; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/head_bench.py || exit 1; done; done
  for v in p1 p1w; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_ppo_kernels_gpu.py tests/test_ppo_flagship_parity_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -3 || exit 1; done
  ;;
m)
  # round 6: the weight-gradient x6 GEMM's schedule, alternating on one box
  # (wgrad_ab.py, the trainer's shape): wg0 = HEAD; wg1 / wg2 = iglp_opt(0 / 1);
  # wg3 = a sched_group_barrier pipeline; wsj1 / wsj2 = the two waves of a SIMD
  # splitting the next stage at different points of the stage (j 1 / 3, 0 / 2)
  for i in 1 2 3; do for v in wg0 wg1 wg2 wg3 wsj1 wsj2; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/wgrad_ab.py || exit 1; done; done
  ;;
n)
  # round 6: iglp_opt(0) on the weight-gradient GEMM, alone and with the SIMD's
  # two waves splitting at different points (wg1sj1 / wg1sj2), and two
  # sched_group_barrier pipelines (wg5: a transposed read every 2 MFMAs;
  # wg3sj2), alternating on one box against HEAD (wg0)
  for i in 1 2 3; do for v in wg0 wg1 wg1sj1 wg1sj2 wg3 wg5 wg3sj2; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/wgrad_ab.py || exit 1; done; done
  ;;
o)
  # round 6: the weight-gradient GEMM with iglp_opt(0) (wgnew) against HEAD
  # (wg0) in the trainer: PPO updates/s from bench.py, alternating; then the
  # x6 GEMM and flagship parity tests on the new in-tree library
  mkdir -p gpurun_out/r6o
  for i in 1 2 3; do for v in wg0 wgnew; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion > gpurun_out/r6o/b_${v}_$i.log 2>&1 || exit 1; python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ppo']['updates_per_s'], d['ppo']['roofline']['kernels_per_minibatch']['gemm_x6_wgrad'].get('isolated_us'))" gpurun_out/r6o/b_${v}_$i.log $v; done; done
  timeout -k 10 400 python -u -m pytest tests/test_gemm_x6_gpu.py tests/test_gemm_x6_fl_gpu.py tests/test_ppo_flagship_parity_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -3
  ;;
p)
  # the first-layer forward (dr_linear_tanh2_x6, the trainer's form, and the
  # plain dr_linear_tanh2) under launch shapes: lt0 = HEAD (64 rows per
  # block, <= 1,024 blocks per net); ltb512 = <= 512 blocks; ltb2k = 32 rows
  # per block, <= 2,048; ltr128 = 128 rows, <= 512
  for i in 1 2 3; do for v in lt0 ltb512 ltb2k ltr128; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/lt_ab.py || exit 1; done; done
  ;;
q)
  # the first-layer forward with its input rows loaded 1 (HEAD) / 2 / 3 / 4
  # rows ahead (DR_LT_PF; scalar loads; the knob is not kept); lth / lthpf2: two waves per row
  # (DR_LT_HALF: 50 VGPRs, 8 waves per SIMD), with PF 1 / 2
  for i in 1 2 3; do for v in ltpf1 ltpf2 ltpf3 ltpf4 lth lthpf2; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/lt_ab.py || exit 1; done; done
  ;;
r)
  # the record gather with the block's records loaded cooperatively into LDS
  # (gc1: eight threads per 128-B record) against HEAD (gc0)
  for i in 1 2 3; do for v in gc0 gc1; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/gather_bench.py || exit 1; done; done
  ;;
s)
  # the weight gradient's stage-start reads: H tile 0 and G tile 0 issued
  # first (wgo1, with iglp_opt(0); wgo1n without) against the product (wgc)
  for i in 1 2 3; do for v in wgc wgo1 wgo1n; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/wgrad_ab.py || exit 1; done; done
  ;;
t)
  # the driver's multi-rank command form on the one-GPU box, both ranks on the
  # card over gloo (RCCL refuses two ranks per device), then a second seed of
  # the staged-curriculum convergence run on the final kernels
  DRONERL_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --steps 20 --warmup 5 > gpurun_out/r06_n2_gloo.log 2>&1 || exit 1
  grep '^{' gpurun_out/r06_n2_gloo.log | tail -1 > gpurun_out/r06_n2_gloo.json
  ENT=0.01 TAG=r06_ppo_c3_staged_ent01 SEEDS=1 bash scripts/c3_staged.sh > gpurun_out/r06_c3_s1.log 2>&1
  ;;
u)
  # the first layer's dot products on the x6 MFMA path (lm1: 512 blocks per
  # net, 4-byte column stores; lm2 / lm2b: the transposed product with 16-byte
  # row stores, 512 / 1,024 blocks) against the FMA-chain kernel (lm0); then the
  # first-layer, x6 and PPO tests on lm2
  for i in 1 2 3; do for v in lm0 lm1 lm2 lm2b; do DRONERL_LIB=scripts/micro/build/lib_$v.so timeout -k 10 120 python scripts/micro/lt_ab.py || exit 1; done; done
  DRONERL_LIB=scripts/micro/build/lib_lm2.so timeout -k 10 600 python -u -m pytest tests/test_ppo_kernels_gpu.py tests/test_gemm_x6_fl_gpu.py tests/test_trainer_knobs_gpu.py tests/test_ppo_flagship_parity_gpu.py tests/test_ppo_gpu.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -15
  ;;
*) echo "usage: $0 b|c|...|o"; exit 2 ;;
esac
