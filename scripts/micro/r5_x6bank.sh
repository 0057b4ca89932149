#!/bin/bash
# Round 5: the x6 split-write swizzle.  Digests of the old (lib_base) and new
# library on the fixed-seed worker, alternating A/B timing, the x6 GPU tests,
# and the bank-conflict PMC pass of the new kernel.
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b; mkdir -p $O
B=$PWD/scripts/micro/build/lib_base.so
export PYTHONPATH=$PWD
for m in "384 1" "65536 64"; do
  timeout -k 10 120 env DRONERL_LIB=$B python tests/x6_forms_worker.py $m > $O/dig_base_${m// /_}.txt 2>&1 || exit 1
  timeout -k 10 120 python tests/x6_forms_worker.py $m > $O/dig_new_${m// /_}.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  timeout -k 10 120 env DRONERL_LIB=$B python scripts/micro/gemm_x6_bench.py > $O/ab_base_$i.json 2>$O/ab_base_$i.err || exit 1
  timeout -k 10 120 python scripts/micro/gemm_x6_bench.py > $O/ab_new_$i.json 2>$O/ab_new_$i.err || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 tests/test_gemm_x6_gpu.py > $O/test_x6.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc -o run -- python3 scripts/micro/gemm_x6_bench.py --reps 10 > $O/pmc.log 2>&1
echo pmc rc=$?
