# round 6: PMC passes over the 16x16x32 x6 kernels and the head kernel
set -o pipefail
bash scripts/micro/gemm_x6_pmc.sh > gpurun_out/r6f_gx6.log 2>&1; echo "gx6 rc=$?"; tail -4 gpurun_out/r6f_gx6.log
FL=1 bash scripts/micro/gemm_x6_pmc.sh > gpurun_out/r6f_fl.log 2>&1; echo "fl rc=$?"; tail -3 gpurun_out/r6f_fl.log
HEAD=1 bash scripts/micro/gemm_x6_pmc.sh > gpurun_out/r6f_head.log 2>&1; echo "head rc=$?"; tail -3 gpurun_out/r6f_head.log
