#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only; never
# combined with sys/runtime traces) over a short eager bench run.
# Usage: scripts/pmc.sh <tag> <bench args...>
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$PWD/bench.py" --no-cpu-baseline --no-companion --no-graph "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -2 "$OUT/p$i.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
