#!/bin/bash
# gather_minibatch_kernel: FETCH_SIZE / WRITE_SIZE per dispatch against its
# algorithmic bytes, and its kernel-trace duration (separate passes)
cd "$(dirname "$0")/../.."
O=$PWD/gpurun_out/r5g; mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $PWD/scripts/micro/gather_pmc.py 1 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/p$i.log; exit $rc; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $PWD/scripts/micro/gather_pmc.py 1 > $O/kt.log 2>&1 || exit 1
rm -f $O/kt/*kernel_trace.csv
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gather_minibatch" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, len(v), sum(v) / len(v))
for f in glob.glob(O + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gather_minibatch" in r["Name"]:
            print("time", r["Calls"], float(r["AverageNs"]) / 1e3)
PY
