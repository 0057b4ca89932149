"""Summarise scripts/pmc.sh output: per-dispatch averages of every collected
counter for one kernel, plus derived HBM traffic.

HBM bytes per dispatch, following MI355X_MICROARCH.md (HBM / rocprofv3):
  FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE = TCC_EA0_RDREQ x 64 B
  and on gfx950 it reports HALF the bytes of a wide coalesced streaming
  read, so the corrected read bytes are TCC_EA0_RDREQ x 128 B when every
  request is a full 128-B line (checked here: the corrected figure is
  compared with the kernel's algorithmic read bytes).  WRITE_SIZE is exact
  for 16-B-per-lane streaming stores.

Usage: python scripts/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, kern):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
        by_dispatch = defaultdict(dict)
        for r in rows:
            by_dispatch[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            by_dispatch[int(r["Dispatch_Id"])]["_grid"] = int(r["Grid_Size"])
            by_dispatch[int(r["Dispatch_Id"])]["_dur"] = (int(r["End_Timestamp"]) -
                                                          int(r["Start_Timestamp"]))
        ids = sorted(by_dispatch)
        ids = ids[len(ids) // 5:]          # drop warm-up dispatches
        for i in ids:
            for k, v in by_dispatch[i].items():
                vals[k].append(v)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    d = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "env_step"
    m = load(d, kern)
    out = dict(m)
    if "TCC_EA0_RDREQ_sum" in m:
        out["hbm_read_bytes_rdreq128"] = m["TCC_EA0_RDREQ_sum"] * 128
        out["hbm_read_bytes_rdreq64"] = m["TCC_EA0_RDREQ_sum"] * 64
    if "FETCH_SIZE" in m:
        out["fetch_bytes_raw"] = m["FETCH_SIZE"] * 1024
        out["fetch_bytes_x2"] = m["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in m:
        out["write_bytes"] = m["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
        out["valu_insts_per_wave"] = m.get("SQ_INSTS_VALU", 0) / max(m.get("SQ_WAVES", 1), 1)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
