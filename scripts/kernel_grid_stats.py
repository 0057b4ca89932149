"""Per-(kernel, grid) duration statistics from a rocprofv3 --kernel-trace csv.

`--stats` averages every dispatch of a kernel name together, so the headline
rollout kernel's K = 32 launches on 65,536 envs share one average with
bench.py's host-floor probe (the same kernel on 64 envs, one step).  This
splits the trace by grid size and writes, per kernel and grid, the dispatch
count and the mean / median / min / max duration in microseconds.

  python scripts/kernel_grid_stats.py <run_kernel_trace.csv> <out.json> [substr ...]
(substr: keep only kernel names containing one of them)
"""
import csv
import json
import statistics
import sys


def grid_of(row):
    if row.get("Grid_Size"):
        return int(row["Grid_Size"])
    g = 1
    for ax in ("X", "Y", "Z"):
        v = row.get(f"Grid_Size_{ax}")
        if v:
            g *= int(v)
    return g


def summarise(path, keep=()):
    groups = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if keep and not any(k in name for k in keep):
                continue
            us = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            groups.setdefault((name, grid_of(row)), []).append(us)
    out = []
    for (name, grid), v in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        out.append({"kernel": name, "grid": grid, "dispatches": len(v),
                    "mean_us": round(statistics.fmean(v), 3),
                    "median_us": round(statistics.median(v), 3),
                    "min_us": round(min(v), 3), "max_us": round(max(v), 3)})
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1], tuple(sys.argv[3:]))
    with open(sys.argv[2], "w") as f:
        json.dump(res, f, indent=1)
    for r in res:
        print(json.dumps(r))
