"""Per-kernel average duration (us) from a rocprofv3 SQLite result
(run_results.db): python scripts/micro/dbstats.py <db> [substr ...]"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
sub = sys.argv[2:]
rows = c.execute("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
                 "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
agg = defaultdict(list)
for name, ns in rows:
    agg[name].append(ns)
for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    if sub and not any(x in name for x in sub):
        continue
    print(f"{len(v):6d} {sum(v) / len(v) / 1e3:9.2f} us  {sum(v) / 1e6:8.2f} ms  {name[:90]}")
