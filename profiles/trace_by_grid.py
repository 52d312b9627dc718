"""Per kernel and grid size totals from a rocprofv3 kernel-trace CSV (a kernel launched at several
sizes, e.g. the 2D prox at C3 and at C2, gets one line per size).
Usage: python profiles/trace_by_grid.py trace.csv > kernel_trace_by_grid.txt"""
import csv
import re
import sys
from collections import defaultdict

d = defaultdict(list)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        d[(r["Kernel_Name"], int(r.get("Grid_Size") or r["Grid_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(" total_ms  calls   avg_ms      grid  kernel")
for (k, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    m = re.match(r"(?:void )?((?:mmx::)?(?:\(anonymous namespace\)::)?[\w:]+(?:<[^>]*>)?)", k)
    print(f"{sum(v) / 1e6:9.3f} {len(v):6d} {sum(v) / len(v) / 1e6:8.4f} {g:9d}  {m.group(1) if m else k}")
