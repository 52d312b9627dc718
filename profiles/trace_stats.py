"""Per-kernel statistics (rocprofv3 --stats layout) from a rocprofv3 kernel-trace CSV
(out_kernel_trace.csv / *_kernel_trace.csv): Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, StdDev.  Usage: python profiles/trace_stats.py trace.csv > kernel_stats.csv"""
import csv
import math
import sys
from collections import defaultdict

d = defaultdict(list)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        d[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    s = sum(v)
    m = s / len(v)
    sd = math.sqrt(sum((x - m) ** 2 for x in v) / len(v))
    w.writerow([k, len(v), s, round(m, 3), round(100.0 * s / tot, 2), min(v), max(v), round(sd, 3)])
