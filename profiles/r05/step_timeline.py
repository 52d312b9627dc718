"""One ADMM step's kernels and the gaps between them, from a rocprofv3 --kernel-trace CSV:
  python3 step_timeline.py run_kernel_trace.csv [step index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts at k_predict or, when the extrapolation is fused (2D, round 5), at the first x-update
# (the z-from-positions instance, k_xupdate<2, false, false, true, ...>)
idx = [i for i, r in enumerate(rows) if "k_predict" in r["Kernel_Name"] or "k_xupdate<2, false, false, true" in r["Kernel_Name"]]
a, b = idx[k], idx[k + 1]
prev = int(rows[a - 1]["End_Timestamp"])
busy = gaps = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void mmx::", "").replace("mmx::", "")
    print("%8.1f us  gap %6.1f us  %s" % ((e - s) / 1e3, (s - prev) / 1e3, name))
    busy += e - s
    gaps += max(0, s - prev)
    prev = e
print("step span %.1f us: kernels %.1f us, gaps %.1f us" % ((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3,
                                                          busy / 1e3, gaps / 1e3))
