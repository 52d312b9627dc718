#!/usr/bin/env python3
"""rocprofv3 --kernel-trace database (rocpd SQLite, the rocprofv3 7.x default output) -> the same
summaries as the CSV runs of earlier rounds: per-kernel statistics (calls, total, average, min,
max ns; kernel_stats_*.csv) and per-(kernel, grid size) averages (kernel_trace_by_grid.txt, the form
bench.py's roofline is checked against: one kernel name serves several workloads of different
sizes).  Usage: rocpd_summary.py run_results.db out_dir [tag]"""
import csv
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    db, out = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else "bench"
    os.makedirs(out, exist_ok=True)
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, accum_vgpr_count, "
                     "scratch_size, lds_size from kernels").fetchall()
    by = defaultdict(list)
    grid = defaultdict(list)
    res = {}
    for name, dur, gx, gy, gz, wx, vg, ag, scr, lds in rows:
        by[name].append(dur)
        grid[(name, gx * gy * gz)].append(dur)
        res[name] = (wx, vg, ag, scr, lds)
    tot = sum(sum(v) for v in by.values())
    with open(os.path.join(out, "kernel_stats_%s.csv" % tag), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "Workgroup",
                    "VGPRs", "AGPRs", "ScratchBytesPerLane", "LDSBytes"])
        for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            wx, vg, ag, scr, lds = res[name]
            w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / tot, 3), min(v), max(v),
                        wx, vg, ag, scr, lds])
    with open(os.path.join(out, "kernel_trace_by_grid_%s.txt" % tag), "w") as f:
        f.write("# kernel | grid (work-items) | launches | average us | min us | max us\n")
        for (name, g), v in sorted(grid.items(), key=lambda kv: -sum(kv[1])):
            if sum(v) < 1e-3 * tot:
                continue
            f.write("%s | %d | %d | %.2f | %.2f | %.2f\n" % (name, g, len(v), sum(v) / len(v) / 1e3, min(v) / 1e3,
                                                            max(v) / 1e3))


if __name__ == "__main__":
    main()
