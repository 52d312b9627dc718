"""SQ stall summary of one rocprofv3 --pmc pass (SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES): per prox / x-update
kernel, the fractions of a wave's cycles waiting on memory (wait_any), on instruction dependencies
(wait_inst), issuing (active) and issuing VALU, VALU instructions and cycles per wave.
Usage: python sq_report.py <rocprofv3 output dir>"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in d.items():
    if "prox" not in k and "xupdate" not in k:
        continue
    n = len(c["SQ_WAVES"])
    avg = {m: sum(v) / len(v) for m, v in c.items()}
    wc = avg["SQ_WAVE_CYCLES"]
    print(k[:60], "launches", n, "waves %.0f" % avg["SQ_WAVES"],
          "wait_any %.2f wait_inst %.2f active %.2f active_valu %.2f" % (
              avg["SQ_WAIT_ANY"] / wc, avg["SQ_WAIT_INST_ANY"] / wc, avg["SQ_ACTIVE_INST_ANY"] / wc,
              avg["SQ_ACTIVE_INST_VALU"] / wc),
          "valu_insts/wave %.0f" % (avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]),
          "wave_cycles/wave %.0f" % (4 * wc / avg["SQ_WAVES"]))
