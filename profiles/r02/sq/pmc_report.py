import csv, sys, glob, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in d.items():
    if "prox" not in k and "xupdate" not in k: continue
    n = len(c["SQ_WAVES"])
    avg = {m: sum(v) / len(v) for m, v in c.items()}
    wc = avg["SQ_WAVE_CYCLES"]
    print(k[:60], "launches", n, "waves %.0f" % avg["SQ_WAVES"],
          "wait_any %.2f wait_inst %.2f active %.2f active_valu %.2f" % (avg["SQ_WAIT_ANY"] / wc, avg["SQ_WAIT_INST_ANY"] / wc, avg["SQ_ACTIVE_INST_ANY"] / wc, avg["SQ_ACTIVE_INST_VALU"] / wc),
          "valu_insts/wave %.0f" % (avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]), "wave_cycles/wave %.0f" % (4 * wc / avg["SQ_WAVES"]))
