"""Per-kernel HBM traffic from the two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: they cannot
share a pass on gfx950) -> profiles/pmc_summary.json, read by bench.py for roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of 16-byte-per-lane
coalesced streaming reads (MI355X_MICROARCH.md §HBM); `hbm_bytes_per_launch` applies that x2 to the
fetch side (the prox kernel's bulk read, Bkinv, is such a stream), `hbm_bytes_raw_per_launch` does
not.  Other access widths are uncalibrated, so the truth lies between the two for mixed kernels.

  python profiles/make_pmc_summary.py profiles/r01/pmc/fetch_size_counter_collection.csv \
         profiles/r01/pmc/write_size_counter_collection.csv
"""
import collections
import csv
import json
import os
import re
import sys


def load(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def short(name):
    m = re.match(r"(?:void )?mmx::(\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name


def main(fetch, write):
    f, w = load(fetch), load(write)
    out = {"source": [os.path.relpath(fetch), os.path.relpath(write)], "units": "bytes per launch"}
    for k in f:
        if not k.startswith(("void mmx::", "mmx::")):
            continue
        fk = sum(f[k]) / len(f[k])
        wk = sum(w.get(k, [0.0])) / max(len(w.get(k, [])), 1)
        out[short(k)] = {"launches": len(f[k]), "fetch_kib_raw": round(fk, 1), "write_kib": round(wk, 1),
                         "hbm_bytes_per_launch": round((2 * fk + wk) * 1024),
                         "hbm_bytes_raw_per_launch": round((fk + wk) * 1024)}
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "pmc_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
