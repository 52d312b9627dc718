"""Per-kernel HBM traffic from the two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: they cannot
share a pass on gfx950) -> profiles/pmc_summary.json, read by bench.py for roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of 16-byte-per-lane
coalesced streaming reads (MI355X_MICROARCH.md §HBM); round 4 calibrated the kernels' other read
widths the same way (8 B per lane, 24-B records, random records: also half, 128-B lines tallied at
64 B; WRITE_SIZE exact for 8-B plain and nontemporal stores; profiles/r04/calib/), so
`hbm_bytes_per_launch` applies the x2 to every kernel's fetch side; `hbm_bytes_raw_per_launch` is
the uncorrected figure.

  python profiles/make_pmc_summary.py profiles/r05/pmc/fetch_counter_collection.csv.gz \
         profiles/r05/pmc/write_counter_collection.csv.gz profiles/r05/pmc/f64_counter_collection.csv.gz \
         bfgs_heavy=profiles/r05/pmc/f64b_counter_collection.csv.gz

(round 5, as round 4: each pass is its own rocprofv3 run of `bench.py --steps 10 --warmup 2 --no-cpu-baseline
--no-bfgs`, dev/r5_final_pmc.sh; the f64 pass of the BFGS-heavy section alone is profiles/r04/bfgs_only.py;
the summary holds only the kernels those runs launched)

The optional third pass (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, wave instructions) gives
`fp64_flops_per_launch` = 64 lanes x (ADD + MUL + 2 FMA + TRANS): executed fp64 work, including
the correctly rounded powers' double-double arithmetic.
"""
import collections
import csv
import gzip
import json
import os
import re
import sys


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def load(path):
    """kernel -> grid size -> counter values (a kernel launched at several sizes, e.g. the 2D prox
    at C3 and at C2, is summarised per size)"""
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(_open(path)):
        d[r["Kernel_Name"]][int(r["Grid_Size"])].append(float(r["Counter_Value"]))
    return d


def short(name):
    m = re.match(r"(?:void )?mmx::(?:\(anonymous namespace\)::)?(\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name


def load_f64(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(_open(path)):
        d[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in d.items():
        mean = {name: sum(v) / len(v) for name, v in c.items()}
        out[k] = round(64 * (mean.get("SQ_INSTS_VALU_ADD_F64", 0) + mean.get("SQ_INSTS_VALU_MUL_F64", 0) +
                             2 * mean.get("SQ_INSTS_VALU_FMA_F64", 0) + mean.get("SQ_INSTS_VALU_TRANS_F64", 0)))
    return out


def main(fetch, write, f64=None, *tagged):
    """tagged: "name=path" f64 passes of single workloads, summarised as "<kernel>@name" (largest grid)"""
    f, w = load(fetch), load(write)
    fl = load_f64(f64) if f64 else {}
    out = {"source": [os.path.relpath(p) for p in (fetch, write, f64) if p], "units": "bytes per launch",
           "note": "per kernel: the launches of its largest grid (the headline-size workload); other grid "
                   "sizes under by_grid"}

    def entry(k, g):
        fk = sum(f[k][g]) / len(f[k][g])
        wl = w.get(k, {}).get(g, [])
        wk = sum(wl) / max(len(wl), 1)
        e = {"grid_size": g, "launches": len(f[k][g]), "fetch_kib_raw": round(fk, 1), "write_kib": round(wk, 1),
             "hbm_bytes_per_launch": round((2 * fk + wk) * 1024), "hbm_bytes_raw_per_launch": round((fk + wk) * 1024)}
        if (k, g) in fl:
            e["fp64_flops_per_launch"] = fl[(k, g)]
        return e

    for k in f:
        if not k.startswith(("void mmx::", "mmx::")):
            continue
        grids = sorted(f[k], reverse=True)
        e = entry(k, grids[0])
        if len(grids) > 1:
            e["by_grid"] = {str(g): entry(k, g) for g in grids[1:]}
        out[short(k)] = e
    for t in tagged:
        name, path = t.split("=", 1)
        out["source"].append(os.path.relpath(path))
        best = {}
        for (k, g), v in load_f64(path).items():
            if k.startswith(("void mmx::", "mmx::")) and g >= best.get(k, (0, 0))[0]:
                best[k] = (g, v)
        for k, (g, v) in best.items():
            out[short(k) + "@" + name] = {"grid_size": g, "fp64_flops_per_launch": v}
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "pmc_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
