"""Per-kernel HBM traffic of the LASolver kernels from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
dev/r5_la_pmc.sh (FETCH_SIZE x2 on gfx950, as profiles/make_pmc_summary.py), against the algorithmic
bytes of a triangular sweep, 12 nnz(triangle) + 16 n (values + column indices, right-hand side + result)."""
import collections, csv, json, sys


def load(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def short(k):
    return k.replace("void ", "").replace("mmx::(anonymous namespace)::", "").replace("mmx::", "").split("(")[0]


out = {}
for tag, f, w, n, nnz in (("3d_c4", sys.argv[1], sys.argv[2], 1536573, 68267943),
                          ("2d_n2M", sys.argv[3], sys.argv[4], 2002226, 28008516)):
    F, W = load(f), load(w)
    alg = 12 * (nnz - n) / 2 + 16 * n
    for k in F:
        if "sweep" not in k and "factor" not in k:
            continue
        fb = 2 * 1024 * sum(F[k]) / len(F[k])
        wb = 1024 * sum(W.get(k, [0])) / max(len(W.get(k, [])), 1)
        e = {"launches": len(F[k]), "hbm_bytes_per_launch": round(fb + wb), "fetch_bytes": round(fb), "write_bytes": round(wb)}
        if "sweep" in k:
            e["algorithmic_bytes"] = round(alg)
            e["ratio"] = round((fb + wb) / alg, 2)
        out[tag + ":" + short(k)] = e
print(json.dumps(out, indent=1))
