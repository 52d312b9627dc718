"""Numeric ILU(0) factor times by method on the bench's patterns: 3D C4 (SquareGrid n=63, 1,536,573
rows) and 2D (SquareGrid n=707, 2,002,226 rows): one wavefront per row (MMX_FACTOR=wave), the
lane-per-row level factor (level), and in 2D the chain/band factor (default); factors must be
bit-identical."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "..", "mm-admm_amd", "python"))
import numpy as np
import lasolver_amd as la
import mmadmm_amd as mx
MODES = sys.argv[1:] or None
for dim, n, modes in ((3, 63, ["wave", "level", "wave"]), (2, 707, ["chain", "wave", "level", "chain", "wave"])):
    if MODES:
        modes = [m for m in MODES if not (dim == 3 and m.startswith("chain"))]
    mesh = mx.MeshData.rect(dim, n)
    s = la.MatrixStruc(dim * mesh.nP)
    s.mesh_pattern(dim, mesh.F)
    s.pack()
    ia, ja = s.getia(), s.getja()
    N = len(ia) - 1
    rng = np.random.default_rng(5)
    a = rng.uniform(-1, 1, len(ja))
    rows = np.repeat(np.arange(N), np.diff(ia))
    d = np.nonzero(ja == rows)[0]
    a[d] = np.add.reduceat(np.abs(a), ia[:-1]) * 0.5 + 1.0
    ref = None
    for mode in modes:
        os.environ["MMX_FACTOR_GRAN"] = "1" if mode.endswith("-gran") else "0"
        mode0 = mode.split("-")[0]
        if mode0 == "chain":
            os.environ.pop("MMX_FACTOR", None)
        else:
            os.environ["MMX_FACTOR"] = mode0
        A = la.MatrixIter(s)
        A.a[:] = a
        A.b[:] = np.ones(N)
        A.sfac(la.ParamIter.mesh())
        A.factor()
        A.set_timing(True)
        A.reset_stats()
        for _ in range(3):
            A.factor()
        st = A.stats()
        af = A.get_factor()[2]
        same = None if ref is None else bool(np.array_equal(af.view(np.int64), ref.view(np.int64)))
        if ref is None:
            ref = af
        print(json.dumps({"dim": dim, "rows": N, "mode": mode, "factor_mode": st["factor_mode"],
                          "factor_ms": round(st["t_factor_ms"] / max(st["n_factor_timed"], 1), 3),
                          "bitwise_vs_first": same}), flush=True)
        A.close()
