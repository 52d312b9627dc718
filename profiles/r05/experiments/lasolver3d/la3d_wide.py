"""3D LASolver at C4 (SquareGrid n=63 Jacobian pattern, 1,536,573 rows): sweep times with the
backward triangle's rows (up to 44 entries) in one 48-entry stage position (default) against two
32-entry segments (MMX_CHAIN_E48=0) and the level schedule; every ILU solve must be bit-identical."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "..", "mm-admm_amd", "python"))
import numpy as np
import lasolver_amd as la
import mmadmm_amd as mx
n = int(sys.argv[1]) if len(sys.argv) > 1 else 63
mesh = mx.MeshData.rect(3, n)
s = la.MatrixStruc(3 * mesh.nP)
s.mesh_pattern(3, mesh.F)
s.pack()
ia, ja = s.getia(), s.getja()
N = len(ia) - 1
rng = np.random.default_rng(5)
a = rng.uniform(-1, 1, len(ja))
rows = np.repeat(np.arange(N), np.diff(ia))
d = np.nonzero(ja == rows)[0]
a[d] = np.add.reduceat(np.abs(a), ia[:-1]) * 0.5 + 1.0
b = rng.uniform(-1, 1, N)
ref = None
for mode in sys.argv[2:] if len(sys.argv) > 2 else ["wide", "seg", "level", "wide"]:
    os.environ["MMX_SWEEP"] = "level" if mode == "level" else "auto"
    os.environ["MMX_CHAIN_E48"] = "0" if mode == "seg" else "1"
    A = la.MatrixIter(s)
    A.a[:] = a
    A.b[:] = b
    p = la.ParamIter.mesh()
    t0 = time.perf_counter()
    A.sfac(p)
    tsf = time.perf_counter() - t0
    A.factor()
    A.set_timing(True)
    A.reset_stats()
    for _ in range(5):
        y = A.ilu_solve(b)
    st = A.stats()
    x = np.zeros(N)
    A.reset_stats()
    it = A.solve(p, x)
    st2 = A.stats()
    same = None if ref is None else bool(np.array_equal(y.view(np.int64), ref[0].view(np.int64)) and
                                         np.array_equal(x.view(np.int64), ref[1].view(np.int64)))
    if ref is None:
        ref = (y, x)
    print(json.dumps({"mode": mode, "rows": N, "nnz": len(ja), "sfac_s": round(tsf, 2), "sweep_mode": st["sweep_mode"],
                      "sweep_ms": round(st["t_sweep_ms"] / max(st["n_sweep_timed"], 1), 3),
                      "n_sweeps": st["n_sweep_timed"], "solve_ms": round(st2["t_solve_ms"], 3), "cg_iters": it,
                      "bitwise_vs_first": same}), flush=True)
    A.close()
