"""n = 2,002,226 (SquareGrid n=707 Jacobian pattern) ILU(0)-CG-STAB: sweep and solve times with the
loaders moving only a band's used entry slots (MMX_CHAIN_TRIM=1, default) or the whole stage (0),
alternating; the solutions must be bit-identical."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "..", "mm-admm_amd", "python"))
import numpy as np
import mmadmm_amd as mx, lasolver_amd as la
mesh = mx.MeshData.rect(2, 707)
s = la.MatrixStruc(2 * mesh.nP); s.mesh_pattern(2, mesh.F); s.pack()
ia, ja = s.getia(), s.getja(); n = len(ia) - 1
rng = np.random.default_rng(20221015)
a = rng.uniform(-1.0, 1.0, len(ja))
rows = np.repeat(np.arange(n), np.diff(ia)); d = np.nonzero(ja == rows)[0]
a[d] = np.add.reduceat(np.abs(a), ia[:-1]) * 0.5 + 1.0
b = rng.uniform(-1.0, 1.0, n)
ref = None
for mode in sys.argv[1:] if len(sys.argv) > 1 else ["1", "0", "1", "0"]:
    os.environ["MMX_CHAIN_TRIM"] = mode
    A = la.MatrixIter(s)
    A.a[:] = a; A.b[:] = b
    p = la.ParamIter.mesh(); A.sfac(p); A.set_timing(True)
    xs = np.zeros(n); A.solve(p, xs)  # warm-up (factor)
    res = []
    for rep in range(3):
        A.reset_stats(); xs = np.zeros(n); nitr = A.solve(p, xs); st = A.stats()
        res.append((st["t_solve_ms"], st["t_sweep_ms"] / max(st["n_sweep_timed"], 1)))
    same = None if ref is None else bool(np.array_equal(xs.view(np.int64), ref.view(np.int64)))
    if ref is None:
        ref = xs.copy()
    print(json.dumps({"trim": mode, "nitr": nitr, "solve_ms": [round(r[0], 3) for r in res],
                      "sweep_ms": [round(r[1], 3) for r in res], "bitwise_vs_first": same}), flush=True)
    A.close()
