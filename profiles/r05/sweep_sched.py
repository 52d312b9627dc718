"""CG-STAB solve / sweep times at n = 2,002,226 (the bench's n = 707 Jacobian, diagonally shifted)
under the schedule settings in the environment (MMX_CHAIN_ALIGN, MMX_CHAIN_LAT, ...): one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mm-admm_amd", "python"))
import numpy as np
import mmadmm_amd as mx
import lasolver_amd as la

mesh = mx.MeshData.rect(2, 707)
s = la.MatrixStruc(2 * mesh.nP)
s.mesh_pattern(2, mesh.F)
s.pack()
ia, ja = s.getia(), s.getja()
n = len(ia) - 1
rng = np.random.default_rng(20221015)
a = rng.uniform(-1.0, 1.0, len(ja))
x = rng.uniform(-1.0, 1.0, n)
rows = np.repeat(np.arange(n), np.diff(ia))
d = np.nonzero(ja == rows)[0]
a2 = a.copy()
a2[d] = np.add.reduceat(np.abs(a2), ia[:-1]) * 0.5 + 1.0
b = rng.uniform(-1.0, 1.0, n)
A = la.MatrixIter(s)
A.a[:] = a2
A.b[:] = b
p = la.ParamIter.mesh()
A.sfac(p)
A.set_timing(True)
res = []
ref = None
for rep in range(3):
    A.reset_stats()
    xs = np.zeros(n)
    nitr = A.solve(p, xs)
    st = A.stats()
    if ref is None:
        ref = xs.copy()
    res.append({"solve_ms": round(st["t_solve_ms"], 2), "sweep_ms": round(st["t_sweep_ms"] / max(st["n_sweep_timed"], 1), 3),
                "factor_ms": round(st["t_factor_ms"], 2), "nitr": nitr, "same_x": bool(np.array_equal(xs, ref))})
env = {k: v for k, v in os.environ.items() if k.startswith("MMX_")}
print(json.dumps({"env": env, "runs": res}))
