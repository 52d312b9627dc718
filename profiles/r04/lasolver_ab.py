"""Same-box comparison of library builds on bench.py's n = 2,002,226 ILU(0)-CG-STAB solve (SquareGrid
n = 707 Jacobian pattern, values as bench.py spmv_bench): for each library (MMADMM_LIB) in a fresh
process, the solve / factor / sweep times of 3 solves after a warm-up one, and a hash of the
solution (builds must be bit-identical).  Usage: python lasolver_ab.py <lib>[+VAR=VALUE...] [...]"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one():
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))
    import lasolver_amd as la
    import mmadmm_amd as mx
    mesh = mx.MeshData.rect(2, 707)
    s = la.MatrixStruc(2 * mesh.nP)
    s.mesh_pattern(2, mesh.F)
    s.pack()
    ia, ja = s.getia(), s.getja()
    n = len(ia) - 1
    rng = np.random.default_rng(20221015)
    a = rng.uniform(-1.0, 1.0, len(ja))
    rng.uniform(-1.0, 1.0, n)
    rows = np.repeat(np.arange(n), np.diff(ia))
    d = np.nonzero(ja == rows)[0]
    a2 = a.copy()
    a2[d] = np.add.reduceat(np.abs(a2), ia[:-1]) * 0.5 + 1.0
    b = rng.uniform(-1.0, 1.0, n)
    A = la.MatrixIter(s)
    A.set_timing(True)
    A.a[:] = a2
    A.b[:] = b
    p = la.ParamIter.mesh()
    A.sfac(p)
    xs = np.zeros(n)
    A.solve(p, xs)
    res = []
    for _ in range(3):
        A.reset_stats()
        xs = np.zeros(n)
        nitr = A.solve(p, xs)
        st = A.stats()
        res.append((st["t_solve_ms"], st["t_factor_ms"], st["t_sweep_ms"] / max(st["n_sweep_timed"], 1)))
    A.close()
    best = min(res)
    return {"lib": os.environ.get("MMADMM_LIB", "default"), "nitr": nitr, "solve_ms": round(best[0], 2),
            "factor_ms": round(best[1], 2), "sweep_ms": round(best[2], 3),
            "xhash": hashlib.sha1(xs.tobytes()).hexdigest()[:16]}


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        print(json.dumps(one()), flush=True)
        sys.exit(0)
    for rep in range(2):
        for spec in sys.argv[1:]:
            lib, *sets = spec.split("+")
            env = dict(os.environ)
            env.update(kv.split("=", 1) for kv in sets)
            if lib != "default":
                env["MMADMM_LIB"] = os.path.abspath(lib)
            r = subprocess.run([sys.executable, __file__, "--one"], env=env, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(json.dumps({"spec": spec, "error": r.stderr[-2000:]}), flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            d["round"], d["spec"] = rep, spec
            print(json.dumps(d), flush=True)
