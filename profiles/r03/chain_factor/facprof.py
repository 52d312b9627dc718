"""Chain-factor profile at n = 707 (MMX_FACTOR=chain, MMX_CHAIN_PROF=1): compute / stage-wait /
import-wait cycles per iteration and importer cycles, from the counters at prof[480..485]."""
import ctypes, os, sys
os.environ["MMX_FACTOR"] = "chain"
os.environ.setdefault("MMX_CHAIN_PROF", "1")
sys.path.insert(0, "mm-admm_amd/python")
import numpy as np
import mmadmm_amd as mx, lasolver_amd as la
mesh = mx.MeshData.rect(2, 707)
s = la.MatrixStruc(2 * mesh.nP); s.mesh_pattern(2, mesh.F); s.pack()
ia, ja = s.getia(), s.getja(); n = len(ia) - 1
rng = np.random.default_rng(20221015)
a = rng.uniform(-1.0, 1.0, len(ja))
rows = np.repeat(np.arange(n), np.diff(ia)); d = np.nonzero(ja == rows)[0]
a[d] = np.add.reduceat(np.abs(a), ia[:-1]) * 0.5 + 1.0
A = la.MatrixIter(s); A.a[:] = a
p = la.ParamIter.mesh(); A.sfac(p); A.set_timing(True)
L = la.lib()
L.mmx_matrix_chain_prof.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
out = (ctypes.c_ulonglong * 1024)()
for rep in range(3):
    L.mmx_matrix_chain_prof(A.h, out, 1)
    A.reset_stats(); A.factor(); st = A.stats()
    L.mmx_matrix_chain_prof(A.h, out, 0)
    c = [out[480 + i] for i in range(6)]
    it = max(c[3], 1)
    print("factor_ms %.2f mode %d bands %d iters %d: per iteration compute %.0f stage-wait %.0f import-wait %.0f; importer %.0f per band"
          % (st["t_factor_ms"], st["factor_mode"], c[4], c[3], c[0] / it, c[1] / it, c[2] / it, c[5] / max(c[4], 1)))
for b in range(16):
    q = [out[480 + 320 + 4 * b + j] for j in range(4)]
    if q[3]:
        print("  band %d T %d cyc/it %.0f stage %.0f import %.0f" % (b, q[3], q[0] / q[3], q[1] / q[3], q[2] / q[3]))
