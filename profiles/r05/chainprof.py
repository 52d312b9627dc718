import os, sys, ctypes
os.environ.setdefault("MMX_CHAIN_PROF", "2")
sys.path.insert(0, "mm-admm_amd/python")
import numpy as np
import mmadmm_amd as mx, lasolver_amd as la
mesh = mx.MeshData.rect(2, 707)
s = la.MatrixStruc(2 * mesh.nP); s.mesh_pattern(2, mesh.F); s.pack()
ia, ja = s.getia(), s.getja(); n = len(ia) - 1
rng = np.random.default_rng(20221015)
a = rng.uniform(-1.0, 1.0, len(ja)); x = rng.uniform(-1.0, 1.0, n)
A = la.MatrixIter(s)
rows = np.repeat(np.arange(n), np.diff(ia)); d = np.nonzero(ja == rows)[0]
a2 = a.copy(); a2[d] = np.add.reduceat(np.abs(a2), ia[:-1]) * 0.5 + 1.0
b = rng.uniform(-1.0, 1.0, n)
A.a[:] = a2; A.b[:] = b
p = la.ParamIter.mesh(); A.sfac(p); A.set_timing(True)
for rep in range(3):
    A.reset_stats(); xs = np.zeros(n); nitr = A.solve(p, xs); st = A.stats()
    print("nitr", nitr, "solve_ms", st["t_solve_ms"], "sweep_ms", st["t_sweep_ms"] / max(st["n_sweep_timed"], 1), "n_sweep", st["n_sweep_timed"])
L = la.lib()
out = (ctypes.c_ulonglong * 1024)()
L.mmx_matrix_chain_prof.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
rc = L.mmx_matrix_chain_prof(A.h, out, 0)
print("rc", rc)
for k, base in (("fwd", 0), ("bwd", 512)):
    c = [out[base + i] for i in range(16)]
    it = max(c[3], 1)
    print(k, "loader flush %d slot %d inflight %d importer %d" % (c[4], c[5], c[6], c[7]))
    print(k, "bands", c[8], "iters", c[3], "compute cyc/iter %.0f" % (c[0] / it), "stage %.0f" % (c[1] / it), "import %.0f" % (c[2] / it),
          "fine: to chain end %.0f, to prog %.0f, to next %.0f" % (c[9] / it, c[10] / it, c[11] / it))
    for slot in range(64):
        q = [out[base + 16 + 4 * slot + j] for j in range(4)]
        if q[3]:
            print("  band slot", slot, "cyc/it %.0f" % (q[0] / q[3]), "stage %.0f" % (q[1] / q[3]), "imp %.0f" % (q[2] / q[3]), "T", q[3])
