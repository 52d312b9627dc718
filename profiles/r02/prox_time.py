import os, sys, time, json
sys.path.insert(0, '/root/repo/mm-admm_amd/python')
import mmadmm_amd as mx
n = int(os.environ.get("C4N", "63"))
if os.environ.get("WL") == "c3":
    mesh = mx.MeshData.hexdisc(577, 0.5, 0.5, 0.5)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5)
    E = mx.Engine(M, 0.055)
else:
    mesh = mx.MeshData.rect(3, n)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5)
    E = mx.Engine(M, 0.025)
E.step(10, -1.0); E.step(10, -1.0); E.sync()
E.set_timing(True); E.reset_stats(); E.sync()
t0 = time.perf_counter()
for _ in range(3): E.step(10, -1.0)
E.sync(); el = time.perf_counter() - t0
st = E.stats()
X = E.get("x")
import hashlib, numpy as np
h = hashlib.sha1(np.ascontiguousarray(X).tobytes()).hexdigest()[:12] if X is not None else '-'
print(json.dumps({"wl": os.environ.get("WL", "c4"), "lib": os.environ.get("MMADMM_LIB", "default"), "prox_ms": round(st["t_prox_ms"] / max(st["n_prox"], 1), 4), "xup_ms": round(st["t_xupdate_ms"] / max(st["n_xupdate"], 1), 4),
                  "it_s": round(30 / el, 2), "hash": h}))
