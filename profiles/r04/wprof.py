"""Phase probe of the 3D steady prox (build: profiles/r04/variants.sh wprof "-DMMX_WAVE_PROF"):
C4 (MonType 6), 3 steps, then the per-block shader-clock stamps of the last steady launch
(mmx_wprof_dump) -> median and mean phase durations over all blocks.  Usage (on the GPU box):
MMADMM_LIB=dev/lib_wprof/libmmadmm.so python profiles/r04/wprof.py [c4|c5]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))
import mmadmm_amd as mx  # noqa: E402

work = sys.argv[1] if len(sys.argv) > 1 else "c4"
n = 63 if work == "c4" else 118
m = mx.MeshData.rect(3, n)
M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5)
E = mx.Engine(M, 0.025)
for _ in range(3):
    E.step(10, -1.0)
E.set_timing(True)
E.reset_stats()
E.step(10, -1.0)
E.sync()
st = E.stats()
lib = ctypes.CDLL(os.environ["MMADMM_LIB"])
lib.mmx_wprof_dump.argtypes = [ctypes.c_char_p]
path = os.path.join(ROOT, "gpurun_out", f"wprof_{work}.bin")
os.makedirs(os.path.dirname(path), exist_ok=True)
nb = lib.mmx_wprof_dump(path.encode())
t = np.fromfile(path, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
ok = (t[:, :7] > 0).all(axis=1)
t = t[ok]
names = ["entry (inputs, cached gradient)", "pass 1 (p = -B G)", "blockGrad", "pass 2 (By, yBy, yB)",
         "pass 3 (update)", "write-back + partials"]
out = {"work": work, "blocks": int(nb), "blocks_stamped": int(ok.sum()),
       "prox_ms": round(st["t_prox_ms"] / st["n_prox"], 4)}
for i, nm in enumerate(names):
    d = t[:, i + 1] - t[:, i]
    out[nm] = {"median": int(np.median(d)), "mean": int(d.mean()), "p90": int(np.percentile(d, 90))}
life = t[:, 6] - t[:, 0]
out["lifetime"] = {"median": int(np.median(life)), "mean": int(life.mean())}
span = (t[:, 6].max() - t[:, 0].min())
out["launch_span_clocks"] = int(span)
print(json.dumps(out, indent=1), flush=True)
