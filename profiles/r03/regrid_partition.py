"""Partitioned regrid at C4 (3D SquareGrid n = 63, 512,191 vertices, MonType 7 rebuilt every step):
grid rows each rank rebuilds and vertex bytes each rank receives per rebuild, N = 1/2/4/8 ranks on
the loopback communicator (one GPU, one engine per thread).  Prints one JSON line per N.
Usage: python profiles/r03/regrid_partition.py [n]"""
import json
import os
import sys
import threading

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mm-admm_amd", "python"))
import mmadmm_amd as mx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 63
mesh = mx.MeshData.rect(3, n)
M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(3, 7), rho=2000.0, tau=0.5, device=0)
for N in (1, 2, 4, 8):
    comm = mx.Comm.loopback(N) if N > 1 else None
    eng = [mx.Engine(M, 0.025, rank=r, nranks=N, comm=comm) if N > 1 else mx.Engine(M, 0.025) for r in range(N)]
    for e in eng:
        e.set_regrid(True)
    th = [threading.Thread(target=e.step, args=(1, -1.0)) for e in eng]
    for t in th:
        t.start()
    for t in th:
        t.join()
    total = len(eng[0].get("grid")) // 9
    rows = [e.stats()["regrid_rows"] for e in eng]
    gb = [e.stats()["regrid_gather_bytes"] for e in eng]
    print(json.dumps({"workload": "c4", "n": n, "vertices": mesh.nP, "tets": mesh.nF, "ranks": N, "grid_rows_total": total,
                      "grid_rows_per_rank": rows, "max_rows_frac": round(max(rows) / total, 4),
                      "gathered_bytes_per_rank": gb}), flush=True)
    for e in eng:
        e.close()
    if comm:
        comm.close()
