"""Partitioned regrid (MonType 7 rebuilt every step) at C4 (3D SquareGrid n = 63, 512,191 vertices)
and C5 (n = 136, 5,086,809 vertices): per rank, the grid rows rebuilt, the candidate vertices of
the nearest-vertex fill and the bytes received per rebuild -- the near-box exchange of round 4
(regridNear) against the round-3 all-gather of every owned vertex -- N = 2/4/8 ranks on the
loopback communicator (one GPU, one engine per thread), 2 steps x 3 ADMM iterations; positions
checked equal between the two modes.  Prints one JSON line per (workload, N, mode).
Usage: python profiles/r04/regrid_partition.py [c4|c5|both]"""
import hashlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mm-admm_amd", "python"))
import mmadmm_amd as mx  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
for wl, n in (("c4", 63), ("c5", 136)):
    if which not in (wl, "both"):
        continue
    mesh = mx.MeshData.rect(3, n)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(3, 7), rho=2000.0, tau=0.5, device=0)
    for N in (2, 4, 8):
        hashes = {}
        for mode in ("near", "all"):
            if mode == "all":
                os.environ["MMX_REGRID_GATHER"] = "all"
            else:
                os.environ.pop("MMX_REGRID_GATHER", None)
            t0 = time.perf_counter()
            comm = mx.Comm.loopback(N)
            eng = []
            for r in range(N):
                eng.append(mx.Engine(M, 0.025, rank=r, nranks=N, comm=comm))
                print(f"{wl} N={N} {mode}: rank {r} set up", file=sys.stderr, flush=True)
            setup = time.perf_counter() - t0
            for e in eng:
                e.set_regrid(True)

            def run(e):
                for _ in range(2):
                    e.step(3, -1.0)
            th = [threading.Thread(target=run, args=(e,)) for e in eng]
            t0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            el = time.perf_counter() - t0
            st = [e.stats() for e in eng]
            h = hashlib.sha1()
            for e in eng:
                h.update(e.get("x").tobytes())
            hashes[mode] = h.hexdigest()[:16]
            print(json.dumps({"workload": wl, "n": n, "vertices": mesh.nP, "ranks": N, "mode": mode,
                              "grid_rows_per_rank": [s["regrid_rows"] for s in st],
                              "candidates_per_rank": [s["regrid_cand"] for s in st],
                              "bytes_received_per_rank": [s["regrid_gather_bytes"] for s in st],
                              "fallbacks": [s["regrid_fallbacks"] for s in st], "setup_s": round(setup, 1),
                              "two_steps_s_loopback": round(el, 2), "xhash": hashes[mode]}), flush=True)
            for e in eng:
                e.close()
            comm.close()
        print(json.dumps({"workload": wl, "ranks": N, "positions_equal": hashes["near"] == hashes["all"]}), flush=True)
