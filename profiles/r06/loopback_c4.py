"""C4 step on one rank against the same C4 cut in two (RCB element partition, loopback
communicator: two engines on one GPU driven from two threads), VERDICT r5 #3's check of what a
partitioned rank costs per simplex.  Prints one JSON line per configuration.

The two ranks share the card, so their kernels run concurrently; the comparison is whole-step wall
time (both ranks' steps) minus the exchange time the engines record, against the one-rank step.
Usage: python profiles/r06/loopback_c4.py [steps]
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))
import mmadmm_amd as mx  # noqa: E402

ITERS = 10


def run_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if errs:
        raise errs[0]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    mesh = mx.MeshData.rect(3, 63)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5)

    E = mx.Engine(M, 0.025)
    E.step(ITERS, -1.0)
    E.step(ITERS, -1.0)
    E.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        E.step(ITERS, -1.0)
    E.sync()
    t1 = (time.perf_counter() - t0) / steps
    E.close()
    print(json.dumps({"config": "C4 one rank", "ms_per_step": round(t1 * 1e3, 3), "nF": mesh.nF}), flush=True)

    for overlap in ("1", "0"):
        os.environ["MMX_OVERLAP"] = overlap
        comm = mx.Comm.loopback(2)
        parts = [mx.Engine(M, 0.025, rank=r, nranks=2, comm=comm) for r in range(2)]

        def go(k):
            return [lambda e=e: [e.step(ITERS, -1.0) for _ in range(k)] for e in parts]

        run_threads(go(2))
        for e in parts:
            e.sync()
            e.set_timing(True)
            e.reset_stats()
        t0 = time.perf_counter()
        run_threads(go(steps))
        for e in parts:
            e.sync()
        t2 = (time.perf_counter() - t0) / steps
        st = [e.stats() for e in parts]
        ex = max(s["t_exchange_ms"] for s in st) / steps
        nloc = [e.nF for e in parts]
        rec = {"config": "C4 two ranks, loopback, one GPU", "overlap": int(overlap),
               "ms_per_step": round(t2 * 1e3, 3), "exchange_ms_per_step_max_rank": round(ex, 3),
               "ms_per_step_minus_exchange": round(t2 * 1e3 - ex, 3),
               "ratio_to_one_rank": round((t2 * 1e3 - ex) / (t1 * 1e3), 4), "nF_per_rank": nloc,
               "interior_nodes": [s["interior_nodes"] for s in st],
               "halo_send_bytes_per_step": [round(s["halo_send_bytes"] / steps) for s in st],
               "prox_ms": [round(s["t_prox_ms"] / max(s["n_prox"], 1), 4) for s in st],
               "xupdate_ms": [round(s["t_xupdate_ms"] / max(s["n_xupdate"], 1), 4) for s in st]}
        print(json.dumps(rec), flush=True)
        for e in parts:
            e.close()


if __name__ == "__main__":
    main()
