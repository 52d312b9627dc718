#!/usr/bin/env python3
"""bench.py -- ADMM iterations/s of the MM-ADMM integrator on MI355X (BASELINE.json metric).

Workload (C3): 2D circular mesh with 1,000,519 nodes / 1,997,574 triangles
(hexagonal disc N=577, radius 0.5, centre (0.5, 0.5), rim FIXED), monitor MEx1 (static
isotropic bump), dt 0.055, tau 0.5, rho 50 (Experiments/InputFiles/Monitor2320.json family).
A "step" is one MeshIntegrator::step with exactly AdmmIter = 10 ADMM iterations (the early exit
disabled, SURVEY §8d protocol); value = ADMM iterations per second over the timed steps.  The
first warm-up step (finite-difference Hessians) is reported separately.

  python bench.py [--gpus N] [--steps K] [--warmup W]
For N > 1 launch with torch.distributed.run: each rank runs its own element-partitioned share
(weak scaling).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--admm-iter", type=int, default=10)
    ap.add_argument("--disc-n", type=int, default=577)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def pmc_traffic(kernel_prefix):
    """Per-launch HBM bytes of a kernel from the committed rocprofv3 PMC summary, or None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_prefix, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(mesh, admm_iter, threads):
    """Reference-equivalent CPU path (the oracle: CPU restatement of the reference, OpenMP prox,
    serial consensus algebra, -O3 -msse2) on the same mesh; bounded sample: set-up and the
    FD-Hessian step untimed, then one timed step of admm_iter iterations."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py

    om = oracle_py.Mesh(2, mesh.Xp, mesh.F, mesh.mask)
    O = oracle_py.Integrator(om, 1, 0.055, 0.5, 50.0, nthreads=threads)
    O.step(admm_iter, -1.0)
    t0 = time.perf_counter()
    O.step(admm_iter, -1.0)
    dt = time.perf_counter() - t0
    return {"value": round(admm_iter / dt, 3), "unit": "ADMM it/s", "cores": threads, "kind": "port",
            "sample": f"C3 mesh, 1 timed step of {admm_iter} ADMM iterations after set-up and the "
                      f"FD-Hessian step (oracle/oracle.cpp, g++ -O3 -msse2 -fopenmp, {threads} threads)"}


def main():
    args = parse()
    import torch  # first, so libmmadmm binds to the same HIP runtime
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import mmadmm_amd as mx

    mesh = mx.MeshData.hexdisc(args.disc_n, 0.5, 0.5, 0.5)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5, device=local)
    t_setup = time.perf_counter()
    eng = mx.Engine(M, 0.055)
    t_setup = time.perf_counter() - t_setup

    first_ms = None
    for w in range(max(args.warmup, 1)):
        t0 = time.perf_counter()
        eng.step(args.admm_iter, -1.0)
        if w == 0:
            first_ms = (time.perf_counter() - t0) * 1e3
    eng.set_timing(True)
    eng.reset_stats()

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step(args.admm_iter, -1.0)
    eng.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    st = eng.stats()
    iters = args.steps * args.admm_iter * world
    prox_ms = st["t_prox_ms"] / max(st["n_prox"], 1)
    xup_ms = st["t_xupdate_ms"] / max(st["n_xupdate"], 1)
    prox_gbs = st["prox_bytes"] / (prox_ms * 1e-3) / 1e9
    xup_gbs = st["xupdate_bytes"] / (xup_ms * 1e-3) / 1e9
    traffic = pmc_traffic("k_prox")
    result = {
        "metric": "ADMM iterations/sec on 1M-node 2D mesh; achieved HBM GB/s in SpMV",
        "value": round(iters / elapsed, 3),
        "unit": "ADMM it/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "C3: 2D circular mesh (hexagonal disc N=%d), %d nodes, %d triangles, MEx1 "
                               "monitor, dt 0.055 tau 0.5 rho 50, %d ADMM iterations per step"
                               % (args.disc_n, mesh.nP, mesh.nF, args.admm_iter),
                   "nodes_per_gpu": mesh.nP, "simplices_per_gpu": mesh.nF, "admm_iter": args.admm_iter,
                   "parallelism": "replicas" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": "k_prox_lds<2>",
                     "achieved": round(prox_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(prox_gbs / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "bytes_per_launch": st["prox_bytes"],
                     "avg_launch_ms": round(prox_ms, 4)},
        "kernels": {"k_prox_ms": round(prox_ms, 4), "k_xupdate_ms": round(xup_ms, 4),
                    "k_xupdate_GBs": round(xup_gbs, 1), "bfgs_iters_per_prox":
                        round(st["bfgs_iters"] / max(st["admm_iters"], 1) / mesh.nF, 4)},
        "first_step_ms": round(first_ms, 2),
        "setup_s": round(t_setup, 2),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count(), 16)
        result["cpu_baseline"] = cpu_baseline(mesh, args.admm_iter, threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
