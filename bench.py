#!/usr/bin/env python3
"""bench.py -- ADMM iterations/s of the MM-ADMM integrator on MI355X (BASELINE.json metric).

Workload (C3): 2D circular mesh with 1,000,519 nodes / 1,997,574 triangles
(hexagonal disc N=577, radius 0.5, centre (0.5, 0.5), rim FIXED), monitor MEx1 (static
isotropic bump), dt 0.055, tau 0.5, rho 50 (Experiments/InputFiles/Monitor2320.json family).
A "step" is one MeshIntegrator::step with exactly AdmmIter = 10 ADMM iterations (the early exit
disabled, SURVEY §8d protocol); value = ADMM iterations per second over the timed steps.  The
first warm-up step (finite-difference Hessians) is reported separately.

  python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 runs N ranks, one per GPU: under a launcher (torch.distributed.run, WORLD_SIZE = N) directly,
otherwise bench.py re-launches itself under torch.distributed.run before anything touches the GPU
(fewer than N visible GPUs, or WORLD_SIZE != N: exit status 2, no line).  The global mesh grows with N (hexagonal disc of
N_disc = 577*sqrt(N), ~N million nodes) and is element-partitioned across the ranks, one per GPU,
exchanging interface-slot values with their neighbouring ranks over RCCL send/recv (recursive
coordinate bisection of the simplex centroids; weak scaling).
value = ADMM iterations per second x (global nodes / 1,000,519): whole-job throughput in units of
C3-sized meshes.

The second half of the metric, achieved HBM GB/s in SpMV, is measured on the backward-Euler
Jacobian CSR of the 2D SquareGrid n=707 mesh (n = 2,002,226 rows, nnz = 28,008,516, SURVEY §8d
microbenchmark ii) with the LASolver replacement's matmult, and reported under "spmv" together
with one ILU(0)-preconditioned CG-STAB solve of that matrix.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, spec)
# CPU-baseline legs, run after all GPU timing so host threads (OpenMP workers still spinning after a
# parallel region) cannot delay the launches of a measured GPU section
DEFERRED = []


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE, else 1); without WORLD_SIZE, N > 1 re-launches "
                         "this script under torch.distributed.run with N processes")
    ap.add_argument("--comm", choices=("rccl", "host"), default="rccl",
                    help="N > 1: rccl (one GPU per rank, RCCL send/recv over xGMI; the measurement) or host (the halo "
                         "exchange through pinned host buffers over a gloo group, ranks may share a GPU: a rehearsal of "
                         "the N-rank path on a box with fewer GPUs, not a measurement)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--admm-iter", type=int, default=10)
    ap.add_argument("--disc-n", type=int, default=577)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-spmv", action="store_true")
    ap.add_argument("--no-be", action="store_true", help="skip the backward-Euler (method 2) section")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 (2D unit square, 99,905 nodes) section")
    ap.add_argument("--no-3d", action="store_true", help="skip the 3D (BASELINE config 4) section")
    ap.add_argument("--no-bfgs", action="store_true", help="skip the BFGS-heavy (rho = 1) 2D section")
    ap.add_argument("--c5", action="store_true",
                    help="add BASELINE config 5 on one GPU: 3D 5.09M-node mesh, time-varying monitor")
    ap.add_argument("--budget-s", type=float, default=1500.0,
                    help="N > 1: wall-clock budget of every rank (a watchdog ends a rank that exceeds it with exit "
                         "status 124, naming its phase) and of the re-launched job (the launcher's process group is "
                         "killed after the budget + 60 s, naming the ranks that never finished set-up)")
    ap.add_argument("--comm-timeout", type=float, default=300.0,
                    help="N > 1: deadline (s) of the RCCL communicator's creation and of every wait of a "
                         "partitioned step (MMADMM_ERR_RCCL after ncclCommAbort, never a hang)")
    ap.add_argument("--rendezvous-only", action="store_true",
                    help="N > 1: launch the ranks, rendezvous over gloo, report the phases and exit (no GPU; a CI "
                         "check of the launch path and its failure handling)")
    ap.add_argument("--workload", choices=("c3", "c4", "c5"), default="c3",
                    help="c3: 2D 1M-node disc (the headline); c4: 3D 512k-node cube per GPU, anisotropic monitor "
                         "(weak scaling); c5: 3D 5.09M-node cube, time-varying monitor rebuilt every step, fixed "
                         "size (strong scaling)")
    return ap.parse_args()


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


T_START = time.time()
_PHASE = {"name": "start"}


def phase(name):
    """One stderr progress line per rank per phase, also appended to $MMX_BENCH_PROGRESS/rank<r> when
    bench.py re-launched itself (so that the parent can name a rank that never got past a phase)."""
    rank = os.environ.get("RANK", "0")
    _PHASE["name"] = name
    log("rank %s/%s: phase %s (+%.1f s)" % (rank, os.environ.get("WORLD_SIZE", "1"), name, time.time() - T_START))
    d = os.environ.get("MMX_BENCH_PROGRESS")
    if d:
        try:
            with open(os.path.join(d, "rank%s" % rank), "a") as f:
                f.write(name + "\n")
        except OSError:
            pass


def start_watchdog(budget_s, rank):
    """A rank that is still running after budget_s seconds (a peer that never joined, a collective
    that never completed) prints its phase and exits with status 124 -- the launcher then ends the
    other ranks.  os._exit: no interpreter shutdown, which could itself wait on the stuck call."""
    import threading

    def run():
        if threading.Event().wait(budget_s):
            return
        log("rank %d: wall-clock budget of %.0f s exceeded in phase '%s' -- a peer rank missing or stuck? "
            "exiting with status 124" % (rank, budget_s, _PHASE["name"]))
        os._exit(124)

    threading.Thread(target=run, name="bench-watchdog", daemon=True).start()


def rank_phases(progress_dir, n):
    """the phases each rank reported (rank -> list)"""
    out = {}
    for r in range(n):
        try:
            with open(os.path.join(progress_dir, "rank%d" % r)) as f:
                out[r] = [ln.strip() for ln in f if ln.strip()]
        except OSError:
            out[r] = []
    return out


def report_ranks(progress_dir, n):
    """stderr: the ranks that never finished set-up, with their last phase; returns that list"""
    ph = rank_phases(progress_dir, n)
    missing = [r for r in range(n) if "setup" not in ph[r]]
    absent = [r for r in range(n) if "rendezvous" not in ph[r]]
    for r in range(n):
        log("rank %d: last phase %s" % (r, ph[r][-1] if ph[r] else "none (never started)"))
    if absent:
        log("ranks that never reached the rendezvous: %s" % ", ".join(str(r) for r in absent))
    if missing:
        log("ranks that printed no 'setup' line: %s" % ", ".join(str(r) for r in missing))
    return missing


def launch_plan(gpus, env, n_visible, share=False):
    """How a `bench.py --gpus N` invocation runs (the reference's one parallelism knob is its thread
    count, main.cpp:788-799 -> src/Mesh.cpp:436-438; here it is N ranks, one per GPU):
      ("run", world)  -- this process is one rank of `world` (WORLD_SIZE set by a launcher, or N = 1)
      ("spawn", N)    -- no launcher: re-launch under torch.distributed.run with N processes
      ("error", msg)  -- N and the launcher disagree, or fewer than N GPUs are visible
    n_visible: a callable giving the visible GPU count (only called when it matters); share: ranks may
    share a GPU (--comm host), so the count is not checked.  A --gpus N run never falls back to fewer
    ranks."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if gpus is not None and gpus != world:
            return ("error", "bench.py --gpus %d launched with WORLD_SIZE=%d" % (gpus, world))
        if world > 1 and not share and n_visible() < world:
            return ("error", "bench.py: WORLD_SIZE=%d but only %d GPU(s) visible" % (world, n_visible()))
        return ("run", world)
    n = 1 if gpus is None else gpus
    if n < 1:
        return ("error", "bench.py --gpus %d: need at least one GPU" % n)
    if n == 1:
        return ("run", 1)
    have = n if share else n_visible()
    if have < n:
        return ("error", "bench.py --gpus %d: only %d GPU(s) visible, device %d is missing" % (n, have, have))
    return ("spawn", n)


def parallelism_label(world, comm="rccl"):
    return ("single" if world == 1 else
            "element-partition x%d (RCB, RCCL halo send/recv of interface slots)" % world if comm == "rccl" else
            "element-partition x%d (RCB, halo exchange over a gloo host transport; rehearsal)" % world)


def visible_gpus():
    """GPU count from a child process, so this one never touches the GPU before it re-launches."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(n, budget_s=None):
    """N ranks under torch.distributed.run (127.0.0.1 rendezvous); this process only waits for them
    and exits with their status (a child process, not an exec).  With a budget the launcher runs in
    its own process group; past budget_s + 60 s the group is killed (SIGTERM, then SIGKILL) and the
    call returns 124.  On any failure the ranks' last phases are printed and the ranks that never
    finished set-up are named."""
    import shutil
    import signal
    import subprocess
    import tempfile
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    log("re-launching %d ranks:" % n, " ".join(cmd))
    if budget_s is None:
        return subprocess.run(cmd).returncode
    prog = tempfile.mkdtemp(prefix="mmx_bench_progress_")
    try:
        p = subprocess.Popen(cmd, env=dict(os.environ, MMX_BENCH_PROGRESS=prog), start_new_session=True)
        try:
            rc = p.wait(timeout=budget_s + 60.0)
        except subprocess.TimeoutExpired:
            log("the %d-rank job exceeded its budget of %.0f s (+60 s): killing its process group" % (n, budget_s))
            report_ranks(prog, n)
            for sig, grace in ((signal.SIGTERM, 15.0), (signal.SIGKILL, 15.0)):
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    break
                try:
                    p.wait(timeout=grace)
                    break
                except subprocess.TimeoutExpired:
                    continue
            return 124
        if rc != 0:
            log("the %d-rank job failed with status %d" % (n, rc))
            report_ranks(prog, n)
        return rc
    finally:
        shutil.rmtree(prog, ignore_errors=True)


def rendezvous_only(world, budget_s):
    """--rendezvous-only: the N-rank launch and its failure handling without a GPU -- each rank
    reports its phases, meets the others over gloo (bounded by the budget) and exits.
    MMX_BENCH_TEST_STALL_RANK=r makes rank r stall before the rendezvous (test hook)."""
    import datetime
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        start_watchdog(budget_s, rank)
    phase("start")
    stall = os.environ.get("MMX_BENCH_TEST_STALL_RANK")
    if stall is not None and int(stall) == rank:
        log("rank %d: stalling before the rendezvous (MMX_BENCH_TEST_STALL_RANK)" % rank)
        time.sleep(10 * budget_s + 600)
    import torch.distributed as dist
    phase("rendezvous")
    if world > 1:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(budget_s, 1.0)))
        dist.barrier()
    phase("setup")
    if world > 1:
        dist.destroy_process_group()
    phase("done")
    return 0


def spmv_bench(torch, la, mx, with_cpu):
    """matmult on the n=707 Jacobian (28.0 M nonzeros) + one ILU(0)-CG-STAB solve."""
    import numpy as np
    mesh = mx.MeshData.rect(2, 707)
    s = la.MatrixStruc(2 * mesh.nP)
    s.mesh_pattern(2, mesh.F)
    s.pack()
    ia, ja = s.getia(), s.getja()
    n = len(ia) - 1
    rng = np.random.default_rng(20221015)
    a = rng.uniform(-1.0, 1.0, len(ja))
    x = rng.uniform(-1.0, 1.0, n)
    A = la.MatrixIter(s)
    A.a[:] = a
    A.upload()
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    for _ in range(5):
        A.matmult_device(xd.data_ptr(), yd.data_ptr())
    A.set_timing(True)
    A.reset_stats()
    reps = 50
    for _ in range(reps):
        A.matmult_device(xd.data_ptr(), yd.data_ptr())
    st = A.stats()
    ms = st["t_spmv_ms"] / st["n_spmv_timed"]
    gbs = st["spmv_bytes"] / (ms * 1e-3) / 1e9
    out = {"matrix": "SquareGrid n=707 backward-Euler Jacobian pattern (src/Mesh.cpp:309-345), values U(-1,1)",
           "rows": n, "nnz": int(len(ja)), "bytes_per_spmv": st["spmv_bytes"], "avg_ms": round(ms, 5),
           "achieved_GBs": round(gbs, 1), "peak_GBs": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4),
           "kernel": "k_spmv2<0>", "reps": reps}
    tr, trr = pmc_traffic("k_spmv2<0>")
    out["traffic"], out["traffic_fetch_uncorrected"] = tr, trr
    # one timed solve after a warm-up one: diagonally dominant values, src/Mesh.cpp parameters
    rows = np.repeat(np.arange(n), np.diff(ia))
    d = np.nonzero(ja == rows)[0]
    a2 = a.copy()
    a2[d] = np.add.reduceat(np.abs(a2), ia[:-1]) * 0.5 + 1.0
    b = rng.uniform(-1.0, 1.0, n)
    A.a[:] = a2
    A.b[:] = b
    p = la.ParamIter.mesh()
    A.sfac(p)
    xs = np.zeros(n)
    A.solve(p, xs)  # untimed warm-up solve (first launches); every solve re-factors (values re-uploaded)
    A.reset_stats()
    xs = np.zeros(n)
    nitr = A.solve(p, xs)
    st = A.stats()
    out["cgstab"] = _solve_stats(st, nitr)
    A.close()
    # the same solve on the C4 cube's Jacobian pattern (3D SquareGrid n = 63, 1,536,573 rows; the
    # backward-Euler C4 line's solver), diagonally dominant values of the same form
    mesh3 = mx.MeshData.rect(3, 63)
    s3 = la.MatrixStruc(3 * mesh3.nP)
    s3.mesh_pattern(3, mesh3.F)
    s3.pack()
    ia3, ja3 = s3.getia(), s3.getja()
    n3 = len(ia3) - 1
    rng3 = np.random.default_rng(5)
    a3 = rng3.uniform(-1.0, 1.0, len(ja3))
    d3 = np.nonzero(ja3 == np.repeat(np.arange(n3), np.diff(ia3)))[0]
    a3[d3] = np.add.reduceat(np.abs(a3), ia3[:-1]) * 0.5 + 1.0
    b3 = rng3.uniform(-1.0, 1.0, n3)
    A3 = la.MatrixIter(s3)
    A3.a[:] = a3
    A3.b[:] = b3
    A3.sfac(p)
    A3.set_timing(True)
    xs3 = np.zeros(n3)
    A3.solve(p, xs3)
    A3.reset_stats()
    xs3 = np.zeros(n3)
    nitr3 = A3.solve(p, xs3)
    out["cgstab_c4"] = dict(_solve_stats(A3.stats(), nitr3), rows=n3, nnz=int(len(ja3)),
                            matrix="3D SquareGrid n=63 (C4) Jacobian pattern, diagonally dominant U(-1,1) values")
    A3.close()
    A = None
    def _cpu():
        import time as _t
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import lasolver_py as L
        t0 = _t.perf_counter()
        for _ in range(3):
            L.matmult(ia, ja, a, x)
        cms = (_t.perf_counter() - t0) / 3 * 1e3
        t0 = _t.perf_counter()
        _, cit, _ = L.solve(ia, ja, a2, b)
        csolve = (_t.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"matmult_ms": round(cms, 2), "solve_ms": round(csolve, 1), "nitr": cit, "cores": 1,
                               "kind": "port", "sample": "oracle/lasolver.cpp (bit-identical restatement of "
                               "lib/LASolver, itself pinned to the reference build): 3 matmults + 1 solve"}
        t0 = _t.perf_counter()
        _, cit3, _ = L.solve(ia3, ja3, a3, b3)
        c3 = (_t.perf_counter() - t0) * 1e3
        out["cgstab_c4"]["cpu_baseline"] = {"solve_ms": round(c3, 1), "nitr": cit3, "cores": 1, "kind": "port",
                                            "gpu_speedup": round(c3 / out["cgstab_c4"]["solve_ms"], 1),
                                            "sample": "oracle/lasolver.cpp, the same C4-pattern solve"}
    if with_cpu:  # CPU baselines run after every GPU measurement (main)
        DEFERRED.append(_cpu)
    return out


def _solve_stats(st, nitr):
    fk = {0: "k_ilu_factor_lds", 1: "k_chain_factor", 2: "k_ilu_factor_wave"}
    return {"nitr": nitr, "solve_ms": round(st["t_solve_ms"], 2), "factor_ms": round(st["t_factor_ms"], 2),
            "sweep_ms": round(st["t_sweep_ms"] / max(st["n_sweep_timed"], 1), 3),
            "sweep_kernel": ("k_chain_sweep (E=%d/%d fwd/bwd)" % (st["sweep_e"], st["sweep_e_bwd"])
                             if st["sweep_mode"] else "k_sweep"),
            "factor_kernel": fk.get(st["factor_mode"], "?"),
            "ms_per_iter": round((st["t_solve_ms"] - st["t_factor_ms"]) / max(nitr, 1), 2)}


def be_bench(mx, with_cpu, dim=2):
    """Method 2 (Mesh::backwardsEulerStep, src/Mesh.cpp:1263-1341) on the device.  dim 2: SquareGrid
    n = 707 (1,001,113 nodes, the SpMV matrix's mesh), MEx3, dt 0.025, tau 0.5, rho 100 (the
    Monitor220 family).  dim 3: the C4 cube (3D SquareGrid n = 63, 512,191 nodes, a 1,536,573-row
    Jacobian whose upper rows take the 48-entry chain-sweep stages), the C4 monitor (MonType 6), dt 0.025,
    tau 0.5.  First step (pattern, symbolic ILU, sweep schedules, FD Jacobian) and the steady steps
    after it are timed separately; the CPU leg runs the oracle on the same mesh."""
    if dim == 2:
        mesh = mx.MeshData.rect(2, 707)
        mon, rho, steps, csteps = 3, 100.0, 3, 2
        desc = "SquareGrid n=707 (%d nodes, %d triangles), MEx3, dt 0.025 tau 0.5 rho 100" % (mesh.nP, mesh.nF)
    else:
        mesh = mx.MeshData.rect(3, 63)
        mon, rho, steps, csteps = 6, 2000.0, 2, 1
        desc = ("C4: 3D SquareGrid n=63 (%d nodes, %d tetrahedra), MonType 6 (anisotropic shell), dt 0.025 "
                "tau 0.5" % (mesh.nP, mesh.nF))
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, mon), rho=rho, tau=0.5)
    E = mx.Engine(M, 0.025)
    t0 = time.perf_counter()
    E.backwards_euler_step(0.025)
    first = time.perf_counter() - t0
    E.reset_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        E.backwards_euler_step(0.025)
    dt = (time.perf_counter() - t0) / steps
    st = E.stats()
    out = {"workload": desc, "first_step_s": round(first, 3), "step_ms": round(dt * 1e3, 2), "steps": steps,
           "newton_per_step": st["newton_iters"] / steps, "cg_iters_per_step": st["cg_iters"] / steps,
           "solve_ms_per_step": round(st["t_solve_ms"] / steps, 2)}
    E.close()
    def _cpu():  # the oracle's restatement, one core, on the same mesh and parameters
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py
        om = oracle_py.Mesh(dim, mesh.Xp, mesh.F, mesh.mask)
        O = oracle_py.Integrator(om, mon, 0.025, 0.5, rho, nthreads=1)
        O.backwards_euler_step(0.025)
        t0 = time.perf_counter()
        for _ in range(csteps):
            O.backwards_euler_step(0.025)
        cdt = (time.perf_counter() - t0) / csteps
        out["cpu_baseline"] = {"step_ms": round(cdt * 1e3, 1), "nodes": int(om.nP), "cores": 1, "kind": "port",
                               "gpu_speedup": round(cdt * 1e3 / out["step_ms"], 1),
                               "sample": "oracle/oracle.cpp backwards_euler_step (FD Jacobian + LASolver "
                                         "restatement) on the same mesh, %d steady step(s) after the first" % csteps}
    if with_cpu:  # CPU baselines run after every GPU measurement (main)
        DEFERRED.append(_cpu)
    return out


def c2_bench(mx, with_cpu, threads, admm_iter, steps=20):
    """BASELINE config 2 / SURVEY C2 on one GPU: 2D SquareGrid n = 223 (99,905 nodes, 198,916
    triangles), MEx1 (static Gaussian bump), dt 0.055 tau 0.5 rho 50, admm_iter ADMM iterations per
    step with the early exit off; the CPU path on the same mesh beside it."""
    mesh = mx.MeshData.rect(2, 223)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5)
    E = mx.Engine(M, 0.055)
    t0 = time.perf_counter()
    E.step(admm_iter, -1.0)
    E.sync()
    first = time.perf_counter() - t0
    for _ in range(2):
        E.step(admm_iter, -1.0)
    E.set_timing(True)
    E.reset_stats()
    E.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        E.step(admm_iter, -1.0)
    E.sync()
    el = time.perf_counter() - t0
    st = E.stats()
    prox_ms = st["t_prox_ms"] / max(st["n_prox"], 1)
    prox_gbs = st["prox_bytes"] / (prox_ms * 1e-3) / 1e9
    out = {"workload": "C2: 2D SquareGrid n=223, %d nodes, %d triangles, MEx1, dt 0.055 tau 0.5 rho 50, %d ADMM "
                       "iterations per step" % (mesh.nP, mesh.nF, admm_iter),
           "value": round(steps * admm_iter / el, 3), "unit": "ADMM it/s", "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 3), "first_step_ms": round(first * 1e3, 1),
           "kernels": {"k_prox_ms": round(prox_ms, 4)},
           "roofline": {"bound": "hbm", "kernel": prox2d_name(), "achieved": round(prox_gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(prox_gbs / HBM_PEAK_GBS, 4),
                        "bytes_per_launch": st["prox_bytes"], "avg_launch_ms": round(prox_ms, 4)}}
    E.close()

    def _cpu():
        out["cpu_baseline"] = cpu_baseline(mesh, admm_iter, threads, label="C2", steps1=CPU_STEPS)
    if with_cpu:  # CPU baselines run after every GPU measurement (main)
        DEFERRED.append(_cpu)
    return out


def c4_bench(mx, with_cpu, threads, admm_iter):
    """BASELINE config 4 / SURVEY C4 on one GPU: 3D SquareGrid n = 63 (512,191 nodes, 3,000,564
    tetrahedra), the anisotropic shell monitor (MonType 6), dt 0.025 tau 0.5 (the 3DMonitor2x0
    family) and rho 2000 (at the family's rho 50 this monitor inverts elements under the reference
    algorithm -- the CPU oracle asserts by the third step on n = 16; at rho 500 the n = 63 mesh
    inverts by the fifth step), 10 ADMM iterations per step, early exit off.  The
    element-partitioned multi-GPU form of this workload is `bench.py --workload c4` under
    torch.distributed.run."""
    mesh = mx.MeshData.rect(3, 63)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5)
    E = mx.Engine(M, 0.025)
    t0 = time.perf_counter()
    E.step(admm_iter, -1.0)
    E.sync()
    first = time.perf_counter() - t0
    E.step(admm_iter, -1.0)
    E.set_timing(True)
    E.reset_stats()
    E.sync()
    steps = 3
    t0 = time.perf_counter()
    for _ in range(steps):
        E.step(admm_iter, -1.0)
    E.sync()
    el = time.perf_counter() - t0
    st = E.stats()
    prox_ms = st["t_prox_ms"] / max(st["n_prox"], 1)
    xup_ms = st["t_xupdate_ms"] / max(st["n_xupdate"], 1)
    prox_gbs = st["prox_bytes"] / (prox_ms * 1e-3) / 1e9
    out = {"workload": "C4: 3D SquareGrid n=63, %d nodes, %d tetrahedra, anisotropic shell monitor (MonType 6), "
                       "dt 0.025 tau 0.5 rho 2000, %d ADMM iterations per step" % (mesh.nP, mesh.nF, admm_iter),
           "value": round(steps * admm_iter / el, 3), "unit": "ADMM it/s", "first_step_ms": round(first * 1e3, 1),
           "kernels": {"k_prox_wave_ms": round(prox_ms, 4), "k_xupdate_ms": round(xup_ms, 4),
                       "bfgs_iters_per_prox": round(st["bfgs_iters"] / max(st["admm_iters"], 1) / mesh.nF, 4)},
           "roofline": {"bound": "hbm", "kernel": PROX3D_NAME, "achieved": round(prox_gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(prox_gbs / HBM_PEAK_GBS, 4),
                        "bytes_per_launch": st["prox_bytes"], "avg_launch_ms": round(prox_ms, 4)}}
    tr, trr = pmc_traffic(PROX3D_NAME)
    out["roofline"]["traffic"], out["roofline"]["traffic_fetch_uncorrected"] = tr, trr
    E.close()
    def _cpu():  # the oracle (OpenMP prox), same mesh and protocol: the FD-Hessian step untimed, then
        # C4_CPU_STEPS steps of admm_iter iterations (a bounded sample: ~25 s on 16 cores)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py
        om = oracle_py.Mesh(3, mesh.Xp, mesh.F, mesh.mask)
        O = oracle_py.Integrator(om, 6, 0.025, 0.5, 2000.0, nthreads=threads)
        O.step(admm_iter, -1.0)
        t0 = time.perf_counter()
        for _ in range(C4_CPU_STEPS):
            O.step(admm_iter, -1.0)
        cdt = (time.perf_counter() - t0) / C4_CPU_STEPS
        out["cpu_baseline"] = {"value": round(admm_iter / cdt, 3), "unit": "ADMM it/s", "cores": threads, "kind": "port",
                               "host": host_info(threads),
                               "sample": "C4 mesh, %d timed steps of %d ADMM iterations after set-up and the FD-Hessian "
                                         "step (oracle/oracle.cpp, g++ -O3 -msse2 -fopenmp, %d threads)"
                                         % (C4_CPU_STEPS, admm_iter, threads)}
    if with_cpu:  # CPU baselines run after every GPU measurement (main)
        DEFERRED.append(_cpu)
    return out


def bfgs_bench(mx, with_cpu, threads, admm_iter, steps=3):
    """The compute-heavy prox regime: every other section runs at ~1.0 BFGS
    iteration per simplex per prox, where the prox is one blockGrad plus a Bkinv stream.  Here the
    1M-node SquareGrid n = 707 (1,001,113 nodes, 2,000,000 triangles) with MEx1 at rho = 1 (a weak
    ADMM penalty: the prox minimises the functional almost freely), dt 0.055 tau 0.5, where the
    BFGS loop (src/Mesh.cpp:827-856) takes ~3-4 iterations per simplex once the mesh moves.  Two
    untimed steps, then `steps` timed steps of admm_iter iterations; the CPU leg runs the oracle on
    the same mesh and trajectory (16 threads, 1 step after the same two)."""
    mesh = mx.MeshData.rect(2, 707)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 1), rho=1.0, tau=0.5)
    E = mx.Engine(M, 0.055)
    for _ in range(2):
        E.step(admm_iter, -1.0)
    E.set_timing(True)
    E.reset_stats()
    E.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        E.step(admm_iter, -1.0)
    E.sync()
    el = time.perf_counter() - t0
    st = E.stats()
    prox_ms = st["t_prox_ms"] / max(st["n_prox"], 1)
    xup_ms = st["t_xupdate_ms"] / max(st["n_xupdate"], 1)
    bpp = st["bfgs_iters"] / max(st["admm_iters"], 1) / mesh.nF
    # algorithmic bytes grow with the BFGS iterations only through Bkinv's LDS image (read once,
    # written once per prox): the same per-launch bytes as one iteration
    prox_gbs = st["prox_bytes"] / (prox_ms * 1e-3) / 1e9
    out = {"workload": "SquareGrid n=707, %d nodes, %d triangles, MEx1, rho 1, dt 0.055 tau 0.5, %d ADMM iterations "
                       "per step, steps 3-5 of the run" % (mesh.nP, mesh.nF, admm_iter),
           "value": round(steps * admm_iter / el, 3), "unit": "ADMM it/s", "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 3),
           "kernels": {"k_prox_ms": round(prox_ms, 4), "k_xupdate_ms": round(xup_ms, 4),
                       "bfgs_iters_per_prox": round(bpp, 4), "max_bfgs": st["max_bfgs"]},
           "prox_GBs_algorithmic": round(prox_gbs, 1),
           "prox_us_per_bfgs_iteration": round(prox_ms * 1e3 / max(bpp, 1e-9), 2)}
    fl = pmc_entry(prox2d_name() + "@bfgs_heavy").get("fp64_flops_per_launch")
    if fl:
        out["prox_fp64"] = {"executed_flops_per_launch": fl, "achieved_TFLOPs": round(fl / (prox_ms * 1e-3) / 1e12, 2),
                            "peak_TFLOPs": 78.6, "frac": round(fl / (prox_ms * 1e-3) / 1e12 / 78.6, 4),
                            "source": "builder-measured rocprofv3 SQ_INSTS_VALU_*_F64 pass of this section "
                                      "(profiles/pmc_summary.json)"}
    E.close()

    def _cpu():
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py
        om = oracle_py.Mesh(2, mesh.Xp, mesh.F, mesh.mask)
        O = oracle_py.Integrator(om, 1, 0.055, 0.5, 1.0, nthreads=threads)
        for _ in range(2):
            O.step(admm_iter, -1.0)
        b0 = O.bfgs_iters()
        t0 = time.perf_counter()
        O.step(admm_iter, -1.0)
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(admm_iter / cdt, 3), "unit": "ADMM it/s", "cores": threads,
                               "kind": "port", "bfgs_iters_per_prox": round((O.bfgs_iters() - b0) / admm_iter / mesh.nF, 4),
                               "gpu_speedup": round(out["value"] * cdt / admm_iter, 1),
                               "sample": "the same mesh and trajectory: 2 untimed steps, then 1 timed step of %d ADMM "
                                         "iterations (oracle/oracle.cpp, %d threads)" % (admm_iter, threads)}
    if with_cpu:
        DEFERRED.append(_cpu)
    return out


def tv_bench(mx, n, admm_iter, steps=3):
    """Time-varying monitor (BASELINE config 5's "time-varying monitor") on one GPU:
    3D SquareGrid n (63: the C4 mesh; 136: C5, 5.09 M nodes), MonType 7 (a bump moving on a circle),
    the monitor grid rebuilt on the device at every step start (mmadmm_set_regrid), dt 0.025 tau 0.5
    rho 2000, admm_iter ADMM iterations per step.  value = ADMM it/s including the rebuilds."""
    mesh = mx.MeshData.rect(3, n)
    t0 = time.perf_counter()
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(3, 7), rho=2000.0, tau=0.5)
    E = mx.Engine(M, 0.025)
    E.set_regrid(True)
    setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    E.step(admm_iter, -1.0)
    E.sync()
    first = time.perf_counter() - t0
    E.step(admm_iter, -1.0)
    E.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        E.step(admm_iter, -1.0)
    E.sync()
    el = time.perf_counter() - t0
    E.set_regrid(False)
    reps = 3
    t1 = time.perf_counter()
    for r in range(reps):
        E.regrid(0.1 * r)
    E.sync()
    rg = (time.perf_counter() - t1) / reps
    out = {"workload": "3D SquareGrid n=%d, %d nodes, %d tetrahedra, time-varying moving-bump monitor (MonType 7), "
                       "grid rebuilt on the device every step, dt 0.025 tau 0.5 rho 2000, %d ADMM iterations per step"
                       % (n, mesh.nP, mesh.nF, admm_iter),
           "value": round(steps * admm_iter / el, 3), "unit": "ADMM it/s", "ms_per_step": round(el / steps * 1e3, 2),
           "regrid_ms": round(rg * 1e3, 3), "first_step_ms": round(first * 1e3, 1), "setup_s": round(setup, 2),
           "regrids": E.stats()["regrids"]}
    E.close()
    return out


def prox2d_name():
    """the steady 2D prox kernel the engine launches (workgroup size: MMX_PROX_BLOCK, default 64)"""
    return "k_prox_lds<2, %d>" % int(os.environ.get("MMX_PROX_BLOCK", "64"))


# the steady 3D prox on the full-row (anisotropic) monitor grid; isotropic grids launch the <3, false, true>
# instance
PROX3D_NAME = "k_prox_wave<3, false, false>"


def pmc_entry(kernel):
    """The committed rocprofv3 PMC summary of a kernel (profiles/pmc_summary.json); `kernel` is the
    short name, template arguments included, or a prefix of it ending in ','."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    if kernel in d:
        return d[kernel]
    for k, v in d.items():
        if k.startswith(kernel):
            return v
    return {}


def pmc_traffic(kernel):
    """Per-launch HBM bytes of a kernel from the PMC passes (FETCH_SIZE x2 per the gfx950
    correction + WRITE_SIZE; and raw)."""
    d = pmc_entry(kernel)
    return d.get("hbm_bytes_per_launch"), d.get("hbm_bytes_raw_per_launch")


def host_info(threads):
    """The GPU box's host as the CPU baseline saw it: nproc, the CPUs this job may run
    on, the lscpu model and physical core count, and the threads the baseline used."""
    info = {"threads_used": threads, "nproc": os.cpu_count(), "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "threads_note": "the all-core leg uses the CPU share this job is granted (the harness sets OMP_NUM_THREADS "
                            "on the GPU box; the box's other cores serve other jobs), not every physical core "
                            "nproc reports"}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = dict((a.strip(), b.strip()) for a, b in (ln.split(":", 1) for ln in out.splitlines() if ":" in ln))
        info["model"] = kv.get("Model name")
        if kv.get("Core(s) per socket") and kv.get("Socket(s)"):
            info["physical_cores"] = int(kv["Core(s) per socket"]) * int(kv["Socket(s)"])
        info["threads_per_core"] = kv.get("Thread(s) per core")
    except (OSError, ValueError):
        pass
    return info


def cpu_threads(args):
    """Threads of the CPU baseline: --cpu-threads, else every CPU the job is granted (the harness's
    CPU share: OMP_NUM_THREADS when it sets one, else the affinity mask)."""
    if args.cpu_threads:
        return args.cpu_threads
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env:
        return env
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


CPU_STEPS = 5  # >= 5 timed steps
C4_CPU_STEPS = 2  # C4 on the CPU: ~1.3 ADMM it/s on 16 cores, so 2 steps of 10 iterations bound the sample


def cpu_baseline(mesh, admm_iter, threads, mon=1, dt=0.055, tau=0.5, rho=50.0, label="C3", steps1=1):
    """Reference-equivalent CPU path (the oracle: CPU restatement of the reference, OpenMP prox,
    serial consensus algebra, -O3 -msse2) on the same mesh; bounded sample: set-up and the
    FD-Hessian step untimed, then CPU_STEPS timed steps of admm_iter iterations on `threads`
    threads, and steps1 further steps of admm_iter iterations on one thread (like for like)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py

    om = oracle_py.Mesh(mesh.dim, mesh.Xp, mesh.F, mesh.mask)
    O = oracle_py.Integrator(om, mon, dt, tau, rho, nthreads=threads)
    O.step(admm_iter, -1.0)
    t0 = time.perf_counter()
    for _ in range(CPU_STEPS):
        O.step(admm_iter, -1.0)
    el = time.perf_counter() - t0
    oracle_py.set_threads(1)  # all cores and 1 thread, the same protocol (steps of admm_iter)
    t0 = time.perf_counter()
    for _ in range(steps1):
        O.step(admm_iter, -1.0)
    el1 = time.perf_counter() - t0
    return {"value": round(CPU_STEPS * admm_iter / el, 3), "unit": "ADMM it/s", "cores": threads, "kind": "port",
            "value_1thread": round(steps1 * admm_iter / el1, 3), "host": host_info(threads),
            "sample": f"{label} mesh, {CPU_STEPS} timed steps of {admm_iter} ADMM iterations after set-up and the "
                      f"FD-Hessian step (oracle/oracle.cpp, g++ -O3 -msse2 -fopenmp, {threads} threads); "
                      f"value_1thread: {steps1} further step(s) of {admm_iter} ADMM iterations on 1 thread"}


def stream_copy_ceiling(torch, la):
    """Measured HBM ceiling on this box: a 1 GiB device-to-device copy (read + write bytes / time)
    with the library's 16-B-per-lane streaming kernels (the fastest of its variants), and with
    torch's copy_ for comparison."""
    n = 1 << 27  # doubles
    x = torch.ones(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    dev = torch.cuda.current_device()
    ms = min(la.stream_copy_ms(x.data_ptr(), y.data_ptr(), n, reps=20, device=dev, variant=v) for v in (0, 1, 2))
    kern = 2 * 8 * n / (ms * 1e-3) / 1e9
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 20
    for _ in range(reps):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    tms = e0.elapsed_time(e1) / reps
    del x, y
    return round(kern, 1), round(2 * 8 * n / (tms * 1e-3) / 1e9, 1)


def lib_provenance(mx):
    """the library's embedded source hash against the sources of the tree this run is in"""
    info = mx.build_info()
    sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "tools"))
    try:
        import src_hash
        tree = src_hash.source_hash()
    except Exception:  # noqa: BLE001 -- reported as unknown
        tree = None
    return {"lib_src_hash": info.get("src_hash"), "lib_git": info.get("git"), "tree_src_hash": tree,
            "lib_matches_tree": tree is not None and tree == info.get("src_hash")}


def pmc_flops(kernel):
    """Executed fp64 flops per launch from the SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 pass."""
    return pmc_entry(kernel).get("fp64_flops_per_launch")


def main():
    args = parse()
    # before anything touches the GPU: a --gpus N run is N ranks, or it fails
    share = args.comm == "host" or args.rendezvous_only
    plan, val = launch_plan(args.gpus, os.environ, visible_gpus, share=share)
    if plan == "error":
        log(val)
        sys.exit(2)
    if plan == "spawn":
        sys.exit(relaunch(val, args.budget_s))
    world = val
    if args.rendezvous_only:
        sys.exit(rendezvous_only(world, args.budget_s))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        start_watchdog(args.budget_s, rank)
        phase("start")
    import datetime

    import torch  # first, so libmmadmm binds to the same HIP runtime
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    host_comm = world > 1 and args.comm == "host"
    if host_comm:  # rehearsal: ranks may share the visible GPUs
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(local)
        phase("rendezvous")
        dist.init_process_group("gloo" if host_comm else "nccl",
                                timeout=datetime.timedelta(seconds=max(args.budget_s, 60.0)))
    import mmadmm_amd as mx
    import lasolver_amd as la

    c5 = args.workload == "c5"
    c4 = args.workload == "c4" or c5  # 3D
    base_nodes = 5086809 if c5 else (512191 if c4 else 1000519)
    dt = 0.025 if c4 else 0.055
    disc_n = args.disc_n if world == 1 else int(round(args.disc_n * world ** 0.5))
    cube_n = 63 if world == 1 else int(round(63 * world ** (1.0 / 3.0)))

    used = {}

    def make_mesh(n_ranks):
        if c5:
            used["n"] = 136
            log(f"rank {rank}/{world}: 3D cube n=136 (C5), time-varying monitor")
            m = mx.MeshData.rect(3, 136)
            return m, mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 7), rho=2000.0, tau=0.5, device=local)
        if c4:
            n = 63 if n_ranks == 1 else cube_n
            used["n"] = n
            log(f"rank {rank}/{world}: 3D cube n={n}")
            m = mx.MeshData.rect(3, n)
            return m, mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5, device=local)
        n = args.disc_n if n_ranks == 1 else disc_n
        used["n"] = n
        log(f"rank {rank}/{world}: hexdisc N={n}")
        m = mx.MeshData.hexdisc(n, 0.5, 0.5, 0.5)
        return m, mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5, device=local)

    if world > 1:
        phase("mesh")
    mesh, M = make_mesh(world)
    t_setup = time.perf_counter()
    parallelism = parallelism_label(world, args.comm)
    comm = None
    rccl_nranks = comm_nranks = None
    if world > 1:
        # the element-partitioned engine or nothing: a failure here ends the run with a non-zero
        # exit status (no silent fallback to replicas)
        phase("communicator")
        if host_comm:
            comm = mx.Comm.host(world, rank, mx.TorchDistTransport())
        else:
            uid = [mx.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = mx.Comm.rccl(world, rank, uid[0], local, timeout_s=args.comm_timeout)
        phase("engine")
        eng = mx.Engine(M, dt, rank=rank, nranks=world, comm=comm)
        # ncclCommCount for RCCL; the host transport only knows the count it was made with
        comm_nranks = comm.nranks()
        rccl_nranks = None if host_comm else comm_nranks
        if comm_nranks != world:
            raise RuntimeError("communicator has %d ranks, expected %d" % (comm_nranks, world))
    else:
        eng = mx.Engine(M, dt)
    if c5:
        eng.set_regrid(True)  # the monitor grid rebuilt on the device at every step start
    t_setup = time.perf_counter() - t_setup
    log(f"rank {rank}: setup {t_setup:.1f}s, local nodes {eng.nP}, local simplices {eng.nF}")
    if world > 1:
        phase("setup")
        phase("warmup")

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

    if world > 1:
        phase("timed")
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
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if host_comm else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if world > 1:
        phase("report")
    st = eng.stats()
    # per rank: local nodes and simplices, the halo exchange's device time per ADMM iteration (pack +
    # send/recv on its stream, overlapped with the interior x-update), its bytes, the interior nodes
    mine = (eng.nP, eng.nF, (st["t_exchange_ms"] * 1e3 / st["n_exchange"]) if st["n_exchange"] else None,
            st["halo_send_bytes"], st["halo_recv_bytes"], st["interior_nodes"], st["overlap"])
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    # a second run with the early exit enabled reports the iterations actually executed
    eng.reset_stats()
    for _ in range(3):
        eng.step(args.admm_iter, 1e-3)
    st_early = eng.stats()
    iters = args.steps * args.admm_iter
    # whole-job throughput: C5 is one fixed mesh (strong scaling); C3/C4 in units of the
    # single-GPU mesh (the global mesh grows with the ranks: weak scaling)
    scale = 1.0 if c5 else mesh.nP / base_nodes
    prox_ms = st["t_prox_ms"] / max(st["n_prox"], 1)
    xup_ms = st["t_xupdate_ms"] / max(st["n_xupdate"], 1)
    prox_gbs = st["prox_bytes"] / (prox_ms * 1e-3) / 1e9
    xup_gbs = st["xupdate_bytes"] / (xup_ms * 1e-3) / 1e9
    # 3D: the isotropic-grid instance when the monitor grid is isotropic (C5's moving bump)
    prox_name = (PROX3D_NAME.replace("false>", "true>") if st["monitor_iso"] else PROX3D_NAME) if c4 else prox2d_name()
    # the committed PMC passes profile the default run (C3 and the C4 section): per-launch figures
    # of another mesh size do not apply to C5
    traffic, traffic_raw = pmc_traffic(prox_name) if not c5 else (None, None)
    result = {
        "metric": ("ADMM iterations/sec on 5.09M-node 3D mesh, time-varying monitor (BASELINE config 5)" if c5 else
                   "ADMM iterations/sec on 512k-node 3D mesh (BASELINE config 4)" if c4 else
                   "ADMM iterations/sec on 1M-node 2D mesh; achieved HBM GB/s in SpMV"),
        "value": round(iters / elapsed * scale, 3),
        "unit": "ADMM it/s",
        "n_gpus": min(world, torch.cuda.device_count()) if host_comm else world,
        "ranks": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if c5 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": ("C5: 3D SquareGrid n=136, %d nodes, %d tetrahedra, time-varying moving-bump monitor "
                                "(MonType 7) with the grid rebuilt on the device every step, dt 0.025 tau 0.5 rho 2000, "
                                "%d ADMM iterations per step" % (mesh.nP, mesh.nF, args.admm_iter)) if c5 else
                               ("C4: 3D SquareGrid n=%d, %d nodes, %d tetrahedra, anisotropic shell monitor "
                                "(MonType 6), dt 0.025 tau 0.5 rho 2000, %d ADMM iterations per step"
                                % (used["n"], mesh.nP, mesh.nF, args.admm_iter)) if c4 else
                               ("C3: 2D circular mesh (hexagonal disc N=%d), %d nodes, %d triangles, MEx1 "
                                "monitor, dt 0.055 tau 0.5 rho 50, %d ADMM iterations per step"
                                % (used["n"], mesh.nP, mesh.nF, args.admm_iter)),
                   "global_nodes": mesh.nP, "global_simplices": mesh.nF, "nodes_rank0": eng.nP,
                   "simplices_rank0": eng.nF, "nodes_per_rank": [p[0] for p in per_rank],
                   "simplices_per_rank": [p[1] for p in per_rank], "rccl_nranks": rccl_nranks,
                   "comm_nranks": (comm_nranks if world > 1 else None),
                   "exchange_us_per_iter": ([None if p[2] is None else round(p[2], 2) for p in per_rank]
                                            if world > 1 else None),
                   "halo_bytes_per_iter": ([{"send": int(p[3]), "recv": int(p[4])} for p in per_rank]
                                           if world > 1 else None),
                   "interior_nodes_per_rank": ([p[5] for p in per_rank] if world > 1 else None),
                   "halo_overlap": (bool(per_rank[0][6]) if world > 1 else None),
                   "imbalance": (round(max(p[1] for p in per_rank) / (sum(p[1] for p in per_rank) / world), 4)
                                 if world > 1 else None),
                   "admm_iter": args.admm_iter, "parallelism": parallelism,
                   "comm": (args.comm if world > 1 else None),
                   "value_unit_note": "ADMM it/s x global nodes / %d" % base_nodes},
        "roofline": {"bound": "hbm", "kernel": prox_name,
                     "achieved": round(prox_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(prox_gbs / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_fetch_uncorrected": traffic_raw,
                     "traffic_source": "builder-measured, not this run: profiles/pmc_summary.json (rocprofv3 "
                                       "FETCH_SIZE, WRITE_SIZE passes of the committed tree)",
                     "bytes_per_launch": st["prox_bytes"],
                     "avg_launch_ms": round(prox_ms, 4)},
        "prox_fp64": None,
        "kernels": {"k_prox_ms": round(prox_ms, 4), "k_xupdate_ms": round(xup_ms, 4),
                    "k_xupdate_GBs": round(xup_gbs, 1), "bfgs_iters_per_prox":
                        round(st["bfgs_iters"] / max(st["admm_iters"], 1) / mesh.nF, 4)},
        "early_exit": {"tol": 1e-3, "steps": 3,
                       "admm_iters_per_step": round(st_early["admm_iters"] / 3, 2)},
        "first_step_ms": round(first_ms, 2),
        "setup_s": round(t_setup, 2),
        "build": lib_provenance(mx),
    }
    fl = pmc_flops(prox_name) if not c5 else None
    if fl:
        result["prox_fp64"] = {"executed_flops_per_launch": fl, "achieved_TFLOPs": round(fl / (prox_ms * 1e-3) / 1e12, 2),
                               "peak_TFLOPs": 78.6, "frac": round(fl / (prox_ms * 1e-3) / 1e12 / 78.6, 4),
                               "source": "rocprofv3 SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 x 64 lanes "
                                         "(profiles/pmc_summary.json); peak: AMD MI355X fp64 vector spec"}
    if not c4:
        # SURVEY §8(d)'s compulsory bytes exclude the entry-gradient cache (16 K B per simplex,
        # read and written every launch): an implementation choice that saves a blockGrad
        comp = st["prox_bytes"] - 16 * 6 * eng.nF
        result["roofline"]["compulsory_bytes_per_launch"] = comp
        result["roofline"]["frac_compulsory"] = round(comp / (prox_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        result["roofline"]["compulsory_note"] = ("bytes_per_launch minus the prox-entry gradient cache "
                                                 "(16 K B per simplex, K = 6)")
    if rank == 0 and world == 1:
        cc, tc = stream_copy_ceiling(torch, la)
        result["roofline"]["measured_copy_ceiling_GBs"] = cc
        result["roofline"]["torch_copy_GBs"] = tc
        result["roofline"]["frac_of_copy_ceiling"] = round(prox_gbs / cc, 4)
    if not args.no_spmv and not c4:
        log("spmv microbenchmark")
        result["spmv"] = spmv_bench(torch, la, mx, with_cpu=(rank == 0 and world == 1 and not args.no_cpu_baseline))
    if not args.no_be and world == 1 and not c4:
        log("backward Euler")
        result["backward_euler"] = be_bench(mx, with_cpu=not args.no_cpu_baseline)
    threads = cpu_threads(args)
    if not args.no_c2 and world == 1 and not c4:
        log("C2 square grid")
        result["c2"] = c2_bench(mx, not args.no_cpu_baseline, threads, args.admm_iter)
    if not args.no_bfgs and world == 1 and not c4:
        log("BFGS-heavy 2D (rho 1)")
        try:
            result["bfgs_heavy"] = bfgs_bench(mx, not args.no_cpu_baseline, threads, args.admm_iter)
        except Exception as e:  # noqa: BLE001 -- reported in the line, the headline stands
            result["bfgs_heavy"] = {"error": str(e)}
    if not args.no_3d and world == 1 and not c4:
        log("3D C4")
        result["c4_3d"] = c4_bench(mx, not args.no_cpu_baseline, threads, args.admm_iter)
        log("3D time-varying monitor")
        result["c4_time_varying"] = tv_bench(mx, 63, args.admm_iter)
        if not args.no_be:
            log("3D backward Euler (C4)")
            try:
                result["backward_euler_c4"] = be_bench(mx, not args.no_cpu_baseline, dim=3)
            except Exception as e:  # noqa: BLE001 -- reported in the line, the headline stands
                result["backward_euler_c4"] = {"error": str(e)}
    if args.c5 and world == 1 and rank == 0:
        log("3D C5 time-varying (5.09 M nodes)")
        result["c5_time_varying"] = tv_bench(mx, 136, args.admm_iter, steps=2)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not c4:
        log("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(mesh, args.admm_iter, threads, steps1=CPU_STEPS)
    for f in DEFERRED:  # the sections' CPU baselines, after every GPU measurement
        log("cpu baseline:", f.__qualname__.split(".")[0])
        f()
    # the GPU speed-up against the CPU path on all cores and on one (reported, not a target)
    cb = result.get("cpu_baseline")
    if cb and cb.get("value"):
        cb["gpu_speedup"] = round(result["value"] / cb["value"], 1)
        if cb.get("value_1thread"):
            cb["gpu_speedup_1thread"] = round(result["value"] / cb["value_1thread"], 1)
    c4r = result.get("c4_3d", {})
    c2r = result.get("c2", {})
    if c2r.get("cpu_baseline", {}).get("value"):
        c2r["cpu_baseline"]["gpu_speedup"] = round(c2r["value"] / c2r["cpu_baseline"]["value"], 1)
    if c4r.get("cpu_baseline", {}).get("value"):
        c4r["cpu_baseline"]["gpu_speedup"] = round(c4r["value"] / c4r["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()
        phase("done")


if __name__ == "__main__":
    main()
