"""Element-partitioned ADMM on one GPU: nranks engines (one per thread) exchanging interface-slot
values through the loopback communicator.  Node positions must equal the single-engine run BIT
FOR BIT for fixed iteration counts (the interface sums run in ascending global simplex order on
every rank); energies and residual norms are sums over ranks and agree to rounding."""
import os
import sys
import threading

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "mm-admm_amd", "python"))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    import torch  # noqa: F401
    import mmadmm_amd
    return mmadmm_amd


def _run_parallel(fns):
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


CASES = [
    ("rect2d", lambda mx: mx.MeshData.rect(2, 12), 2, 3, 1000.0, 0.5, 0.025, 2, "rcb"),
    ("rect2d_3ranks", lambda mx: mx.MeshData.rect(2, 14), 2, 5, 50.0, 0.5, 0.05, 3, "rcb"),
    ("hexdisc", lambda mx: mx.MeshData.hexdisc(10, 0.5, 0.5, 0.5), 2, 1, 50.0, 0.5, 0.055, 2, "rcb"),
    ("hexdisc_4ranks", lambda mx: mx.MeshData.hexdisc(14, 0.5, 0.5, 0.5), 2, 1, 50.0, 0.5, 0.055, 4, "rcb"),
    ("hexdisc_ranges", lambda mx: mx.MeshData.hexdisc(10, 0.5, 0.5, 0.5), 2, 1, 50.0, 0.5, 0.055, 3, "ranges"),
    ("rect3d", lambda mx: mx.MeshData.rect(3, 3), 3, 1, 20.0, 0.5, 0.05, 2, "rcb"),
    ("rect3d_4ranks", lambda mx: mx.MeshData.rect(3, 4), 3, 6, 2000.0, 0.5, 0.025, 4, "rcb"),
]


@pytest.mark.parametrize("name,gen,dim,mon,rho,tau,dt,nranks,method", CASES, ids=[c[0] for c in CASES])
def test_partitioned_equals_single(mx, name, gen, dim, mon, rho, tau, dt, nranks, method):
    mesh = gen(mx)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, mon), rho=rho, tau=tau, device=0)
    ref = mx.Engine(M, dt)
    comm = mx.Comm.loopback(nranks)
    parts = [mx.Engine(M, dt, rank=r, nranks=nranks, comm=comm, partition=method) for r in range(nranks)]
    # 5 steps: 2D partitions take z from the positions and fuse predictX into the first x-update
    # from the fourth step on (round 6), and overlap every x-update's interior nodes with the exchange
    steps, iters = 5, 6
    ih_ref = [ref.step(iters, -1.0)[0] for _ in range(steps)]
    ih = [[None] * steps for _ in range(nranks)]

    def run(r):
        def f():
            for k in range(steps):
                ih[r][k] = parts[r].step(iters, -1.0)[0]
        return f

    _run_parallel([run(r) for r in range(nranks)])
    xr = ref.get("x").reshape(-1, dim)
    covered = np.zeros(mesh.nP, bool)
    for r, e in enumerate(parts):
        ids = e.local_nodes()
        x = e.get("x").reshape(-1, dim)
        assert np.array_equal(x, xr[ids]), f"rank {r}: node positions differ from the single-GPU run"
        covered[ids] = True
        # every rank sees the same combined energy, equal to the single-GPU one to rounding
        for k in range(steps):
            assert ih[r][k] == ih[0][k]
            assert abs(ih[r][k] - ih_ref[k]) <= 1e-12 * abs(ih_ref[k])
    assert covered.all()
    # the early-exit path agrees too (same iteration decisions)
    ref2 = mx.Engine(M, dt)
    parts2 = [mx.Engine(M, dt, rank=r, nranks=nranks, comm=comm, partition=method) for r in range(nranks)]
    it_ref = ref2.step(50, 1e-3)[1]
    its = [None] * nranks

    def run2(r):
        def f():
            its[r] = parts2[r].step(50, 1e-3)[1]
        return f

    _run_parallel([run2(r) for r in range(nranks)])
    assert all(i == it_ref for i in its), (its, it_ref)
    for e in parts + parts2:
        e.close()
    comm.close()


def _check_rank_grid(e, gr, r):
    """A rank's rebuilt grid: the rows of its box equal the single-GPU grid, the others are NaN."""
    g = e.get("grid")
    ok = ~np.isnan(g)
    assert ok.any(), f"rank {r}: empty box"
    assert np.array_equal(g[ok], gr[ok]), f"rank {r}: grid rows differ"
    st = e.stats()
    assert 0 < st["regrid_rows"] <= len(g) // (e.dim * e.dim)


@pytest.mark.parametrize("gather", ["near", "all"])
@pytest.mark.parametrize("mon,dim,nranks,n", [(7, 2, 2, 12), (1, 2, 3, 12), (7, 3, 2, 4), (7, 2, 4, 40), (7, 3, 4, 10)])
def test_partitioned_regrid_equals_single(mx, mon, dim, nranks, n, gather, monkeypatch):
    """Time-varying monitor on a partition: every rank rebuilds the grid rows its simplices can
    reach (NaN elsewhere) from the vertices near them (gather "near": the ranks exchange only the
    owned vertices inside each other's search boxes; "all": every owned vertex all-gathered, the
    fallback); node positions stay bit-identical to the single-GPU run."""
    if gather == "all":
        monkeypatch.setenv("MMX_REGRID_GATHER", "all")
    else:
        monkeypatch.delenv("MMX_REGRID_GATHER", raising=False)
    mesh = mx.MeshData.rect(dim, n)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, mon), rho=200.0, tau=0.5, device=0)
    ref = mx.Engine(M, 0.05)
    ref.set_regrid(True)
    comm = mx.Comm.loopback(nranks)
    parts = [mx.Engine(M, 0.05, rank=r, nranks=nranks, comm=comm) for r in range(nranks)]
    for e in parts:
        e.set_regrid(True)
    steps = 4
    for _ in range(steps):
        ref.step(5, -1.0)

    def run(r):
        def f():
            for _ in range(steps):
                parts[r].step(5, -1.0)
        return f

    _run_parallel([run(r) for r in range(nranks)])
    xr = ref.get("x").reshape(-1, dim)
    gr = ref.get("grid")
    for r, e in enumerate(parts):
        _check_rank_grid(e, gr, r)
        assert np.array_equal(e.get("x").reshape(-1, dim), xr[e.local_nodes()]), f"rank {r}: positions differ"
        st = e.stats()
        assert st["regrids"] == steps
        if gather == "near":  # the candidate exchange sufficed at every rebuild
            assert st["regrid_fallbacks"] == 0 and 0 < st["regrid_cand"] <= mesh.nP + e.nP, st
    for e in parts:
        e.close()
    comm.close()


def _regrid_parts(mx, mesh, dim, nranks, steps, rho=200.0, dt=0.05):
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, 7), rho=rho, tau=0.5, device=0)
    ref = mx.Engine(M, dt)
    ref.set_regrid(True)
    for _ in range(steps):
        ref.step(5, -1.0)
    comm = mx.Comm.loopback(nranks)
    parts = [mx.Engine(M, dt, rank=r, nranks=nranks, comm=comm) for r in range(nranks)]
    for e in parts:
        e.set_regrid(True)
    _run_parallel([(lambda e: (lambda: [e.step(5, -1.0) for _ in range(steps)]))(e) for e in parts])
    xr = ref.get("x").reshape(-1, dim)
    for r, e in enumerate(parts):
        assert np.array_equal(e.get("x").reshape(-1, dim), xr[e.local_nodes()]), f"rank {r}: positions differ"
    ref.close()
    return comm, parts


@pytest.mark.parametrize("nranks", [2, 4])
def test_partitioned_regrid_disc_no_fallback(mx, nranks):
    """A non-rectangular domain (the hexagonal disc): the grid box's corners lie outside the disc, far
    from every vertex.  The exactness check of the near exchange only counts the sides of a rank's
    search box that lie inside the global vertex box (no vertex can lie beyond the others), so no
    rebuild falls back to the all-gather."""
    mesh = mx.MeshData.hexdisc(40, 0.5, 0.5, 0.5)
    comm, parts = _regrid_parts(mx, mesh, 2, nranks, 3)
    for r, e in enumerate(parts):
        st = e.stats()
        assert st["regrids"] == 3 and st["regrid_fallbacks"] == 0, (r, st)
        e.close()
    comm.close()


def test_partitioned_regrid_forced_fallback(mx, monkeypatch):
    """MMX_REGRID_MARGIN=0 shrinks the search box to the rank's own rows: the nearest-vertex check
    fails at the cut, every rank falls back to all-gathering the vertices (regridNear ->
    regridAll), and the result is still the single-GPU one."""
    monkeypatch.setenv("MMX_REGRID_MARGIN", "0")
    mesh = mx.MeshData.rect(2, 24)
    comm, parts = _regrid_parts(mx, mesh, 2, 3, 2)
    for r, e in enumerate(parts):
        st = e.stats()
        assert st["regrids"] == 2 and st["regrid_fallbacks"] == 2, (r, st)
        e.close()
    comm.close()


@pytest.mark.parametrize("dim,n,nranks", [(2, 24, 3), (3, 8, 2)])
def test_partitioned_regrid_long_run_equals_single(mx, dim, n, nranks):
    """20 steps with the moving-bump monitor (MonType 7) rebuilt at every step on a partition: the
    mesh stretches as the bump travels, and each rank's grid box follows it (the margin is the
    widest local simplex re-measured at every rebuild).  Node positions stay bit-identical to one
    GPU at every step, and no evaluation leaves a rank's box (no NonFiniteEnergyError)."""
    mesh = mx.MeshData.rect(dim, n)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, 7), rho=200.0, tau=0.5, device=0)
    dt = 0.05
    ref = mx.Engine(M, dt)
    ref.set_regrid(True)
    comm = mx.Comm.loopback(nranks)
    parts = [mx.Engine(M, dt, rank=r, nranks=nranks, comm=comm) for r in range(nranks)]
    for e in parts:
        e.set_regrid(True)
    steps = 20
    xs = []
    for _ in range(steps):
        ref.step(5, -1.0)
        xs.append(ref.get("x").reshape(-1, dim))
    got = [[None] * steps for _ in range(nranks)]

    def run(r):
        def f():
            for k in range(steps):
                parts[r].step(5, -1.0)
                got[r][k] = parts[r].get("x").reshape(-1, dim)
        return f

    _run_parallel([run(r) for r in range(nranks)])
    moved = np.abs(xs[-1] - mesh.Xp).max()
    assert moved > 1e-3, moved  # the bump moved the mesh
    for r, e in enumerate(parts):
        ids = e.local_nodes()
        for k in range(steps):
            assert np.array_equal(got[r][k], xs[k][ids]), f"rank {r} step {k}: positions differ"
        assert e.stats()["regrids"] == steps and e.stats()["regrid_fallbacks"] == 0
        e.close()
    comm.close()
    ref.close()


def test_c4_eight_ranks_regrid_equals_single(mx):
    """C4 (3D SquareGrid n = 63, 512,191 nodes, 3,000,564 tets) on an 8-rank loopback partition
    with the time-varying monitor rebuilt every step: one step of 3 ADMM iterations, node
    positions bit-identical to one GPU, each rank's grid rows equal to the single-GPU grid inside
    its box, and each rank fills well under the whole grid."""
    mesh = mx.MeshData.rect(3, 63)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(3, 7), rho=2000.0, tau=0.5, device=0)
    ref = mx.Engine(M, 0.025)
    ref.set_regrid(True)
    ref.step(3, -1.0)
    xr = ref.get("x").reshape(-1, 3)
    gr = ref.get("grid")
    total = len(gr) // 9
    ref.close()
    nranks = 8
    comm = mx.Comm.loopback(nranks)
    parts = [mx.Engine(M, 0.025, rank=r, nranks=nranks, comm=comm) for r in range(nranks)]
    for e in parts:
        e.set_regrid(True)
    _run_parallel([(lambda e: (lambda: e.step(3, -1.0)))(e) for e in parts])
    for r, e in enumerate(parts):
        assert np.array_equal(e.get("x").reshape(-1, 3), xr[e.local_nodes()]), f"rank {r}: positions differ"
        _check_rank_grid(e, gr, r)
        st = e.stats()
        assert st["regrid_rows"] < 0.5 * total, (r, st["regrid_rows"], total)
        # only the vertices near the rank's box travel: a fraction of the all-gather's bytes
        assert st["regrid_fallbacks"] == 0 and st["regrid_cand"] < 0.5 * mesh.nP, st
        assert st["regrid_gather_bytes"] < 0.5 * 8 * 3 * mesh.nP, st
        e.close()
    comm.close()


def test_rccl_communicator_single_rank(mx):
    """The RCCL communicator bench.py uses for N > 1 (ncclGetUniqueId, ncclCommInitRank,
    ncclAllGather on the engine's stream), driven at one rank: the partitioned engine over it
    equals the plain engine bit for bit. Ranks on several GPUs are left to the multi-GPU run."""
    mesh = mx.MeshData.rect(2, 12)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 3), rho=1000.0, tau=0.5, device=0)
    ref = mx.Engine(M, 0.025)
    comm = mx.Comm.rccl(1, 0, mx.Comm.unique_id(), 0)
    assert comm.nranks() == 1  # ncclCommCount, as bench.py's rccl_nranks
    part = mx.Engine(M, 0.025, rank=0, nranks=1, comm=comm)
    for _ in range(3):
        ref.step(5, -1.0)
        part.step(5, -1.0)
    ids = part.local_nodes()
    assert np.array_equal(part.get("x").reshape(-1, 2), ref.get("x").reshape(-1, 2)[ids])


def test_partitioned_early_exit_equals_single(mx):
    """Early exit (tol > 0) on a partition: the residual norms are summed over ranks, so every rank
    stops at the same iteration as the single-GPU engine (bench.py's early-exit run at N > 1)."""
    mesh = mx.MeshData.hexdisc(10, 0.5, 0.5, 0.5)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5, device=0)
    ref = mx.Engine(M, 0.055)
    nranks = 2
    comm = mx.Comm.loopback(nranks)
    parts = [mx.Engine(M, 0.055, rank=r, nranks=nranks, comm=comm) for r in range(nranks)]
    for _ in range(3):
        ref.step(10, 1e-3)

    def run(r):
        def f():
            for _ in range(3):
                parts[r].step(10, 1e-3)
        return f

    _run_parallel([run(r) for r in range(nranks)])
    xr = ref.get("x").reshape(-1, 2)
    n_ref = ref.stats()["n_prox"]
    for e in parts:
        assert np.array_equal(e.get("x").reshape(-1, 2), xr[e.local_nodes()])
        assert e.stats()["n_prox"] == n_ref


@pytest.mark.parametrize("knob", ["MMX_OVERLAP", "MMX_ZX", "MMX_FUSE_PRED"])
@pytest.mark.parametrize("dim,nranks", [(2, 3), (3, 2)])
def test_partition_step_variants_bitwise(mx, dim, nranks, knob, monkeypatch):
    """Round 6: the partitioned step overlaps the interior x-update with the
    halo exchange and, in 2D, keeps the one-rank step start (z from the positions, predictX fused).
    Each against engines with it turned off: node positions, xPrev, xBar, z, u bit-identical; the
    exchange is timed on its stream and its bytes reported."""
    mesh = mx.MeshData.hexdisc(14, 0.5, 0.5, 0.5) if dim == 2 else mx.MeshData.rect(3, 4)
    mon, rho, dt = (1, 50.0, 0.055) if dim == 2 else (6, 2000.0, 0.025)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, mon), rho=rho, tau=0.5, device=0)
    comm_a, comm_b = mx.Comm.loopback(nranks), mx.Comm.loopback(nranks)
    A = [mx.Engine(M, dt, rank=r, nranks=nranks, comm=comm_a) for r in range(nranks)]
    monkeypatch.setenv(knob, "0")
    B = [mx.Engine(M, dt, rank=r, nranks=nranks, comm=comm_b) for r in range(nranks)]
    monkeypatch.delenv(knob)
    for e in A + B:
        e.set_timing(True)
    steps = 5

    def run(es, r):
        def f():
            for _ in range(steps):
                es[r].step(6, -1.0)
        return f

    _run_parallel([run(A, r) for r in range(nranks)] + [run(B, r) for r in range(nranks)])
    for r in range(nranks):
        for f in ("x", "xPrev", "xBar", "z", "u"):
            assert np.array_equal(A[r].get(f), B[r].get(f)), f"{knob}=0, rank {r}: {f} differs"
        st = A[r].stats()
        assert st["overlap"] == 1 and 0 < st["interior_nodes"] < A[r].nP
        assert st["n_exchange"] == steps * 7 and st["t_exchange_ms"] > 0
        assert st["halo_send_bytes"] > 0 and st["halo_recv_bytes"] > 0
        if knob == "MMX_OVERLAP":
            sb = B[r].stats()
            assert sb["overlap"] == 0 and sb["interior_nodes"] == B[r].nP
    for e in A + B:
        e.close()
    comm_a.close()
    comm_b.close()
