"""BASELINE.json's configurations at their stated sizes on the GPU, against the oracle.

SURVEY.md §8 sizes: C2 SquareGrid n = 223 (99,905 nodes), C3 the 1,000,519-node disc of the
headline bench, C4 3D SquareGrid n = 63 (512,191 nodes, 3,000,564 tetrahedra), C5 3D n = 136
(5,086,809 nodes, 30,185,472 tetrahedra, time-varying monitor).  The size-dependent code paths
meet the oracle here: the deferred per-iteration reduction slices (maxBlocks), the XCD block
ranges of the prox, the LDS chunk tail of the 2D prox and 64-bit Bkinv indexing.

* C2, C3, C4: bit-identical device state (x, z, u, Bkinv) to the oracle with correctly rounded pow
  and the exact diagonal solve, fixed iteration counts (the oracle runs on OMP_NUM_THREADS host
  cores); C2, C3 and C4 also at reference semantics (glibc pow, Jacobi-CG, early exit on): same
  ADMM and BFGS iteration counts and <= 1e-10 relative node-position error.
* C4 partitioned over two ranks (loopback communicator, one GPU) equals one GPU bit for bit.
* C5 (too large for the oracle in a test): one GPU equals a three-rank partition bit for bit.  On
  one GPU the Bkinv offsets of the last tetrahedra exceed 2^32 doubles; on the partition every
  rank's offsets stay below 2^31, so equality checks the 64-bit index path.  Plus properties: no
  inverted element, one grid rebuild per step, finite energies.
"""
import os
import threading

import numpy as np
import pytest

import mmadmm_amd as mx
import oracle_py

pytestmark = pytest.mark.gpu

POS_TOL = 1e-10


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)


@pytest.fixture(autouse=True)
def _pow_mode_reset():
    yield
    oracle_py.set_pow_mode(0)


def _pair(m, mon, dt, tau, rho, pow_mode=1, cg_mode=1):
    oracle_py.set_pow_mode(pow_mode)
    om = oracle_py.Mesh(m.dim, m.Xp, m.F, m.mask)
    O = oracle_py.Integrator(om, mon, dt, tau, rho, nthreads=_threads(), cgMode=cg_mode)
    G = mx.Engine(mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(m.dim, mon), rho=rho, tau=tau), dt)
    return O, G


def _bitwise(O, G, fields=("x", "z", "u", "hess")):
    for f in fields:
        a, b = G.get(f), O.get(f)
        assert np.array_equal(a, b), f"{f}: {np.count_nonzero(a != b)} of {a.size} entries differ"


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
        t.join(timeout=900)
    if errs:
        raise errs[0]


def _partitioned(M, dt, nranks, steps, iters, regrid=False):
    comm = mx.Comm.loopback(nranks)
    parts = [mx.Engine(M, dt, rank=r, nranks=nranks, comm=comm) for r in range(nranks)]
    ih = [[None] * steps for _ in range(nranks)]
    for e in parts:
        if regrid:
            e.set_regrid(True)

    def run(r):
        def f():
            for k in range(steps):
                ih[r][k] = parts[r].step(iters, -1.0)[0]
        return f

    _run_parallel([run(r) for r in range(nranks)])
    return comm, parts, ih


def test_c2_square_grid_bitwise():
    """C2: SquareGrid n = 223, MEx1, Monitor2320-family parameters; 2 steps x 10 iterations."""
    m = mx.MeshData.rect(2, 223)
    assert (m.nP, m.nF) == (99905, 198916)
    O, G = _pair(m, 1, 0.055, 0.5, 50.0)
    for s in range(2):
        ih_o = O.step(10, -1.0)[0]
        ih_g = G.step(10, -1.0)[0]
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
    _bitwise(O, G)
    assert G.stats()["bfgs_iters"] == O.bfgs_iters()


def test_c2_square_grid_reference_semantics():
    """C2 with the reference's arithmetic (glibc pow, Jacobi-CG) and its early exit (tol 1e-3)."""
    m = mx.MeshData.rect(2, 223)
    O, G = _pair(m, 1, 0.055, 0.5, 50.0, pow_mode=0, cg_mode=0)
    for s in range(3):
        ih_o, it_o = O.step(10, 1e-3)[:2]
        ih_g, it_g = G.step(10, 1e-3)
        assert it_o == it_g, f"ADMM iteration count differs at step {s}"
        assert abs(ih_o - ih_g) <= 1e-11 * abs(ih_o)
    xo, xg = O.get("x"), G.get("x")
    assert np.abs(xo - xg).max() / np.abs(xo).max() <= POS_TOL


def test_c3_disc_bitwise():
    """C3: the bench's 1,000,519-node disc, MEx1, dt 0.055 tau 0.5 rho 50; 2 steps x 10 iterations
    (the first with the FD-Hessian prox and the gradient predictor)."""
    m = mx.MeshData.hexdisc(577, 0.5, 0.5, 0.5)
    assert m.nP == 1000519
    O, G = _pair(m, 1, 0.055, 0.5, 50.0)
    for s in range(2):
        ih_o = O.step(10, -1.0)[0]
        ih_g = G.step(10, -1.0)[0]
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
    _bitwise(O, G)
    assert G.stats()["bfgs_iters"] == O.bfgs_iters()


def test_c3_disc_reference_semantics():
    """C3 at the headline size against the reference's own arithmetic -- glibc pow, Jacobi-CG on the
    block-diagonal t (tol = eps), and the ADMM early exit at tol 1e-3 (src/MeshIntegrator.cpp:144-172)
    -- for 3 steps: the same ADMM iteration count every step, the same BFGS iteration total over
    2 M triangles (the L1 < 1e-5 exit of src/Mesh.cpp:850 decided alike for every one of them), and
    node positions within north_star's 1e-10 relative."""
    m = mx.MeshData.hexdisc(577, 0.5, 0.5, 0.5)
    O, G = _pair(m, 1, 0.055, 0.5, 50.0, pow_mode=0, cg_mode=0)
    for s in range(3):
        ih_o, it_o = O.step(10, 1e-3)[:2]
        ih_g, it_g = G.step(10, 1e-3)
        assert it_o == it_g, f"ADMM iteration count differs at step {s}"
        assert abs(ih_o - ih_g) <= 1e-11 * abs(ih_o)
        assert G.stats()["bfgs_iters"] == O.bfgs_iters(), f"BFGS iteration total differs after step {s}"
    xo, xg = O.get("x"), G.get("x")
    assert np.abs(xo - xg).max() / np.abs(xo).max() <= POS_TOL


def _ref_semantics_protocol(m, mon, dt, tau, rho, steps, iters):
    """The bench's protocol (early exit off: exactly `iters` ADMM iterations per step, the timed
    trajectory of bench.py) against the reference-semantics oracle (glibc pow, Jacobi-CG on the
    block-diagonal t with tol = eps; src/MeshIntegrator.cpp:144-172).  After every step: the same
    BFGS iteration total (every L1 < 1e-5 exit of src/Mesh.cpp:850 decided alike) and the maximum
    relative node-position error, which is returned per step."""
    O, G = _pair(m, mon, dt, tau, rho, pow_mode=0, cg_mode=0)
    errs = []
    for s in range(steps):
        ih_o, it_o = O.step(iters, -1.0)[:2]
        ih_g, it_g = G.step(iters, -1.0)
        assert it_o == it_g == iters
        xo, xg = O.get("x"), G.get("x")
        errs.append(float(np.abs(xo - xg).max() / np.abs(xo).max()))
        bo, bg = O.bfgs_iters(), G.stats()["bfgs_iters"]
        print(f"step {s}: max relative position error {errs[-1]:.3e}, BFGS total {bo} / {bg}", flush=True)
        assert bg == bo, f"BFGS iteration total differs after step {s}"
        assert abs(ih_o - ih_g) <= 1e-11 * abs(ih_o), f"step {s}"
    print("max relative node-position error per step:", ", ".join(f"{e:.3e}" for e in errs))
    assert errs[-1] <= POS_TOL, errs
    G.close()
    return errs


def test_c3_disc_reference_semantics_bench_protocol():
    """C3 (1,000,519 nodes) over the bench's timed protocol: 5 steps x 10 ADMM iterations, early
    exit off, glibc pow + Jacobi-CG in the oracle; <= 1e-10 relative positions after the last step."""
    m = mx.MeshData.hexdisc(577, 0.5, 0.5, 0.5)
    _ref_semantics_protocol(m, 1, 0.055, 0.5, 50.0, 5, 10)


def test_c4_cube_reference_semantics_bench_protocol():
    """C4 (512,191 nodes, 3,000,564 tetrahedra) over the bench's protocol: 2 steps x 10 ADMM
    iterations, early exit off, reference arithmetic in the oracle."""
    m = mx.MeshData.rect(3, 63)
    _ref_semantics_protocol(m, 6, 0.025, 0.5, 2000.0, 2, 10)


def test_c4_cube_reference_semantics():
    """C4 (512,191 nodes, 3,000,564 tetrahedra) at reference semantics: one step with the early exit
    on, the same ADMM and BFGS iteration counts and node positions within 1e-10 relative."""
    m = mx.MeshData.rect(3, 63)
    O, G = _pair(m, 6, 0.025, 0.5, 2000.0, pow_mode=0, cg_mode=0)
    ih_o, it_o = O.step(10, 1e-3)[:2]
    ih_g, it_g = G.step(10, 1e-3)
    assert it_o == it_g
    assert abs(ih_o - ih_g) <= 1e-11 * abs(ih_o)
    assert G.stats()["bfgs_iters"] == O.bfgs_iters()
    xo, xg = O.get("x"), G.get("x")
    assert np.abs(xo - xg).max() / np.abs(xo).max() <= POS_TOL
    G.close()


def test_c4_cube_bitwise_and_partitioned():
    """C4: 3D SquareGrid n = 63, anisotropic shell monitor (MonType 6), dt 0.025 tau 0.5 rho 2000;
    1 step x 10 iterations bit-identical to the oracle, then the same step on a two-rank
    element partition bit-identical to one GPU."""
    m = mx.MeshData.rect(3, 63)
    assert (m.nP, m.nF) == (512191, 3000564)
    O, G = _pair(m, 6, 0.025, 0.5, 2000.0)
    ih_o = O.step(10, -1.0)[0]
    ih_g = G.step(10, -1.0)[0]
    assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
    _bitwise(O, G)
    assert G.stats()["bfgs_iters"] == O.bfgs_iters()
    del O
    M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5)
    comm, parts, ih = _partitioned(M, 0.025, 2, 1, 10)
    xr = G.get("x").reshape(-1, 3)
    for r, e in enumerate(parts):
        assert np.array_equal(e.get("x").reshape(-1, 3), xr[e.local_nodes()]), f"rank {r}"
        assert abs(ih[r][0] - ih_g) <= 1e-12 * abs(ih_g)
        e.close()
    comm.close()
    G.close()


# The BFGS-heavy regime (VERDICT r4 missing #2): bench.py's `bfgs_heavy` section -- SquareGrid
# n = 707 (1,001,113 nodes, 1,999,396 triangles), MEx1 at rho 1 (a weak ADMM penalty, so the prox
# minimises the functional almost freely), dt 0.055 tau 0.5.  Every other at-size test runs at ~1.0
# BFGS iteration per simplex per prox; here the repeated rank-two updates, the c2 divisions and the
# L1 < 1e-5 exit of bfgsOptSimplex (/root/reference/src/Mesh.cpp:827-856, 850) run ~2.6-3.0 times
# per simplex per prox after the first step.
BFGS_HEAVY = dict(mon=1, dt=0.055, tau=0.5, rho=1.0)


def _bfgs_per_prox(G, before, nF, iters=10):
    return (G.stats()["bfgs_iters"] - before) / iters / nF


def test_bfgs_heavy_1m_bitwise():
    """3 steps x 10 ADMM iterations at 1 M nodes, bit-identical to the oracle (correctly rounded
    pow, exact diagonal solve): x, z, u, Bkinv after every step and equal BFGS totals; the steps
    after the first average >= 2.5 BFGS iterations per simplex per prox."""
    m = mx.MeshData.rect(2, 707)
    assert (m.nP, m.nF) == (1001113, 1999396)
    p = BFGS_HEAVY
    O, G = _pair(m, p["mon"], p["dt"], p["tau"], p["rho"])
    per = []
    for s in range(3):
        b0 = G.stats()["bfgs_iters"]
        ih_o = O.step(10, -1.0)[0]
        ih_g = G.step(10, -1.0)[0]
        per.append(_bfgs_per_prox(G, b0, m.nF))
        assert G.stats()["bfgs_iters"] == O.bfgs_iters(), f"BFGS iteration total differs after step {s}"
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o), f"step {s}"
        _bitwise(O, G)
        print(f"step {s}: bitwise, {per[-1]:.3f} BFGS iterations per simplex per prox", flush=True)
    assert sum(per[1:]) / len(per[1:]) >= 2.5, per
    assert G.stats()["max_bfgs"] >= 4, G.stats()["max_bfgs"]
    G.close()


# Relative node-position error allowed after each step of the BFGS-heavy run at reference semantics.
# This regime amplifies ulp-level differences about 10-100x per step: the oracle against ITSELF with
# only the block-diagonal solve changed (exact division instead of the reference's Jacobi-CG, both
# with glibc pow; sub-ulp differences per x-update) differs by 4.4e-16, 1.5e-14, 1.1e-10, 2.1e-10
# after steps 1-4, and with only the powers changed (correctly rounded instead of glibc's, which
# misrounds ~1 in 1,200) by 9.3e-13, 7.1e-11, 1.0e-9, 2.0e-9 (profiles/r05/bfgs_heavy_sensitivity.log).
# The GPU is bit-identical to the correctly rounded restatement (test above), so its distance to the
# reference's arithmetic is exactly the latter row: within north_star's 1e-10 for two steps, then
# the regime's own amplification.  The BFGS totals stay equal at every step.
BFGS_HEAVY_REFSEM_TOL = (1e-10, 1e-10, 1e-8)


def test_bfgs_heavy_1m_reference_semantics():
    """The same 3 steps against the reference's arithmetic (glibc pow, Jacobi-CG), early exit off:
    equal BFGS totals after every step (every L1 < 1e-5 exit of /root/reference/src/Mesh.cpp:850
    decided alike over 2 M triangles x ~3 iterations) and node positions within
    BFGS_HEAVY_REFSEM_TOL per step."""
    m = mx.MeshData.rect(2, 707)
    p = BFGS_HEAVY
    O, G = _pair(m, p["mon"], p["dt"], p["tau"], p["rho"], pow_mode=0, cg_mode=0)
    errs = []
    for s, tol in enumerate(BFGS_HEAVY_REFSEM_TOL):
        ih_o = O.step(10, -1.0)[0]
        ih_g = G.step(10, -1.0)[0]
        xo, xg = O.get("x"), G.get("x")
        errs.append(float(np.abs(xo - xg).max() / np.abs(xo).max()))
        print(f"step {s}: max relative position error {errs[-1]:.3e}", flush=True)
        assert G.stats()["bfgs_iters"] == O.bfgs_iters(), f"BFGS iteration total differs after step {s}"
        assert abs(ih_o - ih_g) <= 1e-11 * abs(ih_o), f"step {s}"
        assert errs[-1] <= tol, (s, errs)
    G.close()


def test_c5_cube_partition_equals_single():
    """C5: 3D n = 136, time-varying monitor (MonType 7, grid rebuilt on the device every step),
    dt 0.025 tau 0.5 rho 2000; 1 step x 3 iterations on one GPU and on a three-rank partition."""
    m = mx.MeshData.rect(3, 136)
    assert (m.nP, m.nF) == (5086809, 30185472)
    assert m.nF * 144 > 2 ** 32  # one GPU: Bkinv offsets beyond 32 bits
    assert (m.nF // 3 + 64) * 144 < 2 ** 31  # partition: every rank's offsets within 31 bits
    M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 7), rho=2000.0, tau=0.5)
    G = mx.Engine(M, 0.025)
    G.set_regrid(True)
    e0 = G.energy()
    ih_g, it_g = G.step(3, -1.0)
    assert it_g == 3 and np.isfinite(ih_g) and np.isfinite(e0)
    st = G.stats()
    assert st["regrids"] == 1 and st["steps"] == 1
    assert st["bfgs_iters"] > 0
    xg = G.get("x").reshape(-1, 3)
    assert np.isfinite(xg).all()
    assert np.isfinite(G.energy())
    G.close()
    comm, parts, ih = _partitioned(M, 0.025, 3, 1, 3, regrid=True)
    for r, e in enumerate(parts):
        assert np.array_equal(e.get("x").reshape(-1, 3), xg[e.local_nodes()]), f"rank {r}"
        assert abs(ih[r][0] - ih_g) <= 1e-12 * abs(ih_g)
        e.close()
    comm.close()
