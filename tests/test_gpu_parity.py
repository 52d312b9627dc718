"""GPU (libmmadmm, HIP on MI355X) against the CPU oracle, through the C-ABI.

Two bars:
  * bit-for-bit: oracle with correctly rounded pow and the exact block-diagonal solve (the
    arithmetic the kernels implement) -- x, z, u and Bkinv must be identical after several
    steps with fixed ADMM iteration counts;
  * reference semantics: oracle with glibc pow and Eigen's Jacobi-CG solve -- relative node
    position error <= 1e-10 (north-star tolerance), energies <= 1e-12.
"""
import os

import numpy as np
import pytest

import mmadmm_amd as mx
import oracle_py
from conftest import GOLDEN, circle_mesh

pytestmark = pytest.mark.gpu

POS_TOL = 1e-10


@pytest.fixture(autouse=True)
def _pow_mode_reset():
    yield
    oracle_py.set_pow_mode(0)


def cases():
    return {
        "C1_circle24_mex5": (lambda: circle_mesh("CircleEx24"), 5, 0.05, 0.1, 5.0, False),
        "rect10_mex3": (lambda: oracle_py.Mesh.rect(2, 10), 3, 0.025, 0.5, 1000.0, False),
        "rect16_mex2": (lambda: oracle_py.Mesh.rect(2, 16), 2, 0.025, 0.5, 100.0, False),
        "hexdisc12_mex1": (lambda: _hexdisc(12), 1, 0.055, 0.5, 50.0, False),
        "rect3d_3_mex1": (lambda: oracle_py.Mesh.rect(3, 3), 1, 0.025, 0.5, 50.0, False),
        "rect3d_4_aniso6": (lambda: oracle_py.Mesh.rect(3, 4), 6, 0.025, 0.5, 50.0, False),
        "circle3d6_compmesh": (lambda: circle_mesh("3DCircleEx6"), 5, 0.1, 0.1, 0.5, True),
    }


def _hexdisc(N):
    m = mx.MeshData.hexdisc(N)
    return oracle_py.Mesh(2, m.Xp, m.F, m.mask)


def make_pair(mesh, mon, dt, tau, rho, comp, pow_mode, cg_mode, gradUse=False):
    oracle_py.set_pow_mode(pow_mode)
    Vc = mesh.Vp.copy() if comp else None
    O = oracle_py.Integrator(mesh, mon, dt, tau, rho, gradUse=gradUse, Vc=Vc, cgMode=cg_mode)
    M = mx.Mesh(mesh.Vp, mesh.F, mesh.mask, mx.BuiltinMonitor(mesh.dim, mon), rho=rho, tau=tau,
                gradUse=gradUse, Xc=Vc)
    G = mx.Engine(M, dt)
    return O, G


def test_devmath_correctly_rounded():
    rng = np.random.default_rng(1)
    x = np.exp(rng.uniform(-30, 30, 200000))
    np.testing.assert_array_equal(mx.devmath(0, x), np.sqrt(x))
    sub = x[:4000]
    for op, y in ((1, 1.5), (2, -0.5), (3, 2.25), (4, 1.25)):
        ref = np.array([oracle_py.crpow(v, y) for v in sub])
        np.testing.assert_array_equal(mx.devmath(op, sub), ref)


def _near_midpoint_args(rng):
    """arguments whose powers sit close to rounding midpoints: a few ulps from 1 and from perfect
    powers (x = k^4, k^2), plus random ones"""
    one = 1.0 + np.arange(-64, 65) * 2.0 ** -52
    k = np.arange(1.0, 3000.0)
    pp = np.concatenate([k ** 2, k ** 4, (k + 0.5) ** 2])
    pp = np.concatenate([np.nextafter(pp, 0), pp, np.nextafter(pp, np.inf)])
    return np.concatenate([one, pp, np.exp(rng.uniform(-20, 20, 6000))])


def test_devmath_fast_path_correct_or_deferred():
    """The prox kernels' fast powers (EXACT = false, with the library's double-double, MMX_DD_FAST
    or not) either return the correctly rounded power or defer (NaN here) to the exact path --
    never a wrong rounding -- and defer rarely on random arguments."""
    rng = np.random.default_rng(7)
    x = _near_midpoint_args(rng)
    for op, y in ((6, 1.5), (7, -0.5), (8, 2.25), (9, 1.25)):
        got = mx.devmath(op, x)
        ref = np.array([oracle_py.crpow(v, y) for v in x])
        ok = ~np.isnan(got)
        np.testing.assert_array_equal(got[ok], ref[ok])
        assert np.isnan(got[-6000:]).mean() < 1e-3, (op, np.isnan(got[-6000:]).mean())


def test_devmath_dd_sqrt_error_bound():
    """The double-double sqrt behind the powers: |s + e - sqrt(x)| < 2^-98 |sqrt(x)| (crmath.h;
    the rounding decision needs 2^-95), checked in 60-digit decimal arithmetic."""
    from decimal import Decimal, getcontext

    getcontext().prec = 60
    rng = np.random.default_rng(11)
    x = np.concatenate([np.exp(rng.uniform(-60, 60, 1500)), 1.0 + np.arange(-200, 200) * 2.0 ** -52])
    out = mx.devmath(10, np.concatenate([x, np.zeros_like(x)]))
    worst = 0.0
    for i, v in enumerate(x):
        s, e = out[2 * i], out[2 * i + 1]
        t = Decimal(float(v)).sqrt()
        err = abs((Decimal(float(s)) + Decimal(float(e)) - t) / t)
        worst = max(worst, float(err))
    assert worst < 2.0 ** -98, worst


@pytest.mark.parametrize("name", list(cases()))
def test_setup_identical(name):
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    O, G = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    np.testing.assert_array_equal(G.get("grid"), O.get("grid"))
    np.testing.assert_array_equal(G.simplices(), O.F())
    np.testing.assert_array_equal(G.get("Ehat"), O.get("Ehat"))
    np.testing.assert_array_equal(G.get("x"), O.get("x"))
    np.testing.assert_array_equal(G.get("z"), O.get("z"))
    e_o, e_g = O.energy(), G.energy()
    assert abs(e_o - e_g) <= 1e-13 * abs(e_o)


@pytest.mark.parametrize("name", list(cases()))
def test_steps_bitwise(name):
    """Fixed iteration counts, cr pow, exact diagonal solve: bit-identical device state."""
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    O, G = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    # 2D: 6 steps, so the predictor fused into the first x-update (steps after the third) runs three
    # times and its xPrev / xBar writes are read by later steps' extrapolations
    nsteps = 6 if mesh.dim == 2 else 3
    for s in range(nsteps):
        ih_o = O.step(5, -1.0)[0]
        ih_g = G.step(5, -1.0)[0]
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
        for f in ("x", "z", "u", "xBar", "xPrev"):
            np.testing.assert_array_equal(G.get(f), O.get(f), err_msg=f"{f} step {s}")
    np.testing.assert_array_equal(G.get("hess"), O.get("hess"))
    assert G.stats()["bfgs_iters"] == O.bfgs_iters()


@pytest.mark.parametrize("name", ["hexdisc12_mex1", "rect16_mex2", "C1_circle24_mex5", "rect3d_3_mex1", "circle3d6_compmesh"])
def test_exact_recompute_path_bitwise(name, monkeypatch):
    """The steady-state prox skips cr_resolve; a block whose powers come near a rounding midpoint
    is recomputed exactly by k_prox_fix.  MMX_FORCE_TIE=2 sends every second block down that path:
    the state and the energies (same partial-sum trees) must not change by a bit."""
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    O, G = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    monkeypatch.setenv("MMX_FORCE_TIE", "2")
    _, Gt = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    monkeypatch.delenv("MMX_FORCE_TIE")
    for s in range(3):
        ih_o = O.step(5, -1.0)[0]
        ih_g = G.step(5, -1.0)[0]
        ih_t = Gt.step(5, -1.0)[0]
        assert ih_t == ih_g
        for f in ("x", "z", "u"):
            np.testing.assert_array_equal(Gt.get(f), O.get(f), err_msg=f"{f} step {s}")
    np.testing.assert_array_equal(Gt.get("hess"), O.get("hess"))
    np.testing.assert_array_equal(Gt.get("hess"), G.get("hess"))
    assert Gt.stats()["bfgs_iters"] == O.bfgs_iters()


@pytest.mark.parametrize("name", list(cases()))
def test_steps_reference_semantics(name):
    """glibc pow + Eigen Jacobi-CG (the reference's arithmetic): <= 1e-10 node positions."""
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    O, G = make_pair(mesh, mon, dt, tau, rho, comp, 0, 0)
    for s in range(5):
        ih_o, it_o = O.step(10, 1e-3)[:2]
        ih_g, it_g = G.step(10, 1e-3)
        assert it_o == it_g, f"ADMM iteration count differs at step {s}"
        assert abs(ih_o - ih_g) <= 1e-11 * abs(ih_o)
    xo, xg = O.get("x"), G.get("x")
    err = np.abs(xo - xg).max() / np.abs(xo).max()
    assert err <= POS_TOL, err


def test_euler_step_parity():
    mesh = oracle_py.Mesh.rect(2, 12)
    O, G = make_pair(mesh, 3, 0.025, 0.5, 1000.0, False, 1, 1)
    for _ in range(3):
        a, b = O.euler_step(), G.euler_step()
        assert abs(a - b) <= 1e-12 * abs(a)
        np.testing.assert_array_equal(G.get("x"), O.get("x"))


def test_grad_use_predictor():
    mesh = oracle_py.Mesh.rect(2, 8)
    O, G = make_pair(mesh, 4, 0.005, 0.1, 50.0, False, 1, 1, gradUse=True)
    for _ in range(4):
        O.step(3, -1.0)
        G.step(3, -1.0)
    np.testing.assert_array_equal(G.get("x"), O.get("x"))


def test_inverted_element_reported():
    """The reference aborts on assert(Edet > 0); the engine returns MMADMM_ERR_INVERTED."""
    mesh = oracle_py.Mesh.levelset2d(40, compact_mask=False)  # reference quirk: all-FIXED simplices
    M = mx.Mesh(mesh.Vp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5)
    G = mx.Engine(M, 0.055)
    with pytest.raises(mx.InvertedElementError):
        for _ in range(3):
            G.step(10, -1.0)


class _HalfNanMonitor(mx.MonitorFunction):
    """identity left of x = 0.6, NaN right of it: a monitor value that is not finite"""
    dim = 2

    def __call__(self, x, M):
        M[:] = np.nan if x[0] > 0.6 else np.eye(2)


def test_nonfinite_monitor_reported_not_as_inverted():
    """A non-finite monitor value with no inverted element: MMADMM_ERR_NONFINITE
    (NonFiniteEnergyError), not MMADMM_ERR_INVERTED (every reporting operation starts from a clear
    inverted flag)."""
    mesh = mx.MeshData.rect(2, 12)
    G = mx.Engine(mx.Mesh(mesh.Xp, mesh.F, mesh.mask, _HalfNanMonitor(), rho=50.0, tau=0.5), 0.055)
    assert np.isnan(G.energy())  # NaN monitor values: energy is NaN, no element inverted
    with pytest.raises(mx.NonFiniteEnergyError):
        G.step(5, -1.0)
    G.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_division_by_reciprocal_is_correctly_rounded(seed):
    """div_mk (crmath.h): RN(x/c) from RN(1/c) + one FMA correction, used for the BFGS update's
    2 K^2 divisions by c2 in the fast prox kernels -- bit-identical to IEEE division inside the
    ranges the kernels check (c in [2^-100, 2^100], c > 0; x = +-0 or |x| in [2^-900, 2^900]) on
    random, wide-range and near-midpoint quotients, signed zeros included."""
    import mmadmm_amd as mx
    rng = np.random.default_rng(seed)
    n = 1 << 21
    c = rng.uniform(1, 2, n) * np.exp2(rng.integers(-100, 100, n))
    c[: n // 4] = rng.uniform(1e-12, 1e-3, n // 4)  # c2 = p.y magnitudes of the prox
    x = rng.uniform(-2, 2, n) * np.exp2(rng.integers(-899, 899, n))
    # near-midpoint quotients: x = RN(c * (q + ulp(q)/2 * (1 + tiny)))
    q = rng.uniform(1, 2, n // 4) * np.exp2(rng.integers(-600, 600, n // 4))
    half = np.spacing(q) / 2
    sl = slice(n // 2, n // 2 + n // 4)
    x[sl] = c[sl] * (q + half * (1 + rng.uniform(-1e-6, 1e-6, n // 4)))
    ok = (np.abs(x) >= 2.0 ** -900) & (np.abs(x) <= 2.0 ** 900)
    x[~ok] = 1.0
    x[-1000:] = 0.0
    x[-500:] = -0.0
    pairs = np.empty(2 * n)
    pairs[0::2], pairs[1::2] = x, c
    out = mx.devmath(5, pairs)[:n]
    ref = x / c
    assert np.array_equal(out.view(np.int64), ref.view(np.int64))


@pytest.mark.parametrize("dim,tol", [(2, -1.0), (2, 1e-3), (3, -1.0)])
def test_long_run_bitwise(dim, tol):
    """Many steps on a mid-size mesh: no drift between the device and the oracle.

    tol < 0 runs the deferred-reduction path (one k_reduce_steps per step), tol > 0 the
    per-iteration early-exit check (reference MeshIntegrator::step, early exit on
    ||x - z|| / ||z - zPrev|| < tol). The meshes move by ~1e-2 over the run."""
    if dim == 2:
        mesh, mon, rho, nsteps = _hexdisc(40), 2, 100.0, 20
    else:
        mesh, mon, rho, nsteps = oracle_py.Mesh.rect(3, 10), 6, 2000.0, 8
    O, G = make_pair(mesh, mon, 0.025, 0.5, rho, False, 1, 1)
    for _ in range(nsteps):
        O.step(5, tol)
        G.step(5, tol)
    np.testing.assert_array_equal(G.get("x"), O.get("x"))
    np.testing.assert_array_equal(G.get("z"), O.get("z"))


@pytest.mark.parametrize("dim,ts", [(2, "1"), (3, "0")])
def test_xupdate_slot_terms_bitwise(dim, ts, monkeypatch):
    """The x-update from the prox's slot terms w(w(z - u)) (DeviceMesh::tslot, on by default in
    3D) and from z and u (the 2D default) give the same bits as the oracle: each engine is run
    with the other choice forced (MMX_TSLOT)."""
    monkeypatch.setenv("MMX_TSLOT", ts)
    if dim == 2:
        mesh, mon, rho = _hexdisc(30), 2, 100.0
    else:
        mesh, mon, rho = oracle_py.Mesh.rect(3, 8), 6, 2000.0
    O, G = make_pair(mesh, mon, 0.025, 0.5, rho, False, 1, 1)
    for tol in (-1.0, 1e-3, -1.0):
        O.step(5, tol)
        G.step(5, tol)
    np.testing.assert_array_equal(G.get("x"), O.get("x"))
    np.testing.assert_array_equal(G.get("z"), O.get("z"))


@pytest.mark.parametrize("name", ["rect3d_3_mex1", "circle3d6_compmesh"])
@pytest.mark.parametrize("force_tie", [0, 2])
def test_quad_lane_prox_bitwise(name, force_tie, monkeypatch):
    """The cooperative 3D prox (k_prox_quad, four lanes per tetrahedron, MMX_PROX3D=quad) against
    the oracle bit for bit, alone and with every second block sent down its exact instance
    (MMX_FORCE_TIE=2), which strides over the tie queue with a grid of workgroups."""
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    monkeypatch.setenv("MMX_PROX3D", "quad")
    if force_tie:
        monkeypatch.setenv("MMX_FORCE_TIE", str(force_tie))
    O, G = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    for s in range(3):
        ih_o = O.step(5, -1.0)[0]
        ih_g = G.step(5, -1.0)[0]
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
        for f in ("x", "z", "u"):
            np.testing.assert_array_equal(G.get(f), O.get(f), err_msg=f"{f} step {s}")
    np.testing.assert_array_equal(G.get("hess"), O.get("hess"))
    assert G.stats()["bfgs_iters"] == O.bfgs_iters()


def test_quad_lane_prox_equals_wave_at_c4(monkeypatch):
    """C4 (3,000,564 tets): one step of 10 iterations with k_prox_quad equals k_prox_wave bit for
    bit (state and Bkinv), with and without forced exact recomputation of every 7th block."""
    m = mx.MeshData.rect(3, 63)
    M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5)
    W = mx.Engine(M, 0.025)
    W.step(10, -1.0)
    W.step(10, -1.0)
    monkeypatch.setenv("MMX_PROX3D", "quad")
    monkeypatch.setenv("MMX_FORCE_TIE", "7")
    Q = mx.Engine(M, 0.025)
    Q.step(10, -1.0)
    Q.step(10, -1.0)
    for f in ("x", "z", "u", "hess"):
        np.testing.assert_array_equal(Q.get(f), W.get(f), err_msg=f)
    assert Q.stats()["bfgs_iters"] == W.stats()["bfgs_iters"]
    W.close()
    Q.close()


@pytest.mark.parametrize("name", ["C1_circle24_mex5", "hexdisc12_mex1"])
@pytest.mark.parametrize("force_tie", [0, 2])
def test_prox2d_wave_bitwise(name, force_tie, monkeypatch):
    """The 2D prox through k_prox_wave<2> (MMX_PROX2D=wave: one wave per workgroup, all six Bkinv
    rows held in LDS, Bkinv double-buffered) against the oracle bit for bit, alone and with every
    second block sent down its exact instance (MMX_FORCE_TIE=2)."""
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    monkeypatch.setenv("MMX_PROX2D", "wave")
    if force_tie:
        monkeypatch.setenv("MMX_FORCE_TIE", str(force_tie))
    O, G = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    for s in range(3):
        ih_o = O.step(5, -1.0)[0]
        ih_g = G.step(5, -1.0)[0]
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
        for f in ("x", "z", "u"):
            np.testing.assert_array_equal(G.get(f), O.get(f), err_msg=f"{f} step {s}")
    np.testing.assert_array_equal(G.get("hess"), O.get("hess"))
    assert G.stats()["bfgs_iters"] == O.bfgs_iters()


@pytest.mark.parametrize("order,sweep", [(0, 0), (1, 0), (0, 2), (1, 4)])
def test_xupdate_order_and_sweep_bitwise(order, sweep, monkeypatch):
    """The 3D slot-term x-update in its forms -- nodes by first incident simplex (order 0) or in eight
    y slabs, one per XCD group (order 1, the default); one node per lane (sweep 0) or walked as a
    per-XCD sweep by a persistent grid of `sweep` workgroups per CU (default 1) -- sums every
    node's slots in the same ascending order: positions bit-identical to the default."""
    m = mx.MeshData.rect(3, 24)
    M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 6), rho=2000.0, tau=0.5)
    W = mx.Engine(M, 0.025)
    W.step(10, -1.0)
    W.step(10, -1.0)
    monkeypatch.setenv("MMX_XUP_ORDER", str(order))
    monkeypatch.setenv("MMX_XUP_SWEEP", str(sweep))
    Q = mx.Engine(M, 0.025)
    Q.step(10, -1.0)
    Q.step(10, -1.0)
    for f in ("x", "z", "u"):
        np.testing.assert_array_equal(Q.get(f), W.get(f), err_msg=f)
    W.close()
    Q.close()


@pytest.mark.parametrize("order,sweep", [(1, 0), (0, 1), (1, 1), (1, 2)])
def test_xupdate_order_and_sweep_bitwise_2d(order, sweep, monkeypatch):
    """The 2D x-update (z and u gathered) in the same forms (opt-in in 2D): bit-identical."""
    m = mx.MeshData.hexdisc(60, 0.5, 0.5, 0.5)
    M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5)
    W = mx.Engine(M, 0.055)
    W.step(10, -1.0)
    W.step(10, -1.0)
    monkeypatch.setenv("MMX_XUP_ORDER", str(order))
    monkeypatch.setenv("MMX_XUP_SWEEP", str(sweep))
    Q = mx.Engine(M, 0.055)
    Q.step(10, -1.0)
    Q.step(10, -1.0)
    for f in ("x", "z", "u"):
        np.testing.assert_array_equal(Q.get(f), W.get(f), err_msg=f)
    W.close()
    Q.close()


ISO_CASES = {  # mesh, MonType, dt, tau, rho, isotropic grid
    "hexdisc40_mex1": (lambda: mx.MeshData.hexdisc(40), 1, 0.055, 0.5, 50.0, 1),
    "rect30_mex3": (lambda: mx.MeshData.rect(2, 30), 3, 0.025, 0.5, 1000.0, 1),
    "rect30_mex2": (lambda: mx.MeshData.rect(2, 30), 2, 0.025, 0.5, 100.0, 0),
    "hexdisc40_movingbump": (lambda: mx.MeshData.hexdisc(40), 7, 0.05, 0.5, 50.0, 1),
    "rect3d_8_mex1": (lambda: mx.MeshData.rect(3, 8), 1, 0.025, 0.5, 50.0, 1),
    "rect3d_8_aniso6": (lambda: mx.MeshData.rect(3, 8), 6, 0.025, 0.5, 50.0, 0),
    "rect3d_8_movingbump": (lambda: mx.MeshData.rect(3, 8), 7, 0.025, 0.5, 2000.0, 1),
}


@pytest.mark.parametrize("name", list(ISO_CASES))
def test_isotropic_grid_path_bitwise(name, monkeypatch):
    """An isotropic monitor grid (every point s I bit for bit) is kept as one value per point and
    interpolated from it (evalMonitor, engine.cpp updateIso): the state after 3 steps x 5 ADMM iterations equals the full-row path (MMX_ISO=0) bit
    for bit, in 2D and 3D (the first prox's FD Hessian, the steady 3D prox and its exact
    recomputation are separate isotropic instances there); MEx2 and MonType 6 are anisotropic and keep
    the full rows; MonType 7 is rebuilt on the device every step and stays isotropic."""
    mk, mon, dt, tau, rho, iso = ISO_CASES[name]
    mesh = mk()
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("MMX_ISO", flag)
        M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(mesh.dim, mon), rho=rho, tau=tau)
        G = mx.Engine(M, dt)
        if mon == 7:
            G.set_regrid(True)
        for _ in range(3):
            G.step(5, -1.0)
        out[flag] = (G.stats()["monitor_iso"], G.get("x"), G.get("z"), G.get("u"), G.get("hess"))
        G.close()
    assert out["0"][0] == 0 and out["1"][0] == iso
    for a, b in zip(out["0"][1:], out["1"][1:]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("knob", ["MMX_ZX", "MMX_FUSE_PRED"])
@pytest.mark.parametrize("name", ["hexdisc12_mex1", "rect16_mex2"])
def test_step_start_fusions_ab_bitwise(name, knob, monkeypatch):
    """The 2D step start: z taken from the positions (DeviceMesh::zx, no k_gather_z) and
    predictX fused into the first x-update, against new engines with each turned off -- x, xPrev,
    xBar, z, u bit-identical over 6 steps (the fused predictor runs from the fourth)."""
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    _, G = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    monkeypatch.setenv(knob, "0")
    _, Gk = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    monkeypatch.delenv(knob)
    for s in range(6):
        assert G.step(5, -1.0)[0] == Gk.step(5, -1.0)[0]
        for f in ("x", "xPrev", "xBar", "z", "u"):
            np.testing.assert_array_equal(G.get(f), Gk.get(f), err_msg=f"{knob}=0: {f} step {s}")


@pytest.mark.parametrize("name", ["hexdisc12_mex1", "rect3d_3_mex1"])
def test_split_reductions_small_mesh(name, monkeypatch):
    """The two-launch reductions (k_reduce_split + k_reduce_combine into the mapped pinned results)
    normally run only at >= 4096 partial rows, i.e. at the at-size meshes.
    MMX_RED_SPLIT_MIN=1 forces them on a small mesh: the energies and BFGS totals must equal the
    oracle's and the one-workgroup path's, and repeated runs must be bit-identical."""
    mk, mon, dt, tau, rho, comp = cases()[name]
    mesh = mk()
    O, G = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    monkeypatch.setenv("MMX_RED_SPLIT_MIN", "1")
    _, Gs = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    _, Gs2 = make_pair(mesh, mon, dt, tau, rho, comp, 1, 1)
    for s in range(3):
        for tol in (-1.0, 1e-3):  # the deferred whole-step reduction and the per-iteration one
            ih_o, it_o = O.step(5, tol)[:2]
            ih_g, it_g = G.step(5, tol)
            ih_s, it_s = Gs.step(5, tol)
            ih_s2, it_s2 = Gs2.step(5, tol)
            assert it_s == it_g == it_o and ih_s == ih_s2
            assert abs(ih_s - ih_o) <= 1e-12 * abs(ih_o) and abs(ih_s - ih_g) <= 1e-12 * abs(ih_g)
    np.testing.assert_array_equal(Gs.get("x"), O.get("x"))
    assert Gs.stats()["bfgs_iters"] == O.bfgs_iters() == Gs2.stats()["bfgs_iters"]
    assert Gs.stats()["last_primal"] == Gs2.stats()["last_primal"]
