"""Backward Euler (method 2, Mesh::backwardsEulerStep, src/Mesh.cpp:1263-1341) on the GPU.

Three bars, as for the ADMM step:
  * the FD Jacobian (buildEulerJac + FSubJac, src/Mesh.cpp:1112-1261) is bit-identical to the
    oracle's (correctly rounded pow, the arithmetic the kernels implement);
  * whole Newton steps are bit-identical to the oracle run with the GPU's CG-STAB summation order
    (tree=True, oracle/lasolver.cpp dotMode 1): x after every step, equal Newton counts;
  * reference semantics: the energy traces of the reference's own method-2 runs
    (Experiments/Results/*/Ih2.txt) to their 6 printed digits and step counts.
"""
import os

import numpy as np
import pytest

import mmadmm_amd as mx
import oracle_py
from conftest import GOLDEN, circle_mesh
from test_gpu_parity import make_pair

pytestmark = pytest.mark.gpu

SIX_DIGITS = 6e-6


@pytest.fixture(autouse=True)
def _pow_mode_reset():
    yield
    oracle_py.set_pow_mode(0)


CASES = {
    "rect12_mex3": (lambda: oracle_py.Mesh.rect(2, 12), 3, 0.025, 0.5, 100.0, False),
    "circle12_mex5": (lambda: circle_mesh("CircleEx12"), 5, 0.05, 0.1, 5.0, False),
    "rect3d_4_mex3": (lambda: oracle_py.Mesh.rect(3, 4), 3, 0.025, 0.5, 50.0, False),
    "circle3d6_compmesh": (lambda: circle_mesh("3DCircleEx6"), 5, 0.1, 0.1, 0.5, True),
}


@pytest.mark.parametrize("name", list(CASES))
def test_jacobian_bitwise(name):
    mk, mon, dt, tau, rho, comp = CASES[name]
    O, G = make_pair(mk(), mon, dt, tau, rho, comp, 1, 1)
    O.backwards_euler_step(dt, 1e-3, tree=True)
    G.backwards_euler_step(dt, 1e-3)
    ia_o, ja_o, a_o = O.jacobian()
    ia_g, ja_g, a_g = G.jacobian()
    np.testing.assert_array_equal(ia_g, ia_o)
    np.testing.assert_array_equal(ja_g, ja_o)
    np.testing.assert_array_equal(a_g, a_o)
    # +0.0 adds of the reference: no -0.0 survives in the assembled values
    assert not np.any((a_g == 0) & np.signbit(a_g))


@pytest.mark.parametrize("name", list(CASES))
def test_newton_steps_bitwise(name):
    mk, mon, dt, tau, rho, comp = CASES[name]
    O, G = make_pair(mk(), mon, dt, tau, rho, comp, 1, 1)
    for s in range(5):
        if s == 3:  # done() moves Vp: the next Jacobian is a new one (and rebuilt on the GPU)
            O.done()
            G.done()
            np.testing.assert_array_equal(G.get("points"), O.get("points"))
        ih_o, n_o = O.backwards_euler_step(dt, 1e-3, tree=True)
        ih_g, n_g = G.backwards_euler_step(dt, 1e-3)
        assert n_o == n_g, f"Newton iterations differ at step {s}"
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
        np.testing.assert_array_equal(G.get("x"), O.get("x"), err_msg=f"x step {s}")
    st = G.stats()
    assert st["newton_iters"] >= 5 and st["jacobians"] >= 1
    ia_o, ja_o, a_o = O.jacobian()
    np.testing.assert_array_equal(G.jacobian()[2], a_o)


# (golden, mesh, MonType, dt, tau, rho, DtTol, nSteps) from Experiments/InputFiles/*.json
BE_TRACES = [
    ("Monitor220", lambda: oracle_py.Mesh.rect(2, 20), 3, 0.025, 0.5, 100, 1e-4, 1000),
    ("Monitor320", lambda: circle_mesh("CircleEx12"), 5, 0.05, 0.1, 5, 1e-5, 10000),
    ("3DMonitor210", lambda: oracle_py.Mesh.rect(3, 10), 3, 0.025, 0.5, 50, 1e-5, 100),
]


@pytest.mark.parametrize("cfg", BE_TRACES, ids=[t[0] for t in BE_TRACES])
def test_reference_ih2_trace(cfg):
    name, mk, mon, dt, tau, rho, dtTol, nSteps = cfg
    mesh = mk()
    M = mx.Mesh(mesh.Vp, mesh.F, mesh.mask, mx.BuiltinMonitor(mesh.dim, mon), rho=rho, tau=tau)
    I = mx.MeshIntegrator(dt, M)
    ours = [I.getEnergy()]
    prev = np.inf
    for i in range(nSteps):  # runAlgo's time loop (main.cpp:172-211), method 2
        Ih = I.backwardsEulerStep(dt, 1e-3)
        ours.append(Ih)
        if i != 0 and abs((Ih - prev) / dt) < dtTol:
            break
        prev = Ih
    ref = np.loadtxt(os.path.join(GOLDEN, name, "Ih2.txt"), delimiter=",")[:, 1]
    assert len(ours) == len(ref), "number of time steps differs"
    rel = np.abs(np.array(ours) - ref) / np.abs(ref)
    assert rel.max() < SIX_DIGITS, rel.max()


def test_argument_and_partition_errors():
    mesh = oracle_py.Mesh.rect(2, 6)
    M = mx.Mesh(mesh.Vp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 3), rho=100.0, tau=0.5)
    G = mx.Engine(M, 0.025)
    with pytest.raises(mx.MMADMMError):
        G.backwards_euler_step(-1.0)
    with pytest.raises(mx.MMADMMError):  # no Jacobian before the first step
        G.jacobian()
    comm = mx.Comm.loopback(2)
    P = mx.Engine(M, 0.025, rank=0, nranks=2, comm=comm)
    with pytest.raises(mx.MMADMMError, match="one rank"):
        P.backwards_euler_step(0.025)
    P.close()
    comm.close()


def test_backward_euler_at_bench_size_bitwise():
    """The bench's method-2 workload (SquareGrid n = 707: 1,001,113 nodes, 2,002,226 unknowns,
    MEx3, dt 0.025 tau 0.5 rho 100): two backward-Euler steps bit-identical to the oracle run with
    the GPU's CG-STAB summation order -- the FD Jacobian, the Newton counts and x after each step --
    so the size-dependent parts of the method-2 path (Jacobian assembly, the n = 2 M factor and
    chain sweeps) meet the restatement at the size the bench times."""
    m = mx.MeshData.rect(2, 707)
    assert m.nP == 1001113
    om = oracle_py.Mesh(2, m.Xp, m.F, m.mask)
    O, G = make_pair(om, 3, 0.025, 0.5, 100.0, False, 1, 1)
    for s in range(2):
        ih_o, n_o = O.backwards_euler_step(0.025, 1e-3, tree=True)
        ih_g, n_g = G.backwards_euler_step(0.025, 1e-3)
        assert n_o == n_g, f"Newton iterations differ at step {s}"
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
        np.testing.assert_array_equal(G.get("x"), O.get("x"), err_msg=f"x step {s}")
    np.testing.assert_array_equal(G.jacobian()[2], O.jacobian()[2])
    G.close()


@pytest.mark.parametrize("dim,n,mon,loose", [(2, 60, 3, 0), (3, 14, 6, 0), (3, 12, 7, 0), (2, 20, 3, 2), (3, 6, 6, 1)])
def test_fd_jac_fast_path_and_assembly_variants_bitwise(dim, n, mon, loose, monkeypatch):
    """Round 6: the FD derivative blocks as a fast pass (no exact tie decision, no scratch) plus the
    exact recomputation of the lanes it queues, and the Jacobian assembled one wavefront per node,
    against the one-pass exact kernel (MMX_FDJ_FAST=0) and the entry-outer assembly
    (MMX_JAC_ASSEMBLE=entry): the Jacobian and two Newton steps bit-identical.  Regular meshes (the
    exact path is common there) with the anisotropic (6) and isotropic (7) 3D monitors; `loose`
    nodes that no simplex references (as the Shoulder meshes have: their Jacobian rows hold only the
    diagonal) inserted at the front of the numbering and appended at its end."""
    mesh = mx.MeshData.rect(dim, n)
    Xp, F, mask = mesh.Xp, mesh.F, mesh.mask
    if loose:
        c = Xp.mean(axis=0, keepdims=True)
        Xp = np.vstack([c] * loose + [Xp, c])
        F = F + loose
        mask = np.concatenate([mask[:1]] * loose + [mask, mask[:1]])
    rho = 2000.0 if dim == 3 else 100.0

    def run():
        M = mx.Mesh(Xp, F, mask, mx.BuiltinMonitor(dim, mon), rho=rho, tau=0.5)
        E = mx.Engine(M, 0.025)
        E.backwards_euler_step(0.025)
        jac = E.jacobian()[2].copy()
        E.backwards_euler_step(0.025)
        x = E.get("x").copy()
        E.close()
        return jac, x

    jac, x = run()
    monkeypatch.setenv("MMX_FDJ_FAST", "0")
    monkeypatch.setenv("MMX_JAC_ASSEMBLE", "entry")
    jac0, x0 = run()
    np.testing.assert_array_equal(jac, jac0)
    np.testing.assert_array_equal(x, x0)
