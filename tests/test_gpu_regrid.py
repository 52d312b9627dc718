"""Time-varying monitors on the device: the monitor grid rebuilt from the current mesh
at every step start (the reference's commented Mesh::setUp hook, src/Mesh.cpp:1006-1014), against
the oracle doing the same on the CPU (tests/test_regrid_oracle.py).  Bit-for-bit: the device
bounding box, nearest-vertex search and smoothing reproduce the host set-up exactly."""
import numpy as np
import pytest

import mmadmm_amd as mx
import oracle_py

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _pow_mode():
    oracle_py.set_pow_mode(1)  # correctly rounded pow: the kernels' arithmetic
    yield
    oracle_py.set_pow_mode(0)


def pair(mesh, mon, dt, tau, rho):
    O = oracle_py.Integrator(mesh, mon, dt, tau, rho, cgMode=1, regrid=True)
    M = mx.Mesh(mesh.Vp, mesh.F, mesh.mask, mx.BuiltinMonitor(mesh.dim, mon), rho=rho, tau=tau)
    G = mx.Engine(M, dt)
    G.set_regrid(True)
    return O, G


@pytest.mark.parametrize("dim,n,mon", [(2, 14, 7), (2, 14, 1), (3, 4, 7), (3, 4, 3)])
def test_regrid_each_step_bitwise(dim, n, mon):
    """MonType 7 moves with t (device-evaluated); 1 and 3 are static (host callback at the moved
    vertices).  Grid, positions and energies identical to the oracle at every step."""
    mesh = oracle_py.Mesh.rect(dim, n)
    O, G = pair(mesh, mon, 0.05, 0.5, 200.0)
    for s in range(4):
        ih_o = O.step(5, -1.0)[0]
        ih_g = G.step(5, -1.0)[0]
        np.testing.assert_array_equal(G.get("grid"), O.get("grid"), err_msg=f"grid step {s}")
        for f in ("x", "z", "u"):
            np.testing.assert_array_equal(G.get(f), O.get(f), err_msg=f"{f} step {s}")
        assert abs(ih_o - ih_g) <= 1e-12 * abs(ih_o)
    assert G.stats()["regrids"] == 4


@pytest.mark.parametrize("dim,maker", [(2, lambda: mx.MeshData.hexdisc(20)), (2, lambda: mx.MeshData.rect(2, 31)),
                                       (3, lambda: mx.MeshData.rect(3, 7))])
def test_regrid_at_setup_positions_equals_host_setup(dim, maker):
    """A rebuild at t = 0 on the unmoved mesh reproduces the host set-up grid bit for bit (the
    device nearest-vertex search, ties to the lowest vertex id, and the smoothing)."""
    m = maker()
    for mon in (1, 3, 7):
        M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(dim, mon), rho=100.0, tau=0.5)
        G = mx.Engine(M, 0.025)
        host = G.get("grid").copy()
        G.regrid(0.0)
        np.testing.assert_array_equal(G.get("grid"), host)
        G.close()


@pytest.mark.parametrize("dim,n,nsteps", [(2, 40, 20), (3, 8, 10)])
def test_regrid_long_run_bitwise(dim, n, nsteps):
    """The moving bump (MonType 7) over a full revolution (t = 0 .. 1 at dt 0.05 in 2D): grid and
    positions stay identical to the oracle across every device regrid."""
    mesh = oracle_py.Mesh.rect(dim, n)
    O, G = pair(mesh, 7, 0.05, 0.5, 200.0)
    for _ in range(nsteps):
        O.step(5, -1.0)
        G.step(5, -1.0)
    np.testing.assert_array_equal(G.get("grid"), O.get("grid"))
    np.testing.assert_array_equal(G.get("x"), O.get("x"))
    assert G.stats()["regrids"] == nsteps
