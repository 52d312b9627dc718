"""The oracle's time-varying-monitor path (the reference's commented Mesh::setUp
hook, src/Mesh.cpp:1006-1014, re-running MeshInterpolator::updateMesh + interpolateMonitor at every
step start).  No reference counterpart exists to pin it (parity unpinned beyond the set-up itself,
which test_oracle_pins.py pins through the t = 0 energies); these are consistency checks."""
import numpy as np

import oracle_py


def test_static_monitor_regrid_first_step_unchanged():
    """At step 0 the mesh has not moved: rebuilding the grid of a static monitor changes nothing."""
    m = oracle_py.Mesh.rect(2, 12)
    A = oracle_py.Integrator(m, 1, 0.025, 0.5, 100.0)
    B = oracle_py.Integrator(m, 1, 0.025, 0.5, 100.0, regrid=True)
    a = A.step(5, -1.0)[0]
    b = B.step(5, -1.0)[0]
    assert a == b
    np.testing.assert_array_equal(A.get("x"), B.get("x"))


def test_static_monitor_regrid_follows_the_mesh():
    m = oracle_py.Mesh.rect(2, 12)
    B = oracle_py.Integrator(m, 1, 0.025, 0.5, 100.0, regrid=True)
    g0 = B.get("grid").copy()
    B.step(5, -1.0)
    B.step(5, -1.0)  # step 2 rebuilds from the positions step 1 produced
    assert not np.array_equal(B.get("grid"), g0)


def test_moving_bump_grid_moves_with_time():
    m = oracle_py.Mesh.rect(2, 12)
    B = oracle_py.Integrator(m, 7, 0.1, 0.5, 100.0, regrid=True)
    g = [B.get("grid").copy()]
    for _ in range(3):
        B.step(5, -1.0)
        g.append(B.get("grid").copy())
    assert np.array_equal(g[0], g[1])  # t = 0 at step 0 (set-up also evaluates t = 0)
    assert not np.array_equal(g[1], g[2]) and not np.array_equal(g[2], g[3])
    assert np.isfinite(B.get("x")).all()


def test_moving_bump_monitor_formula():
    for t in (0.0, 0.3):
        x = np.array([0.4, 0.55])
        c = np.array([0.5 + 0.2 * np.cos(2 * np.pi * t), 0.5 + 0.2 * np.sin(2 * np.pi * t)])
        s = 1 + 5.0 / (1 + 50.0 * np.sum((x - c) ** 2))
        if t == 0.0:
            np.testing.assert_allclose(oracle_py.monitor_at(2, 7, x), [s, 0, 0, s], rtol=1e-15)
