"""Pins the LASolver restatement (oracle/lasolver.cpp) bit for bit: against the golden fixtures the
reference itself produced (tests/golden/make_lasolver_golden.py) and, when the reference has been
compiled in this container (oracle/_ref), against it on fresh seeded systems."""
import glob
import os

import numpy as np
import pytest

import lasolver_py as L
import oracle_py

GOLD = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "lasolver", "*.npz"))
              if not p.endswith("ilu_levels.npz"))


def _same(x, y):
    return np.array_equal(np.asarray(x), np.asarray(y), equal_nan=True)


def test_fixtures_present():
    assert len(GOLD) == 8


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_restatement_matches_reference_fixture(path):
    g = np.load(path)  # allow_pickle defaults to False
    ia, ja, a, b = g["ia"], g["ja"], g["a"], g["b"]
    assert _same(L.matmult(ia, ja, a, b), g["matmult_b"])
    af = L.ilu0(ia, ja, a)
    assert _same(af, g["af"])
    assert _same(L.ilu_solve(ia, ja, af, b), g["ilu_solve_b"])
    x0 = g["x0"] if "x0" in g.files else None
    rr, nitmax, rhat = float(g["resid_reduc"]), int(g["nitmax"]), int(g["new_rhat"])
    for k in (1, 2, 3):
        x, it, _ = L.solve(ia, ja, a, b, nitmax=min(k, nitmax), resid_reduc=rr, new_rhat=rhat, x0=x0)
        assert it == int(g[f"nitr_it{k}"])
        assert _same(x, g[f"x_it{k}"])
    x, it, _ = L.solve(ia, ja, a, b, nitmax=nitmax, resid_reduc=rr, new_rhat=rhat, x0=x0)
    assert it == int(g["nitr"])
    assert _same(x, g["x"])


def test_zero_rhs_is_nan_like_reference():
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "lasolver", "rect2d_4_zero_rhs.npz"))
    assert int(g["nitr"]) == 1 and np.all(np.isnan(g["x"]))


def test_tridiagonal_ilu_exact():
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "lasolver", "tridiag_1000.npz"))
    assert int(g["nitr"]) == 1


def test_mesh_pattern_equals_pack_of_buildmatrix_stream():
    for dim, n in ((2, 3), (2, 6), (3, 2)):
        m = oracle_py.Mesh.rect(dim, n)
        rows, cols = L.mesh_entries(dim, m.F)
        ia, ja = L.pack(dim * m.nP, rows, cols)
        ia2, ja2 = L.mesh_pattern(dim, m.nP, m.F)
        assert _same(ia, ia2) and _same(ja, ja2)


@pytest.mark.skipif(not L.ref_available(), reason="reference LASolver not built (oracle/_ref)")
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_restatement_matches_reference_live(seed):
    rng = np.random.default_rng(seed)
    m = oracle_py.Mesh.rect(2, 5 + seed % 3)
    rows, cols = L.mesh_entries(2, m.F)
    N = 2 * m.nP
    ia, ja = L.pack(N, rows, cols, use_ref=True)
    ia2, ja2 = L.pack(N, rows, cols)
    assert _same(ia, ia2) and _same(ja, ja2)
    a = L.random_values(ia, ja, seed, 0.2 + 0.3 * (seed % 2))
    b = rng.uniform(-1, 1, N)
    xr, nr, _ = L.solve(ia, ja, a, b, use_ref=True)
    xo, no, _ = L.solve(ia, ja, a, b)
    assert nr == no and _same(xr, xo)
    _, _, afr, _ = L.ref_ilu(ia, ja, a)
    assert _same(afr, L.ilu0(ia, ja, a))


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_gpu_reduction_order_vs_reference(path):
    """dotMode 1 (the GPU's tree-shaped dot products) against the reference's sequential sums:
    the rounding-level bounds tests/test_gpu_lasolver.py relies on."""
    g = np.load(path)
    ia, ja, a, b = g["ia"], g["ja"], g["a"], g["b"]
    x0 = g["x0"] if "x0" in g.files else None
    rr, nitmax, rhat = float(g["resid_reduc"]), int(g["nitmax"]), int(g["new_rhat"])
    name = os.path.basename(path)
    x, it, _ = L.solve(ia, ja, a, b, nitmax=nitmax, resid_reduc=rr, new_rhat=rhat, x0=x0, tree=True)
    gx, gi = g["x"], int(g["nitr"])
    rel = np.linalg.norm(x - gx) / np.linalg.norm(gx)
    if "zero_rhs" in name:
        assert it == gi == 1 and np.all(np.isnan(x))
    elif "noconv" in name:
        assert it == gi == -1
    elif "hard" in name:
        assert abs(it - gi) <= 0.05 * gi and rel <= 1e-5
    else:
        assert it == gi and rel <= 1e-14
