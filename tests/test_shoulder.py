"""The Shoulder experiment (main.cpp:403-630): its mesh against a plain restatement of the listed
lines, and whole runs of the oracle against the reference's committed Shoulder results.

The mesh is the rect mesh without the simplices whose centroid lies in the upper quadrant, the
boundary re-marking, and the random moves of interior vertices drawn from glibc rand() after
srand(69) (main.cpp:785) with Eigen's Random() = -1 + 2 rand()/RAND_MAX per coefficient.  The
reference's Experiments/InputFiles/Monitor110.json (and 120/140/1160/1320, 3DMonitor110) run it;
their results (Experiments/Results/<name>/Ih0.txt, points.txt, triangles.txt, copied to
tests/golden/) pin the random sequence (t = 0 energies to 6 digits) and the whole trajectory.
Monitor140's committed trace is a stale artifact: rows 0-6 reproduce, then it follows neither
GradUse setting of its JSON (measured with the oracle).  CPU only."""
import ctypes
import ctypes.util

import numpy as np
import pytest

import mmadmm_amd as mx

libc = ctypes.CDLL(ctypes.util.find_library("c"))
RAND_MAX = 2147483647


def restated(dim, n, btype=mx.BOUNDARY_FIXED):
    base = mx.MeshData.rect(dim, n, btype=btype)
    X = base.Xp.copy()
    F = base.F.copy()
    mask = base.mask.copy()
    c0 = (0 + 1) / 2.0
    keep = []
    for i in range(F.shape[0]):
        x = X[F[i]]
        c = [((x[0, d] + x[1, d]) + x[2, d]) * (1.0 / 3.0) if dim == 2 else
             (((x[0, d] + x[1, d]) + x[2, d]) + x[3, d]) * (1.0 / 4.0) for d in range(dim)]
        if all(c[d] > c0 for d in range(dim)):
            for v in F[i]:
                p = X[v]
                e = lambda a, b: abs(a - b) < 1e-16  # noqa: E731
                if dim == 2:
                    fixed = (e(p[0], c0) and e(p[1], c0)) or (e(p[0], c0) and e(p[1], 1.0)) or (e(p[0], 1.0) and e(p[1], c0))
                else:
                    fixed = ((e(p[0], c0) and e(p[2], c0)) or (e(p[0], c0) and e(p[2], 1.0)) or (e(p[0], 1.0) and e(p[2], c0))
                             or (e(p[1], 0.0) and e(p[2], c0)) or (e(p[1], 1.0) and e(p[2], c0))
                             or (e(p[0], c0) and e(p[1], 0.0)) or (e(p[0], c0) and e(p[1], 1.0)))
                mask[v] = mx.BOUNDARY_FIXED if fixed else btype
        else:
            keep.append(i)
    F = F[keep]
    Xc = X.copy()
    h = np.sqrt(sum((1.0 / n) ** 2 for _ in range(dim)))
    for i in range(X.shape[0]):
        if mask[i] != mx.INTERIOR:
            continue
        d = np.array([-1.0 + 2.0 * float(libc.rand()) / float(RAND_MAX) for _ in range(dim)])
        sq = 0.0
        for k in range(dim):
            sq = d[k] * d[k] if k == 0 else sq + d[k] * d[k]
        d = d / np.sqrt(sq)
        r = (h / 10.0) * float(libc.rand()) / float(RAND_MAX)
        X[i] = X[i] + r * d
    return X, Xc, F, mask


@pytest.mark.parametrize("dim,n", [(2, 8), (2, 13), (3, 4)])
def test_shoulder_matches_restatement(dim, n):
    libc.srand(69)
    m = mx.MeshData.shoulder(dim, n)
    libc.srand(69)
    X, Xc, F, mask = restated(dim, n)
    np.testing.assert_array_equal(m.F, F)
    np.testing.assert_array_equal(m.mask, mask)
    np.testing.assert_array_equal(m.Xc, Xc)
    np.testing.assert_array_equal(m.Xp, X)
    assert m.F.shape[0] < (4 if dim == 2 else 12) * n ** dim  # the quadrant is gone
    assert not np.array_equal(m.Xp, m.Xc)


import oracle_py  # noqa: E402
from ref_runs import (POINTS_ATOL, RUNS, SIX_DIGITS, ih, load_txt, make_mesh, rel_err,  # noqa: E402
                      run_trace)


def _oracle(name, nthreads=0):
    mesh, mon, dt, tau, rho, gu = RUNS[name][:6]
    m = make_mesh(mesh, mx.MeshData)
    om = oracle_py.Mesh(mesh[1], m.Xp, m.F, m.mask)
    return oracle_py.Integrator(om, mon, dt, tau, rho, gradUse=gu, nthreads=nthreads)


@pytest.mark.parametrize("name", ["Monitor110", "Monitor120", "Monitor140", "Monitor1160", "3DMonitor110"])
def test_shoulder_t0_energy_pins_random_sequence(name):
    I = _oracle(name)
    assert abs(I.energy() - ih(name)[0]) / ih(name)[0] < SIX_DIGITS


def test_monitor110_whole_run():
    """All 78 rows of Monitor110/Ih0.txt (GradUse true), the final points and the reoriented
    triangles."""
    mesh, mon, dt, tau, rho, gu, admm, dtTol, nSteps = RUNS["Monitor110"]
    I = _oracle("Monitor110")
    ours = run_trace(lambda n, t: I.step(n, t)[0], I.energy, nSteps, dt, admm, dtTol)
    ref = ih("Monitor110")
    assert len(ours) == len(ref)
    assert rel_err(ours, ref) < SIX_DIGITS
    I.done()
    np.testing.assert_allclose(I.get("points").reshape(-1, 2), load_txt("Monitor110", "points.txt"), rtol=0,
                               atol=POINTS_ATOL)
    np.testing.assert_array_equal(I.F(), load_txt("Monitor110", "triangles.txt", dtype=np.int32))


def test_monitor120_first_200_steps():
    mesh, mon, dt, tau, rho, gu, admm, dtTol, nSteps = RUNS["Monitor120"]
    I = _oracle("Monitor120")
    ours = run_trace(lambda n, t: I.step(n, t)[0], I.energy, nSteps, dt, admm, dtTol, max_steps=200)
    assert rel_err(ours, ih("Monitor120")[:201]) < SIX_DIGITS
    np.testing.assert_array_equal(I.F(), load_txt("Monitor120", "triangles.txt", dtype=np.int32))


def test_monitor140_stale_artifact_prefix():
    """Rows 0-6 of the committed Monitor140 trace reproduce; the rest does not (stale artifact)."""
    mesh, mon, dt, tau, rho, gu, admm, dtTol, nSteps = RUNS["Monitor140"]
    I = _oracle("Monitor140")
    ours = run_trace(lambda n, t: I.step(n, t)[0], I.energy, nSteps, dt, admm, dtTol, max_steps=6)
    assert rel_err(ours, ih("Monitor140")[:7]) < 2e-6


def test_3dmonitor110_orientation():
    """3D Shoulder: the reoriented tetrahedra equal the reference's output triangles.txt."""
    I = _oracle("3DMonitor110")
    np.testing.assert_array_equal(I.F(), load_txt("3DMonitor110", "triangles.txt", dtype=np.int32))
