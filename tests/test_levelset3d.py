"""The 3D LevelSet generator (utils::meshFromLevelSetFun 3D, src/MeshUtils.h:540-667, with
spherePhi, main.cpp:87-97): libmmadmm's O(N) mmadmm_mesh_levelset3d against the
oracle's restatement of the reference's own structure (std::set of used points, std::map pntMap with
the reversed rank), plus structural checks and the driver's TestType LevelSet Dim 3.

The reference's 3D generator loses its result (`delete Vp; Vp = Vpnew;` at 663-666 reassigns the
function's pointer copies) and does not compact the mask; both are repaired here.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import mmadmm_amd as mx
import oracle_py

EPS = 1e-12
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(ROOT, "mm-admm_amd", "bin", "mmadmm_run")


def _cube_cut(n):
    """The kept tetrahedra of the rect cube and the used vertex ids, from the generator's rule."""
    g = mx.MeshData.rect(3, n)
    phi = ((g.Xp - 0.5) ** 2).sum(1) - 0.4 * 0.4
    keep = ~np.all(phi[g.F] > -EPS, axis=1)
    used = np.zeros(g.nP, bool)
    used[g.F[keep].ravel()] = True
    return g, phi, keep, np.nonzero(used)[0]


def _dets(X, F):
    return np.linalg.det(X[F[:, 1:]] - X[F[:, [0]]])


@pytest.mark.parametrize("n", [1, 4, 10, 21])
@pytest.mark.parametrize("compact", [True, False])
@pytest.mark.parametrize("btype", [1, 0])
def test_product_equals_restatement(n, compact, btype):
    a = mx.MeshData.levelset3d(n, btype=btype, compact_mask=compact)
    b = oracle_py.Mesh.levelset3d(n, btype=btype, compact_mask=compact)
    np.testing.assert_array_equal(a.Xp, b.Vp)
    np.testing.assert_array_equal(a.F, b.F)
    np.testing.assert_array_equal(a.mask, b.mask)


@pytest.mark.parametrize("n", [4, 12, 30])
def test_structure(n):
    g, phi, keep, ids = _cube_cut(n)
    a = mx.MeshData.levelset3d(n)
    assert a.nF == int(keep.sum()) and a.nP == len(ids)
    # node numbering: the reference's pntMap, the i-th largest used id -> i (MeshUtils.h:645-651)
    desc = ids[::-1]
    np.testing.assert_array_equal(a.F, np.searchsorted(ids, g.F[keep])[:, :] * -1 + len(ids) - 1)
    # inside vertices unmoved and INTERIOR; outside / on-sphere ones moved and marked bType (FIXED)
    inside = phi[desc] <= -EPS
    np.testing.assert_array_equal(a.Xp[inside], g.Xp[desc][inside])
    assert (a.mask[inside] == mx.INTERIOR).all() and (a.mask[~inside] == mx.BOUNDARY_FIXED).all()
    r = np.linalg.norm(a.Xp[~inside] - 0.5, axis=1)
    # pulled towards the sphere (p - phi n with the squared-distance phi: near it, not onto it)
    assert np.abs(r - 0.4).max() < 0.75 / n
    # no tetrahedron degenerates or flips against the cube it was cut from
    d0, d1 = _dets(g.Xp[desc], a.F), _dets(a.Xp, a.F)
    assert (np.sign(d0) == np.sign(d1)).all() and (np.abs(d1) > 0).all()
    assert (np.abs(d1) / np.abs(d0)).min() > 0.01


def test_driver_levelset_3d(tmp_path):
    cfg = {"TestType": "LevelSet", "Dim": 3, "MonType": 3, "Method": 0, "CompMesh": False, "BoundaryType": 1,
           "GradUse": False, "nSteps": 3, "AdmmIter": 10, "DtTol": 1e-5, "dt": 0.025, "tau": 0.5, "rho": 50,
           "w": 3.53553390593, "nx": 10, "ny": 10, "nz": 10, "xa": 0, "xb": 1, "ya": 0, "yb": 1, "za": 0, "zb": 1}
    inp = tmp_path / "Experiments" / "InputFiles"
    inp.mkdir(parents=True)
    (inp / "Ls3.json").write_text(json.dumps(cfg))
    r = subprocess.run([RUN, "Ls3", "0", "1", "--root", str(tmp_path), "--dry-run"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    a = mx.MeshData.levelset3d(10)
    assert f"size of Vp {a.nP}, 3" in r.stdout and f"size of F {a.nF}, 4" in r.stdout
