"""Host-side logic of the LASolver replacement (no GPU): MatrixStruc packing and the symbolic
ILU(k) of libmmadmm.so against the reference's own outputs (golden fixtures)."""
import os
import sys

import numpy as np
import pytest

import lasolver_py as L
import oracle_py

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "mm-admm_amd", "python"))
la = pytest.importorskip("lasolver_amd")

LEV = os.path.join(os.path.dirname(__file__), "golden", "lasolver", "ilu_levels.npz")


@pytest.mark.parametrize("tag", ["d2", "d3"])
@pytest.mark.parametrize("level", [1, 2])
def test_symbolic_ilu_k_matches_reference(tag, level):
    g = np.load(LEV)
    iaf, jaf, dg = la.ilu_symbolic(g[f"{tag}_ia"], g[f"{tag}_ja"], level)
    assert np.array_equal(iaf, g[f"{tag}_l{level}_iaf"])
    assert np.array_equal(jaf, g[f"{tag}_l{level}_jaf"])
    assert np.array_equal(dg, g[f"{tag}_l{level}_diag"])


def test_symbolic_ilu0_is_the_pattern():
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "lasolver", "rect2d_9_tight.npz"))
    iaf, jaf, dg = la.ilu_symbolic(g["ia"], g["ja"], 0)
    assert np.array_equal(iaf, g["ia"]) and np.array_equal(jaf, g["ja"]) and np.array_equal(dg, g["diag"])


@pytest.mark.parametrize("dim,n", [(2, 4), (2, 7), (3, 2)])
def test_struc_pack_matches_reference_stream(dim, n):
    m = oracle_py.Mesh.rect(dim, n)
    rows, cols = L.mesh_entries(dim, m.F)
    N = dim * m.nP
    s = la.MatrixStruc(N)
    s.set_entries(rows, cols)
    s.pack()
    ia, ja = L.pack(N, rows, cols)  # restatement, itself pinned to the reference
    assert np.array_equal(s.getia(), ia) and np.array_equal(s.getja(), ja)
    s2 = la.MatrixStruc(N)
    s2.mesh_pattern(dim, m.F)
    assert np.array_equal(s2.getia(), ia) and np.array_equal(s2.getja(), ja)


def test_struc_errors_like_reference():
    s = la.MatrixStruc(4)
    with pytest.raises(la.MMADMMError):
        s.set_entry(4, 0)  # "invalid row entry in set_entry"
    s.pack()
    with pytest.raises(la.MMADMMError):
        s.pack()  # "data structure already packed"
    with pytest.raises(la.MMADMMError):
        s.set_entry(0, 1)  # "data structure already compressed"


def test_symbolic_rejects_missing_diagonal():
    ia = np.array([0, 1, 2], np.int32)
    ja = np.array([1, 0], np.int32)
    with pytest.raises(la.MMADMMError):
        la.ilu_symbolic(ia, ja, 0)


def test_param_defaults():
    p = la.ParamIter()
    assert (p.order, p.level, p.iscal, p.nitmax, p.info) == (1, 1, 1, 30, 1)
    q = la.ParamIter.mesh()
    assert (q.order, q.level, q.iscal, q.nitmax, q.resid_reduc, q.new_rhat, q.iaccel) == (0, 0, 0, 10000, 1e-6, 0, 0)
