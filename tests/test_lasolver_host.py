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


@pytest.mark.skipif(not L.ref_available(), reason="the reference LASolver build (oracle/_ref) is not present")
@pytest.mark.parametrize("seed", range(6))
def test_symbolic_ilu_k_random_patterns_match_reference_build(seed):
    """Round 6: the level-of-fill symbolic factor (a heap-driven row merge, sparse.cpp) against the
    reference's own scaler_ILU built in place (oracle/_ref) on random unsymmetric patterns, levels
    1-3, where fill joins the pivots of its own row."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(20, 200))
    rows, cols = [], []
    for i in range(n):
        c = set(rng.integers(0, n, int(rng.integers(1, 8))).tolist()) | {i}
        rows += [i] * len(c)
        cols += sorted(c)
    ia, ja = L.pack(n, np.array(rows, np.int32), np.array(cols, np.int32))
    ia, ja = np.asarray(ia), np.asarray(ja)
    for level in (1, 2, 3):
        iaf, jaf, _ = la.ilu_symbolic(ia, ja, level)
        riaf, rjaf = L.ref_ilu(ia, ja, np.ones(len(ja)), level)[:2]
        assert np.array_equal(iaf, riaf) and np.array_equal(jaf, rjaf), level


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


def _schedule_info(ia, ja, level, fwd):
    import ctypes
    L_ = la.lib()
    L_.mmx_sweep_schedule_info.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p]
    ia = np.ascontiguousarray(ia, np.int32)
    ja = np.ascontiguousarray(ja, np.int32)
    out = np.zeros(16, np.int64)
    rc = L_.mmx_sweep_schedule_info(len(ia) - 1, ia.ctypes.data, ja.ctypes.data, level, int(fwd), out.ctypes.data)
    assert rc == 0, L_.mmx_last_error().decode() if hasattr(L_, "mmx_last_error") else rc
    keys = "ok E R RI bands chains maxLen maxSkew maxT slots imports estIters levels".split()
    return dict(zip(keys, out[:13].tolist()))


@pytest.mark.parametrize("mesh,level", [(("rect", 2, 20), 0), (("rect", 2, 57), 0), (("rect", 2, 20), 1),
                                        (("hexdisc", 30), 0), (("circle", "CircleEx24"), 0), (("rect", 3, 6), 0),
                                        (("rect", 3, 14), 0)])
@pytest.mark.parametrize("pair", ["1", "0"])
def test_chain_schedule_is_valid(mesh, level, pair, monkeypatch):
    """The chain/band sweep schedule (host/chain_sched.cpp) replays correctly on the host: every row
    once with the reference's entry order, ring values live when read, imports right and ordered,
    a pair's forwarded entry its first row (validate_chain_schedule, which mmx_sweep_schedule_info
    runs and fails on)."""
    import mmadmm_amd as mx
    from conftest import circle_mesh
    if mesh[0] == "rect":
        m = oracle_py.Mesh.rect(mesh[1], mesh[2])
        dim, F, nP = mesh[1], m.F, m.nP
    elif mesh[0] == "hexdisc":
        md = mx.MeshData.hexdisc(mesh[1], 0.5, 0.5, 0.5)
        dim, F, nP = 2, md.F, md.nP
    else:
        c = circle_mesh(mesh[1])
        dim, F, nP = 2, c.F, c.Vp.shape[0]
    ia, ja = L.mesh_pattern(dim, nP, F)
    monkeypatch.setenv("MMX_CHAIN_PAIR", pair)  # 2D: two rows per position (default) or one
    for fwd in (True, False):
        info = _schedule_info(ia, ja, level, fwd)
        assert info["ok"] == 1, info
        if dim == 3:
            # 3D: the lower rows fit 32-entry stages, the upper rows (up to 44 entries) 48-entry ones
            # (one position per row); each band's lanes wait for imports from several planes, and the
            # modelled path stays within two DAG depths
            assert info["E"] == (32 if fwd else 48) and info["estIters"] <= 2 * info["levels"] + 64, info
        elif pair == "1":
            # two chain rows per iteration: the critical path is about half the DAG's depth
            assert info["estIters"] <= 0.7 * info["levels"] + 64, info
        else:
            # the critical path stays close to the dependency DAG's depth
            assert info["estIters"] <= 1.3 * info["levels"] + 64, info


@pytest.mark.parametrize("n", [6, 14])
def test_segmented_schedule_is_valid(n, monkeypatch):
    """MMX_CHAIN_E48=0: the 3D upper rows take two 32-entry segments at consecutive positions (the
    round-3 layout) -- still a valid schedule, only a longer one."""
    m = oracle_py.Mesh.rect(3, n)
    ia, ja = L.mesh_pattern(3, m.nP, m.F)
    monkeypatch.setenv("MMX_CHAIN_E48", "0")
    info = _schedule_info(ia, ja, 0, False)
    assert info["ok"] == 1 and info["E"] == 32, info
    assert info["estIters"] <= 4 * info["levels"] + 64, info


@pytest.mark.parametrize("mesh", [("rect", 2, 20), ("rect", 2, 57), ("hexdisc", 30), ("circle", "CircleEx24"),
                                  ("rect", 3, 4)])
def test_factor_schedule_is_valid(mesh):
    """The numeric factor's chain/band schedule (build_factor_schedule) replays correctly on the
    host: every (entry, pivot) update the reference makes reads U(j_q, col e) from the right ring
    cell or imported row, written before and not overwritten; no update the reference does not
    make (validate_factor_schedule).  3D rows exceed the factor's row layout: no schedule."""
    import ctypes
    import mmadmm_amd as mx
    from conftest import circle_mesh
    if mesh[0] == "rect":
        m = oracle_py.Mesh.rect(mesh[1], mesh[2])
        dim, F, nP = mesh[1], m.F, m.nP
    elif mesh[0] == "hexdisc":
        md = mx.MeshData.hexdisc(mesh[1], 0.5, 0.5, 0.5)
        dim, F, nP = 2, md.F, md.nP
    else:
        c = circle_mesh(mesh[1])
        dim, F, nP = 2, c.F, c.Vp.shape[0]
    ia, ja = L.mesh_pattern(dim, nP, F)
    L_ = la.lib()
    L_.mmx_factor_schedule_info.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    ia = np.ascontiguousarray(ia, np.int32)
    ja = np.ascontiguousarray(ja, np.int32)
    out = np.zeros(8, np.int64)
    rc = L_.mmx_factor_schedule_info(len(ia) - 1, ia.ctypes.data, ja.ctypes.data, 0, out.ctypes.data)
    assert rc == 0
    info = dict(zip("ok bands slots R imports maxslots estIters levels".split(), out.tolist()))
    if dim == 3:
        assert info["ok"] == 0
    else:
        assert info["ok"] == 1 and info["maxslots"] <= 384, info
        assert info["estIters"] <= 1.3 * info["levels"] + 64, info
