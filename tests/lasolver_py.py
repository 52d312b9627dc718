"""ctypes access to the LASolver oracle (oracle/liboracle.so: the CPU restatement) and, when it
has been built in this container, the reference itself (oracle/_ref/liblasolver_ref.so).
Test infrastructure only."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ORC = os.path.join(ROOT, "oracle", "liboracle.so")
_REF = os.path.join(ROOT, "oracle", "_ref", "liblasolver_ref.so")

_i = ctypes.c_int
_d = ctypes.c_double
_ip = ctypes.POINTER(ctypes.c_int)
_dp = ctypes.POINTER(ctypes.c_double)


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _lib(path):
    return ctypes.CDLL(path)


_orc = None
_ref = None


def orc():
    global _orc
    if _orc is None:
        _orc = _lib(_ORC)
        _orc.orc_la_pack.argtypes = [_i, _i, _ip, _ip, _i, _ip, _ip, _i]
        _orc.orc_la_mesh_pattern.argtypes = [_i, _i, _i, _ip, _ip, _ip, _i]
        _orc.orc_la_matmult.argtypes = [_i, _ip, _ip, _dp, _dp, _dp]
        _orc.orc_la_ilu0.argtypes = [_i, _ip, _ip, _dp, _dp]
        _orc.orc_la_ilu_solve.argtypes = [_i, _ip, _ip, _dp, _dp, _dp]
        _orc.orc_la_solve.argtypes = [_i, _ip, _ip, _dp, _dp, _dp, _i, _d, _i, _i, _dp, _ip, _dp, _i]
    return _orc


def ref_available():
    return os.path.exists(_REF)


def ref():
    global _ref
    if _ref is None:
        _ref = _lib(_REF)
        _ref.lsr_struc_pack.argtypes = [_i, _i, _ip, _ip, _i, _ip, _ip, _i]
        _ref.lsr_solve.argtypes = [_i, _ip, _ip, _dp, _dp, _dp, _i, _i, _i, _i, _i, _d, _i, _i, _dp, _ip]
        _ref.lsr_ilu.argtypes = [_i, _ip, _ip, _dp, _i, _ip, _ip, _dp, _ip, _i]
        _ref.lsr_ilu_solve.argtypes = [_i, _ip, _ip, _dp, _dp, _dp]
        _ref.lsr_matmult.argtypes = [_i, _ip, _ip, _dp, _dp, _dp]
    return _ref


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def pack(n, rows, cols, no_diag=0, use_ref=False):
    """MatrixStruc(n, no_diag) + set_entry + pack -> (ia, ja)."""
    rows, cols = _i32(rows), _i32(cols)
    fn = ref().lsr_struc_pack if use_ref else orc().orc_la_pack
    ia = np.zeros(n + 1, np.int32)
    nnz = fn(n, len(rows), _ptr(rows, _ip), _ptr(cols, _ip), no_diag, _ptr(ia, _ip), None, 0)
    assert nnz >= 0
    ja = np.zeros(max(nnz, 1), np.int32)
    fn(n, len(rows), _ptr(rows, _ip), _ptr(cols, _ip), no_diag, _ptr(ia, _ip), _ptr(ja, _ip), nnz)
    return ia, ja[:nnz]


def mesh_pattern(dim, nP, F):
    """Backward-Euler Jacobian pattern (src/Mesh.cpp:309-345), packed."""
    F = _i32(F)
    n = dim * nP
    ia = np.zeros(n + 1, np.int32)
    nnz = orc().orc_la_mesh_pattern(dim, nP, len(F), _ptr(F, _ip), _ptr(ia, _ip), None, 0)
    ja = np.zeros(nnz, np.int32)
    orc().orc_la_mesh_pattern(dim, nP, len(F), _ptr(F, _ip), _ptr(ia, _ip), _ptr(ja, _ip), nnz)
    return ia, ja


def mesh_entries(dim, F):
    """The (row, col) set_entry stream buildMatrix issues (src/Mesh.cpp:313-341), in order."""
    F = np.asarray(F)
    rows, cols = [], []
    for s in range(len(F)):
        pl = list(F[s])
        for _ in range(dim + 1):
            for n_ in range(dim + 1):
                for r in range(pl[0] * dim, pl[0] * dim + dim):
                    for c in range(pl[n_] * dim, pl[n_] * dim + dim):
                        rows.append(r)
                        cols.append(c)
            pl = pl[1:] + pl[:1]
    return np.array(rows, np.int32), np.array(cols, np.int32)


def matmult(ia, ja, a, x, use_ref=False):
    n = len(ia) - 1
    ia, ja, a, x = _i32(ia), _i32(ja), _f64(a), _f64(x)
    y = np.zeros(n)
    (ref().lsr_matmult if use_ref else orc().orc_la_matmult)(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), _ptr(x, _dp), _ptr(y, _dp))
    return y


def ilu0(ia, ja, a):
    n = len(ia) - 1
    ia, ja, a = _i32(ia), _i32(ja), _f64(a)
    af = np.zeros(len(a))
    assert orc().orc_la_ilu0(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), _ptr(af, _dp)) == 0
    return af


def ref_ilu(ia, ja, a, level=0):
    """The reference's own ILU factor (sfac2 + factor) -> (iaf, jaf, af, diag row-relative)."""
    n = len(ia) - 1
    ia, ja, a = _i32(ia), _i32(ja), _f64(a)
    iaf = np.zeros(n + 1, np.int32)
    diag = np.zeros(n, np.int32)
    nz = ref().lsr_ilu(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), level, _ptr(iaf, _ip), None, None, None, 0)
    assert nz >= 0
    jaf = np.zeros(nz, np.int32)
    af = np.zeros(nz)
    ref().lsr_ilu(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), level, _ptr(iaf, _ip), _ptr(jaf, _ip),
                  _ptr(af, _dp), _ptr(diag, _ip), nz)
    return iaf, jaf, af, diag


def ref_ilu_solve(ia, ja, a, b):
    n = len(ia) - 1
    ia, ja, a, b = _i32(ia), _i32(ja), _f64(a), _f64(b)
    x = np.zeros(n)
    assert ref().lsr_ilu_solve(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), _ptr(b, _dp), _ptr(x, _dp)) == 0
    return x


def ilu_solve(ia, ja, af, b):
    n = len(ia) - 1
    ia, ja, af, b = _i32(ia), _i32(ja), _f64(af), _f64(b)
    x = np.zeros(n)
    assert orc().orc_la_ilu_solve(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(af, _dp), _ptr(b, _dp), _ptr(x, _dp)) == 0
    return x


def solve(ia, ja, a, b, nitmax=10000, resid_reduc=1e-6, new_rhat=0, x0=None, toler=None, use_ref=False, tree=False):
    """MatrixIter::solve with the src/Mesh.cpp parameters -> (x, nitr, rms history).
    tree=True: dot products in the GPU's fixed reduction order instead of sequential sums."""
    n = len(ia) - 1
    ia, ja, a, b = _i32(ia), _i32(ja), _f64(a), _f64(b)
    tol = _f64(toler) if toler is not None else None
    x = _f64(x0).copy() if x0 is not None else np.zeros(n)
    nitr = ctypes.c_int(0)
    if use_ref:
        rc = ref().lsr_solve(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), _ptr(b, _dp), _ptr(tol, _dp),
                             0, 0, 0, 0, nitmax, resid_reduc, new_rhat, 1 if x0 is not None else 0,
                             _ptr(x, _dp), ctypes.byref(nitr))
        assert rc == 0
        return x, nitr.value, None
    hist = np.zeros(max(nitmax, 1))
    rc = orc().orc_la_solve(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), _ptr(b, _dp), _ptr(tol, _dp),
                            nitmax, resid_reduc, new_rhat, 1 if x0 is not None else 0, _ptr(x, _dp),
                            ctypes.byref(nitr), _ptr(hist, _dp), 1 if tree else 0)
    assert rc == 0
    k = nitr.value if nitr.value > 0 else nitmax
    return x, nitr.value, hist[:k]


def solve_ref_level(ia, ja, a, b, level, nitmax=10000, resid_reduc=1e-6):
    """The reference's MatrixIter::solve with ILU(level)."""
    n = len(ia) - 1
    ia, ja, a, b = _i32(ia), _i32(ja), _f64(a), _f64(b)
    x = np.zeros(n)
    nitr = ctypes.c_int(0)
    assert ref().lsr_solve(n, _ptr(ia, _ip), _ptr(ja, _ip), _ptr(a, _dp), _ptr(b, _dp), None, 0, level, 0, 0,
                           nitmax, resid_reduc, 0, 0, _ptr(x, _dp), ctypes.byref(nitr)) == 0
    return x, nitr.value, None


def random_values(ia, ja, seed, shift=None, dtau=None):
    """Seeded values in the pattern.  shift: diagonal made dominant by |row sum| * shift."""
    rng = np.random.default_rng(seed)
    n = len(ia) - 1
    a = rng.uniform(-1.0, 1.0, len(ja))
    if dtau is not None:  # J = I + dt/tau * H-like
        a *= dtau
    if shift is not None:
        for i in range(n):
            s = ia[i]; e = ia[i + 1]
            d = s + int(np.nonzero(ja[s:e] == i)[0][0])
            a[d] = np.sum(np.abs(a[s:e])) * shift + 1.0
    return a
