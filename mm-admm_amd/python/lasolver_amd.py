"""lasolver_amd -- Python mirror of the reference's LASolver surface (lib/LASolver/MatrixIter.h) on
the MI355X kernels of libmmadmm.so (include/mmx_sparse.h).

  ParamIter                     MatrixIter.h:113-175 (defaults of its constructor; ParamIter.mesh()
                                gives the settings src/Mesh.cpp:264-304 uses)
  MatrixStruc(n, no_diag)       set_entry(row, col), pack(), getia(), getja(), getnja()
  MatrixIter(struc) / MatrixIter(n, ia, ja)
                                aValue / bValue as numpy views (a, b), set_toler, sfac(param),
                                solve(param, x, initial_guess) -> nitr (x updated in place),
                                matmult(x) (the module-level matmult of accel_class.cpp)
There is no CPU fallback: every call runs on the GPU through the C-ABI.
"""
import ctypes

import numpy as np

from mmadmm_amd import MMADMMError, _check, c_double_p, c_int_p, lib as _mlib

_cfg = False


class ParamIter(ctypes.Structure):
    _fields_ = [("order", ctypes.c_int), ("level", ctypes.c_int), ("drop_ilu", ctypes.c_int),
                ("ipiv", ctypes.c_int), ("iscal", ctypes.c_int), ("nitmax", ctypes.c_int),
                ("resid_reduc", ctypes.c_double), ("info", ctypes.c_int), ("drop_tol", ctypes.c_double),
                ("new_rhat", ctypes.c_int), ("iaccel", ctypes.c_int), ("north", ctypes.c_int)]

    def __init__(self):
        super().__init__()
        lib().mmx_param_iter_default(ctypes.byref(self))

    @staticmethod
    def mesh():
        p = ParamIter()
        lib().mmx_param_iter_mesh(ctypes.byref(p))
        return p


class SparseStats(ctypes.Structure):
    _fields_ = [("solves", ctypes.c_longlong), ("iterations", ctypes.c_longlong), ("spmvs", ctypes.c_longlong),
                ("sweeps", ctypes.c_longlong), ("factors", ctypes.c_longlong), ("t_spmv_ms", ctypes.c_double),
                ("t_sweep_ms", ctypes.c_double), ("t_factor_ms", ctypes.c_double), ("t_vec_ms", ctypes.c_double),
                ("t_solve_ms", ctypes.c_double), ("n_spmv_timed", ctypes.c_longlong),
                ("n_sweep_timed", ctypes.c_longlong), ("n_factor_timed", ctypes.c_longlong),
                ("spmv_bytes", ctypes.c_double), ("last_rms", ctypes.c_double), ("rmsi", ctypes.c_double),
                ("sweep_mode", ctypes.c_int), ("sweep_e", ctypes.c_int), ("factor_mode", ctypes.c_int),
                ("sweep_e_bwd", ctypes.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def lib():
    global _cfg
    L = _mlib()
    if _cfg:
        return L
    vp, i, ll, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_double
    pp = ctypes.POINTER(ParamIter)
    L.mmx_param_iter_default.argtypes = [pp]
    L.mmx_param_iter_default.restype = None
    L.mmx_param_iter_mesh.argtypes = [pp]
    L.mmx_param_iter_mesh.restype = None
    L.mmx_struc_create.argtypes = [i, i, ctypes.POINTER(vp)]
    L.mmx_struc_set_entry.argtypes = [vp, i, i]
    L.mmx_struc_set_entries.argtypes = [vp, ll, c_int_p, c_int_p]
    L.mmx_struc_mesh_pattern.argtypes = [vp, i, i, c_int_p]
    L.mmx_struc_pack.argtypes = [vp]
    L.mmx_struc_get.argtypes = [vp, ctypes.POINTER(i), ctypes.POINTER(ll), c_int_p, c_int_p]
    L.mmx_struc_destroy.argtypes = [vp]
    L.mmx_matrix_create.argtypes = [i, i, c_int_p, c_int_p, ctypes.POINTER(vp)]
    L.mmx_matrix_create_from_struc.argtypes = [i, vp, ctypes.POINTER(vp)]
    L.mmx_matrix_sizes.argtypes = [vp, ctypes.POINTER(i), ctypes.POINTER(ll)]
    L.mmx_matrix_stream.argtypes = [vp, ctypes.POINTER(vp)]
    L.mmx_matrix_set_values.argtypes = [vp, c_double_p]
    L.mmx_matrix_set_values_device.argtypes = [vp, vp]
    L.mmx_matrix_set_rhs.argtypes = [vp, c_double_p]
    L.mmx_matrix_set_rhs_device.argtypes = [vp, vp]
    L.mmx_matrix_set_toler.argtypes = [vp, c_double_p]
    L.mmx_matrix_sfac.argtypes = [vp, pp]
    L.mmx_matrix_solve.argtypes = [vp, pp, c_double_p, ctypes.POINTER(i), i]
    L.mmx_matrix_solve_device.argtypes = [vp, pp, vp, ctypes.POINTER(i), i]
    L.mmx_matrix_matmult.argtypes = [vp, c_double_p, c_double_p]
    L.mmx_matrix_matmult_device.argtypes = [vp, vp, vp]
    L.mmx_matrix_factor.argtypes = [vp]
    L.mmx_matrix_ilu_solve.argtypes = [vp, c_double_p, c_double_p]
    L.mmx_matrix_ilu_solve_device.argtypes = [vp, vp, vp]
    L.mmx_matrix_factor_nnz.argtypes = [vp, ctypes.POINTER(ll)]
    L.mmx_matrix_get_factor.argtypes = [vp, c_int_p, c_int_p, c_double_p, c_int_p]
    L.mmx_matrix_set_timing.argtypes = [vp, i]
    L.mmx_matrix_stats_get.argtypes = [vp, ctypes.POINTER(SparseStats)]
    L.mmx_matrix_stats_reset.argtypes = [vp]
    L.mmx_matrix_destroy.argtypes = [vp]
    L.mmx_stream_copy.argtypes = [i, vp, vp, ll, i, i, ctypes.POINTER(ctypes.c_double)]
    L.mmx_occupy.argtypes = [i, i, ctypes.c_double]
    L.mmx_occupy_wait.argtypes = []
    L.mmx_ilu_symbolic.argtypes = [i, c_int_p, c_int_p, i, ctypes.POINTER(ll), c_int_p, c_int_p, c_int_p]
    _cfg = True
    return L


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class MatrixStruc:
    """MatrixStruc(n, no_diag) (lib/LASolver/MatrixIter.h:66-107)."""

    def __init__(self, n, no_diag=0):
        self.h = ctypes.c_void_p()
        _check(lib().mmx_struc_create(int(n), int(no_diag), ctypes.byref(self.h)))
        self.n = int(n)

    def set_entry(self, row, col):
        _check(lib().mmx_struc_set_entry(self.h, int(row), int(col)))

    def set_entries(self, rows, cols):
        rows, cols = _i32(rows), _i32(cols)
        if rows.shape != cols.shape:
            raise ValueError("rows and cols differ in length")
        _check(lib().mmx_struc_set_entries(self.h, len(rows), rows.ctypes.data_as(c_int_p),
                                           cols.ctypes.data_as(c_int_p)))

    def mesh_pattern(self, dim, F):
        """The set_entry loop of Mesh::buildMatrix (src/Mesh.cpp:309-341) for simplices F."""
        F = _i32(F)
        _check(lib().mmx_struc_mesh_pattern(self.h, int(dim), len(F), F.ctypes.data_as(c_int_p)))

    def pack(self):
        _check(lib().mmx_struc_pack(self.h))

    def getnja(self):
        nnz = ctypes.c_longlong()
        _check(lib().mmx_struc_get(self.h, None, ctypes.byref(nnz), None, None))
        return nnz.value

    def getia(self):
        ia = np.zeros(self.n + 1, np.int32)
        _check(lib().mmx_struc_get(self.h, None, None, ia.ctypes.data_as(c_int_p), None))
        return ia

    def getja(self):
        ja = np.zeros(self.getnja(), np.int32)
        _check(lib().mmx_struc_get(self.h, None, None, None, ja.ctypes.data_as(c_int_p)))
        return ja

    def __del__(self):
        if lib is None:  # interpreter shutdown: the library is being torn down
            return
        if getattr(self, "h", None) and self.h.value:
            lib().mmx_struc_destroy(self.h)
            self.h = ctypes.c_void_p()


class MatrixIter:
    """MatrixIter (lib/LASolver/MatrixIter.h:178-383) resident on one MI355X.

    `a` and `b` are host arrays standing in for aValue(k) / bValue(i); they are sent to the GPU
    by sfac/solve/matmult (or explicitly with upload())."""

    def __init__(self, struc_or_n, ia=None, ja=None, device=0):
        self.h = ctypes.c_void_p()
        if isinstance(struc_or_n, MatrixStruc):
            _check(lib().mmx_matrix_create_from_struc(int(device), struc_or_n.h, ctypes.byref(self.h)))
        else:
            ia, ja = _i32(ia), _i32(ja)
            _check(lib().mmx_matrix_create(int(device), int(struc_or_n), ia.ctypes.data_as(c_int_p),
                                           ja.ctypes.data_as(c_int_p), ctypes.byref(self.h)))
        n, nnz = ctypes.c_int(), ctypes.c_longlong()
        _check(lib().mmx_matrix_sizes(self.h, ctypes.byref(n), ctypes.byref(nnz)))
        self.n, self.nnz = n.value, nnz.value
        self.a = np.zeros(self.nnz)
        self.b = np.zeros(self.n)
        self._ia = None
        self._ja = None

    # aValue / bValue: host mirrors, uploaded before use
    def aValue(self, k):
        return self.a[k]

    def bValue(self, i):
        return self.b[i]

    def upload(self):
        _check(lib().mmx_matrix_set_values(self.h, _f64(self.a).ctypes.data_as(c_double_p)))
        _check(lib().mmx_matrix_set_rhs(self.h, _f64(self.b).ctypes.data_as(c_double_p)))

    def set_toler(self, tol):
        _check(lib().mmx_matrix_set_toler(self.h, _f64(tol).ctypes.data_as(c_double_p)))

    def sfac(self, param):
        _check(lib().mmx_matrix_sfac(self.h, ctypes.byref(param)))

    def solve(self, param, x, initial_guess=0):
        """Returns nitr (-1 if not converged); x (float64 array of n) receives the solution."""
        if x.dtype != np.float64 or not x.flags.c_contiguous or len(x) != self.n:
            raise ValueError("x must be a contiguous float64 array of length n")
        self.upload()
        nitr = ctypes.c_int()
        _check(lib().mmx_matrix_solve(self.h, ctypes.byref(param), x.ctypes.data_as(c_double_p),
                                      ctypes.byref(nitr), int(initial_guess)))
        return nitr.value

    def matmult(self, x):
        _check(lib().mmx_matrix_set_values(self.h, _f64(self.a).ctypes.data_as(c_double_p)))
        x = _f64(x)
        y = np.zeros(self.n)
        _check(lib().mmx_matrix_matmult(self.h, x.ctypes.data_as(c_double_p), y.ctypes.data_as(c_double_p)))
        return y

    def factor(self):
        _check(lib().mmx_matrix_set_values(self.h, _f64(self.a).ctypes.data_as(c_double_p)))
        _check(lib().mmx_matrix_factor(self.h))

    def ilu_solve(self, b):
        b = _f64(b)
        x = np.zeros(self.n)
        _check(lib().mmx_matrix_ilu_solve(self.h, b.ctypes.data_as(c_double_p), x.ctypes.data_as(c_double_p)))
        return x

    def get_factor(self):
        nz = ctypes.c_longlong()
        _check(lib().mmx_matrix_factor_nnz(self.h, ctypes.byref(nz)))
        iaf = np.zeros(self.n + 1, np.int32)
        jaf = np.zeros(nz.value, np.int32)
        af = np.zeros(nz.value)
        dg = np.zeros(self.n, np.int32)
        _check(lib().mmx_matrix_get_factor(self.h, iaf.ctypes.data_as(c_int_p), jaf.ctypes.data_as(c_int_p),
                                           af.ctypes.data_as(c_double_p), dg.ctypes.data_as(c_int_p)))
        return iaf, jaf, af, dg

    # device-pointer variants (torch tensors' data_ptr() on the matrix's device)
    def set_values_device(self, ptr):
        _check(lib().mmx_matrix_set_values_device(self.h, ctypes.c_void_p(ptr)))

    def set_rhs_device(self, ptr):
        _check(lib().mmx_matrix_set_rhs_device(self.h, ctypes.c_void_p(ptr)))

    def matmult_device(self, xptr, yptr):
        _check(lib().mmx_matrix_matmult_device(self.h, ctypes.c_void_p(xptr), ctypes.c_void_p(yptr)))

    def solve_device(self, param, xptr, initial_guess=0):
        nitr = ctypes.c_int()
        _check(lib().mmx_matrix_solve_device(self.h, ctypes.byref(param), ctypes.c_void_p(xptr),
                                             ctypes.byref(nitr), int(initial_guess)))
        return nitr.value

    def stream(self):
        s = ctypes.c_void_p()
        _check(lib().mmx_matrix_stream(self.h, ctypes.byref(s)))
        return s.value

    def set_timing(self, on=True):
        _check(lib().mmx_matrix_set_timing(self.h, 1 if on else 0))

    def stats(self):
        s = SparseStats()
        _check(lib().mmx_matrix_stats_get(self.h, ctypes.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        _check(lib().mmx_matrix_stats_reset(self.h))

    def close(self):
        if lib is None:  # interpreter shutdown
            return
        if getattr(self, "h", None) and self.h.value:
            lib().mmx_matrix_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        self.close()


def ilu_symbolic(ia, ja, level):
    """Factor pattern of the level-of-fill ILU (scaler_ILU::sfac2) -> (iaf, jaf, diag row-relative)."""
    ia, ja = _i32(ia), _i32(ja)
    n = len(ia) - 1
    nz = ctypes.c_longlong()
    _check(lib().mmx_ilu_symbolic(n, ia.ctypes.data_as(c_int_p), ja.ctypes.data_as(c_int_p), int(level),
                                  ctypes.byref(nz), None, None, None))
    iaf = np.zeros(n + 1, np.int32)
    jaf = np.zeros(nz.value, np.int32)
    dg = np.zeros(n, np.int32)
    _check(lib().mmx_ilu_symbolic(n, ia.ctypes.data_as(c_int_p), ja.ctypes.data_as(c_int_p), int(level), None,
                                  iaf.ctypes.data_as(c_int_p), jaf.ctypes.data_as(c_int_p), dg.ctypes.data_as(c_int_p)))
    return iaf, jaf, dg


def stream_copy_ms(src_ptr, dst_ptr, n, reps=20, device=0, variant=0):
    """Average ms of a 16-B-per-lane streaming copy of n doubles between two device buffers (the
    achievable HBM ceiling; 16 n bytes moved per copy)."""
    ms = ctypes.c_double()
    _check(lib().mmx_stream_copy(int(device), ctypes.c_void_p(src_ptr), ctypes.c_void_p(dst_ptr), int(n), int(reps),
                                 int(variant), ctypes.byref(ms)))
    return ms.value


def matmult(A, x):
    """accel_class.cpp's matmult(xin, xout, n, a, ia, ja) on the GPU."""
    return A.matmult(x)


__all__ = ["ParamIter", "MatrixStruc", "MatrixIter", "matmult", "ilu_symbolic", "stream_copy_ms", "MMADMMError"]


def occupy(blocks, ms, device=0):
    """test hook: hold `blocks` workgroups' CUs for ms milliseconds on a stream of the library's own
    (asynchronous; occupy_wait() joins it)"""
    _check(lib().mmx_occupy(int(device), int(blocks), float(ms)))


def occupy_wait():
    _check(lib().mmx_occupy_wait())
