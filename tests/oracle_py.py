"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
The oracle is the CPU restatement of the reference ADMM path (see oracle/oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int_p = ctypes.POINTER(ctypes.c_int)


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_mesh_rect.restype = ctypes.c_void_p
        L.orc_mesh_rect.argtypes = [ctypes.c_int] * 4 + [ctypes.c_double] * 6 + [ctypes.c_int]
        L.orc_mesh_levelset2d.restype = ctypes.c_void_p
        L.orc_mesh_levelset2d.argtypes = [ctypes.c_int] * 2 + [ctypes.c_double] * 4 + [ctypes.c_int] * 2
        L.orc_mesh_levelset3d.restype = ctypes.c_void_p
        L.orc_mesh_levelset3d.argtypes = [ctypes.c_int] * 3 + [ctypes.c_double] * 6 + [ctypes.c_int] * 2
        L.orc_mesh_read.restype = ctypes.c_void_p
        L.orc_mesh_read.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.orc_mesh_sizes.argtypes = [ctypes.c_void_p, c_int_p, c_int_p, c_int_p]
        L.orc_mesh_copy.argtypes = [ctypes.c_void_p, c_double_p, c_int_p, c_int_p]
        L.orc_mesh_free.argtypes = [ctypes.c_void_p]
        L.orc_create.restype = ctypes.c_void_p
        L.orc_create.argtypes = [ctypes.c_int, ctypes.c_int, c_double_p, c_double_p, ctypes.c_int,
                                 c_int_p, c_int_p, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_step.restype = ctypes.c_int
        L.orc_step.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, c_double_p, c_int_p,
                               c_double_p, c_double_p]
        L.orc_euler_step.argtypes = [ctypes.c_void_p, c_double_p]
        L.orc_set_regrid.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_energy.restype = ctypes.c_double
        L.orc_energy.argtypes = [ctypes.c_void_p]
        L.orc_done.argtypes = [ctypes.c_void_p]
        L.orc_get.argtypes = [ctypes.c_void_p, ctypes.c_char_p, c_double_p]
        L.orc_get_F.argtypes = [ctypes.c_void_p, c_int_p]
        L.orc_sizes.argtypes = [ctypes.c_void_p] + [c_int_p] * 6
        L.orc_bfgs_iters.restype = ctypes.c_longlong
        L.orc_bfgs_iters.argtypes = [ctypes.c_void_p]
        L.orc_error.restype = ctypes.c_int
        L.orc_error.argtypes = [ctypes.c_void_p]
        L.orc_block_grad.restype = ctypes.c_double
        L.orc_block_grad.argtypes = [ctypes.c_void_p, ctypes.c_int, c_double_p, c_double_p, c_double_p,
                                     ctypes.c_int, ctypes.c_int, c_double_p]
        L.orc_eval_monitor.argtypes = [ctypes.c_void_p, c_double_p, c_double_p]
        L.orc_monitor_at.argtypes = [ctypes.c_int, ctypes.c_int, c_double_p, c_double_p]
        L.orc_destroy.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(c_double_p)


def _ip(a):
    return a.ctypes.data_as(c_int_p)


class Mesh:
    """A mesh from one of the reference generators (src/MeshUtils.h) or files."""

    def __init__(self, dim, Vp, F, mask):
        self.dim = dim
        self.Vp = np.ascontiguousarray(Vp, dtype=np.float64)
        self.F = np.ascontiguousarray(F, dtype=np.int32)
        self.mask = np.ascontiguousarray(mask, dtype=np.int32)

    @property
    def nP(self):
        return self.Vp.shape[0]

    @property
    def nF(self):
        return self.F.shape[0]

    @staticmethod
    def _from_handle(dim, h):
        L = lib()
        nP, nF, ml = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        L.orc_mesh_sizes(h, ctypes.byref(nP), ctypes.byref(nF), ctypes.byref(ml))
        Vp = np.zeros((nP.value, dim))
        F = np.zeros((nF.value, dim + 1), dtype=np.int32)
        mask = np.zeros(ml.value, dtype=np.int32)
        L.orc_mesh_copy(h, _dp(Vp), _ip(F), _ip(mask))
        L.orc_mesh_free(h)
        return Mesh(dim, Vp, F, mask)

    @staticmethod
    def rect(dim, n, xa=0, xb=1, ya=0, yb=1, za=0, zb=1, btype=1):
        h = lib().orc_mesh_rect(dim, n, n, n if dim == 3 else 0, xa, xb, ya, yb, za, zb, btype)
        return Mesh._from_handle(dim, h)

    @staticmethod
    def levelset2d(n, xa=0.0, xb=1.0, ya=0.0, yb=1.0, btype=1, compact_mask=True):
        h = lib().orc_mesh_levelset2d(n, n, xa, xb, ya, yb, btype, int(compact_mask))
        return Mesh._from_handle(2, h)

    @staticmethod
    def levelset3d(n, xa=0.0, xb=1.0, ya=0.0, yb=1.0, za=0.0, zb=1.0, btype=1, compact_mask=True):
        h = lib().orc_mesh_levelset3d(n, n, n, xa, xb, ya, yb, za, zb, btype, int(compact_mask))
        return Mesh._from_handle(3, h)

    @staticmethod
    def read(dim, tri, pnts, mask):
        h = lib().orc_mesh_read(dim, tri.encode(), pnts.encode(), mask.encode())
        if not h:
            raise FileNotFoundError(tri)
        return Mesh._from_handle(dim, h)


def set_threads(n):
    """OpenMP threads of the restatement's prox (process-wide)."""
    lib().orc_set_threads.argtypes = [ctypes.c_int]
    lib().orc_set_threads(int(n))


class Integrator:
    """Mesh<D> + MeshIntegrator<D> of the reference, restated on the CPU."""

    def __init__(self, mesh, monType, dt, tau, rho, gradUse=False, Vc=None, nthreads=0, cgMode=0, regrid=False):
        L = lib()
        self.dim = mesh.dim
        Vc_p = None
        if Vc is not None:
            self._Vc = np.ascontiguousarray(Vc, dtype=np.float64)
            Vc_p = _dp(self._Vc)
        mask = np.ascontiguousarray(mesh.mask[: mesh.nP], dtype=np.int32)
        self.h = L.orc_create(mesh.dim, mesh.nP, _dp(mesh.Vp), Vc_p, mesh.nF, _ip(mesh.F), _ip(mask),
                              monType, dt, tau, rho, int(gradUse), nthreads, cgMode)
        nP, nF, gr, gx, gy, gz = [ctypes.c_int() for _ in range(6)]
        L.orc_sizes(self.h, *[ctypes.byref(v) for v in (nP, nF, gr, gx, gy, gz)])
        self.nP, self.nF, self.gridRows = nP.value, nF.value, gr.value
        self.gridN = (gx.value, gy.value, gz.value)
        self.K = self.dim * (self.dim + 1)
        if regrid:  # time-varying monitor: grid rebuilt at every step start
            L.orc_set_regrid(self.h, 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_destroy(self.h)
            self.h = None

    def step(self, nIters, tol=1e-3):
        Ih, pr, du = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        it = ctypes.c_int()
        e = lib().orc_step(self.h, nIters, tol, ctypes.byref(Ih), ctypes.byref(it), ctypes.byref(pr),
                           ctypes.byref(du))
        if e:
            raise RuntimeError("oracle: inverted element (assert Edet > 0)")
        return Ih.value, it.value, pr.value, du.value

    def euler_step(self):
        Ih = ctypes.c_double()
        lib().orc_euler_step(self.h, ctypes.byref(Ih))
        return Ih.value

    def backwards_euler_step(self, dt, tol=1e-3, tree=False):
        """MeshIntegrator::backwardsEulerStep -> (Ih, Newton iterations).  tree: the GPU's
        reduction order in the CG-STAB dot products."""
        L = lib()
        L.orc_backward_euler_step.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                              c_double_p, c_int_p]
        Ih, it = ctypes.c_double(), ctypes.c_int()
        e = L.orc_backward_euler_step(self.h, dt, tol, 1 if tree else 0, ctypes.byref(Ih), ctypes.byref(it))
        if e:
            raise RuntimeError("oracle: backward Euler failed (inverted element or CG-STAB non-convergence)")
        return Ih.value, it.value

    def jacobian(self):
        """The last backward-Euler Jacobian (ia, ja, a)."""
        L = lib()
        L.orc_jacobian_nnz.argtypes = [ctypes.c_void_p]
        L.orc_jacobian_nnz.restype = ctypes.c_longlong
        L.orc_get_jacobian.argtypes = [ctypes.c_void_p, c_int_p, c_int_p, c_double_p]
        nnz = L.orc_jacobian_nnz(self.h)
        ia = np.zeros(self.dim * self.nP + 1, np.int32)
        ja = np.zeros(nnz, np.int32)
        a = np.zeros(nnz)
        L.orc_get_jacobian(self.h, ia.ctypes.data_as(c_int_p), ja.ctypes.data_as(c_int_p), a.ctypes.data_as(c_double_p))
        return ia, ja, a

    def energy(self):
        return lib().orc_energy(self.h)

    def done(self):
        lib().orc_done(self.h)

    def get(self, what):
        sizes = {"x": self.nP * self.dim, "xPrev": self.nP * self.dim, "xBar": self.nP * self.dim,
                 "points": self.nP * self.dim, "tdiag": self.nP * self.dim,
                 "z": self.nF * self.K, "u": self.nF * self.K, "hess": self.nF * self.K * self.K,
                 "grid": self.gridRows * self.dim * self.dim, "Ih": self.nF,
                 "Ehat": self.dim * self.dim}
        out = np.zeros(sizes[what])
        lib().orc_get(self.h, what.encode(), _dp(out))
        return out

    def F(self):
        out = np.zeros((self.nF, self.dim + 1), dtype=np.int32)
        lib().orc_get_F(self.h, _ip(out))
        return out

    def bfgs_iters(self):
        return lib().orc_bfgs_iters(self.h)

    def block_grad(self, sid, z, dxpu=None, computeGrad=True, regularize=False):
        z = np.ascontiguousarray(z, dtype=np.float64)
        dx = np.ascontiguousarray(dxpu if dxpu is not None else z, dtype=np.float64)
        g = np.zeros(self.K)
        igt = ctypes.c_double()
        e = lib().orc_block_grad(self.h, sid, _dp(z), _dp(dx), _dp(g), int(computeGrad), int(regularize),
                                 ctypes.byref(igt))
        return e, g, igt.value

    def eval_monitor(self, pnt):
        p = np.ascontiguousarray(pnt, dtype=np.float64)
        M = np.zeros(self.dim * self.dim)
        lib().orc_eval_monitor(self.h, _dp(p), _dp(M))
        return M


def monitor_at(dim, monType, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    M = np.zeros(dim * dim)
    lib().orc_monitor_at(dim, monType, _dp(x), _dp(M))
    return M


def set_pow_mode(mode):
    """0: glibc pow (reference semantics); 1: correctly rounded pow (bitwise GPU parity)."""
    L = lib()
    L.orc_set_pow_mode.argtypes = [ctypes.c_int]
    L.orc_set_pow_mode(int(mode))


def crpow(x, y):
    L = lib()
    L.orc_crpow.restype = ctypes.c_double
    L.orc_crpow.argtypes = [ctypes.c_double, ctypes.c_double]
    return L.orc_crpow(float(x), float(y))
