"""mmadmm_amd -- Python mirror of connortannahill/MM-ADMM's integrator surface on libmmadmm.so.

The classes keep the reference's names and argument meaning:
  MonitorFunction          src/MonitorFunction.h:9-21 (operator()(x, M) fills the D x D tensor)
  Mesh(Xp, F, mask, Mon, numThreads, rho, w, tau, integrationMode, gradUse)
                           src/Mesh.h:22-25 (w is ignored: w = 0.5*sqrt(rho), src/Mesh.cpp:451)
  MeshIntegrator(dt, mesh) src/MeshIntegrator.h:12-51: step(nIters, tol), eulerStep(tol),
                           backwardsEulerStep(dt, tol), getEnergy(), done(), outputX/outputZ(fname), proxTime/predTime
Everything runs through the C-ABI in include/mmadmm.h; there is no CPU fallback: importing
this module fails loudly when the HIP library is missing.
"""
import ctypes
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MMADMM_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libmmadmm.so"))

MMADMM_OK = 0
BOUNDARY_FREE, BOUNDARY_FIXED, INTERIOR = 0, 1, 2

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int_p = ctypes.POINTER(ctypes.c_int32)
MONITOR_FN = ctypes.CFUNCTYPE(None, ctypes.c_int, c_double_p, c_double_p, ctypes.c_void_p)
c_ll_p = ctypes.POINTER(ctypes.c_longlong)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, c_double_p, c_double_p, ctypes.c_longlong)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, c_int_p, c_double_p, c_ll_p, c_ll_p,
                               c_double_p, c_ll_p, c_ll_p)


class mmadmm_params(ctypes.Structure):
    _fields_ = [("dt", ctypes.c_double), ("tau", ctypes.c_double), ("rho", ctypes.c_double),
                ("grad_use", ctypes.c_int), ("device", ctypes.c_int), ("rank", ctypes.c_int),
                ("nranks", ctypes.c_int), ("partition", ctypes.c_int)]


PARTITION = {"rcb": 0, "ranges": 1}  # MMADMM_PART_RCB / MMADMM_PART_RANGES


class mmadmm_stats(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_longlong), ("admm_iters", ctypes.c_longlong),
                ("bfgs_iters", ctypes.c_longlong), ("max_bfgs", ctypes.c_int),
                ("last_primal", ctypes.c_double), ("last_dual", ctypes.c_double),
                ("t_prox_ms", ctypes.c_double), ("t_xupdate_ms", ctypes.c_double),
                ("t_step_ms", ctypes.c_double), ("n_prox", ctypes.c_longlong),
                ("n_xupdate", ctypes.c_longlong), ("n_steps_timed", ctypes.c_longlong),
                ("prox_bytes", ctypes.c_double), ("xupdate_bytes", ctypes.c_double),
                ("newton_iters", ctypes.c_longlong), ("jacobians", ctypes.c_longlong),
                ("cg_iters", ctypes.c_longlong), ("t_jac_ms", ctypes.c_double), ("t_solve_ms", ctypes.c_double),
                ("t_be_ms", ctypes.c_double), ("regrids", ctypes.c_longlong), ("regrid_rows", ctypes.c_longlong),
                ("regrid_gather_bytes", ctypes.c_double), ("regrid_cand", ctypes.c_longlong),
                ("regrid_fallbacks", ctypes.c_longlong), ("monitor_iso", ctypes.c_int),
                ("t_exchange_ms", ctypes.c_double), ("n_exchange", ctypes.c_longlong),
                ("halo_send_bytes", ctypes.c_double), ("halo_recv_bytes", ctypes.c_double),
                ("interior_nodes", ctypes.c_int), ("overlap", ctypes.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class MMADMMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"mmadmm error {code}: {msg}")
        self.code = code


class InvertedElementError(MMADMMError):
    """The reference aborts on assert(Edet > 0) (src/AdaptationFunctional.cpp:174)."""


class NonFiniteEnergyError(MMADMMError):
    """MMADMM_ERR_NONFINITE: a NaN energy with no inverted element -- a monitor value that is not
    finite (on an element partition with a time-varying monitor: an evaluation outside the rank's
    rebuilt grid box)."""


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libmmadmm.so not built ({LIB_PATH}); run `make -C mm-admm_amd`")
    L = ctypes.CDLL(LIB_PATH)
    L.mmadmm_last_error.restype = ctypes.c_char_p
    L.mmadmm_builtin_monitor.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(MONITOR_FN),
                                         ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_create.argtypes = [ctypes.c_int, ctypes.c_int, c_double_p, c_double_p, ctypes.c_int, c_int_p,
                                c_int_p, ctypes.POINTER(mmadmm_params), MONITOR_FN, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_step.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, c_double_p,
                              ctypes.POINTER(ctypes.c_int)]
    L.mmadmm_euler_step.argtypes = [ctypes.c_void_p, c_double_p]
    L.mmadmm_energy.argtypes = [ctypes.c_void_p, c_double_p]
    L.mmadmm_backward_euler_step.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, c_double_p,
                                             ctypes.POINTER(ctypes.c_int)]
    L.mmadmm_get_jacobian.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), c_int_p, c_int_p,
                                      c_double_p]
    L.mmadmm_done.argtypes = [ctypes.c_void_p]
    L.mmadmm_get.argtypes = [ctypes.c_void_p, ctypes.c_char_p, c_double_p]
    L.mmadmm_get_simplices.argtypes = [ctypes.c_void_p, c_int_p]
    L.mmadmm_sizes.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int)] * 3
    L.mmadmm_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.mmadmm_stats_get.argtypes = [ctypes.c_void_p, ctypes.POINTER(mmadmm_stats)]
    L.mmadmm_stats_reset.argtypes = [ctypes.c_void_p]
    L.mmadmm_sync.argtypes = [ctypes.c_void_p]
    L.mmadmm_regrid.argtypes = [ctypes.c_void_p, ctypes.c_double]
    L.mmadmm_set_regrid.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.mmadmm_destroy.argtypes = [ctypes.c_void_p]
    L.mmadmm_mesh_rect.argtypes = [ctypes.c_int] * 4 + [ctypes.c_double] * 6 + [ctypes.c_int,
                                                                                 ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_mesh_levelset2d.argtypes = [ctypes.c_int] * 2 + [ctypes.c_double] * 4 + [
        ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_mesh_levelset3d.argtypes = [ctypes.c_int] * 3 + [ctypes.c_double] * 6 + [
        ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_mesh_hexdisc.argtypes = [ctypes.c_int] + [ctypes.c_double] * 3 + [ctypes.c_int,
                                                                               ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_mesh_shoulder.argtypes = [ctypes.c_int] * 4 + [ctypes.c_double] * 6 + [ctypes.c_int,
                                                                                     ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_mesh_reference_points.argtypes = [ctypes.c_void_p, c_double_p]
    L.mmadmm_mesh_read.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_void_p)]
    L.mmadmm_mesh_sizes.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int)] * 4
    L.mmadmm_mesh_copy.argtypes = [ctypes.c_void_p, c_double_p, c_int_p, c_int_p]
    L.mmadmm_mesh_free.argtypes = [ctypes.c_void_p]
    L.mmadmm_write_points.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, c_double_p]
    L.mmadmm_write_simplices.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, c_int_p]
    L.mmadmm_debug_blockgrad.argtypes = [ctypes.c_void_p, ctypes.c_int, c_double_p, c_double_p, ctypes.c_int,
                                         c_double_p]
    L.mmadmm_devmath.argtypes = [ctypes.c_int, ctypes.c_int, c_double_p, c_double_p]
    vp = ctypes.c_void_p
    L.mmadmm_comm_unique_id.argtypes = [vp, ctypes.c_int]
    L.mmadmm_comm_create_rccl.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.POINTER(vp)]
    L.mmadmm_comm_create_rccl_timeout.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_double,
                                                  ctypes.POINTER(vp)]
    L.mmadmm_comm_create_loopback.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.mmadmm_comm_destroy.argtypes = [vp]
    L.mmadmm_comm_nranks.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.mmadmm_build_info.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.mmadmm_comm_create_host.argtypes = [ctypes.c_int, ctypes.c_int, ALLGATHER_FN, EXCHANGE_FN, vp, ctypes.POINTER(vp)]
    L.mmadmm_be_begin.argtypes = [vp, ctypes.c_double, c_double_p]
    L.mmadmm_be_residual.argtypes = [vp, ctypes.c_double, c_double_p, c_double_p, c_double_p]
    L.mmadmm_be_fsubjac.argtypes = [vp, c_double_p]
    L.mmadmm_be_add.argtypes = [vp, c_double_p]
    L.mmadmm_create_partitioned.argtypes = [ctypes.c_int, ctypes.c_int, c_double_p, c_double_p, ctypes.c_int, c_int_p,
                                            c_int_p, ctypes.POINTER(mmadmm_params), MONITOR_FN, vp, vp,
                                            ctypes.POINTER(vp)]
    L.mmadmm_local_nodes.argtypes = [vp, ctypes.POINTER(ctypes.c_int), c_int_p]
    L.mmadmm_plan_create.argtypes = [ctypes.c_int, ctypes.c_int, c_double_p, ctypes.c_int, c_int_p, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.mmadmm_plan_sizes.argtypes = [vp] + [ctypes.POINTER(ctypes.c_int)] * 7
    L.mmadmm_plan_get.argtypes = [vp] + [c_int_p] * 6
    L.mmadmm_plan_destroy.argtypes = [vp]
    _lib = L
    return L


def build_info():
    """{"src_hash": ..., "git": ..., "arch": ...} embedded in libmmadmm.so at build time"""
    buf = ctypes.create_string_buffer(256)
    _check(lib().mmadmm_build_info(buf, 256))
    return dict(kv.split("=", 1) for kv in buf.value.decode().split())


def _close_at_exit(obj):
    """__del__ of a handle owner: close it, unless the interpreter is tearing down (module globals
    such as the ctypes library may already be gone; the process exit releases the device)."""
    try:
        obj.close()
    except (TypeError, AttributeError, NameError):
        pass


def _check(rc):
    if rc != MMADMM_OK:
        msg = lib().mmadmm_last_error().decode(errors="replace")
        if rc == 3:
            raise InvertedElementError(rc, msg)
        if rc == 7:
            raise NonFiniteEnergyError(rc, msg)
        raise MMADMMError(rc, msg)


def _dp(a):
    return a.ctypes.data_as(c_double_p)


def _ip(a):
    return a.ctypes.data_as(c_int_p)


# ---------------------------------------------------------------- meshes (src/MeshUtils.h)
class MeshData:
    """Vertices Xp (nP x D), simplices F (nF x D+1), node mask (NodeType values)."""

    def __init__(self, dim, Xp, F, mask):
        self.dim = dim
        self.Xp = np.ascontiguousarray(Xp, dtype=np.float64)
        self.F = np.ascontiguousarray(F, dtype=np.int32)
        self.mask = np.ascontiguousarray(mask, dtype=np.int32)

    @property
    def nP(self):
        return self.Xp.shape[0]

    @property
    def nF(self):
        return self.F.shape[0]

    @staticmethod
    def _take(h):
        L = lib()
        d, nP, nF, ml = (ctypes.c_int() for _ in range(4))
        _check(L.mmadmm_mesh_sizes(h, ctypes.byref(d), ctypes.byref(nP), ctypes.byref(nF), ctypes.byref(ml)))
        Xp = np.zeros((nP.value, d.value))
        F = np.zeros((nF.value, d.value + 1), dtype=np.int32)
        mask = np.zeros(ml.value, dtype=np.int32)
        _check(L.mmadmm_mesh_copy(h, _dp(Xp), _ip(F), _ip(mask)))
        Xc = np.zeros_like(Xp)
        _check(L.mmadmm_mesh_reference_points(h, _dp(Xc)))
        L.mmadmm_mesh_free(h)
        m = MeshData(d.value, Xp, F, mask)
        m.Xc = Xc  # reference positions (CompMesh): equal to Xp except for Shoulder meshes
        return m

    @staticmethod
    def shoulder(dim, n, xa=0, xb=1, ya=0, yb=1, za=0, zb=1, btype=BOUNDARY_FIXED):
        """setUpShoulderExperiment's mesh (main.cpp:403-630); draws from the C library's rand()
        (seed with srand(69) for the reference's sequence, main.cpp:785)."""
        h = ctypes.c_void_p()
        _check(lib().mmadmm_mesh_shoulder(dim, n, n, n if dim == 3 else 0, xa, xb, ya, yb, za, zb, btype,
                                          ctypes.byref(h)))
        return MeshData._take(h)

    @staticmethod
    def rect(dim, n, xa=0, xb=1, ya=0, yb=1, za=0, zb=1, btype=BOUNDARY_FIXED):
        h = ctypes.c_void_p()
        _check(lib().mmadmm_mesh_rect(dim, n, n, n if dim == 3 else 0, xa, xb, ya, yb, za, zb, btype,
                                      ctypes.byref(h)))
        return MeshData._take(h)

    @staticmethod
    def levelset2d(n, xa=0.0, xb=1.0, ya=0.0, yb=1.0, btype=BOUNDARY_FIXED, compact_mask=True):
        h = ctypes.c_void_p()
        _check(lib().mmadmm_mesh_levelset2d(n, n, xa, xb, ya, yb, btype, int(compact_mask), ctypes.byref(h)))
        return MeshData._take(h)

    @staticmethod
    def levelset3d(n, xa=0.0, xb=1.0, ya=0.0, yb=1.0, za=0.0, zb=1.0, btype=BOUNDARY_FIXED, compact_mask=True):
        """utils::meshFromLevelSetFun 3D with spherePhi (src/MeshUtils.h:540-667, main.cpp:87-97)."""
        h = ctypes.c_void_p()
        _check(lib().mmadmm_mesh_levelset3d(n, n, n, xa, xb, ya, yb, za, zb, btype, int(compact_mask),
                                            ctypes.byref(h)))
        return MeshData._take(h)

    @staticmethod
    def hexdisc(N, r=0.5, cx=0.5, cy=0.5, btype=BOUNDARY_FIXED):
        h = ctypes.c_void_p()
        _check(lib().mmadmm_mesh_hexdisc(N, r, cx, cy, btype, ctypes.byref(h)))
        return MeshData._take(h)

    @staticmethod
    def read(dim, tri, pnts, mask):
        h = ctypes.c_void_p()
        _check(lib().mmadmm_mesh_read(dim, tri.encode(), pnts.encode(), mask.encode(), ctypes.byref(h)))
        return MeshData._take(h)


def write_points(path, Xp):
    Xp = np.ascontiguousarray(Xp, dtype=np.float64)
    _check(lib().mmadmm_write_points(path.encode(), Xp.shape[1], Xp.shape[0], _dp(Xp)))


def write_simplices(path, F):
    F = np.ascontiguousarray(F, dtype=np.int32)
    _check(lib().mmadmm_write_simplices(path.encode(), F.shape[1] - 1, F.shape[0], _ip(F)))


# ---------------------------------------------------------------- monitors
class MonitorFunction:
    """User monitor (src/MonitorFunction.h:13): override __call__(x, M) to fill M (D x D)."""

    dim = 2

    def __call__(self, x, M):
        raise NotImplementedError

    def _cfunc(self):
        def tramp(dim, xp, Mp, _user):
            x = np.ctypeslib.as_array(xp, shape=(dim,))
            M = np.ctypeslib.as_array(Mp, shape=(dim, dim))
            self(x, M)

        self._keep = MONITOR_FN(tramp)
        return self._keep, None


class BuiltinMonitor(MonitorFunction):
    """Experiments/TestMonitors/MEx* by MonType (main.cpp:836-864), evaluated natively."""

    def __init__(self, dim, mon_type):
        self.dim = dim
        self.mon_type = mon_type

    def _cfunc(self):
        fn = MONITOR_FN()
        user = ctypes.c_void_p()
        _check(lib().mmadmm_builtin_monitor(self.dim, self.mon_type, ctypes.byref(fn), ctypes.byref(user)))
        return fn, user


# ---------------------------------------------------------------- Mesh<D> / MeshIntegrator<D>
class Mesh:
    """Mesh<D> (src/Mesh.h:16-126).  Holds the problem; the device state is created by
    MeshIntegrator, which knows dt (src/MeshIntegrator.cpp:15-62)."""

    def __init__(self, Xp, F, boundaryMask, Mon, numThreads=1, rho=50.0, w=None, tau=0.5,
                 integrationMode=0, gradUse=False, Xc=None, device=-1):
        self.Xp = np.ascontiguousarray(Xp, dtype=np.float64)
        self.dim = self.Xp.shape[1]
        self.F = np.ascontiguousarray(F, dtype=np.int32)
        self.mask = np.ascontiguousarray(np.asarray(boundaryMask)[: self.Xp.shape[0]], dtype=np.int32)
        self.Mon = Mon
        self.numThreads = numThreads
        self.rho = float(rho)
        self.w = 0.5 * np.sqrt(self.rho)  # src/Mesh.cpp:451 ignores the w argument
        self.tau = float(tau)
        self.integrationMode = integrationMode
        self.gradUse = bool(gradUse)
        self.Xc = None if Xc is None else np.ascontiguousarray(Xc, dtype=np.float64)
        self.device = device


UNIQUE_ID_BYTES = 128


class Comm:
    """Communicator of an element-partitioned run: RCCL between processes (one per GPU) or a
    loopback shared by the engines of one process (driven from threads; tests)."""

    def __init__(self, h):
        self.h = h

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        _check(lib().mmadmm_comm_unique_id(buf, UNIQUE_ID_BYTES))
        return buf.raw

    @staticmethod
    def rccl(nranks, rank, uid, device, timeout_s=None):
        """RCCL communicator (collective over the ranks).  timeout_s bounds its creation and every
        wait of a partitioned step (default: MMX_COMM_TIMEOUT_S, else 300 s; <= 0: none): a rank
        that never joins or stops makes the others fail with MMADMM_ERR_RCCL, not hang."""
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), UNIQUE_ID_BYTES)
        if timeout_s is None:
            _check(lib().mmadmm_comm_create_rccl(int(nranks), int(rank), buf, int(device), ctypes.byref(h)))
        else:
            _check(lib().mmadmm_comm_create_rccl_timeout(int(nranks), int(rank), buf, int(device),
                                                         ctypes.c_double(float(timeout_s)), ctypes.byref(h)))
        return Comm(h)

    @staticmethod
    def loopback(nranks):
        h = ctypes.c_void_p()
        _check(lib().mmadmm_comm_create_loopback(int(nranks), ctypes.byref(h)))
        return Comm(h)

    @staticmethod
    def host(nranks, rank, transport):
        """A communicator over the caller's host transport (one process per rank; `transport` has
        allgather(send, recv) and exchange(peers, sends, recvs) on numpy arrays, e.g.
        TorchDistTransport over a gloo process group): the engine stages its blocks through pinned
        host memory and calls the transport in the same order on every rank.

        Failure: a transport call that raises is reported to that rank's engine as MMADMM_ERR_RCCL,
        and the transport's abort() (if it has one) is called first, so that the other ranks, blocked
        in the same collective, fail too instead of waiting forever.  TorchDistTransport.abort ends
        the gloo process group; without an abort the caller must tear down every rank when any rank
        reports MMADMM_ERR_RCCL."""

        def ag(_user, send, recv, count):
            try:
                n = int(count)
                s = np.ctypeslib.as_array(send, shape=(max(n, 1),))[:n]
                r = np.ctypeslib.as_array(recv, shape=(max(n * nranks, 1),))[: n * nranks]
                transport.allgather(s, r)
                return 0
            except BaseException:  # noqa: BLE001 -- reported to the engine as a status
                import traceback
                traceback.print_exc()
                _abort(transport)
                return 1

        def ex(_user, npeers, peer, send, so, sc, recv, ro, rc):
            try:
                peers, sends, recvs = [], [], []
                for i in range(npeers):
                    peers.append(int(peer[i]))
                    n_s, n_r = int(sc[i]), int(rc[i])
                    sends.append(np.ctypeslib.as_array(ctypes.cast(ctypes.byref(send.contents, 8 * int(so[i])),
                                                                   c_double_p), shape=(max(n_s, 1),))[:n_s])
                    recvs.append(np.ctypeslib.as_array(ctypes.cast(ctypes.byref(recv.contents, 8 * int(ro[i])),
                                                                   c_double_p), shape=(max(n_r, 1),))[:n_r])
                transport.exchange(peers, sends, recvs)
                return 0
            except BaseException:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                _abort(transport)
                return 1

        cag, cex = ALLGATHER_FN(ag), EXCHANGE_FN(ex)
        h = ctypes.c_void_p()
        _check(lib().mmadmm_comm_create_host(int(nranks), int(rank), cag, cex, None, ctypes.byref(h)))
        c = Comm(h)
        c._keep = (cag, cex, transport)  # the callbacks must outlive the communicator
        return c

    def nranks(self):
        """ranks as the transport reports them (RCCL: ncclCommCount)"""
        n = ctypes.c_int()
        _check(lib().mmadmm_comm_nranks(self.h, ctypes.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "h", None):
            lib().mmadmm_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            _close_at_exit(self)
        except TypeError:  # interpreter shutdown: the module's globals are gone
            pass


def _abort(transport):
    ab = getattr(transport, "abort", None)
    if ab is not None:
        try:
            ab()
        except BaseException:  # noqa: BLE001 -- best effort: the status is reported either way
            pass


class TorchDistTransport:
    """Host transport over an initialised torch.distributed CPU process group (gloo): all_gather
    for the block all-gathers, tagged isend/irecv with the neighbouring ranks for the halo
    exchange (messages matched by the engine's call order, which is the same on every rank)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.world = dist.get_world_size(group)
        self.calls = 0
        self.bytes_sent = 0

    def allgather(self, send, recv):
        t = self.torch
        n = send.size
        out = t.from_numpy(recv).view(self.world, n) if n else None
        if n:
            self.dist.all_gather(list(out.unbind(0)), t.from_numpy(send.copy()), group=self.group)
            self.bytes_sent += 8 * n

    def exchange(self, peers, sends, recvs):
        t, d = self.torch, self.dist
        tag = self.calls % (1 << 20)
        self.calls += 1
        reqs = []
        for q, s, r in zip(peers, sends, recvs):
            if s.size:
                reqs.append(d.isend(t.from_numpy(s.copy()), q, group=self.group, tag=tag))
                self.bytes_sent += 8 * s.size
            if r.size:
                reqs.append(d.irecv(t.from_numpy(r), q, group=self.group, tag=tag))
        for q in reqs:
            q.wait()

    def abort(self):
        """End the process group (Comm.host calls this when a transfer failed on this rank): the
        ranks blocked in a collective or a receive with this one then fail instead of hanging."""
        self.dist.destroy_process_group(self.group)


def partition_plan(dim, Xp, F, nranks, rank, method="rcb"):
    """The element partition of rank `rank` (host only) -> dict of numpy arrays: localNodes,
    localSimplices (global ids, ascending), incPtr/incSrc (per local node its incident slot sources
    in ascending global simplex order: >= 0 local slot offset, < 0 row -1-src of the receive
    buffer), sendOff (local slot offsets sent, per peer), peers (rows: rank, rows sent, rows
    received), recvRows, interfaceNodes."""
    L = lib()
    Xp = np.ascontiguousarray(Xp, dtype=np.float64).reshape(-1, dim)
    F = np.ascontiguousarray(F, dtype=np.int32)
    h = ctypes.c_void_p()
    _check(L.mmadmm_plan_create(int(dim), Xp.shape[0], _dp(Xp), len(F), _ip(F), int(nranks), int(rank),
                                PARTITION[method], ctypes.byref(h)))
    try:
        v = [ctypes.c_int() for _ in range(7)]
        _check(L.mmadmm_plan_sizes(h, *[ctypes.byref(x) for x in v]))
        nl, nfl, ns, nsend, nrecv, npeers, nif = [x.value for x in v]
        out = dict(localNodes=np.zeros(nl, np.int32), localSimplices=np.zeros(nfl, np.int32),
                   incPtr=np.zeros(nl + 1, np.int32), incSrc=np.zeros(ns, np.int32), sendOff=np.zeros(nsend, np.int32),
                   peers=np.zeros((npeers, 3), np.int32))
        _check(L.mmadmm_plan_get(h, *[_ip(out[k]) for k in ("localNodes", "localSimplices", "incPtr", "incSrc",
                                                             "sendOff", "peers")]))
        out.update(recvRows=nrecv, interfaceNodes=nif)
        return out
    finally:
        L.mmadmm_plan_destroy(h)


class Engine:
    """Direct handle on one libmmadmm integrator (what MeshIntegrator wraps)."""

    def __init__(self, mesh, dt, rank=0, nranks=1, comm=None, partition="rcb"):
        """rank/nranks/comm: element-partitioned run (include/mmadmm.h); `mesh` is the global mesh
        on every rank and this engine owns the simplices the partition ("rcb": recursive coordinate
        bisection of the centroids; "ranges": contiguous id ranges) gives rank `rank`."""
        L = lib()
        p = mmadmm_params(dt=float(dt), tau=mesh.tau, rho=mesh.rho, grad_use=int(mesh.gradUse),
                          device=mesh.device, rank=int(rank), nranks=int(nranks), partition=PARTITION[partition])
        fn, user = mesh.Mon._cfunc()
        self._fn = fn
        h = ctypes.c_void_p()
        Xc = _dp(mesh.Xc) if mesh.Xc is not None else None
        if nranks == 1 and comm is None:
            _check(L.mmadmm_create(mesh.dim, mesh.Xp.shape[0], _dp(mesh.Xp), Xc, mesh.F.shape[0], _ip(mesh.F),
                                   _ip(mesh.mask), ctypes.byref(p), fn, user, ctypes.byref(h)))
        else:
            _check(L.mmadmm_create_partitioned(mesh.dim, mesh.Xp.shape[0], _dp(mesh.Xp), Xc, mesh.F.shape[0],
                                               _ip(mesh.F), _ip(mesh.mask), ctypes.byref(p), fn, user,
                                               comm.h if comm is not None else None, ctypes.byref(h)))
        self.h = h
        self.comm = comm
        self.dim = mesh.dim
        nP, nF, gr = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(L.mmadmm_sizes(h, ctypes.byref(nP), ctypes.byref(nF), ctypes.byref(gr)))
        self.nP, self.nF, self.gridRows = nP.value, nF.value, gr.value
        self.K = self.dim * (self.dim + 1)

    def local_nodes(self):
        """Global ids of this engine's nodes (all nodes for a single-GPU engine)."""
        ids = np.zeros(self.nP, dtype=np.int32)
        _check(lib().mmadmm_local_nodes(self.h, None, _ip(ids)))
        return ids

    def close(self):
        if getattr(self, "h", None):
            lib().mmadmm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            _close_at_exit(self)
        except TypeError:  # interpreter shutdown: the module's globals are gone
            pass

    def step(self, nIters, tol=1e-3):
        Ih = ctypes.c_double()
        it = ctypes.c_int()
        _check(lib().mmadmm_step(self.h, nIters, tol, ctypes.byref(Ih), ctypes.byref(it)))
        return Ih.value, it.value

    def euler_step(self):
        Ih = ctypes.c_double()
        _check(lib().mmadmm_euler_step(self.h, ctypes.byref(Ih)))
        return Ih.value

    def backwards_euler_step(self, dt, tol=1e-3):
        """Mesh::backwardsEulerStep (src/Mesh.cpp:1263-1341) -> (Ih, Newton iterations)."""
        Ih = ctypes.c_double()
        it = ctypes.c_int()
        _check(lib().mmadmm_backward_euler_step(self.h, dt, tol, ctypes.byref(Ih), ctypes.byref(it)))
        return Ih.value, it.value

    def jacobian(self):
        """The last backward-Euler Jacobian as CSR (ia, ja, a)."""
        nnz = ctypes.c_longlong()
        _check(lib().mmadmm_get_jacobian(self.h, ctypes.byref(nnz), None, None, None))
        ia = np.zeros(self.nP * self.dim + 1, dtype=np.int32)
        ja = np.zeros(nnz.value, dtype=np.int32)
        a = np.zeros(nnz.value)
        _check(lib().mmadmm_get_jacobian(self.h, None, _ip(ia), _ip(ja), _dp(a)))
        return ia, ja, a

    def energy(self):
        E = ctypes.c_double()
        _check(lib().mmadmm_energy(self.h, ctypes.byref(E)))
        return E.value

    def done(self):
        _check(lib().mmadmm_done(self.h))

    def get(self, what):
        n = {"x": self.nP * self.dim, "xPrev": self.nP * self.dim, "xBar": self.nP * self.dim,
             "points": self.nP * self.dim, "z": self.nF * self.K, "u": self.nF * self.K,
             "hess": self.nF * self.K * self.K, "gs": self.nF * self.K, "grid": self.gridRows * self.dim * self.dim,
             "Ehat": self.dim * self.dim}[what]
        out = np.zeros(n)
        _check(lib().mmadmm_get(self.h, what.encode(), _dp(out)))
        return out

    def simplices(self):
        F = np.zeros((self.nF, self.dim + 1), dtype=np.int32)
        _check(lib().mmadmm_get_simplices(self.h, _ip(F)))
        return F

    def set_timing(self, on):
        _check(lib().mmadmm_set_timing(self.h, int(on)))

    def stats(self):
        s = mmadmm_stats()
        _check(lib().mmadmm_stats_get(self.h, ctypes.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        _check(lib().mmadmm_stats_reset(self.h))

    def sync(self):
        _check(lib().mmadmm_sync(self.h))

    def regrid(self, t):
        """Rebuild the monitor grid on the device from the current mesh at time t (the reference's
        commented Mesh::setUp hook, src/Mesh.cpp:1006-1014)."""
        _check(lib().mmadmm_regrid(self.h, t))

    def set_regrid(self, every_step=True):
        """Time-varying monitor: rebuild the grid at the start of every step, t = steps * dt."""
        _check(lib().mmadmm_set_regrid(self.h, 1 if every_step else 0))

    def block_grad(self, sid, z, dxpu=None, computeGrad=True, regularize=False):
        """Device Mesh::computeBlockGrad of one simplex -> (energy, grad, Igt)."""
        z = np.ascontiguousarray(z, dtype=np.float64)
        dx = np.ascontiguousarray(dxpu if dxpu is not None else z, dtype=np.float64)
        out = np.zeros(self.K + 2)
        _check(lib().mmadmm_debug_blockgrad(self.h, sid, _dp(z), _dp(dx),
                                            int(computeGrad) | (2 * int(regularize)), _dp(out)))
        return out[0], out[2:], out[1]


class MeshIntegrator:
    """MeshIntegrator<D> (src/MeshIntegrator.h:12-51)."""

    def __init__(self, dt, a):
        self.a = a
        self.dt = float(dt)
        self.engine = Engine(a, dt)
        self.proxTime = 0.0
        self.predTime = 0.0
        self.stepsTaken = 0

    def step(self, nIters, tol):
        t0 = time.perf_counter()
        Ih, _ = self.engine.step(nIters, tol)
        self.proxTime += time.perf_counter() - t0
        self.stepsTaken += 1
        return Ih

    def eulerStep(self, tol=1e-3):
        return self.engine.euler_step()

    def backwardsEulerStep(self, dt, tol):
        return self.engine.backwards_euler_step(dt, tol)[0]

    def getEnergy(self):
        return self.engine.energy()

    def done(self):
        self.engine.done()

    def outputX(self, fname):
        write_points(fname, self.engine.get("x").reshape(-1, self.a.dim))

    def outputZ(self, fname):
        write_points(fname, self.engine.get("z").reshape(-1, self.a.dim))


def devmath(op, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    _check(lib().mmadmm_devmath(op, x.size, _dp(x), _dp(out)))
    return out
