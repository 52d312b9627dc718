"""Built-in monitor plugins of libmmadmm (host code, evaluated once at set-up) against the
oracle's restatement of Experiments/TestMonitors/MEx*.h and of the build's MonType 6
anisotropic shell (no reference counterpart).  CPU only: the monitors never touch the GPU."""
import ctypes

import numpy as np
import pytest

import mmadmm_amd as mx
import oracle_py

def product_monitor(dim, mon):
    fn, user = mx.MONITOR_FN(), ctypes.c_void_p()
    assert mx.lib().mmadmm_builtin_monitor(dim, mon, ctypes.byref(fn), ctypes.byref(user)) == 0
    f = fn

    def ev(x):
        xa = np.ascontiguousarray(x, dtype=np.float64)
        M = np.zeros(dim * dim)
        f(dim, xa.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), M.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
          user.value)
        return M
    return ev


@pytest.mark.parametrize("dim,mon", [(d, m) for d in (2, 3) for m in range(8)])
def test_builtin_monitor_matches_oracle(dim, mon):
    rng = np.random.default_rng(10 * dim + mon)
    ev = product_monitor(dim, mon)
    for x in rng.uniform(-0.1, 1.1, (200, dim)):
        np.testing.assert_array_equal(ev(x), oracle_py.monitor_at(dim, mon, x))


def test_aniso_shell_is_anisotropic():
    ev = product_monitor(3, 6)
    M = ev(np.array([0.8, 0.5, 0.5])).reshape(3, 3)  # on the shell, normal along x
    w = np.linalg.eigvalsh(M)  # MEx2-style: lam1 = 1 + sech(0) = 2 along n, 1/lam1 across
    np.testing.assert_allclose(w, [0.5, 0.5, 2.0])
    np.testing.assert_allclose(M @ np.array([1.0, 0, 0]), [2.0, 0, 0])


def test_builtin_monitor_range_checked():
    fn, user = mx.MONITOR_FN(), ctypes.c_void_p()
    assert mx.lib().mmadmm_builtin_monitor(3, 8, ctypes.byref(fn), ctypes.byref(user)) != 0
