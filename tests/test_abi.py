"""The drop-in boundary (no GPU needed): libmmadmm.so loads, exports every function the public
headers declare, and refuses compute without a GPU instead of falling back to the CPU."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mm-admm_amd", "lib", "libmmadmm.so")
HEADERS = [os.path.join(ROOT, "include", h) for h in ("mmadmm.h", "mmx_sparse.h")]


def declared(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(mm\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("libmmadmm.so is not built (run __graft_entry__.build())")
    return ctypes.CDLL(LIB)


@pytest.mark.parametrize("header", HEADERS, ids=[os.path.basename(h) for h in HEADERS])
def test_every_declared_symbol_is_exported(lib, header):
    names = declared(header)
    assert len(names) > 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_no_cpu_fallback(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib.mmadmm_last_error.restype = ctypes.c_char_p
    mesh = ctypes.c_void_p()
    assert lib.mmadmm_mesh_rect(2, 4, 4, 4, ctypes.c_double(0), ctypes.c_double(1), ctypes.c_double(0),
                                ctypes.c_double(1), ctypes.c_double(0), ctypes.c_double(1), 1,
                                ctypes.byref(mesh)) == 0  # host-side generator works
    lib.mmadmm_mesh_free(mesh)
    out = np.zeros(4)
    inp = np.ones(4)
    rc = lib.mmadmm_devmath(1, 4, inp.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 2  # MMADMM_ERR_HIP: no device, no silent CPU path
    ia = np.array([0, 1], np.int32)
    ja = np.array([0], np.int32)
    h = ctypes.c_void_p()
    rc = lib.mmx_matrix_create(0, 1, ia.ctypes.data_as(ctypes.c_void_p), ja.ctypes.data_as(ctypes.c_void_p),
                               ctypes.byref(h))
    assert rc == 2 and b"no HIP device" in lib.mmadmm_last_error()


def test_python_mirror_refuses_without_library(tmp_path):
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import mmadmm_amd\n"
            "try:\n    mmadmm_amd.lib()\nexcept ImportError:\n    sys.exit(0)\nsys.exit(3)"
            % os.path.join(ROOT, "mm-admm_amd", "python"))
    env = dict(os.environ, MMADMM_LIB=str(tmp_path / "missing.so"))
    assert subprocess.run([sys.executable, "-c", code], env=env, timeout=120).returncode == 0
