"""One source of truth for buffer-layout switches.

Round 5 reached the GPU with host code and kernels disagreeing on the 2D z/u layout (MMX_ZU_INTER
honoured by the kernels, hard-wired in engine.cpp).  Every such switch now lives in
mm-admm_amd/csrc/kernels/layout.h, each kernel object exports the layout word it was compiled with,
and the engine / the LASolver matrix compare it with their own before any HIP call.

Here (no GPU): a library whose engine.cpp is rebuilt with MMX_ZU_INTER=1 against the default kernel
objects must refuse mmadmm_create with MMADMM_ERR_INVALID and a message naming the mismatch; the
consistent library passes the same check (it then fails later, for want of a GPU)."""
import ctypes
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mm-admm_amd")
BUILD = os.path.join(PKG, "build")
OUT = os.path.join(ROOT, "tests", "_build")

_CREATE = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, %(py)r)
import mmadmm_amd as mx
L = ctypes.CDLL(%(lib)r)
w = ctypes.c_uint(0)
rc_layout = L.mmadmm_layout_check(ctypes.byref(w))
m = mx.MeshData.rect(2, 4)
p = mx.mmadmm_params(dt=0.05, tau=0.5, rho=50.0, grad_use=0, device=-1, rank=0, nranks=1, partition=0)
fn = mx.MONITOR_FN(lambda d, x, M, u: None)
h = ctypes.c_void_p()
L.mmadmm_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, mx.MONITOR_FN, ctypes.c_void_p,
                            ctypes.c_void_p]
L.mmadmm_last_error.restype = ctypes.c_char_p
Xp = np.ascontiguousarray(m.Xp, dtype=np.float64); F = np.ascontiguousarray(m.F, dtype=np.int32)
mask = np.ascontiguousarray(m.mask, dtype=np.int32)
rc = L.mmadmm_create(2, m.nP, Xp.ctypes.data, None, m.nF, F.ctypes.data, mask.ctypes.data, ctypes.byref(p), fn,
                     None, ctypes.byref(h))
print("LAYOUT", rc_layout, hex(w.value))
print("CREATE", rc, L.mmadmm_last_error().decode())
"""


def _run_create(lib):
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    r = subprocess.run([sys.executable, "-c", _CREATE % {"py": os.path.join(PKG, "python"), "lib": lib}],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = dict(ln.split(" ", 1) for ln in r.stdout.splitlines() if ln.startswith(("LAYOUT", "CREATE")))
    return out


def _mismatched_lib():
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, "libmmadmm_mismatch.so")
    eng = os.path.join(OUT, "engine_zuinter.o")
    flags = ["-std=c++17", "-O1", "-fPIC", "-ffp-contract=off", "-fopenmp", "-I" + BUILD]
    subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["-DMMX_ZU_INTER=1", "-x", "hip", "--offload-arch=gfx950", "-c",
                    os.path.join(PKG, "csrc", "host", "engine.cpp"), "-o", eng], check=True, capture_output=True)
    objs = [o for o in sorted(glob.glob(os.path.join(BUILD, "*.o"))) if os.path.basename(o) != "engine.o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fopenmp", "-o", lib] + objs + [eng] +
                   ["-Wl,-rpath,/opt/rocm/lib", "-lrccl"], check=True, capture_output=True)
    return lib


def test_consistent_library_passes_the_check():
    import mmadmm_amd as mx
    w = ctypes.c_uint(0)
    assert mx.lib().mmadmm_layout_check(ctypes.byref(w)) == 0
    assert (w.value >> 24) == 0x4d  # the word's tag


def test_mismatched_objects_fail_at_create():
    if not os.path.exists(os.path.join(BUILD, "engine.o")):
        pytest.skip("library objects not built (run __graft_entry__.build())")
    lib = _mismatched_lib()
    try:
        out = _run_create(lib)
    finally:  # a test artefact: not left in the tree (it would travel with every GPU call)
        for f in (lib, os.path.join(OUT, "engine_zuinter.o")):
            if os.path.exists(f):
                os.remove(f)
    # the LASolver side (sparse.cpp) was built with the kernels' flags: its check passes
    assert out["LAYOUT"].split()[0] == "0"
    rc, msg = out["CREATE"].split(" ", 1)
    assert int(rc) == 1, out  # MMADMM_ERR_INVALID, before any HIP call
    assert "buffer layout mismatch" in msg and "admm_kernels" in msg, msg
    # the consistent library gets past the check (then reports no GPU here, or creates on a GPU box)
    good = _run_create(os.path.join(PKG, "lib", "libmmadmm.so"))
    rc2, msg2 = good["CREATE"].split(" ", 1)
    assert "layout mismatch" not in msg2 and int(rc2) in (0, 2), good
