"""The reference's committed experiment runs used as pins (tests/golden/, copied by
tests/golden/make_golden.py from Experiments/Results/*).  Each entry restates the run's
Experiments/InputFiles/<name>.json: the mesh (generator or BaseCircle files), MonType, dt, tau, rho,
GradUse, AdmmIter, DtTol, nSteps.  `run_trace` is runAlgo's time loop (main.cpp:172-211).

Shoulder meshes (main.cpp:403-630) draw from glibc rand() after srand(69) (main.cpp:785) and Eigen's
Random() = -1 + 2 rand()/RAND_MAX per coefficient; the t = 0 energies of Monitor110/120/1160 and
3DMonitor110 reproduce to the printed 6 digits, which pins that sequence.
"""
import ctypes
import ctypes.util
import gzip
import os
import shutil
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
SIX_DIGITS = 6e-6  # relative tolerance of a 6-significant-digit print

_libc = ctypes.CDLL(ctypes.util.find_library("c"))

# name: (mesh, MonType, dt, tau, rho, GradUse, AdmmIter, DtTol, nSteps)
# mesh = ("rect", D, n) | ("shoulder", D, n) | ("file", "CircleEx48")
RUNS = {
    "Monitor110": (("shoulder", 2, 10), 0, 0.005, 0.1, 50, True, 10, 1e-5, 1000),
    "Monitor120": (("shoulder", 2, 20), 0, 0.005, 0.1, 50, False, 10, 1e-5, 1000),
    "Monitor140": (("shoulder", 2, 40), 0, 0.005, 0.1, 50, False, 10, 1e-5, 1000),
    "Monitor1160": (("shoulder", 2, 160), 0, 0.0005, 0.1, 50, False, 10, 1e-5, 1000),
    "Monitor1320": (("shoulder", 2, 320), 0, 0.0005, 0.1, 50, False, 10, 1e-5, 1000),
    "3DMonitor110": (("shoulder", 3, 10), 0, 0.025, 10.0, 75, False, 50, 1e-5, 100),
    "Monitor2160": (("rect", 2, 160), 3, 0.055, 0.5, 50, False, 10, 1e-4, 1000),
    "Monitor2320": (("rect", 2, 320), 3, 0.055, 0.5, 50, False, 10, 1e-4, 1000),
    "3DMonitor220": (("rect", 3, 20), 3, 0.025, 0.5, 50, False, 100, 1e-5, 100),
    "Monitor380": (("file", "CircleEx48"), 5, 0.05, 0.1, 5, False, 100, 1e-5, 10000),
    "Monitor3160": (("file", "CircleEx96"), 5, 0.05, 0.1, 5, False, 100, 1e-5, 10000),
}


def golden_path(*parts):
    """Path of a golden file; a compressed copy (<file>.gz) is returned when that is what exists."""
    p = os.path.join(GOLDEN, *parts)
    return p if os.path.exists(p) else p + ".gz"


def load_txt(*parts, dtype=float):
    return np.loadtxt(golden_path(*parts), delimiter=",", dtype=dtype)


def ih(name, method=0):
    return load_txt(name, f"Ih{method}.txt")[:, 1]


def _plain_copy(src, dst):
    if src.endswith(".gz"):
        with gzip.open(src, "rb") as fi, open(dst, "wb") as fo:
            shutil.copyfileobj(fi, fo)
    else:
        shutil.copyfile(src, dst)


def file_mesh_paths(name, tmpdir):
    """(triangles, points, mask) plain-text paths of a BaseCircle mesh (decompressed into tmpdir)."""
    sub = "BaseCircle3D" if name.startswith("3D") else "BaseCircle"
    out = []
    for kind in ("triangles", "points", "mask"):
        dst = os.path.join(tmpdir, f"{name}{kind}.txt")
        _plain_copy(golden_path(sub, f"{name}{kind}.txt"), dst)
        out.append(dst)
    return out


def make_mesh(mesh, MeshData):
    """The run's initial mesh through `MeshData` (mmadmm_amd.MeshData) -> object with Xp, F, mask."""
    kind = mesh[0]
    if kind == "rect":
        return MeshData.rect(mesh[1], mesh[2])
    if kind == "shoulder":
        _libc.srand(69)  # main.cpp:785
        return MeshData.shoulder(mesh[1], mesh[2])
    with tempfile.TemporaryDirectory() as d:
        tri, pts, mask = file_mesh_paths(mesh[1], d)
        return MeshData.read(3 if mesh[1].startswith("3D") else 2, tri, pts, mask)


def mesh_dim(mesh):
    return 3 if (mesh[0] == "file" and mesh[1].startswith("3D")) else mesh[1] if mesh[0] != "file" else 2


def run_trace(step, energy, nSteps, dt, admm, dtTol, max_steps=None):
    """runAlgo's time loop (main.cpp:172-211): Ih(t=0), then step(admm, 1e-3) until
    |Ih - Ihprev| / dt < DtTol for i != 0.  step(nIters, tol) -> Ih."""
    Iv = [energy()]
    Ihprev = np.inf
    n = nSteps if max_steps is None else min(nSteps, max_steps)
    for i in range(n):
        Ih = step(admm, 1e-3)
        Iv.append(Ih)
        if i != 0 and abs((Ih - Ihprev) / dt) < dtTol:
            break
        Ihprev = Ih
    return np.array(Iv)


def rel_err(ours, ref):
    return float((np.abs(np.asarray(ours) - ref) / np.abs(ref)).max())


# Final positions are printed with 6 significant digits (default ostream precision): coordinates
# in [0, 1] carry an absolute print error <= 5e-7.  The trajectories of the reference (glibc pow,
# Eigen) and of the engine (correctly rounded pow) differ by rounding only; 2e-6 bounds both.
POINTS_ATOL = 2e-6
