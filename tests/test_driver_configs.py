"""The reference's 36 experiment configs (Experiments/InputFiles/*.json, committed unchanged under
tests/golden/InputFiles) through the experiment driver mm-admm_amd/bin/mmadmm_run (SURVEY §8f row 1,
main.cpp:784-907), and the reference's committed traces through the driver on the GPU.

* CPU (dry run: parse the config and build the mesh on the host): every config either builds a
  mesh of exactly the size of the reference's own result files (points.txt / triangles.txt row
  counts, tests/golden/result_sizes.json), or -- when its input mesh was never committed to the
  reference (.MISSING_LARGE_BLOBS: CircleEx192, 3DCircleEx24/48/96/192) -- is reported as
  unavailable with exit status 2.
* GPU: `mmadmm_run <name> <method> 1` for every trace Ih<method>.txt of the reference whose t = 0
  row agrees with the config (methods 0, 1 and 2: ADMM, explicit Euler, backward Euler), every row
  to the printed 6 digits with the same number of time steps; the final points.txt / triangles.txt
  of the method-0 runs as well.
"""
import gzip
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(ROOT, "mm-admm_amd", "bin", "mmadmm_run")
GOLDEN = os.path.join(ROOT, "tests", "golden")
INPUTS = os.path.join(GOLDEN, "InputFiles")
CONFIGS = sorted(f[:-5] for f in os.listdir(INPUTS) if f.endswith(".json"))
SIZES = json.load(open(os.path.join(GOLDEN, "result_sizes.json")))
SIX_DIGITS = 6e-6
POINTS_ATOL = 2e-6  # see tests/ref_runs.py

# Input meshes the reference never committed: the configs that name them are unavailable
MISSING = {"3DMonitor3160", "3DMonitor3320", "3DMonitor340", "3DMonitor380", "Monitor3320"}
# 3DMonitor310's artifacts were produced with dt = tau = 0.1, rho = 0.5 (the committed JSON was
# edited after the runs; tests/test_oracle_pins.py): the GPU runs use those values
OVERRIDE = {"3DMonitor310": {"dt": 0.1, "tau": 0.1, "rho": 0.5}}
# the 3D Shoulder/SquareGrid n = 320 configs build ~170-200 M tetrahedra (8 GB of host arrays);
# their dry runs are left out of the CPU suite (MMX_DRIVER_HUGE=1 runs them)
HUGE = {"3DMonitor1320", "3DMonitor2320"}


def _plain_copy(src, dst):
    if src.endswith(".gz"):
        with gzip.open(src, "rb") as fi, open(dst[:-3], "wb") as fo:
            shutil.copyfileobj(fi, fo)
    else:
        shutil.copyfile(src, dst)


@pytest.fixture(scope="module")
def root(tmp_path_factory):
    """A reference-shaped tree: Experiments/InputFiles (the 36 configs) and the input meshes."""
    if not os.path.exists(RUN):
        pytest.fail("mmadmm_run not built (make -C mm-admm_amd)")
    r = tmp_path_factory.mktemp("ref")
    inp = r / "Experiments" / "InputFiles"
    inp.mkdir(parents=True)
    for name in CONFIGS:
        cfg = json.load(open(os.path.join(INPUTS, name + ".json")))
        cfg.update(OVERRIDE.get(name, {}))
        (inp / f"{name}.json").write_text(json.dumps(cfg, indent=4))
    for sub in ("BaseCircle", "BaseCircle3D"):
        d = r / "Experiments" / "Results" / sub
        d.mkdir(parents=True)
        for f in os.listdir(os.path.join(GOLDEN, sub)):
            _plain_copy(os.path.join(GOLDEN, sub, f), str(d / f))
    return r


def _run(root, *args, timeout=900):
    return subprocess.run([RUN, *args, "--root", str(root)], capture_output=True, text=True, timeout=timeout)


def _sizes(stdout):
    vp = [ln for ln in stdout.splitlines() if ln.startswith("size of Vp ")][0]
    f = [ln for ln in stdout.splitlines() if ln.startswith("size of F ")][0]
    return int(vp.split()[3].rstrip(",")), int(f.split()[3].rstrip(","))


@pytest.mark.parametrize("name", CONFIGS)
def test_dry_run_every_reference_config(root, name):
    if name in HUGE and not os.environ.get("MMX_DRIVER_HUGE"):
        pytest.skip("~200 M tetrahedra: MMX_DRIVER_HUGE=1")
    r = _run(root, name, "0", "1", "--dry-run")
    if name in MISSING:
        assert r.returncode == 2 and "not available" in r.stderr, (r.returncode, r.stderr)
        return
    assert r.returncode == 0, r.stderr
    nP, nF = _sizes(r.stdout)
    cfg = json.load(open(os.path.join(INPUTS, name + ".json")))
    if name in SIZES:  # the reference's own output mesh of this config
        if "points" in SIZES[name]:
            assert nP == SIZES[name]["points"]
        if "triangles" in SIZES[name]:
            assert nF == SIZES[name]["triangles"]
    elif cfg["TestType"] == "SquareGrid":  # generateUniformRectMesh: cell centres; 4 / 12 simplices per cell
        n, D = cfg["nx"], cfg["Dim"]
        assert (nP, nF) == ((n + 1) ** D + n ** D, (4 if D == 2 else 12) * n ** D)
    assert nP > 0 and nF > 0


def test_every_config_is_covered():
    assert len(CONFIGS) == 36
    covered = [n for n in CONFIGS if n in SIZES or n in MISSING]
    # configs with neither a result nor a missing mesh: the large SquareGrid/Shoulder cubes
    assert set(CONFIGS) - set(covered) <= {"3DMonitor1160", "3DMonitor1320", "3DMonitor140", "3DMonitor180",
                                           "3DMonitor2160", "3DMonitor2320", "3DMonitor240", "3DMonitor280",
                                           "3DMonitor320"}


def _golden(name, f):
    p = os.path.join(GOLDEN, name, f)
    return p if os.path.exists(p) else p + ".gz"


# (config, method): every trace Ih<method>.txt of the reference whose first row is the config's
# t = 0 energy (the SquareGrid 2x0 family's Ih1.txt files start elsewhere: older artifacts)
TRACES = sorted((n, m) for n in os.listdir(GOLDEN) if os.path.isdir(os.path.join(GOLDEN, n))
                and n in CONFIGS for m in (0, 1, 2) if os.path.exists(os.path.join(GOLDEN, n, f"Ih{m}.txt")))
# Stale artifacts (tests/test_shoulder.py): the committed trace leaves the trajectory
# its JSON describes after this many rows; only that prefix is a pin.  Run past it, the JSON's
# trajectory inverts an element (the reference would abort on assert(Edet > 0)), so the driver is
# given the config with nSteps = prefix - 1.
STALE_PREFIX = {("Monitor1160", 0): 23, ("Monitor1320", 0): 23, ("Monitor140", 0): 7, ("Monitor180", 0): 7}


@pytest.mark.gpu
@pytest.mark.parametrize("name,method", TRACES, ids=[f"{n}-m{m}" for n, m in TRACES])
def test_driver_reproduces_reference_trace(root, name, method):
    ref = np.loadtxt(os.path.join(GOLDEN, name, f"Ih{method}.txt"), delimiter=",")[:, 1]
    k = STALE_PREFIX.get((name, method))
    run = name
    if k:  # the prefix only: the same config with nSteps = k - 1
        run = f"{name}_prefix"
        cfg = json.load(open(os.path.join(INPUTS, name + ".json")))
        cfg["nSteps"] = k - 1
        (root / "Experiments" / "InputFiles" / f"{run}.json").write_text(json.dumps(cfg, indent=4))
    r = _run(root, run, str(method), "1", timeout=1100)
    assert r.returncode == 0, r.stderr[-2000:]
    out = root / "Experiments" / "Results" / run
    ours = np.loadtxt(out / f"Ih{method}.txt", delimiter=",")[:, 1]
    if k:
        ref = ref[:k]
        assert len(ours) == k
    else:
        assert len(ours) == len(ref), f"{len(ours) - 1} time steps, the reference took {len(ref) - 1}"
    rel = np.abs(ours - ref) / np.abs(ref)
    bad = np.nonzero(rel >= SIX_DIGITS)[0]
    assert rel.max() < SIX_DIGITS, f"{len(bad)} of {len(ref)} rows differ, first at row {bad[0]}: " \
                                    f"{ours[bad[0]]!r} vs {ref[bad[0]]!r} (max rel {rel.max():.3g})"
    if method == 0 and not k and os.path.exists(_golden(name, "points.txt")):
        P = np.loadtxt(out / "points.txt", delimiter=",")
        Pref = np.loadtxt(_golden(name, "points.txt"), delimiter=",")
        assert P.shape == Pref.shape
        np.testing.assert_allclose(P, Pref, rtol=0, atol=POINTS_ATOL, err_msg="final points.txt")
        if os.path.exists(_golden(name, "triangles.txt")):
            T = np.loadtxt(out / "triangles.txt", delimiter=",").astype(np.int64)
            np.testing.assert_array_equal(T, np.loadtxt(_golden(name, "triangles.txt"), delimiter=",").astype(np.int64))
