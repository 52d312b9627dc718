"""Whole reference runs on the GPU engine against the reference's committed results.

Each case is one of the reference's own experiments (tests/ref_runs.py restates its
Experiments/InputFiles/<name>.json) run through runAlgo's time loop on the device: every row of
Ih0.txt to the printed 6 digits with the same number of time steps, the final points.txt to its
print precision, and the reoriented triangles.txt exactly.  Sizes up to 205,441 nodes
(Monitor2320, Monitor1320) and 96,000 tetrahedra (3DMonitor220), so the multi-block reduction
paths, the XCD block ranges and the LDS chunk tails of the prox all meet the reference's numbers.
"""
import os

import numpy as np
import pytest

import mmadmm_amd as mx
from ref_runs import POINTS_ATOL, RUNS, SIX_DIGITS, golden_path, ih, load_txt, make_mesh, rel_err, run_trace

pytestmark = pytest.mark.gpu

CASES = ["Monitor110", "Monitor120", "3DMonitor110", "Monitor2160", "Monitor2320", "3DMonitor220", "Monitor380",
         "Monitor3160"]

# Stale artifacts: the committed trace leaves the trajectory its JSON describes after these many
# rows (the oracle, pinned elsewhere to 6 digits, leaves it at the same row; tests/test_shoulder.py,
# DESIGN.md section 5); only that prefix is a pin.
STALE_PREFIX = {"Monitor1160": 23, "Monitor1320": 23}


def _engine(name):
    mesh, mon, dt, tau, rho, gu = RUNS[name][:6]
    m = make_mesh(mesh, mx.MeshData)
    M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(m.dim, mon), rho=rho, tau=tau, gradUse=gu)
    return m, mx.Engine(M, dt)


@pytest.mark.parametrize("name", CASES)
def test_reference_run(name):
    mesh, mon, dt, tau, rho, gu, admm, dtTol, nSteps = RUNS[name]
    m, G = _engine(name)
    ours = run_trace(lambda n, t: G.step(n, t)[0], G.energy, nSteps, dt, admm, dtTol)
    ref = ih(name)
    assert len(ours) == len(ref), f"{len(ours) - 1} time steps, the reference took {len(ref) - 1}"
    assert rel_err(ours, ref) < SIX_DIGITS
    G.done()
    if os.path.exists(golden_path(name, "points.txt")):
        P = G.get("points").reshape(-1, m.dim)
        Pref = load_txt(name, "points.txt")
        assert P.shape == Pref.shape
        np.testing.assert_allclose(P, Pref, rtol=0, atol=POINTS_ATOL)
    if os.path.exists(golden_path(name, "triangles.txt")):
        np.testing.assert_array_equal(G.simplices(), load_txt(name, "triangles.txt", dtype=np.int32))
    G.close()


@pytest.mark.parametrize("name", list(STALE_PREFIX))
def test_reference_run_stale_prefix(name):
    mesh, mon, dt, tau, rho, gu, admm, dtTol, nSteps = RUNS[name]
    k = STALE_PREFIX[name]
    m, G = _engine(name)
    ours = run_trace(lambda n, t: G.step(n, t)[0], G.energy, nSteps, dt, admm, dtTol, max_steps=k - 1)
    assert rel_err(ours, ih(name)[:k]) < SIX_DIGITS
    G.close()
