"""The GPU engine reproduces the reference's committed energy traces (6 significant digits)."""
import numpy as np
import pytest

import mmadmm_amd as mx
import oracle_py
from conftest import circle_mesh
from test_oracle_pins import SIX_DIGITS, TRACES, ih0

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", TRACES, ids=[t[0] for t in TRACES])
def test_gpu_energy_trace(cfg):
    name, mesh, mon, dt, tau, rho, admm, dtTol, nSteps, vc = cfg
    m = oracle_py.Mesh.rect(mesh[1], mesh[2]) if mesh[0] == "rect" else circle_mesh(mesh[1])
    M = mx.Mesh(m.Vp, m.F, m.mask, mx.BuiltinMonitor(m.dim, mon), rho=rho, tau=tau,
                Xc=m.Vp.copy() if vc else None)
    I = mx.MeshIntegrator(dt, M)
    Iv = [I.getEnergy()]
    Ihprev = np.inf
    for i in range(nSteps):  # runAlgo time loop, main.cpp:180-211
        Ih = I.step(admm, 1e-3)
        Iv.append(Ih)
        if i != 0 and abs((Ih - Ihprev) / dt) < dtTol:
            break
        Ihprev = Ih
    ref = ih0(name)
    assert len(Iv) == len(ref)
    assert (np.abs(np.array(Iv) - ref) / np.abs(ref)).max() < SIX_DIGITS
