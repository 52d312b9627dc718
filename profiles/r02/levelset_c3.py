"""The reference LevelSet circle at C3 size (nx = ny = 1140) on the GPU engine (bit-identical to the
oracle with correctly rounded pow): C3 parameters, 10 ADMM iterations per step, until an inverted
element is reported or 40 steps pass."""
import sys
sys.path.insert(0, 'mm-admm_amd/python')
import numpy as np
import mmadmm_amd as mx

for compact in (False, True):
    mesh = mx.MeshData.levelset2d(1140, compact_mask=compact)
    nfix = int(np.sum(np.asarray(mesh.mask) == mx.BOUNDARY_FIXED))
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5)
    G = mx.Engine(M, 0.055)
    print('compact_mask', compact, 'nodes', mesh.nP, 'simplices', len(mesh.F), 'FIXED nodes', nfix, flush=True)
    for s in range(40):
        try:
            ih, it = G.step(10, -1.0)
        except mx.InvertedElementError:
            print('  step', s, 'InvertedElementError', flush=True)
            break
        if s < 3 or s % 10 == 9:
            print('  step', s, 'Ih', ih, flush=True)
    else:
        print('  40 steps without inversion')
    G.close()
