"""The Shoulder experiment's mesh (main.cpp:403-630) against a plain restatement here: the rect mesh
without the simplices whose centroid lies in the upper quadrant, the boundary re-marking, and the
random moves of interior vertices drawn from glibc rand() after srand(69) (main.cpp:785) with Eigen
3.4's Random() = -1 + 2 rand()/RAND_MAX per coefficient.  The reference ships no Shoulder input or
output (no Experiments/InputFiles entry), and Eigen is un-vendored: parity unpinned beyond this
restatement of the listed source lines.  CPU only."""
import ctypes
import ctypes.util

import numpy as np
import pytest

import mmadmm_amd as mx

libc = ctypes.CDLL(ctypes.util.find_library("c"))
RAND_MAX = 2147483647


def restated(dim, n, btype=mx.BOUNDARY_FIXED):
    base = mx.MeshData.rect(dim, n, btype=btype)
    X = base.Xp.copy()
    F = base.F.copy()
    mask = base.mask.copy()
    c0 = (0 + 1) / 2.0
    keep = []
    for i in range(F.shape[0]):
        x = X[F[i]]
        c = [((x[0, d] + x[1, d]) + x[2, d]) * (1.0 / 3.0) if dim == 2 else
             (((x[0, d] + x[1, d]) + x[2, d]) + x[3, d]) * (1.0 / 4.0) for d in range(dim)]
        if all(c[d] > c0 for d in range(dim)):
            for v in F[i]:
                p = X[v]
                e = lambda a, b: abs(a - b) < 1e-16  # noqa: E731
                if dim == 2:
                    fixed = (e(p[0], c0) and e(p[1], c0)) or (e(p[0], c0) and e(p[1], 1.0)) or (e(p[0], 1.0) and e(p[1], c0))
                else:
                    fixed = ((e(p[0], c0) and e(p[2], c0)) or (e(p[0], c0) and e(p[2], 1.0)) or (e(p[0], 1.0) and e(p[2], c0))
                             or (e(p[1], 0.0) and e(p[2], c0)) or (e(p[1], 1.0) and e(p[2], c0))
                             or (e(p[0], c0) and e(p[1], 0.0)) or (e(p[0], c0) and e(p[1], 1.0)))
                mask[v] = mx.BOUNDARY_FIXED if fixed else btype
        else:
            keep.append(i)
    F = F[keep]
    Xc = X.copy()
    h = np.sqrt(sum((1.0 / n) ** 2 for _ in range(dim)))
    for i in range(X.shape[0]):
        if mask[i] != mx.INTERIOR:
            continue
        d = np.array([-1.0 + 2.0 * float(libc.rand()) / float(RAND_MAX) for _ in range(dim)])
        sq = 0.0
        for k in range(dim):
            sq = d[k] * d[k] if k == 0 else sq + d[k] * d[k]
        d = d / np.sqrt(sq)
        r = (h / 10.0) * float(libc.rand()) / float(RAND_MAX)
        X[i] = X[i] + r * d
    return X, Xc, F, mask


@pytest.mark.parametrize("dim,n", [(2, 8), (2, 13), (3, 4)])
def test_shoulder_matches_restatement(dim, n):
    libc.srand(69)
    m = mx.MeshData.shoulder(dim, n)
    libc.srand(69)
    X, Xc, F, mask = restated(dim, n)
    np.testing.assert_array_equal(m.F, F)
    np.testing.assert_array_equal(m.mask, mask)
    np.testing.assert_array_equal(m.Xc, Xc)
    np.testing.assert_array_equal(m.Xp, X)
    assert m.F.shape[0] < (4 if dim == 2 else 12) * n ** dim  # the quadrant is gone
    assert not np.array_equal(m.Xp, m.Xc)
