"""Generate the LASolver golden fixtures (tests/golden/lasolver/*.npz) from the reference itself.

Run in the build container after `make -f oracle/Makefile.ref` has compiled the reference's
lib/LASolver sources in place into oracle/_ref/liblasolver_ref.so.  Each fixture holds data only:
the packed pattern (MatrixStruc::pack of buildMatrix's set_entry stream), seeded values, the
right-hand side, and the reference's outputs: matmult(a, b), the numeric ILU(0) factor, the ILU
solve of b, and MatrixIter::solve's x / nitr after 1, 2, 3 iterations and to convergence.

Cases: Jacobian patterns of 2D SquareGrid n=4 and n=9 and 3D n=2 with diagonally
shifted random values (converging in a few iterations), a hard case that needs hundreds of
iterations, one that does not converge within nitmax, an initial guess with new_rhat = 1, a zero
right-hand side (the reference returns NaN, 0/0 in alpha), and the tridiagonal probe (ILU(0) exact).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import lasolver_py as L  # noqa: E402
import oracle_py  # noqa: E402

OUT = os.path.join(HERE, "lasolver")


def jac_pattern(dim, n):
    m = oracle_py.Mesh.rect(dim, n)
    rows, cols = L.mesh_entries(dim, m.F)
    N = dim * m.nP
    return L.pack(N, rows, cols, use_ref=True)


def tridiag(n):
    rows = np.concatenate([np.arange(1, n), np.arange(0, n - 1)])
    cols = np.concatenate([np.arange(0, n - 1), np.arange(1, n)])
    return L.pack(n, rows, cols, use_ref=True)


CASES = [
    # name, pattern, value seed, diagonal shift, rhs seed, resid_reduc, nitmax, new_rhat, x0 seed
    ("rect2d_4_easy", lambda: jac_pattern(2, 4), 2, 0.6, 102, 1e-6, 10000, 0, None),
    ("rect2d_9_tight", lambda: jac_pattern(2, 9), 4, 0.3, 104, 1e-10, 10000, 0, None),
    ("rect3d_2_easy", lambda: jac_pattern(3, 2), 1, 1.2, 101, 1e-6, 10000, 0, None),
    ("rect2d_4_hard", lambda: jac_pattern(2, 4), 3, None, 103, 1e-6, 10000, 0, None),
    ("rect2d_9_noconv", lambda: jac_pattern(2, 9), 3, None, 103, 1e-6, 200, 0, None),
    ("rect3d_2_x0_rhat", lambda: jac_pattern(3, 2), 4, 0.3, 104, 1e-6, 10000, 1, 105),
    ("rect2d_4_zero_rhs", lambda: jac_pattern(2, 4), 2, 0.6, None, 1e-6, 10000, 0, None),
    ("tridiag_1000", lambda: tridiag(1000), 5, 1.0, 106, 1e-6, 10000, 0, None),
]


def make(name, pat, vseed, shift, bseed, rr, nitmax, new_rhat, x0seed):
    ia, ja = pat()
    n = len(ia) - 1
    a = L.random_values(ia, ja, vseed, shift)
    b = np.zeros(n) if bseed is None else np.random.default_rng(bseed).uniform(-1.0, 1.0, n)
    x0 = None if x0seed is None else np.random.default_rng(x0seed).uniform(-1.0, 1.0, n)
    iaf, jaf, af, diag = L.ref_ilu(ia, ja, a)
    assert np.array_equal(iaf, ia) and np.array_equal(jaf, ja), "level-0 ILU pattern must equal A's"
    out = dict(ia=ia, ja=ja, a=a, b=b, resid_reduc=np.float64(rr), nitmax=np.int32(nitmax),
               new_rhat=np.int32(new_rhat), af=af, diag=diag,
               matmult_b=L.matmult(ia, ja, a, b, use_ref=True), ilu_solve_b=L.ref_ilu_solve(ia, ja, a, b))
    if x0 is not None:
        out["x0"] = x0
    for k in (1, 2, 3):
        x, it, _ = L.solve(ia, ja, a, b, nitmax=min(k, nitmax), resid_reduc=rr, new_rhat=new_rhat, x0=x0,
                           use_ref=True)
        out[f"x_it{k}"] = x
        out[f"nitr_it{k}"] = np.int32(it)
    x, it, _ = L.solve(ia, ja, a, b, nitmax=nitmax, resid_reduc=rr, new_rhat=new_rhat, x0=x0, use_ref=True)
    out["x"] = x
    out["nitr"] = np.int32(it)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    return n, len(ja), it


def make_levels():
    """Level-of-fill ILU(k) factors (sfac2 + factor) at levels 1 and 2 on a 2D n=6 and a 3D n=2
    Jacobian pattern: pins the symbolic restatement and the numeric factor with fill-in."""
    out = {}
    for tag, (dim, n) in (("d2", (2, 6)), ("d3", (3, 2))):
        ia, ja = jac_pattern(dim, n)
        a = L.random_values(ia, ja, 21, 0.4)
        b = np.random.default_rng(22).uniform(-1.0, 1.0, len(ia) - 1)
        out[f"{tag}_ia"], out[f"{tag}_ja"], out[f"{tag}_a"], out[f"{tag}_b"] = ia, ja, a, b
        for lev in (1, 2):
            iaf, jaf, af, diag = L.ref_ilu(ia, ja, a, level=lev)
            out[f"{tag}_l{lev}_iaf"], out[f"{tag}_l{lev}_jaf"] = iaf, jaf
            out[f"{tag}_l{lev}_af"], out[f"{tag}_l{lev}_diag"] = af, diag
            x, it, _ = L.solve_ref_level(ia, ja, a, b, lev)
            out[f"{tag}_l{lev}_x"], out[f"{tag}_l{lev}_nitr"] = x, np.int32(it)
    np.savez_compressed(os.path.join(OUT, "ilu_levels.npz"), **out)


if __name__ == "__main__":
    assert L.ref_available(), "build oracle/_ref first: make -f oracle/Makefile.ref -C oracle"
    os.makedirs(OUT, exist_ok=True)
    for c in CASES:
        n, nnz, it = make(*c)
        print(f"{c[0]}: n={n} nnz={nnz} nitr={it}")
    make_levels()
    print("ilu_levels")
