// oracle.cpp -- CPU restatement of connortannahill/MM-ADMM's ADMM time step.
//
// TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain C++17: no Eigen, no nanoflann.
// Compiled with the reference's flags (-O3 -msse2 -fopenmp, Makefile:4) plus
// -ffp-contract=off so every product and sum is rounded exactly as written.
//
// Conventions where the reference's arithmetic lives inside un-vendored Eigen:
//  * 2x2 / 3x3 determinant and inverse: Eigen 3.4 closed forms (determinant_impl,
//    compute_inverse_size2/3, cofactor_3x3).
//  * fixed-size products and traces: coefficient sums in ascending inner index.
//  * k x k inverse of the FD Hessian (Eigen PartialPivLU, src/Mesh.cpp:816):
//    unblocked partial-pivot LU (first max-|.| pivot), then forward / backward
//    substitution column by column, diagonal applied as multiply by 1/U_ii.
//  * dynamic-size reductions (VectorXd::sum, squaredNorm, dot): SSE2 packet order
//    (two 2-double packets, Eigen redux_impl LinearVectorizedTraversal).
//  * Eigen ConjugateGradient<Lower|Upper> + DiagonalPreconditioner, x0 = 0, tol = eps
//    (src/MeshIntegrator.cpp:51-55,138,160) restated exactly (cgMode 0); cgMode 1
//    returns the exact block-diagonal solution x = vec / t_ii.
//  * nanoflann kNN(k=1) in the monitor-grid set-up (src/MeshInterpolator.cpp:166-241):
//    exact nearest vertex by a k-d tree, ties -> lowest vertex id (nanoflann's tie order is
//    tree dependent; unpinned on exact ties).
#include "oracle.h"

#include <algorithm>
#include <cassert>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <quadmath.h>

namespace orc {

// powMode 1: correctly rounded pow (long double, with a __float128 fallback when the
// 64-bit result sits within 2 ulps of a double rounding midpoint).  powMode 0 is glibc pow,
// i.e. the reference's semantics; glibc misrounds ~1 in 1200 calls by one ulp.
static double crpow(double x, double y) {
  const long double r = powl((long double)x, (long double)y);
  if (!(r > 0) || !std::isfinite((double)r)) return pow(x, y);
  uint64_t mant;
  std::memcpy(&mant, &r, sizeof(mant));  // x87: 64-bit explicit mantissa in the low 8 bytes
  const uint64_t low = mant & 0x7FF;
  if (low >= 0x3FE && low <= 0x402) return (double)powq((__float128)x, (__float128)y);
  if (low <= 0x002 || low >= 0x7FE) return (double)powq((__float128)x, (__float128)y);
  return (double)r;
}
static int g_powMode = 0;
static inline double opow(double x, double y) { return g_powMode ? crpow(x, y) : pow(x, y); }

enum NodeType { BOUNDARY_FREE = 0, BOUNDARY_FIXED = 1, INTERIOR = 2 };  // src/NodeType.h:4-8

// ---------------------------------------------------------------------------
// Eigen-order helpers
// ---------------------------------------------------------------------------
template <class E>
static double sse2_redux(long n, E e) {  // Eigen redux_impl<..., LinearVectorizedTraversal, NoUnrolling>
  if (n <= 0) return 0.0;
  const long aligned = (n / 2) * 2, aligned2 = (n / 4) * 4;
  double res;
  if (aligned) {
    double a0 = e(0), a1 = e(1);
    if (aligned > 2) {
      double b0 = e(2), b1 = e(3);
      for (long i = 4; i < aligned2; i += 4) {
        a0 += e(i);
        a1 += e(i + 1);
        b0 += e(i + 2);
        b1 += e(i + 3);
      }
      a0 += b0;
      a1 += b1;
      if (aligned > aligned2) {
        a0 += e(aligned2);
        a1 += e(aligned2 + 1);
      }
    }
    res = a0 + a1;
    for (long i = aligned; i < n; ++i) res += e(i);
  } else {
    res = e(0);
    for (long i = 1; i < n; ++i) res += e(i);
  }
  return res;
}

template <int D>
struct Mat {  // row-major small matrix m[r][c]
  double m[D][D];
};

template <int D>
static inline double det(const Mat<D>& a) {
  if (D == 2) return a.m[0][0] * a.m[1][1] - a.m[1][0] * a.m[0][1];
  // Eigen determinant_impl<3>: bruteforce_det3_helper(m,0,1,2) - (m,1,0,2) + (m,2,0,1)
  const double h0 = a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]);
  const double h1 = a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]);
  const double h2 = a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
  return h0 - h1 + h2;
}

static inline double cof3(const double m[3][3], int i, int j) {
  const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
}

template <int D>
static inline Mat<D> inverse(const Mat<D>& a) {
  Mat<D> r;
  if (D == 2) {
    const double invdet = 1.0 / det<D>(a);
    r.m[0][0] = a.m[1][1] * invdet;
    r.m[1][0] = -a.m[1][0] * invdet;
    r.m[0][1] = -a.m[0][1] * invdet;
    r.m[1][1] = a.m[0][0] * invdet;
  } else {
    const double (*m)[3] = reinterpret_cast<const double(*)[3]>(a.m);
    const double c0 = cof3(m, 0, 0), c1 = cof3(m, 1, 0), c2 = cof3(m, 2, 0);
    const double dt = (c0 * m[0][0] + c1 * m[1][0]) + c2 * m[2][0];
    const double invdet = 1.0 / dt;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) r.m[i][j] = cof3(m, j, i) * invdet;
    r.m[0][0] = c0 * invdet;
    r.m[0][1] = c1 * invdet;
    r.m[0][2] = c2 * invdet;
  }
  return r;
}

template <int D>
static inline Mat<D> mul(const Mat<D>& a, const Mat<D>& b) {
  Mat<D> c;
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) {
      double s = a.m[i][0] * b.m[0][j];
      for (int k = 1; k < D; ++k) s += a.m[i][k] * b.m[k][j];
      c.m[i][j] = s;
    }
  return c;
}

template <int D>
static inline Mat<D> transpose(const Mat<D>& a) {
  Mat<D> t;
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) t.m[i][j] = a.m[j][i];
  return t;
}

template <int D>
static inline double trace(const Mat<D>& a) {
  double s = a.m[0][0];
  for (int i = 1; i < D; ++i) s += a.m[i][i];
  return s;
}

// ---------------------------------------------------------------------------
// Monitor functions (Experiments/TestMonitors/MEx*.h) -- host only, set-up time
// ---------------------------------------------------------------------------
static void monIdentity(int D, double* M) {
  for (int i = 0; i < D * D; ++i) M[i] = (i / D == i % D) ? 1.0 : 0.0;
}
static void monScale(int D, double* M, double s) {
  monIdentity(D, M);
  for (int i = 0; i < D * D; ++i) M[i] *= s;
}
// MEx1.h:8-20 / MEx13D.h
static void mex1(int D, const double* x, double* M) {
  const double mu1 = 20, mu2 = 20;
  double sq = 0.0;
  for (int d = 0; d < D; ++d) {
    const double t = x[d] - 0.5;
    sq = (d == 0) ? t * t : sq + t * t;
  }
  monScale(D, M, 1 + mu1 / (1 + mu2 * sq));
}
// MEx2.h:8-22
static void mex2(int D, const double* x, double* M) {
  const double lam1 = 1 + (1.0 / cosh(50 * (x[0] + x[1] - 1.0) * (x[0] + x[1] - 1.0)));
  const double lam2 = 1.0 / lam1;
  const double r = (1.0 / sqrt(2.0)) * 1.0;
  const double v[2] = {r, r}, vo[2] = {r, -(1.0 / sqrt(2.0)) * 1.0};
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) M[i * 2 + j] = ((lam1 * v[i]) * v[j]) + ((lam2 * vo[i]) * vo[j]);
}
// MEx3.h:8-18 / MEx23D.h / MEx33D.h
static void mex3(int D, const double* x, double* M) {
  const double PI = 3.141592653589793238462643383;
  double s;
  if (D == 2)
    s = sqrt(0.01 / (2.0 + cos(8.0 * PI * sqrt(pow(x[0] - 0.5, 2) + pow(x[1] - 0.5, 2)))));
  else
    s = pow(0.01 / (2.0 + cos(8.0 * PI *
                              sqrt(pow(x[0] - 0.5, 2) + pow(x[1] - 0.5, 2) + pow(x[2] - 0.5, 2)))),
            1.0 / 2.0);
  monScale(D, M, s);
}
// MEx4.h:8-23
static void mex4(int D, const double* x, double* M) {
  const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
  const double eps = 0.01;
  double g0 = ((1.0 / (1.0 + exp((x[0] + h + x[1] - 1) / (2.0 * eps)))) -
               (1.0 / (1.0 + exp((x[0] - h + x[1] - 1) / (2.0 * eps))))) /
              (2.0 * h);
  double g1 = ((1.0 / (1.0 + exp((x[0] + x[1] + h - 1) / (2.0 * eps)))) -
               (1.0 / (1.0 + exp((x[0] + x[1] - h - 1) / (2.0 * eps))))) /
              (2.0 * h);
  const double nrm = sqrt(g0 * g0 + g1 * g1);
  monScale(D, M, pow(1 + pow(nrm, 2.0), 1.0 / 4.0));
}
// MEx5.h:8-24
static double mex5u(double x, double y) {
  const double r = sqrt(pow(x - 0.7, 2.0) + pow(y - 0.5, 2.0));
  const double theta = atan((y - 0.5) / (x - 0.7));
  return 1.0 + 9.0 / (1.0 + 100.0 * r * r * pow(cos(theta - 20.0 * r * r), 2.0));
}
static void mex5(int D, const double* x, double* M) {
  const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
  const double g0 = (mex5u(x[0] + h, x[1]) - mex5u(x[0] - h, x[1])) / (2.0 * h);
  const double g1 = (mex5u(x[0], x[1] + h) - mex5u(x[0], x[1] - h)) / (2.0 * h);
  const double nrm = sqrt(g0 * g0 + g1 * g1);
  monScale(D, M, pow(1 + pow(nrm, 2.0), 1.0 / 4.0));
}
// MEx53D.h:8-28 (grad(1) overwritten, Vector<double,2> grad: reference quirk kept)
static double mex53u(double x, double y, double z) {
  const double r = sqrt(pow(x - 0.7, 2.0) + pow(y - 0.5, 2.0) + pow(z - 0.5, 2));
  const double theta = atan((y - 0.5) / (x - 0.7));
  const double psi = atan((z - 0.5) / (x - 0.7));
  return 1.0 + 9.0 / (1.0 + 100.0 * r * r * pow(cos(theta + psi - 20.0 * r * r), 2.0));
}
static void mex53(int D, const double* x, double* M) {
  const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
  double g0 = (mex53u(x[0] + h, x[1], x[2]) - mex53u(x[0] - h, x[1], x[2])) / (2.0 * h);
  double g1 = (mex53u(x[0], x[1] + h, x[2]) - mex53u(x[0], x[1] - h, x[2])) / (2.0 * h);
  g1 = (mex53u(x[0], x[1], x[2] + h) - mex53u(x[0], x[1], x[2] - h)) / (2.0 * h);
  const double nrm = sqrt(g0 * g0 + g1 * g1);
  monScale(D, M, pow(1 + pow(nrm, 2.0), 1.0 / 4.0));
}

// MonType 6: the build's anisotropic shell monitor (mm-admm_amd/csrc/host/monitors.cpp
// anisoShell; no reference counterpart -- BASELINE config 4), restated term for term
static void anisoShell(int D, const double* x, double* M) {
  double d[3], r2 = 0.0;
  for (int i = 0; i < D; ++i) {
    d[i] = x[i] - 0.5;
    r2 = (i == 0) ? d[i] * d[i] : r2 + d[i] * d[i];
  }
  const double r = sqrt(r2);
  const double phi = r - 0.3;
  const double lam1 = 1 + (1.0 / cosh(50 * phi * phi));
  const double lam2 = 1.0 / lam1;
  double n[3];
  for (int i = 0; i < D; ++i) n[i] = (r > 1e-12) ? d[i] / r : (i == 0 ? 1.0 : 0.0);
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) M[i * D + j] = ((i == j) ? lam2 : 0.0) + ((lam1 - lam2) * n[i]) * n[j];
}

// MonType 7: the build's time-varying monitor (no reference counterpart; BASELINE config 5,
// SURVEY §8f-2): a bump moving on a circle, M = (1 + 5 / (1 + 50 |x - c(t)|^2)) I,
// c(t) = (0.5 + 0.2 cos 2 pi t, 0.5 + 0.2 sin 2 pi t, 0.5) -- mm-admm_amd/csrc/host/monitors.cpp
// (moving_bump_centre) and csrc/kernels/regrid_kernels.hip (k_monitor_tv), restated
static void movingBump(int D, const double* x, double t, double* M) {
  const double PI = 3.141592653589793238462643383;
  const double c[3] = {0.5 + 0.2 * cos((2.0 * PI) * t), 0.5 + 0.2 * sin((2.0 * PI) * t), 0.5};
  double sq = 0.0;
  for (int d = 0; d < D; ++d) {
    const double u = x[d] - c[d];
    sq = (d == 0) ? u * u : sq + u * u;
  }
  const double sc = 1 + 5.0 / (1 + 50.0 * sq);
  for (int i = 0; i < D * D; ++i) M[i] = (i / D == i % D) ? sc : 0.0;
}

// Registry by MonType (main.cpp:836-864; 6 = anisoShell, 7 = movingBump at time t)
static void monitorAt(int D, int monType, const double* x, double* M, double t = 0.0) {
  if (monType == 7) {
    movingBump(D, x, t, M);
    return;
  }
  if (D == 2) {
    switch (monType) {
      case 0: monIdentity(2, M); return;
      case 1: mex1(2, x, M); return;
      case 2: mex2(2, x, M); return;
      case 3: mex3(2, x, M); return;
      case 4: mex4(2, x, M); return;
      case 6: anisoShell(2, x, M); return;
      default: mex5(2, x, M); return;
    }
  }
  switch (monType) {  // Mvals3D = {M03D, M13D, M23D, M33D, M03D, M53D}
    case 0: case 4: monIdentity(3, M); return;
    case 1: mex1(3, x, M); return;
    case 2: case 3: mex3(3, x, M); return;
    case 6: anisoShell(3, x, M); return;
    default: mex53(3, x, M); return;
  }
}

// ---------------------------------------------------------------------------
// Meshes (src/MeshUtils.h)
// ---------------------------------------------------------------------------
struct MeshData {
  int dim = 2;
  std::vector<double> Vp;  // nP x dim row-major
  std::vector<int> F;      // nF x (dim+1)
  std::vector<int> mask;   // may be longer than nP (reference quirk)
  int nP() const { return (int)(Vp.size() / dim); }
  int nF() const { return (int)(F.size() / (dim + 1)); }
};

static void linspace(double xa, double xb, int ns, std::vector<double>& x) {  // MeshUtils.h:24-29
  x.resize(ns + 1);
  for (int i = 0; i < ns + 1; i++) x[i] = xa + ((double)i) * (xb - xa) / ns;
}

// MeshUtils.h:82-335 (xa..zb truncated to int as in the reference)
static void genRect(int D, int nx, int ny, int nz, double xaD, double xbD, double yaD, double ybD,
                    double zaD, double zbD, int bType, MeshData& m) {
  const int xa = (int)xaD, xb = (int)xbD, ya = (int)yaD, yb = (int)ybD;
  const int za = (D == 3) ? (int)zaD : 0, zb = (D == 3) ? (int)zbD : 0;
  const double hx = (xb - xa) / ((double)nx), hy = (yb - ya) / ((double)ny);
  const double hz = (D == 3) ? (zb - za) / ((double)nz) : 0;
  m.dim = D;
  if (D == 2) {
    const int nP = (nx + 1) * (ny + 1) + nx * ny;
    m.Vp.assign((size_t)nP * 2, 0.0);
    m.F.assign((size_t)4 * nx * ny * 3, 0);
    m.mask.assign(nP, INTERIOR);
    int off = 0;
    for (int j = 0; j <= ny; j++)
      for (int i = 0; i <= nx; i++) {
        m.Vp[off * 2] = xa + hx * i;
        m.Vp[off * 2 + 1] = ya + hy * j;
        off++;
      }
    for (int j = 0; j < ny; j++)
      for (int i = 0; i < nx; i++) {
        m.Vp[off * 2] = xa + hx * i + hx / 2.0;
        m.Vp[off * 2 + 1] = ya + hy * j + hy / 2.0;
        off++;
      }
    const int stride = (nx + 1) * (ny + 1);
    int* F = m.F.data();
    off = 0;
    for (int j = 0; j < ny; j++)
      for (int i = 0; i < nx; i++) {
        F[off * 3 + 0] = i + j * (nx + 1); F[off * 3 + 1] = stride + i + j * nx; F[off * 3 + 2] = i + (j + 1) * (nx + 1); off++;
        F[off * 3 + 0] = stride + i + j * nx; F[off * 3 + 1] = i + 1 + (j + 1) * (nx + 1); F[off * 3 + 2] = i + (j + 1) * (nx + 1); off++;
        F[off * 3 + 0] = stride + i + j * nx; F[off * 3 + 1] = i + 1 + (j + 1) * (nx + 1); F[off * 3 + 2] = i + 1 + j * (nx + 1); off++;
        F[off * 3 + 0] = i + j * (nx + 1); F[off * 3 + 1] = i + 1 + j * (nx + 1); F[off * 3 + 2] = stride + i + j * nx; off++;
      }
    for (int i = 0; i < (nx + 1) * (ny + 1); i++) {
      const int iOff = i % (nx + 1), jOff = i / (ny + 1);  // MeshUtils.h:162-163 (quirk: ny+1)
      const bool b = (iOff == 0) || (iOff == nx) || (jOff == 0) || (jOff == ny);
      m.mask[i] = b ? bType : INTERIOR;
      if ((iOff == 0 && jOff == 0) || (iOff == nx && jOff == 0) || (iOff == 0 && jOff == ny) ||
          (iOff == nx && jOff == ny))
        m.mask[i] = BOUNDARY_FIXED;
    }
  } else {
    const int nP = (nx + 1) * (ny + 1) * (nz + 1) + nx * ny * nz;
    m.Vp.assign((size_t)nP * 3, 0.0);
    m.F.assign((size_t)12 * nx * ny * nz * 4, 0);
    m.mask.assign(nP, INTERIOR);
    int off = 0;
    for (int k = 0; k <= nz; k++)
      for (int j = 0; j <= ny; j++)
        for (int i = 0; i <= nx; i++) {
          m.Vp[off * 3] = xa + hx * i;
          m.Vp[off * 3 + 1] = ya + hy * j;
          m.Vp[off * 3 + 2] = za + hz * k;
          off++;
        }
    for (int k = 0; k < nz; k++)
      for (int j = 0; j < ny; j++)
        for (int i = 0; i < nx; i++) {
          m.Vp[off * 3] = xa + hx * i + hx / 2.0;
          m.Vp[off * 3 + 1] = ya + hy * j + hy / 2.0;
          m.Vp[off * 3 + 2] = za + hz * k + hz / 2.0;
          off++;
        }
    const int stride = (nx + 1) * (ny + 1) * (nz + 1);
    const int sx = 1, sy = nx + 1, sz = (nx + 1) * (ny + 1);
    int* F = m.F.data();
    off = 0;
    auto put = [&](int a, int b, int c, int d) {
      F[off * 4 + 0] = a; F[off * 4 + 1] = b; F[off * 4 + 2] = c; F[off * 4 + 3] = d; off++;
    };
    for (int k = 0; k < nz; k++)
      for (int j = 0; j < ny; j++)
        for (int i = 0; i < nx; i++) {
          const int mid = stride + i + j * nx + k * (nx * ny);
          auto P = [&](int di, int dj, int dk) { return (i + di) * sx + (j + dj) * sy + (k + dk) * sz; };
          put(P(0, 0, 0), P(1, 0, 0), P(1, 1, 0), mid);  // bot
          put(P(0, 0, 0), P(0, 1, 0), P(1, 1, 0), mid);
          put(P(0, 0, 1), P(1, 0, 1), P(1, 1, 1), mid);  // top
          put(P(0, 0, 1), P(0, 1, 1), P(1, 1, 1), mid);
          put(P(0, 0, 0), P(0, 1, 0), P(0, 1, 1), mid);  // left
          put(P(0, 0, 0), P(0, 0, 1), P(0, 1, 1), mid);
          put(P(1, 0, 0), P(1, 1, 0), P(1, 1, 1), mid);  // right
          put(P(1, 0, 0), P(1, 0, 1), P(1, 1, 1), mid);
          put(P(0, 0, 0), P(1, 0, 0), P(0, 0, 1), mid);  // back
          put(P(1, 0, 0), P(1, 0, 1), P(0, 0, 1), mid);
          put(P(0, 1, 0), P(1, 1, 0), P(0, 1, 1), mid);  // front
          put(P(1, 1, 0), P(1, 1, 1), P(0, 1, 1), mid);
        }
    for (int k = 0; k < nz + 1; k++)
      for (int i = 0; i < (nx + 1) * (ny + 1); i++) {
        const int iOff = i / (nx + 1), jOff = i % (ny + 1);  // MeshUtils.h:302-303
        const bool b = (iOff == 0) || (iOff == nx) || (jOff == 0) || (jOff == ny) || (k == 0) || (k == nz);
        const int o = k * (nx + 1) * (ny + 1) + i;
        if (b) m.mask[o] = bType;
        const bool corner = (iOff == 0 && jOff == 0) || (iOff == nx && jOff == 0) ||
                            (iOff == 0 && jOff == ny) || (iOff == nx && jOff == ny) ||
                            (iOff == 0 && k == 0) || (iOff == nx && k == 0) ||
                            (iOff == 0 && k == nz) || (iOff == nx && k == nz) ||
                            (k == 0 && jOff == 0) || (k == nz && jOff == 0) ||
                            (k == 0 && jOff == ny) || (k == nz && jOff == ny);
        if (corner) m.mask[o] = BOUNDARY_FIXED;
      }
  }
}

static double circlePhi(double x, double y) {  // main.cpp:33-40
  const double r = 0.35, cx = 0.5, cy = 0.5;
  const double xv = (x - cx), yv = (y - cy);
  return sqrt(xv * xv + yv * yv) - r;
}

// MeshUtils.h:404-538 restated with an O(N) ascending-rank compaction in place of the
// O(nP*nF) remap loop at 510-518 (same result).  The mask is NOT compacted: entries
// are written at old point ids (487) and then at new ids (534-535), as in the reference.
// compactMask != 0 remaps the mask to the new ids (the evident intent; without it the
// reference's quirk leaves all-FIXED simplices that make bfgsOptSimplex divide 0/0).
static void genLevelSet2D(int nx, int ny, double xa, double xb, double ya, double yb, int bType,
                          int compactMask, MeshData& m) {
  const double EPS = 1e-12;
  MeshData g;
  genRect(2, nx, ny, 0, xa, xb, ya, yb, 0, 0, bType, g);
  for (auto& v : g.mask) v = INTERIOR;
  const int nF0 = g.nF();
  std::vector<int> keep;
  keep.reserve(nF0);
  for (int s = 0; s < nF0; ++s) {
    const int* f = &g.F[s * 3];
    const double p0 = circlePhi(g.Vp[f[0] * 2], g.Vp[f[0] * 2 + 1]);
    const double p1 = circlePhi(g.Vp[f[1] * 2], g.Vp[f[1] * 2 + 1]);
    const double p2 = circlePhi(g.Vp[f[2] * 2], g.Vp[f[2] * 2 + 1]);
    if (!(p0 > -EPS && p1 > -EPS && p2 > -EPS)) keep.push_back(s);
  }
  const int nP0 = g.nP();
  std::vector<char> used(nP0, 0);
  for (int s : keep)
    for (int j = 0; j < 3; ++j) used[g.F[s * 3 + j]] = 1;
  for (int p = 0; p < nP0; ++p) {  // ascending, like std::set iteration
    if (!used[p]) continue;
    double X = g.Vp[p * 2], Y = g.Vp[p * 2 + 1];
    const double phi = circlePhi(X, Y);
    if (std::abs(phi) < EPS || phi > 0) {  // interpolateBoundaryLocation 2D (369-386)
      const double xv = (X - 0.5), yv = (Y - 0.5);
      const double g0 = (xv) / sqrt(xv * xv + yv * yv);
      const double g1 = (yv) / sqrt(xv * xv + yv * yv);
      const double ph = circlePhi(X, Y);
      X = X - ph * g0;
      Y = Y - ph * g1;
      g.mask[p] = bType;
    }
    g.Vp[p * 2] = X;
    g.Vp[p * 2 + 1] = Y;
  }
  std::vector<int> newId(nP0, -1);
  int cnt = 0;
  for (int p = 0; p < nP0; ++p)
    if (used[p]) newId[p] = cnt++;
  m.dim = 2;
  m.Vp.resize((size_t)cnt * 2);
  for (int p = 0; p < nP0; ++p)
    if (used[p]) {
      m.Vp[newId[p] * 2] = g.Vp[p * 2];
      m.Vp[newId[p] * 2 + 1] = g.Vp[p * 2 + 1];
    }
  m.F.resize(keep.size() * 3);
  for (size_t i = 0; i < keep.size(); ++i)
    for (int j = 0; j < 3; ++j) m.F[i * 3 + j] = newId[g.F[keep[i] * 3 + j]];
  if (compactMask) {
    m.mask.assign(cnt, INTERIOR);
    for (int p = 0; p < nP0; ++p)
      if (used[p]) m.mask[newId[p]] = g.mask[p];
  } else {
    m.mask = g.mask;  // length nP0 (uncompacted, MeshUtils.h:487)
  }
  for (int p = 0; p < cnt; ++p) {
    const double phi = circlePhi(m.Vp[p * 2], m.Vp[p * 2 + 1]);
    if (std::abs(phi) < EPS) m.mask[p] = BOUNDARY_FIXED;
  }
}

static double spherePhi(double x, double y, double z) {  // main.cpp:87-97 (squared form, not a distance)
  const double r = 0.4, cx = 0.5, cy = 0.5, cz = 0.5;
  const double xv = (x - cx), yv = (y - cy), zv = (z - cz);
  return xv * xv + yv * yv + zv * zv - r * r;
}

// MeshUtils.h:540-667 (3D meshFromLevelSetFun with spherePhi, main.cpp:363) restated, with the three
// defects that make the reference's 3D generator unusable repaired:
//  * its result never reaches the caller: `delete Vc; Vc = Vcnew; delete Vp; Vp = Vpnew;`
//    (663-666) reassigns the function's own pointer copies, leaving the caller's Vp/Vc deleted
//    (dangling) while F has been remapped -- here Vp and F are the remapped mesh;
//  * the mask is not compacted (written at the pre-compaction ids, 595-597); compactMask != 0
//    remaps it (the evident intent, as for 2D), 0 keeps the reference's indexing;
//  * F is remapped in place (653-661) by walking the used ids in ASCENDING order with the
//    DESCENDING map, so an entry remapped to a larger used id still to come is remapped again
//    (used ids {0,1,2}: 0 -> 2 -> 0, and 2 -> 0 too) and the reference's F is corrupted -- here
//    each entry is remapped exactly once (the 2D loop, 510-518, maps ids downwards and is sound).
// The node numbering is the reference's: pntMap maps the i-th LARGEST used id to i (645-651, the
// reversed rank) and F is remapped with it once, consistently with Vp.  No final |phi| < EPS pass (the
// 2D generator has one, 531-537; the 3D one does not).  The interior-side projection is
// interpolateBoundaryLocation 3D (388-402): a central-difference gradient of spherePhi with
// h = 2 sqrt(eps), normalised (Eigen normalize: divided by sqrt of the squared norm), and
// p - phi(p) n -- with the squared-distance phi this moves outside points towards, not onto,
// the sphere.
static void genLevelSet3D(int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za,
                          double zb, int bType, int compactMask, MeshData& m) {
  const double EPS = 1e-12;
  MeshData g;
  genRect(3, nx, ny, nz, xa, xb, ya, yb, za, zb, bType, g);
  for (auto& v : g.mask) v = INTERIOR;
  const int nF0 = g.nF();
  auto phiAt = [&](int v) { return spherePhi(g.Vp[v * 3], g.Vp[v * 3 + 1], g.Vp[v * 3 + 2]); };
  std::vector<int> idsToBeRemoved;
  for (int s = 0; s < nF0; ++s) {
    const int* f = &g.F[s * 4];
    const double p0 = phiAt(f[0]), p1 = phiAt(f[1]), p2 = phiAt(f[2]), p3 = phiAt(f[3]);
    if (p0 > -EPS && p1 > -EPS && p2 > -EPS && p3 > -EPS) idsToBeRemoved.push_back(s);
  }
  std::vector<int> Fk;  // removeRow in descending id order == the others kept in order
  {
    size_t r = 0;
    for (int s = 0; s < nF0; ++s) {
      if (r < idsToBeRemoved.size() && idsToBeRemoved[r] == s) {
        ++r;
        continue;
      }
      Fk.insert(Fk.end(), g.F.begin() + (size_t)s * 4, g.F.begin() + (size_t)(s + 1) * 4);
    }
  }
  std::set<int> usedPnts(Fk.begin(), Fk.end());
  const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
  for (int p : usedPnts) {
    double x[3] = {g.Vp[p * 3], g.Vp[p * 3 + 1], g.Vp[p * 3 + 2]};
    if (spherePhi(x[0], x[1], x[2]) > -EPS) {
      double gr[3];
      gr[0] = (spherePhi(x[0] + h, x[1], x[2]) - spherePhi(x[0] - h, x[1], x[2])) / (2.0 * h);
      gr[1] = (spherePhi(x[0], x[1] + h, x[2]) - spherePhi(x[0], x[1] - h, x[2])) / (2.0 * h);
      gr[2] = (spherePhi(x[0], x[1], x[2] + h) - spherePhi(x[0], x[1], x[2] - h)) / (2.0 * h);
      const double sq = gr[0] * gr[0] + gr[1] * gr[1] + gr[2] * gr[2];
      if (sq > 0) {
        const double nrm = sqrt(sq);
        for (int c = 0; c < 3; ++c) gr[c] = gr[c] / nrm;
      }
      const double ph = spherePhi(x[0], x[1], x[2]);
      for (int c = 0; c < 3; ++c) x[c] = x[c] - ph * gr[c];
      g.mask[p] = bType;
    }
    for (int c = 0; c < 3; ++c) g.Vp[p * 3 + c] = x[c];
  }
  std::vector<int> pntsSorted(usedPnts.begin(), usedPnts.end());
  std::map<int, int> pntMap;
  const int cnt = (int)pntsSorted.size();
  m.dim = 3;
  m.Vp.resize((size_t)cnt * 3);
  for (int i = 0; i < cnt; i++) {
    const int off = pntsSorted[cnt - i - 1];
    pntMap[off] = i;
    for (int c = 0; c < 3; ++c) m.Vp[(size_t)i * 3 + c] = g.Vp[(size_t)off * 3 + c];
  }
  m.F.resize(Fk.size());
  for (size_t e = 0; e < Fk.size(); ++e) m.F[e] = pntMap[Fk[e]];
  if (compactMask) {
    m.mask.assign(cnt, INTERIOR);
    for (const auto& kv : pntMap) m.mask[kv.second] = g.mask[kv.first];
  } else {
    m.mask = g.mask;
  }
}

// MeshUtils.h:669-733 (comma separated, one row per line; mask one int per line)
static bool readMesh(int D, const char* tri, const char* pnts, const char* mask, MeshData& m) {
  m.dim = D;
  std::ifstream ft(tri);
  if (!ft) return false;
  std::string line, word;
  std::vector<int> triData;
  while (std::getline(ft, line)) {
    std::stringstream s(line);
    while (std::getline(s, word, ',')) triData.push_back(std::stoi(word));
  }
  std::ifstream fp(pnts);
  if (!fp) return false;
  std::vector<double> pd;
  while (std::getline(fp, line)) {
    std::stringstream s(line);
    while (std::getline(s, word, ',')) pd.push_back(std::stod(word));
  }
  std::ifstream fm(mask);
  if (!fm) return false;
  m.mask.clear();
  int tmp;
  while (fm >> tmp) m.mask.push_back(tmp);
  const size_t nF = triData.size() / (D + 1), nP = pd.size() / D;
  m.F.assign(triData.begin(), triData.begin() + nF * (D + 1));
  m.Vp.assign(pd.begin(), pd.begin() + nP * D);
  return true;
}

// ---------------------------------------------------------------------------
// Monitor grid (src/MeshInterpolator.cpp)
// ---------------------------------------------------------------------------
template <int D>
struct Grid {
  int nx = 0, ny = 0, nz = 0;
  std::vector<double> gx, gy, gz;
  std::vector<double> vals;  // rows x D*D
  int rows() const { return (int)(vals.size() / (D * D)); }
};

// Exact nearest neighbour (ties -> lowest id): recursive k-d tree over index ranges.
template <int D>
struct NN {
  const double* X = nullptr;
  std::vector<int> ord;
  struct Split {
    int axis;
    double val;
  };
  std::vector<Split> splits;  // implicit tree over [lo, hi) ranges, heap-indexed
  void build(const double* Xin, int nin) {
    X = Xin;
    ord.resize(nin);
    for (int i = 0; i < nin; ++i) ord[i] = i;
    splits.assign(4 * (size_t)std::max(nin, 1), Split{-1, 0.0});
    rec(1, 0, nin);
  }
  void rec(size_t node, int lo, int hi) {
    if (hi - lo <= 6) return;
    int axis = 0;
    double best = -1;
    for (int d = 0; d < D; ++d) {
      double a = INFINITY, b = -INFINITY;
      for (int t = lo; t < hi; ++t) {
        a = std::min(a, X[ord[t] * D + d]);
        b = std::max(b, X[ord[t] * D + d]);
      }
      if (b - a > best) {
        best = b - a;
        axis = d;
      }
    }
    const int mid = (lo + hi) / 2;
    std::nth_element(ord.begin() + lo, ord.begin() + mid, ord.begin() + hi, [&](int p, int q) {
      return X[p * D + axis] < X[q * D + axis] || (X[p * D + axis] == X[q * D + axis] && p < q);
    });
    splits[node] = Split{axis, X[ord[mid] * D + axis]};
    rec(2 * node, lo, mid);
    rec(2 * node + 1, mid, hi);
  }
  static double dist(const double* q, const double* p) {  // nanoflann L2_Simple_Adaptor
    double r = 0.0;
    for (int d = 0; d < D; ++d) {
      const double df = q[d] - p[d];
      r += df * df;
    }
    return r;
  }
  void visit(size_t node, int lo, int hi, const double* q, double& best, int& bi) const {
    if (hi - lo <= 6) {
      for (int t = lo; t < hi; ++t) {
        const double dd = dist(q, &X[ord[t] * D]);
        if (dd < best || (dd == best && ord[t] < bi)) {
          best = dd;
          bi = ord[t];
        }
      }
      return;
    }
    const int mid = (lo + hi) / 2;
    const Split s = splits[node];
    const double diff = q[s.axis] - s.val;
    if (diff < 0) {
      visit(2 * node, lo, mid, q, best, bi);
      if (diff * diff <= best) visit(2 * node + 1, mid, hi, q, best, bi);
    } else {
      visit(2 * node + 1, mid, hi, q, best, bi);
      if (diff * diff <= best) visit(2 * node, lo, mid, q, best, bi);
    }
  }
  int query(const double* q) const {
    double best = INFINITY;
    int bi = -1;
    visit(1, 0, (int)ord.size(), q, best, bi);
    return bi;
  }
};

template <int D>
static void buildGrid(const double* X, int nP, int monType, Grid<D>& g, double t = 0.0) {
  // updateMesh (68-130): nx = ny = nz = (int)pow(X.size(), 1/D), bbox of the mesh
  const int sz = (int)std::pow((double)((long)nP * D), 1.0 / D);
  g.nx = sz;
  g.ny = sz;
  g.nz = (D == 2) ? 1 : sz;
  double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < nP; i++)
    for (int d = 0; d < D; ++d) {
      const double v = X[i * D + d];
      mn[d] = (v < mn[d]) ? v : mn[d];
      mx[d] = (v > mx[d]) ? v : mx[d];
    }
  linspace(mn[0], mx[0], g.nx, g.gx);
  linspace(mn[1], mx[1], g.ny, g.gy);
  if (D == 3) linspace(mn[2], mx[2], g.nz, g.gz);
  const long rows = (long)(g.nx + 1) * (g.ny + 1) * (g.nz + 1);
  g.vals.assign(rows * D * D, 0.0);
  // evaluateAtVertices (MonitorFunction.cpp:16-32)
  std::vector<double> monVals((size_t)nP * D * D);
  for (int v = 0; v < nP; ++v) monitorAt(D, monType, &X[v * D], &monVals[(size_t)v * D * D], t);
  NN<D> nn;
  nn.build(X, nP);
  const int nx = g.nx, ny = g.ny;
  if (D == 2) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nx + 1; i++)
      for (int j = 0; j < ny + 1; j++) {
        const double q[2] = {g.gx[i], g.gy[j]};
        const int id = nn.query(q);
        std::memcpy(&g.vals[((size_t)j * (nx + 1) + i) * 4], &monVals[(size_t)id * 4], 4 * sizeof(double));
      }
  } else {
    const int nz = g.nz;
#pragma omp parallel for schedule(static)
    for (int k = 0; k < nz + 1; k++)
      for (int i = 0; i < nx + 1; i++)
        for (int j = 0; j < ny + 1; j++) {
          const double q[3] = {g.gx[i], g.gy[j], g.gz[k]};
          const int id = nn.query(q);
          // MeshInterpolator.cpp:234 -- row (nx+1)(ny+1)k + i(nx+1) + j (x/y swapped)
          std::memcpy(&g.vals[((size_t)(nx + 1) * (ny + 1) * k + (size_t)i * (nx + 1) + j) * 9],
                      &monVals[(size_t)id * 9], 9 * sizeof(double));
        }
  }
  // smoothMonitorGrid (366-404)
  const int nIters = (D == 2) ? 5 : 2;
  std::vector<double> tmp;
  for (int it = 0; it < nIters; ++it) {
    tmp = g.vals;
    if (D == 2) {
      for (int i = 1; i < nx; i++)
        for (int j = 1; j < ny; j++) {
          double* o = &g.vals[((size_t)j * (nx + 1) + i) * 4];
          const double* c = &tmp[((size_t)j * (nx + 1) + i) * 4];
          const double* e = &tmp[((size_t)j * (nx + 1) + i + 1) * 4];
          const double* w = &tmp[((size_t)j * (nx + 1) + i - 1) * 4];
          const double* n = &tmp[((size_t)(j + 1) * (nx + 1) + i) * 4];
          const double* s = &tmp[((size_t)(j - 1) * (nx + 1) + i) * 4];
          for (int q = 0; q < 4; ++q) {
            double v = 0.6 * c[q];
            v += 0.1 * e[q];
            v += 0.1 * w[q];
            v += 0.1 * n[q];
            v += 0.1 * s[q];
            o[q] = v;
          }
        }
    } else {
      const double h = 0.4 / 6.0;
      const int nz = g.nz;
      const size_t P = (size_t)(nx + 1) * (ny + 1);
      for (int k = 1; k < nz; k++)
        for (int i = 1; i < nx; i++)
          for (int j = 1; j < ny; j++) {
            const size_t c = P * k + (size_t)j * (nx + 1) + i;
            for (int q = 0; q < 9; ++q) {
              g.vals[c * 9 + q] = 0.6 * tmp[c * 9 + q] + h * tmp[(c + 1) * 9 + q] +
                                  h * tmp[(c - 1) * 9 + q] + h * tmp[(c + nx + 1) * 9 + q] +
                                  h * tmp[(c - nx - 1) * 9 + q] + h * tmp[(c + P) * 9 + q] +
                                  h * tmp[(c - P) * 9 + q];
            }
          }
    }
  }
}

static inline int findLimInf(double w, const std::vector<double>& m) {  // MeshUtils.h:45-54
  uint32_t guess = (int)((w - m[0]) / (m[1] - m[0]));
  if (guess > m.size() - 2) guess = (uint32_t)(m.size() - 2);
  return (int)guess;
}

template <int D>
static void evalMonitor(const Grid<D>& g, const double* pnt, Mat<D>& mVal) {  // 287-342
  const int xInd = findLimInf(pnt[0], g.gx), yInd = findLimInf(pnt[1], g.gy);
  const int nx = g.nx, ny = g.ny;
  if (D == 2) {
    const double xm0 = g.gx[xInd], xm1 = g.gx[xInd + 1], ym0 = g.gy[yInd], ym1 = g.gy[yInd + 1];
    const double x = pnt[0], y = pnt[1];
    const double norm = (1 / ((xm1 - xm0) * (ym1 - ym0)));
    const double c0 = norm * (xm1 - x) * (ym1 - y), c1 = norm * (x - xm0) * (ym1 - y);
    const double c2 = norm * (xm1 - x) * (y - ym0), c3 = norm * (x - xm0) * (y - ym0);
    const double* g00 = &g.vals[((size_t)yInd * (nx + 1) + xInd) * 4];
    const double* g10 = g00 + 4;
    const double* g01 = &g.vals[((size_t)(yInd + 1) * (nx + 1) + xInd) * 4];
    const double* g11 = g01 + 4;
    for (int n = 0; n < 4; n++) mVal.m[n / 2][n % 2] = c0 * g00[n] + c1 * g10[n] + c2 * g01[n] + c3 * g11[n];
  } else {
    const int zInd = findLimInf(pnt[2], g.gz);
    const double xd = (pnt[0] - g.gx[xInd]) / (g.gx[xInd + 1] - g.gx[xInd]);
    const double yd = (pnt[1] - g.gy[yInd]) / (g.gy[yInd + 1] - g.gy[yInd]);
    const double zd = (pnt[2] - g.gz[zInd]) / (g.gz[zInd + 1] - g.gz[zInd]);
    const double c[8] = {(1 - xd) * (1 - yd) * (1 - zd), xd * (1 - yd) * (1 - zd),
                         (1 - xd) * yd * (1 - zd),       xd * yd * (1 - zd),
                         (1 - xd) * (1 - yd) * zd,       xd * (1 - yd) * zd,
                         (1 - xd) * yd * zd,             xd * yd * zd};
    const size_t P = (size_t)(nx + 1) * (ny + 1);
    const size_t r[8] = {zInd * P + (size_t)yInd * (nx + 1) + xInd,
                         zInd * P + (size_t)yInd * (nx + 1) + xInd + 1,
                         zInd * P + (size_t)(yInd + 1) * (nx + 1) + xInd,
                         zInd * P + (size_t)(yInd + 1) * (nx + 1) + xInd + 1,
                         (zInd + 1) * P + (size_t)yInd * (nx + 1) + xInd,
                         (zInd + 1) * P + (size_t)yInd * (nx + 1) + xInd + 1,
                         (zInd + 1) * P + (size_t)(yInd + 1) * (nx + 1) + xInd,
                         (zInd + 1) * P + (size_t)(yInd + 1) * (nx + 1) + xInd + 1};
    double f[9];
    for (int n = 0; n < 9; ++n) f[n] = 0.0;
    for (int q = 0; q < 8; ++q)
      for (int n = 0; n < 9; ++n) f[n] += c[q] * g.vals[r[q] * 9 + n];
    for (int n = 0; n < 9; ++n) mVal.m[n / 3][n % 3] = f[n];
  }
}

// ---------------------------------------------------------------------------
// The integrator state
// ---------------------------------------------------------------------------
struct Base {
  virtual ~Base() {}
  int dim = 2;
  int err = 0;
  int regrid = 0;   // rebuild the monitor grid at every step start (time-varying monitors)
  int monType = 0;
};

template <int D>
struct Integrator : Base {
  static constexpr int K = D * (D + 1);
  int nP = 0, nF = 0;
  bool compMesh = false;
  std::vector<double> Vp, Vc;  // nP x D row-major
  std::vector<int> F, mask;
  Grid<D> grid;
  Mat<D> EhatConst;
  double tau = 0, rho = 0, w = 0, dt = 0;
  int gradUse = 0, cgMode = 0;
  // integrator state (MeshIntegrator.h:29-49)
  std::vector<double> x, xPrev, xBar, z, zPrev, uBar, DXpU, vec, tdiag, invdiag;
  std::vector<double> hess;  // nF x K x K, row-major per simplex
  std::vector<double> IhVec;
  bool hessComputed = false, stepTaken = false;
  int stepsTaken = 0;
  long long bfgsIters = 0;

  void init(int nP_, const double* Vp_, const double* Vc_, int nF_, const int* F_, const int* mask_,
            int monType_, double dt_, double tau_, double rho_, int gradUse_, int cgMode_) {
    dim = D;
    nP = nP_;
    nF = nF_;
    Vp.assign(Vp_, Vp_ + (size_t)nP * D);
    monType = monType_;
    compMesh = (Vc_ != nullptr);
    if (compMesh) Vc.assign(Vc_, Vc_ + (size_t)nP * D);
    F.assign(F_, F_ + (size_t)nF * (D + 1));
    mask.assign(mask_, mask_ + nP);
    dt = dt_;
    tau = tau_;
    rho = rho_;
    gradUse = gradUse_;
    cgMode = cgMode_;
    // reOrientElements (Mesh.cpp:243-260)
    for (int i = 0; i < nF; i++) {
      Mat<D> E;
      for (int j = 0; j < D; j++)
        for (int r = 0; r < D; ++r) E.m[r][j] = Vp[F[i * (D + 1) + j + 1] * D + r] - Vp[F[i * (D + 1)] * D + r];
      if (det<D>(E) < 0) std::swap(F[i * (D + 1) + 1], F[i * (D + 1) + 2]);
    }
    buildGrid<D>(Vp.data(), nP, monType, grid);
    w = 0.5 * sqrt(rho);  // Mesh.cpp:451
    // Ehat for !compMesh (AdaptationFunctional.cpp:176-201), N = F.rows()
    if (D == 2) {
      EhatConst.m[0][0] = 1.0; EhatConst.m[1][0] = 0.0;
      EhatConst.m[0][1] = 1.0 / 2.0; EhatConst.m[1][1] = sqrt(3) / 2.0;
    } else {
      const double v[3][3] = {{-2.0, 0.0, -2.0}, {0.0, -2.0, -2.0}, {-2.0, -2.0, 0.0}};
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) EhatConst.m[r][c] = v[r][c];
    }
    const double dFact = (D == 2) ? 2.0 : 6.0;
    const double s1 = pow((dFact / std::abs(det<D>(EhatConst))), 1.0 / ((double)D));
    for (int r = 0; r < D; ++r)
      for (int c = 0; c < D; ++c) EhatConst.m[r][c] *= s1;
    const double s2 = (double)pow(nF, 1.0 / D);
    for (int r = 0; r < D; ++r)
      for (int c = 0; c < D; ++c) EhatConst.m[r][c] /= s2;
    // MeshIntegrator ctor (MeshIntegrator.cpp:15-62)
    x.resize((size_t)nP * D);
    copyX(x);
    xPrev = x;
    xBar = x;
    z.resize((size_t)nF * K);
    gatherD(x, z);
    zPrev = z;
    uBar.assign(z.size(), 0.0);
    DXpU = z;
    vec.assign((size_t)nP * D, 0.0);
    // t = M + dt^2 WD_T W D, block diagonal: t_ii = tau + dt^2 * (sum_{s ∋ v} w*w)
    std::vector<int> val(nP, 0);
    for (int s = 0; s < nF; ++s)
      for (int n = 0; n < D + 1; ++n) val[F[s * (D + 1) + n]]++;
    tdiag.resize((size_t)nP * D);
    invdiag.resize((size_t)nP * D);
    const double dtsq = dt * dt;
    for (int v = 0; v < nP; ++v) {
      double S = 0.0;
      for (int c = 0; c < val[v]; ++c) S = (c == 0) ? (w * w) * 1.0 : S + (w * w) * 1.0;
      for (int m = 0; m < D; ++m) {
        tdiag[v * D + m] = tau + dtsq * S;
        invdiag[v * D + m] = 1.0 / tdiag[v * D + m];
      }
    }
    hess.assign((size_t)nF * K * K, 0.0);
    for (int s = 0; s < nF; ++s)
      for (int i = 0; i < K; ++i) hess[(size_t)s * K * K + i * K + i] = 1.0;
    IhVec.assign(nF, 0.0);
  }

  void copyX(std::vector<double>& tar) const {  // Mesh.cpp:996-1004
    for (int i = 0; i < nP; i++)
      for (int j = 0; j < D; j++) tar[i * D + j] = Vp[i * D + j];
  }
  void gatherD(const std::vector<double>& xv, std::vector<double>& out) const {  // Dmat * x
    for (int s = 0; s < nF; ++s)
      for (int n = 0; n < D + 1; ++n)
        for (int m = 0; m < D; ++m) out[(size_t)s * K + n * D + m] = xv[F[s * (D + 1) + n] * D + m];
  }

  // AdaptationFunctional<D>::blockGrad (AdaptationFunctional.cpp:102-287)
  double blockGrad(int zId, const double* z, const double* xi, double* grad, bool computeGrad,
                   bool regularize, double* Igt, const double* dxpu) const {
    const double dFact = (D == 2) ? 2.0 : 6.0;
    Mat<D> mPre[D + 1], M;
    for (int i = 0; i < D + 1; i++) {
      evalMonitor<D>(grid, &z[i * D], mPre[i]);
      for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) M.m[r][c] = ((i == 0) ? 0.0 : M.m[r][c]) + mPre[i].m[r][c];
    }
    Mat<D> Minv = inverse<D>(M);
    for (int r = 0; r < D; ++r)
      for (int c = 0; c < D; ++c) Minv.m[r][c] = Minv.m[r][c] / ((double)D + 1);
    Mat<D> E, Ehat;
    for (int j = 0; j < D; ++j) {
      const int n = j + 1;
      for (int r = 0; r < D; ++r) {
        E.m[r][j] = z[D * n + r] - z[r];
        if (compMesh) Ehat.m[r][j] = xi[D * n + r] - xi[r];
      }
    }
    const double Edet = det<D>(E);
    if (!(Edet > 0)) {  // assert(Edet > 0) (AdaptationFunctional.cpp:174): reported, not aborted
      const double nan = std::numeric_limits<double>::quiet_NaN();
      if (computeGrad)
        for (int i = 0; i < K; ++i) grad[i] = nan;
      return nan;
    }
    if (!compMesh) Ehat = EhatConst;
    const Mat<D> Einv = inverse<D>(E);
    const Mat<D> FJ = mul<D>(Ehat, Einv);
    const double detFJ = det<D>(FJ);
    const double d = (double)D;
    const double p = 1.5;
    const double theta = 1.0 / 3.0;
    const Mat<D> FJt = transpose<D>(FJ);
    const Mat<D> MinvJt = mul<D>(Minv, FJt);
    const Mat<D> JMJt = mul<D>(FJ, MinvJt);
    const double trJMJt = trace<D>(JMJt);
    const double detM = sqrt(1.0 / det<D>(Minv));
    const double G = theta * detM * opow(trJMJt, d * p / 2.0) +
                     (1.0 - 2.0 * theta) * pow(d, d * p / 2.0) * detM * opow(detFJ / detM, p);
    const double absK = std::abs(Edet / dFact);
    auto regTerm = [&]() {
      double sq = 0.0;
      for (int i = 0; i < K; ++i) {
        const double t = dxpu[i] - z[i];
        sq = (i == 0) ? t * t : sq + t * t;
      }
      return 0.5 * w * w * sq;
    };
    if (!computeGrad) {
      if (regularize) return absK * G + regTerm();
      return absK * G;
    }
    Mat<D> dGdJ;
    {
      const double s = d * p * theta * detM * opow(trJMJt, d * p / 2.0 - 1);
      for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) dGdJ.m[r][c] = s * MinvJt.m[r][c];
    }
    const double dGddet = p * (1.0 - 2.0 * theta) * pow(d, (d * p) / 2.0) * opow(detM, 1.0 - p) * opow(detFJ, p - 1);
    Mat<D> dGdM;
    {
      const double s1 = -0.5 * theta * d * p * detM * opow(trJMJt, d * p / 2.0 - 1);
      Mat<D> T;
      const Mat<D> MinvT = transpose<D>(Minv);
      for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) T.m[r][c] = s1 * MinvT.m[r][c];
      T = mul<D>(mul<D>(mul<D>(T, FJt), FJ), Minv);
      const double s2 = 0.5 * theta * detM * opow(trJMJt, d * p / 2.0) +
                        ((0.5 - theta) * (1.0 - p) * pow(d, d * p / 2.0)) * opow(detM, 1 - p) * opow(detFJ, p);
      for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) dGdM.m[r][c] = T.m[r][c] + s2 * Minv.m[r][c];
    }
    double basisComb[D];
    for (int c = 0; c < D; ++c) basisComb[c] = 0.0;
    for (int j = 0; j < D; ++j) {
      const int n = j + 1;
      Mat<D> dm;
      for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) dm.m[r][c] = mPre[n].m[r][c] - mPre[0].m[r][c];
      const double tr = trace<D>(mul<D>(dGdM, dm));
      for (int c = 0; c < D; ++c) basisComb[c] += Einv.m[j][c] * tr;
    }
    const double c1 = (-G + dGddet * detFJ);
    Mat<D> vLoc;
    {
      const Mat<D> P = mul<D>(mul<D>(Einv, dGdJ), FJ);
      for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) vLoc.m[r][c] = c1 * Einv.m[r][c] + P.m[r][c];
    }
    for (int n = 0; n < D; n++)
      for (int c = 0; c < D; ++c) vLoc.m[n][c] -= (basisComb[c]) / ((double)D + 1.0);
    double gs[D];
    for (int c = 0; c < D; ++c) {
      double s = 0.0;
      for (int n = 0; n < D; n++) s += vLoc.m[n][c];
      gs[c] = s + (basisComb[c] + 0.0);
    }
    for (int l = 0; l < D; l++) grad[l] = gs[l];
    for (int n = 1; n < D + 1; n++)
      for (int l = 0; l < D; l++) grad[D * n + l] = -vLoc.m[n - 1][l];
    for (int i = 0; i < K; ++i) grad[i] *= absK;
    double Ih = absK * G;
    if (Igt) *Igt = Ih;
    if (regularize) {
      Ih += regTerm();
      for (int i = 0; i < K; ++i) grad[i] += w * w * (-dxpu[i] + z[i]);
    }
    return Ih;
  }

  // Mesh<D>::computeBlockGrad (Mesh.cpp:755-772)
  double computeBlockGrad(int zId, const double* z, const double* xi, double* grad, bool computeGrad,
                          bool regularize, double* Igt, const double* dxpu) const {
    const double Ix = blockGrad(zId, z, xi, grad, computeGrad, regularize, Igt, dxpu);
    for (int i = 0; i < D + 1; i++)
      if (mask[F[zId * (D + 1) + i]] == BOUNDARY_FIXED)
        for (int m = 0; m < D; ++m) grad[D * i + m] = 0.0;
    return Ix;
  }

  void simplexXi(int s, double* xi) const {
    if (!compMesh) return;
    for (int n = 0; n < D + 1; ++n)
      for (int l = 0; l < D; ++l) xi[n * D + l] = Vc[F[s * (D + 1) + n] * D + l];
  }

  // k x k inverse: unblocked partial-pivot LU + substitution (Eigen PartialPivLU::inverse)
  static bool invertK(double* A /* K*K row-major, in place */) {
    double lu[K][K];
    int perm[K];
    for (int i = 0; i < K; ++i) {
      perm[i] = i;
      for (int j = 0; j < K; ++j) lu[i][j] = A[i * K + j];
    }
    for (int k = 0; k < K; ++k) {
      int piv = k;
      double big = std::abs(lu[k][k]);
      for (int i = k + 1; i < K; ++i)
        if (std::abs(lu[i][k]) > big) {
          big = std::abs(lu[i][k]);
          piv = i;
        }
      if (big != 0.0) {
        if (piv != k) {
          for (int j = 0; j < K; ++j) std::swap(lu[k][j], lu[piv][j]);
          std::swap(perm[k], perm[piv]);
        }
        for (int i = k + 1; i < K; ++i) lu[i][k] /= lu[k][k];
      }
      for (int i = k + 1; i < K; ++i)
        for (int j = k + 1; j < K; ++j) lu[i][j] -= lu[i][k] * lu[k][j];
    }
    // X = P * I, then L (unit) and U solves, column by column
    for (int c = 0; c < K; ++c) {
      double xcol[K];
      for (int i = 0; i < K; ++i) xcol[i] = (perm[i] == c) ? 1.0 : 0.0;
      for (int i = 0; i < K; ++i) {
        const double b = xcol[i];
        for (int r = i + 1; r < K; ++r) xcol[r] -= b * lu[r][i];
      }
      for (int i = K - 1; i >= 0; --i) {
        const double a = 1.0 / lu[i][i];
        const double b = (xcol[i] *= a);
        for (int r = 0; r < i; ++r) xcol[r] -= b * lu[r][i];
      }
      for (int i = 0; i < K; ++i) A[i * K + c] = xcol[i];
    }
    return true;
  }

  // Mesh<D>::bfgsOptSimplex (Mesh.cpp:777-872); returns Ihsave, *iters = BFGS iterations
  double bfgsOptSimplex(int zId, double* z, const double* xi, int nIter, double tol, const double* dxpu,
                        int* itersOut, int* errOut) {
    const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
    double Gk[K], Gkp1[K], zPurt[K];
    double Igt = 0.0;
    double* B = &hess[(size_t)zId * K * K];
    if (std::isnan(computeBlockGrad(zId, z, xi, Gk, true, true, &Igt, dxpu))) *errOut = 1;
    const double Ihsave = Igt;
    if (!hessComputed) {
      for (int i = 0; i < K; ++i) zPurt[i] = z[i];
      for (int i = 0; i < K; i++) {
        zPurt[i] += h;
        computeBlockGrad(zId, zPurt, xi, Gkp1, true, true, &Igt, dxpu);
        for (int r = 0; r < K; ++r) B[r * K + i] = (Gkp1[r] - Gk[r]) / h;
        zPurt[i] = z[i];
      }
      for (int n = 0; n < D + 1; n++)
        if (mask[F[zId * (D + 1) + n]] != INTERIOR)
          for (int m = 0; m < D; m++) B[(D * n + m) * K + D * n + m] = 1.0;
      invertK(B);
    }
    double pk[K], yk[K], By[K], yB[K];
    int iter;
    for (iter = 0; iter < nIter; iter++) {
      for (int i = 0; i < K; ++i) {
        double s = (-B[i * K]) * Gk[0];
        for (int j = 1; j < K; ++j) s += (-B[i * K + j]) * Gk[j];
        pk[i] = s;
      }
      for (int i = 0; i < K; ++i) z[i] += pk[i];
      if (std::isnan(computeBlockGrad(zId, z, xi, Gkp1, true, true, &Igt, dxpu))) *errOut = 1;
      double Ix = 0;
      for (int i = 0; i < K; i++) Ix += std::abs(Gkp1[i]);
      for (int i = 0; i < K; ++i) yk[i] = Gkp1[i] - Gk[i];
      double c2 = pk[0] * yk[0];
      for (int i = 1; i < K; ++i) c2 += pk[i] * yk[i];
      for (int i = 0; i < K; ++i) {
        double s = B[i * K] * yk[0];
        for (int j = 1; j < K; ++j) s += B[i * K + j] * yk[j];
        By[i] = s;
      }
      double yBy = yk[0] * By[0];
      for (int i = 1; i < K; ++i) yBy += yk[i] * By[i];
      const double c1 = (c2 + yBy) / (pow(c2, 2.0));
      for (int j = 0; j < K; ++j) {
        double s = yk[0] * B[j];
        for (int i = 1; i < K; ++i) s += yk[i] * B[i * K + j];
        yB[j] = s;
      }
      double Bn[K * K];
      for (int i = 0; i < K; ++i)
        for (int j = 0; j < K; ++j) {
          double by = B[i * K] * (yk[0] * pk[j]);  // (Bkinv * (yk pk^T))_ij
          for (int q = 1; q < K; ++q) by += B[i * K + q] * (yk[q] * pk[j]);
          Bn[i * K + j] = B[i * K + j] + (((c1 * (pk[i] * pk[j])) - by / c2) - (pk[i] * yB[j]) / c2);
        }
      std::memcpy(B, Bn, sizeof(Bn));
      if (Ix < tol) {
        for (int i = 0; i < K; ++i) Gk[i] = Gkp1[i];
        break;
      }
      for (int i = 0; i < K; ++i) Gk[i] = Gkp1[i];
    }
    *itersOut = (iter == nIter) ? nIter : iter + 1;
    return Ihsave;
  }

  // Mesh<D>::prox (Mesh.cpp:930-994)
  double prox(const std::vector<double>& dxpu, std::vector<double>& zv, double tol) {
    long long iters = 0;
    int errAny = 0;
#pragma omp parallel for schedule(static) reduction(+ : iters) reduction(| : errAny)
    for (int i = 0; i < nF; i++) {
      double zi[K], xi[K];
      simplexXi(i, xi);
      for (int l = 0; l < K; ++l) zi[l] = zv[(size_t)K * i + l];
      int it = 0, e = 0;
      IhVec[i] = bfgsOptSimplex(i, zi, xi, 50, tol / 100, &dxpu[(size_t)K * i], &it, &e);
      for (int l = 0; l < K; ++l) zv[(size_t)K * i + l] = zi[l];
      iters += it;
      errAny |= e;
    }
    if (errAny) err = 1;
    bfgsIters += iters;
    hessComputed = true;
    return sse2_redux(nF, [&](long i) { return IhVec[i]; });
  }

  // Mesh<D>::eulerGrad (Mesh.cpp:582-624)
  double eulerGrad(const std::vector<double>& xv, std::vector<double>& grad) {
    std::fill(grad.begin(), grad.end(), 0.0);
    double Ihorig = 0.0;
    double zi[K], xi[K], g[K], Igt;
    for (int i = 0; i < nF; i++) {
      simplexXi(i, xi);
      for (int n = 0; n < D + 1; n++)
        for (int l = 0; l < D; l++) zi[n * D + l] = xv[D * F[i * (D + 1) + n] + l];
      Ihorig += computeBlockGrad(i, zi, xi, g, true, false, &Igt, nullptr);
      for (int n = 0; n < D + 1; n++) {
        const int off = F[i * (D + 1) + n];
        for (int l = 0; l < D; ++l) grad[D * off + l] += g[D * n + l];
      }
    }
    return Ihorig;
  }

  // Mesh<D>::predictX (Mesh.cpp:649-674)
  void predictX(int steps) {
    if (gradUse || steps <= 2) {
      std::vector<double> grad(x.size());
      eulerGrad(x, grad);
      for (size_t i = 0; i < x.size(); ++i) xBar[i] = x[i] - (dt / tau) * grad[i];
    } else {
      for (size_t i = 0; i < x.size(); ++i) xBar[i] = 2 * x[i] - xPrev[i];
    }
  }

  // cg->solve(vec): Eigen ConjugateGradient<Lower|Upper>, Jacobi preconditioner
  void cgSolve(const std::vector<double>& rhs, std::vector<double>& out) {
    const long n = (long)rhs.size();
    if (cgMode == 1) {
      for (long i = 0; i < n; ++i) out[i] = rhs[i] * invdiag[i];
      return;
    }
    std::vector<double> xs(n, 0.0), r(rhs), p(n), zz(n), tmp(n);
    const double rhsNorm2 = sse2_redux(n, [&](long i) { return rhs[i] * rhs[i]; });
    if (rhsNorm2 == 0) {
      out.assign(n, 0.0);
      return;
    }
    const double tol = std::numeric_limits<double>::epsilon();
    const double threshold = std::max(tol * tol * rhsNorm2, DBL_MIN);
    double residualNorm2 = sse2_redux(n, [&](long i) { return r[i] * r[i]; });
    if (residualNorm2 < threshold) {
      out = xs;
      return;
    }
    for (long i = 0; i < n; ++i) p[i] = invdiag[i] * r[i];
    double absNew = sse2_redux(n, [&](long i) { return r[i] * p[i]; });
    long it = 0;
    const long maxIters = 2 * n;
    while (it < maxIters) {
      for (long i = 0; i < n; ++i) tmp[i] = tdiag[i] * p[i];
      const double alpha = absNew / sse2_redux(n, [&](long i) { return p[i] * tmp[i]; });
      for (long i = 0; i < n; ++i) xs[i] += alpha * p[i];
      for (long i = 0; i < n; ++i) r[i] -= alpha * tmp[i];
      residualNorm2 = sse2_redux(n, [&](long i) { return r[i] * r[i]; });
      if (residualNorm2 < threshold) break;
      for (long i = 0; i < n; ++i) zz[i] = invdiag[i] * r[i];
      const double absOld = absNew;
      absNew = sse2_redux(n, [&](long i) { return r[i] * zz[i]; });
      const double beta = absNew / absOld;
      for (long i = 0; i < n; ++i) p[i] = zz[i] + beta * p[i];
      it++;
    }
    out = xs;
  }

  // vec = m*xBar + dt^2 * WD_T * (w*(z - uBar)); x = cg.solve(vec)
  void xUpdate() {
    const double dtsq = dt * dt;
    std::vector<double> P((size_t)nP * D, 0.0);
    for (int s = 0; s < nF; ++s)
      for (int n = 0; n < D + 1; ++n) {
        const int v = F[s * (D + 1) + n];
        for (int m = 0; m < D; ++m) {
          const size_t j = (size_t)s * K + n * D + m;
          P[v * D + m] += w * (w * (z[j] - uBar[j]));
        }
      }
    for (size_t i = 0; i < P.size(); ++i) vec[i] = (tau * xBar[i]) + dtsq * P[i];
    cgSolve(vec, x);
  }

  // MeshIntegrator<D>::step (MeshIntegrator.cpp:101-191)
  double step(int nIters, double tol, int* itersOut, double* primalOut, double* dualOut) {
    // Mesh<D>::setUp (src/Mesh.cpp:1006-1014, commented in the reference): with regrid on, the
    // monitor grid is rebuilt from the current Vp and the monitor at t = steps * dt
    if (regrid) buildGrid<D>(Vp.data(), nP, monType, grid, stepsTaken * dt);
    predictX(stepsTaken);
    xPrev = x;
    x = xBar;
    gatherD(x, z);
    if (!stepTaken) std::fill(uBar.begin(), uBar.end(), 0.0);
    if (stepsTaken == 0) gatherD(xPrev, z);
    double Ihstart = 0;
    xUpdate();
    int i;
    double primal = 0, dual = 0;
    const bool earlyExit = tol >= 0;
    const double proxTol = earlyExit ? tol : 1e-3;
    const long nz = (long)z.size();
    for (i = 0; i < nIters; i++) {
      for (long j = 0; j < nz; ++j) DXpU[j] = 0.0;
      gatherD(x, DXpU);
      for (long j = 0; j < nz; ++j) DXpU[j] = DXpU[j] + uBar[j];
      zPrev = z;
      const double IhCur = prox(DXpU, z, proxTol);
      if (i == 0) Ihstart = IhCur;
      stepTaken = true;
      for (long j = 0; j < nz; ++j) uBar[j] = DXpU[j] - z[j];
      xUpdate();
      std::vector<double> Dx(nz);
      gatherD(x, Dx);
      primal = sqrt(sse2_redux(nz, [&](long j) {
        const double t = Dx[j] - z[j];
        return t * t;
      }));
      dual = sqrt(sse2_redux(nz, [&](long j) {
        const double t = z[j] - zPrev[j];
        return t * t;
      }));
      if (earlyExit && primal < tol && dual < tol) break;
    }
    if (itersOut) *itersOut = (i < nIters) ? i + 1 : nIters;
    if (primalOut) *primalOut = primal;
    if (dualOut) *dualOut = dual;
    updateAfterStep();
    stepsTaken++;
    return Ihstart;
  }

  void updateAfterStep() {  // Mesh.cpp:1016-1036
    for (int i = 0; i < nP; i++)
      for (int j = 0; j < D; j++) Vp[i * D + j] = x[i * D + j];
  }

  // MeshIntegrator::eulerStep -> Mesh::eulerStepMod (Mesh.cpp:532-579): interior nodes only,
  // blockGrad without FIXED-row zeroing, x -= (dt/tau) grad.
  double eulerStep() {
    std::vector<double> grad(x.size(), 0.0);
    double Ihorig = 0.0;
    double zi[K], xi[K], g[K], Igt;
    for (int i = 0; i < nF; i++) {
      simplexXi(i, xi);
      for (int n = 0; n < D + 1; n++)
        for (int l = 0; l < D; l++) zi[n * D + l] = x[D * F[i * (D + 1) + n] + l];
      Ihorig += blockGrad(i, zi, xi, g, true, false, &Igt, nullptr);
      for (int n = 0; n < D + 1; n++) {
        const int off = F[i * (D + 1) + n];
        if (mask[off] == INTERIOR)
          for (int l = 0; l < D; ++l) grad[D * off + l] += g[D * n + l];
      }
    }
    for (size_t i = 0; i < x.size(); ++i) x[i] -= (dt / tau) * grad[i];
    return Ihorig;
  }

  // ---- backward Euler (method 2) ------------------------------------------------------------
  // Mesh<D>::eulerStepMod (Mesh.cpp:532-579): blockGrad (no FIXED zeroing) scattered to INTERIOR
  // nodes; returns the summed energy.
  double eulerStepMod(const std::vector<double>& xv, std::vector<double>& grad) {
    std::fill(grad.begin(), grad.end(), 0.0);
    double Ihorig = 0.0;
    double zi[K], xi[K], g[K], Igt;
    for (int i = 0; i < nF; i++) {
      simplexXi(i, xi);
      for (int n = 0; n < D + 1; n++)
        for (int l = 0; l < D; l++) zi[n * D + l] = xv[D * F[i * (D + 1) + n] + l];
      Ihorig += blockGrad(i, zi, xi, g, true, false, &Igt, nullptr);
      for (int n = 0; n < D + 1; n++) {
        const int off = F[i * (D + 1) + n];
        if (mask[off] == INTERIOR)
          for (int l = 0; l < D; ++l) grad[D * off + l] += g[D * n + l];
      }
    }
    return Ihorig;
  }

  std::vector<int> jia, jja;  // buildMatrix pattern (Mesh.cpp:309-345)
  std::vector<double> jval;
  bool beStepTaken = false;
  int lastNewton = 0;

  // Mesh<D>::buildEulerJac + FSubJac (Mesh.cpp:1112-1261): finite-difference Jacobian of the
  // gradient, evaluated at Vp (the initial mesh: Vp is only updated by done(), App. A-16).
  void buildEulerJac(double dtBE) {
    std::fill(jval.begin(), jval.end(), 0.0);
    std::vector<std::vector<int>> conn(nP);  // simplexConnects: ascending simplex ids
    for (int s = 0; s < nF; ++s)
      for (int n = 0; n < D + 1; ++n) conn[F[s * (D + 1) + n]].push_back(s);
    const double h = 10.0 * sqrt(std::numeric_limits<double>::epsilon());
    double xLoc[K], xiLoc[K], Gk[K], Gkp1[K], xPurt[K], derivs[D][K], Igt;
    for (int pntId = 0; pntId < nP; ++pntId) {
      auto& sids = conn[pntId];
      sids.erase(std::unique(sids.begin(), sids.end()), sids.end());
      for (int sId : sids) {
        int off = 0;
        simplexXi(sId, xiLoc);
        for (int n = 0; n < D + 1; n++) {
          const int v = F[sId * (D + 1) + n];
          if (v == pntId) off = n;
          for (int l = 0; l < D; l++) xLoc[n * D + l] = Vp[(size_t)v * D + l];
        }
        blockGrad(sId, xLoc, xiLoc, Gk, true, false, &Igt, nullptr);
        for (int i = 0; i < K; ++i) xPurt[i] = xLoc[i];
        if (mask[pntId] == BOUNDARY_FIXED) {
          for (int r = 0; r < D; r++)
            for (int c = 0; c < K; c++) derivs[r][c] = 0.0;
          for (int r = 0; r < D; r++)
            for (int c = D * off; c < D * (off + 1); c++)
              if (r == c) derivs[r][c] = 1.0;  // only for off == 0 (App. A-17)
        } else {
          for (int i = 0; i < D; i++) {
            xPurt[D * off + i] += h;
            blockGrad(sId, xPurt, xiLoc, Gkp1, true, false, &Igt, nullptr);
            for (int c = 0; c < K; ++c) derivs[i][c] = (Gkp1[c] - Gk[c]) / h;
            xPurt[D * off + i] = xLoc[D * off + i];
          }
        }
        int sorted[D + 1], rel[D + 1];  // pairsort by node id
        for (int r = 0; r < D + 1; r++) {
          sorted[r] = F[sId * (D + 1) + r];
          rel[r] = r;
        }
        for (int a = 1; a < D + 1; ++a)
          for (int b = a; b > 0 && sorted[b - 1] > sorted[b]; --b) {
            std::swap(sorted[b - 1], sorted[b]);
            std::swap(rel[b - 1], rel[b]);
          }
        for (int pp = 0; pp < D; pp++) {
          const int row = D * pntId + pp;
          for (int i = jia[row]; i < jia[row + 1]; i++) {
            const int colIndex = jja[i] / D, colOff = jja[i] % D;
            for (int j = 0; j < D + 1; j++) {
              if (sorted[j] == colIndex)
                jval[i] += derivs[pp][D * rel[j] + colOff];
              else
                jval[i] += 0.0;
            }
          }
        }
      }
    }
    const int n = D * nP;
    for (int r = 0; r < n; r++)
      for (int i = jia[r]; i < jia[r + 1]; i++) {
        jval[i] *= (dtBE / tau);
        if (jja[i] == r) jval[i] += 1.0;
      }
  }

  // Mesh<D>::backwardsEulerStep (Mesh.cpp:1263-1341): Newton on F(x) = (dt/tau) grad + (x - xn)
  // with the ILU(0)-CG-STAB solve (lib/LASolver); returns the last eulerStepMod energy.
  double backwardsEulerStep(double dtBE, double tol, int dotMode) {
    const int n = D * nP;
    if (jia.empty()) {  // buildMatrix
      jia.resize(n + 1);
      const int nnz = orc_la_mesh_pattern(D, nP, nF, F.data(), jia.data(), nullptr, 0);
      jja.resize(nnz);
      orc_la_mesh_pattern(D, nP, nF, F.data(), jia.data(), jja.data(), nnz);
      jval.assign(nnz, 0.0);
    }
    const std::vector<double> xn = x;
    const double SAFETY_FAC = 1.0 / 10.0;
    std::vector<double> grad(n, 0.0), rhs(n), dx(n);
    double Ih = eulerStepMod(x, grad);
    for (int i = 0; i < n; ++i) x[i] -= (dtBE / tau) * grad[i];
    const int MAX_ITERS = 1000;
    int nIter = 0;
    double gradOneN = 0, gradOneNPrev = INFINITY;
    if (!beStepTaken) buildEulerJac(dtBE);  // (+ sfac)
    do {
      Ih = eulerStepMod(x, grad);
      for (int i = 0; i < n; ++i) grad[i] *= (dtBE / tau);
      for (int i = 0; i < n; ++i) grad[i] += (x[i] - xn[i]);
      gradOneN = sse2_redux(n, [&](long i) { return std::fabs(grad[i]); });
      if (gradOneN < SAFETY_FAC * tol) break;
      if (!beStepTaken || std::fabs(gradOneN - gradOneNPrev) / (gradOneN) < 0.25) {
        buildEulerJac(dtBE);
        beStepTaken = true;
      }
      for (int i = 0; i < n; ++i) rhs[i] = -grad[i];
      int cgIter = 0;
      orc_la_solve(n, jia.data(), jja.data(), jval.data(), rhs.data(), nullptr, 10000, 1e-6, 0, 0, dx.data(), &cgIter,
                   nullptr, dotMode);
      if (cgIter <= 0) {  // the reference asserts cgIter > 0
        err = 1;
        break;
      }
      for (int i = 0; i < n; ++i) x[i] += dx[i];
      nIter++;
      gradOneNPrev = gradOneN;
    } while (nIter < MAX_ITERS);
    lastNewton = nIter;
    return Ih;
  }

  // Mesh<D>::computeEnergy (Mesh.cpp:496-530) on Vp
  double energy() const {
    double Ih = 0.0;
    double zi[K], xi[K], g[K];
    for (int i = 0; i < nF; i++) {
      simplexXi(i, xi);
      for (int n = 0; n < D + 1; n++)
        for (int l = 0; l < D; l++) zi[n * D + l] = Vp[F[i * (D + 1) + n] * D + l];
      Ih += computeBlockGrad(i, zi, xi, g, false, false, nullptr, nullptr);
    }
    return Ih;
  }
};

}  // namespace orc

using namespace orc;

extern "C" {

// OpenMP threads of the prox restatement (process-wide, like the reference's Mesh ctor, Mesh.cpp:428-438)
void orc_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}

void* orc_mesh_rect(int dim, int nx, int ny, int nz, double xa, double xb, double ya, double yb,
                    double za, double zb, int btype) {
  auto* m = new MeshData();
  genRect(dim, nx, ny, nz, xa, xb, ya, yb, za, zb, btype, *m);
  return m;
}
void* orc_mesh_levelset2d(int nx, int ny, double xa, double xb, double ya, double yb, int btype,
                          int compactMask) {
  auto* m = new MeshData();
  genLevelSet2D(nx, ny, xa, xb, ya, yb, btype, compactMask, *m);
  return m;
}
void* orc_mesh_levelset3d(int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za,
                          double zb, int btype, int compactMask) {
  auto* m = new MeshData();
  genLevelSet3D(nx, ny, nz, xa, xb, ya, yb, za, zb, btype, compactMask, *m);
  return m;
}
void* orc_mesh_read(int dim, const char* tri, const char* pnts, const char* mask) {
  auto* m = new MeshData();
  if (!readMesh(dim, tri, pnts, mask, *m)) {
    delete m;
    return nullptr;
  }
  return m;
}
void orc_mesh_sizes(void* h, int* nP, int* nF, int* maskLen) {
  auto* m = (MeshData*)h;
  *nP = m->nP();
  *nF = m->nF();
  *maskLen = (int)m->mask.size();
}
void orc_mesh_copy(void* h, double* Vp, int* F, int* mask) {
  auto* m = (MeshData*)h;
  std::memcpy(Vp, m->Vp.data(), m->Vp.size() * sizeof(double));
  std::memcpy(F, m->F.data(), m->F.size() * sizeof(int));
  std::memcpy(mask, m->mask.data(), m->mask.size() * sizeof(int));
}
void orc_mesh_free(void* h) { delete (MeshData*)h; }

void* orc_create(int dim, int nP, const double* Vp, const double* Vc, int nF, const int* F,
                 const int* mask, int monType, double dt, double tau, double rho, int gradUse,
                 int nthreads, int cgMode) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  if (dim == 2) {
    auto* s = new Integrator<2>();
    s->init(nP, Vp, Vc, nF, F, mask, monType, dt, tau, rho, gradUse, cgMode);
    return (Base*)s;
  }
  auto* s = new Integrator<3>();
  s->init(nP, Vp, Vc, nF, F, mask, monType, dt, tau, rho, gradUse, cgMode);
  return (Base*)s;
}

#define DISPATCH(h, expr2, expr3)                    \
  do {                                               \
    Base* b_ = (Base*)(h);                           \
    if (b_->dim == 2) {                              \
      auto* s = static_cast<Integrator<2>*>(b_);     \
      expr2;                                         \
    } else {                                         \
      auto* s = static_cast<Integrator<3>*>(b_);     \
      expr3;                                         \
    }                                                \
  } while (0)

int orc_step(void* h, int nIters, double tol, double* Ih, int* admmIters, double* primal, double* dual) {
  double r = 0;
  int e = 0;
  DISPATCH(h, (r = s->step(nIters, tol, admmIters, primal, dual), e = s->err),
           (r = s->step(nIters, tol, admmIters, primal, dual), e = s->err));
  *Ih = r;
  return e;
}
void orc_set_regrid(void* h, int on) { ((Base*)h)->regrid = on; }
int orc_euler_step(void* h, double* Ih) {
  double r = 0;
  DISPATCH(h, r = s->eulerStep(), r = s->eulerStep());
  *Ih = r;
  return 0;
}
int orc_backward_euler_step(void* h, double dt, double tol, int dotMode, double* Ih, int* newtonIters) {
  double r = 0;
  int e = 0, it = 0;
  DISPATCH(h, (r = s->backwardsEulerStep(dt, tol, dotMode), e = s->err, it = s->lastNewton),
           (r = s->backwardsEulerStep(dt, tol, dotMode), e = s->err, it = s->lastNewton));
  *Ih = r;
  if (newtonIters) *newtonIters = it;
  return e;
}
void orc_get_jacobian(void* h, int* ia, int* ja, double* a) {
  DISPATCH(h, (std::copy(s->jia.begin(), s->jia.end(), ia), std::copy(s->jja.begin(), s->jja.end(), ja),
               std::copy(s->jval.begin(), s->jval.end(), a)),
           (std::copy(s->jia.begin(), s->jia.end(), ia), std::copy(s->jja.begin(), s->jja.end(), ja),
            std::copy(s->jval.begin(), s->jval.end(), a)));
}
long long orc_jacobian_nnz(void* h) {
  long long r = 0;
  DISPATCH(h, r = (long long)s->jja.size(), r = (long long)s->jja.size());
  return r;
}
double orc_energy(void* h) {
  double r = 0;
  DISPATCH(h, r = s->energy(), r = s->energy());
  return r;
}
void orc_done(void* h) { DISPATCH(h, s->updateAfterStep(), s->updateAfterStep()); }

}  // extern "C"
template <class S>
static void getVec(S* s, const char* what, double* out) {
  const std::vector<double>* v = nullptr;
  std::string w(what);
  if (w == "x") v = &s->x;
  else if (w == "xPrev") v = &s->xPrev;
  else if (w == "xBar") v = &s->xBar;
  else if (w == "z") v = &s->z;
  else if (w == "u") v = &s->uBar;
  else if (w == "points") v = &s->Vp;
  else if (w == "hess") v = &s->hess;
  else if (w == "grid") v = &s->grid.vals;
  else if (w == "tdiag") v = &s->tdiag;
  else if (w == "Ih") v = &s->IhVec;
  else if (w == "Ehat") {
    for (int r = 0; r < s->dim; ++r)
      for (int c = 0; c < s->dim; ++c) out[r * s->dim + c] = s->EhatConst.m[r][c];
    return;
  }
  if (v) std::memcpy(out, v->data(), v->size() * sizeof(double));
}
extern "C" {
void orc_get(void* h, const char* what, double* out) { DISPATCH(h, getVec(s, what, out), getVec(s, what, out)); }
void orc_get_F(void* h, int* F) {
  DISPATCH(h, std::memcpy(F, s->F.data(), s->F.size() * sizeof(int)),
           std::memcpy(F, s->F.data(), s->F.size() * sizeof(int)));
}
void orc_sizes(void* h, int* nP, int* nF, int* gridRows, int* gnx, int* gny, int* gnz) {
  DISPATCH(h,
           (*nP = s->nP, *nF = s->nF, *gridRows = s->grid.rows(), *gnx = s->grid.nx, *gny = s->grid.ny, *gnz = s->grid.nz),
           (*nP = s->nP, *nF = s->nF, *gridRows = s->grid.rows(), *gnx = s->grid.nx, *gny = s->grid.ny, *gnz = s->grid.nz));
}
long long orc_bfgs_iters(void* h) {
  long long r = 0;
  DISPATCH(h, r = s->bfgsIters, r = s->bfgsIters);
  return r;
}
int orc_error(void* h) { return ((Base*)h)->err; }
double orc_block_grad(void* h, int sid, const double* z, const double* dxpu, double* grad, int computeGrad,
                      int regularize, double* Igt) {
  double r = 0;
  DISPATCH(h,
           {
             double xi[6];
             s->simplexXi(sid, xi);
             r = s->computeBlockGrad(sid, z, xi, grad, computeGrad, regularize, Igt, dxpu);
           },
           {
             double xi[12];
             s->simplexXi(sid, xi);
             r = s->computeBlockGrad(sid, z, xi, grad, computeGrad, regularize, Igt, dxpu);
           });
  return r;
}
void orc_eval_monitor(void* h, const double* pnt, double* M) {
  DISPATCH(h,
           {
             Mat<2> m;
             evalMonitor<2>(s->grid, pnt, m);
             for (int i = 0; i < 4; ++i) M[i] = m.m[i / 2][i % 2];
           },
           {
             Mat<3> m;
             evalMonitor<3>(s->grid, pnt, m);
             for (int i = 0; i < 9; ++i) M[i] = m.m[i / 3][i % 3];
           });
}
void orc_monitor_at(int dim, int monType, const double* x, double* M) { monitorAt(dim, monType, x, M); }
void orc_set_pow_mode(int mode) { g_powMode = mode; }
double orc_crpow(double x, double y) { return crpow(x, y); }
void orc_destroy(void* h) { delete (Base*)h; }

}  // extern "C"
