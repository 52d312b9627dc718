// admm_device.h -- per-simplex Huang-functional arithmetic for the CDNA4 ADMM kernels.
//
// One lane owns one simplex.  Every function follows the operation order of the reference
// (src/AdaptationFunctional.cpp:102-287, src/MeshInterpolator.cpp:287-342,
// src/MeshUtils.h:45-80) with the small-matrix conventions documented in DESIGN.md
// (Eigen 3.4 closed-form 2x2/3x3 determinant and inverse, ascending inner sums).  The
// translation unit is compiled with -ffp-contract=off, so no multiply-add is fused unless
// written as fma(); the powers go through crmath.h.  The result is bit-identical to the
// CPU oracle run with correctly rounded pow (tests/test_gpu_parity.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crmath.h"

namespace mmx {

enum : int { BOUNDARY_FREE = 0, BOUNDARY_FIXED = 1, INTERIOR = 2 };  // src/NodeType.h:4-8

template <int D>
struct GridView {  // the smoothed monitor grid, rows of D*D doubles
  const double* gx;
  const double* gy;
  const double* gz;
  const double* vals;
  const double* pad;  // 3D: the grid rows padded to 10 doubles (16-byte aligned rows)
  const double* cell[3];  // 3D: per axis and cell i {g_i, h_i = g_{i+1} - g_i, RN(1/h_i), 0}
  const double* iso;      // isotropic grid: one value per point (the diagonal), else nullptr
  int nx, ny, nz;
  double hx, hy, hz;     // gx[1]-gx[0] etc., the divisors of findLimInfMeshPoint
  double rhx, rhy, rhz;  // RN(1/h)
  // linspace (src/MeshUtils.h:24-29) parameters: g[i] = a + (i * span) / ns, recomputed on the
  // device instead of loaded (saves a dependent load before every monitor gather)
  double ax, ay, az, spx, spy, spz, nsx, nsy, nsz, rnsx, rnsy, rnsz;
  // set to 1 by a blockGrad that meets a finite Edet <= 0 (a NaN Edet -- NaN positions -- does
  // not set it): tells an inverted element from a non-finite monitor value at the step's end
  unsigned* invFlag;
};

// grid coordinate i of an axis, bit-identical to the host linspace (div_nr is exact here:
// i*span >= 0 and ns >= 1 are normal or zero)
__device__ __forceinline__ double gridCoord(double a, double span, double ns, double rns, int i) {
  return a + div_nr(((double)i) * span, ns, rns);
}

template <int D>
constexpr double kRecipD1 = 1.0 / ((double)D + 1.0);  // RN(1/(D+1))

template <int D>
struct FunctionalConsts {
  double Ehat[D * D];  // row-major, !CompMesh reference simplex (host computed, std::pow)
  double powd;         // pow(d, d*p/2) computed on the host with std::pow
  double w;            // 0.5*sqrt(rho)
  int compMesh;
};

template <int D>
struct M {  // row-major small matrix
  double m[D][D];
};

template <int D>
__device__ __forceinline__ double det(const M<D>& a) {
  if constexpr (D == 2) {
    return a.m[0][0] * a.m[1][1] - a.m[1][0] * a.m[0][1];
  } else {
    const double h0 = a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]);
    const double h1 = a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]);
    const double h2 = a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
    return h0 - h1 + h2;
  }
}

__device__ __forceinline__ double cof3(const M<3>& a, int i, int j) {
  const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return a.m[i1][j1] * a.m[i2][j2] - a.m[i1][j2] * a.m[i2][j1];
}

template <int D>
__device__ __forceinline__ M<D> inverse(const M<D>& a) {
  M<D> r;
  if constexpr (D == 2) {
    const double invdet = 1.0 / det<D>(a);
    r.m[0][0] = a.m[1][1] * invdet;
    r.m[1][0] = -a.m[1][0] * invdet;
    r.m[0][1] = -a.m[0][1] * invdet;
    r.m[1][1] = a.m[0][0] * invdet;
  } else {
    const double c0 = cof3(a, 0, 0), c1 = cof3(a, 1, 0), c2 = cof3(a, 2, 0);
    const double dt = (c0 * a.m[0][0] + c1 * a.m[1][0]) + c2 * a.m[2][0];
    const double invdet = 1.0 / dt;
#pragma unroll
    for (int i = 1; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) r.m[i][j] = cof3(a, j, i) * invdet;
    r.m[0][0] = c0 * invdet;
    r.m[0][1] = c1 * invdet;
    r.m[0][2] = c2 * invdet;
  }
  return r;
}

template <int D>
__device__ __forceinline__ M<D> mul(const M<D>& a, const M<D>& b) {
  M<D> c;
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double s = a.m[i][0] * b.m[0][j];
#pragma unroll
      for (int k = 1; k < D; ++k) s += a.m[i][k] * b.m[k][j];
      c.m[i][j] = s;
    }
  return c;
}

template <int D>
__device__ __forceinline__ M<D> transpose(const M<D>& a) {
  M<D> t;
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) t.m[i][j] = a.m[j][i];
  return t;
}

template <int D>
__device__ __forceinline__ double trace(const M<D>& a) {
  double s = a.m[0][0];
#pragma unroll
  for (int i = 1; i < D; ++i) s += a.m[i][i];
  return s;
}

// utils::findLimInfMeshPoint (src/MeshUtils.h:45-54): (int) cast, then uint32 clamp
__device__ __forceinline__ int findLimInf(double w, double m0, int size, double h, double rh) {
  // (w - m[0]) / (m[1] - m[0]); operands normal or zero, so div_nr is exact
  uint32_t guess = (uint32_t)(int)div_nr(w - m0, h, rh);
  if (guess > (uint32_t)(size - 2)) guess = (uint32_t)(size - 2);
  return (int)guess;
}

#ifndef MMX_MON_BATCH
#define MMX_MON_BATCH 1
#endif
#ifndef MMX_MON_PIPE
#define MMX_MON_PIPE 1
#endif
// 3D evalMonitorOnGrid in two halves, the loads of one point (monLoad3: the cell's coordinates
// and its eight corner rows) and the trilinear interpolation (monEval3), so blockGrad can request
// the next vertex's cell while it interpolates the current one: the same operations as the 3D
// branch of evalMonitor below
// MMX_MON_RECIP: the cell's coordinate, width and RN(1/width) from the per-axis cell tables, and
// the fraction (p - g_i) / (g_{i+1} - g_i) as div_nr (exact: both operands normal or zero, as for
// findLimInf) instead of an IEEE division
#ifndef MMX_MON_RECIP
#define MMX_MON_RECIP 0
#endif
struct MonIn3 {
  double x0, x1, y0, y1, z0, z1;  // MMX_MON_RECIP: x1 etc. hold the cell widths
#if MMX_MON_RECIP
  double rx, ry, rz;
#endif
  double r[8][9];
};
__device__ __forceinline__ void monLoad3(const GridView<3>& g, const double* pnt, MonIn3& in) {
  const int xInd = findLimInf(pnt[0], g.ax, g.nx + 1, g.hx, g.rhx);
  const int yInd = findLimInf(pnt[1], g.ay, g.ny + 1, g.hy, g.rhy);
  const int zInd = findLimInf(pnt[2], g.az, g.nz + 1, g.hz, g.rhz);
  const int nx = g.nx;
#if MMX_MON_RECIP
  {
    const double2* cx = reinterpret_cast<const double2*>(g.cell[0]) + 2 * xInd;
    const double2* cy = reinterpret_cast<const double2*>(g.cell[1]) + 2 * yInd;
    const double2* cz = reinterpret_cast<const double2*>(g.cell[2]) + 2 * zInd;
    const double2 ax = cx[0], bx = cx[1], ay = cy[0], by = cy[1], az = cz[0], bz = cz[1];
    in.x0 = ax.x;
    in.x1 = ax.y;
    in.rx = bx.x;
    in.y0 = ay.x;
    in.y1 = ay.y;
    in.ry = by.x;
    in.z0 = az.x;
    in.z1 = az.y;
    in.rz = bz.x;
  }
#else
#ifdef MMX_GRID_RECOMPUTE3
  in.x0 = gridCoord(g.ax, g.spx, g.nsx, g.rnsx, xInd);
  in.x1 = gridCoord(g.ax, g.spx, g.nsx, g.rnsx, xInd + 1);
  in.y0 = gridCoord(g.ay, g.spy, g.nsy, g.rnsy, yInd);
  in.y1 = gridCoord(g.ay, g.spy, g.nsy, g.rnsy, yInd + 1);
  in.z0 = gridCoord(g.az, g.spz, g.nsz, g.rnsz, zInd);
  in.z1 = gridCoord(g.az, g.spz, g.nsz, g.rnsz, zInd + 1);
#else
  in.x0 = g.gx[xInd];
  in.x1 = g.gx[xInd + 1];
  in.y0 = g.gy[yInd];
  in.y1 = g.gy[yInd + 1];
  in.z0 = g.gz[zInd];
  in.z1 = g.gz[zInd + 1];
#endif
#endif
  const size_t P = (size_t)(nx + 1) * (g.ny + 1);
  const size_t base = zInd * P + (size_t)yInd * (nx + 1) + xInd;
  const size_t rows[8] = {base, base + 1, base + nx + 1, base + nx + 2,
                          base + P, base + P + 1, base + P + nx + 1, base + P + nx + 2};
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const double2* rp = reinterpret_cast<const double2*>(g.pad + rows[q] * 10);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const double2 v = rp[e];
      in.r[q][2 * e] = v.x;
      in.r[q][2 * e + 1] = v.y;
    }
    in.r[q][8] = g.pad[rows[q] * 10 + 8];
  }
}
__device__ __forceinline__ void monEval3(const MonIn3& in, const double* pnt, M<3>& mv) {
#if MMX_MON_RECIP
  const double xd = div_nr(pnt[0] - in.x0, in.x1, in.rx);
  const double yd = div_nr(pnt[1] - in.y0, in.y1, in.ry);
  const double zd = div_nr(pnt[2] - in.z0, in.z1, in.rz);
#else
  const double xd = (pnt[0] - in.x0) / (in.x1 - in.x0);
  const double yd = (pnt[1] - in.y0) / (in.y1 - in.y0);
  const double zd = (pnt[2] - in.z0) / (in.z1 - in.z0);
#endif
  const double c[8] = {(1 - xd) * (1 - yd) * (1 - zd), xd * (1 - yd) * (1 - zd),
                       (1 - xd) * yd * (1 - zd),       xd * yd * (1 - zd),
                       (1 - xd) * (1 - yd) * zd,       xd * (1 - yd) * zd,
                       (1 - xd) * yd * zd,             xd * yd * zd};
  double f[9];
#pragma unroll
  for (int n = 0; n < 9; ++n) f[n] = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int n = 0; n < 9; ++n) f[n] += c[q] * in.r[q][n];
#pragma unroll
  for (int n = 0; n < 9; ++n) mv.m[n / 3][n % 3] = f[n];
}
// the same two halves on an isotropic grid (one value per point, GridView::iso): the corner values
// and the sums of monEval3 on the diagonal value and on the off-diagonal +0 (bit-identical)
struct MonIso3 {
  double x0, x1, y0, y1, z0, z1;
  double r[8];
};
__device__ __forceinline__ void monLoad3Iso(const GridView<3>& g, const double* pnt, MonIso3& in) {
  const int xInd = findLimInf(pnt[0], g.ax, g.nx + 1, g.hx, g.rhx);
  const int yInd = findLimInf(pnt[1], g.ay, g.ny + 1, g.hy, g.rhy);
  const int zInd = findLimInf(pnt[2], g.az, g.nz + 1, g.hz, g.rhz);
  const int nx = g.nx;
#ifdef MMX_GRID_RECOMPUTE3
  in.x0 = gridCoord(g.ax, g.spx, g.nsx, g.rnsx, xInd);
  in.x1 = gridCoord(g.ax, g.spx, g.nsx, g.rnsx, xInd + 1);
  in.y0 = gridCoord(g.ay, g.spy, g.nsy, g.rnsy, yInd);
  in.y1 = gridCoord(g.ay, g.spy, g.nsy, g.rnsy, yInd + 1);
  in.z0 = gridCoord(g.az, g.spz, g.nsz, g.rnsz, zInd);
  in.z1 = gridCoord(g.az, g.spz, g.nsz, g.rnsz, zInd + 1);
#else
  in.x0 = g.gx[xInd];
  in.x1 = g.gx[xInd + 1];
  in.y0 = g.gy[yInd];
  in.y1 = g.gy[yInd + 1];
  in.z0 = g.gz[zInd];
  in.z1 = g.gz[zInd + 1];
#endif
  const size_t P = (size_t)(nx + 1) * (g.ny + 1);
  const size_t base = zInd * P + (size_t)yInd * (nx + 1) + xInd;
  const size_t rows[8] = {base, base + 1, base + nx + 1, base + nx + 2,
                          base + P, base + P + 1, base + P + nx + 1, base + P + nx + 2};
#pragma unroll
  for (int q = 0; q < 8; ++q) in.r[q] = g.iso[rows[q]];
}
__device__ __forceinline__ void monEval3Iso(const MonIso3& in, const double* pnt, M<3>& mv) {
  const double xd = (pnt[0] - in.x0) / (in.x1 - in.x0);
  const double yd = (pnt[1] - in.y0) / (in.y1 - in.y0);
  const double zd = (pnt[2] - in.z0) / (in.z1 - in.z0);
  const double c[8] = {(1 - xd) * (1 - yd) * (1 - zd), xd * (1 - yd) * (1 - zd),
                       (1 - xd) * yd * (1 - zd),       xd * yd * (1 - zd),
                       (1 - xd) * (1 - yd) * zd,       xd * (1 - yd) * zd,
                       (1 - xd) * yd * zd,             xd * yd * zd};
  double d = 0.0, o = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    d += c[q] * in.r[q];
    o += c[q] * 0.0;
  }
#pragma unroll
  for (int n = 0; n < 9; ++n) mv.m[n / 3][n % 3] = (n / 3 == n % 3) ? d : o;
}
// MeshInterpolator<D>::evalMonitorOnGrid (src/MeshInterpolator.cpp:287-342)
template <int D>
__device__ __forceinline__ void evalMonitor(const GridView<D>& g, const double* pnt, M<D>& mv) {
  const int xInd = findLimInf(pnt[0], g.ax, g.nx + 1, g.hx, g.rhx);
  const int yInd = findLimInf(pnt[1], g.ay, g.ny + 1, g.hy, g.rhy);
  const int nx = g.nx;
  if constexpr (D == 2) {
    // the cell's coordinates recomputed (gridCoord, bit-identical to the host linspace) rather than
    // loaded: the loads were a dependent round trip after the index (round 4, C3 prox 0.365 ->
    // 0.323 ms with the isotropic grid; round 1, with four 32-byte corner rows behind them, loading
    // measured cheaper)
#ifdef MMX_GRID_LOAD
    const double xm0 = g.gx[xInd], xm1 = g.gx[xInd + 1], ym0 = g.gy[yInd], ym1 = g.gy[yInd + 1];
#else
    const double xm0 = gridCoord(g.ax, g.spx, g.nsx, g.rnsx, xInd), xm1 = gridCoord(g.ax, g.spx, g.nsx, g.rnsx, xInd + 1);
    const double ym0 = gridCoord(g.ay, g.spy, g.nsy, g.rnsy, yInd), ym1 = gridCoord(g.ay, g.spy, g.nsy, g.rnsy, yInd + 1);
#endif
    const double x = pnt[0], y = pnt[1];
    const double norm = (1 / ((xm1 - xm0) * (ym1 - ym0)));
    const double c0 = norm * (xm1 - x) * (ym1 - y), c1 = norm * (x - xm0) * (ym1 - y);
    const double c2 = norm * (xm1 - x) * (y - ym0), c3 = norm * (x - xm0) * (y - ym0);
    if (g.iso) {
      // an isotropic grid (every point s I, off-diagonals +0): the same sums as below on one value
      // per corner -- 8 bytes gathered per corner instead of 32; the off-diagonal sums of +0 are
      // formed as below, so they are bit-identical too (NaN positions included)
      const double* r0 = g.iso + (size_t)yInd * (nx + 1) + xInd;
      const double* r1 = r0 + (nx + 1);
      const double a = r0[0], b = r0[1], e = r1[0], f = r1[1];
      const double d = c0 * a + c1 * b + c2 * e + c3 * f;
      const double o = c0 * 0.0 + c1 * 0.0 + c2 * 0.0 + c3 * 0.0;
      mv.m[0][0] = d;
      mv.m[0][1] = o;
      mv.m[1][0] = o;
      mv.m[1][1] = d;
      return;
    }
    const double2* r0 = reinterpret_cast<const double2*>(g.vals + ((size_t)yInd * (nx + 1) + xInd) * 4);
    const double2* r1 = reinterpret_cast<const double2*>(g.vals + ((size_t)(yInd + 1) * (nx + 1) + xInd) * 4);
    const double2 a0 = r0[0], a1 = r0[1], b0 = r0[2], b1 = r0[3];  // g00, g10
    const double2 e0 = r1[0], e1 = r1[1], f0 = r1[2], f1 = r1[3];  // g01, g11
    mv.m[0][0] = c0 * a0.x + c1 * b0.x + c2 * e0.x + c3 * f0.x;
    mv.m[0][1] = c0 * a0.y + c1 * b0.y + c2 * e0.y + c3 * f0.y;
    mv.m[1][0] = c0 * a1.x + c1 * b1.x + c2 * e1.x + c3 * f1.x;
    mv.m[1][1] = c0 * a1.y + c1 * b1.y + c2 * e1.y + c3 * f1.y;
  } else {
    const int zInd = findLimInf(pnt[2], g.az, g.nz + 1, g.hz, g.rhz);
    const double x0 = g.gx[xInd], x1 = g.gx[xInd + 1];
    const double y0 = g.gy[yInd], y1 = g.gy[yInd + 1];
    const double z0 = g.gz[zInd], z1 = g.gz[zInd + 1];
    const double xd = (pnt[0] - x0) / (x1 - x0);
    const double yd = (pnt[1] - y0) / (y1 - y0);
    const double zd = (pnt[2] - z0) / (z1 - z0);
    const double c[8] = {(1 - xd) * (1 - yd) * (1 - zd), xd * (1 - yd) * (1 - zd),
                         (1 - xd) * yd * (1 - zd),       xd * yd * (1 - zd),
                         (1 - xd) * (1 - yd) * zd,       xd * (1 - yd) * zd,
                         (1 - xd) * yd * zd,             xd * yd * zd};
    const size_t P = (size_t)(nx + 1) * (g.ny + 1);
    const size_t base = zInd * P + (size_t)yInd * (nx + 1) + xInd;
    const size_t rows[8] = {base, base + 1, base + nx + 1, base + nx + 2,
                            base + P, base + P + 1, base + P + nx + 1, base + P + nx + 2};
    if (g.iso) {  // an isotropic grid (monEval3)
      double d = 0.0, o = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        d += c[q] * g.iso[rows[q]];
        o += c[q] * 0.0;
      }
#pragma unroll
      for (int n = 0; n < 9; ++n) mv.m[n / 3][n % 3] = (n / 3 == n % 3) ? d : o;
      return;
    }
    // rows read from the 10-double padded copy: 5 16-byte loads per row instead of 9 8-byte ones
    // (the same values; the sums below are unchanged).  All eight rows are requested before the
    // first is used: loaded row by row, the compiler waited for each corner before requesting the
    // next (eight dependent cache round trips per vertex)
    double f[9];
#pragma unroll
    for (int n = 0; n < 9; ++n) f[n] = 0.0;
#if MMX_MON_BATCH
    double r[8][10];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double2* rp = reinterpret_cast<const double2*>(g.pad + rows[q] * 10);
#pragma unroll
      for (int e = 0; e < 5; ++e) {
        const double2 v = rp[e];
        r[q][2 * e] = v.x;
        r[q][2 * e + 1] = v.y;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int n = 0; n < 9; ++n) f[n] += c[q] * r[q][n];
#else
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double2* rp = reinterpret_cast<const double2*>(g.pad + rows[q] * 10);
      double r[10];
#pragma unroll
      for (int e = 0; e < 5; ++e) {
        const double2 v = rp[e];
        r[2 * e] = v.x;
        r[2 * e + 1] = v.y;
      }
#pragma unroll
      for (int n = 0; n < 9; ++n) f[n] += c[q] * r[n];
    }
#endif
#pragma unroll
    for (int n = 0; n < 9; ++n) mv.m[n / 3][n % 3] = f[n];
  }
}

// exponents d*p/2, d*p/2-1 for this dimension
template <int D, bool EXACT>
__device__ __forceinline__ double pow_dp2(double x, bool& tie) {
  if constexpr (D == 2) return cr_pow_p15<EXACT>(x, tie);
  else return cr_pow_p225<EXACT>(x, tie);
}
template <int D, bool EXACT>
__device__ __forceinline__ double pow_dp2m1(double x, bool& tie) {
  if constexpr (D == 2) return cr_pow_p05(x);
  else return cr_pow_p125<EXACT>(x, tie);
}

// AdaptationFunctional<D>::blockGrad (src/AdaptationFunctional.cpp:102-287).
// Returns the (regularised if REG) energy, sets Igt = |K| G, grad (if GRAD).
// An inverted element (assert(Edet > 0), line 174) returns NaN and a NaN gradient.
// ghuang (optional): receives the unregularised gradient |K| dG (K values) -- the part of the
// result that depends on z alone, reused by the next prox at the same z.  (Igt is not kept: the
// energy a prox reports is only read for the first prox of a step, which never uses the cache.)
// EXACT = false (prox fast path): a power too close to a rounding midpoint, or outside the
// double-double ranges, raises *tie instead of being resolved; the results are then void.
template <int D, bool GRAD, bool REG, bool EXACT = true>
__device__ __forceinline__ double blockGrad(const GridView<D>& g, const FunctionalConsts<D>& fc,
                                            const double* z, const double* xi, const double* dxpu,
                                            double* grad, double& Igt, double* ghuang = nullptr,
                                            bool* tiep = nullptr) {
  bool tie = false;
  constexpr int K = D * (D + 1);
  const double dFact = (D == 2) ? 2.0 : 6.0;
  M<D> mPre[D + 1], Msum;
  if constexpr (D == 3 && MMX_MON_PIPE) {  // vertex i + 1's cell requested while vertex i interpolates
    if (g.iso) {
      MonIso3 ja, jb;
      monLoad3Iso(g, &z[0], ja);
      monLoad3Iso(g, &z[3], jb);
      monEval3Iso(ja, &z[0], mPre[0]);
      monLoad3Iso(g, &z[6], ja);
      monEval3Iso(jb, &z[3], mPre[1]);
      monLoad3Iso(g, &z[9], jb);
      monEval3Iso(ja, &z[6], mPre[2]);
      monEval3Iso(jb, &z[9], mPre[3]);
    } else {
      MonIn3 ia, ib;
      monLoad3(g, &z[0], ia);
      monLoad3(g, &z[3], ib);
      monEval3(ia, &z[0], mPre[0]);
      monLoad3(g, &z[6], ia);
      monEval3(ib, &z[3], mPre[1]);
      monLoad3(g, &z[9], ib);
      monEval3(ia, &z[6], mPre[2]);
      monEval3(ib, &z[9], mPre[3]);
    }
  }
#pragma unroll
  for (int i = 0; i < D + 1; i++) {
    if constexpr (!(D == 3 && MMX_MON_PIPE)) evalMonitor<D>(g, &z[i * D], mPre[i]);
#pragma unroll
    for (int r = 0; r < D; ++r)
#pragma unroll
      for (int c = 0; c < D; ++c) Msum.m[r][c] = ((i == 0) ? 0.0 : Msum.m[r][c]) + mPre[i].m[r][c];
  }
  // the vertex differences the gradient needs (formed here, so only D matrices stay live instead
  // of the D + 1 vertex monitors; the values are the same)
  M<D> dmv[D];
#pragma unroll
  for (int j = 0; j < D; ++j)
#pragma unroll
    for (int r = 0; r < D; ++r)
#pragma unroll
      for (int c = 0; c < D; ++c) dmv[j].m[r][c] = mPre[j + 1].m[r][c] - mPre[0].m[r][c];
  M<D> Minv = inverse<D>(Msum);
#pragma unroll
  for (int r = 0; r < D; ++r)
#pragma unroll
    for (int c = 0; c < D; ++c) Minv.m[r][c] = Minv.m[r][c] / ((double)D + 1);
  M<D> E, Ehat;
#pragma unroll
  for (int j = 0; j < D; ++j) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
      E.m[r][j] = z[D * (j + 1) + r] - z[r];
      Ehat.m[r][j] = fc.compMesh ? (xi[D * (j + 1) + r] - xi[r]) : fc.Ehat[r * D + j];
    }
  }
  const double Edet = det<D>(E);
  if (!(Edet > 0)) {
    if (Edet <= 0 && g.invFlag) *g.invFlag = 1u;  // cold path: a vector store to global memory
    const double nan = __builtin_nan("");
    if constexpr (GRAD) {
#pragma unroll
      for (int i = 0; i < K; ++i) grad[i] = nan;
      if (ghuang)
#pragma unroll
        for (int i = 0; i < K; ++i) ghuang[i] = nan;
    }
    Igt = nan;
    return nan;
  }
  const M<D> Einv = inverse<D>(E);
  const M<D> FJ = mul<D>(Ehat, Einv);
  const double detFJ = det<D>(FJ);
  const double d = (double)D;
  const double p = 1.5;
  const double theta = 1.0 / 3.0;
  const M<D> FJt = transpose<D>(FJ);
  const M<D> MinvJt = mul<D>(Minv, FJt);
  const M<D> JMJt = mul<D>(FJ, MinvJt);
  const double trJMJt = trace<D>(JMJt);
  const double detM = cr_sqrt(1.0 / det<D>(Minv));
  const double tr_dp2 = pow_dp2<D, EXACT>(trJMJt, tie);
  const double G = theta * detM * tr_dp2 + (1.0 - 2.0 * theta) * fc.powd * detM * cr_pow_p15<EXACT>(detFJ / detM, tie);
  const double absK = __builtin_fabs(Edet / dFact);
  double sq = 0.0;
  if constexpr (REG) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const double t = dxpu[i] - z[i];
      sq = (i == 0) ? t * t : sq + t * t;
    }
  }
  if constexpr (!EXACT) *tiep = *tiep || tie;
  if constexpr (!GRAD) {
    Igt = absK * G;
    if constexpr (REG) return absK * G + 0.5 * fc.w * fc.w * sq;
    return absK * G;
  } else {
    const double tr_dp2m1 = pow_dp2m1<D, EXACT>(trJMJt, tie);
    const double detM_1mp = cr_pow_m05<EXACT>(detM, tie);
    M<D> dGdJ;
    {
      const double s = d * p * theta * detM * tr_dp2m1;
#pragma unroll
      for (int r = 0; r < D; ++r)
#pragma unroll
        for (int c = 0; c < D; ++c) dGdJ.m[r][c] = s * MinvJt.m[r][c];
    }
    const double dGddet = p * (1.0 - 2.0 * theta) * fc.powd * detM_1mp * cr_pow_p05(detFJ);
    M<D> dGdM;
    {
      const double s1 = -0.5 * theta * d * p * detM * tr_dp2m1;
      const M<D> MinvT = transpose<D>(Minv);
      M<D> T;
#pragma unroll
      for (int r = 0; r < D; ++r)
#pragma unroll
        for (int c = 0; c < D; ++c) T.m[r][c] = s1 * MinvT.m[r][c];
      T = mul<D>(mul<D>(mul<D>(T, FJt), FJ), Minv);
      const double s2 = 0.5 * theta * detM * tr_dp2 +
                        ((0.5 - theta) * (1.0 - p) * fc.powd) * detM_1mp * cr_pow_p15<EXACT>(detFJ, tie);
#pragma unroll
      for (int r = 0; r < D; ++r)
#pragma unroll
        for (int c = 0; c < D; ++c) dGdM.m[r][c] = T.m[r][c] + s2 * Minv.m[r][c];
    }
    double basisComb[D];
#pragma unroll
    for (int c = 0; c < D; ++c) basisComb[c] = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const double tr = trace<D>(mul<D>(dGdM, dmv[j]));
#pragma unroll
      for (int c = 0; c < D; ++c) basisComb[c] += Einv.m[j][c] * tr;
    }
    const double c1 = (-G + dGddet * detFJ);
    M<D> vLoc;
    {
      const M<D> P = mul<D>(mul<D>(Einv, dGdJ), FJ);
#pragma unroll
      for (int r = 0; r < D; ++r)
#pragma unroll
        for (int c = 0; c < D; ++c) vLoc.m[r][c] = c1 * Einv.m[r][c] + P.m[r][c];
    }
#pragma unroll
    for (int n = 0; n < D; n++)
#pragma unroll
      for (int c = 0; c < D; ++c) vLoc.m[n][c] -= (basisComb[c]) / ((double)D + 1.0);
#pragma unroll
    for (int c = 0; c < D; ++c) {
      double s = 0.0;
#pragma unroll
      for (int n = 0; n < D; n++) s += vLoc.m[n][c];
      grad[c] = s + (basisComb[c] + 0.0);
    }
#pragma unroll
    for (int n = 1; n < D + 1; n++)
#pragma unroll
      for (int l = 0; l < D; l++) grad[D * n + l] = -vLoc.m[n - 1][l];
#pragma unroll
    for (int i = 0; i < K; ++i) grad[i] *= absK;
    double Ih = absK * G;
    Igt = Ih;
    if constexpr (!EXACT) *tiep = *tiep || tie;
    if (ghuang) {
#pragma unroll
      for (int i = 0; i < K; ++i) ghuang[i] = grad[i];
    }
    if constexpr (REG) {
      Ih += 0.5 * fc.w * fc.w * sq;
#pragma unroll
      for (int i = 0; i < K; ++i) grad[i] += fc.w * fc.w * (-dxpu[i] + z[i]);
    }
    return Ih;
  }
}

// Mesh<D>::computeBlockGrad (src/Mesh.cpp:755-772): zero the gradient of FIXED vertices
template <int D>
__device__ __forceinline__ void zeroFixed(double* grad, unsigned fixedBits) {
#pragma unroll
  for (int i = 0; i < D + 1; i++)
    if (fixedBits & (1u << i))
#pragma unroll
      for (int m = 0; m < D; ++m) grad[D * i + m] = 0.0;
}

}  // namespace mmx
