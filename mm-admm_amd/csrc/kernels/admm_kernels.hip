// admm_kernels.hip -- CDNA4 (gfx950) kernels of one ADMM time step of the MMPDE integrator.
//
// Reference hot path: MeshIntegrator<D>::step (src/MeshIntegrator.cpp:101-191) ->
// Mesh<D>::prox (src/Mesh.cpp:930-994) -> bfgsOptSimplex (777-872) -> blockGrad
// (src/AdaptationFunctional.cpp:102-287), plus the Eigen consensus algebra (D x, D^T v,
// block-diagonal CG).  Kernels per ADMM iteration:
//   k_prox     one lane per simplex: gather DXpU = D x + u, BFGS prox (persistent Bkinv),
//              u <- DXpU - z, partial sums of energy, |z - zPrev|^2, BFGS iterations.
//   k_xupdate  one lane per node: x = (tau xBar + dt^2 sum_{s ∋ v} w (w (z - u))) / t_vv in
//              ascending simplex order (Eigen's column-major D^T product order), and
//              partial sums of |D x - z|^2.
// Partial sums go to per-workgroup slots and are reduced in a fixed order (deterministic).
// Build: -ffp-contract=off (no fused multiply-add unless written), see DESIGN.md.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "admm_device.h"
#include "admm_kernels.h"

namespace mmx {

constexpr int kBlock = 256;
constexpr int kLdsStride = kBlock + 1;  // padded SoA stride of the LDS Bkinv image
constexpr int kProxBlock = 64;          // steady-state 2D prox workgroup (round 4, with the isotropic grid and recomputed
                                        // coordinates: 64 0.322 ms, 128 0.327-0.348, 256 0.366 at C3; round 3: 128 > 256 > 64)

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// Workgroup reduction of NV values into partials[blockIdx.x * kNumPartials + i].
// Values 0..3 are summed, 4 is or-ed (as a sum of flags), 5 is a max.
template <int NV, int BS = kBlock>
__device__ __forceinline__ void block_partials(double (&v)[NV], double* partials, int slot = -1) {
  __shared__ double red[BS / 64][kNumPartials];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = (i == 5) ? wave_max(v[i]) : wave_sum(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < kNumPartials; ++i) red[wid][i] = (i < NV) ? v[i] : 0.0;
  }
  __syncthreads();
  if (threadIdx.x < kNumPartials) {
    double s = red[0][threadIdx.x];
    for (int w = 1; w < BS / 64; ++w)
      s = (threadIdx.x == 5) ? fmax(s, red[w][threadIdx.x]) : s + red[w][threadIdx.x];
    partials[(size_t)(slot < 0 ? (int)blockIdx.x : slot) * kNumPartials + threadIdx.x] = s;
  }
}

__device__ __forceinline__ int logical_block(int xcd) {
  return xcd ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
}

// any grid size: XCD x (= blockIdx % 8) takes a contiguous range of q or q + 1 logical blocks
__device__ __forceinline__ int logical_block_any() {
  const int g = (int)gridDim.x, q = g / 8, r = g % 8, x = (int)(blockIdx.x % 8);
  return x * q + min(x, r) + (int)(blockIdx.x / 8);
}

// z and u of simplex s, slot layout i = n D + c (the reference's D x order).  With MMX_ZU_INTER=1
// (2D, a build option, off: measured slower) the two are interleaved per vertex slot,
// [z_n0 z_n1 u_n0 u_n1] (32 B), so the x-update's two gathers of a slot fall in one cache line; the
// buffer then holds 2 K doubles per simplex and u = z + D.  Default: two arrays.
template <int D>
constexpr bool kZUInter = (D == 2) && MMX_ZU_INTER;
template <int D>
__device__ __forceinline__ size_t zu_base(int s) {
  return (size_t)s * (kZUInter<D> ? 2 : 1) * (D * (D + 1));
}
template <int D>
__device__ __forceinline__ int zu_i(int i) {
  return kZUInter<D> ? (i / D) * 2 * D + i % D : i;
}
// an incidence entry's slot offset s K + n D -> where its z values start
template <int D>
__device__ __forceinline__ size_t zu_off(int off) {
  return kZUInter<D> ? 2 * (size_t)off : (size_t)off;
}

// ISO: -1 the monitor path chosen at run time from m.giso; 0 the full-row path only; 1 the
// isotropic path only (m.giso set).  3D kernels are instantiated per path and launched by m.giso
// (launch_iso3), so neither path's registers count against the other's.
template <int D, int ISO = -1>
__device__ __forceinline__ GridView<D> gridOf(const DeviceMesh<D>& m) {
  GridView<D> g;
  g.gx = m.gx;
  g.gy = m.gy;
  g.gz = m.gz;
  g.vals = m.gvals;
  g.pad = m.gpad;
  g.cell[0] = m.gcell[0];
  g.cell[1] = m.gcell[1];
  g.cell[2] = m.gcell[2];
  g.iso = m.giso;
  g.nx = m.gnx;
  g.ny = m.gny;
  g.nz = m.gnz;
  g.hx = m.ghx;
  g.hy = m.ghy;
  g.hz = m.ghz;
  g.rhx = m.grhx;
  g.rhy = m.grhy;
  g.rhz = m.grhz;
  g.ax = m.gax;
  g.ay = m.gay;
  g.az = m.gaz;
  g.spx = m.gspx;
  g.spy = m.gspy;
  g.spz = m.gspz;
  g.nsx = m.gnsx;
  g.nsy = m.gnsy;
  g.nsz = m.gnsz;
  g.rnsx = m.grnsx;
  g.rnsy = m.grnsy;
  g.rnsz = m.grnsz;
  g.invFlag = m.invFlag;
  if constexpr (ISO == 0)
    g.iso = nullptr;
  else if constexpr (ISO == 1)
    __builtin_assume(g.iso != nullptr);
  return g;
}

template <int D>
__device__ __forceinline__ FunctionalConsts<D> constsOf(const DeviceMesh<D>& m) {
  FunctionalConsts<D> c;
#pragma unroll
  for (int i = 0; i < D * D; ++i) c.Ehat[i] = m.Ehat[i];
  c.powd = m.powd;
  c.w = m.w;
  c.compMesh = m.compMesh;
  return c;
}

template <int D>
__device__ __forceinline__ void loadVerts(const DeviceMesh<D>& m, int s, int (&f)[D + 1]) {
#pragma unroll
  for (int n = 0; n < D + 1; ++n) f[n] = m.F[(size_t)s * (D + 1) + n];
}

template <int D>
__device__ __forceinline__ void gatherX(const double* x, const int (&f)[D + 1], double* out) {
#pragma unroll
  for (int n = 0; n < D + 1; ++n) {
    if constexpr (D == 2) {
      const double2 v = *reinterpret_cast<const double2*>(x + (size_t)f[n] * 2);
      out[n * 2] = v.x;
      out[n * 2 + 1] = v.y;
    } else {
#pragma unroll
      for (int c = 0; c < D; ++c) out[n * D + c] = x[(size_t)f[n] * D + c];
    }
  }
}

template <int D>
__device__ __forceinline__ void loadXi(const DeviceMesh<D>& m, const int (&f)[D + 1], double* xi) {
  if (m.compMesh) gatherX<D>(m.Vc, f, xi);
}

// the x-update's term of the simplex's slots (DeviceMesh::tslot, the layout of z): the same
// expression the x-update forms from z and u (bit-identical)
template <int D>
__device__ __forceinline__ void write_tslot(const DeviceMesh<D>& m, int s, const double* z, const double* u) {
  if (!m.tslot) return;
  constexpr int K = D * (D + 1);
  double* ts = m.tslot + (size_t)s * K;
#pragma unroll
  for (int i = 0; i < K; ++i) ts[i] = m.w * (m.w * (z[i] - u[i]));
}

// z = D x (Dmat * x, src/MeshIntegrator.cpp:121,126): exact gather into simplex copies
template <int D>
__global__ void __launch_bounds__(kBlock) k_gather_z(DeviceMesh<D> m, const double* __restrict__ x,
                                                      double* __restrict__ z) {
  constexpr int K = D * (D + 1);
  const int s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= m.nF) return;
  int f[D + 1];
  loadVerts<D>(m, s, f);
  double v[K];
  gatherX<D>(x, f, v);
#pragma unroll
  for (int i = 0; i < K; ++i) z[zu_base<D>(s) + zu_i<D>(i)] = v[i];
}

// per-simplex gradient of the unregularised functional (Mesh::eulerGrad / eulerStepMod)
template <int D, int ISO = -1>
__global__ void __launch_bounds__(kBlock) k_grad_simplex(DeviceMesh<D> m, const double* __restrict__ x,
                                                          double* __restrict__ gs, int zeroFixedRows,
                                                          double* __restrict__ partials) {
  constexpr int K = D * (D + 1);
  const int s = blockIdx.x * kBlock + threadIdx.x;
  double pv[5] = {0, 0, 0, 0, 0};
  if (s < m.nF) {
    int f[D + 1];
    loadVerts<D>(m, s, f);
    double z[K], xi[K], g[K], Igt;
    gatherX<D>(x, f, z);
    loadXi<D>(m, f, xi);
    const double e = blockGrad<D, true, false>(gridOf<D, ISO>(m), constsOf<D>(m), z, xi, nullptr, g, Igt);
    if (zeroFixedRows) zeroFixed<D>(g, m.sbits[s] & 0xF);
#pragma unroll
    for (int i = 0; i < K; ++i) gs[(size_t)s * K + i] = g[i];
    pv[0] = e;
    pv[4] = (e == e) ? 0.0 : 1.0;
  }
  block_partials<5>(pv, partials);
}

// predictX (src/Mesh.cpp:649-674) fused with xPrev = x (src/MeshIntegrator.cpp:119):
// mode 0: xBar = x - (dt/tau) * sum_{s ∋ v} gs (ascending s);  mode 1: xBar = 2x - xPrev
template <int D>
__global__ void __launch_bounds__(kBlock) k_predict(DeviceMesh<D> m, int mode, const double* __restrict__ gs,
                                                     const double* __restrict__ x, double* __restrict__ xPrev,
                                                     double* __restrict__ xBar, double dt_over_tau, int xcd) {
  const int idx = logical_block(xcd) * kBlock + threadIdx.x;
  if (idx >= m.nP) return;
  // mode 0 gathers the incident gradients: in the x-update's order (neighbouring simplices); mode 1
  // streams x and xPrev in node-id order
  const int v = (mode == 0 && m.nodeOrder) ? m.nodeOrder[idx] : idx;
  double xv[D], xb[D];
#pragma unroll
  for (int c = 0; c < D; ++c) xv[c] = x[(size_t)v * D + c];
  if (mode == 0) {
    double g[D];
#pragma unroll
    for (int c = 0; c < D; ++c) g[c] = 0.0;
    const int b = m.inc_ptr[v], e = m.inc_ptr[v + 1];
    for (int t = b; t < e; ++t) {
      const int off = m.inc_off[t];
      const double* src = (off >= 0) ? gs + off : m.remote + (size_t)(-1 - off) * D;
#pragma unroll
      for (int c = 0; c < D; ++c) g[c] += src[c];
    }
#pragma unroll
    for (int c = 0; c < D; ++c) xb[c] = xv[c] - dt_over_tau * g[c];
  } else {
#pragma unroll
    for (int c = 0; c < D; ++c) xb[c] = 2 * xv[c] - xPrev[(size_t)v * D + c];
  }
#pragma unroll
  for (int c = 0; c < D; ++c) {
    xBar[(size_t)v * D + c] = xb[c];
    xPrev[(size_t)v * D + c] = xv[c];
  }
}

// x-update: vec = tau*xBar + dt^2 WD_T (w (z - u)), x = vec / t_vv (block-diagonal t),
// optional |D x - z|^2 partial sums (primal residual, src/MeshIntegrator.cpp:162).
// A node's incident slots are taken 8 at a time: their offsets, then all their z and u values
// are requested before the first is added (branch-free: lanes past the end re-read the last
// slot, a slot of another rank reads its gathered row), then summed in ascending order.
template <int D, bool RESID, bool TS, int CH = 8, bool ZX = false, bool PRED = false, bool REM = false>
__device__ __forceinline__ void xupdate_node(const DeviceMesh<D>& m, const StepScalars& sc,
                                             const double* __restrict__ xBar, const double* __restrict__ z,
                                             const double* __restrict__ u, double* __restrict__ x, int idx,
                                             double (&pv)[3]) {
  {
    // processing order: nodes by first incident simplex, so a workgroup's nodes share simplices
    const int v = m.nodeOrder ? m.nodeOrder[idx] : idx;
    double acc[D];
#pragma unroll
    for (int c = 0; c < D; ++c) acc[c] = 0.0;
    const int b = m.inc_ptr[v], e = m.inc_ptr[v + 1];
    double xb[D], zn[D];
    if constexpr (PRED) {  // predictX mode 1 for this node (k_predict): xBar = 2 x - xPrev, xPrev = x
      double xv[D];
#pragma unroll
      for (int c = 0; c < D; ++c) {
        xv[c] = x[(size_t)v * D + c];
        xb[c] = 2 * xv[c] - m.predPrev[(size_t)v * D + c];
      }
#pragma unroll
      for (int c = 0; c < D; ++c) {
        m.predBar[(size_t)v * D + c] = xb[c];
        m.predPrev[(size_t)v * D + c] = xv[c];
      }
    } else {
#pragma unroll
      for (int c = 0; c < D; ++c) xb[c] = xBar[(size_t)v * D + c];
    }
    // ZX: a step's first x-update without z (DeviceMesh::zx): every local slot of node v holds z = zx_v
    // (with PRED, zx is this step's xBar: the node's own xb); REM: an element partition, whose
    // remote slots still come from the exchange (their terms formed by launch_pack_export)
    constexpr bool zv0 = ZX && !TS;
    if constexpr (zv0) {
      if constexpr (PRED) {
#pragma unroll
        for (int c = 0; c < D; ++c) zn[c] = xb[c];
      } else {
#pragma unroll
        for (int c = 0; c < D; ++c) zn[c] = m.zx[(size_t)v * D + c];
      }
    }
    const double inv = m.invdiag[v];
    for (int t0 = b; t0 < e; t0 += CH) {
      int off[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j) off[j] = m.inc_off[min(t0 + j, e - 1)];
      double zv[CH][D], uv[CH][D];
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const bool loc = off[j] >= 0;
        if constexpr (TS) {  // the prox's terms; another rank's slot from `remote`
          const double* pt = loc ? m.tslot + off[j] : m.remote + (size_t)(-1 - off[j]) * D;
#pragma unroll
          for (int c = 0; c < D; ++c) zv[j][c] = pt[c];
        } else {
          const double* pz = loc ? z + zu_off<D>(off[j]) : m.remote + (size_t)(-1 - off[j]) * D;
          const double* pu = loc ? u + zu_off<D>(off[j]) : pz;
#pragma unroll
          for (int c = 0; c < D; ++c) {
            if constexpr (zv0 && REM)
              zv[j][c] = loc ? zn[c] : pz[c];
            else if constexpr (zv0)  // (one rank only: no slot of another rank)
              zv[j][c] = zn[c];
            else
              zv[j][c] = pz[c];
            uv[j][c] = pu[c];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        if (t0 + j < e) {
#pragma unroll
          for (int c = 0; c < D; ++c) {  // another rank's slot: the term formed there (launch_pack_export mode 0)
            if constexpr (TS)
              acc[c] += zv[j][c];
            else
              acc[c] += (off[j] >= 0) ? sc.w * (sc.w * (zv[j][c] - uv[j][c])) : zv[j][c];
          }
        }
      }
    }
    double xn[D];
#pragma unroll
    for (int c = 0; c < D; ++c) {
      xn[c] = ((sc.tau * xb[c]) + sc.dtsq * acc[c]) * inv;
      x[(size_t)v * D + c] = xn[c];
    }
    if constexpr (RESID) {  // same chunking; a slot of another rank is counted by its owner
      double r2 = 0.0;
      for (int t0 = b; t0 < e; t0 += CH) {
        int off[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) off[j] = m.inc_off[min(t0 + j, e - 1)];
        double zv[CH][D];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const double* pz = z + zu_off<D>(off[j] >= 0 ? off[j] : 0);
#pragma unroll
          for (int c = 0; c < D; ++c) zv[j][c] = pz[c];
        }
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          if (t0 + j < e && off[j] >= 0) {
#pragma unroll
            for (int c = 0; c < D; ++c) {
              const double d = xn[c] - zv[j][c];
              r2 += d * d;
            }
          }
        }
      }
      pv[2] = r2;
    }
  }
}
#ifndef MMX_XU_CH2D
#define MMX_XU_CH2D 6  // 2D: incident slots requested at once per node (C3: 8 0.066 ms, 6 0.0645, 4 0.079)
#endif
template <int D, bool RESID, bool TS, bool ZX = false, bool PRED = false, bool REM = false>
__global__ void __launch_bounds__(kBlock) k_xupdate(DeviceMesh<D> m, StepScalars sc,
                                                     const double* __restrict__ xBar,
                                                     const double* __restrict__ z,
                                                     const double* __restrict__ u, double* __restrict__ x,
                                                     double* __restrict__ partials, int xcd) {
  const int lb = logical_block(xcd);
  const int idx = m.xupLo + lb * kBlock + threadIdx.x;
  double pv[3] = {0, 0, 0};
  if (idx < m.xupHi)
    xupdate_node<D, RESID, TS, (D == 2 ? MMX_XU_CH2D : 8), ZX, PRED, REM>(m, sc, xBar, z, u, x, idx, pv);
  if constexpr (RESID) block_partials<3>(pv, partials, lb);
}
// The slot-term x-update (no residual) as a sweep: XCD c (= blockIdx % 8) takes the node-order
// positions [c n8, (c + 1) n8) and its gridDim / 8 workgroups walk them in rounds, so the slot
// terms a round gathers are mostly still in that XCD's L2 for the neighbouring rounds.
// CH: incident slots requested at once per node (3D slot terms: 24 covers a grid vertex's
// tetrahedra in one batch)
// RESID: the primal residual too (a step's last iteration, or every iteration with the early exit):
// each lane sums its nodes' terms in its round order and the workgroup's partial record is
// blockIdx.x -- a fixed grouping for a fixed grid, so runs are bit-reproducible
template <int D, bool TS, int CH, bool RESID = false>
__global__ void __launch_bounds__(kBlock) k_xupdate_sweep(DeviceMesh<D> m, StepScalars sc,
                                                           const double* __restrict__ xBar,
                                                           const double* __restrict__ z, const double* __restrict__ u,
                                                           double* __restrict__ x, int n8, double* __restrict__ partials) {
  const int c = (int)(blockIdx.x % 8), w = (int)(blockIdx.x / 8), per = (int)(gridDim.x / 8);
  const int lo = m.xupLo + c * n8, hi = min(lo + n8, m.xupHi);
  double pv[3], r2 = 0.0;
  for (int idx = lo + w * kBlock + (int)threadIdx.x; idx < hi; idx += per * kBlock) {
    xupdate_node<D, RESID, TS, CH>(m, sc, xBar, z, u, x, idx, pv);
    if constexpr (RESID) r2 += pv[2];
  }
  if constexpr (RESID) {
    double q[3] = {0.0, 0.0, r2};
    block_partials<3>(q, partials, (int)blockIdx.x);
  }
}

// k x k inverse: unblocked partial-pivot LU + substitution (mirrors the oracle's restatement
// of Eigen PartialPivLU::inverse, src/Mesh.cpp:816).  Dynamic pivoting: first prox only.
template <int K>
__device__ void invertK(double* A) {
  double lu[K * K];
  int perm[K];
  for (int i = 0; i < K; ++i) {
    perm[i] = i;
    for (int j = 0; j < K; ++j) lu[i * K + j] = A[i * K + j];
  }
  for (int k = 0; k < K; ++k) {
    int piv = k;
    double big = __builtin_fabs(lu[k * K + k]);
    for (int i = k + 1; i < K; ++i)
      if (__builtin_fabs(lu[i * K + k]) > big) {
        big = __builtin_fabs(lu[i * K + k]);
        piv = i;
      }
    if (big != 0.0) {
      if (piv != k) {
        for (int j = 0; j < K; ++j) {
          const double t = lu[k * K + j];
          lu[k * K + j] = lu[piv * K + j];
          lu[piv * K + j] = t;
        }
        const int t = perm[k];
        perm[k] = perm[piv];
        perm[piv] = t;
      }
      for (int i = k + 1; i < K; ++i) lu[i * K + k] /= lu[k * K + k];
    }
    for (int i = k + 1; i < K; ++i)
      for (int j = k + 1; j < K; ++j) lu[i * K + j] -= lu[i * K + k] * lu[k * K + j];
  }
  for (int c = 0; c < K; ++c) {
    double xc[K];
    for (int i = 0; i < K; ++i) xc[i] = (perm[i] == c) ? 1.0 : 0.0;
    for (int i = 0; i < K; ++i) {
      const double b = xc[i];
      for (int r = i + 1; r < K; ++r) xc[r] -= b * lu[r * K + i];
    }
    for (int i = K - 1; i >= 0; --i) {
      const double a = 1.0 / lu[i * K + i];
      const double b = (xc[i] *= a);
      for (int r = 0; r < i; ++r) xc[r] -= b * lu[r * K + i];
    }
    for (int i = 0; i < K; ++i) A[i * K + c] = xc[i];
  }
}


// Bkinv accessors: registers (first prox), the workgroup's LDS image (2D steady state) or the
// wave-interleaved global layout (3D steady state).  get/set address one entry; advance() is
// called after each BFGS update (the global accessor then reads what it wrote).
template <int K>
struct RegB {
  static constexpr bool kRowFence = false;
  static constexpr int kHeld = 0;
  static constexpr bool kCarry = false;
  static constexpr bool kRolled = false;
  static constexpr int kPipe = 0;
  static constexpr int kPipe1 = 0, kPipe2 = 0, kPipe3 = 0;
  static constexpr bool kPre = false;
  double* b;
  __device__ __forceinline__ double get(int i, int j) const { return b[i * K + j]; }
  __device__ __forceinline__ double heldRow(int, int) const { return 0.0; }
  __device__ __forceinline__ void holdRow(int, int, double) const {}
  __device__ __forceinline__ void set(int i, int j, double v) const { b[i * K + j] = v; }
  __device__ __forceinline__ void advance() {}
  __device__ __forceinline__ void fresh() {}
};
// LDS image: a scheduling fence per matrix row keeps one row live at a time (otherwise the
// scheduler hoists all K*K reads and the kernel spills)
template <int K, int STRIDE = kLdsStride>
struct LdsB {
  static constexpr bool kRowFence = true;
  static constexpr int kHeld = 0;
  static constexpr bool kCarry = false;
  static constexpr bool kRolled = true;  // the update pass one row per trip (code size; 2D: same speed)
  static constexpr int kPipe = 0;
  static constexpr int kPipe1 = 0, kPipe2 = 0, kPipe3 = 0;
  static constexpr bool kPre = false;
  double* base;  // &lds[tid], entries strided by STRIDE
  __device__ __forceinline__ double get(int i, int j) const { return base[(i * K + j) * STRIDE]; }
  __device__ __forceinline__ double heldRow(int, int) const { return 0.0; }
  __device__ __forceinline__ void holdRow(int, int, double) const {}
  __device__ __forceinline__ void set(int i, int j, double v) const { base[(i * K + j) * STRIDE] = v; }
  __device__ __forceinline__ void advance() {}
  // 2D: keeping the previous pass's K*K = 36 values in registers is cheaper than re-reading LDS
  __device__ __forceinline__ void fresh() {}
};
// address-space-qualified pointers: they keep global (and LDS) accesses as global_/ds_ instructions
// through the pointer laundering below (a plain pointer out of an asm operand becomes flat)
typedef __attribute__((address_space(1))) double gdouble;
#ifndef MMX_WAVE_CARRY
#define MMX_WAVE_CARRY 1  // C4: -1.5..2% (the first streamed rows of passes 2 and 3 ready when they start)
#endif
#ifndef MMX_WAVE_HELD
#define MMX_WAVE_HELD 6  // Bkinv rows kept in LDS (36 KB per wave at one wave per SIMD); C4: 4 rows -1.8%, 6 -3.1%
#endif
#ifndef MMX_ROW_PIPE
#define MMX_ROW_PIPE 2  // global Bkinv rows: request row i+2 before working on row i (C4: 1 -> 2 rows -1.6%, 3 spills)
#endif
typedef __attribute__((address_space(3))) double ldouble;

// Global, wave-interleaved (entry ij of simplex s at ((s/64)*K*K + ij)*64 + s%64: a wavefront's
// access to one entry is 512 contiguous bytes).  Double-buffered across proxes: the first BFGS
// iteration reads the previous prox's buffer `rd` and writes `wr`, later iterations work in `wr`,
// so `rd` stays intact for an exact recomputation of the block.
#ifndef MMX_WAVE_DMA
#define MMX_WAVE_DMA 1
#endif
#ifndef MMX_ROW_PIPE_FULL
#define MMX_ROW_PIPE_FULL 3  // the same for the 3D prox with a general (full-row) monitor grid
#endif
#ifndef MMX_ROW_PIPE1
#define MMX_ROW_PIPE1 6  // pass 1: global rows requested ahead (with kPre all of rows 6-11 while 0-5 come from LDS); C4 2 -> 6: -1.1%
#endif
#ifndef MMX_ROW_PIPE2
#define MMX_ROW_PIPE2 6  // pass 2: rows 8-11 requested when it starts (6, 7 carried), read after rows 0-5 (LDS)
#endif
#ifndef MMX_ROW_PIPE3
#define MMX_ROW_PIPE3 2  // pass 3
#endif
// 2D (K = 6, k_prox_wave<2>): every row held in LDS, so no streamed-row queues
template <int K, int PIPE = MMX_ROW_PIPE>
struct WaveB {
  static constexpr bool k2 = (K == 6);
  static constexpr bool kRowFence = true;
  static constexpr bool kRolled = true;
  static constexpr int kPipe = k2 ? 0 : PIPE;
  static constexpr int kPipe1 = k2 ? 0 : MMX_ROW_PIPE1, kPipe2 = k2 ? 0 : MMX_ROW_PIPE2, kPipe3 = k2 ? 0 : MMX_ROW_PIPE3;
  static constexpr int kHeld = k2 ? K : MMX_WAVE_HELD;  // rows kept in LDS from pass 1 to passes 2 and 3
  static constexpr bool kCarry = !k2 && MMX_WAVE_CARRY;
  // the held rows of the entry matrix DMA'd into LDS at the start of the block (prox_wave_block),
  // so the first pass 1 reads them from there
  static constexpr bool kPre = MMX_WAVE_DMA && kHeld > 0;
  // 3D with MMX_B3_PAIRS (bidx): the lane's base is 2 lane and entry e at (e & ~1) 64 + (e & 1), so
  // a row's twelve entries are six 16-byte accesses; otherwise base lane, entry e at e 64
  static constexpr bool kPairs = !k2 && MMX_B3_PAIRS;
  static constexpr int kLaneMul = kPairs ? 2 : 1;
  static __device__ __forceinline__ int eo(int e) { return kPairs ? (e & ~1) * 64 + (e & 1) : e * 64; }
  const gdouble* rd;
  gdouble* wr;
  ldouble* held;  // &lds[kLaneMul lane], kHeld rows in the same layout
  __device__ __forceinline__ double get(int i, int j) const { return rd[eo(i * K + j)]; }
  __device__ __forceinline__ double heldRow(int i, int j) const { return held[eo(i * K + j)]; }
  __device__ __forceinline__ void holdRow(int i, int j, double v) const { held[eo(i * K + j)] = v; }
  // the new Bkinv is read by the next prox only: nontemporal stores keep it out of the way of the
  // rows still to be re-read (C4 prox 2.97 -> 2.77 ms; nontemporal loads: no gain)
  __device__ __forceinline__ void set(int i, int j, double v) const { __builtin_nontemporal_store(v, &wr[eo(i * K + j)]); }
  __device__ __forceinline__ void advance() { rd = wr; }
  // a pass over the matrix re-reads it: an opaque pointer stops the compiler from forwarding the
  // previous pass's K*K = 144 loads in registers (3D spilled)
  // the memory clobber keeps the LDS rows in LDS (no store-to-load forwarding into registers)
  __device__ __forceinline__ void fresh() { asm volatile("" : "+v"(rd), "+v"(wr)::"memory"); }
};

// index of Bkinv entry ij of simplex s, wave-interleaved in 2D and 3D: the 2D LDS kernel's chunk
// is then its LDS image (a straight copy), and WaveB's accesses are 512 contiguous bytes
template <int D>
__device__ __forceinline__ size_t bidx(int s, int ij) {
  constexpr int KK = D * (D + 1) * D * (D + 1);
  if constexpr (D == 3 && MMX_B3_PAIRS)  // (layout.h) a lane's entries ij, ij + 1 (ij even) adjacent
    return ((size_t)(s >> 6) * KK + (ij & ~1)) * 64 + 2 * (s & 63) + (ij & 1);
  return ((size_t)(s >> 6) * KK + ij) * 64 + (s & 63);
}

#define MMX_ROW_FENCE(BA) \
  if constexpr (BA::kRowFence) __builtin_amdgcn_sched_barrier(0)

// Timing probe (build option -DMMX_WAVE_PROF, never in the product build): per-block shader-clock
// stamps of the phases of the 3D steady prox's first BFGS iteration, written by lane 0 with a
// vector store; the host side is mmx_wprof_dump (below).  `dep` is a value the phase produces, so
// the stamp is taken once it is available.
#ifdef MMX_WAVE_PROF
__device__ unsigned long long* g_wprof;
#define WPROF(slot, dep)                                                                     \
  do {                                                                                       \
    asm volatile("" ::"v"(dep));                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    const unsigned long long t_ = __builtin_readcyclecounter();                              \
    if (threadIdx.x == 0 && g_wprof) g_wprof[(size_t)blockIdx.x * 8 + (slot)] = t_;          \
    __builtin_amdgcn_sched_barrier(0);                                                       \
  } while (0)
#else
#define WPROF(slot, dep) \
  do {                   \
  } while (0)
#endif

template <int K, class BA>
__device__ __forceinline__ void load_row(const BA& B, int i, double (&r)[K]) {
#pragma unroll
  for (int j = 0; j < K; ++j) r[j] = B.get(i, j);
}
// row i of a pass: rows below BA::kHeld (when `held`) from the accessor's LDS copy; the others
// with PIPE > 0 from rn[0] (requested PIPE rows earlier), after which the queue shifts and row
// i+PIPE is requested.  i may be a run-time value (the rolled update pass).
template <int K, int PIPE, class BA>
__device__ __forceinline__ void next_row(const BA& B, int i, double (&row)[K], double (&rn)[PIPE > 0 ? PIPE : 1][K],
                                         bool held = false) {
  if (held && i < BA::kHeld) {
#pragma unroll
    for (int j = 0; j < K; ++j) row[j] = B.heldRow(i, j);
  } else if constexpr (PIPE > 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) row[j] = rn[0][j];
#pragma unroll
    for (int d = 0; d + 1 < PIPE; ++d)
#pragma unroll
      for (int j = 0; j < K; ++j) rn[d][j] = rn[d + 1][j];
    if (i + PIPE < K) load_row<K>(B, i + PIPE, rn[PIPE - 1]);
  } else {
    load_row<K>(B, i, row);
  }
}
// the first PIPE streamed rows of a pass (from row `first`)
template <int K, int PIPE, class BA>
__device__ __forceinline__ void start_rows(const BA& B, double (&rn)[PIPE > 0 ? PIPE : 1][K], int first = 0) {
#pragma unroll
  for (int d = 0; d < PIPE; ++d)
    if (first + d < K) load_row<K>(B, first + d, rn[d]);
}

// Row i of the BFGS update (src/Mesh.cpp:848):
// B_ij += c1 p_i p_j - (B (y p^T))_ij / c2 - p_i (y^T B)_j / c2.  EXACT = false divides by
// Markstein's correction (div_mk) and folds the range data into eBy / fin for the caller's check.
template <int D, bool EXACT, class BA, int K>
__device__ __forceinline__ void bfgs_update_row(BA& B, int i, double pki, const double (&row)[K], const double (&yk)[K],
                                                const double (&pk)[K], const double (&yB)[K], double c1, double c2,
                                                double rc2, unsigned& eBy, double& fin) {
  double nrow[K], ykr[K];
  // 3D: (y p^T)_qj is formed again for every row -- laundering y per row stops the compiler
  // from keeping all K*K = 144 products live across the rows (they spilled); 2D keeps its 36
#pragma unroll
  for (int q = 0; q < K; ++q) {
    ykr[q] = yk[q];
    if constexpr (D == 3) asm volatile("" : "+v"(ykr[q]));
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double by = row[0] * (ykr[0] * pk[j]);
#pragma unroll
    for (int q = 1; q < K; ++q) by += row[q] * (ykr[q] * pk[j]);
    if constexpr (EXACT) {
      nrow[j] = row[j] + (((c1 * (pki * pk[j])) - by / c2) - (pki * yB[j]) / c2);
    } else {
      eBy = max(eBy, mk_exp(by, 900));
      nrow[j] = row[j] + (((c1 * (pki * pk[j])) - div_mk(by, c2, rc2)) - div_mk(pki * yB[j], c2, rc2));
      fin = cr_fma(nrow[j], 0.0, fin);
    }
  }
#pragma unroll
  for (int j = 0; j < K; ++j) B.set(i, j, nrow[j]);
}

// UR consecutive rows i..i+UR-1 of the update in one trip (3D): the products y_q p_j are formed
// once for the UR rows instead of once per row; every entry's operations are bfgs_update_row's.
#ifndef MMX_UPD_ROWS
#define MMX_UPD_ROWS 2  // 3D: rows of the update pass per trip (round 3: 1 -> 3 rows 2.755 -> 2.719 ms; round 6, paired layout: 3 -> 2 rows 2.272 -> 2.255 ms, 4 rows 2.29)
#endif
template <int D, bool EXACT, int UR, class BA, int K>
__device__ __forceinline__ void bfgs_update_rows(BA& B, int i, const double (&pki)[UR], const double (&row)[UR][K],
                                                 const double (&yk)[K], const double (&pk)[K], const double (&yB)[K],
                                                 double c1, double c2, double rc2, unsigned& eBy, double& fin) {
  double nrow[UR][K], ykr[K];
#pragma unroll
  for (int q = 0; q < K; ++q) {
    ykr[q] = yk[q];
    asm volatile("" : "+v"(ykr[q]));
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double yp[K];
#pragma unroll
    for (int q = 0; q < K; ++q) yp[q] = ykr[q] * pk[j];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      double by = row[u][0] * yp[0];
#pragma unroll
      for (int q = 1; q < K; ++q) by += row[u][q] * yp[q];
      if constexpr (EXACT) {
        nrow[u][j] = row[u][j] + (((c1 * (pki[u] * pk[j])) - by / c2) - (pki[u] * yB[j]) / c2);
      } else {
        eBy = max(eBy, mk_exp(by, 900));
        nrow[u][j] = row[u][j] + (((c1 * (pki[u] * pk[j])) - div_mk(by, c2, rc2)) - div_mk(pki[u] * yB[j], c2, rc2));
        fin = cr_fma(nrow[u][j], 0.0, fin);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < UR; ++u)
#pragma unroll
    for (int j = 0; j < K; ++j) B.set(i + u, j, nrow[u][j]);
}

// Mesh<D>::bfgsOptSimplex iteration loop (src/Mesh.cpp:827-856): inverse-BFGS without line
// search, <= 50 iterations, stop when ||grad||_1 < tol.  Returns the iteration count.
// EXACT = false: the fast path; a power near a rounding midpoint raises *tie (the caller then
// recomputes the simplex exactly) and the loop stops.
template <int D, class BA, bool EXACT = true>
__device__ __forceinline__ int bfgs_iterations(BA B, const GridView<D>& g, const FunctionalConsts<D>& fc,
                                               double* z, const double* xi, const double* dx, double* G,
                                               unsigned fixedBits, double tol, bool& bad, double* gcache,
                                               bool* tie = nullptr) {
  constexpr int K = D * (D + 1);
  constexpr int kPipe = BA::kPipe;
  int iter;
  for (iter = 0; iter < 50; iter++) {
    B.fresh();
    double pk[K];
    double rn[kPipe > 0 ? kPipe : 1][K];  // kPipe rows requested ahead of the row being worked on
    // kCarry: the first kPipe streamed rows of a pass are kept in registers from the previous pass
    // (the next pass starts without waiting for their loads)
    constexpr bool kCarry = BA::kCarry && kPipe > 0;
    double rc[kPipe > 0 ? kPipe : 1][K];
    // kPre: the first iteration's held rows are in LDS already (DMA'd at the start of the block)
    const bool pre = BA::kPre && iter == 0;
    constexpr int kP1 = BA::kPipe1;
    double rn1[kP1 > 0 ? kP1 : 1][K];  // pass 1's queue of requested rows
    start_rows<K, kP1>(B, rn1, pre ? BA::kHeld : 0);
#pragma unroll
    for (int i = 0; i < K; ++i) {
      MMX_ROW_FENCE(BA);
      double row[K];
      next_row<K, kP1>(B, i, row, rn1, pre);
      if constexpr (BA::kHeld > 0) {  // the first kHeld rows wait in LDS for passes 2 and 3
        if (!pre && i < BA::kHeld)
#pragma unroll
          for (int j = 0; j < K; ++j) B.holdRow(i, j, row[j]);
      }
      if constexpr (kCarry) {
        if (i >= BA::kHeld && i < BA::kHeld + kPipe)
#pragma unroll
          for (int j = 0; j < K; ++j) rc[i - BA::kHeld][j] = row[j];
      }
      double sacc = (-row[0]) * G[0];
#pragma unroll
      for (int j = 1; j < K; ++j) sacc += (-row[j]) * G[j];
      pk[i] = sacc;
    }
    MMX_ROW_FENCE(BA);
    if constexpr (BA::kPipe > 0 && !EXACT) {
      if (iter == 0) WPROF(2, pk[K - 1]);
    }
#pragma unroll
    for (int i = 0; i < K; ++i) z[i] += pk[i];
    double G1[K], Igt;
    {
      const double e = blockGrad<D, true, true, EXACT>(g, fc, z, xi, dx, G1, Igt, gcache, tie);
      bad |= (e != e);
    }
    if constexpr (BA::kPipe > 0 && !EXACT) {
      if (iter == 0) WPROF(3, G1[K - 1]);
    }
    if constexpr (!EXACT) {
      if (*tie) break;
    }
    zeroFixed<D>(G1, fixedBits);
    double Ix = 0;
#pragma unroll
    for (int i = 0; i < K; i++) Ix += __builtin_fabs(G1[i]);
    double yk[K];
#pragma unroll
    for (int i = 0; i < K; ++i) yk[i] = G1[i] - G[i];
    double c2 = pk[0] * yk[0];
#pragma unroll
    for (int i = 1; i < K; ++i) c2 += pk[i] * yk[i];
    B.fresh();
    // one pass over B: By_i = sum_j B_ij y_j, yBy = sum_i y_i By_i, yB_j = sum_i y_i B_ij
    double yBy = 0.0, yB[K];
    constexpr int kP2 = BA::kPipe2 > kPipe ? BA::kPipe2 : kPipe;
    double rn2[kP2 > 0 ? kP2 : 1][K];
    if constexpr (kCarry) {
#pragma unroll
      for (int d = 0; d < kPipe; ++d)
#pragma unroll
        for (int j = 0; j < K; ++j) rn2[d][j] = rc[d][j];
#pragma unroll
      for (int d = kPipe; d < kP2; ++d)
        if (BA::kHeld + d < K) load_row<K>(B, BA::kHeld + d, rn2[d]);
    } else {
      start_rows<K, kP2>(B, rn2, BA::kHeld);
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
      MMX_ROW_FENCE(BA);
      double row[K];
      next_row<K, kP2>(B, i, row, rn2, true);
      if constexpr (kCarry) {
        if (i >= BA::kHeld && i < BA::kHeld + kPipe)
#pragma unroll
          for (int j = 0; j < K; ++j) rc[i - BA::kHeld][j] = row[j];
      }
      double by = row[0] * yk[0];
#pragma unroll
      for (int j = 1; j < K; ++j) by += row[j] * yk[j];
      yBy = (i == 0) ? yk[0] * by : yBy + yk[i] * by;
#pragma unroll
      for (int j = 0; j < K; ++j) yB[j] = (i == 0) ? yk[0] * row[j] : yB[j] + yk[i] * row[j];
    }
    MMX_ROW_FENCE(BA);
    const double c1 = (c2 + yBy) / cr_pow_2(c2);
    if constexpr (BA::kPipe > 0 && !EXACT) {
      if (iter == 0) WPROF(4, c1);
    }
    // fast path (EXACT = false): the 2 K^2 divisions by c2 below by Markstein's correction from
    // one reciprocal (div_mk, bit-identical inside the ranges checked after the pass; outside
    // them the block is recomputed exactly, as for a near-midpoint power)
    const double rc2 = 1.0 / c2;
    unsigned eBy = 0u;  // max of mk_exp(by, 900) over the pass
    double fin = 0.0;   // stays +0 while every new entry is finite
    B.fresh();
    // B_ij += c1 p_i p_j - (B (y p^T))_ij / c2 - p_i (y^T B)_j / c2, row by row
    if constexpr (BA::kRolled) {
      // one row per trip (3D: the unrolled pass is ~60 KB of code, more than the instruction
      // cache; measured C4 prox 3.12 -> 2.93 ms), rows requested kPipe ahead
      constexpr int kP3 = BA::kPipe3 > kPipe ? BA::kPipe3 : kPipe;
      double rn3[kP3 > 0 ? kP3 : 1][K];
      if constexpr (kCarry) {
#pragma unroll
        for (int d = 0; d < kPipe; ++d)
#pragma unroll
          for (int j = 0; j < K; ++j) rn3[d][j] = rc[d][j];
#pragma unroll
        for (int d = kPipe; d < kP3; ++d)
          if (BA::kHeld + d < K) load_row<K>(B, BA::kHeld + d, rn3[d]);
      } else {
        start_rows<K, kP3>(B, rn3, BA::kHeld);
      }
      constexpr int UR = (D == 3 && K % MMX_UPD_ROWS == 0) ? MMX_UPD_ROWS : 1;
      if constexpr (UR == 1) {
#pragma unroll 1
        for (int i = 0; i < K; ++i) {
          double pki = pk[0];
#pragma unroll
          for (int k = 1; k < K; ++k) pki = (i == k) ? pk[k] : pki;
          double row[K];
          next_row<K, kP3>(B, i, row, rn3, true);
          bfgs_update_row<D, EXACT>(B, i, pki, row, yk, pk, yB, c1, c2, rc2, eBy, fin);
        }
      } else {
#pragma unroll 1
        for (int i = 0; i < K; i += UR) {
          double pki[UR], rows[UR][K];
#pragma unroll
          for (int u = 0; u < UR; ++u) {
            pki[u] = pk[0];
#pragma unroll
            for (int k = 1; k < K; ++k) pki[u] = (i + u == k) ? pk[k] : pki[u];
            next_row<K, kP3>(B, i + u, rows[u], rn3, true);
          }
          bfgs_update_rows<D, EXACT, UR>(B, i, pki, rows, yk, pk, yB, c1, c2, rc2, eBy, fin);
        }
      }
    } else {
      start_rows<K, kPipe>(B, rn);
#pragma unroll
      for (int i = 0; i < K; ++i) {
        MMX_ROW_FENCE(BA);
        double row[K];
        next_row<K, kPipe>(B, i, row, rn);
        bfgs_update_row<D, EXACT>(B, i, pk[i], row, yk, pk, yB, c1, c2, rc2, eBy, fin);
      }
    }
    MMX_ROW_FENCE(BA);
    if constexpr (BA::kPipe > 0 && !EXACT) {
      if (iter == 0) WPROF(5, fin);
    }
    B.advance();
    if constexpr (!EXACT) {
      // div_mk's ranges: c2 in [2^-100, 2^100]; by = 0 or in [2^-900, 2^900]; p_i yB_j likewise,
      // which p and yB = 0 or in [2^-450, 2^450] guarantee; every new entry finite
      unsigned ePY = 0u;
#pragma unroll
      for (int k = 0; k < K; ++k) ePY = max(ePY, max(mk_exp(pk[k], 450), mk_exp(yB[k], 450)));
      if (!(c2 >= 0x1p-100 && c2 <= 0x1p100) || eBy > 1799u || ePY > 899u || fin != 0.0) *tie = true;
      if (*tie) break;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) G[i] = G1[i];
    if (Ix < tol) break;
  }
  return (iter == 50) ? 50 : iter + 1;
}

// Entry gradient of the prox: the full regularised blockGrad, or -- when z is unchanged since the
// previous prox -- its cached unregularised part plus the regulariser, added exactly as blockGrad
// adds it (bit-identical).
template <int D, bool EXACT = true>
__device__ __forceinline__ void entry_grad(const GridView<D>& g, const FunctionalConsts<D>& fc, const double* z,
                                           const double* xi, const double* dx, const double* cache, bool useCache,
                                           double* G, double& Igt, bool& bad, bool* tie = nullptr) {
  constexpr int K = D * (D + 1);
  if (useCache) {
#pragma unroll
    for (int i = 0; i < K; ++i) G[i] = cache[i];
    Igt = 0.0;  // unused: a step reports the energy of its first prox, which never takes the cache
#pragma unroll
    for (int i = 0; i < K; ++i) G[i] += fc.w * fc.w * (-dx[i] + z[i]);
    bad |= (cache[0] != cache[0]);  // an inverted element's cached gradient is all NaN
  } else {
    const double e = blockGrad<D, true, true, EXACT>(g, fc, z, xi, dx, G, Igt, nullptr, tie);
    bad |= (e != e);
  }
}

// The prox (src/Mesh.cpp:930-994 / 777-872), one lane per simplex.  FIRST = the first prox of
// the run, which builds the finite-difference Hessian and inverts it.
template <int D, bool FIRST, int ISO = -1>
__device__ __forceinline__ void prox_simplex(const DeviceMesh<D>& m, double tol, const double* __restrict__ x,
                                             double* __restrict__ zg, double* __restrict__ ug,
                                             const double* Bin, double* Bout, bool useCache, int s,
                                             double (&pv)[6]) {
  constexpr int K = D * (D + 1);
  const GridView<D> g = gridOf<D, ISO>(m);
  const FunctionalConsts<D> fc = constsOf<D>(m);
  int f[D + 1];
  loadVerts<D>(m, s, f);
  const unsigned bits = m.sbits[s];
  const unsigned fixedBits = bits & 0xF;
  double xi[K];
  loadXi<D>(m, f, xi);
  double dx[K], z[K], zold[K];
  gatherX<D>(x, f, dx);
  double* zs = zg + zu_base<D>(s);
  double* us = ug + zu_base<D>(s);
  if (m.zx)
    gatherX<D>(m.zx, f, z);  // the step's first prox: z = D zx (DeviceMesh::zx)
  else
#pragma unroll
    for (int i = 0; i < K; ++i) z[i] = zs[zu_i<D>(i)];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    dx[i] = dx[i] + us[zu_i<D>(i)];  // DXpU = D x + uBar
    zold[i] = z[i];
  }
  double B[K * K];
  if constexpr (!FIRST) {
#pragma unroll
    for (int i = 0; i < K * K; ++i) B[i] = Bin[bidx<D>(s, i)];
  }
  double G[K], G1[K], Igt;
  bool bad = false;
  (void)G1;
  double* gc = m.gcache + (size_t)s * K;
  entry_grad<D>(g, fc, z, xi, dx, gc, !FIRST && useCache, G, Igt, bad);
  zeroFixed<D>(G, fixedBits);
  const double Ihsave = Igt;
  if constexpr (FIRST) {
    const double h = 2.0 * cr_sqrt(2.220446049250313080847e-16);
    double zp[K];
#pragma unroll
    for (int i = 0; i < K; ++i) zp[i] = z[i];
    for (int i = 0; i < K; i++) {
      zp[i] += h;
      double Ig2;
      blockGrad<D, true, true>(g, fc, zp, xi, dx, G1, Ig2);
      zeroFixed<D>(G1, fixedBits);
#pragma unroll
      for (int r = 0; r < K; ++r) B[r * K + i] = (G1[r] - G[r]) / h;
      zp[i] = z[i];
    }
#pragma unroll
    for (int n = 0; n < D + 1; n++)
      if (bits & (1u << (4 + n)))
#pragma unroll
        for (int c = 0; c < D; c++) B[(D * n + c) * K + D * n + c] = 1.0;
    invertK<K>(B);
  }
  RegB<K> Bacc{B};
  const int its = bfgs_iterations<D>(Bacc, g, fc, z, xi, dx, G, fixedBits, tol, bad, gc);
  double dual2 = 0.0;
  double un[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    zs[zu_i<D>(i)] = z[i];
    un[i] = dx[i] - z[i];  // uBar = DXpU - z
    us[zu_i<D>(i)] = un[i];
    const double d = z[i] - zold[i];
    dual2 += d * d;
  }
  write_tslot<D>(m, s, z, un);
#pragma unroll
  for (int i = 0; i < K * K; ++i) Bout[bidx<D>(s, i)] = B[i];
  pv[0] = Ihsave;
  pv[1] = dual2;
  pv[3] = (double)its;
  pv[4] = bad ? 1.0 : 0.0;
  pv[5] = (double)its;
}

template <int D, bool FIRST, int ISO = -1>
__global__ void __launch_bounds__(kBlock) k_prox(DeviceMesh<D> m, double tol, const double* __restrict__ x,
                                                  double* __restrict__ zg, double* __restrict__ ug,
                                                  const double* Bin, double* Bout, double* __restrict__ partials,
                                                  int useCache) {
  const int s = blockIdx.x * kBlock + threadIdx.x;
  double pv[6] = {0, 0, 0, 0, 0, 0};
  if (s < m.nF) prox_simplex<D, FIRST, ISO>(m, tol, x, zg, ug, Bin, Bout, useCache != 0, s, pv);
  block_partials<6>(pv, partials);
}

// Exact recomputation of the steady-state prox for the blocks whose fast pass (k_prox_lds) met a
// power within 2^-95 of a rounding midpoint (or outside the double-double ranges): such a block
// wrote nothing back (z, u, Bkinv unchanged), so each of its simplices restarts from its inputs
// with cr_resolve, Bkinv in registers and a full entry blockGrad (bit-identical to the cached
// form, which the fast pass may have overwritten), and the block's partials are formed with the
// same workgroup shape -- the same values in the same tree.  The workgroups of a fixed grid (one
// per CU at most) stride over the list, so a prox with many ties is not serialised on one CU (with
// no ties each workgroup only reads the counter).  The queue counters are double-buffered over the
// steady proxes: this prox's recomputation clears the previous prox's counter (whose recomputation
// has finished, stream order), which the next prox appends to -- a plain store, no completion
// atomics.
__device__ __forceinline__ void rearm_tie_queue(unsigned* tieStale) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *tieStale = 0u;
}
template <int D, int BS>
__global__ void __launch_bounds__(BS) k_prox_fix(DeviceMesh<D> m, double tol, const double* __restrict__ x,
                                                 double* __restrict__ zg, double* __restrict__ ug,
                                                 const double* Bin, double* Bout, double* __restrict__ partials) {
  const unsigned n = *m.tieCount;
  for (unsigned i = blockIdx.x; i < n; i += gridDim.x) {
    const int b = m.tieList[i];
    const int s = b * BS + (int)threadIdx.x;
    double pv[6] = {0, 0, 0, 0, 0, 0};
    if (s < m.nF) prox_simplex<D, false>(m, tol, x, zg, ug, Bin, Bout, false, s, pv);
    block_partials<6, BS>(pv, partials, b);
    __syncthreads();
  }
  rearm_tie_queue(m.tieStale);
}

// Steady-state prox (every prox after the first), Bkinv staged through LDS.  The workgroup's
// BS simplices own one contiguous Bkinv chunk of BS/64 wave blocks (bidx: [block][K*K][64]), which
// is also the LDS image: entry ij of a lane's matrix sits 64 doubles after entry ij-1, so each
// lane's BFGS reads its own matrix conflict-free, and the chunk moves in and out as a straight
// 16-byte-per-lane copy (in: DMA'd to LDS, no registers; out: nontemporal stores).  The
// registers this frees give two waves per SIMD.  Each lane's own inputs (vertices, z, u, the
// cached gradient) are requested around the chunk, so their latency hides under it.
// Fast path: the powers are not tie-resolved here (EXACT = false).  If any lane of the block
// meets a near-midpoint power the whole block writes nothing back and is queued for k_prox_fix,
// which recomputes it exactly from the untouched inputs.
typedef double v2nt __attribute__((ext_vector_type(2)));
#ifndef MMX_ZU_NT
#define MMX_ZU_NT 0  // 2D prox: z and u written with nontemporal stores (experiment)
#endif
#ifndef MMX_LDS_DMA
#define MMX_LDS_DMA 0  // 1: the chunk DMA'd to LDS after the gathers (C3 prox 0.380 ms); 0: through registers, requested before them (0.370 ms)
#endif
template <int D, int BS>
__global__ void __launch_bounds__(BS, 2) k_prox_lds(DeviceMesh<D> m, double tol, const double* __restrict__ x,
                                                        double* __restrict__ zg, double* __restrict__ ug,
                                                        double* __restrict__ Bg, double* __restrict__ partials,
                                                        int useCache) {
  constexpr int K = D * (D + 1), KK = K * K;
  static_assert(BS % 64 == 0, "whole wave blocks per chunk");
  __shared__ __attribute__((aligned(16))) double lds[KK * BS];
  const int tid = threadIdx.x;
  const int lb = (int)blockIdx.x;  // (an XCD-contiguous mapping measured no gain: a 2D workgroup's simplices already share lines)
  const int s0 = lb * BS;
  const int nIn = min(BS, m.nF - s0);
  const bool act = tid < nIn;
  const int s = act ? s0 + tid : s0;  // inactive lanes shadow the first simplex, store nothing
  // the lane's inputs, requested first
  int f[D + 1];
  loadVerts<D>(m, s, f);
  const unsigned fixedBits = m.sbits[s] & 0xF;
  double* zs = zg + zu_base<D>(s);
  double* us = ug + zu_base<D>(s);
  double* gc = m.gcache + (size_t)s * K;
  double z[K], z0[K], dx[K], gcv[K];
  if (m.zx)
    gatherX<D>(m.zx, f, z);  // the step's first prox: z = D zx (DeviceMesh::zx)
  else
#pragma unroll
    for (int i = 0; i < K; ++i) z[i] = zs[zu_i<D>(i)];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    z0[i] = z[i];  // the entry z, for ||z - zPrev||^2 (no reload at the end)
    dx[i] = us[zu_i<D>(i)];
  }
  if (useCache) {
#pragma unroll
    for (int i = 0; i < K; ++i) gcv[i] = gc[i];
  }
  // the chunk: BS/64 whole wave blocks (the buffer is padded to whole chunks of 256 simplices, so a
  // short last chunk copies -- and writes back unchanged -- its padding)
  double* chunk = Bg + (size_t)s0 * KK;
  constexpr int NL = KK / 2;  // 16-byte pieces per lane; piece r of lane tid at 16 (tid + r BS)
  v2nt cv[MMX_LDS_DMA ? 1 : NL];
  if constexpr (!MMX_LDS_DMA) {
    // the chunk is read once and written once: nontemporal (C3 prox 0.412 -> 0.399 ms)
#pragma unroll
    for (int r = 0; r < NL; ++r) cv[r] = __builtin_nontemporal_load(reinterpret_cast<const v2nt*>(chunk) + tid + r * BS);
  }
  double xi[K], dxv[K];
  loadXi<D>(m, f, xi);
  gatherX<D>(x, f, dxv);
  if constexpr (MMX_LDS_DMA) {
    // requested after the gathers (a wait for loads issued before an LDS DMA waits for the DMA
    // too): wave w's lanes fill bytes [16 (r BS + 64 w), +1 KB) of the image, a wave-uniform base
    __builtin_amdgcn_sched_barrier(0);
    const char* src = reinterpret_cast<const char*>(chunk) + tid * 16;
    const int wofs = __builtin_amdgcn_readfirstlane((tid >> 6) * 1024);
#pragma unroll
    for (int r = 0; r < NL; ++r)
      __builtin_amdgcn_global_load_lds(src + r * BS * 16,
                                       (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(lds) + wofs + r * BS * 16),
                                       16, 0, 0);
    __builtin_amdgcn_sched_barrier(0);  // (the DMA issued as one batch: nothing that waits moves into it)
    __builtin_amdgcn_s_waitcnt(0);      // this wave's DMA has landed (the barrier then covers the workgroup's)
  } else {
#pragma unroll
    for (int r = 0; r < NL; ++r) reinterpret_cast<v2nt*>(lds)[tid + r * BS] = cv[r];
  }
#pragma unroll
  for (int i = 0; i < K; ++i) dx[i] = dxv[i] + dx[i];  // DXpU = D x + uBar
  __syncthreads();
  double pv[6] = {0, 0, 0, 0, 0, 0};
  bool tie = false;
  if (act) {
    const GridView<D> g = gridOf<D>(m);
    const FunctionalConsts<D> fc = constsOf<D>(m);
    double G[K], Igt;
    bool bad = false;
    entry_grad<D, false>(g, fc, z, xi, dx, gcv, useCache != 0, G, Igt, bad, &tie);
    zeroFixed<D>(G, fixedBits);
    const double Ihsave = Igt;
    LdsB<K, 64> Bacc{lds + (tid >> 6) * KK * 64 + (tid & 63)};
    const int its =
        tie ? 0 : bfgs_iterations<D, LdsB<K, 64>, false>(Bacc, g, fc, z, xi, dx, G, fixedBits, tol, bad, gc, &tie);
    double dual2 = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const double d = z[i] - z0[i];
      dual2 += d * d;
    }
    pv[0] = Ihsave;
    pv[1] = dual2;
    pv[3] = (double)its;
    pv[4] = bad ? 1.0 : 0.0;
    pv[5] = (double)its;
  }
  if (m.forceTie > 0 && tid == 0 && (int)((unsigned)lb % (unsigned)m.forceTie) == 0) tie = true;
  if (__syncthreads_or(tie ? 1 : 0)) {  // rare: leave the block to k_prox_fix
    if (tid == 0) m.tieList[atomicAdd(m.tieCount, 1u)] = lb;
    return;
  }
  if (act) {
    double un[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      un[i] = dx[i] - z[i];  // uBar = DXpU - z
      if constexpr (MMX_ZU_NT) {
        __builtin_nontemporal_store(z[i], &zs[zu_i<D>(i)]);
        __builtin_nontemporal_store(un[i], &us[zu_i<D>(i)]);
      } else {
        zs[zu_i<D>(i)] = z[i];
        us[zu_i<D>(i)] = un[i];
      }
    }
    write_tslot<D>(m, s, z, un);
  }
#pragma unroll
  for (int r = 0; r < NL; ++r)
    __builtin_nontemporal_store(reinterpret_cast<const v2nt*>(lds)[tid + r * BS], reinterpret_cast<v2nt*>(chunk) + tid + r * BS);
  block_partials<6, BS>(pv, partials, lb);
}

// Steady-state 3D prox: one wavefront per workgroup, one lane per tetrahedron, Bkinv (144
// doubles per tet, 1152 B: too large to stage in LDS) read straight from global memory in the
// wave-interleaved layout -- every access of a wavefront to one entry is 512 contiguous bytes --
// and double-buffered (WaveB): the previous prox's buffer is only read, so a block whose fast
// pass meets a near-midpoint power (EXACT = false) is abandoned unwritten and recomputed exactly
// by k_prox_wave_fix from the untouched inputs, as in the 2D kernel.
#ifndef MMX_WAVE_OCC
#define MMX_WAVE_OCC 1  // measured: one wave per SIMD (310 VGPRs); two (12-53 spills, p/G/DXpU parked in LDS) gain < 2%
#endif
#ifndef MMX_WAVE_OCC2
#define MMX_WAVE_OCC2 2  // k_prox_wave<2> (MMX_PROX2D=wave): waves per SIMD
#endif
#ifndef MMX_WAVE_PERSIST
#define MMX_WAVE_PERSIST 0  // 3D: a persistent grid of this many one-wave workgroups (a multiple of 8), 0: one per block
#endif
#ifndef MMX_HELD_DMA_CPOL
// cache policy of the held rows' DMA: 2 = nontemporal (they are read from global once and kept in
// LDS, so streaming them leaves L2 to the rows re-read by passes 2 and 3): C4 prox 2.31 -> 2.29 ms.
// Not kept: the update pass's (last) row reads streamed (no change), u and the cached gradient
// loaded nontemporal (2.29 -> 2.46 ms); profiles/r06/experiments/c4_streaming_hints.jsonl
#define MMX_HELD_DMA_CPOL 2
#endif
#ifndef MMX_WAVE_XCD
#define MMX_WAVE_XCD 1  // measured C4: prox 3.42 -> 3.29 ms (neighbouring tets share x and monitor-grid lines in one L2)
#endif
// One block (64 tets) of the 3D steady-state prox.  EXACT = false (k_prox_wave): the fast path;
// returns false, having written nothing, when a power met a near-midpoint (the block is queued).
// EXACT = true (k_prox_wave_fix): the exact recomputation of a queued block, entry gradient
// included (the fast pass may have left the cache at a point it then abandoned).
// DRAIN = false (the persistent loop): the block ends without waiting for its stores, so they drain
// while the wave's next block issues its loads
template <int D, bool COMP, bool EXACT, bool ISO = false, bool DRAIN = true>
__device__ __forceinline__ void prox_wave_block(const DeviceMesh<D>& m, double tol, const double* __restrict__ x,
                                                double* __restrict__ zg, double* __restrict__ ug, const double* Bin,
                                                double* Bout, double* __restrict__ partials, int useCache, int lb,
                                                double* ldsHeld) {
  constexpr int K = D * (D + 1), KK = K * K;
  const int tid = threadIdx.x;
  const int s0 = lb * 64;
  const bool act = s0 + tid < m.nF;
  const int s = act ? s0 + tid : s0;
  if constexpr (!EXACT) WPROF(0, s);
  int f[D + 1];
  loadVerts<D>(m, s, f);
  const unsigned fixedBits = m.sbits[s] & 0xF;
  double* zs = zg + zu_base<D>(s);
  double* us = ug + zu_base<D>(s);
  double* gc = m.gcache + (size_t)s * K;
  double z[K], dx[K], gcv[K];
  if (m.zx)
    gatherX<D>(m.zx, f, z);  // the step's first prox: z = D zx (DeviceMesh::zx)
  else
#pragma unroll
    for (int i = 0; i < K; ++i) z[i] = zs[zu_i<D>(i)];
#pragma unroll
  for (int i = 0; i < K; ++i) dx[i] = us[zu_i<D>(i)];
  if (!EXACT && useCache) {
#pragma unroll
    for (int i = 0; i < K; ++i) gcv[i] = gc[i];
  }
  double xi[K];
  if constexpr (COMP) gatherX<D>(m.Vc, f, xi);
  {
    double dxv[K];
    gatherX<D>(x, f, dxv);
#pragma unroll
    for (int i = 0; i < K; ++i) dx[i] = dxv[i] + dx[i];  // DXpU = D x + uBar
    if constexpr (WaveB<K>::kPre) {
      __builtin_amdgcn_sched_barrier(0);  // (not hoisted above the gathers' wait)
      // the held rows of the block's matrix (contiguous in the wave-interleaved layout, and in
      // the same order in ldsHeld) straight into LDS, 1 KB per instruction, requested once the
      // lane's inputs are in (the wait for the gathers, requested before the DMA, would otherwise
      // exceed the 63 loads vmcnt tracks and wait for the DMA too); the first pass 1 finds them
      // there
      const char* src = reinterpret_cast<const char*>(Bin + (size_t)lb * KK * 64) + tid * 16;
      char* dst = reinterpret_cast<char*>(ldsHeld);
#pragma unroll
      for (int c = 0; c < WaveB<K>::kHeld * K * 64 * 8 / 1024; ++c)
        __builtin_amdgcn_global_load_lds(src + c * 1024, (__attribute__((address_space(3))) void*)(dst + c * 1024),
                                         16, 0, MMX_HELD_DMA_CPOL);
    }
  }
  double pv[6] = {0, 0, 0, 0, 0, 0};
  bool tie = false;
  if (act) {
    // ISO: the isotropic-grid instance (GridView::iso set); otherwise the full-row instance, whose
    // monitor code is then exactly the general one (no second path competing for registers)
    GridView<D> g = gridOf<D>(m);
    if constexpr (ISO)
      __builtin_assume(g.iso != nullptr);
    else
      g.iso = nullptr;
    FunctionalConsts<D> fc = constsOf<D>(m);
    fc.compMesh = COMP ? 1 : 0;
    double G[K], Igt;
    bool bad = false;
    entry_grad<D, EXACT>(g, fc, z, xi, dx, gcv, !EXACT && useCache != 0, G, Igt, bad, &tie);
    zeroFixed<D>(G, fixedBits);
    const double Ihsave = Igt;
    if constexpr (!EXACT) WPROF(1, G[K - 1]);
    const size_t gb = (size_t)lb * KK * 64 + WaveB<K>::kLaneMul * tid;
    int its;
    {
      // the general-monitor instance requests its update-pass rows one further ahead (C4 prox
      // 2.291 -> 2.264 ms; the isotropic instance is slower with it: C4 moving bump 408 -> 405 it/s)
      using WB = WaveB<K, ISO ? MMX_ROW_PIPE : MMX_ROW_PIPE_FULL>;
      WB Bacc{(const gdouble*)(Bin + gb), (gdouble*)(Bout + gb), (ldouble*)(ldsHeld + WaveB<K>::kLaneMul * tid)};
      its = tie ? 0 : bfgs_iterations<D, WB, EXACT>(Bacc, g, fc, z, xi, dx, G, fixedBits, tol, bad, gc, &tie);
    }
    double dual2 = 0.0, z0[K];  // the entry z again (from zx on a step's first prox)
    if (m.zx)
      gatherX<D>(m.zx, f, z0);
    else
#pragma unroll
      for (int i = 0; i < K; ++i) z0[i] = zs[zu_i<D>(i)];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const double d = z[i] - z0[i];
      dual2 += d * d;
    }
    pv[0] = Ihsave;
    pv[1] = dual2;
    pv[3] = (double)its;
    pv[4] = bad ? 1.0 : 0.0;
    pv[5] = (double)its;
  }
  if constexpr (!EXACT) {
    if (m.forceTie > 0 && tid == 0 && (int)((unsigned)lb % (unsigned)m.forceTie) == 0) tie = true;
    if (__syncthreads_or(tie ? 1 : 0)) {  // rare: leave the block to k_prox_wave_fix
      if (tid == 0) m.tieList[atomicAdd(m.tieCount, 1u)] = lb;
      __builtin_amdgcn_s_waitcnt(0);  // (an entry tie skips pass 1: no DMA left in flight)
      return;
    }
  }
  if (act) {
    double un[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      zs[zu_i<D>(i)] = z[i];  // (nontemporal z/u stores measured slower: the x-update and the next prox read them)
      un[i] = dx[i] - z[i];  // uBar = DXpU - z
      us[zu_i<D>(i)] = un[i];
    }
    write_tslot<D>(m, s, z, un);
  }
  block_partials<6, 64>(pv, partials, lb);
  if constexpr (!EXACT && DRAIN) {
    __builtin_amdgcn_s_waitcnt(0);
    WPROF(6, pv[0]);
  }
}

template <int D, bool COMP, bool ISO = false>
__global__ void __launch_bounds__(64, D == 2 ? MMX_WAVE_OCC2 : MMX_WAVE_OCC) k_prox_wave(DeviceMesh<D> m, double tol, const double* __restrict__ x,
                                                     double* __restrict__ zg, double* __restrict__ ug,
                                                     const double* Bin, double* Bout, double* __restrict__ partials,
                                                     int useCache) {
  constexpr int K = D * (D + 1);
  __shared__ __attribute__((aligned(16))) double ldsHeld[WaveB<K>::kHeld > 0 ? WaveB<K>::kHeld * K * 64 : 2];
#if MMX_WAVE_PERSIST
  if constexpr (D == 3) {
    // persistent waves (experiment): workgroup w on XCD c = w % 8 walks the XCD's contiguous range of
    // blocks with stride gridDim / 8, so a wave starts its next block without ending (no drain of its
    // stores before the next block's loads are issued by a new wave)
    // (the grid is a multiple of 8: launch_prox rounds it up)
    const int nb = (m.nF + 63) / 64, g8 = max(1, (int)gridDim.x / 8), c = (int)(blockIdx.x % 8), j = (int)(blockIdx.x / 8);
    const int q = nb / 8, r = nb % 8, lo = c * q + min(c, r), hi = lo + q + (c < r ? 1 : 0);
    for (int lb = lo + j; lb < hi; lb += g8) {
      // (the next block's held-row DMA into ldsHeld is issued after this block's last reads of it
      // have returned: the final rows' stores consume them)
      prox_wave_block<D, COMP, false, ISO, false>(m, tol, x, zg, ug, Bin, Bout, partials, useCache, lb, ldsHeld);
    }
    return;
  }
#endif
  const int lb = MMX_WAVE_XCD ? logical_block_any() : (int)blockIdx.x;  // XCD-contiguous tet ranges
  prox_wave_block<D, COMP, false, ISO>(m, tol, x, zg, ug, Bin, Bout, partials, useCache, lb, ldsHeld);
}

// The exact recomputation of the blocks k_prox_wave queued, with the same Bkinv streaming (the
// generic one-lane k_prox_fix holds a tet's 144 Bkinv entries in registers and spills: ~0.3 ms
// for one block).  A fixed grid strides over the queue, as k_prox_fix.
template <int D, bool COMP, bool ISO = false>
__global__ void __launch_bounds__(64, D == 2 ? MMX_WAVE_OCC2 : MMX_WAVE_OCC) k_prox_wave_fix(DeviceMesh<D> m, double tol,
                                                         const double* __restrict__ x, double* __restrict__ zg,
                                                         double* __restrict__ ug, const double* Bin, double* Bout,
                                                         double* __restrict__ partials) {
  constexpr int K = D * (D + 1);
  __shared__ __attribute__((aligned(16))) double ldsHeld[WaveB<K>::kHeld > 0 ? WaveB<K>::kHeld * K * 64 : 2];
  const unsigned n = *m.tieCount;
  for (unsigned i = blockIdx.x; i < n; i += gridDim.x) {
    prox_wave_block<D, COMP, true, ISO>(m, tol, x, zg, ug, Bin, Bout, partials, 0, m.tieList[i], ldsHeld);
    __syncthreads();
  }
  rearm_tie_queue(m.tieStale);
}

// ---- 3D steady-state prox, four lanes per tetrahedron (k_prox_quad) ------------------------------
// Lane 4t + k of a workgroup works on tetrahedron t with quad lane k: it holds rows 3k..3k+2 of the
// tet's Bkinv in registers for the whole prox (Bkinv is read once and written once) and the
// components of vertex k (z, DXpU, gradient, p, y).  Full 12-vectors are assembled on demand from
// the four lanes with DPP quad broadcasts; every value any lane computes is formed with exactly the
// operations, in exactly the order, of the one-lane kernel (bit-identical): values that depend on
// the whole simplex (the 3x3 algebra of blockGrad, the powers, the scalar sums c2, yBy, |G|_1,
// ||z - zPrev||^2, the regulariser's ||DXpU - z||^2) are computed by all four lanes alike; the
// four vertex monitors of blockGrad are evaluated one per lane; the row-wise work (p = -B G,
// B y, the rank-two update) is split by rows; the column sums y^T B, sequential over the rows
// (src/Mesh.cpp:848), pass from quad lane to quad lane in row order.
template <int Q>
__device__ __forceinline__ double qb(double v) {  // quad lane Q's value, in every lane of the quad
  const int2 i = __builtin_bit_cast(int2, v);
  int2 r;
  r.x = __builtin_amdgcn_update_dpp(0, i.x, Q * 0x55, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp(0, i.y, Q * 0x55, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ int qb_or(int v) {  // OR over the quad
  int r = v;
  r |= __builtin_amdgcn_update_dpp(0, v, 1 * 0x55, 0xF, 0xF, false);
  r |= __builtin_amdgcn_update_dpp(0, v, 0 * 0x55, 0xF, 0xF, false);
  r |= __builtin_amdgcn_update_dpp(0, v, 2 * 0x55, 0xF, 0xF, false);
  r |= __builtin_amdgcn_update_dpp(0, v, 3 * 0x55, 0xF, 0xF, false);
  return r;
}
// full[3q + c] = own[c] of quad lane q
__device__ __forceinline__ void qfull(const double (&own)[3], double (&full)[12]) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    full[c] = qb<0>(own[c]);
    full[3 + c] = qb<1>(own[c]);
    full[6 + c] = qb<2>(own[c]);
    full[9 + c] = qb<3>(own[c]);
  }
}
template <int Q>
__device__ __forceinline__ M<3> qbM(const M<3>& a) {
  M<3> r;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) r.m[i][j] = qb<Q>(a.m[i][j]);
  return r;
}

// AdaptationFunctional<3>::blockGrad (src/AdaptationFunctional.cpp:102-287) with GRAD and REG,
// cooperatively: z = the tet's 12 coordinates (all lanes), zo / dxo = this lane's vertex (k) of z
// and DXpU; returns the regularised energy (all lanes) and this lane's 3 gradient components in
// go.  ghuang (the gradient cache of the simplex, or nullptr): this lane's unregularised
// components, and Igt from quad lane 0.  Same operations in the same order as blockGrad<3, true,
// true, EXACT> (admm_device.h), so every value is bit-identical to it.
template <bool EXACT>
__device__ __forceinline__ double blockGradQuad(const GridView<3>& g, const FunctionalConsts<3>& fc, int k,
                                                const double (&z)[12], const double* xi, const double (&zo)[3],
                                                const double (&dxo)[3], double (&go)[3], double& Igt,
                                                double* ghuang, bool* tiep) {
  bool tie = false;
  const double dFact = 6.0;
  // the vertex monitors: this lane's, then M = ((0 + m0) + m1) + m2) + m3 and the lane's own
  // difference m_k - m0 (the gradient's monitor-variation term needs m_{j+1} - m0 from lane j+1)
  M<3> mk;
  evalMonitor<3>(g, zo, mk);
  M<3> Msum, dmk;
  {
    const M<3> m0 = qbM<0>(mk);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        Msum.m[r][c] = 0.0 + m0.m[r][c];
        dmk.m[r][c] = mk.m[r][c] - m0.m[r][c];
      }
  }
  {
    const M<3> t = qbM<1>(mk);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) Msum.m[r][c] = Msum.m[r][c] + t.m[r][c];
  }
  {
    const M<3> t = qbM<2>(mk);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) Msum.m[r][c] = Msum.m[r][c] + t.m[r][c];
  }
  {
    const M<3> t = qbM<3>(mk);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) Msum.m[r][c] = Msum.m[r][c] + t.m[r][c];
  }
  M<3> Minv = inverse<3>(Msum);
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) Minv.m[r][c] = Minv.m[r][c] / ((double)3 + 1);
  M<3> E, Ehat;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      E.m[r][j] = z[3 * (j + 1) + r] - z[r];
      Ehat.m[r][j] = fc.compMesh ? (xi[3 * (j + 1) + r] - xi[r]) : fc.Ehat[r * 3 + j];
    }
  }
  // the regulariser's ||DXpU - z||^2, summed in index order over the four lanes' components
  double sq;
  {
    double t[3], tf[12];
#pragma unroll
    for (int c = 0; c < 3; ++c) t[c] = dxo[c] - zo[c];
    qfull(t, tf);
    sq = tf[0] * tf[0];
#pragma unroll
    for (int i = 1; i < 12; ++i) sq = sq + tf[i] * tf[i];
  }
  const double Edet = det<3>(E);
  if (!(Edet > 0)) {
    if (Edet <= 0 && g.invFlag) *g.invFlag = 1u;
    const double nan = __builtin_nan("");
#pragma unroll
    for (int c = 0; c < 3; ++c) go[c] = nan;
    if (ghuang) {
#pragma unroll
      for (int c = 0; c < 3; ++c) ghuang[3 * k + c] = nan;
    }
    Igt = nan;
    return nan;
  }
  const M<3> Einv = inverse<3>(E);
  const M<3> FJ = mul<3>(Ehat, Einv);
  const double detFJ = det<3>(FJ);
  const double d = 3.0;
  const double p = 1.5;
  const double theta = 1.0 / 3.0;
  const M<3> FJt = transpose<3>(FJ);
  const M<3> MinvJt = mul<3>(Minv, FJt);
  const M<3> JMJt = mul<3>(FJ, MinvJt);
  const double trJMJt = trace<3>(JMJt);
  const double detM = cr_sqrt(1.0 / det<3>(Minv));
  const double tr_dp2 = pow_dp2<3, EXACT>(trJMJt, tie);
  const double G = theta * detM * tr_dp2 + (1.0 - 2.0 * theta) * fc.powd * detM * cr_pow_p15<EXACT>(detFJ / detM, tie);
  const double absK = __builtin_fabs(Edet / dFact);
  const double tr_dp2m1 = pow_dp2m1<3, EXACT>(trJMJt, tie);
  const double detM_1mp = cr_pow_m05<EXACT>(detM, tie);
  M<3> dGdJ;
  {
    const double s = d * p * theta * detM * tr_dp2m1;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) dGdJ.m[r][c] = s * MinvJt.m[r][c];
  }
  const double dGddet = p * (1.0 - 2.0 * theta) * fc.powd * detM_1mp * cr_pow_p05(detFJ);
  M<3> dGdM;
  {
    const double s1 = -0.5 * theta * d * p * detM * tr_dp2m1;
    const M<3> MinvT = transpose<3>(Minv);
    M<3> T;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) T.m[r][c] = s1 * MinvT.m[r][c];
    T = mul<3>(mul<3>(mul<3>(T, FJt), FJ), Minv);
    const double s2 = 0.5 * theta * detM * tr_dp2 +
                      ((0.5 - theta) * (1.0 - p) * fc.powd) * detM_1mp * cr_pow_p15<EXACT>(detFJ, tie);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) dGdM.m[r][c] = T.m[r][c] + s2 * Minv.m[r][c];
  }
  // trace(dGdM (m_{j+1} - m0)) from lane j + 1 (lane 0's value is not used)
  const double trk = trace<3>(mul<3>(dGdM, dmk));
  const double trj[3] = {qb<1>(trk), qb<2>(trk), qb<3>(trk)};
  double basisComb[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) basisComb[c] = 0.0;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int c = 0; c < 3; ++c) basisComb[c] += Einv.m[j][c] * trj[j];
  const double c1 = (-G + dGddet * detFJ);
  M<3> vLoc;
  {
    const M<3> P = mul<3>(mul<3>(Einv, dGdJ), FJ);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) vLoc.m[r][c] = c1 * Einv.m[r][c] + P.m[r][c];
  }
#pragma unroll
  for (int n = 0; n < 3; n++)
#pragma unroll
    for (int c = 0; c < 3; ++c) vLoc.m[n][c] -= (basisComb[c]) / ((double)3 + 1.0);
  // this lane's gradient components: vertex 0 sums the columns of vLoc, vertex n >= 1 is -vLoc[n-1]
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double s = 0.0;
#pragma unroll
    for (int n = 0; n < 3; n++) s += vLoc.m[n][c];
    const double g0 = s + (basisComb[c] + 0.0);
    const double gn = (k == 1) ? -vLoc.m[0][c] : (k == 2) ? -vLoc.m[1][c] : -vLoc.m[2][c];
    go[c] = ((k == 0) ? g0 : gn) * absK;
  }
  double Ih = absK * G;
  Igt = Ih;
  if constexpr (!EXACT) *tiep = *tiep || tie;
  if (ghuang) {
#pragma unroll
    for (int c = 0; c < 3; ++c) ghuang[3 * k + c] = go[c];
  }
  Ih += 0.5 * fc.w * fc.w * sq;
#pragma unroll
  for (int c = 0; c < 3; ++c) go[c] += fc.w * fc.w * (-dxo[c] + zo[c]);
  return Ih;
}

// The steady-state 3D prox with four lanes per tetrahedron (see above).  A workgroup of QW lanes
// takes QW / 4 consecutive tets (a quarter or all of one group of the wave-interleaved Bkinv layout,
// bidx<3>); Bkinv is double-buffered as for k_prox_wave (Bin only read, Bout written).  EXACT =
// false is the fast path (no tie resolution, Markstein divisions): a block that meets a
// near-midpoint power or a quotient outside div_mk's range writes nothing back and is queued;
// EXACT = true recomputes the queued blocks (the workgroups stride over the queue) with the exact
// decisions, a full entry blockGrad and the same partial-sum tree, and the last workgroup to finish
// re-arms the queue.
template <int TB>
constexpr int kQuadImg = 36 * TB + 8;  // doubles per quad-lane block of the LDS image (bank offset 16 dwords)
template <bool COMP, bool EXACT, int QW>
__global__ void __launch_bounds__(QW, 2) k_prox_quad(DeviceMesh<3> m, double tol, const double* __restrict__ x,
                                                             double* __restrict__ zg, double* __restrict__ ug,
                                                             const double* Bin, double* Bout,
                                                             double* __restrict__ partials, int useCache) {
  constexpr int K = 12, KK = 144, TB = QW / 4, KB = kQuadImg<TB>;
  // LDS image of the block's Bkinv: quad lane k's rows of the TB tets in block k (3 x 12 entries of
  // TB tets); the four blocks 16 dwords apart in the banks, so the 32 lanes of a half-wavefront (8
  // tets x 4 quad lanes) reading one entry hit 64 distinct banks
  __shared__ __attribute__((aligned(16))) double img[4 * KB];
  const int tid = threadIdx.x, k = tid & 3, tl = tid >> 2;
  const unsigned nWork = EXACT ? *m.tieCount : 1u;
  for (unsigned w = EXACT ? blockIdx.x : 0u; w < nWork; w += EXACT ? gridDim.x : 1u) {
    const int lb = EXACT ? m.tieList[w] : logical_block_any();
    const int s0 = lb * TB;
    const bool act = s0 + tl < m.nF;
    const int s = act ? s0 + tl : s0;
    const int fk = m.F[(size_t)s * 4 + k];
    const unsigned fixedBits = m.sbits[s] & 0xF;
    const bool ownFixed = (fixedBits >> k) & 1u;
    double* zs = zg + (size_t)s * K + 3 * k;
    double* us = ug + (size_t)s * K + 3 * k;
    double* gc = m.gcache + (size_t)s * K;
    double zo[3], z0[3], dxo[3], go[3], Igt = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      zo[c] = m.zx ? m.zx[(size_t)fk * 3 + c] : zs[c];  // a step's first prox: z = D zx (DeviceMesh::zx)
      z0[c] = zo[c];
      dxo[c] = x[(size_t)fk * 3 + c] + us[c];  // DXpU = D x + uBar
    }
    const bool cached = !EXACT && useCache;
    if (cached) {
#pragma unroll
      for (int c = 0; c < 3; ++c) go[c] = gc[3 * k + c];
    }
    double xi[K];
    if constexpr (COMP) {
      double xo[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) xo[c] = m.Vc[(size_t)fk * 3 + c];
      qfull(xo, xi);
    }
    // the block's Bkinv chunk (64 tets x 144, contiguous in the wave-interleaved layout) staged
    // through LDS with 16-byte coalesced loads, then this lane's three rows into registers
    // the block's TB tets in their group of 64: entry ij of tet s0 + t at gb + ij 64 + t
    const size_t gb = (size_t)(s0 >> 6) * KK * 64 + (s0 & 63);
    static_assert(!MMX_B3_PAIRS || TB == 64, "paired Bkinv layout: whole wave blocks per quad workgroup");
#pragma unroll 6
    for (int e = tid * 2; e < KK * TB; e += 2 * QW) {
      if constexpr (MMX_B3_PAIRS) {  // 16 bytes = entries ij, ij + 1 of one tet (bidx<3>)
        const int ij = (e / (2 * TB)) * 2, t = (e % (2 * TB)) / 2;
        const v2nt v = __builtin_nontemporal_load(reinterpret_cast<const v2nt*>(Bin + gb - (s0 & 63) + (size_t)e));
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = (ij + h) / K, j = ij + h - K * i, kk = i / 3, r = i - 3 * kk;
          img[kk * KB + (r * K + j) * TB + t] = v[h];
        }
      } else {
        const int ij = e / TB, t = e % TB, i = ij / K, j = ij - K * i, kk = i / 3, r = i - 3 * kk;
        const v2nt v = __builtin_nontemporal_load(reinterpret_cast<const v2nt*>(Bin + gb + (size_t)ij * 64 + t));
        *reinterpret_cast<v2nt*>(&img[kk * KB + (r * K + j) * TB + t]) = v;
      }
    }
    // entry (r, j) of this lane's rows at mine[(r K + j) 64]: read into registers by each pass (not
    // held across the blockGrad), the new values written back by the update pass
    double* const mine = img + k * KB + tl;
    __syncthreads();
    double pv[6] = {0, 0, 0, 0, 0, 0};
    bool tie = false;
    if (act) {
      const GridView<3> g = gridOf<3>(m);
      FunctionalConsts<3> fc = constsOf<3>(m);
      fc.compMesh = COMP ? 1 : 0;
      bool bad = false;
      if (cached) {  // entry_grad with the cache: the unregularised part plus the regulariser
#pragma unroll
        for (int c = 0; c < 3; ++c) go[c] += fc.w * fc.w * (-dxo[c] + zo[c]);
        bad |= (go[0] != go[0]);  // an inverted element's cached gradient is all NaN
      } else {
        double zf[K];
        qfull(zo, zf);
        const double e = blockGradQuad<EXACT>(g, fc, k, zf, xi, zo, dxo, go, Igt, nullptr, &tie);
        bad |= (e != e);
      }
      if (ownFixed)
#pragma unroll
        for (int c = 0; c < 3; ++c) go[c] = 0.0;
      const double Ihsave = Igt;
      int iter;
      for (iter = 0; iter < 50 && !tie; iter++) {
        // p = -B G (rows 3k..3k+2)
        double po[3];
        {
          double Gf[K];
          qfull(go, Gf);
#pragma unroll
          for (int r = 0; r < 3; ++r) {
            double row[K];
#pragma unroll
            for (int j = 0; j < K; ++j) row[j] = mine[(r * K + j) * TB];
            double sacc = (-row[0]) * Gf[0];
#pragma unroll
            for (int j = 1; j < K; ++j) sacc += (-row[j]) * Gf[j];
            po[r] = sacc;
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) zo[c] += po[c];
        double G1o[3], Ig1;
        {
          double zf[K];
          qfull(zo, zf);
          const double e = blockGradQuad<EXACT>(g, fc, k, zf, xi, zo, dxo, G1o, Ig1, gc, &tie);
          bad |= (e != e);
        }
        if constexpr (!EXACT) {
          if (qb_or(tie ? 1 : 0)) {
            tie = true;
            break;
          }
        }
        if (ownFixed)
#pragma unroll
          for (int c = 0; c < 3; ++c) G1o[c] = 0.0;
        double Ix = 0;
        double yo[3], yf[K];
        {
          double G1f[K];
          qfull(G1o, G1f);
#pragma unroll
          for (int i = 0; i < K; i++) Ix += __builtin_fabs(G1f[i]);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) yo[c] = G1o[c] - go[c];
        qfull(yo, yf);
        double c2;
        {
          double pf[K];
          qfull(po, pf);
          c2 = pf[0] * yf[0];
#pragma unroll
          for (int i = 1; i < K; ++i) c2 += pf[i] * yf[i];
        }
        // pass 2: By (rows), yBy = sum_i y_i By_i, yB_j = sum_i y_i B_ij (i ascending: lane to lane);
        // yB ends in quad lane 3 and is handed out as slices like p: yBo[c] = yB_{3k+c}
        double yBy, yBo[3];
        double rows[3][K];  // live through passes 2 and 3 (the update reads the old rows throughout)
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int j = 0; j < K; ++j) rows[r][j] = mine[(r * K + j) * TB];
        {
          double byo[3], byf[K];
#pragma unroll
          for (int r = 0; r < 3; ++r) {
            double by = rows[r][0] * yf[0];
#pragma unroll
            for (int j = 1; j < K; ++j) by += rows[r][j] * yf[j];
            byo[r] = by;
          }
          qfull(byo, byf);
          yBy = yf[0] * byf[0];
#pragma unroll
          for (int i = 1; i < K; ++i) yBy = yBy + yf[i] * byf[i];
          double P[K];
#pragma unroll
          for (int j = 0; j < K; ++j) P[j] = (yo[0] * rows[0][j] + yo[1] * rows[1][j]) + yo[2] * rows[2][j];
#pragma unroll
          for (int j = 0; j < K; ++j) P[j] = ((qb<0>(P[j]) + yo[0] * rows[0][j]) + yo[1] * rows[1][j]) + yo[2] * rows[2][j];
#pragma unroll
          for (int j = 0; j < K; ++j) P[j] = ((qb<1>(P[j]) + yo[0] * rows[0][j]) + yo[1] * rows[1][j]) + yo[2] * rows[2][j];
#pragma unroll
          for (int j = 0; j < K; ++j) P[j] = ((qb<2>(P[j]) + yo[0] * rows[0][j]) + yo[1] * rows[1][j]) + yo[2] * rows[2][j];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const double a0 = qb<3>(P[c]), a1 = qb<3>(P[3 + c]), a2 = qb<3>(P[6 + c]), a3 = qb<3>(P[9 + c]);
            yBo[c] = (k == 0) ? a0 : (k == 1) ? a1 : (k == 2) ? a2 : a3;
          }
        }
        const double c1 = (c2 + yBy) / cr_pow_2(c2);
        const double rc2 = 1.0 / c2;
        unsigned eBy = 0u;
        double fin = 0.0;
        // pass 3: B_ij += c1 p_i p_j - (B (y p^T))_ij / c2 - p_i (y^T B)_j / c2, column by column
        // (column j's products y_q p_j shared by the three rows), into the LDS image
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const double pj = (j < 3) ? qb<0>(po[j % 3]) : (j < 6) ? qb<1>(po[j % 3]) : (j < 9) ? qb<2>(po[j % 3]) : qb<3>(po[j % 3]);
          const double yBj =
              (j < 3) ? qb<0>(yBo[j % 3]) : (j < 6) ? qb<1>(yBo[j % 3]) : (j < 9) ? qb<2>(yBo[j % 3]) : qb<3>(yBo[j % 3]);
          double v[K];
#pragma unroll
          for (int q = 0; q < K; ++q) v[q] = yf[q] * pj;
#pragma unroll
          for (int r = 0; r < 3; ++r) {
            double by = rows[r][0] * v[0];
#pragma unroll
            for (int q = 1; q < K; ++q) by += rows[r][q] * v[q];
            double nb;
            if constexpr (EXACT) {
              nb = rows[r][j] + (((c1 * (po[r] * pj)) - by / c2) - (po[r] * yBj) / c2);
            } else {
              eBy = max(eBy, mk_exp(by, 900));
              nb = rows[r][j] + (((c1 * (po[r] * pj)) - div_mk(by, c2, rc2)) - div_mk(po[r] * yBj, c2, rc2));
              fin = cr_fma(nb, 0.0, fin);
            }
            mine[(r * K + j) * TB] = nb;
          }
        }
        if constexpr (!EXACT) {
          // the ranges of p and yB: each lane checks its slices (a max: order-free), the quad ORs
          unsigned ePY = 0u;
#pragma unroll
          for (int c = 0; c < 3; ++c) ePY = max(ePY, max(mk_exp(po[c], 450), mk_exp(yBo[c], 450)));
          const bool out = !(c2 >= 0x1p-100 && c2 <= 0x1p100) || eBy > 1799u || ePY > 899u || fin != 0.0;
          if (qb_or(out ? 1 : 0)) {
            tie = true;
            break;
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) go[c] = G1o[c];
        if (Ix < tol) break;
      }
      const int its = (iter == 50) ? 50 : iter + 1;
      double dual2 = 0.0;
      {
        double dz[3], dzf[K];
#pragma unroll
        for (int c = 0; c < 3; ++c) dz[c] = zo[c] - z0[c];
        qfull(dz, dzf);
#pragma unroll
        for (int i = 0; i < K; ++i) dual2 += dzf[i] * dzf[i];
      }
      if (k == 0) {
        pv[0] = Ihsave;
        pv[1] = dual2;
        pv[3] = (double)its;
        pv[4] = bad ? 1.0 : 0.0;
        pv[5] = (double)its;
      }
    }
    if constexpr (!EXACT) {
      if (m.forceTie > 0 && tid == 0 && (int)((unsigned)lb % (unsigned)m.forceTie) == 0) tie = true;
      if (__syncthreads_or(tie ? 1 : 0)) {  // rare: leave the block to the exact instance
        if (tid == 0) m.tieList[atomicAdd(m.tieCount, 1u)] = lb;
        return;
      }
    }
    if (act) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double un = dxo[c] - zo[c];  // uBar = DXpU - z
        zs[c] = zo[c];
        us[c] = un;
        if (m.tslot) m.tslot[(size_t)s * K + 3 * k + c] = m.w * (m.w * (zo[c] - un));
      }
    }
    if constexpr (EXACT) __syncthreads();  // (the fast path's __syncthreads_or orders the image)
    // the new Bkinv chunk back with 16-byte coalesced stores (inactive tets: the unchanged image)
#pragma unroll 6
    for (int e = tid * 2; e < KK * TB; e += 2 * QW) {
      if constexpr (MMX_B3_PAIRS) {
        const int ij = (e / (2 * TB)) * 2, t = (e % (2 * TB)) / 2;
        v2nt v;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = (ij + h) / K, j = ij + h - K * i, kk = i / 3, r = i - 3 * kk;
          v[h] = img[kk * KB + (r * K + j) * TB + t];
        }
        __builtin_nontemporal_store(v, reinterpret_cast<v2nt*>(Bout + gb - (s0 & 63) + (size_t)e));
      } else {
        const int ij = e / TB, t = e % TB, i = ij / K, j = ij - K * i, kk = i / 3, r = i - 3 * kk;
        const v2nt v = *reinterpret_cast<const v2nt*>(&img[kk * KB + (r * K + j) * TB + t]);
        __builtin_nontemporal_store(v, reinterpret_cast<v2nt*>(Bout + gb + (size_t)ij * 64 + t));
      }
    }
    block_partials<6, QW>(pv, partials, lb);
    if constexpr (EXACT) __syncthreads();  // the partials scratch is reused by the next block
  }
  if constexpr (EXACT) rearm_tie_queue(m.tieStale);
}

// Mesh::computeEnergy (src/Mesh.cpp:496-530) on positions x
template <int D, int ISO = -1>
__global__ void __launch_bounds__(kBlock) k_energy(DeviceMesh<D> m, const double* __restrict__ x,
                                                    double* __restrict__ partials) {
  constexpr int K = D * (D + 1);
  const int s = blockIdx.x * kBlock + threadIdx.x;
  double pv[5] = {0, 0, 0, 0, 0};
  if (s < m.nF) {
    int f[D + 1];
    loadVerts<D>(m, s, f);
    double z[K], xi[K], Igt;
    gatherX<D>(x, f, z);
    loadXi<D>(m, f, xi);
    const double e = blockGrad<D, false, false>(gridOf<D, ISO>(m), constsOf<D>(m), z, xi, nullptr, nullptr, Igt);
    pv[0] = e;
    pv[4] = (e == e) ? 0.0 : 1.0;
  }
  block_partials<5>(pv, partials);
}

// Mesh::eulerStepMod scatter (src/Mesh.cpp:566-572): INTERIOR nodes only; x -= (dt/tau) grad
template <int D>
__global__ void __launch_bounds__(kBlock) k_euler_apply(DeviceMesh<D> m, const double* __restrict__ gs,
                                                         double* __restrict__ x, double dt_over_tau, int xcd) {
  const int idx = logical_block(xcd) * kBlock + threadIdx.x;
  if (idx >= m.nP) return;
  // nodes in the x-update's processing order (first incident simplex; 3D: y slabs): a workgroup's
  // nodes gather from neighbouring simplices (C4: 0.58 ms in node-id order)
  const int v = m.nodeOrder ? m.nodeOrder[idx] : idx;
  double g[D];
#pragma unroll
  for (int c = 0; c < D; ++c) g[c] = 0.0;
  if (m.nodeInterior[v]) {
    const int b = m.inc_ptr[v], e = m.inc_ptr[v + 1];
    for (int t = b; t < e; ++t) {
      const int off = m.inc_off[t];
      const double* src = (off >= 0) ? gs + off : m.remote + (size_t)(-1 - off) * D;
#pragma unroll
      for (int c = 0; c < D; ++c) g[c] += src[c];
    }
  }
#pragma unroll
  for (int c = 0; c < D; ++c) x[(size_t)v * D + c] -= dt_over_tau * g[c];
}

// ---- backward Euler -------------------------------------------------------------------------
// FSubJac's derivative blocks (src/Mesh.cpp:1173-1230), simplex-centric: thread (s, n) evaluates
// blockGrad at the vertices Vp (pass -1, the reference's Gk) and with coordinate i of vertex n
// moved by h (pass i), and writes derivs(i, :) = (Gkp1 - Gk) / h.  A BOUNDARY_FIXED vertex gets
// the reference's identity pattern, which is nonzero only for n == 0 (r == c in D*n..D*n+D-1).
// The node-centric reference evaluates Gk once per (node, simplex); the values are the same.
// EXACT = false (with `work`): the fast path -- a lane whose powers meet a rounding midpoint (or
// leave the double-double ranges) writes nothing and queues itself (work[0] counts, work[1 + q]
// lists), and k_fd_jac_fix recomputes the queued lanes with the exact decision.  On the regular
// initial meshes the exact path is common, and in the one-kernel form every wave with one such
// lane ran it, with its expansion arithmetic in 5 KB of scratch per lane (C4: 110 ms)
template <int D, int ISO, bool EXACT>
__device__ __forceinline__ void fd_jac_lane(const DeviceMesh<D>& m, const double* __restrict__ Vp, double h,
                                            double* __restrict__ dv, long long t, unsigned* work) {
  constexpr int K = D * (D + 1);
  const int s = (int)(t / (D + 1)), n = (int)(t % (D + 1));
  double* out = dv + (size_t)t * D * K;
  if (m.sbits[s] & (1u << n)) {
    for (int r = 0; r < D; ++r)
#pragma unroll
      for (int c = 0; c < K; ++c) out[r * K + c] = (c == r && c >= D * n && c < D * (n + 1)) ? 1.0 : 0.0;
    return;
  }
  int f[D + 1];
  loadVerts<D>(m, s, f);
  double xl[K], xi[K], gk[K], g1[K], xp[K], Igt;
  gatherX<D>(Vp, f, xl);
  loadXi<D>(m, f, xi);
  const GridView<D> g = gridOf<D, ISO>(m);
  const FunctionalConsts<D> fc = constsOf<D>(m);
  bool tie = false;
#pragma unroll 1
  for (int it = -1; it < D; ++it) {
    const int moved = (it < 0) ? -1 : D * n + it;
#pragma unroll
    for (int c = 0; c < K; ++c) xp[c] = (c == moved) ? xl[c] + h : xl[c];
    blockGrad<D, true, false, EXACT>(g, fc, xp, xi, nullptr, g1, Igt, nullptr, &tie);
    if (it < 0) {
#pragma unroll
      for (int c = 0; c < K; ++c) gk[c] = g1[c];
    } else {  // (a queued lane's rows are all written again by k_fd_jac_fix)
#pragma unroll
      for (int c = 0; c < K; ++c) out[it * K + c] = (g1[c] - gk[c]) / h;
    }
  }
  if constexpr (!EXACT) {
    if (tie) work[1 + atomicAdd(work, 1u)] = (unsigned)t;
  }
}
template <int D, int ISO = -1, bool EXACT = true>
__global__ void __launch_bounds__(kBlock) k_fd_jac(DeviceMesh<D> m, const double* __restrict__ Vp, double h,
                                                    double* __restrict__ dv, unsigned* work) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (long long)m.nF * (D + 1)) return;
  fd_jac_lane<D, ISO, EXACT>(m, Vp, h, dv, t, work);
}
// the lanes k_fd_jac<.., false> queued, exactly (a fixed grid striding over the queue)
template <int D, int ISO = -1>
__global__ void __launch_bounds__(kBlock) k_fd_jac_fix(DeviceMesh<D> m, const double* __restrict__ Vp, double h,
                                                        double* __restrict__ dv, const unsigned* __restrict__ work) {
  const unsigned nq = work[0];
  for (unsigned q = blockIdx.x * kBlock + threadIdx.x; q < nq; q += gridDim.x * kBlock)
    fd_jac_lane<D, ISO, true>(m, Vp, h, dv, (long long)work[1 + q], nullptr);
}

// buildEulerJac + FSubJac's scatter (src/Mesh.cpp:1112-1136, 1232-1258), row-centric: row
// r = D*pnt + p, entry (col node ci, offset co).  The reference adds, for each incident simplex
// in ascending id and each vertex j in pairsort order, derivs(p, D*rel[j]+co) where the sorted id
// equals ci and +0.0 elsewhere; the +0.0 adds only turn a -0.0 sum into +0.0, so the same value
// is v + 0.0 before the matching vertex (if it is not first), + d, + 0.0 after (if not last).
template <int D>
__global__ void __launch_bounds__(kBlock) k_jac_assemble(DeviceMesh<D> m, const int* __restrict__ ia,
                                                          const int* __restrict__ ja, const double* __restrict__ dv,
                                                          double dt_over_tau, int finish, double* __restrict__ a) {
  constexpr int K = D * (D + 1);
  const int r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= m.nP * D) return;
  const int pnt = r / D, p = r % D;
  const int tb = m.inc_ptr[pnt], te = m.inc_ptr[pnt + 1];
  for (int i = ia[r]; i < ia[r + 1]; ++i) {
    const int col = ja[i], ci = col / D, co = col % D;
    double v = 0.0;
    for (int t = tb; t < te; ++t) {
      const int off = m.inc_off[t];
      const int s = off / K, nl = (off % K) / D;
      int f[D + 1];
      loadVerts<D>(m, s, f);
      int hit = -1, rank = 0;
#pragma unroll
      for (int k = 0; k < D + 1; ++k) {
        if (f[k] == ci) hit = k;
        rank += (f[k] < ci) ? 1 : 0;
      }
      if (hit >= 0) {
        if (rank > 0) v = v + 0.0;
        v = v + dv[((size_t)(s * (D + 1) + nl) * D + p) * K + D * hit + co];
        if (rank < D) v = v + 0.0;
      } else {
        v = v + 0.0;
      }
    }
    if (finish) {  // buildEulerJac's scaling and identity (src/Mesh.cpp:1125-1134); else the FSubJac sums
      v *= dt_over_tau;
      if (col == r) v += 1.0;
    }
    a[i] = v;
  }
}

// The same sums simplex-outer: row r walks its node's incident simplices once (ascending id) and
// adds each simplex's derivative block to the entries of its D + 1 vertices, found by a binary
// search over the row's node-major columns.  Every entry receives its terms in the same order as
// above; the +0.0 adds are dropped because they change nothing here -- an entry starts at +0.0, and
// a sum that starts at +0.0 is never -0.0 under round-to-nearest (+0 + -0 = +0, x + -x = +0), so
// v + 0.0 = v at every step (bit-identical; C4: 26 ms for the entry-outer form, which loaded the
// node's incident simplices again for every entry of the row)
template <int D>
__global__ void __launch_bounds__(kBlock) k_jac_assemble_s(DeviceMesh<D> m, const int* __restrict__ ia,
                                                            const int* __restrict__ ja, const double* __restrict__ dv,
                                                            double dt_over_tau, int finish, double* __restrict__ a) {
  constexpr int K = D * (D + 1);
  const int r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= m.nP * D) return;
  const int pnt = r / D, p = r % D;
  const int rb = ia[r], re = ia[r + 1], nn = (re - rb) / D;
  for (int i = rb; i < re; ++i) a[i] = 0.0;
  const int tb = m.inc_ptr[pnt], te = m.inc_ptr[pnt + 1];
  for (int t = tb; t < te; ++t) {
    const int off = m.inc_off[t];
    const int s = off / K, nl = (off % K) / D;
    int f[D + 1];
    loadVerts<D>(m, s, f);
    const double* d = dv + ((size_t)(s * (D + 1) + nl) * D + p) * K;
#pragma unroll
    for (int k = 0; k < D + 1; ++k) {
      int lo = 0, hi = nn - 1;  // the node f[k] among the row's nodes (ascending; it is there)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ja[rb + mid * D] / D < f[k])
          lo = mid + 1;
        else
          hi = mid;
      }
      double* e = a + rb + lo * D;
#pragma unroll
      for (int co = 0; co < D; ++co) e[co] = e[co] + d[D * k + co];
    }
  }
  if (finish) {
    for (int i = rb; i < re; ++i) {
      double v = a[i] * dt_over_tau;
      if (ja[i] == r) v += 1.0;
      a[i] = v;
    }
  }
}

// The same sums with one wavefront per node: lane q holds the D x D entries (rows p, offsets co)
// of the node's q-th column node (the node's D rows share their node-major columns) and the wave
// walks the node's incident simplices once, in ascending id (uniform loads); the lanes of the
// simplex's vertices add its derivative values -- every entry its terms in the same order
// (bit-identical; at most 64 column nodes, checked by the launch).  A node that no simplex
// references (the Shoulder meshes have such nodes) has rows holding only their diagonal entry
// (mmx_struc_mesh_pattern), not node blocks: its entries are +0.0 (and the identity) as in the
// other forms.
template <int D>
__global__ void __launch_bounds__(256) k_jac_assemble_w(DeviceMesh<D> m, const int* __restrict__ ia,
                                                         const int* __restrict__ ja, const double* __restrict__ dv,
                                                         double dt_over_tau, int finish, double* __restrict__ a) {
  constexpr int K = D * (D + 1);
  const int pnt = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6), lane = (int)threadIdx.x & 63;
  if (pnt >= m.nP) return;
  const int tb = m.inc_ptr[pnt], te = m.inc_ptr[pnt + 1];
  if (tb == te) {
#pragma unroll
    for (int p = 0; p < D; ++p) {
      const int r = pnt * D + p;
      for (int i = ia[r] + lane; i < ia[r + 1]; i += 64) {
        double v = 0.0;
        if (finish) {
          v *= dt_over_tau;
          if (ja[i] == r) v += 1.0;
        }
        a[i] = v;
      }
    }
    return;
  }
  const int r0 = pnt * D, rb = ia[r0], nn = (ia[r0 + 1] - rb) / D;
  const bool act = lane < nn;
  const int ci = act ? ja[rb + lane * D] / D : -1;
  double acc[D][D];
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int co = 0; co < D; ++co) acc[p][co] = 0.0;
  for (int t = tb; t < te; ++t) {
    const int off = m.inc_off[t];
    const int s = off / K, nl = (off % K) / D;
    int f[D + 1];
    loadVerts<D>(m, s, f);
    int hit = -1;
#pragma unroll
    for (int k = 0; k < D + 1; ++k)
      if (f[k] == ci) hit = k;
    if (hit >= 0) {
      const double* d = dv + ((size_t)(s * (D + 1) + nl) * D) * K + D * hit;
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int co = 0; co < D; ++co) acc[p][co] = acc[p][co] + d[p * K + co];
    }
  }
  if (!act) return;
#pragma unroll
  for (int p = 0; p < D; ++p) {
    const int r = r0 + p, i0 = ia[r] + lane * D;
#pragma unroll
    for (int co = 0; co < D; ++co) {
      double v = acc[p][co];
      if (finish) {  // buildEulerJac's scaling and identity (src/Mesh.cpp:1125-1134)
        v *= dt_over_tau;
        if (ja[i0 + co] == r) v += 1.0;
      }
      a[i0 + co] = v;
    }
  }
}

// Newton residual of backwardsEulerStep (src/Mesh.cpp:1301-1306): grad from eulerStepMod's
// INTERIOR-only scatter (ascending simplex id), F = grad * (dt/tau) + (x - xn), rhs = -F.
// ORD: the nodes in the x-update's processing order (their gathers from neighbouring simplices; C4
// 0.58 ms in node-id order) and no partials -- k_abs_partials then forms them from rhs in node-id
// order with this kernel's blocks, the same sums in the same order (bit-identical)
template <int D, bool ORD = false>
__global__ void __launch_bounds__(kBlock) k_be_residual(DeviceMesh<D> m, const double* __restrict__ gs,
                                                         const double* __restrict__ x, const double* __restrict__ xn,
                                                         double dt_over_tau, double* __restrict__ rhs,
                                                         double* __restrict__ partials, int xcd) {
  const int lb = logical_block(xcd);
  const int idx = lb * kBlock + threadIdx.x;
  const int v = (ORD && idx < m.nP) ? m.nodeOrder[idx] : idx;
  double pv[1] = {0.0};
  if (v < m.nP) {
    double g[D];
#pragma unroll
    for (int c = 0; c < D; ++c) g[c] = 0.0;
    if (m.nodeInterior[v]) {
      const int b = m.inc_ptr[v], e = m.inc_ptr[v + 1];
      for (int t = b; t < e; ++t) {
        const double* src = gs + m.inc_off[t];
#pragma unroll
        for (int c = 0; c < D; ++c) g[c] += src[c];
      }
    }
#pragma unroll
    for (int c = 0; c < D; ++c) {
      const double F = g[c] * dt_over_tau + (x[(size_t)v * D + c] - xn[(size_t)v * D + c]);
      pv[0] += __builtin_fabs(F);
      rhs[(size_t)v * D + c] = -F;
    }
  }
  if constexpr (!ORD) block_partials<1>(pv, partials, lb);
}
// the partials of k_be_residual<D, false> from rhs = -F (|-F| = |F| exactly)
template <int D>
__global__ void __launch_bounds__(kBlock) k_abs_partials(int nP, const double* __restrict__ rhs,
                                                          double* __restrict__ partials, int xcd) {
  const int lb = logical_block(xcd);
  const int v = lb * kBlock + threadIdx.x;
  double pv[1] = {0.0};
  if (v < nP) {
#pragma unroll
    for (int c = 0; c < D; ++c) pv[0] += __builtin_fabs(rhs[(size_t)v * D + c]);
  }
  block_partials<1>(pv, partials, lb);
}

__global__ void __launch_bounds__(kBlock) k_add_inplace(int n, double* __restrict__ x, const double* __restrict__ dx) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) x[i] += dx[i];
}

template <int D>
__global__ void __launch_bounds__(kBlock) k_pack_export(int mode, int nExp, const int* __restrict__ expOff,
                                                         const double* __restrict__ z, const double* __restrict__ u,
                                                         const double* __restrict__ gs, double w,
                                                         double* __restrict__ out, PackZX zx) {
  constexpr int K = D * (D + 1);
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= nExp) return;
  const size_t off = (size_t)expOff[e], zo = zu_off<D>(expOff[e]);
  double zv[D];
  if (mode == 0 && zx.zx) {  // z of the slot = zx of its node (DeviceMesh::zx); predicted: 2 x - xPrev
    const int s = expOff[e] / K, n = (expOff[e] % K) / D;
    const size_t v = (size_t)zx.F[(size_t)s * (D + 1) + n];
#pragma unroll
    for (int c = 0; c < D; ++c) zv[c] = zx.x ? 2 * zx.x[v * D + c] - zx.xPrev[v * D + c] : zx.zx[v * D + c];
  } else {
#pragma unroll
    for (int c = 0; c < D; ++c) zv[c] = z[zo + c];
  }
#pragma unroll
  for (int c = 0; c < D; ++c)
    out[(size_t)e * D + c] = (mode == 0) ? w * (w * (zv[c] - u[zo + c])) : gs[off + c];
}

constexpr int kRed = 1024;
__device__ void reduce_set(const double* __restrict__ partials, int nblocks, double* __restrict__ out);

__global__ void __launch_bounds__(kRed) k_reduce_partials(const double* __restrict__ partials, int nblocks,
                                                           double* __restrict__ out, const double* __restrict__ partials2,
                                                           int nblocks2, double* __restrict__ out2) {
  if (blockIdx.x == 1)  // second set in the same launch
    reduce_set(partials2, nblocks2, out2);
  else
    reduce_set(partials, nblocks, out);
}

// a whole step's reductions in one launch (early exit off): workgroup i < n reduces the prox
// partials of iteration i (slices of `stride` doubles), workgroup n the last x-update's
__global__ void __launch_bounds__(kRed) k_reduce_steps(const double* __restrict__ partA, size_t stride, int nbA,
                                                        const double* __restrict__ partB, int nbB, int n,
                                                        double* __restrict__ results) {
  const int i = blockIdx.x;
  if (i < n)
    reduce_set(partA + (size_t)i * stride, nbA, results + (size_t)i * 2 * kNumPartials);
  else
    reduce_set(partB, nbB, results + (size_t)(n - 1) * 2 * kNumPartials + kNumPartials);
}

// The split form, two launches (a kernel boundary orders them: no fences or counters, which on the
// eight-XCD chip cost a device-wide L2 write-back each -- the one-launch form with an arrival counter
// measured 93 us against 45 us for one workgroup per set): k_reduce_split's workgroup (set q, range
// r) reduces range r of set q into the scratch, k_reduce_combine sums the kRedSplit range results of
// each set in range order.  Sets: q < nA are slices of partA (stride apart), q = nA the set partB
// (when nbB >= 0).
constexpr int kRedLanes = 256;
__global__ void __launch_bounds__(kRedLanes) k_reduce_split(const double* __restrict__ partA, size_t stride, int nbA,
                                                            int nA, const double* __restrict__ partB, int nbB,
                                                            double* __restrict__ scratch) {
  __shared__ double red[kRedLanes / 64][kNumPartials];
  const int q = (int)blockIdx.x / kRedSplit, r = (int)blockIdx.x % kRedSplit;
  const bool isA = q < nA;
  const double* p = isA ? partA + (size_t)q * stride : partB;
  const int nb = isA ? nbA : nbB;
  const int per = (nb + kRedSplit - 1) / kRedSplit, lo = min(nb, r * per), hi = min(nb, lo + per);
  const int tid = (int)threadIdx.x;
  double acc[kNumPartials];
#pragma unroll
  for (int i = 0; i < kNumPartials; ++i) acc[i] = 0.0;
  for (int b = lo + tid; b < hi; b += kRedLanes)
#pragma unroll
    for (int i = 0; i < kNumPartials; ++i) {
      const double v = p[(size_t)b * kNumPartials + i];
      acc[i] = (i == 5) ? fmax(acc[i], v) : acc[i] + v;
    }
#pragma unroll
  for (int i = 0; i < kNumPartials; ++i) acc[i] = (i == 5) ? wave_max(acc[i]) : wave_sum(acc[i]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int i = 0; i < kNumPartials; ++i) red[tid >> 6][i] = acc[i];
  __syncthreads();
  if (tid < kNumPartials) {
    double v = red[0][tid];
    for (int w = 1; w < kRedLanes / 64; ++w) v = (tid == 5) ? fmax(v, red[w][tid]) : v + red[w][tid];
    scratch[(size_t)blockIdx.x * kNumPartials + tid] = v;
  }
}
__global__ void __launch_bounds__(64) k_reduce_combine(const double* __restrict__ scratch, int nA,
                                                       double* __restrict__ outA, size_t outStride,
                                                       double* __restrict__ outB) {
  const int q = (int)blockIdx.x, t = (int)threadIdx.x;
  if (t >= kNumPartials) return;
  const double* base = scratch + (size_t)q * kRedSplit * kNumPartials + t;
  double acc = base[0];
  for (int k = 1; k < kRedSplit; ++k) acc = (t == 5) ? fmax(acc, base[(size_t)k * kNumPartials]) : acc + base[(size_t)k * kNumPartials];
  (q < nA ? outA + (size_t)q * outStride : outB)[t] = acc;
}

__device__ void reduce_set(const double* __restrict__ partials, int nblocks, double* __restrict__ out) {
  // one workgroup of 1024: lane-strided sums in a fixed order (four rows requested at a time),
  // then the wavefront butterflies and the 16 wavefront results in order -- a fixed shape
  __shared__ double red[kRed / 64][kNumPartials];
  const int tid = threadIdx.x;
  double acc[kNumPartials];
#pragma unroll
  for (int i = 0; i < kNumPartials; ++i) acc[i] = 0.0;  // entry 5 (a max of counts >= 0) too
  int b = tid;
  for (; b + 3 * kRed < nblocks; b += 4 * kRed) {
    double v[4][kNumPartials];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kNumPartials; ++i) v[q][i] = partials[(size_t)(b + q * kRed) * kNumPartials + i];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kNumPartials; ++i) acc[i] = (i == 5) ? fmax(acc[i], v[q][i]) : acc[i] + v[q][i];
  }
  for (; b < nblocks; b += kRed)
#pragma unroll
    for (int i = 0; i < kNumPartials; ++i) {
      const double v = partials[(size_t)b * kNumPartials + i];
      acc[i] = (i == 5) ? fmax(acc[i], v) : acc[i] + v;
    }
#pragma unroll
  for (int i = 0; i < kNumPartials; ++i) acc[i] = (i == 5) ? wave_max(acc[i]) : wave_sum(acc[i]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int i = 0; i < kNumPartials; ++i) red[tid >> 6][i] = acc[i];
  __syncthreads();
  if (tid < kNumPartials) {
    double r = red[0][tid];
    for (int w = 1; w < kRed / 64; ++w) r = (tid == 5) ? fmax(r, red[w][tid]) : r + red[w][tid];
    out[tid] = r;
  }
}

// one-simplex evaluation for tests: Mesh::computeBlockGrad (regularised, FIXED rows zeroed)
template <int D>
__global__ void k_debug_blockgrad(DeviceMesh<D> m, int s, const double* __restrict__ zin,
                                  const double* __restrict__ dxin, double* __restrict__ out, int flags) {
  constexpr int K = D * (D + 1);
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int f[D + 1];
  loadVerts<D>(m, s, f);
  double z[K], dx[K], xi[K], g[K], Igt = 0;
  for (int i = 0; i < K; ++i) {
    z[i] = zin[i];
    dx[i] = dxin[i];
    g[i] = 0;
  }
  loadXi<D>(m, f, xi);
  double e;
  if (flags & 1) {
    e = (flags & 2) ? blockGrad<D, true, true>(gridOf<D>(m), constsOf<D>(m), z, xi, dx, g, Igt)
                    : blockGrad<D, true, false>(gridOf<D>(m), constsOf<D>(m), z, xi, dx, g, Igt);
    zeroFixed<D>(g, m.sbits[s] & 0xF);
  } else {
    e = (flags & 2) ? blockGrad<D, false, true>(gridOf<D>(m), constsOf<D>(m), z, xi, dx, g, Igt)
                    : blockGrad<D, false, false>(gridOf<D>(m), constsOf<D>(m), z, xi, dx, g, Igt);
  }
  out[0] = e;
  out[1] = Igt;
  for (int i = 0; i < K; ++i) out[2 + i] = g[i];
}

__global__ void k_devmath(int op, int n, const double* __restrict__ in, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (op == 5) {  // quotient pairs (x, c) -> RN(x/c) by div_mk (no range check here)
    if (2 * i + 1 < n) {
      const double xx = in[2 * i], c = in[2 * i + 1];
      out[i] = div_mk(xx, c, 1.0 / c);
    }
    return;
  }
  if (op == 10) {  // the double-double sqrt the powers use: pairs (s, e) for in[0 .. n/2)
    if (2 * i + 1 < n) {
      double sv, ev, hv;
      dd_sqrt_h(in[i], sv, ev, hv);
      out[2 * i] = sv;
      out[2 * i + 1] = ev;
    }
    return;
  }
  const double x = in[i];
  double r;
  bool tie = false;
  switch (op) {
    case 0: r = cr_sqrt(x); break;
    case 1: r = cr_pow_p15(x); break;
    case 2: r = cr_pow_m05(x); break;
    case 3: r = cr_pow_p225(x); break;
    case 4: r = cr_pow_p125(x); break;
    // the prox kernels' fast path (no tie resolution): NaN where it would defer to the exact path
    case 6: r = cr_pow_p15<false>(x, tie); break;
    case 7: r = cr_pow_m05<false>(x, tie); break;
    case 8: r = cr_pow_p225<false>(x, tie); break;
    default: r = cr_pow_p125<false>(x, tie); break;
  }
  out[i] = tie ? __builtin_nan("") : r;
}

// ---------------------------------------------------------------------------------------
static inline int nblk(int n) { return (n + kBlock - 1) / kBlock; }
// node kernels: grid padded to a multiple of the 8 XCDs, logical blocks dealt in contiguous runs
// per XCD (blocks b and b+8 share an XCD, MI355X_MICROARCH.md §Workgroup dispatch), so the z/u
// lines a run of nodes shares stay in one L2.  MMX_XCD_MAP=0 restores the identity mapping.
static int xcd_map() {
  static int v = [] {
    const char* e = getenv("MMX_XCD_MAP");
    return e ? atoi(e) : 1;
  }();
  return v;
}
static inline int nblk_xcd(int n) { return xcd_map() ? (nblk(n) + 7) / 8 * 8 : nblk(n); }

template <int D>
void launch_gather_z(const DeviceMesh<D>& m, const double* x, double* z, hipStream_t st) {
  if (m.nF == 0) return;
  hipLaunchKernelGGL(k_gather_z<D>, dim3(nblk(m.nF)), dim3(kBlock), 0, st, m, x, z);
}
template <int D>
void launch_grad_simplex(const DeviceMesh<D>& m, const double* x, double* gs, bool zeroFixedRows,
                         double* partials, int* nblocks, hipStream_t st) {
  *nblocks = nblk(m.nF);
  if (m.nF == 0) return;
  if (D == 3 && m.giso)
    hipLaunchKernelGGL((k_grad_simplex<D, 1>), dim3(*nblocks), dim3(kBlock), 0, st, m, x, gs,
                     zeroFixedRows ? 1 : 0, partials);
  else if (D == 3)
    hipLaunchKernelGGL((k_grad_simplex<D, 0>), dim3(*nblocks), dim3(kBlock), 0, st, m, x, gs,
                     zeroFixedRows ? 1 : 0, partials);
  else
    hipLaunchKernelGGL((k_grad_simplex<D, -1>), dim3(*nblocks), dim3(kBlock), 0, st, m, x, gs,
                     zeroFixedRows ? 1 : 0, partials);
}
template <int D>
void launch_predict(const DeviceMesh<D>& m, int mode, const double* gs, double* x, double* xPrev,
                    double* xBar, double dt_over_tau, hipStream_t st) {
  if (m.nP == 0) return;
  hipLaunchKernelGGL(k_predict<D>, dim3(nblk_xcd(m.nP)), dim3(kBlock), 0, st, m, mode, gs, x, xPrev, xBar,
                     dt_over_tau, xcd_map());
}
static bool xup_sweep_resid() {
  const char* e = getenv("MMX_XUP_SWEEP_RESID");
  return !(e && atoi(e) == 0);
}
template <int D>
void launch_xupdate(const DeviceMesh<D>& m, const StepScalars& sc, const double* xBar, const double* z,
                    const double* u, double* x, double* partials, int* nblocks, bool resid, hipStream_t st,
                    bool useTslot) {
  const int nsub = m.xupHi - m.xupLo;  // the launch's share of the node order
  *nblocks = nblk_xcd(nsub);
  if (nsub <= 0) {
    *nblocks = 0;
    return;
  }
  const bool ts = useTslot && m.tslot;
  const bool rem = m.remote != nullptr;
  if (m.zx && !resid && !ts) {  // a step's first x-update: z from DeviceMesh::zx
#define MMX_XU_ZX(P, R)                                                                                        \
  hipLaunchKernelGGL((k_xupdate<D, false, false, true, P, R>), dim3(*nblocks), dim3(kBlock), 0, st, m, sc, xBar, z, \
                     u, x, partials, xcd_map())
    if (m.predBar && rem)  // ... and predictX's extrapolation fused in
      MMX_XU_ZX(true, true);
    else if (m.predBar)
      MMX_XU_ZX(true, false);
    else if (rem)
      MMX_XU_ZX(false, true);
    else
      MMX_XU_ZX(false, false);
#undef MMX_XU_ZX
    return;
  }
  // the fused extrapolation exists only in the form above: a caller that set it for another form
  // would lose predictX silently
  if (m.predBar || m.predPrev)
    throw std::logic_error("launch_xupdate: predBar set for an x-update that cannot fuse predictX");
  // the sweep (persistent) form, MMX_XUP_SWEEP workgroups per CU; with the residual in the slot-term
  // form (3D): C4's last x-update of a step 0.334 -> ~0.17 ms (MMX_XUP_SWEEP_RESID=0: one node per lane)
  const bool sweepResid = resid && ts && xup_sweep_resid();
  if (m.xupSweep > 0 && (!resid || sweepResid)) {
    const int n8 = ((nsub + kBlock - 1) / kBlock + 7) / 8 * kBlock;  // = the node order's XCD groups
    const dim3 g(256 * m.xupSweep);
    if (sweepResid) {
      *nblocks = (int)g.x;
      hipLaunchKernelGGL((k_xupdate_sweep<D, true, 8, true>), g, dim3(kBlock), 0, st, m, sc, xBar, z, u, x, n8,
                         partials);
    } else if (ts && m.xupCh >= 24)
      hipLaunchKernelGGL((k_xupdate_sweep<D, true, 24>), g, dim3(kBlock), 0, st, m, sc, xBar, z, u, x, n8, nullptr);
    else if (ts && m.xupCh >= 16)
      hipLaunchKernelGGL((k_xupdate_sweep<D, true, 16>), g, dim3(kBlock), 0, st, m, sc, xBar, z, u, x, n8, nullptr);
    else if (ts)
      hipLaunchKernelGGL((k_xupdate_sweep<D, true, 8>), g, dim3(kBlock), 0, st, m, sc, xBar, z, u, x, n8, nullptr);
    else
      hipLaunchKernelGGL((k_xupdate_sweep<D, false, (D == 2 ? MMX_XU_CH2D : 8)>), g, dim3(kBlock), 0, st, m, sc, xBar,
                         z, u, x, n8, nullptr);
    return;
  }
#define MMX_XU(R, T)                                                                                               \
  hipLaunchKernelGGL((k_xupdate<D, R, T>), dim3(*nblocks), dim3(kBlock), 0, st, m, sc, xBar, z, u, x, partials, \
                     xcd_map())
  if (resid && ts)
    MMX_XU(true, true);
  else if (resid)
    MMX_XU(true, false);
  else if (ts)
    MMX_XU(false, true);
  else
    MMX_XU(false, false);
#undef MMX_XU
}
__global__ void __launch_bounds__(kBlock) k_pad_rows(const double* __restrict__ vals, long long rows,
                                                      double* __restrict__ pad) {
  const long long r = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (r >= rows) return;
  for (int n = 0; n < 9; ++n) pad[r * 10 + n] = vals[r * 9 + n];
  pad[r * 10 + 9] = 0.0;
}
template <int D>
__global__ void __launch_bounds__(kBlock) k_iso_compact(const double* __restrict__ vals, long long n,
                                                        double* __restrict__ iso, int* __restrict__ notIso) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double* v = vals + i * D * D;
  const unsigned long long d0 = __double_as_longlong(v[0]);
  bool ok = true, nan = true;
#pragma unroll
  for (int k = 0; k < D * D; ++k) {
    const unsigned long long b = __double_as_longlong(v[k]);
    ok = ok && (b == ((k / D == k % D) ? d0 : 0ull));
    nan = nan && (v[k] != v[k]);
  }
  if (!(ok || nan)) *notIso = 1;  // (every writer stores the same value)
  iso[i] = v[0];
}
template <int D>
void launch_iso_compact(const double* vals, long long points, double* iso, int* notIso, hipStream_t st) {
  if (points > 0)
    hipLaunchKernelGGL(k_iso_compact<D>, dim3((unsigned)((points + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, vals,
                       points, iso, notIso);
}
template void launch_iso_compact<2>(const double*, long long, double*, int*, hipStream_t);
template void launch_iso_compact<3>(const double*, long long, double*, int*, hipStream_t);

void launch_pad_rows(const double* vals, long long rows, double* pad, hipStream_t st) {
  if (rows > 0) hipLaunchKernelGGL(k_pad_rows, dim3((unsigned)((rows + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, vals, rows, pad);
}
// hessInvs = I (src/Mesh.cpp:456-464) on the device, in the layout of bidx<D> (the caller zeroes
// the buffer first): one lane per (simplex, diagonal entry)
template <int D>
__global__ void k_bkinv_identity(int nF, double* B) {
  constexpr int K = D * (D + 1);
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)nF * K) return;
  const int s = (int)(t / K), i = (int)(t % K);
  B[bidx<D>(s, i * K + i)] = 1.0;
}
template <int D>
void launch_bkinv_identity(int nF, double* B, hipStream_t st) {
  constexpr int K = D * (D + 1);
  const long long n = (long long)nF * K;
  if (n > 0) hipLaunchKernelGGL(k_bkinv_identity<D>, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, nF, B);
}
template void launch_bkinv_identity<2>(int, double*, hipStream_t);
template void launch_bkinv_identity<3>(int, double*, hipStream_t);
// reuse of the previous prox's last gradient at the prox entry (MMX_GRAD_CACHE=0 disables)
static int cache_enabled() {
  static int v = [] {
    const char* e = getenv("MMX_GRAD_CACHE");
    return e ? atoi(e) : 1;
  }();
  return v;
}
// workgroup size of the steady-state 2D prox (MMX_PROX_BLOCK = 64 | 128 | 256 overrides)
static int prox_block() {
  static int b = [] {
    const char* e = getenv("MMX_PROX_BLOCK");
    const int v = e ? atoi(e) : 0;
    return (v == 64 || v == 128 || v == 256) ? v : kProxBlock;
  }();
  return b;
}

// 3D steady-state prox kernel: k_prox_wave (one lane per tet, default: C4 2.77 ms) or k_prox_quad
// (four lanes per tet, MMX_PROX3D=quad: bit-identical, C4 3.92 ms -- DESIGN.md §3).  Read at every
// launch, so a test can switch kernels between steps.
// 2D steady-state prox kernel: k_prox_lds (default) or k_prox_wave<2> (DeviceMesh::prox2dWave, set
// from MMX_PROX2D=wave when the engine is built: one wave per workgroup, every Bkinv row held in
// LDS, double-buffered, rows written as the update forms them; measured slower)
bool prox_double_buffered(int D, bool wave2d) { return D == 3 || wave2d; }
bool prox2d_wave_requested() {
  const char* e = getenv("MMX_PROX2D");
  return e && std::string(e) == "wave";
}
static int prox3d_quad() {
  const char* e = getenv("MMX_PROX3D");
  return (e && std::string(e) == "quad") ? 1 : 0;
}
constexpr int kFixGrid = 256;  // workgroups of the exact (tie) recomputation: at most one per CU
#ifndef MMX_QUAD_TETS
#define MMX_QUAD_TETS 64
#endif
constexpr int kQuadTets = MMX_QUAD_TETS;  // tets per k_prox_quad workgroup (64: 4.03 ms at C4, 16: 4.37 ms)

#ifdef MMX_WAVE_PROF
static unsigned long long* g_wprofHost = nullptr;
static size_t g_wprofN = 0;
static void wprof_arm(int nblocks) {
  if (g_wprofN >= (size_t)nblocks * 8) return;
  if (g_wprofHost) (void)hipFree(g_wprofHost);
  g_wprofN = (size_t)nblocks * 8;
  (void)hipMalloc((void**)&g_wprofHost, g_wprofN * sizeof(unsigned long long));
  (void)hipMemset(g_wprofHost, 0, g_wprofN * sizeof(unsigned long long));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wprof), &g_wprofHost, sizeof(g_wprofHost));
}
#endif
template <int D>
void launch_prox(const DeviceMesh<D>& m, bool first, bool useCache, double tol, const double* x, double* z, double* u,
                 const double* Bin, double* Bout, double* partials, int* nblocks, hipStream_t st) {
#ifdef MMX_WAVE_PROF
  if (D == 3 && !first) wprof_arm((m.nF + 63) / 64);
#endif
  const int uc = (useCache && cache_enabled()) ? 1 : 0;
  *nblocks = nblk(m.nF);
  if (m.nF == 0) return;
  if (first) {
    if (D == 3 && m.giso)
      hipLaunchKernelGGL((k_prox<D, true, 1>), dim3(*nblocks), dim3(kBlock), 0, st, m, tol, x, z, u, Bin, Bout, partials, 0);
    else if (D == 3)
      hipLaunchKernelGGL((k_prox<D, true, 0>), dim3(*nblocks), dim3(kBlock), 0, st, m, tol, x, z, u, Bin, Bout, partials, 0);
    else
      hipLaunchKernelGGL((k_prox<D, true, -1>), dim3(*nblocks), dim3(kBlock), 0, st, m, tol, x, z, u, Bin, Bout, partials, 0);
  } else if (D == 2 && m.prox2dWave) {
    *nblocks = (m.nF + 63) / 64;
    const dim3 fg(std::min(*nblocks, kFixGrid));
    if (m.compMesh) {
      hipLaunchKernelGGL((k_prox_wave<D, true>), dim3(*nblocks), dim3(64), 0, st, m, tol, x, z, u, Bin, Bout, partials, uc);
      hipLaunchKernelGGL((k_prox_wave_fix<D, true>), fg, dim3(64), 0, st, m, tol, x, z, u, Bin, Bout, partials);
    } else {
      hipLaunchKernelGGL((k_prox_wave<D, false>), dim3(*nblocks), dim3(64), 0, st, m, tol, x, z, u, Bin, Bout, partials, uc);
      hipLaunchKernelGGL((k_prox_wave_fix<D, false>), fg, dim3(64), 0, st, m, tol, x, z, u, Bin, Bout, partials);
    }
  } else if constexpr (D == 2) {
    double* B = Bout;  // in place (LDS image)
    const int bs = prox_block();
    *nblocks = (m.nF + bs - 1) / bs;
    const dim3 fg(std::min(*nblocks, kFixGrid));
    if (bs == 64) {
      hipLaunchKernelGGL((k_prox_lds<D, 64>), dim3(*nblocks), dim3(64), 0, st, m, tol, x, z, u, B, partials, uc);
      hipLaunchKernelGGL((k_prox_fix<D, 64>), fg, dim3(64), 0, st, m, tol, x, z, u, B, B, partials);
    } else if (bs == 128) {
      hipLaunchKernelGGL((k_prox_lds<D, 128>), dim3(*nblocks), dim3(128), 0, st, m, tol, x, z, u, B, partials, uc);
      hipLaunchKernelGGL((k_prox_fix<D, 128>), fg, dim3(128), 0, st, m, tol, x, z, u, B, B, partials);
    } else {
      hipLaunchKernelGGL((k_prox_lds<D, 256>), dim3(*nblocks), dim3(256), 0, st, m, tol, x, z, u, B, partials, uc);
      hipLaunchKernelGGL((k_prox_fix<D, 256>), fg, dim3(256), 0, st, m, tol, x, z, u, B, B, partials);
    }
  } else {
    *nblocks = (m.nF + 63) / 64;
    const dim3 fg(std::min(*nblocks, kFixGrid));
    if (prox3d_quad()) {  // four lanes per tetrahedron, 16 per workgroup; the exact instance recomputes queued blocks
      *nblocks = (m.nF + kQuadTets - 1) / kQuadTets;
      const dim3 qg(std::min(*nblocks, kFixGrid));
      if (m.compMesh) {
        hipLaunchKernelGGL((k_prox_quad<true, false, 4 * kQuadTets>), dim3(*nblocks), dim3(4 * kQuadTets), 0, st, m,
                           tol, x, z, u, Bin, Bout, partials, uc);
        hipLaunchKernelGGL((k_prox_quad<true, true, 4 * kQuadTets>), qg, dim3(4 * kQuadTets), 0, st, m, tol, x, z, u,
                           Bin, Bout, partials, 0);
      } else {
        hipLaunchKernelGGL((k_prox_quad<false, false, 4 * kQuadTets>), dim3(*nblocks), dim3(4 * kQuadTets), 0, st, m,
                           tol, x, z, u, Bin, Bout, partials, uc);
        hipLaunchKernelGGL((k_prox_quad<false, true, 4 * kQuadTets>), qg, dim3(4 * kQuadTets), 0, st, m, tol, x, z, u,
                           Bin, Bout, partials, 0);
      }
      return;
    }
#define MMX_WAVE3(C, I)                                                                                            \
  do {                                                                                                           \
    hipLaunchKernelGGL((k_prox_wave<D, C, I>), dim3(MMX_WAVE_PERSIST ? (std::min(*nblocks, MMX_WAVE_PERSIST) + 7) / 8 * 8 : *nblocks), dim3(64), 0, st, m, tol, x, z, u, Bin, Bout, partials, uc); \
    hipLaunchKernelGGL((k_prox_wave_fix<D, C, I>), fg, dim3(64), 0, st, m, tol, x, z, u, Bin, Bout, partials);          \
  } while (0)
    if (m.compMesh) {
      if (m.giso) MMX_WAVE3(true, true); else MMX_WAVE3(true, false);
    } else {
      if (m.giso) MMX_WAVE3(false, true); else MMX_WAVE3(false, false);
    }
#undef MMX_WAVE3
  }
}
template <int D>
void launch_energy(const DeviceMesh<D>& m, const double* x, double* partials, int* nblocks, hipStream_t st) {
  *nblocks = nblk(m.nF);
  if (m.nF == 0) return;
  if (D == 3 && m.giso)
    hipLaunchKernelGGL((k_energy<D, 1>), dim3(*nblocks), dim3(kBlock), 0, st, m, x, partials);
  else if (D == 3)
    hipLaunchKernelGGL((k_energy<D, 0>), dim3(*nblocks), dim3(kBlock), 0, st, m, x, partials);
  else
    hipLaunchKernelGGL((k_energy<D, -1>), dim3(*nblocks), dim3(kBlock), 0, st, m, x, partials);
}
template <int D>
void launch_euler_apply(const DeviceMesh<D>& m, const double* gs, double* x, double dt_over_tau,
                        hipStream_t st) {
  if (m.nP == 0) return;
  hipLaunchKernelGGL(k_euler_apply<D>, dim3(nblk_xcd(m.nP)), dim3(kBlock), 0, st, m, gs, x, dt_over_tau, xcd_map());
}
// one workgroup per set reads its partials at ~0.1 TB/s (C3: 10 sets of 31 k prox partials took 45 us
// per step); the split form spreads each set over kRedSplit workgroups
// MMX_RED_SPLIT_MIN overrides kRedSplitMin (tests force the split form on small meshes)
static bool split_ok(const RedWork& w, int nblocks) {
  const char* e = getenv("MMX_RED_SPLIT_MIN");
  return w.scratch && nblocks >= (e ? atoi(e) : kRedSplitMin);
}
static void reduce_split(const double* partA, size_t stride, int nbA, int nA, double* outA, size_t outStride,
                         const double* partB, int nbB, double* outB, const RedWork& w, hipStream_t st) {
  const int sets = nA + (nbB >= 0 ? 1 : 0);
  hipLaunchKernelGGL(k_reduce_split, dim3(sets * kRedSplit), dim3(kRedLanes), 0, st, partA, stride, nbA, nA, partB,
                     nbB, w.scratch);
  hipLaunchKernelGGL(k_reduce_combine, dim3(sets), dim3(64), 0, st, w.scratch, nA, outA, outStride, outB);
}
void launch_reduce_partials(const double* partials, int nblocks, double* out, hipStream_t st, const RedWork& w) {
  if (split_ok(w, nblocks))
    reduce_split(partials, 0, nblocks, 1, out, 0, partials, -1, out, w, st);
  else
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kRed), 0, st, partials, nblocks, out, partials, nblocks, out);
}
void launch_reduce_steps(const double* partA, size_t stride, int nbA, const double* partB, int nbB, int n,
                         double* results, hipStream_t st, const RedWork& w) {
  if (split_ok(w, nbA) && n + 1 <= kRedSets)
    reduce_split(partA, stride, nbA, n, results, (size_t)2 * kNumPartials, partB, nbB,
                 results + (size_t)(n - 1) * 2 * kNumPartials + kNumPartials, w, st);
  else
    hipLaunchKernelGGL(k_reduce_steps, dim3(n + 1), dim3(kRed), 0, st, partA, stride, nbA, partB, nbB, n, results);
}
void launch_reduce_partials2(const double* partials, int nblocks, double* out, const double* partials2, int nblocks2,
                             double* out2, hipStream_t st, const RedWork& w) {
  if (split_ok(w, nblocks))
    reduce_split(partials, 0, nblocks, 1, out, 0, partials2, nblocks2, out2, w, st);
  else
    hipLaunchKernelGGL(k_reduce_partials, dim3(2), dim3(kRed), 0, st, partials, nblocks, out, partials2, nblocks2,
                       out2);
}
template <int D>
void launch_debug_blockgrad(const DeviceMesh<D>& m, int s, const double* z, const double* dx, double* out, int flags,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_debug_blockgrad<D>, dim3(1), dim3(64), 0, st, m, s, z, dx, out, flags);
}
template void launch_debug_blockgrad<2>(const DeviceMesh<2>&, int, const double*, const double*, double*, int,
                                        hipStream_t);
template void launch_debug_blockgrad<3>(const DeviceMesh<3>&, int, const double*, const double*, double*, int,
                                        hipStream_t);
template <int D>
void launch_pack_export(int mode, int nExp, const int* expOff, const double* z, const double* u, const double* gs,
                        double w, double* out, hipStream_t st, const PackZX& zx) {
  if (nExp <= 0) return;
  hipLaunchKernelGGL(k_pack_export<D>, dim3((nExp + kBlock - 1) / kBlock), dim3(kBlock), 0, st, mode, nExp, expOff, z, u,
                     gs, w, out, zx);
}
template void launch_pack_export<2>(int, int, const int*, const double*, const double*, const double*, double, double*,
                                    hipStream_t, const PackZX&);
template void launch_pack_export<3>(int, int, const int*, const double*, const double*, const double*, double, double*,
                                    hipStream_t, const PackZX&);

void launch_devmath(int op, int n, const double* in, double* out, hipStream_t st) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_devmath, dim3((n + 255) / 256), dim3(256), 0, st, op, n, in, out);
}

template <int D>
void launch_fd_jac(const DeviceMesh<D>& m, const double* Vp, double h, double* dv, hipStream_t st, unsigned* work) {
  const long long nt = (long long)m.nF * (D + 1);
  if (nt == 0) return;
  // the fix pass: one lane per possible queue entry (the queue's length is known on the device only;
  // lanes past it exit at once) -- the exact path is long, so every queued lane gets its own
  const dim3 gj((unsigned)((nt + kBlock - 1) / kBlock)), gf = gj;
  if (work) {  // fast pass + the exact recomputation of its queued lanes
    if (hipMemsetAsync(work, 0, sizeof(unsigned), st) != hipSuccess) throw std::runtime_error("launch_fd_jac: memset");
#define MMX_FDJ(I)                                                                                       \
  do {                                                                                                   \
    hipLaunchKernelGGL((k_fd_jac<D, I, false>), gj, dim3(kBlock), 0, st, m, Vp, h, dv, work);            \
    hipLaunchKernelGGL((k_fd_jac_fix<D, I>), gf, dim3(kBlock), 0, st, m, Vp, h, dv, (const unsigned*)work); \
  } while (0)
    if (D == 3 && m.giso)
      MMX_FDJ(1);
    else if (D == 3)
      MMX_FDJ(0);
    else
      MMX_FDJ(-1);
#undef MMX_FDJ
    return;
  }
  if (D == 3 && m.giso)
    hipLaunchKernelGGL((k_fd_jac<D, 1>), gj, dim3(kBlock), 0, st, m, Vp, h, dv, nullptr);
  else if (D == 3)
    hipLaunchKernelGGL((k_fd_jac<D, 0>), gj, dim3(kBlock), 0, st, m, Vp, h, dv, nullptr);
  else
    hipLaunchKernelGGL((k_fd_jac<D, -1>), gj, dim3(kBlock), 0, st, m, Vp, h, dv, nullptr);
}
template <int D>
void launch_jac_assemble(const DeviceMesh<D>& m, const int* ia, const int* ja, const double* dv, double dt_over_tau,
                         double* a, hipStream_t st, bool finish, int maxColNodes) {
  if (m.nP == 0) return;
  const char* ev = getenv("MMX_JAC_ASSEMBLE");  // "entry": the entry-outer form (once per assembly)
  const bool entryOuter = ev && std::string(ev) == "entry";
  if (entryOuter)
    hipLaunchKernelGGL(k_jac_assemble<D>, dim3(nblk(m.nP * D)), dim3(kBlock), 0, st, m, ia, ja, dv, dt_over_tau,
                       finish ? 1 : 0, a);
  else if (maxColNodes <= 64)
    hipLaunchKernelGGL(k_jac_assemble_w<D>, dim3((m.nP + 3) / 4), dim3(256), 0, st, m, ia, ja, dv, dt_over_tau,
                       finish ? 1 : 0, a);
  else
    hipLaunchKernelGGL(k_jac_assemble_s<D>, dim3(nblk(m.nP * D)), dim3(kBlock), 0, st, m, ia, ja, dv, dt_over_tau,
                       finish ? 1 : 0, a);
}
template <int D>
void launch_be_residual(const DeviceMesh<D>& m, const double* gs, const double* x, const double* xn,
                        double dt_over_tau, double* rhs, double* partials, int* nblocks, hipStream_t st) {
  *nblocks = nblk_xcd(m.nP);
  if (m.nP == 0) return;
  if (m.nodeOrder) {  // the node-ordered residual, then its partials in node-id order
    hipLaunchKernelGGL((k_be_residual<D, true>), dim3(*nblocks), dim3(kBlock), 0, st, m, gs, x, xn, dt_over_tau, rhs,
                       partials, xcd_map());
    hipLaunchKernelGGL(k_abs_partials<D>, dim3(*nblocks), dim3(kBlock), 0, st, m.nP, rhs, partials, xcd_map());
    return;
  }
  hipLaunchKernelGGL(k_be_residual<D>, dim3(*nblocks), dim3(kBlock), 0, st, m, gs, x, xn, dt_over_tau, rhs, partials,
                     xcd_map());
}
void launch_add_inplace(int n, double* x, const double* dx, hipStream_t st) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_add_inplace, dim3(nblk(n)), dim3(kBlock), 0, st, n, x, dx);
}

#define MMX_INST(D)                                                                                     \
  template void launch_gather_z<D>(const DeviceMesh<D>&, const double*, double*, hipStream_t);          \
  template void launch_grad_simplex<D>(const DeviceMesh<D>&, const double*, double*, bool, double*, int*, \
                                       hipStream_t);                                                    \
  template void launch_predict<D>(const DeviceMesh<D>&, int, const double*, double*, double*, double*,   \
                                  double, hipStream_t);                                                 \
  template void launch_xupdate<D>(const DeviceMesh<D>&, const StepScalars&, const double*, const double*, \
                                  const double*, double*, double*, int*, bool, hipStream_t, bool);      \
  template void launch_prox<D>(const DeviceMesh<D>&, bool, bool, double, const double*, double*, double*,      \
                               const double*,                                                                \
                               double*, double*, int*, hipStream_t);                                    \
  template void launch_energy<D>(const DeviceMesh<D>&, const double*, double*, int*, hipStream_t);       \
  template void launch_euler_apply<D>(const DeviceMesh<D>&, const double*, double*, double, hipStream_t);     \
  template void launch_fd_jac<D>(const DeviceMesh<D>&, const double*, double, double*, hipStream_t, unsigned*);          \
  template void launch_jac_assemble<D>(const DeviceMesh<D>&, const int*, const int*, const double*, double,   \
                                       double*, hipStream_t, bool, int);                                                 \
  template void launch_be_residual<D>(const DeviceMesh<D>&, const double*, const double*, const double*,      \
                                      double, double*, double*, int*, hipStream_t);
MMX_INST(2)
MMX_INST(3)

}  // namespace mmx

#ifdef MMX_WAVE_PROF
// the probe's stamps of the last 3D steady prox launch: 8 per block, written to `path` (binary)
extern "C" int mmx_wprof_dump(const char* path) {
  if (!mmx::g_wprofHost) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  std::vector<unsigned long long> h(mmx::g_wprofN);
  if (hipMemcpy(h.data(), mmx::g_wprofHost, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return -3;
  FILE* f = fopen(path, "wb");
  if (!f) return -4;
  fwrite(h.data(), 8, h.size(), f);
  fclose(f);
  return (int)(h.size() / 8);
}
#endif

// the layout word this kernel object was compiled with (layout.h; checked by the host at create)
extern "C" unsigned mmx_layout_admm(void) { return mmx::kLayoutWord; }
