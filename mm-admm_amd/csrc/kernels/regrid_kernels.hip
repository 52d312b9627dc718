// regrid_kernels.hip -- the monitor-grid set-up on the device, for time-varying monitors
// (SURVEY §8f-2): the reference's commented Mesh<D>::setUp hook (src/Mesh.cpp:1006-1014) would
// re-run MeshInterpolator::updateMesh + interpolateMonitor (src/MeshInterpolator.cpp:68-130,
// 166-259, 366-404) at the start of every step.  Here that is: bounding box of the current
// vertices, monitor at the vertices, nearest vertex of every grid point, Jacobi smoothing --
// all on the device, bit-identical to the host set-up (csrc/host/monitor_grid.cpp):
//   * the nearest vertex is exact: vertices are binned into a uniform cell grid, a grid point
//     searches Chebyshev rings of cells until no unvisited cell can hold a vertex as near as the
//     best one, with the host's squared-distance sums and lowest-id tie rule;
//   * min/max and the smoothing stencil are order-independent / written in the host's order.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "regrid_kernels.h"

namespace mmx {
namespace {

constexpr int kRB = 256;

template <int D>
__global__ void __launch_bounds__(kRB) k_bbox(const double* __restrict__ X, int n, double* __restrict__ part) {
  __shared__ double sm[2 * D][kRB];
  double lo[D], hi[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    lo[d] = INFINITY;
    hi[d] = -INFINITY;
  }
  for (int v = blockIdx.x * kRB + threadIdx.x; v < n; v += gridDim.x * kRB)
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const double x = X[(size_t)v * D + d];
      lo[d] = x < lo[d] ? x : lo[d];
      hi[d] = x > hi[d] ? x : hi[d];
    }
#pragma unroll
  for (int d = 0; d < D; ++d) {
    sm[d][threadIdx.x] = lo[d];
    sm[D + d][threadIdx.x] = hi[d];
  }
  __syncthreads();
  for (int w = kRB / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const double a = sm[d][threadIdx.x + w], b = sm[D + d][threadIdx.x + w];
        sm[d][threadIdx.x] = a < sm[d][threadIdx.x] ? a : sm[d][threadIdx.x];
        sm[D + d][threadIdx.x] = b > sm[D + d][threadIdx.x] ? b : sm[D + d][threadIdx.x];
      }
    __syncthreads();
  }
  if (threadIdx.x < 2 * D) part[(size_t)blockIdx.x * 2 * D + threadIdx.x] = sm[threadIdx.x][0];
}

// the widest simplex per axis (max over simplices of max - min of its vertices' coordinate):
// the partitioned regrid's margin, re-measured from the current positions at every rebuild
template <int D>
__global__ void __launch_bounds__(kRB) k_extent(const double* __restrict__ X, const int* __restrict__ F, int nF,
                                                double* __restrict__ part) {
  __shared__ double sm[D][kRB];
  double ext[D];
#pragma unroll
  for (int d = 0; d < D; ++d) ext[d] = 0.0;
  for (int s = blockIdx.x * kRB + threadIdx.x; s < nF; s += gridDim.x * kRB) {
    int v[D + 1];
#pragma unroll
    for (int n = 0; n <= D; ++n) v[n] = F[(size_t)s * (D + 1) + n];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      double a = X[(size_t)v[0] * D + d], b = a;
#pragma unroll
      for (int n = 1; n <= D; ++n) {
        const double c = X[(size_t)v[n] * D + d];
        a = c < a ? c : a;
        b = c > b ? c : b;
      }
      const double e = b - a;
      ext[d] = e > ext[d] ? e : ext[d];
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) sm[d][threadIdx.x] = ext[d];
  __syncthreads();
  for (int w = kRB / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const double a = sm[d][threadIdx.x + w];
        sm[d][threadIdx.x] = a > sm[d][threadIdx.x] ? a : sm[d][threadIdx.x];
      }
    __syncthreads();
  }
  if (threadIdx.x < D) part[(size_t)blockIdx.x * D + threadIdx.x] = sm[threadIdx.x][0];
}

template <int D>
__device__ __forceinline__ int cellOf(const double* x, const CellGrid& cg, int (&c)[3]) {
  int id = 0;
#pragma unroll
  for (int d = D - 1; d >= 0; --d) {
    int k = (int)((x[d] - cg.lo[d]) * cg.inv[d]);
    k = k < 0 ? 0 : (k >= cg.n[d] ? cg.n[d] - 1 : k);
    c[d] = k;
    id = id * cg.n[d] + k;
  }
  return id;  // x fastest
}

template <int D>
__global__ void __launch_bounds__(kRB) k_bin_count(const double* __restrict__ X, int n, CellGrid cg,
                                                   int* __restrict__ cellOfV, int* __restrict__ counts) {
  const int v = blockIdx.x * kRB + threadIdx.x;
  if (v >= n) return;
  double x[D];
#pragma unroll
  for (int d = 0; d < D; ++d) x[d] = X[(size_t)v * D + d];
  int c[3];
  const int id = cellOf<D>(x, cg, c);
  cellOfV[v] = id;
  atomicAdd(&counts[id], 1);
}

__global__ void __launch_bounds__(kRB) k_bin_fill(int n, const int* __restrict__ cellOfV,
                                                  const int* __restrict__ starts, int* __restrict__ fill,
                                                  int* __restrict__ cellNodes) {
  const int v = blockIdx.x * kRB + threadIdx.x;
  if (v >= n) return;
  const int c = cellOfV[v];
  cellNodes[starts[c] + atomicAdd(&fill[c], 1)] = v;
}

// MonType 7 (time-varying moving bump): M = (1 + 5 / (1 + 50 |x - c(t)|^2)) I, c(t) from the host
template <int D>
__global__ void __launch_bounds__(kRB) k_monitor_tv(const double* __restrict__ X, int n, double c0, double c1,
                                                    double c2, double* __restrict__ monVals) {
  const int v = blockIdx.x * kRB + threadIdx.x;
  if (v >= n) return;
  const double c[3] = {c0, c1, c2};
  double sq = 0.0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const double t = X[(size_t)v * D + d] - c[d];
    sq = (d == 0) ? t * t : sq + t * t;
  }
  const double s = 1 + 5.0 / (1 + 50.0 * sq);
#pragma unroll
  for (int i = 0; i < D * D; ++i) monVals[(size_t)v * D * D + i] = (i / D == i % D) ? s : 0.0;
}

// storage coordinates (sx, sy, k) of the p-th row of a box, and the row
__device__ __forceinline__ size_t box_row(const GridBox& b, long long p, int nx, int ny, int& sx, int& sy, int& sk) {
  const long long bx = b.hi[0] - b.lo[0] + 1, by = b.hi[1] - b.lo[1] + 1;
  sx = b.lo[0] + (int)(p % bx);
  sy = b.lo[1] + (int)((p / bx) % by);
  sk = b.lo[2] + (int)(p / (bx * by));
  return ((size_t)sk * (ny + 1) + sy) * (nx + 1) + sx;
}
__device__ __forceinline__ long long box_rows(const GridBox& b) {
  return (long long)(b.hi[0] - b.lo[0] + 1) * (b.hi[1] - b.lo[1] + 1) * (b.hi[2] - b.lo[2] + 1);
}

// nearest vertex of the grid point of every row of the box; the row takes that vertex's monitor
// value.  Rows are enumerated in storage order (coalesced writes); the row's grid point follows
// the host set-up's layout: 2D row j(nx+1) + i holds point (i, j); 3D row (nx+1)(ny+1)k + i(nx+1) + j
// holds point (i, j, k) (src/MeshInterpolator.cpp:234: x and y swapped), i.e. storage (sx, sy) is
// point (sy, sx).
// Candidates restricted to a search box S (partitioned regrid, cand != nullptr): vertices are
// compared by their global ids cand->gid (the host's lowest-id tie rule), and every grid point
// checks that its nearest candidate is strictly nearer than the boundary of S -- no vertex outside
// S (which this rank does not hold) can then be as near; otherwise *cand->fail is set and the
// caller rebuilds from every vertex.
template <int D>
__global__ void __launch_bounds__(kRB) k_nn_fill(const double* __restrict__ X, CellGrid cg,
                                                 const int* __restrict__ starts, const int* __restrict__ cellNodes,
                                                 const double* __restrict__ gx, const double* __restrict__ gy,
                                                 const double* __restrict__ gz, int nx, int ny, int nz,
                                                 const double* __restrict__ monVals, double* __restrict__ vals,
                                                 GridBox box, NnCand cand) {
  constexpr int DD = D * D;
  const long long p = (long long)blockIdx.x * kRB + threadIdx.x;
  if (p >= box_rows(box)) return;
  int sx, sy, k;
  const size_t row = box_row(box, p, nx, ny, sx, sy, k);
  const int i = (D == 2) ? sx : sy, j = (D == 2) ? sy : sx;
  double q[3] = {gx[i], gy[j], D == 3 ? gz[k] : 0.0};
  int c[3] = {0, 0, 0};
  cellOf<D>(q, cg, c);
  double best = INFINITY;
  int bi = -1, bg = -1;  // nearest candidate: index, global id (tie rule)
  int rmax = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) rmax = max(rmax, max(c[d], cg.n[d] - 1 - c[d]));
  for (int r = 0; r <= rmax; ++r) {
    const int z0 = (D == 3) ? max(c[2] - r, 0) : 0, z1 = (D == 3) ? min(c[2] + r, cg.n[2] - 1) : 0;
    const int y0 = max(c[1] - r, 0), y1 = min(c[1] + r, cg.n[1] - 1);
    const int x0 = max(c[0] - r, 0), x1 = min(c[0] + r, cg.n[0] - 1);
    for (int cz = z0; cz <= z1; ++cz)
      for (int cy = y0; cy <= y1; ++cy)
        for (int cx = x0; cx <= x1; ++cx) {
          const int dz = (D == 3) ? abs(cz - c[2]) : 0;
          if (max(max(abs(cx - c[0]), abs(cy - c[1])), dz) != r) continue;  // ring r only
          const int cell = (cz * cg.n[1] + cy) * cg.n[0] + cx;
          for (int t = starts[cell]; t < starts[cell + 1]; ++t) {
            const int v = cellNodes[t];
            const int gv = cand.gid ? cand.gid[v] : v;
            double dd = 0.0;
#pragma unroll
            for (int d = 0; d < D; ++d) {
              const double df = q[d] - X[(size_t)v * D + d];
              dd += df * df;
            }
            if (dd < best || (dd == best && gv < bg)) {
              best = dd;
              bi = v;
              bg = gv;
            }
          }
        }
    // every unvisited vertex lies >= r cells away along some axis: at distance >= r * h_min
    // (less a margin for the binning's rounding); stop once the best is strictly nearer
    const double lb = ((double)r - 1e-6) * cg.hmin;
    if (bi >= 0 && r > 0 && best < lb * lb) break;
  }
  if (cand.gid) {
    double gap = INFINITY;  // distance from q to the outside of the search box
#pragma unroll
    for (int d = 0; d < D; ++d) gap = fmin(gap, fmin(q[d] - cand.slo[d], cand.shi[d] - q[d]));
    if (!(bi >= 0 && gap > 0.0 && best < gap * gap * (1.0 - 1e-9))) {
      atomicOr(cand.fail, 1);
      if (bi < 0) return;
    }
  }
#pragma unroll
  for (int e = 0; e < DD; ++e) vals[row * DD + e] = monVals[(size_t)bi * DD + e];
}

// partitioned regrid: this rank's owned vertices inside another rank's search box S_q are appended
// (position, global id) to the send block of rank q (rows of D + 1 doubles at q * cap)
template <int D>
__global__ void __launch_bounds__(kRB) k_select_owned(const double* __restrict__ X, const int* __restrict__ ownLocal,
                                                      const int* __restrict__ ownGid, int nOwned, int nranks, int rank,
                                                      const double* __restrict__ sboxes, int* __restrict__ counts,
                                                      double* __restrict__ send, int cap) {
  const int i = blockIdx.x * kRB + threadIdx.x;
  if (i >= nOwned) return;
  const int v = ownLocal[i];
  double x[D];
#pragma unroll
  for (int d = 0; d < D; ++d) x[d] = X[(size_t)v * D + d];
  for (int q = 0; q < nranks; ++q) {
    if (q == rank) continue;
    const double* s = sboxes + (size_t)q * 2 * D;
    bool in = true;
#pragma unroll
    for (int d = 0; d < D; ++d) in = in && x[d] >= s[d] && x[d] <= s[D + d];
    if (in) {
      const int k = atomicAdd(&counts[q], 1);
      double* r = send + ((size_t)q * cap + k) * (D + 1);
#pragma unroll
      for (int d = 0; d < D; ++d) r[d] = x[d];
      r[D] = (double)ownGid[i];
    }
  }
}

// the candidates: this rank's vertices (positions, global ids) then the received rows
template <int D>
__global__ void __launch_bounds__(kRB) k_build_cand(const double* __restrict__ X, const int* __restrict__ gidLocal,
                                                    int nLocal, const double* __restrict__ recv, int nRecv,
                                                    double* __restrict__ cx, int* __restrict__ cgid) {
  const int i = blockIdx.x * kRB + threadIdx.x;
  if (i >= nLocal + nRecv) return;
  if (i < nLocal) {
#pragma unroll
    for (int d = 0; d < D; ++d) cx[(size_t)i * D + d] = X[(size_t)i * D + d];
    cgid[i] = gidLocal[i];
  } else {
    const double* r = recv + (size_t)(i - nLocal) * (D + 1);
#pragma unroll
    for (int d = 0; d < D; ++d) cx[(size_t)i * D + d] = r[d];
    cgid[i] = (int)r[D];
  }
}

// smoothMonitorGrid (src/MeshInterpolator.cpp:366-404): one Jacobi pass, interior points
template <int D>
__global__ void __launch_bounds__(kRB) k_smooth(const double* __restrict__ in, double* __restrict__ out, int nx,
                                                int ny, int nz, GridBox box) {
  constexpr int DD = D * D;
  const long long p = (long long)blockIdx.x * kRB + threadIdx.x;
  const long long P = (long long)(nx + 1) * (ny + 1);
  if (p >= box_rows(box)) return;
  int i, j, k;
  const long long c = (long long)box_row(box, p, nx, ny, i, j, k);
  const bool interior = i >= 1 && i < nx && j >= 1 && j < ny && (D == 2 || (k >= 1 && k < nz));
  for (int q = 0; q < DD; ++q) {
    double v;
    if (!interior) {
      v = in[c * DD + q];
    } else if constexpr (D == 2) {
      v = 0.6 * in[c * DD + q];
      v += 0.1 * in[(c + 1) * DD + q];
      v += 0.1 * in[(c - 1) * DD + q];
      v += 0.1 * in[(c + nx + 1) * DD + q];
      v += 0.1 * in[(c - nx - 1) * DD + q];
    } else {
      const double h = 0.4 / 6.0;
      v = 0.6 * in[c * DD + q] + h * in[(c + 1) * DD + q] + h * in[(c - 1) * DD + q] + h * in[(c + nx + 1) * DD + q] +
          h * in[(c - nx - 1) * DD + q] + h * in[(c + P) * DD + q] + h * in[(c - P) * DD + q];
    }
    out[c * DD + q] = v;
  }
}

template <int D>
__global__ void __launch_bounds__(kRB) k_box_commit(const double* __restrict__ src, double* __restrict__ vals,
                                                    double* __restrict__ pad, int nx, int ny, int nz, GridBox box) {
  constexpr int DD = D * D;
  const long long c = (long long)blockIdx.x * kRB + threadIdx.x;
  const long long P = (long long)(nx + 1) * (ny + 1);
  if (c >= P * (D == 3 ? nz + 1 : 1)) return;
  const int i = (int)(c % (nx + 1)), j = (int)((c / (nx + 1)) % (ny + 1)), k = (D == 3) ? (int)(c / P) : 0;
  const bool in = i >= box.lo[0] && i <= box.hi[0] && j >= box.lo[1] && j <= box.hi[1] && k >= box.lo[2] &&
                  k <= box.hi[2];
  const double nan = __builtin_nan("");
  for (int q = 0; q < DD; ++q) vals[c * DD + q] = in ? src[c * DD + q] : nan;
  if (D == 3 && pad) {
    for (int q = 0; q < DD; ++q) pad[c * 10 + q] = in ? src[c * DD + q] : nan;
    pad[c * 10 + 9] = 0.0;
  }
}

// partitioned regrid: rows of D doubles gathered by index (pack a rank's owned vertices) or
// scattered by index (place every rank's vertices at their global ids; idx < 0 = padding)
__global__ void __launch_bounds__(kRB) k_rows_gather(int D, const int* __restrict__ idx, int n,
                                                     const double* __restrict__ in, double* __restrict__ out) {
  const int i = blockIdx.x * kRB + threadIdx.x;
  if (i >= n) return;
  for (int c = 0; c < D; ++c) out[(size_t)i * D + c] = in[(size_t)idx[i] * D + c];
}
__global__ void __launch_bounds__(kRB) k_rows_scatter(int D, const int* __restrict__ idx, int n,
                                                      const double* __restrict__ in, double* __restrict__ out) {
  const int i = blockIdx.x * kRB + threadIdx.x;
  if (i >= n || idx[i] < 0) return;
  for (int c = 0; c < D; ++c) out[(size_t)idx[i] * D + c] = in[(size_t)i * D + c];
}

inline unsigned blocks(long long n) { return (unsigned)((n + kRB - 1) / kRB); }

}  // namespace

template <int D>
void launch_bbox(const double* X, int n, double* partials, int nblocks, hipStream_t st) {
  hipLaunchKernelGGL(k_bbox<D>, dim3(nblocks), dim3(kRB), 0, st, X, n, partials);
}

template <int D>
void launch_extent(const double* X, const int* F, int nF, double* partials, int nblocks, hipStream_t st) {
  hipLaunchKernelGGL(k_extent<D>, dim3(nblocks), dim3(kRB), 0, st, X, F, nF, partials);
}

template <int D>
void launch_bin(const double* X, int n, const CellGrid& cg, int* cellOfV, int* counts, int* starts, int* fill,
                int* cellNodes, void* scanTmp, size_t scanTmpBytes, hipStream_t st) {
  const int ncell = cg.n[0] * cg.n[1] * cg.n[2];
  (void)hipMemsetAsync(counts, 0, sizeof(int) * (ncell + 1), st);
  (void)hipMemsetAsync(fill, 0, sizeof(int) * ncell, st);
  hipLaunchKernelGGL(k_bin_count<D>, dim3(blocks(n)), dim3(kRB), 0, st, X, n, cg, cellOfV, counts);
  size_t bytes = scanTmpBytes;
  (void)hipcub::DeviceScan::ExclusiveSum(scanTmp, bytes, counts, starts, ncell + 1, st);
  hipLaunchKernelGGL(k_bin_fill, dim3(blocks(n)), dim3(kRB), 0, st, n, cellOfV, starts, fill, cellNodes);
}

size_t bin_scan_bytes(int ncell) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (int*)nullptr, (int*)nullptr, ncell + 1, (hipStream_t)0);
  return bytes;
}

template <int D>
void launch_monitor_tv(const double* X, int n, const double* c, double* monVals, hipStream_t st) {
  hipLaunchKernelGGL(k_monitor_tv<D>, dim3(blocks(n)), dim3(kRB), 0, st, X, n, c[0], c[1], c[2], monVals);
}

static long long host_box_rows(const GridBox& b) {
  return (long long)(b.hi[0] - b.lo[0] + 1) * (b.hi[1] - b.lo[1] + 1) * (b.hi[2] - b.lo[2] + 1);
}

template <int D>
void launch_nn_fill(const double* X, const CellGrid& cg, const int* starts, const int* cellNodes, const double* gx,
                    const double* gy, const double* gz, int nx, int ny, int nz, const double* monVals, double* vals,
                    const GridBox& box, hipStream_t st, const NnCand& cand) {
  const long long n = host_box_rows(box);
  if (n > 0)
    hipLaunchKernelGGL(k_nn_fill<D>, dim3(blocks(n)), dim3(kRB), 0, st, X, cg, starts, cellNodes, gx, gy, gz, nx, ny,
                       nz, monVals, vals, box, cand);
}

template <int D>
void launch_select_owned(const double* X, const int* ownLocal, const int* ownGid, int nOwned, int nranks, int rank,
                         const double* sboxes, int* counts, double* send, int cap, hipStream_t st) {
  if (nOwned > 0)
    hipLaunchKernelGGL(k_select_owned<D>, dim3(blocks(nOwned)), dim3(kRB), 0, st, X, ownLocal, ownGid, nOwned, nranks,
                       rank, sboxes, counts, send, cap);
}

template <int D>
void launch_build_cand(const double* X, const int* gidLocal, int nLocal, const double* recv, int nRecv, double* cx,
                       int* cgid, hipStream_t st) {
  if (nLocal + nRecv > 0)
    hipLaunchKernelGGL(k_build_cand<D>, dim3(blocks(nLocal + nRecv)), dim3(kRB), 0, st, X, gidLocal, nLocal, recv,
                       nRecv, cx, cgid);
}

template <int D>
void launch_smooth(const double* in, double* out, int nx, int ny, int nz, const GridBox& box, hipStream_t st) {
  const long long n = host_box_rows(box);
  if (n > 0) hipLaunchKernelGGL(k_smooth<D>, dim3(blocks(n)), dim3(kRB), 0, st, in, out, nx, ny, nz, box);
}

template <int D>
void launch_box_commit(const double* src, double* vals, double* pad, int nx, int ny, int nz, const GridBox& box,
                       hipStream_t st) {
  const long long rows = (long long)(nx + 1) * (ny + 1) * (D == 3 ? nz + 1 : 1);
  hipLaunchKernelGGL(k_box_commit<D>, dim3(blocks(rows)), dim3(kRB), 0, st, src, vals, pad, nx, ny, nz, box);
}

void launch_rows_gather(int D, const int* idx, int n, const double* in, double* out, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_rows_gather, dim3(blocks(n)), dim3(kRB), 0, st, D, idx, n, in, out);
}
void launch_rows_scatter(int D, const int* idx, int n, const double* in, double* out, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_rows_scatter, dim3(blocks(n)), dim3(kRB), 0, st, D, idx, n, in, out);
}

#define MMX_REGRID_INST(D)                                                                                       \
  template void launch_bbox<D>(const double*, int, double*, int, hipStream_t);                                 \
  template void launch_extent<D>(const double*, const int*, int, double*, int, hipStream_t);                    \
  template void launch_bin<D>(const double*, int, const CellGrid&, int*, int*, int*, int*, int*, void*, size_t, \
                              hipStream_t);                                                                    \
  template void launch_monitor_tv<D>(const double*, int, const double*, double*, hipStream_t);                  \
  template void launch_nn_fill<D>(const double*, const CellGrid&, const int*, const int*, const double*,        \
                                  const double*, const double*, int, int, int, const double*, double*,          \
                                  const GridBox&, hipStream_t, const NnCand&);                                 \
  template void launch_select_owned<D>(const double*, const int*, const int*, int, int, int, const double*, int*, \
                                       double*, int, hipStream_t);                                               \
  template void launch_build_cand<D>(const double*, const int*, int, const double*, int, double*, int*,          \
                                     hipStream_t);                                                               \
  template void launch_smooth<D>(const double*, double*, int, int, int, const GridBox&, hipStream_t);           \
  template void launch_box_commit<D>(const double*, double*, double*, int, int, int, const GridBox&, hipStream_t);
MMX_REGRID_INST(2)
MMX_REGRID_INST(3)
#undef MMX_REGRID_INST

}  // namespace mmx
