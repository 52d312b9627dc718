// monitor_grid.cpp -- set-up of the smoothed monitor grid the hot path interpolates.
//
// MeshInterpolator<D>::updateMesh + interpolateMonitor (src/MeshInterpolator.cpp:68-130,
// 244-259): grid size (int)pow(nP*D, 1/D) over the initial mesh bounding box, monitor at
// every vertex, nearest vertex per grid point, then Jacobi smoothing (5 passes 2D, 2 passes
// 3D; 366-404).  The reference's nanoflann kNN(k=1) is replaced by an exact bucket-grid
// search; ties between equidistant vertices resolve to the lowest vertex id.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "common.h"

namespace mmx {
namespace {

void linspace(double xa, double xb, int ns, std::vector<double>& x) {  // src/MeshUtils.h:24-29
  x.resize(ns + 1);
  for (int i = 0; i < ns + 1; i++) x[i] = xa + ((double)i) * (xb - xa) / ns;
}

template <int D>
class BucketNN {
 public:
  BucketNN(const double* X, int n) : X_(X), n_(n) {
    double hi[3];
    for (int d = 0; d < D; ++d) {
      lo_[d] = INFINITY;
      hi[d] = -INFINITY;
    }
    for (int i = 0; i < n; ++i)
      for (int d = 0; d < D; ++d) {
        lo_[d] = std::min(lo_[d], X[(size_t)i * D + d]);
        hi[d] = std::max(hi[d], X[(size_t)i * D + d]);
      }
    const double per = (D == 2) ? std::sqrt((double)n / 2.0) : std::cbrt((double)n / 2.0);
    long tot = 1;
    for (int d = 0; d < D; ++d) {
      nb_[d] = std::max(1, (int)per);
      h_[d] = (hi[d] - lo_[d]) / nb_[d];
      if (!(h_[d] > 0)) h_[d] = 1.0;
      tot *= nb_[d];
    }
    start_.assign(tot + 1, 0);
    std::vector<int> cell(n);
    for (int i = 0; i < n; ++i) {
      cell[i] = cellOf(&X[(size_t)i * D]);
      start_[cell[i] + 1]++;
    }
    for (long c = 0; c < tot; ++c) start_[c + 1] += start_[c];
    items_.resize(n);
    std::vector<int> fill(start_.begin(), start_.end() - 1);
    for (int i = 0; i < n; ++i) items_[fill[cell[i]]++] = i;
  }

  int nearest(const double* q) const {
    int c[3] = {0, 0, 0};
    for (int d = 0; d < D; ++d) c[d] = coord(q[d], d);
    double best = INFINITY;
    int bi = -1;
    const int maxr = std::max(nb_[0], std::max(nb_[1], D == 3 ? nb_[2] : 1));
    for (int r = 0; r <= maxr; ++r) {
      const int zr = (D == 3) ? r : 0;
      for (int dz = -zr; dz <= zr; ++dz)
        for (int dy = -r; dy <= r; ++dy)
          for (int dx = -r; dx <= r; ++dx) {
            if (std::max(std::abs(dx), std::max(std::abs(dy), std::abs(dz))) != r) continue;
            const int cx = c[0] + dx, cy = c[1] + dy, cz = (D == 3) ? c[2] + dz : 0;
            if (cx < 0 || cx >= nb_[0] || cy < 0 || cy >= nb_[1]) continue;
            if (D == 3 && (cz < 0 || cz >= nb_[2])) continue;
            const long cell = cx + (long)nb_[0] * (cy + (long)nb_[1] * cz);
            for (int t = start_[cell]; t < start_[cell + 1]; ++t) {
              const int i = items_[t];
              double dd = 0.0;  // nanoflann L2_Simple_Adaptor: sum of squared differences
              for (int d = 0; d < D; ++d) {
                const double df = q[d] - X_[(size_t)i * D + d];
                dd += df * df;
              }
              if (dd < best || (dd == best && i < bi)) {
                best = dd;
                bi = i;
              }
            }
          }
      double guard = INFINITY;  // distance from q to the unsearched region
      for (int d = 0; d < D; ++d) {
        if (c[d] - r > 0) guard = std::min(guard, q[d] - (lo_[d] + (c[d] - r) * h_[d]));
        if (c[d] + r + 1 < nb_[d]) guard = std::min(guard, (lo_[d] + (c[d] + r + 1) * h_[d]) - q[d]);
      }
      if (bi >= 0) {
        if (guard == INFINITY) break;
        const double g = guard * (1.0 - 1e-9);
        if (g > 0 && best < g * g) break;
      }
    }
    return bi;
  }

 private:
  int coord(double v, int d) const {
    const int c = (int)std::floor((v - lo_[d]) / h_[d]);
    return std::min(std::max(c, 0), nb_[d] - 1);
  }
  int cellOf(const double* p) const {
    int c = 0, mul = 1;
    for (int d = 0; d < D; ++d) {
      c += coord(p[d], d) * mul;
      mul *= nb_[d];
    }
    return c;
  }
  const double* X_;
  int n_;
  double lo_[3], h_[3];
  int nb_[3];
  std::vector<int> start_, items_;
};

template <int D>
void buildGrid(const double* X, int nP, mmadmm_monitor_fn fn, void* user, HostGrid& g) {
  constexpr int DD = D * D;
  const int sz = (int)std::pow((double)((long)nP * D), 1.0 / D);  // src/MeshInterpolator.cpp:78-84
  g.nx = sz;
  g.ny = sz;
  g.nz = (D == 2) ? 1 : sz;
  double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < nP; i++)
    for (int d = 0; d < D; ++d) {
      const double v = X[(size_t)i * D + d];
      mn[d] = (v < mn[d]) ? v : mn[d];
      mx[d] = (v > mx[d]) ? v : mx[d];
    }
  linspace(mn[0], mx[0], g.nx, g.gx);
  linspace(mn[1], mx[1], g.ny, g.gy);
  if (D == 3) linspace(mn[2], mx[2], g.nz, g.gz);
  const size_t rows = (size_t)(g.nx + 1) * (g.ny + 1) * (g.nz + 1);
  g.vals.assign(rows * DD, 0.0);
  // MonitorFunction<D>::evaluateAtVertices (src/MonitorFunction.cpp:16-32)
  std::vector<double> monVals((size_t)nP * DD);
  for (int v = 0; v < nP; ++v) {
    double M[9];
    for (int i = 0; i < DD; ++i) M[i] = 0.0;  // monTemp.setZero()
    fn(D, &X[(size_t)v * D], M, user);
    std::memcpy(&monVals[(size_t)v * DD], M, DD * sizeof(double));
  }
  BucketNN<D> nn(X, nP);
  const int nx = g.nx, ny = g.ny;
  if (D == 2) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < nx + 1; i++)
      for (int j = 0; j < ny + 1; j++) {
        const double q[2] = {g.gx[i], g.gy[j]};
        const int id = nn.nearest(q);
        std::memcpy(&g.vals[((size_t)j * (nx + 1) + i) * DD], &monVals[(size_t)id * DD], DD * sizeof(double));
      }
  } else {
    const int nz = g.nz;
#pragma omp parallel for schedule(dynamic, 1)
    for (int k = 0; k < nz + 1; k++)
      for (int i = 0; i < nx + 1; i++)
        for (int j = 0; j < ny + 1; j++) {
          const double q[3] = {g.gx[i], g.gy[j], g.gz[k]};
          const int id = nn.nearest(q);
          // src/MeshInterpolator.cpp:234: row (nx+1)(ny+1)k + i(nx+1) + j (x and y swapped)
          std::memcpy(&g.vals[((size_t)(nx + 1) * (ny + 1) * k + (size_t)i * (nx + 1) + j) * DD],
                      &monVals[(size_t)id * DD], DD * sizeof(double));
        }
  }
  // smoothMonitorGrid: Jacobi passes on interior grid points
  const int nIters = (D == 2) ? 5 : 2;
  std::vector<double> tmp;
  for (int it = 0; it < nIters; ++it) {
    tmp = g.vals;
    if (D == 2) {
#pragma omp parallel for schedule(static)
      for (int i = 1; i < nx; i++)
        for (int j = 1; j < ny; j++) {
          const size_t c = (size_t)j * (nx + 1) + i;
          for (int q = 0; q < DD; ++q) {
            double v = 0.6 * tmp[c * DD + q];
            v += 0.1 * tmp[(c + 1) * DD + q];
            v += 0.1 * tmp[(c - 1) * DD + q];
            v += 0.1 * tmp[(c + nx + 1) * DD + q];
            v += 0.1 * tmp[(c - nx - 1) * DD + q];
            g.vals[c * DD + q] = v;
          }
        }
    } else {
      const double h = 0.4 / 6.0;
      const int nz = g.nz;
      const size_t P = (size_t)(nx + 1) * (ny + 1);
#pragma omp parallel for schedule(static)
      for (int k = 1; k < nz; k++)
        for (int i = 1; i < nx; i++)
          for (int j = 1; j < ny; j++) {
            const size_t c = P * k + (size_t)j * (nx + 1) + i;
            for (int q = 0; q < DD; ++q)
              g.vals[c * DD + q] = 0.6 * tmp[c * DD + q] + h * tmp[(c + 1) * DD + q] + h * tmp[(c - 1) * DD + q] +
                                   h * tmp[(c + nx + 1) * DD + q] + h * tmp[(c - nx - 1) * DD + q] +
                                   h * tmp[(c + P) * DD + q] + h * tmp[(c - P) * DD + q];
          }
    }
  }
}

}  // namespace

void build_monitor_grid(int dim, const double* X, int nP, mmadmm_monitor_fn fn, void* user, HostGrid& g) {
  if (dim == 2)
    buildGrid<2>(X, nP, fn, user, g);
  else
    buildGrid<3>(X, nP, fn, user, g);
}

}  // namespace mmx
