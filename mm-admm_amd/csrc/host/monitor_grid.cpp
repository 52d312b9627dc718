// monitor_grid.cpp -- set-up of the smoothed monitor grid the hot path interpolates.
//
// MeshInterpolator<D>::updateMesh + interpolateMonitor (src/MeshInterpolator.cpp:68-130,
// 244-259): grid size (int)pow(nP*D, 1/D) over the initial mesh bounding box, monitor at
// every vertex, nearest vertex per grid point, then Jacobi smoothing (5 passes 2D, 2 passes
// 3D; 366-404).  The reference's nanoflann kNN(k=1) is replaced by an exact k-d tree search;
// ties between equidistant vertices resolve to the lowest vertex id.
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

// Exact nearest vertex by a median-split k-d tree (the role of nanoflann's KDTreeSingleIndexAdaptor,
// src/MeshInterpolator.h:61-84).  Distances are nanoflann's L2_Simple_Adaptor sums of squared
// differences; a far subtree is pruned only when its lower bound strictly exceeds the best
// distance, so equidistant vertices resolve to the lowest id.
template <int D>
class KdNN {
 public:
  KdNN(const double* X, int n) : X_(X), idx_(n) {
    for (int i = 0; i < n; ++i) idx_[i] = i;
    nodes_.reserve(2 * (n / kLeaf + 1));
    build(0, n);
  }

  int nearest(const double* q) const {
    double best = INFINITY;
    int bi = -1;
    search(0, q, best, bi);
    return bi;
  }

 private:
  static constexpr int kLeaf = 8;
  struct Node {
    int lo, hi;    // point range (leaf) or split position (inner: [lo, mid), [mid, hi))
    int axis;      // -1 for a leaf
    double split;
    int left, right;
  };

  int build(int lo, int hi) {
    const int id = (int)nodes_.size();
    nodes_.push_back(Node{lo, hi, -1, 0.0, -1, -1});
    if (hi - lo <= kLeaf) return id;
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int t = lo; t < hi; ++t)
      for (int d = 0; d < D; ++d) {
        const double v = X_[(size_t)idx_[t] * D + d];
        mn[d] = std::min(mn[d], v);
        mx[d] = std::max(mx[d], v);
      }
    int axis = 0;
    for (int d = 1; d < D; ++d)
      if (mx[d] - mn[d] > mx[axis] - mn[axis]) axis = d;
    const int mid = lo + (hi - lo) / 2;
    std::nth_element(idx_.begin() + lo, idx_.begin() + mid, idx_.begin() + hi, [&](int a, int b) {
      const double va = X_[(size_t)a * D + axis], vb = X_[(size_t)b * D + axis];
      return va < vb || (va == vb && a < b);
    });
    const double split = X_[(size_t)idx_[mid] * D + axis];
    const int l = build(lo, mid);
    const int r = build(mid, hi);
    nodes_[id].axis = axis;
    nodes_[id].split = split;
    nodes_[id].left = l;
    nodes_[id].right = r;
    return id;
  }

  void search(int id, const double* q, double& best, int& bi) const {
    const Node& nd = nodes_[id];
    if (nd.axis < 0) {
      for (int t = nd.lo; t < nd.hi; ++t) {
        const int i = idx_[t];
        double dd = 0.0;
        for (int d = 0; d < D; ++d) {
          const double df = q[d] - X_[(size_t)i * D + d];
          dd += df * df;
        }
        if (dd < best || (dd == best && i < bi)) {
          best = dd;
          bi = i;
        }
      }
      return;
    }
    const double diff = q[nd.axis] - nd.split;
    const int nearC = (diff < 0) ? nd.left : nd.right, farC = (diff < 0) ? nd.right : nd.left;
    search(nearC, q, best, bi);
    if (diff * diff <= best) search(farC, q, best, bi);
  }

  const double* X_;
  std::vector<int> idx_;
  std::vector<Node> nodes_;
};

template <int D>
void buildGrid(const double* X, int nP, mmadmm_monitor_fn fn, void* user, HostGrid& g) {
  constexpr int DD = D * D;
  double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = 0; i < nP; i++)
    for (int d = 0; d < D; ++d) {
      const double v = X[(size_t)i * D + d];
      mn[d] = (v < mn[d]) ? v : mn[d];
      mx[d] = (v > mx[d]) ? v : mx[d];
    }
  grid_geometry(D, nP, mn, mx, g);
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
  KdNN<D> nn(X, nP);
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

void grid_geometry(int dim, int nP, const double* lo, const double* hi, HostGrid& g) {
  const int sz = (int)std::pow((double)((long)nP * dim), 1.0 / dim);  // src/MeshInterpolator.cpp:78-84
  g.nx = sz;
  g.ny = sz;
  g.nz = (dim == 2) ? 1 : sz;
  for (int d = 0; d < 3; ++d) {
    g.lo[d] = d < dim ? lo[d] : 0.0;
    g.hi[d] = d < dim ? hi[d] : 0.0;
  }
  linspace(lo[0], hi[0], g.nx, g.gx);
  linspace(lo[1], hi[1], g.ny, g.gy);
  if (dim == 3) linspace(lo[2], hi[2], g.nz, g.gz);
}

void build_monitor_grid(int dim, const double* X, int nP, mmadmm_monitor_fn fn, void* user, HostGrid& g) {
  if (dim == 2)
    buildGrid<2>(X, nP, fn, user, g);
  else
    buildGrid<3>(X, nP, fn, user, g);
}

}  // namespace mmx

extern "C" int mmadmm_monitor_grid(int dim, int nP, const double* Xp, mmadmm_monitor_fn fn, void* user, int* rows,
                                   double* vals) {
  return mmx::guarded([&] {
    if ((dim != 2 && dim != 3) || nP < 1 || !Xp || !fn || !rows)
      throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_monitor_grid: bad arguments");
    mmx::HostGrid g;
    mmx::build_monitor_grid(dim, Xp, nP, fn, user, g);
    *rows = (int)(g.vals.size() / ((size_t)dim * dim));
    if (vals) std::copy(g.vals.begin(), g.vals.end(), vals);
  });
}
