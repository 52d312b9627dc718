// meshgen.cpp -- host mesh generators, reader and writers.
//
//   mmadmm_mesh_rect        utils::generateUniformRectMesh<D> (src/MeshUtils.h:82-335), including
//                           its int truncation of xa..zb and its 2D jOff = i/(ny+1) boundary rule
//   mmadmm_mesh_levelset2d  utils::meshFromLevelSetFun 2D with circlePhi (src/MeshUtils.h:404-538,
//                           main.cpp:33-40); the O(nP*nF) remap loop (510-518) is replaced by an
//                           O(N) ascending-rank compaction with the same result
//   mmadmm_mesh_levelset3d  utils::meshFromLevelSetFun 3D with spherePhi (src/MeshUtils.h:540-667,
//                           main.cpp:87-97), O(N), with the reference's hand-back defect repaired
//   mmadmm_mesh_hexdisc     a well-shaped disc mesh (not in the reference)
//   mmadmm_mesh_shoulder    setUpShoulderExperiment's mesh (main.cpp:403-630): the rect mesh without
//                           the simplices whose centroid lies in the upper (x, y[, z]) quadrant, its
//                           boundary re-marking, and the interior vertices moved by up to h/10 in a
//                           random direction -- glibc rand() (the caller seeds it; main.cpp:785 does
//                           srand(69)) and Eigen 3.4's Random() (x + (y - x) rand() / RAND_MAX, in
//                           [-1, 1], coefficient order); Eigen is un-vendored (its version unpinned)
//   mmadmm_mesh_read        utils::readTriangles (src/MeshUtils.h:669-733)
//   mmadmm_write_points / mmadmm_write_simplices: Mesh::outputPoints / outputSimplices
//                           (src/Mesh.cpp:1067-1095), default ostream formatting (%.6g)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>

#include "common.h"

namespace mmx {
namespace {

constexpr int kFree = MMADMM_BOUNDARY_FREE, kFixed = MMADMM_BOUNDARY_FIXED, kInterior = MMADMM_INTERIOR;

void rect2d(int nx, int ny, int xa, int xb, int ya, int yb, int bType, MeshBuf& m) {
  const double hx = (xb - xa) / ((double)nx), hy = (yb - ya) / ((double)ny);
  const int nP = (nx + 1) * (ny + 1) + nx * ny;
  m.dim = 2;
  m.Vp.assign((size_t)nP * 2, 0.0);
  m.F.assign((size_t)4 * nx * ny * 3, 0);
  m.mask.assign(nP, kInterior);
  size_t off = 0;
  for (int j = 0; j <= ny; j++)
    for (int i = 0; i <= nx; i++, off++) {
      m.Vp[off * 2] = xa + hx * i;
      m.Vp[off * 2 + 1] = ya + hy * j;
    }
  for (int j = 0; j < ny; j++)  // cell midpoints
    for (int i = 0; i < nx; i++, off++) {
      m.Vp[off * 2] = xa + hx * i + hx / 2.0;
      m.Vp[off * 2 + 1] = ya + hy * j + hy / 2.0;
    }
  const int stride = (nx + 1) * (ny + 1);
  int32_t* F = m.F.data();
  size_t t = 0;
  auto tri = [&](int a, int b, int c) {
    F[t * 3] = a;
    F[t * 3 + 1] = b;
    F[t * 3 + 2] = c;
    ++t;
  };
  for (int j = 0; j < ny; j++)
    for (int i = 0; i < nx; i++) {
      const int c00 = i + j * (nx + 1), c10 = i + 1 + j * (nx + 1);
      const int c01 = i + (j + 1) * (nx + 1), c11 = i + 1 + (j + 1) * (nx + 1);
      const int mid = stride + i + j * nx;
      tri(c00, mid, c01);  // left
      tri(mid, c11, c01);  // top
      tri(mid, c11, c10);  // right
      tri(c00, c10, mid);  // bottom
    }
  for (int i = 0; i < (nx + 1) * (ny + 1); i++) {
    const int iOff = i % (nx + 1), jOff = i / (ny + 1);
    const bool boundary = (iOff == 0) || (iOff == nx) || (jOff == 0) || (jOff == ny);
    m.mask[i] = boundary ? bType : kInterior;
    const bool corner = (iOff == 0 || iOff == nx) && (jOff == 0 || jOff == ny);
    if (corner) m.mask[i] = kFixed;
  }
}

void rect3d(int nx, int ny, int nz, int xa, int xb, int ya, int yb, int za, int zb, int bType, MeshBuf& m) {
  const double hx = (xb - xa) / ((double)nx), hy = (yb - ya) / ((double)ny), hz = (zb - za) / ((double)nz);
  const int nP = (nx + 1) * (ny + 1) * (nz + 1) + nx * ny * nz;
  m.dim = 3;
  m.Vp.assign((size_t)nP * 3, 0.0);
  m.F.assign((size_t)12 * nx * ny * nz * 4, 0);
  m.mask.assign(nP, kInterior);
  size_t off = 0;
  for (int k = 0; k <= nz; k++)
    for (int j = 0; j <= ny; j++)
      for (int i = 0; i <= nx; i++, off++) {
        m.Vp[off * 3] = xa + hx * i;
        m.Vp[off * 3 + 1] = ya + hy * j;
        m.Vp[off * 3 + 2] = za + hz * k;
      }
  for (int k = 0; k < nz; k++)
    for (int j = 0; j < ny; j++)
      for (int i = 0; i < nx; i++, off++) {
        m.Vp[off * 3] = xa + hx * i + hx / 2.0;
        m.Vp[off * 3 + 1] = ya + hy * j + hy / 2.0;
        m.Vp[off * 3 + 2] = za + hz * k + hz / 2.0;
      }
  const int stride = (nx + 1) * (ny + 1) * (nz + 1);
  const int sy = nx + 1, sz = (nx + 1) * (ny + 1);
  int32_t* F = m.F.data();
  size_t t = 0;
  for (int k = 0; k < nz; k++)
    for (int j = 0; j < ny; j++)
      for (int i = 0; i < nx; i++) {
        const int mid = stride + i + j * nx + k * (nx * ny);
        auto P = [&](int di, int dj, int dk) { return (i + di) + (j + dj) * sy + (k + dk) * sz; };
        // 12 tets per cell, two per face, each closed by the cell centre
        const int faces[12][3][3] = {
            {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}}, {{0, 0, 0}, {0, 1, 0}, {1, 1, 0}},  // z-
            {{0, 0, 1}, {1, 0, 1}, {1, 1, 1}}, {{0, 0, 1}, {0, 1, 1}, {1, 1, 1}},  // z+
            {{0, 0, 0}, {0, 1, 0}, {0, 1, 1}}, {{0, 0, 0}, {0, 0, 1}, {0, 1, 1}},  // x-
            {{1, 0, 0}, {1, 1, 0}, {1, 1, 1}}, {{1, 0, 0}, {1, 0, 1}, {1, 1, 1}},  // x+
            {{0, 0, 0}, {1, 0, 0}, {0, 0, 1}}, {{1, 0, 0}, {1, 0, 1}, {0, 0, 1}},  // y-
            {{0, 1, 0}, {1, 1, 0}, {0, 1, 1}}, {{1, 1, 0}, {1, 1, 1}, {0, 1, 1}}};  // y+
        for (int q = 0; q < 12; ++q, ++t) {
          for (int v = 0; v < 3; ++v) F[t * 4 + v] = P(faces[q][v][0], faces[q][v][1], faces[q][v][2]);
          F[t * 4 + 3] = mid;
        }
      }
  for (int k = 0; k < nz + 1; k++)
    for (int i = 0; i < (nx + 1) * (ny + 1); i++) {
      const int iOff = i / (nx + 1), jOff = i % (ny + 1);
      const bool boundary = iOff == 0 || iOff == nx || jOff == 0 || jOff == ny || k == 0 || k == nz;
      const int o = k * (nx + 1) * (ny + 1) + i;
      if (boundary) m.mask[o] = bType;
      const bool ie = (iOff == 0 || iOff == nx), je = (jOff == 0 || jOff == ny), ke = (k == 0 || k == nz);
      if ((ie && je) || (ie && ke) || (ke && je)) m.mask[o] = kFixed;  // the 12 cube edges
    }
}

double circlePhi(double x, double y) {  // main.cpp:33-40
  const double r = 0.35, cx = 0.5, cy = 0.5;
  const double xval = (x - cx), yval = (y - cy);
  return sqrt(xval * xval + yval * yval) - r;
}

void levelset2d(int nx, int ny, double xa, double xb, double ya, double yb, int bType, bool compact, MeshBuf& m) {
  const double EPS = 1e-12;
  MeshBuf g;
  rect2d(nx, ny, (int)xa, (int)xb, (int)ya, (int)yb, bType, g);
  for (auto& v : g.mask) v = kInterior;
  const int nF0 = g.nF(), nP0 = g.nP();
  std::vector<int> keep;
  keep.reserve(nF0);
  for (int s = 0; s < nF0; ++s) {  // drop simplices with every vertex outside (phi > -EPS)
    bool out = true;
    for (int j = 0; j < 3; ++j) {
      const int v = g.F[(size_t)s * 3 + j];
      out = out && circlePhi(g.Vp[(size_t)v * 2], g.Vp[(size_t)v * 2 + 1]) > -EPS;
    }
    if (!out) keep.push_back(s);
  }
  std::vector<char> used(nP0, 0);
  for (int s : keep)
    for (int j = 0; j < 3; ++j) used[g.F[(size_t)s * 3 + j]] = 1;
  for (int p = 0; p < nP0; ++p) {  // project outside / on-boundary points (369-386, 478-491)
    if (!used[p]) continue;
    double X = g.Vp[(size_t)p * 2], Y = g.Vp[(size_t)p * 2 + 1];
    const double phi = circlePhi(X, Y);
    if (std::abs(phi) < EPS || phi > 0) {
      const double xv = X - 0.5, yv = Y - 0.5;
      const double n0 = xv / sqrt(xv * xv + yv * yv), n1 = yv / sqrt(xv * xv + yv * yv);
      const double ph = circlePhi(X, Y);
      X = X - ph * n0;
      Y = Y - ph * n1;
      g.mask[p] = bType;
    }
    g.Vp[(size_t)p * 2] = X;
    g.Vp[(size_t)p * 2 + 1] = Y;
  }
  std::vector<int> rank(nP0, -1);
  int cnt = 0;
  for (int p = 0; p < nP0; ++p)
    if (used[p]) rank[p] = cnt++;
  m.dim = 2;
  m.Vp.resize((size_t)cnt * 2);
  for (int p = 0; p < nP0; ++p)
    if (used[p]) {
      m.Vp[(size_t)rank[p] * 2] = g.Vp[(size_t)p * 2];
      m.Vp[(size_t)rank[p] * 2 + 1] = g.Vp[(size_t)p * 2 + 1];
    }
  m.F.resize(keep.size() * 3);
  for (size_t i = 0; i < keep.size(); ++i)
    for (int j = 0; j < 3; ++j) m.F[i * 3 + j] = rank[g.F[(size_t)keep[i] * 3 + j]];
  if (compact) {
    m.mask.assign(cnt, kInterior);
    for (int p = 0; p < nP0; ++p)
      if (used[p]) m.mask[rank[p]] = g.mask[p];
  } else {
    m.mask = g.mask;  // the reference leaves it indexed by pre-compaction ids
  }
  for (int p = 0; p < cnt; ++p)
    if (std::abs(circlePhi(m.Vp[(size_t)p * 2], m.Vp[(size_t)p * 2 + 1])) < EPS) m.mask[p] = kFixed;
}

double spherePhi(double x, double y, double z) {  // main.cpp:87-97 (squared form)
  const double r = 0.4, cx = 0.5, cy = 0.5, cz = 0.5;
  const double xval = (x - cx), yval = (y - cy), zval = (z - cz);
  return xval * xval + yval * yval + zval * zval - r * r;
}

// utils::meshFromLevelSetFun 3D (src/MeshUtils.h:540-667) with spherePhi (main.cpp:363), O(N):
// the cube cut to the tetrahedra with a vertex inside (phi <= -EPS), the used vertices with
// phi > -EPS moved by interpolateBoundaryLocation 3D (388-402: central-difference normal,
// h = 2 sqrt(eps), p - phi(p) n) and marked bType, then the used vertices numbered in DESCENDING
// original id (the reference's pntMap, 645-651) with F remapped alike.  Repaired:
// the reference hands nothing back -- `delete Vp; Vp = Vpnew;` (663-666) reassigns its own
// pointer copies, so the caller's arrays are left deleted -- and it does not compact the mask;
// compact = true remaps the mask to the new numbering (false: the reference's old-id indexing).
// A third repair: the reference remaps F in place (653-661), walking the used ids in ASCENDING
// order with the DESCENDING map, so an entry already remapped to a larger id that is itself a used
// id yet to come is remapped again (ids {0,1,2}: 0 -> 2 -> 0, and 2 -> 0 as well); F is remapped
// here once per entry, with pntMap as the reference intends.  (The 2D generator's map is
// ascending, so a remapped id never exceeds its original and that loop is sound.)
void levelset3d(int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za, double zb, int bType,
                bool compact, MeshBuf& m) {
  const double EPS = 1e-12;
  MeshBuf g;
  rect3d(nx, ny, nz, (int)xa, (int)xb, (int)ya, (int)yb, (int)za, (int)zb, bType, g);
  for (auto& v : g.mask) v = kInterior;
  const int nF0 = g.nF(), nP0 = g.nP();
  std::vector<double> phi(nP0);
  for (int p = 0; p < nP0; ++p) phi[p] = spherePhi(g.Vp[(size_t)p * 3], g.Vp[(size_t)p * 3 + 1], g.Vp[(size_t)p * 3 + 2]);
  std::vector<int> keep;
  keep.reserve(nF0);
  for (int s = 0; s < nF0; ++s) {  // drop the tetrahedra with every vertex outside
    bool out = true;
    for (int j = 0; j < 4; ++j) out = out && phi[g.F[(size_t)s * 4 + j]] > -EPS;
    if (!out) keep.push_back(s);
  }
  std::vector<char> used(nP0, 0);
  for (int s : keep)
    for (int j = 0; j < 4; ++j) used[g.F[(size_t)s * 4 + j]] = 1;
  const double h = 2.0 * sqrt(2.220446049250313080847e-16);
  for (int p = 0; p < nP0; ++p) {
    if (!used[p] || !(phi[p] > -EPS)) continue;
    double* x = &g.Vp[(size_t)p * 3];
    double n[3];
    n[0] = (spherePhi(x[0] + h, x[1], x[2]) - spherePhi(x[0] - h, x[1], x[2])) / (2.0 * h);
    n[1] = (spherePhi(x[0], x[1] + h, x[2]) - spherePhi(x[0], x[1] - h, x[2])) / (2.0 * h);
    n[2] = (spherePhi(x[0], x[1], x[2] + h) - spherePhi(x[0], x[1], x[2] - h)) / (2.0 * h);
    const double sq = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];  // Eigen normalize()
    if (sq > 0) {
      const double nrm = sqrt(sq);
      for (int c = 0; c < 3; ++c) n[c] = n[c] / nrm;
    }
    const double ph = phi[p];
    for (int c = 0; c < 3; ++c) x[c] = x[c] - ph * n[c];
    g.mask[p] = bType;
  }
  int cnt = 0;
  for (int p = 0; p < nP0; ++p) cnt += used[p];
  std::vector<int> rank(nP0, -1);
  for (int p = nP0 - 1, r = 0; p >= 0; --p)
    if (used[p]) rank[p] = r++;
  m.dim = 3;
  m.Vp.resize((size_t)cnt * 3);
  for (int p = 0; p < nP0; ++p)
    if (used[p])
      for (int c = 0; c < 3; ++c) m.Vp[(size_t)rank[p] * 3 + c] = g.Vp[(size_t)p * 3 + c];
  m.F.resize(keep.size() * 4);
  for (size_t i = 0; i < keep.size(); ++i)
    for (int j = 0; j < 4; ++j) m.F[i * 4 + j] = rank[g.F[(size_t)keep[i] * 4 + j]];
  if (compact) {
    m.mask.assign(cnt, kInterior);
    for (int p = 0; p < nP0; ++p)
      if (used[p]) m.mask[rank[p]] = g.mask[p];
  } else {
    m.mask = g.mask;
  }
}

void hexdisc(int N, double r, double cx, double cy, int bType, MeshBuf& m) {
  const long nP = 3L * N * (N + 1) + 1;
  m.dim = 2;
  m.Vp.assign((size_t)nP * 2, 0.0);
  m.mask.assign(nP, kInterior);
  m.Vp[0] = cx;
  m.Vp[1] = cy;
  const double third_pi = 1.0471975511965976;  // pi / 3
  for (int k = 1; k <= N; ++k) {
    const long base = 1 + 3L * k * (k - 1);
    const double rad = r * k / N;
    for (int j = 0; j < 6 * k; ++j) {
      const double th = third_pi * ((double)j / k);
      m.Vp[(size_t)(base + j) * 2] = cx + rad * cos(th);
      m.Vp[(size_t)(base + j) * 2 + 1] = cy + rad * sin(th);
      if (k == N) m.mask[base + j] = bType;
    }
  }
  auto gid = [](int k, int s, int t) -> int32_t {
    if (k == 0) return 0;
    s = (s + t / k) % 6;
    t = t % k;
    return (int32_t)(1 + 3L * k * (k - 1) + (long)s * k + t);
  };
  m.F.clear();
  m.F.reserve((size_t)6 * N * N * 3);
  for (int k = 1; k <= N; ++k)
    for (int s = 0; s < 6; ++s) {
      for (int t = 0; t < k; ++t) {
        m.F.push_back(gid(k, s, t));
        m.F.push_back(gid(k, s, t + 1));
        m.F.push_back(k > 1 ? gid(k - 1, s, t) : 0);
      }
      for (int t = 0; t < k - 1; ++t) {
        m.F.push_back(gid(k - 1, s, t));
        m.F.push_back(gid(k, s, t + 1));
        m.F.push_back(gid(k - 1, s, t + 1));
      }
    }
}

void shoulder(int dim, int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za, double zb,
              int bType, MeshBuf& m) {
  if (dim == 2)
    rect2d(nx, ny, (int)xa, (int)xb, (int)ya, (int)yb, bType, m);
  else
    rect3d(nx, ny, nz, (int)xa, (int)xb, (int)ya, (int)yb, (int)za, (int)zb, bType, m);
  const int D = dim, V = D + 1;
  const double cx = (xa + xb) / 2.0, cy = (ya + yb) / 2.0, cz = (za + zb) / 2.0;
  const double EPS = 1e-16;
  const std::vector<double>& X = m.Vp;  // Vc: not yet perturbed
  std::vector<char> removed(m.nF(), 0);
  for (int i = 0; i < m.nF(); i++) {
    double x[4][3] = {{0}};
    for (int n = 0; n < V; ++n)
      for (int d = 0; d < D; ++d) x[n][d] = X[(size_t)m.F[(size_t)i * V + n] * D + d];
    double c[3];
    for (int d = 0; d < D; ++d)  // (1/3)(x0 + x1 + x2) / (1/4)(x0 + x1 + x2 + x3), Eigen order
      c[d] = (D == 2) ? (1.0 / 3.0) * ((x[0][d] + x[1][d]) + x[2][d])
                      : (1.0 / 4.0) * (((x[0][d] + x[1][d]) + x[2][d]) + x[3][d]);
    const bool inQuad = (D == 2) ? (c[0] > cx && c[1] > cy) : (c[0] > cx && c[1] > cy && c[2] > cz);
    if (!inQuad) continue;
    removed[i] = 1;
    for (int n = 0; n < V; ++n) {
      const double* p = x[n];
      bool fixed;
      if (D == 2) {
        fixed = (std::fabs(p[0] - cx) < EPS && std::fabs(p[1] - cy) < EPS) ||
                (std::fabs(p[0] - cx) < EPS && std::fabs(p[1] - yb) < EPS) ||
                (std::fabs(p[0] - xb) < EPS && std::fabs(p[1] - cy) < EPS);
      } else {
        fixed = (std::fabs(p[0] - cx) < EPS && std::fabs(p[2] - cz) < EPS) ||
                (std::fabs(p[0] - cx) < EPS && std::fabs(p[2] - zb) < EPS) ||
                (std::fabs(p[0] - xb) < EPS && std::fabs(p[2] - cz) < EPS) ||
                (std::fabs(p[1] - ya) < EPS && std::fabs(p[2] - cz) < EPS) ||
                (std::fabs(p[1] - yb) < EPS && std::fabs(p[2] - cz) < EPS) ||
                (std::fabs(p[0] - cx) < EPS && std::fabs(p[1] - ya) < EPS) ||
                (std::fabs(p[0] - cx) < EPS && std::fabs(p[1] - yb) < EPS);
      }
      m.mask[m.F[(size_t)i * V + n]] = fixed ? kFixed : bType;
    }
  }
  // utils::removeRow in descending id order == keeping the others in order
  std::vector<int32_t> F2;
  F2.reserve(m.F.size());
  for (int i = 0; i < m.nF(); ++i)
    if (!removed[i]) F2.insert(F2.end(), m.F.begin() + (size_t)i * V, m.F.begin() + (size_t)(i + 1) * V);
  m.F.swap(F2);
  m.Vc = m.Vp;
  const double hx = (xb - xa) / ((double)nx), hy = (yb - ya) / ((double)ny);
  const double hz = (D == 3) ? (zb - za) / ((double)nz) : 0;
  const double h = sqrt(hx * hx + hy * hy + hz * hz);
  for (int i = 0; i < m.nP(); i++) {
    if (m.mask[i] != kInterior) continue;
    double dir[3], sq = 0.0;
    for (int d = 0; d < D; ++d) dir[d] = -1.0 + (1.0 - (-1.0)) * (double)rand() / (double)RAND_MAX;
    for (int d = 0; d < D; ++d) sq = (d == 0) ? dir[d] * dir[d] : sq + dir[d] * dir[d];
    const double nrm = sqrt(sq);
    for (int d = 0; d < D; ++d) dir[d] /= nrm;
    const double r = (h / 10.0) * static_cast<double>(rand()) / static_cast<double>(RAND_MAX);
    for (int d = 0; d < D; ++d) m.Vp[(size_t)i * D + d] += r * dir[d];
  }
}

void readMesh(int dim, const char* tri, const char* pnts, const char* mask, MeshBuf& m) {
  m.dim = dim;
  std::string line, word;
  std::ifstream ft(tri);
  if (!ft) throw Error(MMADMM_ERR_IO, std::string("cannot read ") + tri);
  std::vector<int32_t> triData;
  while (std::getline(ft, line)) {
    std::stringstream s(line);
    while (std::getline(s, word, ',')) triData.push_back(std::stoi(word));
  }
  std::ifstream fp(pnts);
  if (!fp) throw Error(MMADMM_ERR_IO, std::string("cannot read ") + pnts);
  std::vector<double> pd;
  while (std::getline(fp, line)) {
    std::stringstream s(line);
    while (std::getline(s, word, ',')) pd.push_back(std::stod(word));
  }
  std::ifstream fm(mask);
  if (!fm) throw Error(MMADMM_ERR_IO, std::string("cannot read ") + mask);
  m.mask.clear();
  int tmp;
  while (fm >> tmp) m.mask.push_back(tmp);
  const size_t nF = triData.size() / (dim + 1), nP = pd.size() / dim;
  m.F.assign(triData.begin(), triData.begin() + nF * (dim + 1));
  m.Vp.assign(pd.begin(), pd.begin() + nP * dim);
}

}  // namespace
}  // namespace mmx

using mmx::Error;
using mmx::guarded;
using mmx::MeshBuf;

extern "C" {

int mmadmm_mesh_rect(int dim, int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za,
                     double zb, int btype, mmadmm_mesh* out) {
  return guarded([&] {
    if (!out || (dim != 2 && dim != 3) || nx < 1 || ny < 1 || (dim == 3 && nz < 1))
      throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_rect: bad arguments");
    auto* m = new MeshBuf();
    if (dim == 2)
      mmx::rect2d(nx, ny, (int)xa, (int)xb, (int)ya, (int)yb, btype, *m);
    else
      mmx::rect3d(nx, ny, nz, (int)xa, (int)xb, (int)ya, (int)yb, (int)za, (int)zb, btype, *m);
    *out = reinterpret_cast<mmadmm_mesh>(m);
  });
}

int mmadmm_mesh_levelset2d(int nx, int ny, double xa, double xb, double ya, double yb, int btype, int compact_mask,
                           mmadmm_mesh* out) {
  return guarded([&] {
    if (!out || nx < 1 || ny < 1) throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_levelset2d: bad arguments");
    auto* m = new MeshBuf();
    mmx::levelset2d(nx, ny, xa, xb, ya, yb, btype, compact_mask != 0, *m);
    *out = reinterpret_cast<mmadmm_mesh>(m);
  });
}

int mmadmm_mesh_levelset3d(int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za, double zb,
                           int btype, int compact_mask, mmadmm_mesh* out) {
  return guarded([&] {
    if (!out || nx < 1 || ny < 1 || nz < 1) throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_levelset3d: bad arguments");
    auto* m = new MeshBuf();
    mmx::levelset3d(nx, ny, nz, xa, xb, ya, yb, za, zb, btype, compact_mask != 0, *m);
    *out = reinterpret_cast<mmadmm_mesh>(m);
  });
}

int mmadmm_mesh_shoulder(int dim, int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za,
                         double zb, int btype, mmadmm_mesh* out) {
  return guarded([&] {
    if (!out || (dim != 2 && dim != 3) || nx < 1 || ny < 1 || (dim == 3 && nz < 1))
      throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_shoulder: bad arguments");
    auto* m = new MeshBuf();
    mmx::shoulder(dim, nx, ny, nz, xa, xb, ya, yb, za, zb, btype, *m);
    *out = reinterpret_cast<mmadmm_mesh>(m);
  });
}

int mmadmm_mesh_reference_points(mmadmm_mesh h, double* Xc) {
  return guarded([&] {
    auto* m = reinterpret_cast<MeshBuf*>(h);
    if (!m || !Xc) throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_reference_points: null argument");
    const std::vector<double>& src = m->Vc.empty() ? m->Vp : m->Vc;
    std::copy(src.begin(), src.end(), Xc);
  });
}

int mmadmm_mesh_hexdisc(int N, double r, double cx, double cy, int btype, mmadmm_mesh* out) {
  return guarded([&] {
    if (!out || N < 1 || !(r > 0)) throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_hexdisc: bad arguments");
    auto* m = new MeshBuf();
    mmx::hexdisc(N, r, cx, cy, btype, *m);
    *out = reinterpret_cast<mmadmm_mesh>(m);
  });
}

int mmadmm_mesh_read(int dim, const char* tri, const char* pnts, const char* mask, mmadmm_mesh* out) {
  return guarded([&] {
    if (!out || !tri || !pnts || !mask || (dim != 2 && dim != 3))
      throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_read: bad arguments");
    auto* m = new MeshBuf();
    try {
      mmx::readMesh(dim, tri, pnts, mask, *m);
    } catch (...) {
      delete m;
      throw;
    }
    *out = reinterpret_cast<mmadmm_mesh>(m);
  });
}

int mmadmm_mesh_sizes(mmadmm_mesh h, int* dim, int* nP, int* nF, int* mask_len) {
  return guarded([&] {
    if (!h) throw Error(MMADMM_ERR_INVALID, "null mesh");
    const auto* m = reinterpret_cast<const MeshBuf*>(h);
    if (dim) *dim = m->dim;
    if (nP) *nP = m->nP();
    if (nF) *nF = m->nF();
    if (mask_len) *mask_len = (int)m->mask.size();
  });
}

int mmadmm_mesh_copy(mmadmm_mesh h, double* Xp, int32_t* F, int32_t* mask) {
  return guarded([&] {
    if (!h) throw Error(MMADMM_ERR_INVALID, "null mesh");
    const auto* m = reinterpret_cast<const MeshBuf*>(h);
    if (Xp) std::copy(m->Vp.begin(), m->Vp.end(), Xp);
    if (F) std::copy(m->F.begin(), m->F.end(), F);
    if (mask) std::copy(m->mask.begin(), m->mask.end(), mask);
  });
}

int mmadmm_mesh_free(mmadmm_mesh h) {
  delete reinterpret_cast<MeshBuf*>(h);
  return MMADMM_OK;
}

int mmadmm_write_points(const char* path, int dim, int nP, const double* Xp) {
  return guarded([&] {
    FILE* f = std::fopen(path, "w");
    if (!f) throw Error(MMADMM_ERR_IO, std::string("cannot write ") + path);
    for (int i = 0; i < nP; ++i) {
      for (int j = 0; j < dim - 1; ++j) std::fprintf(f, "%.6g, ", Xp[(size_t)i * dim + j]);
      std::fprintf(f, "%.6g\n", Xp[(size_t)i * dim + dim - 1]);
    }
    std::fclose(f);
  });
}

int mmadmm_write_simplices(const char* path, int dim, int nF, const int32_t* F) {
  return guarded([&] {
    FILE* f = std::fopen(path, "w");
    if (!f) throw Error(MMADMM_ERR_IO, std::string("cannot write ") + path);
    for (int i = 0; i < nF; ++i) {
      for (int j = 0; j < dim; ++j) std::fprintf(f, "%d, ", F[(size_t)i * (dim + 1) + j]);
      std::fprintf(f, "%d\n", F[(size_t)i * (dim + 1) + dim]);
    }
    std::fclose(f);
  });
}

}  // extern "C"
