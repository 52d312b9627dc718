// MeshUtils.h -- the reference's utils:: mesh generators and reader (src/MeshUtils.h:19-734) for
// main.cpp-style drivers, over the C-ABI of libmmadmm.so and host code.
//
// Same names, signatures and argument meaning as the reference:
//   linspace                  src/MeshUtils.h:24-29
//   findLimInfMeshPoint       src/MeshUtils.h:45-54 (the (int) cast and uint32 clamp included)
//   generateUniformRectMesh   src/MeshUtils.h:82-335  -> mmadmm_mesh_rect (xa..zb truncated to int,
//                             the 2D jOff = i/(ny+1) boundary rule; Vc / F / mask resized here)
//   removeRow                 src/MeshUtils.h:338-346
//   meshFromLevelSetFun 2D    src/MeshUtils.h:404-538 with any phiFun: simplices with every vertex
//                             at phi > -EPS dropped, the used points with |phi| < EPS or phi > 0
//                             moved by interpolateBoundaryLocation 2D (369-386: the normal about
//                             (0.5, 0.5) the reference hard-codes, the distance phiFun) and marked
//                             bType, renumbered by ascending id; the mask keeps the reference's
//                             pre-compaction indexing (487) and then |phi| < EPS -> FIXED at the new
//                             ids (531-537); Vc is left unset, as in the reference (430-435, 507)
//   meshFromLevelSetFun 3D    src/MeshUtils.h:540-667 with any phiFun: the same cut, the points
//                             with phi > -EPS moved by interpolateBoundaryLocation 3D (388-402:
//                             central-difference normal of phiFun, h = 2 sqrt(eps)), nodes
//                             numbered as the reference's pntMap (the i-th largest used id -> i).
//                             Repaired: the reference never hands its result back (663-666
//                             reassign its own pointer copies and leave the caller's deleted) and
//                             does not compact the mask; here Vc = Vp = the cut mesh and the mask
//                             follows the new numbering
//   readTriangles             src/MeshUtils.h:669-733 -> mmadmm_mesh_read (plus the one extra mask
//                             entry the reference's read loop appends at end of file, 706-711)
// With circlePhi / spherePhi (main.cpp:33-40, 87-97) the level-set meshes equal the library's
// mmadmm_mesh_levelset2d (compact_mask 0) / mmadmm_mesh_levelset3d (compact_mask 1) bit for bit
// (tests/test_cpp_dropin.py).  Header-only; link with -lmmadmm.
#ifndef MESH_UTILS_H
#define MESH_UTILS_H

#include <Eigen/Dense>
#include <cassert>
#include <cmath>
#include <cstdint>
#include <functional>
#include <limits>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../mmadmm.h"
#include "Mesh.h"
#include "NodeType.h"

using namespace std;

namespace utils {

inline void linspace(double xa, double xb, int ns, vector<double> &x) {
    x.resize(ns + 1);
    for (int i = 0; i < ns + 1; i++) x.at(i) = xa + ((double)i) * (xb - xa) / ns;
}

inline int findLimInfMeshPoint(double w, vector<double> &w_mesh) {
    uint32_t guess = (uint32_t)(int)((w - w_mesh.at(0)) / (w_mesh.at(1) - w_mesh.at(0)));
    if (guess > (uint32_t)(w_mesh.size() - 2)) guess = (uint32_t)(w_mesh.size() - 2);
    return (int)guess;
}

namespace detail {
// a library mesh handle into the caller's Eigen matrices (row per node / simplex)
inline void take(mmadmm_mesh h, Eigen::MatrixXd &Vp, Eigen::MatrixXi &F, vector<NodeType> &mask) {
    int dim = 0, nP = 0, nF = 0, ml = 0;
    mmadmm_cxx::check(mmadmm_mesh_sizes(h, &dim, &nP, &nF, &ml));
    std::vector<double> X((size_t)nP * dim);
    std::vector<int32_t> T((size_t)nF * (dim + 1)), m(ml);
    mmadmm_cxx::check(mmadmm_mesh_copy(h, X.data(), T.data(), m.data()));
    mmadmm_mesh_free(h);
    Vp.resize(nP, dim);
    for (int i = 0; i < nP; i++)
        for (int c = 0; c < dim; c++) Vp(i, c) = X[(size_t)i * dim + c];
    F.resize(nF, dim + 1);
    for (int i = 0; i < nF; i++)
        for (int c = 0; c < dim + 1; c++) F(i, c) = T[(size_t)i * (dim + 1) + c];
    mask.assign(m.size(), NodeType::INTERIOR);
    for (size_t i = 0; i < m.size(); i++) mask[i] = (NodeType)m[i];
}
inline double param(unordered_map<string, double> &params, const char *k) {
    return params.count(k) ? params[k] : 0.0;
}
}  // namespace detail

template <int D>
inline void generateUniformRectMesh(unordered_map<string, double> params, Eigen::MatrixXd *Vc, Eigen::MatrixXi *F,
                                    vector<NodeType> *boundaryMask, NodeType bType) {
    const int nx = (int)params["nx"], ny = (int)params["ny"], nz = (D == 3) ? (int)params["nz"] : 0;
    mmadmm_mesh h = nullptr;
    mmadmm_cxx::check(mmadmm_mesh_rect(D, nx, ny, nz, detail::param(params, "xa"), detail::param(params, "xb"),
                                       detail::param(params, "ya"), detail::param(params, "yb"),
                                       detail::param(params, "za"), detail::param(params, "zb"), (int)bType, &h));
    detail::take(h, *Vc, *F, *boundaryMask);
}

inline void removeRow(Eigen::MatrixXi &matrix, unsigned int rowToRemove) {
    const unsigned int numRows = matrix.rows() - 1, numCols = matrix.cols();
    if (rowToRemove > numRows) return;
    Eigen::MatrixXi out((Eigen::Index)numRows, (Eigen::Index)numCols);
    for (unsigned int i = 0, o = 0; i <= numRows; i++) {
        if (i == rowToRemove) continue;
        for (unsigned int j = 0; j < numCols; j++) out(o, j) = matrix(i, j);
        o++;
    }
    matrix = out;
}

inline void readTriangles(int D, const char *triFileName, const char *pntFileName, const char *maskFileName,
                          Eigen::MatrixXi &F, Eigen::MatrixXd &Vp, vector<NodeType> &boundaryMask) {
    mmadmm_mesh h = nullptr;
    mmadmm_cxx::check(mmadmm_mesh_read(D, triFileName, pntFileName, maskFileName, &h));
    detail::take(h, Vp, F, boundaryMask);
    boundaryMask.push_back((NodeType)0);  // the read loop's extra entry at end of file (706-711)
}

// meshFromLevelSetFun 2D (src/MeshUtils.h:404-538)
inline void meshFromLevelSetFun(std::function<double(double, double)> phiFun, std::vector<int> &nVals,
                                std::vector<std::tuple<double, double>> &bb, Eigen::MatrixXd *Vc, Eigen::MatrixXd *Vp,
                                Eigen::MatrixXi *F, vector<NodeType> *boundaryMask, NodeType bType) {
    const double EPS = 1e-12;
    const int nx = nVals.at(0), ny = nVals.at(1);
    unordered_map<string, double> params;
    params["nx"] = nx;
    params["ny"] = ny;
    params["xa"] = std::get<0>(bb.at(0));
    params["xb"] = std::get<1>(bb.at(0));
    params["ya"] = std::get<0>(bb.at(1));
    params["yb"] = std::get<1>(bb.at(1));
    Eigen::MatrixXd G;
    Eigen::MatrixXi T;
    vector<NodeType> mask;
    generateUniformRectMesh<2>(params, &G, &T, &mask, bType);
    for (auto &m : mask) m = NodeType::INTERIOR;
    const int nP0 = G.rows(), nF0 = T.rows();
    std::vector<int> keep;
    for (int s = 0; s < nF0; s++) {
        bool out = true;
        for (int j = 0; j < 3; j++) out = out && phiFun(G(T(s, j), 0), G(T(s, j), 1)) > -EPS;
        if (!out) keep.push_back(s);
    }
    std::vector<char> used(nP0, 0);
    for (int s : keep)
        for (int j = 0; j < 3; j++) used[T(s, j)] = 1;
    for (int p = 0; p < nP0; p++) {
        if (!used[p]) continue;
        double x = G(p, 0), y = G(p, 1);
        const double phi = phiFun(x, y);
        if (std::abs(phi) < EPS || phi > 0) {  // interpolateBoundaryLocation 2D (369-386)
            const double xv = x - 0.5, yv = y - 0.5;
            const double n0 = xv / sqrt(xv * xv + yv * yv), n1 = yv / sqrt(xv * xv + yv * yv);
            const double ph = phiFun(x, y);
            x = x - ph * n0;
            y = y - ph * n1;
            mask[p] = bType;
        }
        G(p, 0) = x;
        G(p, 1) = y;
    }
    std::vector<int> rank(nP0, -1);
    int cnt = 0;
    for (int p = 0; p < nP0; p++)
        if (used[p]) rank[p] = cnt++;
    Vp->resize(cnt, 2);
    Vc->resize(cnt, 2);  // (left unset by the reference)
    for (int p = 0; p < nP0; p++)
        if (used[p]) {
            (*Vp)(rank[p], 0) = G(p, 0);
            (*Vp)(rank[p], 1) = G(p, 1);
        }
    F->resize((Eigen::Index)keep.size(), 3);
    for (size_t i = 0; i < keep.size(); i++)
        for (int j = 0; j < 3; j++) (*F)(i, j) = rank[T(keep[i], j)];
    *boundaryMask = mask;  // pre-compaction indexing (the reference's quirk, 487)
    for (int p = 0; p < cnt; p++)
        if (std::abs(phiFun((*Vp)(p, 0), (*Vp)(p, 1))) < EPS) boundaryMask->at(p) = NodeType::BOUNDARY_FIXED;
}

// meshFromLevelSetFun 3D (src/MeshUtils.h:540-667), its hand-back and mask indexing repaired
inline void meshFromLevelSetFun(std::function<double(double, double, double)> phiFun, std::vector<int> &nVals,
                                std::vector<std::tuple<double, double>> &bb, Eigen::MatrixXd *Vc, Eigen::MatrixXd *Vp,
                                Eigen::MatrixXi *F, vector<NodeType> *boundaryMask, NodeType bType) {
    const double EPS = 1e-12;
    unordered_map<string, double> params;
    params["nx"] = nVals.at(0);
    params["ny"] = nVals.at(1);
    params["nz"] = nVals.at(2);
    params["xa"] = std::get<0>(bb.at(0));
    params["xb"] = std::get<1>(bb.at(0));
    params["ya"] = std::get<0>(bb.at(1));
    params["yb"] = std::get<1>(bb.at(1));
    params["za"] = std::get<0>(bb.at(2));
    params["zb"] = std::get<1>(bb.at(2));
    Eigen::MatrixXd G;
    Eigen::MatrixXi T;
    vector<NodeType> mask;
    generateUniformRectMesh<3>(params, &G, &T, &mask, bType);
    for (auto &m : mask) m = NodeType::INTERIOR;
    const int nP0 = G.rows(), nF0 = T.rows();
    std::vector<double> phi(nP0);
    for (int p = 0; p < nP0; p++) phi[p] = phiFun(G(p, 0), G(p, 1), G(p, 2));
    std::vector<int> keep;
    for (int s = 0; s < nF0; s++) {
        bool out = true;
        for (int j = 0; j < 4; j++) out = out && phi[T(s, j)] > -EPS;
        if (!out) keep.push_back(s);
    }
    std::vector<char> used(nP0, 0);
    for (int s : keep)
        for (int j = 0; j < 4; j++) used[T(s, j)] = 1;
    const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
    for (int p = 0; p < nP0; p++) {
        if (!used[p] || !(phi[p] > -EPS)) continue;
        const double x = G(p, 0), y = G(p, 1), z = G(p, 2);
        double n[3];  // interpolateBoundaryLocation 3D (388-402)
        n[0] = (phiFun(x + h, y, z) - phiFun(x - h, y, z)) / (2.0 * h);
        n[1] = (phiFun(x, y + h, z) - phiFun(x, y - h, z)) / (2.0 * h);
        n[2] = (phiFun(x, y, z + h) - phiFun(x, y, z - h)) / (2.0 * h);
        const double sq = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
        if (sq > 0) {
            const double nrm = sqrt(sq);
            for (int c = 0; c < 3; c++) n[c] = n[c] / nrm;
        }
        const double ph = phiFun(x, y, z);
        for (int c = 0; c < 3; c++) G(p, c) = G(p, c) - ph * n[c];
        mask[p] = bType;
    }
    std::vector<int> rank(nP0, -1);
    int cnt = 0;
    for (int p = nP0 - 1; p >= 0; p--)
        if (used[p]) rank[p] = cnt++;
    Vp->resize(cnt, 3);
    for (int p = 0; p < nP0; p++)
        if (used[p])
            for (int c = 0; c < 3; c++) (*Vp)(rank[p], c) = G(p, c);
    *Vc = *Vp;
    F->resize((Eigen::Index)keep.size(), 4);
    for (size_t i = 0; i < keep.size(); i++)
        for (int j = 0; j < 4; j++) (*F)(i, j) = rank[T(keep[i], j)];
    boundaryMask->assign(cnt, NodeType::INTERIOR);
    for (int p = 0; p < nP0; p++)
        if (used[p]) boundaryMask->at(rank[p]) = mask[p];
}

}  // namespace utils

#endif  // MESH_UTILS_H
