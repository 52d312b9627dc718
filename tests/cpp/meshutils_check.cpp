// meshutils_check.cpp -- include/mmadmm/MeshUtils.h (the reference's utils:: generators and reader,
// src/MeshUtils.h) against the library's C-ABI generators.  Test infrastructure
// (tests/test_cpp_dropin.py::test_meshutils_header); host only.
//   meshutils_check <dir-with-CircleEx24 files>
// prints one "name ok|FAIL detail" line per check.
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "MeshUtils.h"

static double circlePhi(double x, double y) {  // main.cpp:33-40
    double r = 0.35, cx = 0.5, cy = 0.5;
    double xval = (x - cx), yval = (y - cy);
    return sqrt(xval * xval + yval * yval) - r;
}
static double spherePhi(double x, double y, double z) {  // main.cpp:87-97
    double r = 0.4, cx = 0.5, cy = 0.5, cz = 0.5;
    double xval = (x - cx), yval = (y - cy), zval = (z - cz);
    return xval * xval + yval * yval + zval * zval - r * r;
}

static bool same(const Eigen::MatrixXd &V, const Eigen::MatrixXi &F, const vector<NodeType> &mask, mmadmm_mesh h,
                 std::string &why) {
    int dim = 0, nP = 0, nF = 0, ml = 0;
    mmadmm_mesh_sizes(h, &dim, &nP, &nF, &ml);
    std::vector<double> X((size_t)nP * dim);
    std::vector<int32_t> T((size_t)nF * (dim + 1)), m(ml);
    mmadmm_mesh_copy(h, X.data(), T.data(), m.data());
    mmadmm_mesh_free(h);
    if (V.rows() != nP || F.rows() != nF || (int)mask.size() != ml) {
        why = "sizes " + std::to_string(V.rows()) + "/" + std::to_string(nP) + " " + std::to_string(F.rows()) + "/" +
              std::to_string(nF) + " " + std::to_string(mask.size()) + "/" + std::to_string(ml);
        return false;
    }
    for (int i = 0; i < nP; i++)
        for (int c = 0; c < dim; c++)
            if (V(i, c) != X[(size_t)i * dim + c]) return why = "points", false;
    for (int i = 0; i < nF; i++)
        for (int c = 0; c <= dim; c++)
            if (F(i, c) != T[(size_t)i * (dim + 1) + c]) return why = "simplices", false;
    for (int i = 0; i < ml; i++)
        if ((int)mask[i] != m[i]) return why = "mask", false;
    return true;
}

static void report(const char *name, bool ok, const std::string &why) {
    std::printf("%s %s %s\n", name, ok ? "ok" : "FAIL", ok ? "" : why.c_str());
}

int main(int argc, char **argv) {
    std::string why;
    {  // linspace / findLimInfMeshPoint (MeshUtils.h:24-54), incl. the negative-guess clamp
        vector<double> x;
        utils::linspace(0.0, 1.0, 10, x);
        bool ok = x.size() == 11 && x[10] == 1.0 && x[3] == 0.0 + 3.0 * (1.0 - 0.0) / 10;
        ok = ok && utils::findLimInfMeshPoint(0.35, x) == 3 && utils::findLimInfMeshPoint(-0.2, x) == 9 &&
             utils::findLimInfMeshPoint(5.0, x) == 9;
        report("linspace_findLimInf", ok, "values");
    }
    for (int D = 2; D <= 3; D++) {  // generateUniformRectMesh (82-335)
        unordered_map<string, double> p{{"nx", 7}, {"ny", 7}, {"nz", 7}, {"xa", 0}, {"xb", 1}, {"ya", 0}, {"yb", 1},
                                        {"za", 0}, {"zb", 1}};
        Eigen::MatrixXd V;
        Eigen::MatrixXi F;
        vector<NodeType> mask;
        if (D == 2) utils::generateUniformRectMesh<2>(p, &V, &F, &mask, NodeType::BOUNDARY_FIXED);
        else utils::generateUniformRectMesh<3>(p, &V, &F, &mask, NodeType::BOUNDARY_FIXED);
        mmadmm_mesh h = nullptr;
        mmadmm_mesh_rect(D, 7, 7, D == 3 ? 7 : 0, 0, 1, 0, 1, 0, 1, MMADMM_BOUNDARY_FIXED, &h);
        report(D == 2 ? "rect2d" : "rect3d", same(V, F, mask, h, why), why);
    }
    {  // meshFromLevelSetFun 2D (404-538) with circlePhi == mmadmm_mesh_levelset2d, reference mask
        vector<int> n{40, 40};
        vector<std::tuple<double, double>> bb{{0.0, 1.0}, {0.0, 1.0}};
        Eigen::MatrixXd Vc, V;
        Eigen::MatrixXi F;
        vector<NodeType> mask;
        utils::meshFromLevelSetFun(circlePhi, n, bb, &Vc, &V, &F, &mask, NodeType::BOUNDARY_FIXED);
        mmadmm_mesh h = nullptr;
        mmadmm_mesh_levelset2d(40, 40, 0, 1, 0, 1, MMADMM_BOUNDARY_FIXED, 0, &h);
        report("levelset2d", same(V, F, mask, h, why), why);
    }
    {  // meshFromLevelSetFun 3D (540-667) with spherePhi == mmadmm_mesh_levelset3d (repaired)
        vector<int> n{12, 12, 12};
        vector<std::tuple<double, double>> bb{{0.0, 1.0}, {0.0, 1.0}, {0.0, 1.0}};
        Eigen::MatrixXd Vc, V;
        Eigen::MatrixXi F;
        vector<NodeType> mask;
        utils::meshFromLevelSetFun(spherePhi, n, bb, &Vc, &V, &F, &mask, NodeType::BOUNDARY_FIXED);
        mmadmm_mesh h = nullptr;
        mmadmm_mesh_levelset3d(12, 12, 12, 0, 1, 0, 1, 0, 1, MMADMM_BOUNDARY_FIXED, 1, &h);
        bool ok = same(V, F, mask, h, why) && Vc.rows() == V.rows();
        report("levelset3d", ok, why);
    }
    {  // removeRow (338-346)
        Eigen::MatrixXi M(4, 2);
        for (int i = 0; i < 4; i++) M(i, 0) = i, M(i, 1) = 10 * i;
        utils::removeRow(M, 1);
        report("removeRow", M.rows() == 3 && M(1, 0) == 2 && M(2, 1) == 30, "rows");
    }
    if (argc > 1) {  // readTriangles (669-733): the file's rows, the mask plus the extra EOF entry
        const std::string d = argv[1];
        Eigen::MatrixXi F;
        Eigen::MatrixXd V;
        vector<NodeType> mask;
        utils::readTriangles(2, (d + "/CircleEx24triangles.txt").c_str(), (d + "/CircleEx24points.txt").c_str(),
                             (d + "/CircleEx24mask.txt").c_str(), F, V, mask);
        report("readTriangles", V.rows() == 2084 && F.rows() == 4015 && (int)mask.size() == 2085, "sizes");
    }
    return 0;
}
