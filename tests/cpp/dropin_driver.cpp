// dropin_driver.cpp -- a main.cpp-style driver (reference main.cpp:142-255, 784-907) built against
// the C++ drop-in surface include/mmadmm/{Mesh,MeshIntegrator,MonitorFunction,NodeType}.h and the
// reference's own monitor plugins, Experiments/TestMonitors/MEx*.h, compiled UNCHANGED from where
// they lie (-I <reference>/Experiments/TestMonitors).  Test infrastructure (tests/test_cpp_dropin.py).
//
//   dropin_driver grid <dim> <n>
//       For every MonType of main.cpp's registry (Mvals / Mvals3D, main.cpp:836-864): the monitor
//       grid of the n x n (x n) SquareGrid mesh built from the MEx plugin through the
//       MonitorFunction<D> adapter, and from the engine's built-in restatement; prints
//       "montype <k> rows <r> diff <count>" per type (host only, no device).
//   dropin_driver run <dim> <n> <MonType> <dt> <tau> <rho> <AdmmIter> <nSteps> <DtTol> <outdir>
//       runAlgo (main.cpp:142-255) with Mesh<D> / MeshIntegrator<D>: prints "t, Ih" rows and
//       writes <outdir>/points.txt and <outdir>/triangles.txt (needs a GPU).
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "Mesh.h"
#include "MeshIntegrator.h"
#include "MEx0.h"
#include "MEx1.h"
#include "MEx2.h"
#include "MEx3.h"
#include "MEx4.h"
#include "MEx5.h"
#include "MEx13D.h"
#include "MEx23D.h"
#include "MEx33D.h"
#include "MEx53D.h"

template <int D>
std::vector<MonitorFunction<D> *> registry();
template <>
std::vector<MonitorFunction<2> *> registry<2>() {  // Mvals (main.cpp:836-855)
    return {new MEx0<2>(), new MEx1<2>(), new MEx2<2>(), new MEx3<2>(), new MEx4<2>(), new MEx5<2>()};
}
template <>
std::vector<MonitorFunction<3> *> registry<3>() {  // Mvals3D (main.cpp:842-863)
    auto *m0 = new MEx0<3>();
    return {m0, new MEx13D<3>(), new MEx23D<3>(), new MEx33D<3>(), m0, new MEx53D<3>()};
}

struct RectMesh {
    int dim, nP, nF;
    std::vector<double> X;
    std::vector<int32_t> F, mask;
};

static RectMesh rect(int dim, int n) {
    mmadmm_mesh h = nullptr;
    mmadmm_cxx::check(mmadmm_mesh_rect(dim, n, n, dim == 3 ? n : 0, 0, 1, 0, 1, 0, 1, MMADMM_BOUNDARY_FIXED, &h));
    RectMesh m;
    int ml = 0;
    mmadmm_cxx::check(mmadmm_mesh_sizes(h, &m.dim, &m.nP, &m.nF, &ml));
    m.X.resize((size_t)m.nP * dim);
    m.F.resize((size_t)m.nF * (dim + 1));
    m.mask.resize(ml);
    mmadmm_cxx::check(mmadmm_mesh_copy(h, m.X.data(), m.F.data(), m.mask.data()));
    mmadmm_mesh_free(h);
    return m;
}

template <int D>
int grids(int n) {
    RectMesh m = rect(D, n);
    auto mons = registry<D>();
    for (int k = 0; k < (int)mons.size(); k++) {
        int rows = 0, rows2 = 0;
        mmadmm_cxx::check(mmadmm_monitor_grid(D, m.nP, m.X.data(), &mmadmm_cxx::monitor_trampoline<D>, mons[k],
                                              &rows, nullptr));
        std::vector<double> user((size_t)rows * D * D), builtin((size_t)rows * D * D);
        mmadmm_cxx::check(mmadmm_monitor_grid(D, m.nP, m.X.data(), &mmadmm_cxx::monitor_trampoline<D>, mons[k],
                                              &rows, user.data()));
        mmadmm_monitor_fn fn = nullptr;
        void *u = nullptr;
        mmadmm_cxx::check(mmadmm_builtin_monitor(D, k, &fn, &u));
        mmadmm_cxx::check(mmadmm_monitor_grid(D, m.nP, m.X.data(), fn, u, &rows2, builtin.data()));
        long long diff = 0;
        for (size_t i = 0; i < user.size(); i++) diff += (user[i] != builtin[i]) || std::signbit(user[i]) != std::signbit(builtin[i]);
        std::printf("montype %d rows %d diff %lld\n", k, rows, diff + (rows != rows2));
    }
    return 0;
}

// runAlgo (main.cpp:142-255) on a SquareGrid mesh, through the reference's classes
template <int D>
int run(int n, int monType, double dt, double tau, double rho, int admmIter, int nSteps, double dtTol,
        const std::string &outDir) {
    RectMesh m = rect(D, n);
    Eigen::MatrixXd Vp(m.nP, D);
    Eigen::MatrixXi F(m.nF, D + 1);
    vector<NodeType> boundaryMask(m.nP);
    for (int i = 0; i < m.nP; i++) {
        for (int j = 0; j < D; j++) Vp(i, j) = m.X[(size_t)i * D + j];
        boundaryMask[i] = (NodeType)m.mask[i];
    }
    for (int i = 0; i < m.nF; i++)
        for (int j = 0; j < D + 1; j++) F(i, j) = m.F[(size_t)i * (D + 1) + j];
    MonitorFunction<D> *mon = registry<D>().at(monType);
    double w = 3.53553390593;  // the JSON's w: ignored, as in the reference
    Mesh<D> adaptiveMesh(Vp, F, boundaryMask, mon, 1, rho, w, tau, 0, false);
    MeshIntegrator<D> solver(dt, adaptiveMesh);
    std::vector<double> Ivals{solver.getEnergy()};
    double Ihprev = INFINITY;
    for (int i = 0; i < nSteps; i++) {
        double Ih = solver.step(admmIter, 1e-3);
        Ivals.push_back(Ih);
        if (i != 0 && std::abs((Ih - Ihprev) / dt) < dtTol) break;
        Ihprev = Ih;
    }
    solver.done();
    adaptiveMesh.outputPoints((outDir + "/points.txt").c_str());
    adaptiveMesh.outputSimplices((outDir + "/triangles.txt").c_str());
    for (size_t i = 0; i < Ivals.size(); i++) std::printf("%zu, %.17g\n", i, Ivals[i]);
    return 0;
}

int main(int argc, char **argv) {
    try {
        const std::string mode = argc > 1 ? argv[1] : "";
        if (mode == "grid" && argc == 4) {
            const int dim = std::atoi(argv[2]), n = std::atoi(argv[3]);
            return dim == 2 ? grids<2>(n) : grids<3>(n);
        }
        if (mode == "run" && argc == 12) {
            const int dim = std::atoi(argv[2]), n = std::atoi(argv[3]), mt = std::atoi(argv[4]);
            const double dt = std::atof(argv[5]), tau = std::atof(argv[6]), rho = std::atof(argv[7]);
            const int admm = std::atoi(argv[8]), nSteps = std::atoi(argv[9]);
            const double dtTol = std::atof(argv[10]);
            return dim == 2 ? run<2>(n, mt, dt, tau, rho, admm, nSteps, dtTol, argv[11])
                            : run<3>(n, mt, dt, tau, rho, admm, nSteps, dtTol, argv[11]);
        }
        std::fprintf(stderr, "usage: dropin_driver grid <dim> <n> | run <dim> <n> <MonType> <dt> <tau> <rho> "
                             "<AdmmIter> <nSteps> <DtTol> <outdir>\n");
        return 2;
    } catch (const mmadmm_cxx::Error &e) {
        std::fprintf(stderr, "mmadmm error %d: %s\n", e.code, e.what());
        return 3;
    }
}
