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
//   dropin_driver be <dim> <n> <MonType> <dt> <tau> <rho> <nSteps> <DtTol> [engine]
//       runAlgo with Method 2, the backward Euler step driven from the host through the LASolver
//       classes of include/mmadmm/MatrixIter.h in the reference's own call sequence --
//       Mesh<D>::buildMatrix (src/Mesh.cpp:262-382: ParamIter fields, MatrixStruc + set_entry over
//       every simplex's rotated vertex list, pack, MatrixIter(MatrixStruc&), tol/rhs arrays) and
//       Mesh<D>::backwardsEulerStep (1263-1341: sfac, set_toler, bValue, solve, assert(cgIter > 0)),
//       with the gradient and the FSubJac sums from the engine (mmadmm_be_*); prints "t, Ih" rows
//       and the Newton/CG-STAB counts.  "engine": the engine's own mmadmm_backward_euler_step.
#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "Mesh.h"
#include "MeshIntegrator.h"
#include "SparseItObj.h"

using namespace SparseItObj;  // as src/Mesh.h:14
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

// Mesh<D>'s backward-Euler state (src/Mesh.h: jac, cgParams, tol, rhs, stepTaken) over one engine
template <int D>
struct HostBackwardEuler {
    mmadmm_handle h = nullptr;
    int nP = 0;
    std::vector<int32_t> F;  // re-oriented simplices (the engine's)
    double tau = 0;
    ParamIter *cgParams = nullptr;
    MatrixIter *jac = nullptr;
    double *tol = nullptr, *rhs = nullptr;
    bool stepTaken = false;
    long long newton = 0, cg = 0;

    // Mesh<D>::buildMatrix (src/Mesh.cpp:262-382)
    void buildMatrix() {
        cgParams = new ParamIter();
        const int ILU_LEVEL = 0;
        cgParams->order = 0;
        cgParams->level = ILU_LEVEL;
        cgParams->drop_ilu = 0;
        cgParams->iscal = 0;
        cgParams->nitmax = 10000;
        cgParams->ipiv = 0;
        cgParams->resid_reduc = 1.e-6;
        cgParams->info = 0;
        cgParams->drop_tol = 1.e-3;
        cgParams->new_rhat = 0;
        cgParams->iaccel = 0;
        cgParams->north = 10;
        MatrixStruc *matrixBuilder = new MatrixStruc(D * nP, 0);
        const int nF = (int)F.size() / (D + 1);
        for (int i = 0; i < nF; i++) {
            std::vector<int> pntList(F.begin() + (size_t)i * (D + 1), F.begin() + (size_t)(i + 1) * (D + 1));
            for (int iter = 0; iter < D + 1; iter++) {  // every vertex's D rows against all D+1 vertices
                const int rowStart = pntList.at(0) * D;
                for (int n = 0; n < D + 1; n++) {
                    const int colStart = pntList.at(n) * D;
                    for (int r = rowStart; r < rowStart + D; r++)
                        for (int c = colStart; c < colStart + D; c++) matrixBuilder->set_entry(r, c);
                }
                std::rotate(pntList.begin(), pntList.begin() + 1, pntList.end());
            }
        }
        matrixBuilder->pack();
        jac = new MatrixIter(*matrixBuilder);
        delete matrixBuilder;
        const int nPts = D * nF;  // the reference sizes tol and rhs by D * F->rows() (>= D * nP)
        tol = new double[nPts];
        rhs = new double[nPts];
        for (int i = 0; i < nPts; i++) tol[i] = rhs[i] = 0.0;
    }

    // buildEulerJac (src/Mesh.cpp:1112-1136): zero, the FSubJac sums (device), a *= dt/tau, +1 diag
    void buildEulerJac(double dt) {
        for (int r = 0; r < D * nP; r++)
            for (int i = jac->rowBegin(r); i < jac->rowEndPlusOne(r); i++) jac->aValue(i) = 0;
        std::vector<double> sums(jac->rowEndPlusOne(D * nP - 1));
        mmadmm_cxx::check(mmadmm_be_fsubjac(h, sums.data()));
        for (size_t k = 0; k < sums.size(); k++) jac->aValue((int)k) += sums[k];
        for (int r = 0; r < D * nP; r++)
            for (int i = jac->rowBegin(r); i < jac->rowEndPlusOne(r); i++) {
                const int colIndex = jac->getColIndex(i);
                jac->aValue(i) *= (dt / tau);
                if (colIndex == r) jac->aValue(i) += 1.0;
            }
    }

    // Mesh<D>::backwardsEulerStep (src/Mesh.cpp:1263-1341)
    double backwardsEulerStep(double dt, double tolN) {
        const double SAFETY_FAC = 1.0 / 10.0;
        double Ih = 0;
        mmadmm_cxx::check(mmadmm_be_begin(h, dt, &Ih));  // xn = x; Ih = eulerStepMod(x); x -= dt/tau grad
        const int MAX_ITERS = 1000;
        int nIter = 0;
        double gradOneN = 0, gradOneNPrev = INFINITY;
        std::vector<double> grad(D * nP);
        if (!stepTaken) {
            buildEulerJac(dt);
            jac->sfac(*cgParams);
        }
        do {
            mmadmm_cxx::check(mmadmm_be_residual(h, dt, grad.data(), &gradOneN, &Ih));  // F, ||F||_1
            if (gradOneN < SAFETY_FAC * tolN) break;
            if (!stepTaken || std::abs(gradOneN - gradOneNPrev) / (gradOneN) < 0.25) {
                buildEulerJac(dt);
                if (!stepTaken) jac->sfac(*cgParams);
                jac->set_toler(this->tol);
                stepTaken = true;
            }
            int cgIter = 0;
            for (size_t i = 0; i < grad.size(); i++) jac->bValue((int)i) = -grad[i];
            jac->solve(*cgParams, rhs, cgIter);
            mmadmm_cxx::check(mmadmm_be_add(h, rhs));  // x += dx
            if (!(cgIter > 0)) throw mmadmm_cxx::Error(MMADMM_ERR_NOCONV, "assert(cgIter > 0)");
            cg += cgIter;
            nIter++;
            gradOneNPrev = gradOneN;
        } while (nIter < MAX_ITERS);
        newton += nIter;
        return Ih;
    }
};

// runAlgo (main.cpp:142-255) with Method 2 on a SquareGrid mesh
template <int D>
int runBE(int n, int monType, double dt, double tau, double rho, int nSteps, double dtTol, bool engineOwn) {
    RectMesh m = rect(D, n);
    MonitorFunction<D> *mon = registry<D>().at(monType);
    mmadmm_params p{};
    p.dt = dt;
    p.tau = tau;
    p.rho = rho;
    p.device = -1;
    p.nranks = 1;
    HostBackwardEuler<D> be;
    be.nP = m.nP;
    be.tau = tau;
    mmadmm_cxx::check(mmadmm_create(D, m.nP, m.X.data(), nullptr, m.nF, m.F.data(), m.mask.data(), &p,
                                    &mmadmm_cxx::monitor_trampoline<D>, mon, &be.h));
    be.F.resize(m.F.size());
    mmadmm_cxx::check(mmadmm_get_simplices(be.h, be.F.data()));
    be.buildMatrix();
    double E0 = 0;
    mmadmm_cxx::check(mmadmm_energy(be.h, &E0));
    std::vector<double> Ivals{E0};
    double Ihprev = INFINITY;
    for (int i = 0; i < nSteps; i++) {
        double Ih = 0;
        if (engineOwn) {
            int newton = 0;
            mmadmm_cxx::check(mmadmm_backward_euler_step(be.h, dt, 1e-3, &Ih, &newton));
            be.newton += newton;
        } else {
            Ih = be.backwardsEulerStep(dt, 1e-3);
        }
        Ivals.push_back(Ih);
        if (i != 0 && std::abs((Ih - Ihprev) / dt) < dtTol) break;
        Ihprev = Ih;
    }
    if (!engineOwn) {  // the pattern the mirror built is the engine's buildMatrix pattern
        long long nnz = 0;
        mmadmm_cxx::check(mmadmm_get_jacobian(be.h, &nnz, nullptr, nullptr, nullptr));
        std::vector<int32_t> ia(D * m.nP + 1), ja(nnz);
        mmadmm_cxx::check(mmadmm_get_jacobian(be.h, &nnz, ia.data(), ja.data(), nullptr));
        const bool same = std::equal(ia.begin(), ia.end(), be.jac->get_ia()) &&
                          std::equal(ja.begin(), ja.end(), be.jac->get_ja());
        std::printf("pattern %s nnz %lld\n", same ? "equal" : "DIFFERS", nnz);
    }
    for (size_t i = 0; i < Ivals.size(); i++) std::printf("%zu, %.17g\n", i, Ivals[i]);
    std::vector<double> x((size_t)m.nP * D);
    mmadmm_cxx::check(mmadmm_get(be.h, "x", x.data()));
    unsigned long long hsh = 1469598103934665603ull;  // FNV-1a over the node positions' bits
    for (double v : x) {
        unsigned long long b;
        std::memcpy(&b, &v, 8);
        for (int k = 0; k < 8; k++) hsh = (hsh ^ ((b >> (8 * k)) & 0xff)) * 1099511628211ull;
    }
    std::printf("newton %lld cg %lld xhash %016llx\n", be.newton, be.cg, hsh);
    mmadmm_destroy(be.h);
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
        if (mode == "be" && (argc == 10 || argc == 11)) {
            const int dim = std::atoi(argv[2]), n = std::atoi(argv[3]), mt = std::atoi(argv[4]);
            const double dt = std::atof(argv[5]), tau = std::atof(argv[6]), rho = std::atof(argv[7]);
            const int nSteps = std::atoi(argv[8]);
            const double dtTol = std::atof(argv[9]);
            const bool own = argc == 11 && std::string(argv[10]) == "engine";
            return dim == 2 ? runBE<2>(n, mt, dt, tau, rho, nSteps, dtTol, own)
                            : runBE<3>(n, mt, dt, tau, rho, nSteps, dtTol, own);
        }
        std::fprintf(stderr, "usage: dropin_driver grid <dim> <n> | run <dim> <n> <MonType> <dt> <tau> <rho> "
                             "<AdmmIter> <nSteps> <DtTol> <outdir> | be <dim> <n> <MonType> <dt> <tau> <rho> "
                             "<nSteps> <DtTol> [engine]\n");
        return 2;
    } catch (const mmadmm_cxx::Error &e) {
        std::fprintf(stderr, "mmadmm error %d: %s\n", e.code, e.what());
        return 3;
    } catch (const SparseItObj::General_Exception &e) {
        std::fprintf(stderr, "LASolver error: %s\n", e.p);
        return 4;
    }
}
