// MeshIntegrator.h -- the reference's MeshIntegrator<D> (src/MeshIntegrator.h:12-51) over the
// C-ABI of libmmadmm.so.
//
//   MeshIntegrator(double dt, Mesh<D> &a)      src/MeshIntegrator.cpp:15-62 -> mmadmm_create
//   double step(int nIters, double tol)         src/MeshIntegrator.cpp:101-191 -> mmadmm_step
//   double eulerStep(double tol)                src/MeshIntegrator.cpp:87-94 -> mmadmm_euler_step
//   double backwardsEulerStep(double dt, double tol)
//                                               src/MeshIntegrator.cpp:68-76 -> mmadmm_backward_euler_step
//   double getEnergy()                          src/MeshIntegrator.cpp:79-81 -> mmadmm_energy
//   void done()                                 src/MeshIntegrator.cpp:193-196 -> mmadmm_done
//   void outputX / outputZ(const char *fname)   src/MeshIntegrator.cpp:218-246
//   double proxTime, predTime, multTime, cgTime public timers (wall seconds; the device does the
//                                               whole step, so proxTime holds step() time)
// step() writes the positions back into the Mesh's Xp after every step, as the reference's
// updateAfterStep does; eulerStep/backwardsEulerStep leave Xp to done(), as in the reference.
// One integrator per Mesh (the reference's is not re-entrant either).
#ifndef SOLVER_H
#define SOLVER_H

#include <chrono>
#include <cmath>
#include <string>
#include <vector>

#include "Mesh.h"

using namespace std;

template <int D>
class MeshIntegrator {
public:
    MeshIntegrator(double dt, Mesh<D> &a) : a(&a), dt(dt), dtPrev(dt) {
        if (a.h_) throw mmadmm_cxx::Error(MMADMM_ERR_INVALID, "MeshIntegrator: the Mesh already has an integrator");
        std::vector<double> xp = Mesh<D>::rowMajor(*a.Vp), xc;
        if (a.compMesh) xc = Mesh<D>::rowMajor(*a.Vc);
        std::vector<int32_t> f = Mesh<D>::rowMajor(*a.F);
        const int nP = (int)a.Vp->rows();
        std::vector<int32_t> mask(nP);
        for (int i = 0; i < nP; i++) mask[i] = (int32_t)a.boundaryMask->at(i);
        mmadmm_params p{};
        p.dt = dt;
        p.tau = a.tau;
        p.rho = a.rho;
        p.grad_use = a.gradUse ? 1 : 0;
        p.device = -1;
        p.rank = 0;
        p.nranks = 1;
        mmadmm_cxx::check(mmadmm_create(D, nP, xp.data(), a.compMesh ? xc.data() : nullptr, (int)a.F->rows(), f.data(),
                                        mask.data(), &p, &mmadmm_cxx::monitor_trampoline<D>, a.Mon, &a.h_));
        h_ = a.h_;
    }
    ~MeshIntegrator() {
        if (h_) mmadmm_destroy(h_);
        if (a) a->h_ = nullptr;
    }
    MeshIntegrator(const MeshIntegrator &) = delete;
    MeshIntegrator &operator=(const MeshIntegrator &) = delete;

    double step(int nIters, double tol) {
        const auto t0 = std::chrono::steady_clock::now();
        double Ih = 0;
        int iters = 0;
        mmadmm_cxx::check(mmadmm_step(h_, nIters, tol, &Ih, &iters));
        a->updateAfterStep();
        proxTime += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        stepsTaken++;
        energyCur = Ih;
        return Ih;
    }
    double eulerStep(double tol) {
        (void)tol;
        double Ih = 0;
        mmadmm_cxx::check(mmadmm_euler_step(h_, &Ih));
        stepsTaken++;
        return Ih;
    }
    double backwardsEulerStep(double dtStep, double tol) {
        double Ih = 0;
        int newton = 0;
        mmadmm_cxx::check(mmadmm_backward_euler_step(h_, dtStep, tol, &Ih, &newton));
        stepsTaken++;
        return Ih;
    }
    // the reference's commented Mesh<D>::setUp hook (src/Mesh.cpp:1006-1014): rebuild the monitor
    // grid from the current mesh at the start of every step (no reference counterpart; off by default)
    void setTimeVarying(bool on) { mmadmm_cxx::check(mmadmm_set_regrid(h_, on ? 1 : 0)); }

    double getEnergy() {
        double E = 0;
        mmadmm_cxx::check(mmadmm_energy(h_, &E));
        return E;
    }
    void done() {
        mmadmm_cxx::check(mmadmm_done(h_));
        a->updateAfterStep();
    }
    void outputX(const char *fname) { output("x", fname); }
    void outputZ(const char *fname) { output("z", fname); }

    double proxTime = 0;
    double multTime = 0;
    double cgTime = 0;
    double predTime = 0;
    Mesh<D> *a;
    double dt;
    double dtPrev;
    double energyCur = INFINITY;
    int stepsTaken = 0;

private:
    mmadmm_handle h_ = nullptr;

    void output(const char *what, const char *fname) {
        int nP = 0, nF = 0, rows = 0;
        mmadmm_cxx::check(mmadmm_sizes(h_, &nP, &nF, &rows));
        const size_t n = (what[0] == 'x') ? (size_t)nP * D : (size_t)nF * D * (D + 1);
        std::vector<double> v(n);
        mmadmm_cxx::check(mmadmm_get(h_, what, v.data()));
        mmadmm_cxx::check(mmadmm_write_points(fname, D, (int)(n / D), v.data()));
    }
};

#endif
