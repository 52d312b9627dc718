// Mesh.h -- the reference's Mesh<D> (src/Mesh.h:14-104) over the C-ABI of libmmadmm.so.
//
// Same constructors and argument meaning as src/Mesh.h:22-25:
//   Mesh(Xc, Xp, F, boundaryMask, Mon, numThreads, rho, w, tau, integrationMode, gradUse)
//   Mesh(Xp, F, boundaryMask, Mon, numThreads, rho, w, tau, integrationMode, gradUse)
// and the reference's ownership (src/Mesh.cpp:384-494): the mesh keeps non-owning pointers to
// the caller's Xp/Xc/F/mask and monitor, re-orients the caller's F in place (reOrientElements,
// src/Mesh.cpp:243-260) and writes the node positions back into the caller's Xp after every ADMM
// step and at done() (updateAfterStep, src/Mesh.cpp:1016-1036).  w is ignored, as in the reference
// (w = 0.5 sqrt(rho), src/Mesh.cpp:451); numThreads sized the reference's OpenMP pool and has
// no role on the device.  The device state lives in the engine that MeshIntegrator<D> creates
// (the C-ABI needs dt, which the reference gives the integrator).
//
// Header-only; link with -lmmadmm.  Eigen: the real library or include/mmadmm/eigen_shim.
// Errors: the reference asserts (inverted element, src/AdaptationFunctional.cpp:174) or exits;
// here they are thrown as mmadmm_cxx::Error carrying the C-ABI status code.
#ifndef MESH_H
#define MESH_H

#include <Eigen/Dense>
#include <stdexcept>
#include <string>
#include <vector>

#include "../mmadmm.h"
#include "MonitorFunction.h"
#include "NodeType.h"

using namespace std;

namespace mmadmm_cxx {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string &what) : std::runtime_error(what), code(code) {}
    int code;
};

inline void check(int rc) {
    if (rc != MMADMM_OK) throw Error(rc, mmadmm_last_error());
}

// MonitorFunction<D>::operator() behind the C-ABI's monitor callback (row-major tensor, as
// evaluateAtVertices flattens it, src/MonitorFunction.cpp:16-32; M zeroed before the call)
template <int D>
void monitor_trampoline(int dim, const double *x, double *M, void *user) {
    (void)dim;
    MonitorFunction<D> *mon = static_cast<MonitorFunction<D> *>(user);
    Eigen::Vector<double,D> xv;
    for (int c = 0; c < D; c++) xv(c) = x[c];
    Eigen::Matrix<double,D,D> Mv;
    Mv.setZero();
    (*mon)(xv, Mv);
    for (int i = 0; i < D*D; i++) M[i] = Mv(i/D, i%D);
}

}  // namespace mmadmm_cxx

template <int D> class MeshIntegrator;

template <int D=-1>
class Mesh {
public:
    int integrationMode;
    int gradUse;
    bool compMesh = true;
    double rho, tau;
    Eigen::MatrixXd *Vc;
    Eigen::MatrixXd *Vp;
    Eigen::MatrixXi *F;
    vector<NodeType> *boundaryMask;
    MonitorFunction<D> *Mon;

    Mesh(Eigen::MatrixXd &Xc, Eigen::MatrixXd &Xp, Eigen::MatrixXi &F, vector<NodeType> &boundaryMask,
            MonitorFunction<D> *M, int numThreads, double rho, double w, double tau, int integrationMode, bool gradUse) {
        meshInit(&Xc, Xp, F, boundaryMask, M, numThreads, rho, w, tau, integrationMode, gradUse);
    }
    Mesh(Eigen::MatrixXd &Xp, Eigen::MatrixXi &F, vector<NodeType> &boundaryMask,
            MonitorFunction<D> *M, int numThreads, double rho, double w, double tau, int integrationMode, bool gradUse) {
        meshInit(nullptr, Xp, F, boundaryMask, M, numThreads, rho, w, tau, integrationMode, gradUse);
    }
    ~Mesh() {}

    int getNPnts() { return (int)Vp->rows(); }

    // Mesh::outputSimplices / outputPoints (src/Mesh.cpp:1067-1095): "a, b, c" rows, default
    // ostream formatting
    void outputSimplices(const char *fname) {
        std::vector<int32_t> f = rowMajor(*F);
        mmadmm_cxx::check(mmadmm_write_simplices(fname, D, (int)F->rows(), f.data()));
    }
    void outputPoints(const char *fname) {
        std::vector<double> x = rowMajor(*Vp);
        mmadmm_cxx::check(mmadmm_write_points(fname, D, (int)Vp->rows(), x.data()));
    }

    template <typename Mat>
    static std::vector<typename Mat::Scalar> rowMajor(const Mat &m) {
        std::vector<typename Mat::Scalar> out((size_t)m.rows() * m.cols());
        for (int i = 0; i < (int)m.rows(); i++)
            for (int j = 0; j < (int)m.cols(); j++) out[(size_t)i * m.cols() + j] = m(i, j);
        return out;
    }

private:
    friend class MeshIntegrator<D>;
    mmadmm_handle h_ = nullptr;  // set by MeshIntegrator<D>

    void meshInit(Eigen::MatrixXd *Xc, Eigen::MatrixXd &Xp, Eigen::MatrixXi &F_, vector<NodeType> &mask,
            MonitorFunction<D> *M, int numThreads, double rho_, double w, double tau_, int mode, bool gradUse_) {
        static_assert(D == 2 || D == 3, "Mesh<D>: D must be 2 or 3");
        (void)numThreads;
        (void)w;
        if ((int)Xp.cols() != D || (int)F_.cols() != D + 1)
            throw mmadmm_cxx::Error(MMADMM_ERR_INVALID, "Mesh: Xp must be nP x D and F nF x (D+1)");
        Vc = Xc;
        Vp = &Xp;
        F = &F_;
        boundaryMask = &mask;
        Mon = M;
        rho = rho_;
        tau = tau_;
        integrationMode = mode;
        gradUse = gradUse_;
        compMesh = (Xc != nullptr);
        // reOrientElements (src/Mesh.cpp:243-260) on the caller's F
        std::vector<double> x = rowMajor(Xp);
        std::vector<int32_t> f = rowMajor(F_);
        mmadmm_cxx::check(mmadmm_mesh_reorient(D, (int)Xp.rows(), x.data(), (int)F_.rows(), f.data()));
        for (int i = 0; i < (int)F_.rows(); i++)
            for (int j = 0; j < D + 1; j++) F_(i, j) = f[(size_t)i * (D + 1) + j];
    }

    // updateAfterStep (src/Mesh.cpp:1016-1036): Vp = x
    void updateAfterStep() {
        std::vector<double> x((size_t)Vp->rows() * D);
        mmadmm_cxx::check(mmadmm_get(h_, "points", x.data()));
        for (int i = 0; i < (int)Vp->rows(); i++)
            for (int j = 0; j < D; j++) (*Vp)(i, j) = x[(size_t)i * D + j];
    }
};

#endif
