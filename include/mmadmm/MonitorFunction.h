// MonitorFunction.h -- the reference's monitor plugin interface (src/MonitorFunction.h:9-21):
// subclass it and override operator()(x, M) to fill the D x D monitor tensor at x.  User monitors
// written for the reference (Experiments/TestMonitors/MEx*.h) compile unchanged against it; they
// reach the engine through the adapter in include/mmadmm/Mesh.h, which calls operator() on the
// host at set-up (the reference evaluates the monitor once, src/MeshInterpolator.cpp:254).
//
// Same include guard as the reference's header: a plugin that includes the reference's
// "../../src/MonitorFunction.h" and a driver that includes this one see one class definition,
// whichever comes first (the two declare the same class).
#ifndef MONITOR_FUNCTION_H
#define MONITOR_FUNCTION_H

#include <Eigen/Dense>
#include <vector>

using namespace std;

template <int D>
class MonitorFunction {
protected:
public:
    virtual void operator()(Eigen::Vector<double,D> &x, Eigen::Matrix<double,D,D> &M) = 0;
    virtual ~MonitorFunction() {};
    // MonitorFunction<D>::evaluateAtVertices (src/MonitorFunction.cpp:16-32): row v of M is the
    // row-major flattened tensor at vertex v (M is nP x D*D)
    void evaluateAtVertices(Eigen::MatrixXd &X, Eigen::MatrixXi &F, Eigen::MatrixXd &M) {
        (void)F;
        Eigen::Matrix<double,D,D> monTemp;
        Eigen::Vector<double,D> xTemp;
        for (int vId = 0; vId < X.rows(); vId++) {
            monTemp.setZero();
            for (int c = 0; c < D; c++) xTemp(c) = X(vId, c);
            (*this)(xTemp, monTemp);
            for (int i = 0; i < D*D; i++) M(vId, i) = monTemp(i/D, i%D);
        }
    }
    void evaluateAtPoint(Eigen::MatrixXd &X, Eigen::MatrixXi &F, Eigen::MatrixXd &M) {
        evaluateAtVertices(X, F, M);
    }
};

#endif
