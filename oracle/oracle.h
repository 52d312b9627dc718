/*
 * oracle.h -- C API of the CPU restatement of connortannahill/MM-ADMM's ADMM path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so.  The product (mm-admm_amd/) never links,
 * imports or executes anything under oracle/; it fails loudly when its own HIP
 * library is missing.
 *
 * The oracle restates (plain C++17, no Eigen, no nanoflann) the reference files
 *   src/AdaptationFunctional.cpp:102-287   (blockGrad)
 *   src/Mesh.cpp:243-260, 496-674, 676-772, 777-872, 930-1036
 *   src/MeshIntegrator.cpp:15-62, 68-94, 101-191
 *   src/MeshInterpolator.cpp:68-130, 166-259, 287-342, 366-404
 *   src/MonitorFunction.cpp:16-32, Experiments/TestMonitors/MEx*.h
 *   src/MeshUtils.h:24-80, 82-335, 404-538, 669-733
 * Pinned against the reference's own committed artifacts (Experiments/Results/
 * * /Ih0.txt t=0 energies and full energy traces, 6 significant digits); see
 * tests/test_oracle_pins.py.  Eigen's internal summation orders are unpinned
 * (Eigen is un-vendored); DESIGN.md §Oracle lists the conventions used.
 */
#ifndef MMADMM_ORACLE_H
#define MMADMM_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

/* ---- meshes (generators + file reader), returned as an opaque handle ---- */
void orc_set_threads(int n);
void* orc_mesh_rect(int dim, int nx, int ny, int nz, double xa, double xb, double ya,
                    double yb, double za, double zb, int btype);
void* orc_mesh_levelset2d(int nx, int ny, double xa, double xb, double ya, double yb,
                          int btype, int compactMask);
// MeshUtils.h:540-667 + main.cpp:87-97 (3D, spherePhi) with the pointer hand-back repaired
void* orc_mesh_levelset3d(int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za,
                          double zb, int btype, int compactMask);
void* orc_mesh_read(int dim, const char* tri, const char* pnts, const char* mask);
void orc_mesh_sizes(void* m, int* nP, int* nF, int* maskLen);
void orc_mesh_copy(void* m, double* Vp, int* F, int* mask);
void orc_mesh_free(void* m);

/* ---- the ADMM integrator (Mesh<D> + MeshIntegrator<D>) ---- */
/* Vc may be NULL (CompMesh false).  mask has nP entries (extra entries ignored). */
void* orc_create(int dim, int nP, const double* Vp, const double* Vc, int nF, const int* F,
                 const int* mask, int monType, double dt, double tau, double rho,
                 int gradUse, int nthreads, int cgMode);
/* One MeshIntegrator::step.  tol < 0 disables the ADMM early exit (fixed nIters). */
int orc_step(void* h, int nIters, double tol, double* Ih, int* admmIters, double* primal,
             double* dual);
int orc_euler_step(void* h, double* Ih);
/* time-varying monitors: rebuild the monitor grid from Vp at every step start,
 * monitor at t = steps * dt (MonType 7 moves with t) */
void orc_set_regrid(void* h, int on);
/* MeshIntegrator::backwardsEulerStep (method 2): Newton with the FD Jacobian at the initial mesh
 * and the LASolver restatement; dotMode 0 reference sums, 1 the GPU's reduction order */
int orc_backward_euler_step(void* h, double dt, double tol, int dotMode, double* Ih, int* newtonIters);
long long orc_jacobian_nnz(void* h);
void orc_get_jacobian(void* h, int* ia, int* ja, double* a);
double orc_energy(void* h);
void orc_done(void* h);
void orc_get(void* h, const char* what, double* out);
void orc_get_F(void* h, int* F);
void orc_sizes(void* h, int* nP, int* nF, int* gridRows, int* gnx, int* gny, int* gnz);
long long orc_bfgs_iters(void* h);
int orc_error(void* h);
/* unit-level entry points */
double orc_block_grad(void* h, int sid, const double* z, const double* dxpu, double* grad,
                      int computeGrad, int regularize, double* Igt);
void orc_eval_monitor(void* h, const double* pnt, double* M);
void orc_monitor_at(int dim, int monType, const double* x, double* M);
void orc_destroy(void* h);
/* 0: glibc pow (reference semantics, default); 1: correctly rounded pow in blockGrad */
void orc_set_pow_mode(int mode);
double orc_crpow(double x, double y);

/* ---- LASolver (backward Euler's ILU(0)-preconditioned CG-STAB), oracle/lasolver.cpp ---- */
int orc_la_pack(int n, int nent, const int* rows, const int* cols, int no_diag, int* ia, int* ja, int cap);
int orc_la_mesh_pattern(int dim, int nP, int nF, const int* F, int* ia, int* ja, int cap);
int orc_la_matmult(int n, const int* ia, const int* ja, const double* a, const double* x, double* y);
int orc_la_ilu0(int n, const int* ia, const int* ja, const double* a, double* af);
int orc_la_ilu_solve(int n, const int* ia, const int* ja, const double* af, const double* b, double* x);
int orc_la_solve(int n, const int* ia, const int* ja, const double* a, const double* b, const double* toler,
                 int nitmax, double resid_reduc, int new_rhat, int initial_guess, double* x, int* nitr,
                 double* rms_hist, int dotMode);

#ifdef __cplusplus
}
#endif
#endif
