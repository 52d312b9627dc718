// sparse_kernels.h -- launch interface of the LASolver HIP kernels (gfx950): CSR SpMV
// (matmult), sync-free ILU(0) factor and triangular sweeps (scaler_ILU::factor / solve) and the
// CG-STAB vector algebra (scaler_cgstab::acc_scaler).  See DESIGN.md §LASolver.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mmx {

// Products staged in LDS per SpMV workgroup (16 KB of fp64).
constexpr int kSpmvTile = 2048;
constexpr int kSpmvBlock = 256;
// Rows per sync-free sweep/factor workgroup (one wavefront).
constexpr int kSweepRows = 64;
// Grid of the vector kernels (fixed for a given n, so their partial sums are deterministic).
constexpr int kVecBlock = 256;
int vec_grid(int n);

// CG-STAB state on the device (scaler_cgstab members, accel_class.h:67-69, plus the per-iteration
// results the host polls).
struct CgsScalars {
  double rho, rholst, alpha, omega, beta, rmsi, rms, ctol, iconv;
  int conv;
  int pad;
};

struct SweepCtl {
  unsigned* tickets;  // one counter per sync-free launch of an iteration (zeroed per iteration)
  unsigned* err;      // set when a dependency wait gives up (bounded spin)
};

// y = A x (matmult, accel_class.cpp:521-549).  EPI 0: none; 1: partial sums of e1.y (per block);
// 2: partial sums of y.e1 and y.y.
void launch_spmv(int epi, int nblk, const int* rowblk, const int* ia, const int* ja, const double* a,
                 const double* x, double* y, const double* e1, double* partials, hipStream_t st);

// ILU(0) numeric factor in the factor pattern (iaf/jaf/dg); amap maps A's entries into it.
void launch_ilu_factor(int n, const int* ia, const int* ja, const double* a, const int* amap, const int* iaf,
                       const int* jaf, const int* dg, double* af, unsigned* flags, unsigned epoch,
                       unsigned* ticket, unsigned* err, hipStream_t st);

// Forward sweep (unit L) into granules gy.  pro 0: b = src; 1: p = res + beta (p - omega avbar),
// b = p (stored to p); 2: s = res - alpha avbar, b = s (stored to p).
void launch_sweep_fwd(int pro, int n, const int* iaf, const int* jaf, const int* dg, const double* af,
                      const double* src, double* p, const double* res, const double* avbar, const CgsScalars* sc,
                      uint64_t* gy, unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st);
// Backward sweep (U with its diagonal) from granules gy (epoch_y) into out and granules gx.
void launch_sweep_bwd(int n, const int* iaf, const int* jaf, const int* dg, const double* af, const uint64_t* gy,
                      double* out, uint64_t* gx, unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st);

// init: x = 0, res = b (mode 0) or res = b - res (mode 1, res holding A x); res0 = res; p = 0;
// avbar = 0.  Partials [sum res^2, sum res0.res] per block.
void launch_cgs_init(int mode, int n, const double* b, double* x, double* res, double* res0, double* p,
                     double* avbar, int copy_res0, double* partials, hipStream_t st);
// partials[b*2+1] = block sum of x.y
void launch_dot_into(int n, const double* x, const double* y, double* partials, hipStream_t st);
// sol += alpha vbar + omega z; res = s - omega t; partials [res^2, res0.res, #|step|>|toler|].
void launch_cgs_update(int n, const double* vbar, const double* z, const double* s, const double* t,
                       const double* res0, const double* toler, double* x, double* res, const CgsScalars* sc,
                       double* partials, hipStream_t st);
// Scalar finalisers (one workgroup).  mode 0 init, 1 alpha, 2 omega, 3 update.
void launch_cgs_fin(int mode, const double* partials, int nblk, CgsScalars* sc, hipStream_t st);

}  // namespace mmx
