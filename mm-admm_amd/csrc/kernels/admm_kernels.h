// admm_kernels.h -- host-side launch interface of the ADMM HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace mmx {

// Slot partial-sum record written by one workgroup; reduced in a fixed order.
// v[0] = sum Ih (BFGS entry energies), v[1] = sum |z_new - z_old|^2, v[2] = sum |Dx - z|^2,
// v[3] = BFGS iterations, v[4] = error flags (inverted element), v[5] = max BFGS iters.
constexpr int kNumPartials = kLayoutPartials;

template <int D>
struct DeviceMesh {
  int nP, nF;
  const int* F;           // nF x (D+1)
  const uint8_t* sbits;   // per simplex: bit n = vertex n FIXED, bit 4+n = vertex n not INTERIOR
  const uint8_t* nodeInterior;  // per node 1 if INTERIOR
  const int* inc_ptr;     // nP+1, node -> incident slots, ascending (global) simplex id
  const int* inc_off;     // offset s*K + n*D of each local incident slot; -1-r for a slot of another
                          // rank: its D values are row r of `remote` (element partition)
  const double* remote;   // gathered interface-slot values of the other ranks (or nullptr)
  // the x-update's term w (w (z - u)) of every local slot, written by the prox in the slot layout
  // of z: the x-update then gathers D values per slot instead of 2 D (nullptr: it gathers z and u)
  double* tslot;
  // 2D, one rank: set for a step's first x-update and first prox only -- z = D zx (zx = xBar, or
  // xPrev in the first step; src/MeshIntegrator.cpp:121,126) is gathered from these positions
  // instead of read from z, so the step needs no k_gather_z pass; the prox then writes z as usual
  const double* zx;
  // 2D, one rank, steps after the third: the step's first x-update also does predictX's
  // extrapolation (k_predict mode 1) for its node -- xBar = 2 x - xPrev, xPrev = x -- into these
  // (nullptr: k_predict ran)
  double* predPrev;
  double* predBar;
  double* gcache;         // per simplex K doubles: the unregularised gradient at the current z
  int* tieList;           // prox blocks left to the exact recomputation (k_prox_fix), tieList[0..*tieCount)
  unsigned* tieCount;
  unsigned* tieStale;      // the previous steady prox's counter, cleared by this prox's recomputation
  unsigned* invFlag;       // set by a blockGrad that meets Edet <= 0 (GridView::invFlag)
  int xupCh;              // slots requested at once per node in the sweep (8, 16, 24)
  int xupSweep;           // 3D slot-term x-update as a per-XCD sweep: workgroups per CU (0: one node per lane)
  int forceTie;           // test hook (MMX_FORCE_TIE=n): every n-th prox block takes the exact path
  const int* nodeOrder;   // x-update processing order (nodes by first incident simplex) or nullptr
  // the x-update's share of that order: positions [xupLo, xupHi) (an element partition launches its
  // interior nodes, which need no remote slot, while the halo exchange runs, then the rest)
  int xupLo, xupHi;
  const double* invdiag;  // per node 1 / t_ii (block-diagonal t = tau I + dt^2 WD^T WD)
  const double* Vc;       // nP x D reference positions (CompMesh) or nullptr
  // monitor grid
  const double* gx;
  const double* gy;
  const double* gz;
  const double* gvals;
  const double* gpad;    // 3D: the grid rows padded to 10 doubles (launch_pad_rows)
  const double* gcell[3];  // 3D: per axis and cell i {g_i, h_i = g_{i+1} - g_i, RN(1/h_i), 0}
  const double* giso;      // an isotropic grid's one value per point (launch_iso_compact), else nullptr
  int gnx, gny, gnz;
  double ghx, ghy, ghz, grhx, grhy, grhz;  // grid spacings of findLimInf and RN(1/h)
  double gax, gay, gaz, gspx, gspy, gspz, gnsx, gnsy, gnsz, grnsx, grnsy, grnsz;  // linspace params
  // functional constants
  double Ehat[9];
  double powd, w;
  int compMesh;
  int prox2dWave;  // 2D steady-state prox through k_prox_wave<2> (engine set-up: MMX_PROX2D=wave)
};

struct StepScalars {
  double tau, dtsq, w, dt_over_tau;
};

template <int D>
void launch_gather_z(const DeviceMesh<D>& m, const double* x, double* z, hipStream_t st);
template <int D>
void launch_grad_simplex(const DeviceMesh<D>& m, const double* x, double* gs, bool zeroFixed,
                         double* partials, int* nblocks, hipStream_t st);
template <int D>
void launch_predict(const DeviceMesh<D>& m, int mode, const double* gs, double* x, double* xPrev,
                    double* xBar, double dt_over_tau, hipStream_t st);
template <int D>
void launch_xupdate(const DeviceMesh<D>& m, const StepScalars& sc, const double* xBar,
                    const double* z, const double* u, double* x, double* partials, int* nblocks,
                    bool resid, hipStream_t st, bool useTslot = false);
// useCache: z is unchanged since the previous prox, whose last blockGrad left the unregularised
// gradient in m.gcache; the entry blockGrad then reduces to adding the regulariser.
// 3D: pad[r 10 + n] = vals[r 9 + n], pad[r 10 + 9] = 0 (rebuilt whenever vals changes)
void launch_pad_rows(const double* vals, long long rows, double* pad, hipStream_t st);
// iso[i] = vals[i D^2] for every grid point; *notIso (zeroed by the caller) is set unless every point
// is a multiple of the identity bit for bit (off-diagonals +0, equal diagonals) or all NaN
template <int D>
void launch_iso_compact(const double* vals, long long points, double* iso, int* notIso, hipStream_t st);
// diagonal entries of the identity Bkinv of nF simplices in the bidx<D> layout (buffer zeroed before)
template <int D>
void launch_bkinv_identity(int nF, double* B, hipStream_t st);

// the steady-state prox reads one Bkinv buffer and writes the other (the engine swaps them):
// always in 3D (k_prox_wave), in 2D with k_prox_wave<2> (DeviceMesh::prox2dWave)
bool prox_double_buffered(int D, bool wave2d);
bool prox2d_wave_requested();  // MMX_PROX2D=wave
template <int D>
void launch_prox(const DeviceMesh<D>& m, bool first, bool useCache, double tol, const double* x, double* z,
                 double* u, const double* Bin, double* Bout, double* partials, int* nblocks, hipStream_t st);
template <int D>
void launch_energy(const DeviceMesh<D>& m, const double* x, double* partials, int* nblocks,
                   hipStream_t st);
template <int D>
void launch_euler_apply(const DeviceMesh<D>& m, const double* gs, double* x, double dt_over_tau,
                        hipStream_t st);
// Work space of the split reductions: each set of partials is cut into kRedSplit fixed ranges, one
// workgroup each, and a second launch combines the kRedSplit range results of each set in range
// order -- a fixed shape, so the sums are deterministic.  scratch: kRedSets x kRedSplit x
// kNumPartials doubles.  A null RedWork (or a set of fewer than kRedSplitMin partials) takes one
// workgroup per set.
constexpr int kRedSplit = 32;
constexpr int kRedSplitMin = 4096;
constexpr int kRedSets = 66;  // kDeferMax (engine.cpp) + 2
struct RedWork {
  double* scratch = nullptr;
};
void launch_reduce_partials(const double* partials, int nblocks, double* out, hipStream_t st, const RedWork& w = {});
// a step's reductions at once: results[i*2*kNumPartials ..] from partA slice i (i < n), the x-update's
// set into the second half of row n-1
void launch_reduce_steps(const double* partA, size_t stride, int nbA, const double* partB, int nbB, int n,
                         double* results, hipStream_t st, const RedWork& w = {});
// two reductions in one launch
void launch_reduce_partials2(const double* partials, int nblocks, double* out, const double* partials2, int nblocks2,
                             double* out2, hipStream_t st, const RedWork& w = {});
// interface-slot values a rank contributes to the exchange: mode 0 the x-update term
// w (w (z - u)) per slot, mode 1 the simplex gradient gs per slot (D values each)
// zx (mode 0, a step's first exchange on a partition with DeviceMesh::zx): z of a slot of node v is
// zx_v (predicted: 2 x_v - xPrev_v, the fused predictX of the x-update that has not run yet), F
// gives the slot's node
struct PackZX {
  const int* F = nullptr;
  const double* zx = nullptr;
  const double* x = nullptr;      // predicted: x and xPrev before the step's first x-update
  const double* xPrev = nullptr;
};
template <int D>
void launch_pack_export(int mode, int nExp, const int* expOff, const double* z, const double* u, const double* gs,
                        double w, double* out, hipStream_t st, const PackZX& zx = {});

// ---- backward Euler (Mesh::backwardsEulerStep, src/Mesh.cpp:1263-1341) ----
// FD derivative blocks of FSubJac (src/Mesh.cpp:1173-1230) at positions Vp: one D x K block per
// (simplex s, local vertex n), row-major at dv + ((s*(D+1)+n)*D)*K.
template <int D>
// work (optional, 1 + nF (D + 1) unsigneds): the fast pass + exact recomputation of its tie lanes
void launch_fd_jac(const DeviceMesh<D>& m, const double* Vp, double h, double* dv, hipStream_t st,
                   unsigned* work = nullptr);
// Jacobian values of buildEulerJac (src/Mesh.cpp:1112-1136, 1232-1258) on the buildMatrix CSR
// pattern (ia, ja over the D*nP unknowns): per entry, the derivative blocks of the node's incident
// simplices in ascending id (pairsort order, +0.0 adds), scaled by dt/tau, +1 on the diagonal
// (finish = false: the sums alone, before the scaling and the identity).
template <int D>
// maxColNodes: the widest row's column nodes (at most 64: one wavefront per node, else one lane per row)
void launch_jac_assemble(const DeviceMesh<D>& m, const int* ia, const int* ja, const double* dv,
                         double dt_over_tau, double* a, hipStream_t st, bool finish = true, int maxColNodes = 65);
// Newton residual F = (dt/tau) grad + (x - xn) with grad the INTERIOR-only scatter of gs
// (eulerStepMod, src/Mesh.cpp:532-579); rhs = -F; partial record v[0] = sum |F_i|.
template <int D>
void launch_be_residual(const DeviceMesh<D>& m, const double* gs, const double* x, const double* xn,
                        double dt_over_tau, double* rhs, double* partials, int* nblocks, hipStream_t st);
// x += dx over n doubles
void launch_add_inplace(int n, double* x, const double* dx, hipStream_t st);

template <int D>
void launch_debug_blockgrad(const DeviceMesh<D>& m, int s, const double* z, const double* dx, double* out,
                            int flags, hipStream_t st);

// device math self test: op 0 sqrt, 1 x^1.5, 2 x^-0.5, 3 x^2.25, 4 x^1.25
void launch_devmath(int op, int n, const double* in, double* out, hipStream_t st);

}  // namespace mmx
