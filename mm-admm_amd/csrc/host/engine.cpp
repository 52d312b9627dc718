// engine.cpp -- the ADMM integrator on one MI355X: set-up, device state, step orchestration.
//
// Host mirror of Mesh<D> (src/Mesh.cpp:384-472) and MeshIntegrator<D> (src/MeshIntegrator.cpp).
// All per-step work runs on the device on one HIP stream; the host only launches kernels and,
// with the early exit enabled, reads back three scalars per ADMM iteration.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/mmx_sparse.h"
#include "../kernels/admm_kernels.h"
#include "../kernels/regrid_kernels.h"
#include "comm.h"
#include "common.h"
#include "partition.h"

#define MMX_SP(expr)                                                                     \
  do {                                                                                   \
    const int rc_ = (expr);                                                              \
    if (rc_ != MMADMM_OK) throw ::mmx::Error(rc_, std::string(#expr) + ": " + mmadmm_last_error()); \
  } while (0)

namespace mmx {

namespace {
thread_local std::string g_last_error;
}
void set_last_error(const std::string& msg) { g_last_error = msg; }


struct EngineBase {
  virtual ~EngineBase() = default;
  int dim = 2;
  virtual void step(int nIters, double tol, double* Ih, int* iters) = 0;
  virtual double eulerStep() = 0;
  virtual double backwardEulerStep(double dt, double tol, int* newton) = 0;
  virtual void jacobian(long long* nnz, int32_t* ia, int32_t* ja, double* a) = 0;
  // the pieces of Mesh::backwardsEulerStep for a host-driven Newton loop (mmadmm_be_*)
  virtual void newtonOp(int op, double dt, const double* in, double* out, double* sc) = 0;
  virtual double energy() = 0;
  virtual void done() = 0;
  virtual void get(const std::string& what, double* out) = 0;
  virtual void getSimplices(int32_t* F) = 0;
  virtual void localNodes(int* n, int32_t* ids) = 0;
  virtual void sizes(int* nP, int* nF, int* gridRows) = 0;
  virtual void setTiming(bool on) = 0;
  virtual void stats(mmadmm_stats* s) = 0;
  virtual void resetStats() = 0;
  virtual void sync() = 0;
  virtual void regrid(double t) = 0;
  virtual void setRegrid(bool on) = 0;
  virtual void debugBlockGrad(int s, const double* z, const double* dx, int flags, double* out) = 0;
};

// Mesh::reOrientElements (src/Mesh.cpp:243-260): swap F(i,1), F(i,2) when det(E) < 0, E the
// edge vectors from vertex 0 as columns, Eigen's 2x2 / 3x3 determinant
void reorient_simplices(int D, const double* Vp, int nF, int32_t* F) {
  for (int s = 0; s < nF; ++s) {
    double E[3][3] = {{0}};
    const int32_t* f = F + (size_t)s * (D + 1);
    for (int j = 0; j < D; ++j)
      for (int r = 0; r < D; ++r) E[r][j] = Vp[(size_t)f[j + 1] * D + r] - Vp[(size_t)f[0] * D + r];
    double det;
    if (D == 2) {
      det = E[0][0] * E[1][1] - E[1][0] * E[0][1];
    } else {
      const double h0 = E[0][0] * (E[1][1] * E[2][2] - E[1][2] * E[2][1]);
      const double h1 = E[0][1] * (E[1][0] * E[2][2] - E[1][2] * E[2][0]);
      const double h2 = E[0][2] * (E[1][0] * E[2][1] - E[1][1] * E[2][0]);
      det = h0 - h1 + h2;
    }
    if (det < 0) std::swap(F[(size_t)s * (D + 1) + 1], F[(size_t)s * (D + 1) + 2]);
  }
}

template <int D>
class Engine final : public EngineBase {
 public:
  static constexpr int K = D * (D + 1);

  Engine(int nP, const double* Xp, const double* Xc, int nF, const int32_t* F, const int32_t* mask,
         const mmadmm_params& p, mmadmm_monitor_fn fn, void* user, Comm* comm) {
    dim = D;
    prm_ = p;
    nranks_ = std::max(1, p.nranks);
    rank_ = nranks_ > 1 ? p.rank : 0;
    comm_ = comm;
    if (nranks_ > 1 && !comm_) throw Error(MMADMM_ERR_INVALID, "partitioned engine needs a communicator");
    if (p.device >= 0) MMX_HIP(hipSetDevice(p.device));
    MMX_HIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    if (nranks_ > 1) {  // the halo exchange's stream (overlapped with the interior x-update)
      MMX_HIP(hipStreamCreateWithFlags(&st2_, hipStreamNonBlocking));
      MMX_HIP(hipEventCreateWithFlags(&evProx_, hipEventDisableTiming));
      MMX_HIP(hipEventCreateWithFlags(&evEx_, hipEventDisableTiming));
    }
    compMesh_ = (Xc != nullptr);
    std::vector<double> Vp(Xp, Xp + (size_t)nP * D);
    Fh_.assign(F, F + (size_t)nF * (D + 1));
    for (int i = 0; i < nF * (D + 1); ++i)
      if (Fh_[i] < 0 || Fh_[i] >= nP) throw Error(MMADMM_ERR_INVALID, "simplex vertex id out of range");
    maskH_.assign(mask, mask + nP);
    reorient_simplices(D, Vp.data(), nF, Fh_.data());
    // monitor grid (MeshInterpolator set-up), once per run on the initial vertices
    build_monitor_grid(D, Vp.data(), nP, fn, user, grid_);
    monFn_ = fn;
    monUser_ = user;
    // functional constants (src/AdaptationFunctional.cpp:176-220, src/Mesh.cpp:451)
    const double w = 0.5 * sqrt(p.rho);
    w_ = w;
    double Ehat[3][3] = {{0}};
    if (D == 2) {
      Ehat[0][0] = 1.0;
      Ehat[1][0] = 0.0;
      Ehat[0][1] = 1.0 / 2.0;
      Ehat[1][1] = sqrt(3) / 2.0;
    } else {
      const double v[3][3] = {{-2.0, 0.0, -2.0}, {0.0, -2.0, -2.0}, {-2.0, -2.0, 0.0}};
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Ehat[r][c] = v[r][c];
    }
    const double dFact = (D == 2) ? 2.0 : 6.0;
    const double s1 = pow((dFact / std::abs(hostDet(Ehat))), 1.0 / ((double)D));
    for (int r = 0; r < D; ++r)
      for (int c = 0; c < D; ++c) Ehat[r][c] *= s1;
    const double s2 = (double)pow(nF, 1.0 / D);
    for (int r = 0; r < D; ++r)
      for (int c = 0; c < D; ++c) Ehat[r][c] /= s2;
    for (int r = 0; r < D; ++r)
      for (int c = 0; c < D; ++c) EhatH_[r * D + c] = Ehat[r][c];
    const double d = (double)D, pp = 1.5;
    powd_ = pow(d, d * pp / 2.0);
    // element partition (a single rank owns everything); node -> incident slots in ascending
    // global simplex id (column-major D^T order), other ranks' slots from the gathered buffer
    plan_ = make_partition_plan(D, nP, Vp.data(), nF, Fh_.data(), nranks_, rank_, p.partition);
    nP_ = (int)plan_.localNodes.size();
    nF_ = (int)plan_.localSimplices.size();
    if (nranks_ > 1) {  // vertex owners for the partitioned regrid: the rank of the lowest incident simplex
      std::vector<std::vector<int>> owned(nranks_);
      for (int v = 0; v < nP; ++v) owned[plan_.nodeOwner[v]].push_back(v);
      size_t mx = 1;
      for (auto& o : owned) mx = std::max(mx, o.size());
      maxOwned_ = (int)mx;
      std::vector<int> all((size_t)nranks_ * mx, -1), mine;
      for (int q = 0; q < nranks_; ++q) std::copy(owned[q].begin(), owned[q].end(), all.begin() + (size_t)q * mx);
      for (int v : owned[rank_])
        mine.push_back((int)(std::lower_bound(plan_.localNodes.begin(), plan_.localNodes.end(), v) - plan_.localNodes.begin()));
      nOwned_ = (int)mine.size();
      ownAllGid_.upload(all.data(), all.size(), st_);
      ownAllGidH_ = all;
      ownLocal_.upload(mine.data(), std::max<size_t>(mine.size(), 1), st_);
      streamWait();
    }
    const int nl = nP_;
    // t = M + dt^2 WD_T W D is block diagonal: t_vv = tau + dt^2 * (w*w summed valence times)
    std::vector<double> invdiag(nl);
    const double dtsq = p.dt * p.dt;
    for (int v = 0; v < nl; ++v) {
      double S = 0.0;
      for (int c = 0; c < plan_.valence[v]; ++c) S = (c == 0) ? (w * w) * 1.0 : S + (w * w) * 1.0;
      invdiag[v] = 1.0 / (p.tau + dtsq * S);
    }
    std::vector<uint8_t> sbits(nF_), interior(nl);
    for (int v = 0; v < nl; ++v) interior[v] = maskH_[plan_.localNodes[v]] == MMADMM_INTERIOR ? 1 : 0;
    for (int s = 0; s < nF_; ++s) {
      unsigned b = 0;
      for (int n = 0; n < D + 1; ++n) {
        const int t = maskH_[plan_.localNodes[plan_.Flocal[(size_t)s * (D + 1) + n]]];
        if (t == MMADMM_BOUNDARY_FIXED) b |= 1u << n;
        if (t != MMADMM_INTERIOR) b |= 1u << (4 + n);
      }
      sbits[s] = (uint8_t)b;
    }
    std::vector<double> Vl((size_t)nl * D), Vcl;
    for (int v = 0; v < nl; ++v)
      for (int c = 0; c < D; ++c) Vl[(size_t)v * D + c] = Vp[(size_t)plan_.localNodes[v] * D + c];
    if (compMesh_) {
      Vcl.resize((size_t)nl * D);
      for (int v = 0; v < nl; ++v)
        for (int c = 0; c < D; ++c) Vcl[(size_t)v * D + c] = Xc[(size_t)plan_.localNodes[v] * D + c];
    }
    // device state
    F_.upload(plan_.Flocal.data(), plan_.Flocal.size(), st_);
    sbits_.upload(sbits.data(), sbits.size(), st_);
    interior_.upload(interior.data(), interior.size(), st_);
    incPtr_.upload(plan_.incPtr.data(), plan_.incPtr.size(), st_);
    incOff_.upload(plan_.incSrc.data(), plan_.incSrc.size(), st_);
    {  // the x-update terms in the slot layout (DeviceMesh::tslot): 3D (C4: prox +0.09 ms, x-update
       // 0.36 -> 0.18 ms) and small 2D meshes, whose prox is under two rounds of the chip's resident
       // waves, so the terms' stores cost it little (C2: 14,754 -> 15,037 it/s; C3: prox +0.034 ms,
       // x-update -0.018 ms, 2,506 -> 2,412 it/s); MMX_TSLOT=0/1 overrides
      const char* ts = getenv("MMX_TSLOT");
      tslotOn_ = ts ? atoi(ts) != 0 : (D == 3 || nF_ <= kTslot2dMax);
      const char* sp = getenv("MMX_SPIN");
      spinWait_ = !(sp && atoi(sp) == 0);
      const char* zx = getenv("MMX_ZX");  // 0: the step's z = D x by k_gather_z (DeviceMesh::zx)
      zFromX_ = !(zx && atoi(zx) == 0);  // 2D and 3D, partitions too: the first pack reads zx (PackZX)
      const char* ov = getenv("MMX_OVERLAP");  // 0: the halo exchange before the whole x-update
      overlap_ = nranks_ > 1 && !(ov && atoi(ov) == 0);
      const char* fp = getenv("MMX_FUSE_PRED");  // 0: k_predict runs in every step (DeviceMesh::predBar)
      fusePred_ = !(fp && atoi(fp) == 0);
      if (tslotOn_) tslot_.alloc(std::max<size_t>((size_t)nF_ * K, 1));
    }
    {  // x-update order: nodes by their first incident (local) simplex, then id -- locality of the
       // slot gathers when the node numbering is not simplex-ordered (e.g. cell centres numbered last)
      std::vector<long long> key(nl);
      for (int v = 0; v < nl; ++v) {
        long long k = (long long)nF_;
        for (int t = plan_.incPtr[v]; t < plan_.incPtr[v + 1]; ++t)
          if (plan_.incSrc[t] >= 0) k = std::min<long long>(k, plan_.incSrc[t] / K);
        key[v] = k;
      }
      // an element partition orders its interior nodes (no slot of another rank) first: their
      // x-update runs while the halo exchange is in flight (overlap_), the rest after it
      std::vector<int32_t> inner, bound;
      for (int v = 0; v < nl; ++v) {
        bool remote = false;
        for (int t = plan_.incPtr[v]; t < plan_.incPtr[v + 1]; ++t) remote |= plan_.incSrc[t] < 0;
        (remote && overlap_ ? bound : inner).push_back(v);
      }
      nInner_ = (int)inner.size();
      const char* xo = getenv("MMX_XUP_ORDER");  // 3D default: y slabs (C4 x-update 0.174 -> 0.152 ms with the sweep)
      const bool slabs = xo ? atoi(xo) == 1 : D == 3;
      auto order = [&](std::vector<int32_t>& ord) {
        const int n = (int)ord.size();
        if (slabs) {
          // eight slabs across the y axis (2D: opt-in), one per XCD group of the node order (the x-update's
          // XCD-contiguous blocks), each by first incident simplex: an XCD's share of every z
          // layer is one slab, so its live slot terms are an eighth of a layer
          const int n8 = ((n + 255) / 256 + 7) / 8 * 256;
          std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return Vl[(size_t)a * D + 1] < Vl[(size_t)b * D + 1]; });
          for (int c = 0; c < 8; ++c) {
            const int lo = std::min(n, c * n8), hi = std::min(n, (c + 1) * n8);
            std::stable_sort(ord.begin() + lo, ord.begin() + hi, [&](int a, int b) { return key[a] < key[b]; });
          }
        } else {
          std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return key[a] < key[b]; });
        }
      };
      order(inner);
      order(bound);
      std::vector<int32_t> ord(inner);
      ord.insert(ord.end(), bound.begin(), bound.end());
      nodeOrder_.upload(ord.data(), std::max<size_t>(ord.size(), 1), st_);
      streamWait();
    }
    invdiag_.upload(invdiag.data(), invdiag.size(), st_);
    if (compMesh_) Vc_.upload(Vcl.data(), Vcl.size(), st_);
    uploadGridCoords();
    gvals_.upload(grid_.vals.data(), grid_.vals.size(), st_);
    if (D == 3) {
      gpad_.alloc(gvals_.n / 9 * 10);
      launch_pad_rows(gvals_.p, (long long)(gvals_.n / 9), gpad_.p, st_);
    }
    updateIso();
    Vp_.upload(Vl.data(), Vl.size(), st_);  // Mesh::Vp
    x_.upload(Vl.data(), Vl.size(), st_);   // MeshIntegrator ctor: x = xPrev = xBar = copyX(Vp)
    xPrev_.upload(Vl.data(), Vl.size(), st_);
    xBar_.upload(Vl.data(), Vl.size(), st_);
    if (nranks_ > 1) {
      expOff_.upload(plan_.sendOff.data(), std::max<size_t>(plan_.sendOff.size(), 1), st_);
      export_.alloc((size_t)std::max<size_t>(plan_.sendOff.size(), 1) * D);
      remote_.alloc((size_t)std::max(plan_.recvRows, 1) * D);
    }
    // z_, u_ (MMX_ZU_INTER=1 builds, 2D: the two interleaved per vertex slot in z_, u = z_ + D)
    z_.alloc((size_t)nF_ * K * (kZUInterleaved ? 2 : 1));
    gcache_.alloc((size_t)nF_ * K);
    tieList_.alloc((size_t)nF_ / 16 + 1);  // prox blocks queued for the exact recomputation
    // [0..1]: queued blocks, double-buffered over the steady proxes (k_prox_fix); [2]: the
    // inverted-element flag (GridView::invFlag), cleared when a failed step reads it
    tieCount_.alloc(3);
    MMX_HIP(hipMemsetAsync(tieCount_.p, 0, 3 * sizeof(unsigned), st_));
    if (!kZUInterleaved) u_.alloc((size_t)nF_ * K);
    gs_.alloc((size_t)nF_ * K);
    clearU();
    {
      // hessInvs = I (src/Mesh.cpp:456-464), wave-interleaved (bidx) and padded to whole chunks of
      // 256 simplices (the 2D prox copies whole chunks); 3D double-buffered (k_prox_wave)
      const size_t nB = (size_t)((nF_ + 255) / 256) * 256 * K * K;
      B_.alloc(nB);
      MMX_HIP(hipMemsetAsync(B_.p, 0, nB * sizeof(double), st_));
      launch_bkinv_identity<D>(nF_, B_.p, st_);
      wave2d_ = D == 2 && prox2d_wave_requested();
      if (prox_double_buffered(D, wave2d_)) B2_.alloc(nB);
    }
    // prox workgroups take 16 (3D quad) to 256 simplices; node kernels pad their grid to a multiple of 8 (XCD map)
    // (k_prox_quad: 16 tets per workgroup)
    // (at least 16 x 256: the persistent x-update sweep writes one record per workgroup, 256 per CU
    // count of MMX_XUP_SWEEP, twice on a partition)
    const size_t maxBlocks = std::max<size_t>(4096, std::max((nF_ + 15) / 16, (nP_ + 255) / 256 + 16));
    maxBlocks_ = maxBlocks;
    partA_.alloc(maxBlocks * kNumPartials);
    partB_.alloc(maxBlocks * kNumPartials);
    redScratch_.alloc((size_t)kRedSets * kRedSplit * kNumPartials);
    red_.scratch = redScratch_.p;
    resultsCap_ = 0;
    ensureResults(64);
    m_ = makeView();
    launch_gather_z<D>(m_, x_.p, z_.p, st_);  // z = D x
    streamWait();
    MMX_HIP(hipGetLastError());
  }

  ~Engine() override {
    if (rgHost_) (void)hipHostFree(rgHost_);
    if (rgnHost_) (void)hipHostFree(rgnHost_);
    if (jac_) (void)mmx_matrix_destroy(jac_);
    for (auto& e : evPool_) (void)hipEventDestroy(e);
    if (evSync_) (void)hipEventDestroy(evSync_);
    if (resH_) (void)hipHostFree(resH_);
    if (evProx_) (void)hipEventDestroy(evProx_);
    if (evEx_) (void)hipEventDestroy(evEx_);
    if (st2_) (void)hipStreamDestroy(st2_);
    if (st_) (void)hipStreamDestroy(st_);
  }

  // MeshIntegrator<D>::step (src/MeshIntegrator.cpp:101-191)
  void step(int nIters, double tol, double* Ih, int* itersOut) override {
    if (nIters < 1) throw Error(MMADMM_ERR_INVALID, "step: nIters must be >= 1");
    // Mesh<D>::setUp (src/Mesh.cpp:1006-1014, commented in the reference): time-varying monitors
    if (regridEachStep_) regrid(stepsTaken_ * prm_.dt);
    ensureResults(nIters);
    // (no clear of the inverted flag here: within a step every blockGrad that sets it is followed by
    // a NaN energy that reports it, and energy() / the FD Jacobian clear what they leave)
    const bool timing = timing_;
    hipEvent_t eStep0 = nullptr, eStep1 = nullptr;
    if (timing) {
      eStep0 = nextEvent();
      MMX_HIP(hipEventRecord(eStep0, st_));
    }
    const double dtOverTau = prm_.dt / prm_.tau;
    // predictX (src/Mesh.cpp:649-674), then xPrev = x
    // (2D, one rank: the extrapolation of steps after the third runs inside the step's first x-update)
    const bool fusePred = zFromX_ && fusePred_ && !wave2d_ && !(prm_.grad_use || stepsTaken_ <= 2);
    if (prm_.grad_use || stepsTaken_ <= 2) {
      int nb = 0;
      launch_grad_simplex<D>(m_, x_.p, gs_.p, true, partA_.p, &nb, st_);
      exchange(1);
      launch_predict<D>(m_, 0, gs_.p, x_.p, xPrev_.p, xBar_.p, dtOverTau, st_);
    } else if (!fusePred) {
      launch_predict<D>(m_, 1, nullptr, x_.p, xPrev_.p, xBar_.p, dtOverTau, st_);
    }
    // x = xBar; z = D x; first step: z = D xPrev.  2D on one rank: no pass over z -- the step's first
    // x-update and first prox take z from these positions (DeviceMesh::zx; C3: -37 us per step)
    const double* zsrc = stepsTaken_ == 0 ? xPrev_.p : xBar_.p;
    const bool zFromX = zFromX_ && !wave2d_;
    if (!stepTaken_) clearU();  // (before z: in 2D the clear takes the whole interleaved buffer)
    if (zFromX)
      m_.zx = zsrc;
    else
      launch_gather_z<D>(m_, zsrc, z_.p, st_);
    gcacheValid_ = false;  // z was reset
    if (!zFromX) m_.zx = nullptr;
    StepScalars sc{prm_.tau, prm_.dt * prm_.dt, w_, dtOverTau};
    int nbx = 0, nbp = 0;
    if (fusePred) {
      m_.predPrev = xPrev_.p;
      m_.predBar = xBar_.p;
    }
    PackZX pz;  // a partition's first pack: z = D zx (predicted: 2 x - xPrev) for the exported slots
    if (zFromX) {
      pz.F = F_.p;
      pz.zx = zsrc;
      if (fusePred) {
        pz.x = x_.p;
        pz.xPrev = xPrev_.p;
      }
    }
    xupdateHalo(sc, &nbx, false, false, pz);
    m_.predPrev = m_.predBar = nullptr;
    const bool early = tol >= 0;
    int done = 0;
    double primal = 0, dual = 0;
    // early exit off: every iteration's prox partials kept in their own slice and reduced in one
    // launch after the loop (no reduction launch inside the loop)
    const bool deferRed = !early && nIters <= kDeferMax;
    const size_t slice = maxBlocks_ * kNumPartials;
    if (deferRed && partA_.n < slice * nIters) partA_.alloc(slice * std::max(nIters, 10));
    int firstDeferred = 0;  // first iteration of the batched reduction
    for (int i = 0; i < nIters; ++i) {
      hipEvent_t a0 = nullptr, a1 = nullptr, b1 = nullptr;
      if (timing) {
        a0 = nextEvent();
        MMX_HIP(hipEventRecord(a0, st_));
      }
      const bool firstProx = !hessComputed_;          // another kernel, another partial count
      const bool swapB = prox_double_buffered(D, wave2d_) && hessComputed_;  // steady state B_ -> B2_, then swap
      if (hessComputed_) {  // fast + exact pair: flip the tie queue
        tiePar_ ^= 1;
        std::swap(m_.tieCount, m_.tieStale);
      }
      launch_prox<D>(m_, !hessComputed_, gcacheValid_, early ? tol / 100 : 1e-3 / 100, x_.p, z_.p, uPtr(), B_.p,
                     swapB ? B2_.p : B_.p, partA_.p + (deferRed ? slice * i : 0), &nbp, st_);
      m_.zx = nullptr;  // z is in z_ from the first prox on
      if (swapB) std::swap(B_.p, B2_.p);
      gcacheValid_ = true;  // the prox's last blockGrad left the gradient at the final z
      if (timing) {
        a1 = nextEvent();
        MMX_HIP(hipEventRecord(a1, st_));
      }
      hessComputed_ = true;
      stepTaken_ = true;
      // the primal residual ||D x - z|| (src/MeshIntegrator.cpp:162) only feeds the early-exit test
      // and the reported last residual: without the early exit it is formed on the last iteration
      const bool resid = early || i == nIters - 1;
      xupdateHalo(sc, &nbx, resid, true, PackZX{});
      if (timing) {
        b1 = nextEvent();
        MMX_HIP(hipEventRecord(b1, st_));
        timed_.push_back({a0, a1, b1});
      }
      if (deferRed) {
        if (firstProx && i < nIters - 1) {  // reduced at once: the batch below assumes one partial count
          launch_reduce_partials(partA_.p + slice * i, nbp, res_ + (size_t)i * 2 * kNumPartials, st_, red_);
          firstDeferred = i + 1;
        } else if (i == nIters - 1) {
          const int i0 = firstProx ? i : firstDeferred;
          launch_reduce_steps(partA_.p + slice * i0, slice, nbp, partB_.p, nbx, nIters - i0,
                              res_ + (size_t)i0 * 2 * kNumPartials, st_, red_);
        }
      } else if (resid) {
        launch_reduce_partials2(partA_.p, nbp, res_ + (size_t)i * 2 * kNumPartials, partB_.p, nbx,
                                res_ + (size_t)i * 2 * kNumPartials + kNumPartials, st_, red_);
      } else {
        launch_reduce_partials(partA_.p, nbp, res_ + (size_t)i * 2 * kNumPartials, st_, red_);
      }
      done = i + 1;
      if (early) {
        std::vector<double> rv;
        fetchResults(res_ + (size_t)i * 2 * kNumPartials, 1, rv);
        const double* r = rv.data();
        primal = sqrt(r[kNumPartials + 2]);
        dual = sqrt(r[1]);
        // an inverted element ends the loop; it is reported below, after the step's bookkeeping
        // (Vp, timers, counters), exactly like one found without the early exit
        if (r[4] > 0 || (primal < tol && dual < tol)) break;
      }
    }
    // Mesh::updateAfterStep: Vp = x
    MMX_HIP(hipMemcpyAsync(Vp_.p, x_.p, (size_t)nP_ * D * sizeof(double), hipMemcpyDeviceToDevice, st_));
    vpVersion_++;
    if (timing) {
      eStep1 = nextEvent();
      MMX_HIP(hipEventRecord(eStep1, st_));
    }
    fetchResults(res_, done, hostRes_);
    MMX_HIP(hipGetLastError());
    bool bad = false;
    long long bf = 0;
    int mx = 0;
    for (int i = 0; i < done; ++i) {
      const double* r = &hostRes_[(size_t)i * 2 * kNumPartials];
      bad |= r[4] > 0;
      bf += (long long)r[3];
      mx = std::max(mx, (int)r[5]);
    }
    const double* last = &hostRes_[(size_t)(done - 1) * 2 * kNumPartials];
    primal = sqrt(last[kNumPartials + 2]);
    dual = sqrt(last[1]);
    st_stats_.admm_iters += done;
    st_stats_.bfgs_iters += bf;
    st_stats_.max_bfgs = mx;
    st_stats_.last_primal = primal;
    st_stats_.last_dual = dual;
    st_stats_.steps += 1;
    if (timing) {  // resolved later (stats, reset, or a full pool): no event queries between steps
      stepEv_.push_back({eStep0, eStep1});
      if (evUsed_ >= kEvResolve) resolveTimed();
    }
    stepsTaken_++;
    if (bad) throwBad("in prox");
    if (Ih) *Ih = hostRes_[0];  // Ihstart
    if (itersOut) *itersOut = done;
  }

  // MeshIntegrator::eulerStep -> Mesh::eulerStepMod (src/Mesh.cpp:532-579)
  double eulerStep() override {
    clearInvFlag();
    int nb = 0;
    launch_grad_simplex<D>(m_, x_.p, gs_.p, false, partA_.p, &nb, st_);
    launch_reduce_partials(partA_.p, nb, res_, st_, red_);
    exchange(1);
    launch_euler_apply<D>(m_, gs_.p, x_.p, prm_.dt / prm_.tau, st_);
    std::vector<double> rv;
    fetchResults(res_, 1, rv);
    const double* r = rv.data();
    if (r[4] > 0) throwBad("in the explicit Euler gradient");
    return r[0];
  }

  // MeshIntegrator::backwardsEulerStep -> Mesh::backwardsEulerStep (src/MeshIntegrator.cpp:68-76,
  // src/Mesh.cpp:1263-1341): Newton on F(x) = (dt/tau) grad(x) + (x - xn), the explicit Euler
  // step as initial guess, J dx = -F by the LASolver replacement (ILU(0) CG-STAB, include/
  // mmx_sparse.h) on the device.  The Jacobian is the FD Jacobian at Vp, built on the first
  // Newton iteration of the run and again whenever ||F||_1 stagnates (ratio < 0.25).
  double backwardEulerStep(double dtBE, double tol, int* newtonOut) override {
    if (nranks_ > 1) throw Error(MMADMM_ERR_INVALID, "backward Euler runs on one rank (no element partition)");
    const auto tStep = Clock::now();
    const int n = nP_ * D;
    ensureJacobian();
    const double dtot = dtBE / prm_.tau;
    const double SAFETY_FAC = 1.0 / 10.0;
    const int MAX_ITERS = 1000;
    clearInvFlag();
    MMX_HIP(hipMemcpyAsync(xn_.p, x_.p, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, st_));
    int nb = 0, nb2 = 0;
    launch_grad_simplex<D>(m_, x_.p, gs_.p, false, partA_.p, &nb, st_);  // initial guess
    launch_euler_apply<D>(m_, gs_.p, x_.p, dtot, st_);
    if (!beStepTaken_) buildJacobian(dtBE);
    int nIter = 0;
    double Ih = 0.0, normPrev = INFINITY;
    std::vector<double> rv;
    void* mst = nullptr;
    MMX_SP(mmx_matrix_stream(jac_, &mst));
    do {
      launch_grad_simplex<D>(m_, x_.p, gs_.p, false, partA_.p, &nb, st_);
      launch_be_residual<D>(m_, gs_.p, x_.p, xn_.p, dtot, rhs_.p, partB_.p, &nb2, st_);
      launch_reduce_partials2(partA_.p, nb, res_, partB_.p, nb2, res_ + kNumPartials, st_, red_);
      fetchResults(res_, 1, rv);
      if (rv[4] > 0) throwBad("in backward Euler");
      Ih = rv[0];
      const double norm = rv[kNumPartials];
      if (norm < SAFETY_FAC * tol) break;
      if (!beStepTaken_ || std::fabs(norm - normPrev) / norm < 0.25) {
        buildJacobian(dtBE);
        beStepTaken_ = true;
      }
      waitStream();  // rhs and the Jacobian values are ready for the solver stream (spin: see waitStream)
      const auto tSolve = Clock::now();
      MMX_SP(mmx_matrix_set_rhs_device(jac_, rhs_.p));
      int cgIter = 0;
      MMX_SP(mmx_matrix_solve_device(jac_, &jprm_, dx_.p, &cgIter, 0));  // (returns once its stream is done)
      st_stats_.t_solve_ms += msSince(tSolve);
      if (cgIter > 0) st_stats_.cg_iters += cgIter;
      if (cgIter <= 0)
        throw Error(MMADMM_ERR_NOCONV, "backward Euler: CG-STAB did not converge (reference: assert(cgIter > 0))");
      launch_add_inplace(n, x_.p, dx_.p, st_);
      nIter++;
      normPrev = norm;
    } while (nIter < MAX_ITERS);
    streamWait();
    st_stats_.steps += 1;
    st_stats_.newton_iters += nIter;
    st_stats_.t_be_ms += msSince(tStep);
    if (newtonOut) *newtonOut = nIter;
    return Ih;
  }

  // Mesh::backwardsEulerStep in pieces (src/Mesh.cpp:1263-1341), so that a host loop can drive the
  // Newton iteration and solve through the reference's LASolver interface (include/mmadmm/
  // MatrixIter.h): op 0 xn = x, Ih = eulerStepMod(x), x -= (dt/tau) grad (1266-1273; sc[0] = Ih);
  // op 1 F = (dt/tau) grad(x) + (x - xn) into out (1289-1294; sc[0] = Ih, sc[1] = ||F||_1 as the
  // engine's own loop forms it); op 2 the FSubJac sums at Vp on the buildMatrix CSR pattern, before
  // buildEulerJac's scaling and identity (1112-1124, 1232-1258); op 3 x += in (1329).
  void newtonOp(int op, double dt, const double* in, double* out, double* sc) override {
    if (nranks_ > 1) throw Error(MMADMM_ERR_INVALID, "backward Euler runs on one rank (no element partition)");
    ensureJacobian();
    const int n = nP_ * D;
    std::vector<double> rv;
    int nb = 0, nb2 = 0;
    if (op == 0 || op == 1) clearInvFlag();
    if (op == 0) {
      MMX_HIP(hipMemcpyAsync(xn_.p, x_.p, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, st_));
      launch_grad_simplex<D>(m_, x_.p, gs_.p, false, partA_.p, &nb, st_);
      launch_reduce_partials(partA_.p, nb, res_, st_, red_);
      launch_euler_apply<D>(m_, gs_.p, x_.p, dt / prm_.tau, st_);
      fetchResults(res_, 1, rv);
      if (rv[4] > 0) throwBad("in backward Euler");
      if (sc) sc[0] = rv[0];
    } else if (op == 1) {
      launch_grad_simplex<D>(m_, x_.p, gs_.p, false, partA_.p, &nb, st_);
      launch_be_residual<D>(m_, gs_.p, x_.p, xn_.p, dt / prm_.tau, rhs_.p, partB_.p, &nb2, st_);
      launch_reduce_partials2(partA_.p, nb, res_, partB_.p, nb2, res_ + kNumPartials, st_, red_);
      fetchResults(res_, 1, rv);
      if (rv[4] > 0) throwBad("in backward Euler");
      std::vector<double> r((size_t)n);
      MMX_HIP(hipMemcpyAsync(r.data(), rhs_.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st_));
      streamWait();
      for (int i = 0; i < n; ++i) out[i] = -r[i];  // rhs = -F on the device: the negation is exact
      if (sc) {
        sc[0] = rv[0];
        sc[1] = rv[kNumPartials];
      }
    } else if (op == 2) {
      const double h = 10.0 * sqrt(std::numeric_limits<double>::epsilon());
      launch_fd_jac<D>(m_, Vp_.p, h, dv_.p, st_, fdWork_.p);
      clearInvFlag();  // the FD blocks report no inversion (their energies are not checked)
      // into a scratch buffer: jval_ keeps the engine's last assembled Jacobian (mmadmm_get_jacobian)
      if (jraw_.n != jja_.n) jraw_.alloc(std::max<size_t>(jja_.n, 1));
      launch_jac_assemble<D>(m_, jia_.p, jja_.p, dv_.p, 1.0, jraw_.p, st_, false, maxColNodes_);
      MMX_HIP(hipMemcpyAsync(out, jraw_.p, jja_.n * sizeof(double), hipMemcpyDeviceToHost, st_));
      streamWait();
    } else if (op == 3) {
      MMX_HIP(hipMemcpyAsync(dx_.p, in, (size_t)n * sizeof(double), hipMemcpyHostToDevice, st_));
      launch_add_inplace(n, x_.p, dx_.p, st_);
      streamWait();
    } else {
      throw Error(MMADMM_ERR_INVALID, "newtonOp: unknown op");
    }
  }

  void jacobian(long long* nnz, int32_t* ia, int32_t* ja, double* a) override {
    if (!jac_) throw Error(MMADMM_ERR_INVALID, "no Jacobian yet: run a backward Euler step first");
    if (nnz) *nnz = (long long)jja_.n;
    if (ia) MMX_HIP(hipMemcpyAsync(ia, jia_.p, jia_.n * sizeof(int32_t), hipMemcpyDeviceToHost, st_));
    if (ja) MMX_HIP(hipMemcpyAsync(ja, jja_.p, jja_.n * sizeof(int32_t), hipMemcpyDeviceToHost, st_));
    if (a) MMX_HIP(hipMemcpyAsync(a, jval_.p, jval_.n * sizeof(double), hipMemcpyDeviceToHost, st_));
    streamWait();
  }

  // Mesh::computeEnergy on Vp (src/Mesh.cpp:496-530)
  double energy() override {
    int nb = 0;
    launch_energy<D>(m_, Vp_.p, partA_.p, &nb, st_);
    clearInvFlag();  // energy() returns NaN for an inverted element without reporting it
    launch_reduce_partials(partA_.p, nb, res_, st_, red_);
    std::vector<double> rv;
    fetchResults(res_, 1, rv);
    return rv[0];
  }

  void done() override {
    MMX_HIP(hipMemcpyAsync(Vp_.p, x_.p, (size_t)nP_ * D * sizeof(double), hipMemcpyDeviceToDevice, st_));
    vpVersion_++;
    streamWait();
  }

  void get(const std::string& what, double* out) override {
    const DevBuf<double>* b = nullptr;
    if (what == "x") b = &x_;
    else if (what == "xPrev") b = &xPrev_;
    else if (what == "xBar") b = &xBar_;
    else if (what == "z" || what == "u") {
      if (!kZUInterleaved) {
        b = what == "z" ? &z_ : &u_;
      } else {  // de-interleave: slot i of simplex s at s 2K + (i / D) 2D + i % D (+ D for u)
        std::vector<double> h(z_.n);
        MMX_HIP(hipMemcpyAsync(h.data(), z_.p, z_.n * sizeof(double), hipMemcpyDeviceToHost, st_));
        streamWait();
        const int sh = what == "u" ? D : 0;
        for (int s = 0; s < nF_; ++s)
          for (int i = 0; i < K; ++i) out[(size_t)s * K + i] = h[(size_t)s * 2 * K + (i / D) * 2 * D + i % D + sh];
        return;
      }
    }
    else if (what == "points") b = &Vp_;
    else if (what == "hess") b = &B_;
    else if (what == "gs") b = &gs_;
    else if (what == "grid") {
      if (gridOnDevice_) {
        MMX_HIP(hipMemcpyAsync(out, gvals_.p, gvals_.n * sizeof(double), hipMemcpyDeviceToHost, st_));
        streamWait();
      } else {
        std::memcpy(out, grid_.vals.data(), grid_.vals.size() * sizeof(double));
      }
      return;
    } else if (what == "Ehat") {
      std::memcpy(out, EhatH_, D * D * sizeof(double));
      return;
    } else {
      throw Error(MMADMM_ERR_INVALID, "mmadmm_get: unknown field '" + what + "'");
    }
    if (b == &B_) {  // wave-interleaved on the device: return simplex-major
      std::vector<double> h(b->n);
      MMX_HIP(hipMemcpyAsync(h.data(), b->p, b->n * sizeof(double), hipMemcpyDeviceToHost, st_));
      streamWait();
      for (int s = 0; s < nF_; ++s)
        for (int ij = 0; ij < K * K; ++ij) out[(size_t)s * K * K + ij] = h[bIndex(s, ij)];
      return;
    }
    MMX_HIP(hipMemcpyAsync(out, b->p, b->n * sizeof(double), hipMemcpyDeviceToHost, st_));
    streamWait();
  }

  // host mirror of bidx<D> (admm_kernels.hip)
  static size_t bIndex(int s, int ij) {
    if (D == 3 && MMX_B3_PAIRS) return ((size_t)(s >> 6) * K * K + (ij & ~1)) * 64 + 2 * (s & 63) + (ij & 1);
    return ((size_t)(s >> 6) * K * K + ij) * 64 + (s & 63);
  }

  void getSimplices(int32_t* F) override {  // this rank's simplices, global node ids, re-oriented
    for (size_t i = 0; i < plan_.Flocal.size(); ++i) F[i] = plan_.localNodes[plan_.Flocal[i]];
  }

  void localNodes(int* n, int32_t* ids) override {
    if (n) *n = nP_;
    if (ids) std::memcpy(ids, plan_.localNodes.data(), plan_.localNodes.size() * sizeof(int32_t));
  }

  void sizes(int* nP, int* nF, int* gridRows) override {
    if (nP) *nP = nP_;
    if (nF) *nF = nF_;
    if (gridRows) *gridRows = (int)(grid_.vals.size() / (D * D));
  }

  void setTiming(bool on) override {
    resolveTimed();
    timing_ = on;
  }

  void stats(mmadmm_stats* s) override {
    resolveTimed();
    *s = st_stats_;
    // algorithmic HBM bytes per launch: prox reads F, sbits, z, u, Bkinv,
    // writes z, u, Bkinv; x is gathered once per node.  x-update reads the incidence CSR,
    // z and u once each, xBar and invdiag, writes x.
    const double nF = nF_, nP = nP_;
    // + the gradient cache: K doubles read at entry and written by the last BFGS iteration
    // with the slot terms (tslot, 3D) the prox also writes K doubles per simplex and the x-update
    // reads those instead of z and u
    const double ts = tslotOn_ ? 1.0 : 0.0;
    s->prox_bytes = nF * (4.0 * (D + 1) + 1 + 8.0 * (2 * K + K * K) * 2 + 8.0 * K * 2 + ts * 8.0 * K) +
                    nP * 8.0 * D;
    s->xupdate_bytes = 4.0 * (nP + 1) + 4.0 * (D + 1) * nF + (16.0 - 8.0 * ts) * K * nF + 8.0 * D * nP * 2 + 8.0 * nP;
    s->monitor_iso = iso_ ? 1 : 0;
    s->halo_send_bytes = 8.0 * D * (double)plan_.sendOff.size();
    s->halo_recv_bytes = nranks_ > 1 ? 8.0 * D * (double)plan_.recvRows : 0.0;
    s->interior_nodes = nInner_;
    s->overlap = overlap_ ? 1 : 0;
  }

  void resetStats() override {
    resolveTimed();
    const mmadmm_stats z{};
    st_stats_ = z;
  }

  // the timed steps' HIP events -> the timers (every step ends with a stream synchronisation, so
  // its events have completed); the pool is then reused
  void resolveTimed() {
    if (stepEv_.empty() && timed_.empty() && exEv_.empty()) return;
    streamWait();
    float ms = 0;
    for (auto& p : stepEv_) {
      MMX_HIP(hipEventElapsedTime(&ms, p.first, p.second));
      st_stats_.t_step_ms += ms;
      st_stats_.n_steps_timed += 1;
    }
    if (st2_) MMX_HIP(hipStreamSynchronize(st2_));
    for (auto& p : exEv_) {
      MMX_HIP(hipEventElapsedTime(&ms, p.first, p.second));
      st_stats_.t_exchange_ms += ms;
      st_stats_.n_exchange += 1;
    }
    exEv_.clear();
    for (auto& t : timed_) {
      MMX_HIP(hipEventElapsedTime(&ms, t.a0, t.a1));
      st_stats_.t_prox_ms += ms;
      st_stats_.n_prox += 1;
      MMX_HIP(hipEventElapsedTime(&ms, t.a1, t.b1));
      st_stats_.t_xupdate_ms += ms;
      st_stats_.n_xupdate += 1;
    }
    stepEv_.clear();
    timed_.clear();
    evUsed_ = 0;
  }

  void sync() override { streamWait(); }

  void debugBlockGrad(int s, const double* z, const double* dx, int flags, double* out) override {
    if (s < 0 || s >= nF_) throw Error(MMADMM_ERR_INVALID, "debug_blockgrad: simplex out of range");
    DevBuf<double> dz, ddx, dout;
    dz.upload(z, K, st_);
    ddx.upload(dx, K, st_);
    dout.alloc(K + 2);
    launch_debug_blockgrad<D>(m_, s, dz.p, ddx.p, dout.p, flags, st_);
    MMX_HIP(hipMemcpyAsync(out, dout.p, (K + 2) * sizeof(double), hipMemcpyDeviceToHost, st_));
    streamWait();
  }

 private:
  struct Timed {
    hipEvent_t a0, a1, b1;
  };

  // buildMatrix (src/Mesh.cpp:262-382): the Jacobian's pattern over the D*nP unknowns, the
  // ParamIter of the reference and the symbolic ILU (sfac, done once as the reference does).
  // MMX_SCHED_PROF=1: the first backward-Euler step's host set-up phases on stderr
  static void profMark(const char* what, std::chrono::steady_clock::time_point& t) {
    static const bool on = getenv("MMX_SCHED_PROF") != nullptr;
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[sched] engine %s %.3f s\n", what, std::chrono::duration<double>(now - t).count());
    t = now;
  }
  void ensureJacobian() {
    if (jac_) return;
    auto tp = std::chrono::steady_clock::now();
    const int n = nP_ * D;
    mmx_struc sp = nullptr;
    MMX_SP(mmx_struc_create(n, 0, &sp));
    std::vector<int32_t> ia(n + 1), ja;
    long long nnz = 0;
    int rc = mmx_struc_mesh_pattern(sp, D, (int)(Fh_.size() / (D + 1)), Fh_.data());
    if (rc == MMADMM_OK) rc = mmx_struc_pack(sp);
    if (rc == MMADMM_OK) rc = mmx_struc_get(sp, nullptr, &nnz, nullptr, nullptr);
    if (rc == MMADMM_OK) {
      ja.resize(nnz);
      rc = mmx_struc_get(sp, nullptr, &nnz, ia.data(), ja.data());
    }
    profMark("pattern", tp);
    int dev = prm_.device;
    if (dev < 0) MMX_HIP(hipGetDevice(&dev));
    if (rc == MMADMM_OK) rc = mmx_matrix_create_from_struc(dev, sp, &jac_);
    (void)mmx_struc_destroy(sp);
    profMark("matrix create", tp);
    if (rc != MMADMM_OK) throw Error(rc, std::string("backward Euler Jacobian: ") + mmadmm_last_error());
    mmx_param_iter_mesh(&jprm_);
    maxColNodes_ = 0;  // the widest row's column nodes (the assembly's wavefront per node needs <= 64)
    for (int r = 0; r < n; ++r) maxColNodes_ = std::max(maxColNodes_, (ia[r + 1] - ia[r]) / D);
    jia_.upload(ia.data(), ia.size(), st_);
    jja_.upload(ja.data(), ja.size(), st_);
    jval_.alloc(std::max<size_t>(nnz, 1));
    dv_.alloc(std::max<size_t>((size_t)nF_ * (D + 1) * D * K, 1));
    // the FD blocks' fast pass queues its near-midpoint lanes here (MMX_FDJ_FAST=0: one exact pass)
    const char* ff = getenv("MMX_FDJ_FAST");
    if (!(ff && atoi(ff) == 0)) fdWork_.alloc((size_t)nF_ * (D + 1) + 1);
    xn_.alloc((size_t)n);
    rhs_.alloc((size_t)n);
    dx_.alloc((size_t)n);
    streamWait();
  }

  // buildEulerJac (src/Mesh.cpp:1112-1136); sfac after the first build (src/Mesh.cpp:1287-1290).
  // The Jacobian is evaluated at Vp, which only step() and done() move: a rebuild with the same
  // Vp and dt reproduces the current values bit for bit and is skipped (and so is the solver's
  // re-factorisation of unchanged values).
  void buildJacobian(double dtBE) {
    if (jacVp_ == vpVersion_ && jacDt_ == dtBE) return;
    jacVp_ = vpVersion_;
    jacDt_ = dtBE;
    const auto t0 = Clock::now();
    auto tp = t0;
    const double h = 10.0 * sqrt(std::numeric_limits<double>::epsilon());
    launch_fd_jac<D>(m_, Vp_.p, h, dv_.p, st_, fdWork_.p);
    clearInvFlag();
    launch_jac_assemble<D>(m_, jia_.p, jja_.p, dv_.p, dtBE / prm_.tau, jval_.p, st_, true, maxColNodes_);
    streamWait();
    profMark("FD Jacobian + assembly", tp);
    MMX_SP(mmx_matrix_set_values_device(jac_, jval_.p));
    if (!jacFactored_) {
      MMX_SP(mmx_matrix_sfac(jac_, &jprm_));
      jacFactored_ = true;
      profMark("sfac", tp);
    }
    streamWait();
    st_stats_.jacobians += 1;
    st_stats_.t_jac_ms += msSince(t0);
  }
  using Clock = std::chrono::steady_clock;
  static double msSince(Clock::time_point t) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t).count();
  }

  static double hostDet(const double (&a)[3][3]) {  // Eigen 2x2 / 3x3 determinant
    if (D == 2) return a[0][0] * a[1][1] - a[1][0] * a[0][1];
    const double h0 = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]);
    const double h1 = a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]);
    const double h2 = a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
    return h0 - h1 + h2;
  }

  // halo exchange of interface-slot values with the neighbouring ranks: mode 0 x-update terms,
  // 1 simplex gradients
  void exchange(int mode, const PackZX& pz = {}, hipStream_t st = nullptr) {
    if (nranks_ == 1) return;
    if (!st) st = st_;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing_ && mode == 0) {
      e0 = nextEvent();
      MMX_HIP(hipEventRecord(e0, st));
    }
    launch_pack_export<D>(mode, (int)plan_.sendOff.size(), expOff_.p, z_.p, uPtr(), gs_.p, w_, export_.p, st, pz);
    comm_->exchange(rank_, export_.p, remote_.p, plan_.peers, D, st);
    if (e0) {
      e1 = nextEvent();
      MMX_HIP(hipEventRecord(e1, st));
      exEv_.push_back({e0, e1});
    }
  }

  // the x-update of every node with the halo exchange (mode 0) before it.  On an element partition
  // (overlap_) the interior nodes -- no slot of another rank, first in the node order -- are updated
  // on the step's stream while the pack and the send/recv run on a second stream; the interface
  // nodes follow once the exchange is in.  Each node's sum is the same either way (ascending
  // global simplex id), so the positions are bit-identical; only the residual partials come as two
  // consecutive sets.  (src/MeshIntegrator.cpp:146-160: the consensus the exchange feeds.)
  void xupdateHalo(const StepScalars& sc, int* nbx, bool resid, bool useTs, const PackZX& pz) {
    if (!overlap_) {
      exchange(0, pz);
      launch_xupdate<D>(m_, sc, xBar_.p, z_.p, uPtr(), x_.p, partB_.p, nbx, resid, st_, useTs);
      return;
    }
    MMX_HIP(hipEventRecord(evProx_, st_));
    DeviceMesh<D> mi = m_;
    mi.xupHi = nInner_;
    int nb1 = 0, nb2 = 0;
    launch_xupdate<D>(mi, sc, xBar_.p, z_.p, uPtr(), x_.p, partB_.p, &nb1, resid, st_, useTs);
    MMX_HIP(hipStreamWaitEvent(st2_, evProx_, 0));
    exchange(0, pz, st2_);
    MMX_HIP(hipEventRecord(evEx_, st2_));
    MMX_HIP(hipStreamWaitEvent(st_, evEx_, 0));
    DeviceMesh<D> mb = m_;
    mb.xupLo = nInner_;
    launch_xupdate<D>(mb, sc, xBar_.p, z_.p, uPtr(), x_.p, partB_.p + (size_t)nb1 * kNumPartials, &nb2, resid, st_,
                      useTs);
    *nbx = nb1 + nb2;
  }

  // rows x 2*kNumPartials scalar records on the device -> combined over ranks on the host
  // (sums in rank order; the max-BFGS entry by max)
  // the stream's work so far has completed: an event polled in a spin (low wake-up latency; the
  // blocking stream wait costs tens of microseconds per step), or the stream wait (MMX_SPIN=0)
  void waitStream() {
    if (!spinWait_) {
      streamWait();
      return;
    }
    if (!evSync_) MMX_HIP(hipEventCreateWithFlags(&evSync_, hipEventDisableTiming));
    MMX_HIP(hipEventRecord(evSync_, st_));
    hipError_t r;
    while ((r = hipEventQuery(evSync_)) == hipErrorNotReady) __builtin_ia32_pause();
    MMX_HIP(r);
  }

  // hipStreamSynchronize, on an element partition bounded by the communicator's deadline (a peer
  // that never sends its halo ends the step with MMADMM_ERR_RCCL, comm_poll.h)
  void streamWait() {
    if (nranks_ > 1 && comm_)
      comm_->wait(st_);
    else
      MMX_HIP(hipStreamSynchronize(st_));
  }

  void fetchResults(const double* dev, int rows, std::vector<double>& out) {
    const size_t cnt = (size_t)rows * 2 * kNumPartials;
    out.resize(cnt);
    if (resH_) {  // pinned, written by the reductions themselves
      waitStream();
      std::memcpy(out.data(), resH_ + (dev - res_), cnt * sizeof(double));
      return;
    }
    if (nranks_ == 1) {
      MMX_HIP(hipMemcpyAsync(out.data(), dev, cnt * sizeof(double), hipMemcpyDeviceToHost, st_));
      streamWait();
      return;
    }
    if (resAll_.n < cnt * nranks_) resAll_.alloc(cnt * nranks_);
    comm_->allgather(rank_, dev, resAll_.p, cnt, st_);
    std::vector<double> all(cnt * nranks_);
    MMX_HIP(hipMemcpyAsync(all.data(), resAll_.p, all.size() * sizeof(double), hipMemcpyDeviceToHost, st_));
    streamWait();
    for (size_t i = 0; i < cnt; ++i) {
      const bool isMax = (i % kNumPartials) == 5;
      double v = all[i];
      for (int q = 1; q < nranks_; ++q) v = isMax ? std::max(v, all[(size_t)q * cnt + i]) : v + all[(size_t)q * cnt + i];
      out[i] = v;
    }
  }

  // The monitor grid rebuilt on the device from the current vertices Vp: bounding
  // box, monitor at the vertices (MonType 7 on the device at time t; any other monitor through its
  // host callback), nearest vertex of every grid point, smoothing -- bit-identical to the host
  // set-up (regrid_kernels.hip).  One 2D-double readback (the bounding box) per call.
  // On an element partition (regridNear) a rank rebuilds only the box of grid rows its monitor
  // evaluations can reach, and receives only the vertices that can be nearest to a point of that
  // box: the ranks all-gather their bounding boxes (the global box sets the grid geometry, the same
  // on every rank) and their search boxes S (the row box widened by a margin), each rank sends
  // the vertices it owns (lowest incident simplex) that lie in another rank's S to that rank, and
  // the nearest-vertex fill over these candidates checks, point by point, that its answer is
  // strictly nearer than S's boundary -- so no vertex it does not hold can be as near, and the
  // rows equal the single-GPU grid's.  If any point of any rank fails the check (all ranks agree
  // on it), the rebuild falls back to regridAll: every owned vertex all-gathered to every rank.
  void setRegrid(bool on) override { regridEachStep_ = on; }

  void regrid(double t) override {
    if (nranks_ > 1) {
      const char* mode = getenv("MMX_REGRID_GATHER");  // "all": the full all-gather (round 3)
      if (!(mode && std::string(mode) == "all") && regridNear(t)) return;
      st_stats_.regrid_fallbacks += (mode && std::string(mode) == "all") ? 0 : 1;
    }
    regridAll(t);
  }

  // the partitioned rebuild from the candidates near this rank's box; false: fall back (collective)
  bool regridNear(double t) {
    constexpr int DD = D * D;
    const int nG = plan_.nP;
    const int nbl = std::max(1, std::min(256, (nP_ + 255) / 256));
    const int nbe = std::max(1, std::min(256, (nF_ + 255) / 256));
    const size_t smallN = (size_t)std::max(2 * D, nranks_);
    if (!rgnPart_.p) {
      rgnPart_.alloc((size_t)256 * 2 * D + 256 * D);
      rgnSmallS_.alloc(smallN);
      rgnSmallR_.alloc(smallN * nranks_);
      rgnSbox_.alloc((size_t)nranks_ * 2 * D);
      rgnCnt_.alloc(nranks_ + 1);  // + the fail flag
      rgnSend_.alloc((size_t)nranks_ * maxOwned_ * (D + 1));
      rgnGid_.upload(plan_.localNodes.data(), plan_.localNodes.size(), st_);
      ownGidH_.assign(ownAllGidH_.begin() + (size_t)rank_ * maxOwned_,
                      ownAllGidH_.begin() + (size_t)rank_ * maxOwned_ + std::max(nOwned_, 1));
      rgnOwnGid_.upload(ownGidH_.data(), ownGidH_.size(), st_);
      rgTmp_.alloc(gvals_.n);
      rgTmp2_.alloc(gvals_.n);
      MMX_HIP(hipHostMalloc((void**)&rgnHost_, sizeof(double) * ((size_t)256 * 3 * D + 2 * smallN * nranks_ + 64),
                            hipHostMallocDefault));
    }
    double* H0 = rgnHost_;
    // this rank's bounding box and widest simplex per axis
    launch_bbox<D>(Vp_.p, nP_, rgnPart_.p, nbl, st_);
    launch_extent<D>(Vp_.p, F_.p, nF_, rgnPart_.p + (size_t)256 * 2 * D, nbe, st_);
    MMX_HIP(hipMemcpyAsync(H0, rgnPart_.p, sizeof(double) * nbl * 2 * D, hipMemcpyDeviceToHost, st_));
    MMX_HIP(hipMemcpyAsync(H0 + (size_t)256 * 2 * D, rgnPart_.p + (size_t)256 * 2 * D, sizeof(double) * nbe * D,
                           hipMemcpyDeviceToHost, st_));
    streamWait();
    double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int b = 0; b < nbl; ++b)
      for (int d = 0; d < D; ++d) {
        llo[d] = std::min(llo[d], H0[(size_t)b * 2 * D + d]);
        lhi[d] = std::max(lhi[d], H0[(size_t)b * 2 * D + D + d]);
      }
    for (int d = 0; d < D; ++d) extMax_[d] = 0.0;
    for (int b = 0; b < nbe; ++b)
      for (int d = 0; d < D; ++d) extMax_[d] = std::max(extMax_[d], H0[(size_t)256 * 2 * D + (size_t)b * D + d]);
    // the global box: every vertex is some rank's, so the union of the ranks' boxes (min / max exact)
    double* hs = H0 + (size_t)256 * 3 * D;  // small host staging
    double* hr = hs + smallN;
    auto smallGather = [&](const double* in, int n) {  // n doubles per rank -> hr[q * n + i]
      MMX_HIP(hipMemcpyAsync(rgnSmallS_.p, in, sizeof(double) * n, hipMemcpyHostToDevice, st_));
      comm_->allgather(rank_, rgnSmallS_.p, rgnSmallR_.p, (size_t)n, st_);
      MMX_HIP(hipMemcpyAsync(hr, rgnSmallR_.p, sizeof(double) * n * nranks_, hipMemcpyDeviceToHost, st_));
      streamWait();
    };
    for (int d = 0; d < D; ++d) {
      hs[d] = llo[d];
      hs[D + d] = lhi[d];
    }
    smallGather(hs, 2 * D);
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int q = 0; q < nranks_; ++q)
      for (int d = 0; d < D; ++d) {
        lo[d] = std::min(lo[d], hr[(size_t)q * 2 * D + d]);
        hi[d] = std::max(hi[d], hr[(size_t)q * 2 * D + D + d]);
      }
    setGridGeometry(nG, lo, hi);
    const CellGrid cg = cellGrid(lo, hi);
    int marg[3] = {0, 0, 0};
    const GridBox R = rowBox(llo, lhi, marg);
    const int passes = smoothPasses();
    const GridBox H = widenBox(R, passes);
    // the search box S: the grid points of H's rows widened by a simplex diameter and two cells (a
    // point inside the mesh lies in some simplex, within its diameter of each of its vertices; the
    // fill checks the margin point by point).  The fill gives storage row (sx, sy, k) the point
    // (gx[sx], gy[sy], gz[k]) in 2D but (gx[sy], gy[sx], gz[k]) in 3D (the host layout's x/y swap,
    // src/MeshInterpolator.cpp:234)
    double slo[3] = {0, 0, 0}, shi[3] = {0, 0, 0};
    double diam = 0.0;
    for (int d = 0; d < D; ++d) diam += extMax_[d] * extMax_[d];
    diam = std::sqrt(diam);
    const char* mg = getenv("MMX_REGRID_MARGIN");  // tests: 0 forces the fallback below
    const double marginScale = mg ? atof(mg) : 1.0;
    for (int d = 0; d < D; ++d) {
      const std::vector<double>& g = d == 0 ? grid_.gx : d == 1 ? grid_.gy : grid_.gz;
      const int sd = (D == 3 && d < 2) ? 1 - d : d;  // the storage axis holding coordinate axis d
      const double mu = marginScale * (diam + 2.0 * (g[1] - g[0]));
      slo[d] = g[H.lo[sd]] - mu;
      shi[d] = g[H.hi[sd]] + mu;
    }
    for (int d = 0; d < D; ++d) {
      hs[d] = slo[d];
      hs[D + d] = shi[d];
    }
    smallGather(hs, 2 * D);
    MMX_HIP(hipMemcpyAsync(rgnSbox_.p, hr, sizeof(double) * nranks_ * 2 * D, hipMemcpyHostToDevice, st_));
    // my owned vertices in the other ranks' boxes, per destination
    MMX_HIP(hipMemsetAsync(rgnCnt_.p, 0, sizeof(int) * (nranks_ + 1), st_));
    launch_select_owned<D>(Vp_.p, ownLocal_.p, rgnOwnGid_.p, nOwned_, nranks_, rank_, rgnSbox_.p, rgnCnt_.p,
                           rgnSend_.p, maxOwned_, st_);
    std::vector<int> cnt(nranks_ + 1);
    MMX_HIP(hipMemcpyAsync(cnt.data(), rgnCnt_.p, sizeof(int) * nranks_, hipMemcpyDeviceToHost, st_));
    streamWait();
    for (int q = 0; q < nranks_; ++q) hs[q] = (double)cnt[q];
    smallGather(hs, nranks_);
    std::vector<HaloPeer> peers;
    int nRecv = 0;
    for (int q = 0; q < nranks_; ++q) {
      if (q == rank_) continue;
      const int sc = cnt[q], rc = (int)hr[(size_t)q * nranks_ + rank_];
      if (sc == 0 && rc == 0) continue;
      HaloPeer p;
      p.rank = q;
      p.sendOff = q * maxOwned_;
      p.sendCount = sc;
      p.recvOff = nRecv;
      p.recvCount = rc;
      nRecv += rc;
      peers.push_back(p);
    }
    const int nCand = nP_ + nRecv;
    if ((int)rgnRecv_.n < std::max(nRecv, 1) * (D + 1)) rgnRecv_.alloc((size_t)std::max(nRecv, 1) * (D + 1) * 2);
    if ((int)rgnCandX_.n < nCand * D) {
      rgnCandX_.alloc((size_t)nCand * D * 2);
      rgnCandGid_.alloc((size_t)nCand * 2);
      rgnCellOf_.alloc((size_t)nCand * 2);
      rgnNodes_.alloc((size_t)nCand * 2);
      rgnMon_.alloc((size_t)nCand * DD * 2);
    }
    comm_->exchange(rank_, rgnSend_.p, rgnRecv_.p, peers, D + 1, st_);
    launch_build_cand<D>(Vp_.p, rgnGid_.p, nP_, rgnRecv_.p, nRecv, rgnCandX_.p, rgnCandGid_.p, st_);
    evalMonitorAt(rgnCandX_.p, nCand, t, rgnMon_.p);
    ensureCells(cg);
    launch_bin<D>(rgnCandX_.p, nCand, cg, rgnCellOf_.p, rgCounts_.p, rgStarts_.p, rgFill_.p, rgnNodes_.p, rgScan_.p,
                  rgScanBytes_, st_);
    // the fill's exactness check: a vertex this rank lacks lies outside S, beyond one of S's sides --
    // but not beyond a side at or past the global vertex box (every vertex x has lo <= x <= hi, and S
    // holds x >= slo, x <= shi): such a side is infinitely far (a disc's grid corners are far from
    // every vertex, nearer S's outer side than any vertex)
    double clo[3], chi[3];
    for (int d = 0; d < 3; ++d) {
      clo[d] = (d < D && slo[d] <= lo[d]) ? -INFINITY : slo[d];
      chi[d] = (d < D && shi[d] >= hi[d]) ? INFINITY : shi[d];
    }
    NnCand nc{rgnCandGid_.p, {clo[0], clo[1], clo[2]}, {chi[0], chi[1], chi[2]}, rgnCnt_.p + nranks_};
    launch_nn_fill<D>(rgnCandX_.p, cg, rgStarts_.p, rgnNodes_.p, gx_.p, gy_.p, D == 3 ? gz_.p : gy_.p, grid_.nx,
                      grid_.ny, grid_.nz, rgnMon_.p, rgTmp_.p, H, st_, nc);
    int fail = 0;
    MMX_HIP(hipMemcpyAsync(&fail, rgnCnt_.p + nranks_, sizeof(int), hipMemcpyDeviceToHost, st_));
    streamWait();
    hs[0] = (double)fail;
    smallGather(hs, 1);
    for (int q = 0; q < nranks_; ++q)
      if (hr[q] != 0.0) return false;  // some point of some rank: rebuild from every vertex
    smoothCommit(R, passes, true);
    st_stats_.regrid_rows = (long long)(H.hi[0] - H.lo[0] + 1) * (H.hi[1] - H.lo[1] + 1) * (H.hi[2] - H.lo[2] + 1);
    st_stats_.regrid_gather_bytes = (double)sizeof(double) * ((size_t)nranks_ * (4 * D + nranks_ + 1) +
                                                              (size_t)nRecv * (D + 1));
    st_stats_.regrid_cand = nCand;
    MMX_HIP(hipGetLastError());
    gridOnDevice_ = true;
    updateIso();
    m_ = makeView();
    st_stats_.regrids += 1;
    return true;
  }

  // An isotropic monitor grid (every point a multiple of the identity, bit for bit: the built-in
  // MEx1/3/4/5 and moving-bump monitors; NaN rows of a partitioned rebuild count as isotropic) is
  // also kept as one value per point, and evalMonitor then gathers 8 bytes per cell corner instead
  // of 8 D^2 (2D: C3 prox -4.6%).  Checked on the device after every
  // (re)build; MMX_ISO=0 keeps the full rows.
  void updateIso() {
    iso_ = false;
    const char* e = getenv("MMX_ISO");
    if (e && atoi(e) == 0) return;
    const long long np = (long long)(gvals_.n / (D * D));
    if (np <= 0) return;
    if ((long long)giso_.n != np) giso_.alloc(np);
    if (!isoFlag_.p) isoFlag_.alloc(1);
    MMX_HIP(hipMemsetAsync(isoFlag_.p, 0, sizeof(int), st_));
    launch_iso_compact<D>(gvals_.p, np, giso_.p, isoFlag_.p, st_);
    int notIso = 1;
    MMX_HIP(hipMemcpyAsync(&notIso, isoFlag_.p, sizeof(int), hipMemcpyDeviceToHost, st_));
    streamWait();
    iso_ = (notIso == 0);
  }
  // the grid coordinates and, in 3D, each axis's cell table {g_i, h_i = g_{i+1} - g_i, RN(1/h_i), 0}
  // (blockGrad's monitor interpolation, MMX_MON_RECIP)
  void uploadGridCoords() {
    gx_.upload(grid_.gx.data(), grid_.gx.size(), st_);
    gy_.upload(grid_.gy.data(), grid_.gy.size(), st_);
    if (D == 3) {
      gz_.upload(grid_.gz.data(), grid_.gz.size(), st_);
      const std::vector<double>* ax[3] = {&grid_.gx, &grid_.gy, &grid_.gz};
      for (int a = 0; a < 3; ++a) {
        const std::vector<double>& g = *ax[a];
        const size_t nc = g.size() > 1 ? g.size() - 1 : 1;
        std::vector<double>& t = gcellH_[a];
        t.assign(4 * nc, 0.0);
        for (size_t i = 0; i + 1 < g.size(); ++i) {
          const double h = g[i + 1] - g[i];
          t[4 * i] = g[i];
          t[4 * i + 1] = h;
          t[4 * i + 2] = 1.0 / h;
        }
        gcell_[a].upload(t.data(), t.size(), st_);
      }
    }
  }
  void setGridGeometry(int nG, const double* lo, const double* hi) {
    grid_geometry(D, nG, lo, hi, grid_);
    uploadGridCoords();
  }
  // vertex cells over the global box: about two vertices per cell
  CellGrid cellGrid(const double* lo, const double* hi) const {
    CellGrid cg{};
    const int gn[3] = {grid_.nx, grid_.ny, grid_.nz};
    cg.hmin = INFINITY;
    for (int d = 0; d < 3; ++d) {
      const double ext = d < D ? hi[d] - lo[d] : 0.0;
      cg.lo[d] = d < D ? lo[d] : 0.0;
      cg.n[d] = (d < D && ext > 0) ? std::max(1, gn[d] / 2) : 1;
      cg.inv[d] = (d < D && ext > 0) ? cg.n[d] / ext : 0.0;
      if (d < D && ext > 0) cg.hmin = std::min(cg.hmin, ext / cg.n[d]);
    }
    if (!(cg.hmin < INFINITY)) cg.hmin = 0.0;
    return cg;
  }
  void ensureCells(const CellGrid& cg) {
    const int ncell = cg.n[0] * cg.n[1] * cg.n[2];
    if ((int)rgStarts_.n < ncell + 1) {
      rgCounts_.alloc(ncell + 1);
      rgStarts_.alloc(ncell + 1);
      rgFill_.alloc(ncell);
      rgScanBytes_ = bin_scan_bytes(ncell);
      rgScan_.alloc(std::max<size_t>(rgScanBytes_, 1));
    }
  }
  static int smoothPasses() { return (D == 2) ? 5 : 2; }  // smoothMonitorGrid
  // the grid rows this rank's monitor evaluations can reach: its vertices' bounding box widened by
  // two local simplex extents and two cells (marg[d] rows) for the motion within a step
  GridBox rowBox(const double* llo, const double* lhi, int* marg) const {
    const int gn3[3] = {grid_.nx, grid_.ny, D == 3 ? grid_.nz : 0};
    GridBox R{{0, 0, 0}, {gn3[0], gn3[1], gn3[2]}};
    for (int d = 0; d < D; ++d) {  // evalMonitor reads rows zInd P + yInd (nx+1) + xInd: storage axis d = axis d
      const std::vector<double>& g = d == 0 ? grid_.gx : d == 1 ? grid_.gy : grid_.gz;
      const double h = g[1] - g[0];
      const int M = (int)std::ceil(2.0 * extMax_[d] / h) + 2;
      marg[d] = M;
      R.lo[d] = std::max(0, std::min(gn3[d], (int)std::floor((llo[d] - g[0]) / h) - M));
      R.hi[d] = std::max(0, std::min(gn3[d], (int)std::floor((lhi[d] - g[0]) / h) + 1 + M));
    }
    return R;
  }
  GridBox widenBox(const GridBox& b, int w) const {
    const int gn3[3] = {grid_.nx, grid_.ny, D == 3 ? grid_.nz : 0};
    GridBox o = b;
    for (int d = 0; d < D; ++d) {
      o.lo[d] = std::max(0, b.lo[d] - w);
      o.hi[d] = std::min(gn3[d], b.hi[d] + w);
    }
    return o;
  }
  // the monitor at n vertices (MonitorFunction::evaluateAtVertices, src/MonitorFunction.cpp:16-32)
  void evalMonitorAt(const double* X, int n, double t, double* mon) {
    constexpr int DD = D * D;
    if (builtin_monitor_kind(monFn_, monUser_) == 7) {
      double c[3];
      moving_bump_centre(t, c);
      launch_monitor_tv<D>(X, n, c, mon, st_);
    } else {  // a host plugin: evaluated on the host at the current vertices, as the reference does
      std::vector<double> Xh((size_t)n * D), mv((size_t)n * DD);
      MMX_HIP(hipMemcpyAsync(Xh.data(), X, Xh.size() * sizeof(double), hipMemcpyDeviceToHost, st_));
      streamWait();
      for (int v = 0; v < n; ++v) {
        double M[9];
        for (int i = 0; i < DD; ++i) M[i] = 0.0;
        monFn_(D, &Xh[(size_t)v * D], M, monUser_);
        std::memcpy(&mv[(size_t)v * DD], M, DD * sizeof(double));
      }
      MMX_HIP(hipMemcpyAsync(mon, mv.data(), mv.size() * sizeof(double), hipMemcpyHostToDevice, st_));
      streamWait();
    }
  }
  // smoothing passes over the box (shrinking halo) and the commit: the rows of R (NaN elsewhere)
  // on a partition, the whole grid on one rank
  void smoothCommit(const GridBox& R, int passes, bool part) {
    double* cur = rgTmp_.p;
    double* oth = part ? rgTmp2_.p : gvals_.p;
    for (int it = 0; it < passes; ++it) {
      launch_smooth<D>(cur, oth, grid_.nx, grid_.ny, grid_.nz, widenBox(R, part ? passes - 1 - it : 0), st_);
      std::swap(cur, oth);
    }
    if (part) {
      launch_box_commit<D>(cur, gvals_.p, D == 3 ? gpad_.p : nullptr, grid_.nx, grid_.ny, grid_.nz, R, st_);
    } else {
      if (cur != gvals_.p)
        MMX_HIP(hipMemcpyAsync(gvals_.p, cur, gvals_.n * sizeof(double), hipMemcpyDeviceToDevice, st_));
      if (D == 3) launch_pad_rows(gvals_.p, (long long)(gvals_.n / 9), gpad_.p, st_);
    }
  }

  // every vertex: on one rank its own; on a partition each rank's owned vertices all-gathered to
  // every rank (the fallback of regridNear, and MMX_REGRID_GATHER=all)
  void regridAll(double t) {
    constexpr int DD = D * D;
    const int nG = (nranks_ > 1) ? plan_.nP : nP_;  // vertices the grid is built from
    const int nb = std::max(1, std::min(256, (nG + 255) / 256));
    if (!rgPart_.p) {
      rgPart_.alloc((size_t)512 * 2 * D + 256 * D);  // global bbox partials, this rank's, its simplex extents
      rgMon_.alloc((size_t)nG * DD);
      rgCellOf_.alloc(nG);
      rgNodes_.alloc(nG);
      rgTmp_.alloc(gvals_.n);
      if (nranks_ > 1) rgTmp2_.alloc(gvals_.n);
      if (nranks_ > 1) {
        rgXg_.alloc((size_t)nG * D);
        rgSend_.alloc((size_t)maxOwned_ * D);
        rgRecv_.alloc((size_t)nranks_ * maxOwned_ * D);
      }
      MMX_HIP(hipHostMalloc((void**)&rgHost_, sizeof(double) * (512 * 2 * D + 256 * D), hipHostMallocDefault));
    }
    const double* X = Vp_.p;
    const bool part = nranks_ > 1;
    const int nbl = part ? std::max(1, std::min(256, (nP_ + 255) / 256)) : 0;  // blocks of the local bbox
    const int nbe = part ? std::max(1, std::min(256, (nF_ + 255) / 256)) : 0;  // blocks of the simplex extents
    double* extPart = rgPart_.p + (size_t)512 * 2 * D;
    if (part) {
      launch_rows_gather(D, ownLocal_.p, nOwned_, Vp_.p, rgSend_.p, st_);
      comm_->allgather(rank_, rgSend_.p, rgRecv_.p, (size_t)maxOwned_ * D, st_);
      launch_rows_scatter(D, ownAllGid_.p, nranks_ * maxOwned_, rgRecv_.p, rgXg_.p, st_);
      X = rgXg_.p;
      launch_bbox<D>(Vp_.p, nP_, rgPart_.p + (size_t)256 * 2 * D, nbl, st_);  // this rank's vertices
      launch_extent<D>(Vp_.p, F_.p, nF_, extPart, nbe, st_);  // its widest simplex per axis, now
    }
    launch_bbox<D>(X, nG, rgPart_.p, nb, st_);
    MMX_HIP(hipMemcpyAsync(rgHost_, rgPart_.p, sizeof(double) * nb * 2 * D, hipMemcpyDeviceToHost, st_));
    if (part) {
      MMX_HIP(hipMemcpyAsync(rgHost_ + (size_t)256 * 2 * D, rgPart_.p + (size_t)256 * 2 * D, sizeof(double) * nbl * 2 * D,
                             hipMemcpyDeviceToHost, st_));
      MMX_HIP(hipMemcpyAsync(rgHost_ + (size_t)512 * 2 * D, extPart, sizeof(double) * nbe * D, hipMemcpyDeviceToHost,
                             st_));
    }
    streamWait();
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int b = 0; b < nb; ++b)
      for (int d = 0; d < D; ++d) {
        lo[d] = std::min(lo[d], rgHost_[(size_t)b * 2 * D + d]);
        hi[d] = std::max(hi[d], rgHost_[(size_t)b * 2 * D + D + d]);
      }
    for (int b = 0; b < nbl; ++b)
      for (int d = 0; d < D; ++d) {
        llo[d] = std::min(llo[d], rgHost_[(size_t)(256 + b) * 2 * D + d]);
        lhi[d] = std::max(lhi[d], rgHost_[(size_t)(256 + b) * 2 * D + D + d]);
      }
    if (part) {  // the box margin follows the mesh: the widest local simplex per axis at these positions
      for (int d = 0; d < D; ++d) extMax_[d] = 0.0;
      for (int b = 0; b < nbe; ++b)
        for (int d = 0; d < D; ++d) extMax_[d] = std::max(extMax_[d], rgHost_[(size_t)512 * 2 * D + (size_t)b * D + d]);
    }
    grid_geometry(D, nG, lo, hi, grid_);
    uploadGridCoords();
    // vertex cells: about two vertices per cell
    CellGrid cg{};
    const int gn[3] = {grid_.nx, grid_.ny, grid_.nz};
    cg.hmin = INFINITY;
    for (int d = 0; d < 3; ++d) {
      const double ext = d < D ? hi[d] - lo[d] : 0.0;
      cg.lo[d] = d < D ? lo[d] : 0.0;
      cg.n[d] = (d < D && ext > 0) ? std::max(1, gn[d] / 2) : 1;
      cg.inv[d] = (d < D && ext > 0) ? cg.n[d] / ext : 0.0;
      if (d < D && ext > 0) cg.hmin = std::min(cg.hmin, ext / cg.n[d]);
    }
    if (!(cg.hmin < INFINITY)) cg.hmin = 0.0;
    const int ncell = cg.n[0] * cg.n[1] * cg.n[2];
    if ((int)rgStarts_.n < ncell + 1) {
      rgCounts_.alloc(ncell + 1);
      rgStarts_.alloc(ncell + 1);
      rgFill_.alloc(ncell);
      rgScanBytes_ = bin_scan_bytes(ncell);
      rgScan_.alloc(std::max<size_t>(rgScanBytes_, 1));
    }
    launch_bin<D>(X, nG, cg, rgCellOf_.p, rgCounts_.p, rgStarts_.p, rgFill_.p, rgNodes_.p, rgScan_.p, rgScanBytes_,
                  st_);
    // the monitor at the vertices (MonitorFunction::evaluateAtVertices, src/MonitorFunction.cpp:16-32)
    if (builtin_monitor_kind(monFn_, monUser_) == 7) {
      double c[3];
      moving_bump_centre(t, c);
      launch_monitor_tv<D>(X, nG, c, rgMon_.p, st_);
    } else {  // a host plugin: evaluated on the host at the current vertices, as the reference does
      std::vector<double> Xh((size_t)nG * D), mv((size_t)nG * DD);
      MMX_HIP(hipMemcpyAsync(Xh.data(), X, Xh.size() * sizeof(double), hipMemcpyDeviceToHost, st_));
      streamWait();
      for (int v = 0; v < nG; ++v) {
        double M[9];
        for (int i = 0; i < DD; ++i) M[i] = 0.0;
        monFn_(D, &Xh[(size_t)v * D], M, monUser_);
        std::memcpy(&mv[(size_t)v * DD], M, DD * sizeof(double));
      }
      MMX_HIP(hipMemcpyAsync(rgMon_.p, mv.data(), mv.size() * sizeof(double), hipMemcpyHostToDevice, st_));
      streamWait();
    }
    // the grid rows to rebuild: all of them on one rank; on an element partition the box of rows
    // this rank's monitor evaluations can reach (its vertices' bounding box, widened by two
    // simplex extents and two cells for the motion within a step), plus the smoothing passes'
    // halo for the nearest-vertex fill.  Every vertex is binned, so each fill is exact; the rows
    // outside the box are set to NaN, so an evaluation that left the box could not pass silently.
    const int passes = (D == 2) ? 5 : 2;  // smoothMonitorGrid
    const int gn3[3] = {grid_.nx, grid_.ny, D == 3 ? grid_.nz : 0};
    GridBox R{{0, 0, 0}, {gn3[0], gn3[1], gn3[2]}};
    if (part) {
      for (int d = 0; d < D; ++d) {  // evalMonitor reads rows zInd P + yInd (nx+1) + xInd: storage axis d = axis d
        const std::vector<double>& g = d == 0 ? grid_.gx : d == 1 ? grid_.gy : grid_.gz;
        const double h = g[1] - g[0];
        const int M = (int)std::ceil(2.0 * extMax_[d] / h) + 2;
        R.lo[d] = std::max(0, std::min(gn3[d], (int)std::floor((llo[d] - g[0]) / h) - M));
        R.hi[d] = std::max(0, std::min(gn3[d], (int)std::floor((lhi[d] - g[0]) / h) + 1 + M));
      }
    }
    auto widen = [&](const GridBox& b, int w) {
      GridBox o = b;
      for (int d = 0; d < D; ++d) {
        o.lo[d] = std::max(0, b.lo[d] - w);
        o.hi[d] = std::min(gn3[d], b.hi[d] + w);
      }
      return o;
    };
    const GridBox H = widen(R, part ? passes : 0);
    launch_nn_fill<D>(X, cg, rgStarts_.p, rgNodes_.p, gx_.p, gy_.p, D == 3 ? gz_.p : gy_.p, grid_.nx, grid_.ny,
                      grid_.nz, rgMon_.p, rgTmp_.p, H, st_);
    double* cur = rgTmp_.p;
    double* oth = part ? rgTmp2_.p : gvals_.p;
    for (int it = 0; it < passes; ++it) {
      launch_smooth<D>(cur, oth, grid_.nx, grid_.ny, grid_.nz, widen(R, part ? passes - 1 - it : 0), st_);
      std::swap(cur, oth);
    }
    if (part) {
      launch_box_commit<D>(cur, gvals_.p, D == 3 ? gpad_.p : nullptr, grid_.nx, grid_.ny, grid_.nz, R, st_);
    } else {
      if (cur != gvals_.p)
        MMX_HIP(hipMemcpyAsync(gvals_.p, cur, gvals_.n * sizeof(double), hipMemcpyDeviceToDevice, st_));
      if (D == 3) launch_pad_rows(gvals_.p, (long long)(gvals_.n / 9), gpad_.p, st_);
    }
    st_stats_.regrid_rows = (long long)(H.hi[0] - H.lo[0] + 1) * (H.hi[1] - H.lo[1] + 1) * (H.hi[2] - H.lo[2] + 1);
    st_stats_.regrid_gather_bytes = part ? (double)nranks_ * maxOwned_ * D * sizeof(double) : 0.0;
    st_stats_.regrid_cand = part ? nG : 0;
    MMX_HIP(hipGetLastError());
    gridOnDevice_ = true;
    updateIso();
    m_ = makeView();
    st_stats_.regrids += 1;
  }

  DeviceMesh<D> makeView() const {
    DeviceMesh<D> m{};
    m.nP = nP_;
    m.nF = nF_;
    m.F = F_.p;
    m.sbits = sbits_.p;
    m.nodeInterior = interior_.p;
    m.inc_ptr = incPtr_.p;
    m.inc_off = incOff_.p;
    m.remote = nranks_ > 1 ? remote_.p : nullptr;
    m.tslot = tslotOn_ ? tslot_.p : nullptr;
    m.gcache = gcache_.p;
    m.tieList = tieList_.p;
    m.tieCount = tieCount_.p + tiePar_;  // keep the queue's parity across a rebuilt view (regrid)
    m.tieStale = tieCount_.p + (tiePar_ ^ 1);
    m.invFlag = tieCount_.p + 2;
    m.nodeOrder = nodeOrder_.p;
    m.xupLo = 0;
    m.xupHi = nP_;
    m.prox2dWave = wave2d_ ? 1 : 0;
    {
      const char* xs = getenv("MMX_XUP_SWEEP");  // 3D default: one workgroup per CU (profiles/r03/xupdate)
      m.xupSweep = xs ? std::max(0, atoi(xs)) : (D == 3 ? 1 : 0);
      const char* xc = getenv("MMX_XUP_CH");
      m.xupCh = xc ? atoi(xc) : 8;
    }
    {
      const char* ft = getenv("MMX_FORCE_TIE");
      m.forceTie = ft ? atoi(ft) : 0;
    }
    m.invdiag = invdiag_.p;
    m.Vc = compMesh_ ? Vc_.p : nullptr;
    m.gx = gx_.p;
    m.gy = gy_.p;
    m.gz = (D == 3) ? gz_.p : gy_.p;
    m.gvals = gvals_.p;
    m.gpad = (D == 3) ? gpad_.p : nullptr;
    for (int a = 0; a < 3; ++a) m.gcell[a] = (D == 3) ? gcell_[a].p : nullptr;
    m.giso = iso_ ? giso_.p : nullptr;
    m.gnx = grid_.nx;
    m.gny = grid_.ny;
    m.gnz = grid_.nz;
    // findLimInfMeshPoint divides by m[1] - m[0] (src/MeshUtils.h:47); the kernels use RN(1/h)
    m.ghx = grid_.gx[1] - grid_.gx[0];
    m.ghy = grid_.gy[1] - grid_.gy[0];
    m.ghz = (D == 3) ? grid_.gz[1] - grid_.gz[0] : 1.0;
    m.grhx = 1.0 / m.ghx;
    m.grhy = 1.0 / m.ghy;
    m.grhz = 1.0 / m.ghz;
    // linspace(xa, xb, ns): g[i] = xa + i*(xb - xa)/ns (src/MeshUtils.h:24-29), recomputed in-kernel
    const int ns[3] = {grid_.nx, grid_.ny, grid_.nz};
    double* A[3] = {&m.gax, &m.gay, &m.gaz};
    double* SP[3] = {&m.gspx, &m.gspy, &m.gspz};
    double* NS[3] = {&m.gnsx, &m.gnsy, &m.gnsz};
    double* RNS[3] = {&m.grnsx, &m.grnsy, &m.grnsz};
    for (int d = 0; d < 3; ++d) {
      const bool on = d < D;
      *A[d] = on ? grid_.lo[d] : 0.0;
      *SP[d] = on ? grid_.hi[d] - grid_.lo[d] : 0.0;
      *NS[d] = on ? (double)ns[d] : 1.0;
      *RNS[d] = 1.0 / *NS[d];
    }
    for (int i = 0; i < D * D; ++i) m.Ehat[i] = EhatH_[i];
    m.powd = powd_;
    m.w = w_;
    m.compMesh = compMesh_ ? 1 : 0;
    return m;
  }

  void ensureResults(int nIters) {
    if (nIters <= resultsCap_) return;
    resultsCap_ = std::max(nIters, 64);
    const size_t n = (size_t)resultsCap_ * 2 * kNumPartials;
    // one rank: the reductions write their results straight into pinned host memory (no copy
    // kernel) and the step waits for them by polling an event (MMX_SPIN=0: the stream wait and a
    // device buffer); C3: the step boundary's host turnaround ~54 us ->
    if (nranks_ == 1 && spinWait_) {
      if (resH_) MMX_HIP(hipHostFree(resH_));
      resH_ = nullptr;
      MMX_HIP(hipHostMalloc((void**)&resH_, n * sizeof(double), hipHostMallocMapped));
      MMX_HIP(hipHostGetDevicePointer((void**)&res_, resH_, 0));
    } else {
      results_.alloc(n);
      res_ = results_.p;
    }
  }

  // A NaN energy: an element met Edet <= 0 (the reference's assert(Edet > 0)) if a blockGrad set
  // the inverted flag, else a monitor value that is not finite -- on an element partition with a
  // time-varying monitor, an evaluation outside the grid box this rank rebuilt (its rows are NaN).
  // the inverted flag is set by any blockGrad that meets Edet <= 0 (energy(), the FD Jacobian
  // included) and read only by throwBad: every operation that can report starts from a clear flag
  void clearInvFlag() { MMX_HIP(hipMemsetAsync(tieCount_.p + 2, 0, sizeof(unsigned), st_)); }

  [[noreturn]] void throwBad(const char* where) {
    unsigned flag = 0;
    MMX_HIP(hipMemcpyAsync(&flag, tieCount_.p + 2, sizeof(unsigned), hipMemcpyDeviceToHost, st_));
    streamWait();
    if (flag) {
      MMX_HIP(hipMemsetAsync(tieCount_.p + 2, 0, sizeof(unsigned), st_));
      streamWait();
      throw Error(MMADMM_ERR_INVERTED, std::string("inverted element ") + where + " (reference: assert(Edet > 0))");
    }
    if (nranks_ > 1 && regridEachStep_)
      throw Error(MMADMM_ERR_NONFINITE, std::string("non-finite energy ") + where +
                                            ": a monitor evaluation left this rank's regrid box (no element inverted)");
    throw Error(MMADMM_ERR_NONFINITE, std::string("non-finite energy ") + where +
                                          " without an inverted element (a monitor value that is not finite)");
  }

  hipEvent_t nextEvent() {
    if (evUsed_ == evPool_.size()) {
      hipEvent_t e;
      // timing only: no system-scope fence at the record (each fenced record cost the stream ~5 us
      // of idle GPU -- C3: ~100 us per timed step; the timers are read after a stream wait)
      MMX_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
      evPool_.push_back(e);
    }
    return evPool_[evUsed_++];
  }

  int nP_ = 0, nF_ = 0;
  mmadmm_params prm_{};
  bool compMesh_ = false;
  double w_ = 0, powd_ = 0;
  double EhatH_[9] = {0};
  std::vector<int32_t> Fh_, maskH_;
  HostGrid grid_;
  // time-varying monitors: the monitor plugin, per-step regrid flag and the device set-up buffers
  mmadmm_monitor_fn monFn_ = nullptr;
  void* monUser_ = nullptr;
  bool regridEachStep_ = false, gridOnDevice_ = false;
  DevBuf<double> rgPart_, rgMon_, rgTmp_, rgTmp2_, rgXg_, rgSend_, rgRecv_;
  double extMax_[3] = {0.0, 0.0, 0.0};  // widest local simplex per axis (partitioned regrid box), per rebuild
  DevBuf<int> ownLocal_, ownAllGid_;  // partitioned regrid: my owned vertices (local ids), all ranks' (global ids)
  std::vector<int> ownAllGidH_, ownGidH_;
  // regridNear: partials, small all-gathers, search boxes, per-destination counts (+ the fail
  // flag), send / receive rows {x, gid}, candidates (positions, global ids, cells, monitor)
  DevBuf<double> rgnPart_, rgnSmallS_, rgnSmallR_, rgnSbox_, rgnSend_, rgnRecv_, rgnCandX_, rgnMon_;
  DevBuf<int> rgnCnt_, rgnGid_, rgnOwnGid_, rgnCandGid_, rgnCellOf_, rgnNodes_;
  double* rgnHost_ = nullptr;
  int nOwned_ = 0, maxOwned_ = 1;
  DevBuf<int> rgCellOf_, rgNodes_, rgCounts_, rgStarts_, rgFill_;
  DevBuf<unsigned char> rgScan_;
  size_t rgScanBytes_ = 0;
  double* rgHost_ = nullptr;
  hipStream_t st_ = nullptr;
  // element partition: the halo exchange's stream, its ordering events, the interior nodes' count
  // (the first nInner_ positions of the node order), the exchange timers
  hipStream_t st2_ = nullptr;
  hipEvent_t evProx_ = nullptr, evEx_ = nullptr;
  bool overlap_ = false;
  int nInner_ = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> exEv_;
  DevBuf<int32_t> F_, incPtr_, incOff_;
  DevBuf<double> tslot_;
  bool tslotOn_ = false;
  DevBuf<uint8_t> sbits_, interior_;
  DevBuf<double> gcell_[3];
  DevBuf<double> giso_;  // isotropic grid: one value per point (updateIso)
  DevBuf<int> isoFlag_;
  bool iso_ = false;
  std::vector<double> gcellH_[3];  // the cell tables' host images (kept until the async uploads finish)
  DevBuf<double> invdiag_, Vc_, gx_, gy_, gz_, gvals_, Vp_, x_, xPrev_, xBar_, z_, u_, gs_, B_, B2_, gcache_, gpad_;
  DevBuf<double> partA_, partB_, results_, export_, remote_, resAll_, redScratch_;
  RedWork red_;  // the split reductions' work space (launch_reduce_*)
  DevBuf<int32_t> expOff_, tieList_, nodeOrder_;
  bool wave2d_ = false;  // 2D prox through k_prox_wave<2> (double-buffered Bkinv)
  DevBuf<unsigned> tieCount_;
  int tiePar_ = 0;
  PartitionPlan plan_;
  Comm* comm_ = nullptr;
  int rank_ = 0, nranks_ = 1;
  int resultsCap_ = 0;
  std::vector<double> hostRes_;
  DeviceMesh<D> m_{};
  bool hessComputed_ = false, stepTaken_ = false, gcacheValid_ = false;
  // backward Euler: Jacobian (pattern, values, FD blocks), Newton vectors, the LASolver matrix
  mmx_matrix jac_ = nullptr;
  mmx_param_iter jprm_{};
  bool beStepTaken_ = false, jacFactored_ = false;
  long long vpVersion_ = 0, jacVp_ = -1;  // Vp generation; the one the Jacobian was built at
  double jacDt_ = 0.0;
  DevBuf<int32_t> jia_, jja_;
  DevBuf<double> jval_, jraw_, dv_, xn_, rhs_, dx_;
  DevBuf<unsigned> fdWork_;  // k_fd_jac's tie queue (count + lanes)
  int maxColNodes_ = 65;
  int stepsTaken_ = 0;
  size_t maxBlocks_ = 1;                 // partial-sum rows per launch (upper bound)
  static constexpr int kDeferMax = 64;   // deferred reductions up to this many ADMM iterations
  bool timing_ = false;
  std::vector<hipEvent_t> evPool_;
  size_t evUsed_ = 0;
  bool zFromX_ = false;
  bool fusePred_ = true;
  static constexpr bool kZUInterleaved = (D == 2) && MMX_ZU_INTER;  // = kZUInter<D> (admm_kernels.hip)
  double* uPtr() const { return kZUInterleaved ? z_.p + D : u_.p; }
  void clearU() {  // u = 0 (2D: the whole interleaved buffer, z included)
    if (kZUInterleaved)
      MMX_HIP(hipMemsetAsync(z_.p, 0, z_.n * sizeof(double), st_));
    else
      MMX_HIP(hipMemsetAsync(u_.p, 0, u_.n * sizeof(double), st_));
  }
  bool spinWait_ = true;         // MMX_SPIN (waitStream)
  static constexpr int kTslot2dMax = 2 * 2048 * 64;  // 2D slot terms up to two rounds of resident prox waves
  double* res_ = nullptr;        // the reductions' results: results_.p, or the device view of resH_
  double* resH_ = nullptr;       // pinned, mapped results (one rank)
  hipEvent_t evSync_ = nullptr;
  std::vector<Timed> timed_;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> stepEv_;
  static constexpr size_t kEvResolve = 4096;  // events outstanding before a resolution
  mmadmm_stats st_stats_{};
};

}  // namespace mmx

using mmx::EngineBase;
using mmx::Error;
using mmx::guarded;

struct mmadmm_engine {
  std::unique_ptr<EngineBase> e;
};

static EngineBase& eng(mmadmm_handle h) {
  if (!h || !h->e) throw Error(MMADMM_ERR_INVALID, "null engine handle");
  return *h->e;
}

extern "C" {

const char* mmadmm_last_error(void) { return mmx::g_last_error.c_str(); }
int mmadmm_version(void) { return 100; }

int mmadmm_mesh_reorient(int dim, int nP, const double* Xp, int nF, int32_t* F) {
  return guarded([&] {
    if ((dim != 2 && dim != 3) || nP < 1 || nF < 0 || !Xp || (nF > 0 && !F))
      throw Error(MMADMM_ERR_INVALID, "mmadmm_mesh_reorient: bad arguments");
    for (long long i = 0; i < (long long)nF * (dim + 1); ++i)
      if (F[i] < 0 || F[i] >= nP) throw Error(MMADMM_ERR_INVALID, "simplex vertex id out of range");
    mmx::reorient_simplices(dim, Xp, nF, F);
  });
}

int mmadmm_create(int dim, int nP, const double* Xp, const double* Xc, int nF, const int32_t* F, const int32_t* mask,
                  const mmadmm_params* p, mmadmm_monitor_fn fn, void* user, mmadmm_handle* out) {
  return guarded([&] {
    if (!out) throw Error(MMADMM_ERR_INVALID, "mmadmm_create: out is NULL");
    *out = nullptr;
    if ((dim != 2 && dim != 3) || nP < dim + 1 || nF < 1 || !Xp || !F || !mask || !p || !fn)
      throw Error(MMADMM_ERR_INVALID, "mmadmm_create: bad arguments");
    if (!(p->dt > 0) || !(p->tau > 0) || !(p->rho > 0))
      throw Error(MMADMM_ERR_INVALID, "mmadmm_create: dt, tau, rho must be positive");
    if (p->nranks > 1) throw Error(MMADMM_ERR_INVALID, "mmadmm_create: use mmadmm_create_partitioned for nranks > 1");
    mmx::check_kernel_layout(mmx::kLayoutWord);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
      throw Error(MMADMM_ERR_HIP, "mmadmm_create: no HIP device (the engine has no CPU fallback)");
    auto* h = new mmadmm_engine();
    try {
      if (dim == 2)
        h->e.reset(new mmx::Engine<2>(nP, Xp, Xc, nF, F, mask, *p, fn, user, nullptr));
      else
        h->e.reset(new mmx::Engine<3>(nP, Xp, Xc, nF, F, mask, *p, fn, user, nullptr));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int mmadmm_create_partitioned(int dim, int nP, const double* Xp, const double* Xc, int nF, const int32_t* F,
                              const int32_t* mask, const mmadmm_params* p, mmadmm_monitor_fn fn, void* user,
                              mmadmm_comm comm, mmadmm_handle* out) {
  return guarded([&] {
    if (!out) throw Error(MMADMM_ERR_INVALID, "mmadmm_create_partitioned: out is NULL");
    *out = nullptr;
    if ((dim != 2 && dim != 3) || nP < dim + 1 || nF < 1 || !Xp || !F || !mask || !p || !fn)
      throw Error(MMADMM_ERR_INVALID, "mmadmm_create_partitioned: bad arguments");
    if (!(p->dt > 0) || !(p->tau > 0) || !(p->rho > 0))
      throw Error(MMADMM_ERR_INVALID, "mmadmm_create_partitioned: dt, tau, rho must be positive");
    if (p->nranks < 1 || p->rank < 0 || p->rank >= p->nranks)
      throw Error(MMADMM_ERR_INVALID, "mmadmm_create_partitioned: bad rank / nranks");
    mmx::Comm* c = mmx::comm_of(comm);
    if (p->nranks > 1 && (!c || c->nranks != p->nranks))
      throw Error(MMADMM_ERR_INVALID, "mmadmm_create_partitioned: communicator missing or of another size");
    mmx::check_kernel_layout(mmx::kLayoutWord);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
      throw Error(MMADMM_ERR_HIP, "mmadmm_create_partitioned: no HIP device (the engine has no CPU fallback)");
    auto* h = new mmadmm_engine();
    try {
      if (dim == 2)
        h->e.reset(new mmx::Engine<2>(nP, Xp, Xc, nF, F, mask, *p, fn, user, c));
      else
        h->e.reset(new mmx::Engine<3>(nP, Xp, Xc, nF, F, mask, *p, fn, user, c));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int mmadmm_local_nodes(mmadmm_handle h, int* n_local, int32_t* global_ids) {
  return guarded([&] { eng(h).localNodes(n_local, global_ids); });
}

int mmadmm_step(mmadmm_handle h, int n_iters, double tol, double* Ih, int* admm_iters) {
  return guarded([&] { eng(h).step(n_iters, tol, Ih, admm_iters); });
}
int mmadmm_euler_step(mmadmm_handle h, double* Ih) {
  return guarded([&] {
    const double r = eng(h).eulerStep();
    if (Ih) *Ih = r;
  });
}
int mmadmm_backward_euler_step(mmadmm_handle h, double dt, double tol, double* Ih, int* newton_iters) {
  return guarded([&] {
    if (!(dt > 0)) throw mmx::Error(MMADMM_ERR_INVALID, "backward Euler: dt must be > 0");
    const double r = eng(h).backwardEulerStep(dt, tol, newton_iters);
    if (Ih) *Ih = r;
  });
}
int mmadmm_be_begin(mmadmm_handle h, double dt, double* Ih) {
  return guarded([&] {
    if (!(dt > 0)) throw mmx::Error(MMADMM_ERR_INVALID, "backward Euler: dt must be > 0");
    double sc[2] = {0.0, 0.0};
    eng(h).newtonOp(0, dt, nullptr, nullptr, sc);
    if (Ih) *Ih = sc[0];
  });
}
int mmadmm_be_residual(mmadmm_handle h, double dt, double* F, double* norm1, double* Ih) {
  return guarded([&] {
    if (!F) throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_be_residual: F is NULL");
    double sc[2] = {0.0, 0.0};
    eng(h).newtonOp(1, dt, nullptr, F, sc);
    if (Ih) *Ih = sc[0];
    if (norm1) *norm1 = sc[1];
  });
}
int mmadmm_be_fsubjac(mmadmm_handle h, double* a) {
  return guarded([&] {
    if (!a) throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_be_fsubjac: a is NULL");
    eng(h).newtonOp(2, 0.0, nullptr, a, nullptr);
  });
}
int mmadmm_be_add(mmadmm_handle h, const double* dx) {
  return guarded([&] {
    if (!dx) throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_be_add: dx is NULL");
    eng(h).newtonOp(3, 0.0, dx, nullptr, nullptr);
  });
}
int mmadmm_get_jacobian(mmadmm_handle h, long long* nnz, int32_t* ia, int32_t* ja, double* a) {
  return guarded([&] { eng(h).jacobian(nnz, ia, ja, a); });
}
int mmadmm_energy(mmadmm_handle h, double* E) {
  return guarded([&] {
    const double r = eng(h).energy();
    if (E) *E = r;
  });
}
int mmadmm_done(mmadmm_handle h) {
  return guarded([&] { eng(h).done(); });
}
int mmadmm_get(mmadmm_handle h, const char* what, double* out) {
  return guarded([&] {
    if (!what || !out) throw Error(MMADMM_ERR_INVALID, "mmadmm_get: NULL argument");
    eng(h).get(what, out);
  });
}
int mmadmm_get_simplices(mmadmm_handle h, int32_t* F) {
  return guarded([&] { eng(h).getSimplices(F); });
}
int mmadmm_sizes(mmadmm_handle h, int* nP, int* nF, int* grid_rows) {
  return guarded([&] { eng(h).sizes(nP, nF, grid_rows); });
}
int mmadmm_set_timing(mmadmm_handle h, int on) {
  return guarded([&] { eng(h).setTiming(on != 0); });
}
int mmadmm_stats_get(mmadmm_handle h, mmadmm_stats* s) {
  return guarded([&] {
    if (!s) throw Error(MMADMM_ERR_INVALID, "NULL stats");
    eng(h).stats(s);
  });
}
int mmadmm_stats_reset(mmadmm_handle h) {
  return guarded([&] { eng(h).resetStats(); });
}
int mmadmm_regrid(mmadmm_handle h, double t) {
  return guarded([&] { eng(h).regrid(t); });
}
int mmadmm_set_regrid(mmadmm_handle h, int every_step) {
  return guarded([&] { eng(h).setRegrid(every_step != 0); });
}
int mmadmm_sync(mmadmm_handle h) {
  return guarded([&] { eng(h).sync(); });
}
int mmadmm_debug_blockgrad(mmadmm_handle h, int s, const double* z, const double* dxpu, int flags, double* out) {
  return guarded([&] {
    if (!z || !dxpu || !out) throw Error(MMADMM_ERR_INVALID, "mmadmm_debug_blockgrad: NULL argument");
    eng(h).debugBlockGrad(s, z, dxpu, flags, out);
  });
}
int mmadmm_destroy(mmadmm_handle h) {
  return guarded([&] { delete h; });
}

int mmadmm_devmath(int op, int n, const double* in, double* out) {
  return guarded([&] {
    if (n < 0 || (n && (!in || !out))) throw Error(MMADMM_ERR_INVALID, "mmadmm_devmath: bad arguments");
    mmx::DevBuf<double> a, b;
    a.upload(in, n, nullptr);
    b.alloc(n);
    mmx::launch_devmath(op, n, a.p, b.p, nullptr);
    MMX_HIP(hipMemcpy(out, b.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
  });
}

}  // extern "C"
