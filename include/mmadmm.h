/*
 * mmadmm.h -- C-ABI of the MI355X-native MM-ADMM engine (libmmadmm.so).
 *
 * Drop-in boundary for the hot path of connortannahill/MM-ADMM: the ADMM time step of the
 * MMPDE integrator (MeshIntegrator<D>::step and what it calls).  Plain pointers and sizes
 * only; every call returns MMADMM_OK (0) or an error code, and mmadmm_last_error() gives
 * the message.  No C++ exception crosses this boundary.  All arrays are caller-owned and
 * copied in or out.  The C++ mirror of the reference classes (Mesh<D>, MeshIntegrator<D>,
 * MonitorFunction<D>) lives in include/mmadmm/ and is implemented on top of this ABI.
 *
 * Reference interface each entry point replaces (paths relative to the reference repo):
 *   mmadmm_create            Mesh<D>::Mesh (src/Mesh.h:22-25, src/Mesh.cpp:384-494)
 *                            + MeshIntegrator<D>::MeshIntegrator (src/MeshIntegrator.h:15,
 *                              src/MeshIntegrator.cpp:15-62)
 *   mmadmm_step              MeshIntegrator<D>::step (src/MeshIntegrator.h:17, .cpp:101-191)
 *   mmadmm_euler_step        MeshIntegrator<D>::eulerStep (src/MeshIntegrator.h:18, .cpp:87-94)
 *   mmadmm_backward_euler_step MeshIntegrator<D>::backwardsEulerStep (src/MeshIntegrator.h:19,
 *                            .cpp:68-76) -> Mesh<D>::backwardsEulerStep (src/Mesh.cpp:1263-1341)
 *   mmadmm_get_jacobian      Mesh<D>::jac after buildEulerJac (src/Mesh.cpp:1112-1136)
 *   mmadmm_be_begin / _residual / _fsubjac / _add
 *                            the pieces of Mesh<D>::backwardsEulerStep (src/Mesh.cpp:1266-1273,
 *                            1289-1294, 1112-1124 + 1232-1258, 1329), so a host loop can drive
 *                            the Newton iteration through the LASolver classes (MatrixIter.h)
 *   mmadmm_energy            MeshIntegrator<D>::getEnergy (src/MeshIntegrator.h:20, .cpp:79-81)
 *   mmadmm_done              MeshIntegrator<D>::done (src/MeshIntegrator.h:23, .cpp:193-196)
 *   mmadmm_get("x"|"z")      MeshIntegrator<D>::outputX / outputZ (src/MeshIntegrator.h:21-22)
 *   mmadmm_get("points")     Mesh<D>::outputPoints (src/Mesh.h:29, src/Mesh.cpp:1082-1095)
 *   mmadmm_get_simplices     Mesh<D>::outputSimplices (src/Mesh.h:27, src/Mesh.cpp:1067-1080)
 *   mmadmm_monitor_fn        MonitorFunction<D>::operator() (src/MonitorFunction.h:13),
 *                            evaluated on the host at set-up only, as the reference does
 *                            (src/MonitorFunction.cpp:16-32 via src/MeshInterpolator.cpp:254)
 *   mmadmm_builtin_monitor   Experiments/TestMonitors/MEx*.h registry (main.cpp:836-864)
 *   mmadmm_mesh_*            utils::generateUniformRectMesh / meshFromLevelSetFun /
 *                            readTriangles (src/MeshUtils.h:82-335, 404-538, 669-733)
 */
#ifndef MMADMM_H
#define MMADMM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMADMM_OK 0
#define MMADMM_ERR_INVALID 1  /* bad argument / state */
#define MMADMM_ERR_HIP 2      /* HIP runtime failure or no GPU */
#define MMADMM_ERR_INVERTED 3 /* inverted element: the reference's assert(Edet > 0) */
#define MMADMM_ERR_IO 4       /* file not readable / writable */
#define MMADMM_ERR_RCCL 5     /* collective failure */
#define MMADMM_ERR_NOCONV 6   /* linear solve did not converge: the reference's assert(cgIter > 0) */
#define MMADMM_ERR_NONFINITE 7 /* non-finite energy with no inverted element: a monitor value that is not
                                  finite (element partition + time-varying monitor: an evaluation outside
                                  the rank's rebuilt grid box) */

/* Node types (src/NodeType.h:4-8); mask arrays use these values. */
#define MMADMM_BOUNDARY_FREE 0
#define MMADMM_BOUNDARY_FIXED 1
#define MMADMM_INTERIOR 2

typedef struct mmadmm_engine* mmadmm_handle;
typedef struct mmadmm_meshbuf* mmadmm_mesh;

/* Monitor tensor M(x) (D x D, row-major), called on the host at set-up. */
typedef void (*mmadmm_monitor_fn)(int dim, const double* x, double* M_rowmajor, void* user);

typedef struct mmadmm_params {
  double dt;      /* time step (MeshIntegrator ctor dt) */
  double tau;     /* mass-matrix weight (Mesh ctor tau) */
  double rho;     /* ADMM penalty; w = 0.5*sqrt(rho) as in src/Mesh.cpp:451 */
  int grad_use;   /* GradUse: predictor always uses the energy gradient */
  int device;     /* HIP device ordinal, -1 = current device */
  int rank;       /* element-partitioned run: this rank (0 for single GPU) */
  int nranks;     /* number of ranks (1 for single GPU) */
  int partition;  /* element partition: MMADMM_PART_RCB (0, default) or MMADMM_PART_RANGES */
} mmadmm_params;

typedef struct mmadmm_stats {
  long long steps;        /* time steps taken */
  long long admm_iters;   /* ADMM iterations executed */
  long long bfgs_iters;   /* BFGS iterations summed over simplices */
  int max_bfgs;           /* largest per-simplex BFGS count in the last prox */
  double last_primal;     /* ||D x - z|| of the last ADMM iteration */
  double last_dual;       /* ||z - zPrev|| of the last ADMM iteration */
  double t_prox_ms;       /* device time in the prox kernel (timing on) */
  double t_xupdate_ms;    /* device time in the x-update kernel (timing on) */
  double t_step_ms;       /* device time of whole steps (timing on) */
  long long n_prox;       /* prox launches timed */
  long long n_xupdate;    /* x-update launches timed */
  long long n_steps_timed;
  double prox_bytes;      /* algorithmic HBM bytes of one prox launch */
  double xupdate_bytes;   /* algorithmic HBM bytes of one x-update launch */
  long long newton_iters; /* backward Euler: Newton iterations summed over steps */
  long long jacobians;    /* backward Euler: FD Jacobian builds */
  long long cg_iters;     /* backward Euler: CG-STAB iterations summed over Newton iterations */
  double t_jac_ms;        /* backward Euler: wall time in Jacobian builds (FD + assembly) */
  double t_solve_ms;      /* backward Euler: wall time in the linear solves (ILU(0) + CG-STAB) */
  double t_be_ms;         /* backward Euler: wall time of whole steps */
  long long regrids;      /* monitor-grid rebuilds on the device (mmadmm_regrid / set_regrid) */
  long long regrid_rows;  /* grid rows the last rebuild filled (an element partition: this rank's box) */
  double regrid_gather_bytes; /* bytes this rank received for the last rebuild (element partition) */
  long long regrid_cand;       /* element partition: candidate vertices of the last rebuild's nearest-
                                  vertex fill (this rank's + those received from its neighbours) */
  long long regrid_fallbacks;  /* element partition: rebuilds that fell back to all-gathering every vertex */
  int monitor_iso;             /* 1: the monitor grid is isotropic (every point a multiple of the identity,
                                  bit for bit) and kept as one value per point; MMX_ISO=0 disables it */
  /* element partition (round 6): the halo exchange of an ADMM iteration (pack + send/recv, device
   * time on its stream, timing on), the bytes this rank sends / receives per exchange, and the
   * nodes whose x-update runs while the exchange is in flight (no slot of another rank) */
  double t_exchange_ms;
  long long n_exchange;
  double halo_send_bytes;
  double halo_recv_bytes;
  int interior_nodes;
  int overlap;                 /* 1: the interior x-update overlaps the exchange (MMX_OVERLAP=0: serial) */
} mmadmm_stats;

/* Time-varying monitors (the reference's Mesh<D>::setUp hook, commented out at
 * src/Mesh.cpp:1006-1014, would re-run MeshInterpolator::updateMesh + interpolateMonitor,
 * src/MeshInterpolator.cpp:68-130, 166-259, 366-404, at every step start).
 * mmadmm_regrid rebuilds the smoothed monitor grid on the device from the current mesh positions,
 * the monitor evaluated at time t (built-in MonType 7 on the device; any other monitor through its
 * host callback at the current vertices); bit-identical to the host set-up.  mmadmm_set_regrid(h, 1)
 * does that at the start of every mmadmm_step with t = steps taken * dt.  On an element partition
 * every rank all-gathers the positions of the vertices it owns and rebuilds the same global grid. */
int mmadmm_regrid(mmadmm_handle h, double t);
int mmadmm_set_regrid(mmadmm_handle h, int every_step);

const char* mmadmm_last_error(void);
int mmadmm_version(void);
/* provenance (no reference counterpart): "src_hash=<16 hex> git=<describe> arch=gfx950", the hash of
 * the library's sources as mm-admm_amd/tools/src_hash.py computes it at build time */
int mmadmm_build_info(char* out, int len);

/* built-in monitors MEx0..MEx5 (dim 2) and MEx0/13D/23D/33D/0/53D (dim 3) by MonType 0..5, MonType 7 a
 * time-varying bump M = (1 + 5 / (1 + 50 |x - c(t)|^2)) I, c(t) = (0.5 + 0.2 cos 2 pi t, 0.5 + 0.2 sin 2 pi t,
 * 0.5) (used with mmadmm_set_regrid; set-up evaluates it at t = 0)
 * (main.cpp:836-864), plus MonType 6: an anisotropic shell monitor M = lam2 I + (lam1 - lam2) n n^T (radial n,
 * lam1 = 1 + sech(50 (|x - c| - 0.3)^2), 1/lam1 across n; MEx2.h's construction around a
 * sphere) with no reference counterpart (BASELINE config 4) */
int mmadmm_builtin_monitor(int dim, int mon_type, mmadmm_monitor_fn* fn, void** user);
/* The smoothed monitor grid the set-up builds from the positions Xp (nP x dim) and the monitor
 * (MeshInterpolator<D>::updateMesh + interpolateMonitor, src/MeshInterpolator.cpp:68-130, 166-259,
 * 366-404): host only, no device needed.  *rows = grid rows; vals (rows x dim*dim, row-major
 * tensors) is filled unless NULL. */
int mmadmm_monitor_grid(int dim, int nP, const double* Xp, mmadmm_monitor_fn fn, void* user, int* rows,
                        double* vals);

/* Mesh::reOrientElements (src/Mesh.cpp:243-260) alone, in place on F (host only): the ordering
 * mmadmm_create applies and mmadmm_get_simplices returns. */
int mmadmm_mesh_reorient(int dim, int nP, const double* Xp, int nF, int32_t* F);

/* Mesh<D> + MeshIntegrator<D>.  Xp: nP x dim row-major; Xc: reference positions (CompMesh)
 * or NULL; F: nF x (dim+1); mask: nP node types.  F is re-oriented (src/Mesh.cpp:243-260)
 * and can be read back with mmadmm_get_simplices. */
int mmadmm_create(int dim, int nP, const double* Xp, const double* Xc, int nF, const int32_t* F,
                  const int32_t* mask, const mmadmm_params* p, mmadmm_monitor_fn fn, void* user,
                  mmadmm_handle* out);
/* One ADMM time step.  tol >= 0: the reference's early exit (primal < tol && dual < tol);
 * tol < 0: exactly n_iters ADMM iterations (prox tolerance 1e-3 as main.cpp:184).
 * *Ih = energy at the first prox of the step (the reference's return value). */
int mmadmm_step(mmadmm_handle h, int n_iters, double tol, double* Ih, int* admm_iters);
int mmadmm_euler_step(mmadmm_handle h, double* Ih);
/* method 2: one backward Euler step (Newton + ILU(0) CG-STAB); single rank only */
int mmadmm_backward_euler_step(mmadmm_handle h, double dt, double tol, double* Ih, int* newton_iters);
/* the last assembled backward-Euler Jacobian (CSR over D*nP unknowns; mmadmm_be_fsubjac does not
 * replace it); null arrays are skipped */
int mmadmm_get_jacobian(mmadmm_handle h, long long* nnz, int32_t* ia, int32_t* ja, double* a);
/* backward Euler in pieces (single rank): xn = x, Ih = eulerStepMod(x), x -= (dt/tau) grad */
int mmadmm_be_begin(mmadmm_handle h, double dt, double* Ih);
/* F = (dt/tau) grad(x) + (x - xn) (D*nP doubles to the host), ||F||_1 and Ih = sum of energies */
int mmadmm_be_residual(mmadmm_handle h, double dt, double* F, double* norm1, double* Ih);
/* the FSubJac sums at the mesh positions on the buildMatrix CSR pattern (mmadmm_get_jacobian's ia,
 * ja), before buildEulerJac's a *= dt/tau and the +1 on the diagonal */
int mmadmm_be_fsubjac(mmadmm_handle h, double* a);
/* x += dx (D*nP doubles) */
int mmadmm_be_add(mmadmm_handle h, const double* dx);
int mmadmm_energy(mmadmm_handle h, double* E);
int mmadmm_done(mmadmm_handle h);
/* what: "x", "xPrev", "xBar", "z", "u", "points", "hess", "grid", "Ehat" */
int mmadmm_get(mmadmm_handle h, const char* what, double* out);
int mmadmm_get_simplices(mmadmm_handle h, int32_t* F);
int mmadmm_sizes(mmadmm_handle h, int* nP, int* nF, int* grid_rows);
int mmadmm_set_timing(mmadmm_handle h, int on);
int mmadmm_stats_get(mmadmm_handle h, mmadmm_stats* s);
int mmadmm_stats_reset(mmadmm_handle h);
int mmadmm_sync(mmadmm_handle h);
int mmadmm_destroy(mmadmm_handle h);

/* meshes: generators and readers (host) */
int mmadmm_mesh_rect(int dim, int nx, int ny, int nz, double xa, double xb, double ya, double yb,
                     double za, double zb, int btype, mmadmm_mesh* out);
/* compact_mask = 0 keeps the reference's pre-compaction mask indexing (MeshUtils.h:487) */
int mmadmm_mesh_levelset2d(int nx, int ny, double xa, double xb, double ya, double yb, int btype,
                           int compact_mask, mmadmm_mesh* out);
/* utils::meshFromLevelSetFun 3D with spherePhi (src/MeshUtils.h:540-667, main.cpp:87-97): the cube
 * cut to the tetrahedra with a vertex inside the sphere r = 0.4 centred (0.5, 0.5, 0.5), outside
 * vertices moved by interpolateBoundaryLocation 3D (388-402), nodes numbered as the reference's
 * pntMap (descending original id).  The reference never hands its result back (663-666 reassign
 * pointer copies); here it is returned.  compact_mask = 0: the reference's pre-compaction mask
 * indexing (595-597); 1: the mask remapped to the new numbering. */
int mmadmm_mesh_levelset3d(int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za,
                           double zb, int btype, int compact_mask, mmadmm_mesh* out);
/* hexagonal disc of radius r centred (cx, cy): 3N(N+1)+1 nodes, 6N^2 triangles, rim FIXED */
/* setUpShoulderExperiment (main.cpp:403-630): rect mesh minus the upper (x, y[, z]) quadrant's
 * simplices, re-marked boundary, interior vertices moved by up to h/10 in a random direction drawn with
 * glibc rand() (seed it as main.cpp:785 does: srand(69)) and Eigen 3.4 Random() semantics (Eigen is
 * un-vendored in the reference: version unpinned).  The unmoved positions (the CompMesh reference
 * Vc) come from mmadmm_mesh_reference_points. */
int mmadmm_mesh_shoulder(int dim, int nx, int ny, int nz, double xa, double xb, double ya, double yb, double za,
                         double zb, int btype, mmadmm_mesh* out);
/* Vc of a mesh (the unmoved positions of a Shoulder mesh; Vp for the other generators) */
int mmadmm_mesh_reference_points(mmadmm_mesh h, double* Xc);
int mmadmm_mesh_hexdisc(int N, double r, double cx, double cy, int btype, mmadmm_mesh* out);
int mmadmm_mesh_read(int dim, const char* tri, const char* pnts, const char* mask, mmadmm_mesh* out);
int mmadmm_mesh_sizes(mmadmm_mesh m, int* dim, int* nP, int* nF, int* mask_len);
int mmadmm_mesh_copy(mmadmm_mesh m, double* Xp, int32_t* F, int32_t* mask);
int mmadmm_mesh_free(mmadmm_mesh m);
/* writers byte-compatible with Mesh::outputPoints / outputSimplices (default ostream) */
int mmadmm_write_points(const char* path, int dim, int nP, const double* Xp);
int mmadmm_write_simplices(const char* path, int dim, int nF, const int32_t* F);

/* one-simplex Mesh::computeBlockGrad on the device (tests): flags bit0 = gradient,
 * bit1 = regularise with dxpu; out = {energy, Igt, grad[D(D+1)]} */
int mmadmm_debug_blockgrad(mmadmm_handle h, int s, const double* z, const double* dxpu, int flags,
                           double* out);

/* ---- element partition across ranks (one process per GPU)
 * Every simplex has one owner rank -- MMADMM_PART_RCB: recursive coordinate bisection of the
 * simplex centroids (compact parts, short interfaces); MMADMM_PART_RANGES: contiguous ranges
 * [r*nF/nranks, (r+1)*nF/nranks) of global ids -- and a rank holds the nodes its simplices touch;
 * interface nodes are replicated.  Their x-update / predictor sums take the other ranks' slot
 * values from a halo exchange with the neighbouring ranks only (RCCL send/recv), summed in
 * ascending global simplex order: node positions are bit-identical to a single-GPU run.  At most
 * 64 ranks.  No reference counterpart (the reference is single-process OpenMP). */
#define MMADMM_PART_RCB 0
#define MMADMM_PART_RANGES 1
#define MMADMM_UNIQUE_ID_BYTES 128
typedef struct mmadmm_comm_s* mmadmm_comm;
typedef struct mmadmm_plan_s* mmadmm_plan;
/* The layout word of the host code (kernels/layout.h: every compile-time switch that changes a buffer
 * shared by host and kernels) into *host_word; MMADMM_ERR_INVALID when a kernel object of this
 * library was built with another (mmadmm_create*, mmx_matrix_create* check the same, first). */
int mmadmm_layout_check(unsigned* host_word);
/* RCCL: rank 0 makes the id, every rank creates its communicator with it (collective) */
int mmadmm_comm_unique_id(void* out, int len);
int mmadmm_comm_create_rccl(int nranks, int rank, const void* uid, int device, mmadmm_comm* out);
/* the same with an explicit deadline (seconds; <= 0: none).  The communicator is non-blocking: its
 * creation, every RCCL call that reports ncclInProgress and every stream wait of a partitioned
 * step are bounded by the deadline, after which the communicator is aborted (ncclCommAbort) and the
 * call returns MMADMM_ERR_RCCL naming the rank and the call -- a missing or stuck peer ends the run,
 * never hangs it.  mmadmm_comm_create_rccl takes MMX_COMM_TIMEOUT_S from the environment (default
 * 300 s). */
int mmadmm_comm_create_rccl_timeout(int nranks, int rank, const void* uid, int device, double timeout_s,
                                    mmadmm_comm* out);
/* one communicator shared by nranks engines driven from threads of one process (tests) */
int mmadmm_comm_create_loopback(int nranks, mmadmm_comm* out);
/* transfers done by the caller's host transport (one process per rank, e.g. torch.distributed over
 * gloo or MPI): the engine stages device blocks through pinned host buffers and calls these, in the
 * same order on every rank; each returns 0 on success.
 *   allgather: recv[q*count .. (q+1)*count) = rank q's send block (count doubles)
 *   exchange: for each of npeers peers, send send[send_off[i] .. + send_count[i]) to rank
 *             peer_rank[i] and receive recv_count[i] doubles from it into recv + recv_off[i]
 *             (called on every halo exchange, also with npeers = 0) */
typedef int (*mmadmm_allgather_fn)(void* user, const double* send, double* recv, long long count);
typedef int (*mmadmm_exchange_fn)(void* user, int npeers, const int* peer_rank, const double* send,
                                  const long long* send_off, const long long* send_count, double* recv,
                                  const long long* recv_off, const long long* recv_count);
int mmadmm_comm_create_host(int nranks, int rank, mmadmm_allgather_fn allgather, mmadmm_exchange_fn exchange,
                            void* user, mmadmm_comm* out);
int mmadmm_comm_destroy(mmadmm_comm c);
/* ranks of the communicator: for RCCL what ncclCommCount reports, else the count it was made with */
int mmadmm_comm_nranks(mmadmm_comm c, int* nranks);
/* like mmadmm_create, given the GLOBAL mesh on every rank; p->rank / p->nranks select the
 * share.  mmadmm_get / mmadmm_get_simplices then return this rank's nodes / simplices (in
 * global ids); mmadmm_local_nodes lists the global ids of the local nodes. */
int mmadmm_create_partitioned(int dim, int nP, const double* Xp, const double* Xc, int nF, const int32_t* F,
                              const int32_t* mask, const mmadmm_params* p, mmadmm_monitor_fn fn, void* user,
                              mmadmm_comm comm, mmadmm_handle* out);
int mmadmm_local_nodes(mmadmm_handle h, int* n_local, int32_t* global_ids);
/* the partition plan alone (host only).  Xp (nP x dim) is needed by MMADMM_PART_RCB.  Sizes: local
 * nodes and simplices, incident-slot sources, rows sent / received, neighbour ranks, interface nodes
 * (local nodes another rank also touches).  Arrays: local node and simplex global ids (ascending),
 * per-node slot sources (incPtr/incSrc: >= 0 local slot offset s*K+n*D, < 0 row -1-src of the
 * receive buffer), the local slot offsets sent (per peer, peers ascending), and per peer
 * {rank, rows sent, rows received} (the receive buffer holds the peers' rows in that order). */
int mmadmm_plan_create(int dim, int nP, const double* Xp, int nF, const int32_t* F, int nranks, int rank, int method,
                       mmadmm_plan* out);
int mmadmm_plan_sizes(mmadmm_plan h, int* nLocalNodes, int* nLocalSimplices, int* nSources, int* nSend, int* nRecv,
                      int* nPeers, int* nInterface);
int mmadmm_plan_get(mmadmm_plan h, int32_t* localNodes, int32_t* localSimplices, int32_t* incPtr, int32_t* incSrc,
                    int32_t* sendOff, int32_t* peers);
int mmadmm_plan_destroy(mmadmm_plan h);

/* device math self-test (correctly rounded powers): op 0 sqrt, 1 x^1.5, 2 x^-0.5, 3 x^2.25,
 * 4 x^1.25; op 5: in = pairs (x, c), out[i] = x_i / c_i by reciprocal + FMA correction;
 * ops 6-9: the prox fast path of ops 1-4 (NaN where it defers to the exact path); op 10: the
 * double-double sqrt of in[i] as out[2i] + out[2i+1], i < n/2 */
int mmadmm_devmath(int op, int n, const double* in, double* out);

#ifdef __cplusplus
}
#endif
#endif
