/* mmx_sparse.h -- C-ABI of the MI355X LASolver replacement (ILU-preconditioned CG-STAB on the GPU).
 *
 * Drop-in for the reference's lib/LASolver as used by backward Euler.  Each
 * entry point names the reference interface it replaces:
 *
 *   mmx_param_iter                 ParamIter                       lib/LASolver/MatrixIter.h:113-175
 *   mmx_param_iter_default         ParamIter::ParamIter()          lib/LASolver/MatrixIter.h:155-168
 *   mmx_param_iter_mesh            buildMatrix's settings          src/Mesh.cpp:264-304
 *   mmx_struc_create               MatrixStruc(n, no_diag)         lib/LASolver/MatrixIter.cpp:88-116
 *   mmx_struc_set_entry(_entries)  MatrixStruc::set_entry          lib/LASolver/MatrixIter.cpp:125-142
 *   mmx_struc_mesh_pattern         buildMatrix's set_entry loop    src/Mesh.cpp:309-341
 *   mmx_struc_pack                 MatrixStruc::pack               lib/LASolver/MatrixIter.cpp:179-257, 895-991
 *   mmx_struc_get                  getia / getja / getnja          lib/LASolver/MatrixIter.cpp:144-177
 *   mmx_matrix_create              MatrixIter(n, ia, ja)           lib/LASolver/MatrixIter.cpp:344-427
 *   mmx_matrix_create_from_struc   MatrixIter(MatrixStruc&)        lib/LASolver/MatrixIter.cpp:320-342
 *   mmx_matrix_set_values(_device) aValue(k) = ... for every k     lib/LASolver/MatrixIter.h:311-312
 *   mmx_matrix_set_rhs(_device)    bValue(i) = ... for every i     lib/LASolver/MatrixIter.h:308-309
 *   mmx_matrix_set_toler           set_toler                       lib/LASolver/MatrixIter.cpp:443-453
 *   mmx_matrix_sfac                sfac (symbolic ILU)             lib/LASolver/MatrixIter.cpp:455-489
 *   mmx_matrix_solve(_device)      solve                           lib/LASolver/MatrixIter.cpp:635-819
 *   mmx_matrix_matmult(_device)    matmult                         lib/LASolver/accel_class.cpp:521-549
 *   mmx_matrix_factor              scaler_ILU::factor              lib/LASolver/ILU_class.cpp:300-444
 *   mmx_matrix_ilu_solve(_device)  scaler_ILU::solve               lib/LASolver/ILU_class.cpp:447-527
 *   mmx_matrix_get_factor          rowsp[i].af (read back)         lib/LASolver/ILU_class.h:24-90
 *   mmx_ilu_symbolic               scaler_ILU::sfac2 / merge2      lib/LASolver/ILU_class.cpp:17-295
 *
 * Supported ParamIter settings: natural order (order 0), level-of-fill ILU (drop_ilu 0) at any
 * level, no scaling (iscal 0), no pivoting, CG-STAB acceleration (iaccel 0), either rhat.  Other
 * settings return MMADMM_ERR_INVALID with a message (the reference's only caller uses exactly
 * order 0, level 0, iscal 0, iaccel 0; src/Mesh.cpp:264-304).
 *
 * Conventions: every function returns a status code of mmadmm.h (0 = ok; message via
 * mmadmm_last_error()); no exception crosses the ABI.  Host arrays are caller-owned and copied;
 * *_device variants take pointers into device memory of the matrix's device and run on its
 * stream (mmx_matrix_stream).  Non-convergence is nitr = -1, as in the reference.
 */
#ifndef MMX_SPARSE_H
#define MMX_SPARSE_H

#include <stdint.h>

#include "mmadmm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mmx_param_iter {
  int order;          /* 0 natural (1 RCM: not supported) */
  int level;          /* level of fill of the ILU */
  int drop_ilu;       /* 0 level-of-fill ILU (1 drop tolerance: not supported) */
  int ipiv;           /* 0 no pivoting */
  int iscal;          /* 0 no scaling (1: not supported) */
  int nitmax;         /* maximum iterations */
  double resid_reduc; /* convergence when ||r|| / ||r0|| < resid_reduc */
  int info;           /* ignored (the reference's output is commented out) */
  double drop_tol;    /* ignored (drop_ilu 0) */
  int new_rhat;       /* 0: rhat = r0; 1: rhat = (LU)^-1 r0 */
  int iaccel;         /* 0 CG-STAB (1 orthomin, -1 CG: not supported) */
  int north;          /* ignored (orthomin only) */
} mmx_param_iter;

typedef struct mmx_struc_s* mmx_struc;
typedef struct mmx_matrix_s* mmx_matrix;

typedef struct mmx_sparse_stats {
  long long solves, iterations, spmvs, sweeps, factors;
  double t_spmv_ms, t_sweep_ms, t_factor_ms, t_vec_ms, t_solve_ms; /* with timing on */
  long long n_spmv_timed, n_sweep_timed, n_factor_timed;
  double spmv_bytes;  /* algorithmic bytes of one SpMV: 12 nnz + 4 (n+1) + 16 n */
  double last_rms, rmsi;
  int sweep_mode;     /* triangular sweeps: 0 level-scheduled, 1 chain/band-scheduled */
  int sweep_e;        /* chain sweeps: entry slots per row of the forward stages (8, 16, 32, 48) */
  int factor_mode;    /* numeric factor: 0 level-scheduled (a row per lane), 1 chain/band-scheduled,
                        2 level order with a wavefront per row */
  int sweep_e_bwd;    /* the same for the backward stages */
} mmx_sparse_stats;

void mmx_param_iter_default(mmx_param_iter* p);
void mmx_param_iter_mesh(mmx_param_iter* p);

int mmx_struc_create(int n, int no_diag, mmx_struc* out);
int mmx_struc_set_entry(mmx_struc s, int row, int col);
int mmx_struc_set_entries(mmx_struc s, long long count, const int32_t* rows, const int32_t* cols);
/* every D x D block between the vertices of each simplex (F: nF x (dim+1) node ids) */
int mmx_struc_mesh_pattern(mmx_struc s, int dim, int nF, const int32_t* F);
int mmx_struc_pack(mmx_struc s);
/* n and nnz of the packed structure; ia (n+1) and ja (nnz) copied out when non-null */
int mmx_struc_get(mmx_struc s, int* n, long long* nnz, int32_t* ia, int32_t* ja);
int mmx_struc_destroy(mmx_struc s);

int mmx_matrix_create(int device, int n, const int32_t* ia, const int32_t* ja, mmx_matrix* out);
int mmx_matrix_create_from_struc(int device, mmx_struc s, mmx_matrix* out);
int mmx_matrix_sizes(mmx_matrix m, int* n, long long* nnz);
int mmx_matrix_stream(mmx_matrix m, void** hip_stream);
int mmx_matrix_set_values(mmx_matrix m, const double* a);
int mmx_matrix_set_values_device(mmx_matrix m, const double* d_a);
int mmx_matrix_set_rhs(mmx_matrix m, const double* b);
int mmx_matrix_set_rhs_device(mmx_matrix m, const double* d_b);
int mmx_matrix_set_toler(mmx_matrix m, const double* tol);
int mmx_matrix_sfac(mmx_matrix m, const mmx_param_iter* p);
/* x: initial guess on entry when initial_guess != 0; solution on exit */
int mmx_matrix_solve(mmx_matrix m, const mmx_param_iter* p, double* x, int* nitr, int initial_guess);
int mmx_matrix_solve_device(mmx_matrix m, const mmx_param_iter* p, double* d_x, int* nitr, int initial_guess);
int mmx_matrix_matmult(mmx_matrix m, const double* x, double* y);
int mmx_matrix_matmult_device(mmx_matrix m, const double* d_x, double* d_y);
int mmx_matrix_factor(mmx_matrix m);
int mmx_matrix_ilu_solve(mmx_matrix m, const double* b, double* x);
int mmx_matrix_ilu_solve_device(mmx_matrix m, const double* d_b, double* d_x);
/* factor in CSR form: iaf (n+1), jaf/af (nnz of the factor), diag (n, row-relative) */
int mmx_matrix_factor_nnz(mmx_matrix m, long long* nnzf);
int mmx_matrix_get_factor(mmx_matrix m, int32_t* iaf, int32_t* jaf, double* af, int32_t* diag);
int mmx_matrix_set_timing(mmx_matrix m, int on);
int mmx_matrix_stats_get(mmx_matrix m, mmx_sparse_stats* out);
int mmx_matrix_stats_reset(mmx_matrix m);
int mmx_matrix_destroy(mmx_matrix m);

/* Host-only symbolic ILU (sfac2 + merge2, lib/LASolver/ILU_class.cpp:17-295), natural order: the
 * factor pattern at `level`.  Call with null arrays to get *nnzf, then with iaf (n+1), jaf (*nnzf)
 * and diag (n, row-relative). */
int mmx_ilu_symbolic(int n, const int32_t* ia, const int32_t* ja, int level, long long* nnzf, int32_t* iaf,
                     int32_t* jaf, int32_t* diag);

/* Diagnostics (host only): the chain/band schedule the sweeps would use for the ILU(level) of this
 * pattern.  info[16]: ok, E, R, RI, bands, chains, max chain length,
 * max skew, max band iterations, slots, imports, simulated critical iterations, levels. */
/* Cycle counters of the chain sweeps when MMX_CHAIN_PROF=1 was set before sfac (1024 values:
 * forward 0..511, backward 512..1023; layout in chain_sweep.hip); reset != 0 zeroes them. */
int mmx_matrix_chain_prof(mmx_matrix m, unsigned long long* out, int reset);
int mmx_sweep_schedule_info(int n, const int32_t* ia, const int32_t* ja, int level, int fwd, long long* info);
/* Diagnostics: the chain/band schedule of the numeric factor (chain_factor.hip) for the pattern,
 * replayed on the host (fails with the reason when invalid).  info[0..7]: ok, bands, slots, ring
 * slots R, imports (rows), most import slots a band uses, modelled critical path, DAG levels. */
int mmx_factor_schedule_info(int n, const int32_t* ia, const int32_t* ja, int level, long long* info);

/* Measurement utility (no reference counterpart): the achievable HBM ceiling.  Copies n doubles
 * (n even, device pointers, 16-byte aligned) reps times with a 16-B-per-lane streaming kernel
 * (variant 0: grid-stride, nontemporal; 1: one element per lane; 2: four per lane) on a private
 * stream; *ms = average milliseconds per copy (bytes moved per copy: 16 n).  Variants 3-8 calibrate
 * the rocprofv3 byte counters on the ADMM kernels' access widths (profiles/r04/calib_counters.py):
 * 3 reads 8 B per lane, 4 a 24-B record per lane (three 8-B loads), 5 16 B per lane, 6 / 7 store
 * 8 B per lane (plain / nontemporal), 8 reads a random 24-B record per lane; each touches 8 n bytes
 * (8: n/3 records). */
int mmx_stream_copy(int device, const double* d_src, double* d_dst, long long n, int reps, int variant, double* ms);
/* test hook: a kernel of `blocks` workgroups (1024 lanes, 64 KB LDS each) on a stream of its own
 * that holds their CUs for ms milliseconds (asynchronous; mmx_occupy_wait waits for it).  The
 * solver's kernels must complete beside it (the wave factor takes rows by ticket: no co-residency
 * assumed; tests/test_gpu_lasolver.py). */
int mmx_occupy(int device, int blocks, double ms);
int mmx_occupy_wait(void);

#ifdef __cplusplus
}
#endif
#endif
