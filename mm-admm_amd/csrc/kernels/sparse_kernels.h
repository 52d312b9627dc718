// sparse_kernels.h -- launch interface of the LASolver HIP kernels (gfx950): CSR SpMV
// (matmult), sync-free ILU(0) factor and triangular sweeps (scaler_ILU::factor / solve) and the
// CG-STAB vector algebra (scaler_cgstab::acc_scaler).  See DESIGN.md §LASolver.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"  // MMX_SPMV_*, MMX_CHAIN_VEC / CODE16

namespace mmx {

// Products staged in LDS per SpMV workgroup (16 KB of fp64; layout.h).
constexpr int kSpmvTile = MMX_SPMV_TILE;
constexpr int kSpmvBlock = MMX_SPMV_BLOCK;
// Rows per chunk of the level-scheduled factor/sweeps (one wavefront per chunk) and the size of
// their persistent grid (wavefronts).
constexpr int kSweepRows = 64;
constexpr int kSweepGrid = 128;  // measured: 2048 waves of pollers slow the chain 3.7x (profiles/r01/lasolver_tune.txt)
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
// The same product and partial sums from per-block descriptors {r0, r1, ia[r0], ia[r1]}; a and ja
// must be readable 2 entries past nnz.
void launch_spmv2(int epi, int nblk, const int4* desc, const int* ia, const int* ja, const double* a,
                  const double* x, double* y, const double* e1, double* partials, hipStream_t st);

// ILU numeric factor in the factor pattern (iaf/jaf/dg); amap maps A's entries into it.  perm: rows
// in forward-level order, padded with -1 to whole chunks of kSweepRows.
// piv[k] for a lower entry k of row i: {dg[id], iaf[id+1]} of its pivot row id = jaf[k].
void launch_ilu_factor(const int* ia, const int* ja, const double* a, const int* amap, const int* iaf, const int* jaf,
                       const int* dg, const int2* piv, const int* perm, int nchunks, double* af, unsigned* flags,
                       unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st);

// The same factor with each lane's row in LDS (rows of at most kFacW entries): toff[k] for a lower
// entry k indexes tgt[], which holds for each upper entry of k's pivot row (after the diagonal)
// the position in row i it updates, or -1.
constexpr int kFacW = 127;
void launch_ilu_factor_lds(const int* ia, const double* a, const int* amap, const int* iaf, const int* jaf, const int* dg,
                           const int2* piv, const int* toff, const signed char* tgt, const int* perm, int nchunks,
                           double* af, unsigned* flags, unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st);

// One wavefront per row (k_ilu_factor_wave): perm = every row once in forward level order (no
// padding); rows of at most kFacW entries, kFacWaveNL lower entries and 64 upper entries per pivot
// row.  Bit-identical to the other factors.  gF (2 x nnz(factor) words, or null): rows publish their
// diagonal and upper part as epoch-tagged granules there instead of drained stores + a flag.
constexpr int kFacWaveNL = 32;
void launch_ilu_factor_wave(const int* ia, const double* a, const int* amap, const int* iaf, const int* dg,
                            const int2* piv, const int* jaf, const int* toff, const signed char* tgt, const int* perm,
                            int nrows, double* af, unsigned* flags, uint64_t* gF, unsigned epoch, unsigned* ticket,
                            unsigned* err, hipStream_t st);
// the factor's precomputed dependent loads, from the factor pattern (iaf, jaf, dg on the device):
// per lower entry k of row i, piv[k] = (diag position, end) of its pivot row (0, 0 elsewhere); with
// toff / tgt: toff[k] = rowTot[i] + the pivot upper lengths of row i's earlier lower entries, and
// tgt[toff[k] + u] = the position in row i of the pivot row's u-th upper column, or -1
void launch_fac_prep(int n, const int* iaf, const int* jaf, const int* dg, const long long* rowTot, int2* piv,
                     int* toff, signed char* tgt, hipStream_t st);
// test hook: blocks x 1024 lanes (64 KB LDS each) holding their CUs for ms milliseconds
void launch_occupy(int blocks, double ms, double* sink, hipStream_t st);

// Sweep over the rows of perm (forward or backward level order).  Forward: unit L into granules
// gout, right-hand side per pro (0: src; 1: p = res + beta (p - omega avbar); 2: s = res - alpha
// avbar, stored to p).  Backward: U from the forward granules gin into out and granules gout.
void launch_sweep(bool fwd, int pro, const int* iaf, const int* jaf, const int* dg, const double* af, const int* perm,
                  int nchunks, const double* src, double* p, const double* res, const double* avbar, const CgsScalars* sc,
                  const uint64_t* gin, uint64_t* gout, double* out, unsigned epoch, unsigned* ticket, unsigned* err,
                  hipStream_t st);

// Band/chain-scheduled sweeps (chain_sweep.hip, schedule host/chain_sched.h): the same rows and
// arithmetic as launch_sweep, with intra-band dependencies resolved in LDS.
inline constexpr bool chain_code16(int ee) { return MMX_CHAIN_CODE16 || ee > 32; }

struct ChainArgs {
  const int* bandSlot;
  const int* bandT;
  const int* bandImp;
  const int* bandNImp;
  const int* laneStart;
  const int* laneLen;
  const int* laneSkew;
  const int* laneNs;   // per band * 64 + lane: segments per row (seg schedules; rows wider than 32 entries)
  const int* bandE;    // per band: entry slots in use (multiple of 4)
  const double* val;   // [slot][E][64] entry values (filled from the factor by launch_chain_fill)
  const void* code;    // [slot][E][64] LDS index of the entry's value (0: the zero cell): uint16 (chain_code16) or int32
  const double* dval;  // [slot][64] diagonals (backward)
  const int* impRow;
  const int* impSlot;  // per import: LDS import slot
  const int* impWait;  // per import: iterations the compute wave completes before it is delivered (-1 none)
  const int* impNeed;  // per slot: highest import index read at that iteration (-1: none)
  const int* bandOrder;  // per ticket: the band taken
  int nbands, R, RI;
  int seg;             // the schedule splits rows into segments of 32 entries (k_chain_sweep<..., 32, true, 1>)
  int G;               // rows per position (2: pairs of consecutive chain rows)
  unsigned long long* prof;  // optional cycle counters (MMX_CHAIN_PROF), see chain_sweep.hip
  int profIter;              // MMX_CHAIN_PROF=2: also time the waits inside iterations (perturbs them)
  int trim;                  // loaders move only bandE entry slots of bands using at most half (MMX_CHAIN_TRIM=0: all)
};
void launch_chain_sweep(bool fwd, int pro, int E, const ChainArgs& ca, const double* src, double* p, const double* res,
                        const double* avbar, const CgsScalars* sc, const uint64_t* gin, uint64_t* gout, double* out,
                        unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st);
// the numeric ILU(0) factor on the forward chain/band schedule (chain_factor.hip; host/chain_sched.h
// build_factor_schedule)
struct FactorArgs {
  const int* bandSlot;
  const int* bandT;
  const int* laneLen;
  const int* laneSkew;
  const int* bandOrder;
  const int* bandImp;
  const int* bandNImp;
  const int* impPos;    // per import: factor position of the row's diagonal
  const int* impCnt;    //   its diagonal + upper entries
  const int* impSlot;
  const int* impWait;
  const int* impNeed;   // per slot
  const double* val;    // [slot][kFacWF / 2][64][2] the row's initial values (launch_chain_fill)
  const uint16_t* code; // [slot][kFacNSC / 8][64][8] LDS indices of the update and pivot values
  const int* meta;      // [slot][64] W | nlow << 8 | 1 << 16
  const int* rowStart;  // [slot][64] factor position of the row's first entry
  int nbands, R;
  unsigned long long* prof;  // optional cycle counters (MMX_CHAIN_PROF): 0 compute total, 1 stage
                             // waits, 2 import waits, 3 iterations, 4 bands, 5 importer cycles
};
void launch_chain_factor(const FactorArgs& fa, double* af, uint64_t* gU, unsigned epoch, unsigned* ticket,
                         unsigned* err, hipStream_t st);
// af[amap[k]] = a[k] over the nnz entries of A (af zeroed before: the fill entries start at 0)
void launch_scatter_a(long long nnz, const int* amap, const double* a, double* af, hipStream_t st);

// val[x] = af[srcIdx[x]] (padValue where srcIdx < 0)
void launch_chain_fill(long long n, const int* srcIdx, const double* af, double* val, double padValue,
                       hipStream_t st);

// init: x = 0, res = b (mode 0) or res = b - res (mode 1, res holding A x); res0 = res; p = 0;
// avbar = 0.  Partials [sum res^2, sum res0.res] per block.
void launch_cgs_init(int mode, int n, const double* b, double* x, double* res, double* res0, double* p,
                     double* avbar, int copy_res0, double* partials, hipStream_t st);
// partials[b*2+1] = block sum of x.y
void launch_dot_into(int n, const double* x, const double* y, double* partials, hipStream_t st);
// sol += alpha vbar + omega z; res = s - omega t; partials [res^2, res0.res, #|step|>|toler|].
// out[i] = the value in row i's granule (gx / gy: {tag | lo, tag | hi})
void launch_gran_extract(int n, const uint64_t* g, double* out, hipStream_t st);
// the forward sweep's prologue as its own pass: mode 1 out = res + beta (out - omega avbar), 2 out = res - alpha avbar
void launch_cgs_pro(int mode, int n, const double* res, const double* avbar, double* out, const CgsScalars* sc,
                    hipStream_t st);
void launch_cgs_update(int n, const double* vbar, const double* z, const double* s, const double* t,
                       const double* res0, const double* toler, double* x, double* res, const CgsScalars* sc,
                       double* partials, hipStream_t st);
// Scalar finalisers (one workgroup).  mode 0 init, 1 alpha, 2 omega, 3 update.
void launch_cgs_fin(int mode, const double* partials, int nblk, CgsScalars* sc, hipStream_t st);

// Measurement utility: dst = src over n2 16-byte elements (streaming copy ceiling; variants in
// sparse_kernels.hip).
void launch_stream_copy(int variant, long long n2, const double* src, double* dst, hipStream_t st);

}  // namespace mmx
