// sparse_kernels.hip -- the LASolver path (backward Euler's ILU(0)-preconditioned CG-STAB,
// lib/LASolver) as HIP kernels for gfx950.  All arithmetic is fp64 and rounds exactly as the
// reference writes it (-ffp-contract=off):
//   * SpMV sums each row sequentially from 0.0 in storage order (matmult, accel_class.cpp:537-548),
//     so y is bit-identical to the reference;
//   * the ILU(0) factor and both sweeps apply every row's updates in ascending column order
//     (ILU_class.cpp:360-420, 470-510), so factors and sweep results are bit-identical;
//   * dot products and norms are deterministic fixed-shape tree sums (not the reference's
//     sequential sums): CG-STAB iterates agree to rounding, see tests/test_gpu_lasolver.py.
//
// The triangular sweeps and the factor are sync-free: rows are handed out to wavefronts in
// dispatch order by a ticket counter (so a wavefront only ever waits on rows owned by wavefronts
// that are already running), each lane owns one row, and a row publishes its value as two
// self-validating 8-byte {epoch, half} granules written by agent-scope (sc1) stores
// (MI355X_MICROARCH.md §inter-workgroup visibility, R2 granules); dependencies inside the
// wavefront are forwarded through LDS.  Every wait is bounded and reports through *err.
#include <hip/hip_runtime.h>

#include "sparse_kernels.h"

namespace mmx {

namespace {

constexpr unsigned kSpinMax = 1u << 24;  // idle rounds before a dependency wait gives up

__device__ __forceinline__ void store_granule(uint64_t* g, unsigned epoch, double v) {
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  const uint64_t tag = (uint64_t)epoch << 32;
  __hip_atomic_store(g, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool load_granule(const uint64_t* g, unsigned epoch, double& v) {
  const uint64_t lo = __hip_atomic_load(const_cast<uint64_t*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t hi = __hip_atomic_load(const_cast<uint64_t*>(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((unsigned)(lo >> 32) != epoch || (unsigned)(hi >> 32) != epoch) return false;
  v = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
  return true;
}

// value of a granule written by an earlier launch (no tag check needed)
__device__ __forceinline__ double granule_value(const uint64_t* g) {
  const uint64_t lo = g[0], hi = g[1];
  return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
}

__device__ __forceinline__ double ld_agent(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((uint64_t*)const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store((uint64_t*)p, (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS word exchange between lanes of one wavefront (relaxed atomics: never cached in registers)
__device__ __forceinline__ double lds_get(uint64_t* p) {
  return __longlong_as_double((long long)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT));
}
__device__ __forceinline__ void lds_put(uint64_t* p, double v) {
  __hip_atomic_store(p, (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ int take_ticket(unsigned* ticket) {
  __shared__ int s_blk;
  if (threadIdx.x == 0) s_blk = (int)atomicAdd(ticket, 1u);
  __syncthreads();
  return s_blk;
}

// fixed-shape block tree over NV values per thread; thread 0 returns the sums
template <int NV, int B>
__device__ __forceinline__ void block_sum(double (&v)[NV], double (*red)[NV]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) red[threadIdx.x][i] = v[i];
  __syncthreads();
  for (int w = B / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
#pragma unroll
      for (int i = 0; i < NV; ++i) red[threadIdx.x][i] = red[threadIdx.x][i] + red[threadIdx.x + w][i];
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[0][i];
}

}  // namespace

int vec_grid(int n) {
  const int g = (n + kVecBlock - 1) / kVecBlock;
  return g < 1 ? 1 : (g > 1024 ? 1024 : g);
}

// ---------------------------------------------------------------------------------------------
// SpMV: one workgroup per row block (host-built, <= kSpmvTile nonzeros or one long row).  The
// block's products a[k]*x[ja[k]] are formed by coalesced streaming loads and staged in LDS; then
// one lane per row sums its products sequentially from 0.0.
template <int EPI>
__global__ void __launch_bounds__(kSpmvBlock) k_spmv(const int* __restrict__ rowblk, const int* __restrict__ ia,
                                                      const int* __restrict__ ja, const double* __restrict__ a,
                                                      const double* __restrict__ x, double* __restrict__ y,
                                                      const double* __restrict__ e1, double* __restrict__ partials) {
  __shared__ double prod[kSpmvTile];
  __shared__ double red[kSpmvBlock][2];
  const int b = blockIdx.x;
  const int r0 = rowblk[b], r1 = rowblk[b + 1];
  const int k0 = ia[r0], k1 = ia[r1];
  double pv[2] = {0.0, 0.0};
  if (k1 - k0 <= kSpmvTile) {
#pragma unroll 8
    for (int k = k0 + (int)threadIdx.x; k < k1; k += kSpmvBlock) prod[k - k0] = a[k] * x[ja[k]];
    __syncthreads();
    for (int r = r0 + (int)threadIdx.x; r < r1; r += kSpmvBlock) {
      const int e = ia[r + 1];
      double s = 0.0;
      for (int kk = ia[r]; kk < e; ++kk) s += prod[kk - k0];
      y[r] = s;
      if (EPI == 1) pv[0] += e1[r] * s;
      if (EPI == 2) {
        pv[0] += s * e1[r];
        pv[1] += s * s;
      }
    }
  } else {  // a single row longer than the tile: chunks, summed in order by lane 0
    double s = 0.0;
    for (int c = k0; c < k1; c += kSpmvTile) {
      const int ce = (c + kSpmvTile < k1) ? c + kSpmvTile : k1;
      for (int k = c + (int)threadIdx.x; k < ce; k += kSpmvBlock) prod[k - c] = a[k] * x[ja[k]];
      __syncthreads();
      if (threadIdx.x == 0)
        for (int k = c; k < ce; ++k) s += prod[k - c];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      y[r0] = s;
      if (EPI == 1) pv[0] += e1[r0] * s;
      if (EPI == 2) {
        pv[0] += s * e1[r0];
        pv[1] += s * s;
      }
    }
  }
  if (EPI != 0) {
    __syncthreads();
    block_sum<2, kSpmvBlock>(pv, red);
    if (threadIdx.x == 0) {
      partials[(size_t)b * 2 + 0] = pv[0];
      partials[(size_t)b * 2 + 1] = pv[1];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// ILU(0) numeric factor (scaler_ILU::factor, ILU_class.cpp:300-444), one row per lane.  The row's
// entries are zeroed, A's values loaded, then for every lower entry id in ascending order
// mult = row[id] / U(id,id) and row[idd] -= mult * U(id, idd) for the entries idd of row id's
// upper part that row i holds (two sorted lists merged).  Rows publish through agent-scope
// stores + a drained flag; readers use agent-scope loads only.
__global__ void __launch_bounds__(kSweepRows) k_ilu_factor(int n, const int* __restrict__ ia, const int* __restrict__ ja,
                                                          const double* __restrict__ a, const int* __restrict__ amap,
                                                          const int* __restrict__ iaf, const int* __restrict__ jaf,
                                                          const int* __restrict__ dg, double* af, unsigned* flags,
                                                          unsigned epoch, unsigned* ticket, unsigned* err) {
  const int blk = take_ticket(ticket);
  const int i = blk * kSweepRows + (int)threadIdx.x;
  const bool valid = i < n;
  int kk = 0, kd = 0, ke = 0;
  if (valid) {
    kk = iaf[i];
    kd = dg[i];
    ke = iaf[i + 1];
    for (int k = kk; k < ke; ++k) st_agent(&af[k], 0.0);
    for (int ii = ia[i]; ii < ia[i + 1]; ++ii) st_agent(&af[amap[ii]], a[ii]);
  }
  bool done = !valid;
  unsigned spins = 0;
  while (true) {
    bool fin = false;
    if (!done) {
      while (kk < kd) {
        const int id = jaf[kk];
        if (__hip_atomic_load(&flags[id], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) break;
        const double mult = ld_agent(&af[kk]) / ld_agent(&af[dg[id]]);
        st_agent(&af[kk], mult);
        int p = kk + 1;
        const int ue = iaf[id + 1];
        for (int iii = dg[id] + 1; iii < ue; ++iii) {
          const int idd = jaf[iii];
          while (p < ke && jaf[p] < idd) ++p;
          if (p < ke && jaf[p] == idd) st_agent(&af[p], ld_agent(&af[p]) - mult * ld_agent(&af[iii]));
        }
        ++kk;
      }
      fin = (kk == kd);
    }
    if (fin) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&flags[i], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      done = true;
    }
    if (__all(done)) break;
    if (__ballot(fin) == 0) {
      if (++spins > kSpinMax) {
        atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Forward sweep L y = b (unit diagonal; ILU_class.cpp:470-481): y_i = b_i - sum_{k<diag} af_k y_jk,
// subtracted one term at a time in ascending column order.
template <int PRO>
__global__ void __launch_bounds__(kSweepRows) k_sweep_fwd(int n, const int* __restrict__ iaf, const int* __restrict__ jaf,
                                                         const int* __restrict__ dg, const double* __restrict__ af,
                                                         const double* __restrict__ src, double* __restrict__ p,
                                                         const double* __restrict__ res, const double* __restrict__ avbar,
                                                         const CgsScalars* __restrict__ sc, uint64_t* gy, unsigned epoch,
                                                         unsigned* ticket, unsigned* err) {
  __shared__ uint64_t s_val[kSweepRows];  // row values forwarded inside the wavefront
  const int blk = take_ticket(ticket);
  const int lane = (int)threadIdx.x;
  const int w0 = blk * kSweepRows;
  const int i = w0 + lane;
  const bool valid = i < n;
  double acc = 0.0;
  int k = 0, ke = 0;
  if (valid) {
    double b;
    if (PRO == 0) {
      b = src[i];
    } else if (PRO == 1) {  // pvec = res + beta*(pvec - omega*avbar)   (accel_class.cpp:339-341)
      b = res[i] + sc->beta * (p[i] - sc->omega * avbar[i]);
      p[i] = b;
    } else {  // svec = res - alpha*avbar   (accel_class.cpp:361-363)
      b = res[i] - sc->alpha * avbar[i];
      p[i] = b;
    }
    acc = b;
    k = iaf[i];
    ke = dg[i];
  }
  bool done = !valid;
  uint64_t ready = 0;
  unsigned spins = 0;
  while (true) {
    bool fin = false;
    if (!done) {
      while (k < ke) {
        const int j = jaf[k];
        double v;
        if (j >= w0) {
          if (!((ready >> (j - w0)) & 1ull)) break;
          v = lds_get(&s_val[j - w0]);
        } else if (!load_granule(gy + 2 * (size_t)j, epoch, v)) {
          break;
        }
        acc -= af[k] * v;
        ++k;
      }
      fin = (k == ke);
    }
    if (fin) {
      lds_put(&s_val[lane], acc);
      store_granule(gy + 2 * (size_t)i, epoch, acc);
      done = true;
    }
    const uint64_t fm = __ballot(fin);
    ready |= fm;
    if (__all(done)) break;
    if (fm == 0) {
      if (++spins > kSpinMax) {
        atomicOr(err, 2u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

// Backward sweep U x = y (ILU_class.cpp:485-499): x_i = (y_i - sum_{k>diag} af_k x_jk) / af_diag,
// rows handed out from the last one down.
__global__ void __launch_bounds__(kSweepRows) k_sweep_bwd(int n, const int* __restrict__ iaf, const int* __restrict__ jaf,
                                                         const int* __restrict__ dg, const double* __restrict__ af,
                                                         const uint64_t* __restrict__ gy, double* __restrict__ out,
                                                         uint64_t* gx, unsigned epoch, unsigned* ticket, unsigned* err) {
  __shared__ uint64_t s_val[kSweepRows];  // row values forwarded inside the wavefront
  const int blk = take_ticket(ticket);
  const int lane = (int)threadIdx.x;
  const int whi = n - 1 - blk * kSweepRows;  // row of lane 0; lane l owns row whi - l
  const int i = whi - lane;
  const bool valid = i >= 0;
  double acc = 0.0;
  int k = 0, ke = 0, kd = 0;
  if (valid) {
    acc = granule_value(gy + 2 * (size_t)i);
    kd = dg[i];
    k = kd + 1;
    ke = iaf[i + 1];
  }
  bool done = !valid;
  uint64_t ready = 0;
  unsigned spins = 0;
  while (true) {
    bool fin = false;
    if (!done) {
      while (k < ke) {
        const int j = jaf[k];
        double v;
        if (j <= whi) {
          if (!((ready >> (whi - j)) & 1ull)) break;
          v = lds_get(&s_val[whi - j]);
        } else if (!load_granule(gx + 2 * (size_t)j, epoch, v)) {
          break;
        }
        acc -= af[k] * v;
        ++k;
      }
      fin = (k == ke);
    }
    if (fin) {
      acc = acc / af[kd];
      lds_put(&s_val[lane], acc);
      out[i] = acc;
      store_granule(gx + 2 * (size_t)i, epoch, acc);
      done = true;
    }
    const uint64_t fm = __ballot(fin);
    ready |= fm;
    if (__all(done)) break;
    if (fm == 0) {
      if (++spins > kSpinMax) {
        atomicOr(err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// CG-STAB vector kernels (scaler_cgstab, accel_class.cpp:263-399).
__global__ void __launch_bounds__(kVecBlock) k_cgs_init(int mode, int n, const double* __restrict__ b, double* __restrict__ x,
                                                       double* __restrict__ res, double* __restrict__ res0,
                                                       double* __restrict__ p, double* __restrict__ avbar, int copy_res0,
                                                       double* __restrict__ partials) {
  __shared__ double red[kVecBlock][2];
  double pv[2] = {0.0, 0.0};
  for (int i = blockIdx.x * kVecBlock + threadIdx.x; i < n; i += gridDim.x * kVecBlock) {
    double r;
    if (mode == 0) {  // MatrixIter.cpp:708-715: x = 0, res = b
      x[i] = 0.0;
      r = b[i];
    } else {  // MatrixIter.cpp:719-724: res = b - A x
      r = b[i] - res[i];
    }
    res[i] = r;
    if (copy_res0) res0[i] = r;
    p[i] = 0.0;
    avbar[i] = 0.0;
    pv[0] += r * r;
  }
  pv[1] = pv[0];
  block_sum<2, kVecBlock>(pv, red);
  if (threadIdx.x == 0) {
    partials[(size_t)blockIdx.x * 2 + 0] = pv[0];
    partials[(size_t)blockIdx.x * 2 + 1] = pv[1];
  }
}

__global__ void __launch_bounds__(kVecBlock) k_dot_into(int n, const double* __restrict__ x, const double* __restrict__ y,
                                                       double* __restrict__ partials) {
  __shared__ double red[kVecBlock][1];
  double pv[1] = {0.0};
  for (int i = blockIdx.x * kVecBlock + threadIdx.x; i < n; i += gridDim.x * kVecBlock) pv[0] += x[i] * y[i];
  block_sum<1, kVecBlock>(pv, red);
  if (threadIdx.x == 0) partials[(size_t)blockIdx.x * 2 + 1] = pv[0];
}

__global__ void __launch_bounds__(kVecBlock) k_cgs_update(int n, const double* __restrict__ vbar, const double* __restrict__ z,
                                                         const double* __restrict__ s, const double* __restrict__ t,
                                                         const double* __restrict__ res0, const double* __restrict__ toler,
                                                         double* __restrict__ x, double* __restrict__ res,
                                                         const CgsScalars* __restrict__ sc, double* __restrict__ partials) {
  __shared__ double red[kVecBlock][3];
  const double alpha = sc->alpha, omega = sc->omega;
  double pv[3] = {0.0, 0.0, 0.0};
  for (int i = blockIdx.x * kVecBlock + threadIdx.x; i < n; i += gridDim.x * kVecBlock) {
    const double step1 = alpha * vbar[i];
    const double step2 = omega * z[i];
    const double step = step1 + step2;
    const double tl = toler ? toler[i] : 0.0;
    if (fabs(step) > fabs(tl)) pv[2] += 1.0;
    x[i] = x[i] + step;
    const double r = s[i] - omega * t[i];
    res[i] = r;
    pv[0] += r * r;
    pv[1] += res0[i] * r;
  }
  block_sum<3, kVecBlock>(pv, red);
  if (threadIdx.x == 0) {
    partials[(size_t)blockIdx.x * 3 + 0] = pv[0];
    partials[(size_t)blockIdx.x * 3 + 1] = pv[1];
    partials[(size_t)blockIdx.x * 3 + 2] = pv[2];
  }
}

// Scalar finalisers: fixed-shape reduction of the per-block partials, then the CG-STAB scalar
// recurrences exactly as written in acc_scaler.
template <int MODE>
__global__ void __launch_bounds__(kVecBlock) k_cgs_fin(const double* __restrict__ partials, int nblk, CgsScalars* sc) {
  constexpr int NV = (MODE == 3) ? 3 : 2;
  __shared__ double red[kVecBlock][NV];
  double v[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = 0.0;
  for (int b = threadIdx.x; b < nblk; b += kVecBlock)
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] += partials[(size_t)b * NV + q];
  block_sum<NV, kVecBlock>(v, red);
  if (threadIdx.x != 0) return;
  const double tiny = 1.e-300;
  if (MODE == 0) {  // scaler_cgstab::init + the rho/beta head of the first acc_scaler call
    sc->rmsi = sqrt(v[0]);
    sc->alpha = 1.0;
    sc->rholst = 1.0;
    sc->omega = 1.0;
    const double rho = v[1];
    double beta = rho / (sc->rholst + tiny);
    beta *= (sc->alpha / (sc->omega + tiny));
    sc->rho = rho;
    sc->beta = beta;
    sc->rholst = rho;
    sc->conv = 0;
  } else if (MODE == 1) {  // alpha = rho / (res0, avbar)
    sc->alpha = sc->rho / v[0];
  } else if (MODE == 2) {  // omega = (t, s) / ((t, t) + tiny)
    sc->omega = v[0] / (v[1] + tiny);
  } else {  // rms, convergence, and the next iteration's rho/beta
    const double rms = sqrt(v[0]);
    sc->rms = rms;
    sc->iconv = v[2];
    sc->conv = (v[2] == 0.0 || (rms / sc->rmsi) < sc->ctol) ? 1 : 0;
    const double rho = v[1];
    double beta = rho / (sc->rholst + tiny);
    beta *= (sc->alpha / (sc->omega + tiny));
    sc->rho = rho;
    sc->beta = beta;
    sc->rholst = rho;
  }
}

// ---------------------------------------------------------------------------------------------
void launch_spmv(int epi, int nblk, const int* rowblk, const int* ia, const int* ja, const double* a, const double* x,
                 double* y, const double* e1, double* partials, hipStream_t st) {
  if (nblk <= 0) return;
  if (epi == 0)
    hipLaunchKernelGGL(k_spmv<0>, dim3(nblk), dim3(kSpmvBlock), 0, st, rowblk, ia, ja, a, x, y, e1, partials);
  else if (epi == 1)
    hipLaunchKernelGGL(k_spmv<1>, dim3(nblk), dim3(kSpmvBlock), 0, st, rowblk, ia, ja, a, x, y, e1, partials);
  else
    hipLaunchKernelGGL(k_spmv<2>, dim3(nblk), dim3(kSpmvBlock), 0, st, rowblk, ia, ja, a, x, y, e1, partials);
}

void launch_ilu_factor(int n, const int* ia, const int* ja, const double* a, const int* amap, const int* iaf,
                       const int* jaf, const int* dg, double* af, unsigned* flags, unsigned epoch, unsigned* ticket,
                       unsigned* err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ilu_factor, dim3((n + kSweepRows - 1) / kSweepRows), dim3(kSweepRows), 0, st, n, ia, ja, a, amap,
                     iaf, jaf, dg, af, flags, epoch, ticket, err);
}

void launch_sweep_fwd(int pro, int n, const int* iaf, const int* jaf, const int* dg, const double* af, const double* src,
                      double* p, const double* res, const double* avbar, const CgsScalars* sc, uint64_t* gy,
                      unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st) {
  if (n <= 0) return;
  const dim3 g((n + kSweepRows - 1) / kSweepRows), b(kSweepRows);
  if (pro == 0)
    hipLaunchKernelGGL(k_sweep_fwd<0>, g, b, 0, st, n, iaf, jaf, dg, af, src, p, res, avbar, sc, gy, epoch, ticket, err);
  else if (pro == 1)
    hipLaunchKernelGGL(k_sweep_fwd<1>, g, b, 0, st, n, iaf, jaf, dg, af, src, p, res, avbar, sc, gy, epoch, ticket, err);
  else
    hipLaunchKernelGGL(k_sweep_fwd<2>, g, b, 0, st, n, iaf, jaf, dg, af, src, p, res, avbar, sc, gy, epoch, ticket, err);
}

void launch_sweep_bwd(int n, const int* iaf, const int* jaf, const int* dg, const double* af, const uint64_t* gy,
                      double* out, uint64_t* gx, unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_sweep_bwd, dim3((n + kSweepRows - 1) / kSweepRows), dim3(kSweepRows), 0, st, n, iaf, jaf, dg, af,
                     gy, out, gx, epoch, ticket, err);
}

void launch_cgs_init(int mode, int n, const double* b, double* x, double* res, double* res0, double* p, double* avbar,
                     int copy_res0, double* partials, hipStream_t st) {
  hipLaunchKernelGGL(k_cgs_init, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, mode, n, b, x, res, res0, p, avbar,
                     copy_res0, partials);
}

void launch_dot_into(int n, const double* x, const double* y, double* partials, hipStream_t st) {
  hipLaunchKernelGGL(k_dot_into, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, n, x, y, partials);
}

void launch_cgs_update(int n, const double* vbar, const double* z, const double* s, const double* t, const double* res0,
                       const double* toler, double* x, double* res, const CgsScalars* sc, double* partials,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_cgs_update, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, n, vbar, z, s, t, res0, toler, x, res, sc,
                     partials);
}

void launch_cgs_fin(int mode, const double* partials, int nblk, CgsScalars* sc, hipStream_t st) {
  const dim3 g(1), b(kVecBlock);
  switch (mode) {
    case 0: hipLaunchKernelGGL(k_cgs_fin<0>, g, b, 0, st, partials, nblk, sc); break;
    case 1: hipLaunchKernelGGL(k_cgs_fin<1>, g, b, 0, st, partials, nblk, sc); break;
    case 2: hipLaunchKernelGGL(k_cgs_fin<2>, g, b, 0, st, partials, nblk, sc); break;
    default: hipLaunchKernelGGL(k_cgs_fin<3>, g, b, 0, st, partials, nblk, sc); break;
  }
}

}  // namespace mmx
