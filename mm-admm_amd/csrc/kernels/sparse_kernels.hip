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

#include <algorithm>

#include <cstdlib>

#include "sparse_kernels.h"

namespace mmx {

namespace {

constexpr unsigned kSpinMax = 1u << 24;  // idle rounds before a dependency wait gives up
constexpr int kBatch = 4;               // granule loads in flight per lane in a sweep
constexpr int kFactorBatch = 8;         // pivot-row entries loaded at once in the factor

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

int sweep_grid() {  // persistent wavefronts of the factor/sweeps (MMX_SWEEP_GRID overrides)
  static int g = [] {
    const char* e = getenv("MMX_SWEEP_GRID");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : kSweepGrid;
  }();
  return g;
}

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

// SpMV v2: the same blocks and the same sums, with the block's memory requests all issued up
// front.  The block descriptor {r0, r1, k0, k1} comes from one 16-byte load (no rowblk -> ia
// chain); each lane loads up to 5 aligned pairs of (a, ja) as 16-byte / 8-byte vectors with
// nontemporal hints (read once: they should not evict x from L2), then gathers x, so a
// workgroup has its whole tile in flight; the row bounds and e1 are fetched before the tile
// lands.  Logical blocks are XCD-chunked (each XCD walks a contiguous range of rows, so the x
// windows of consecutive blocks hit its own L2).  a and ja carry 2 padding entries (host) so the
// last pair never reads past the arrays.  Partial sums are indexed by logical block: the same
// rows per partial as k_spmv, so the reductions are unchanged.
constexpr int kSpmvPairs = kSpmvTile / (2 * kSpmvBlock) + 1;  // 5: covers an odd start
typedef int v2i_t __attribute__((ext_vector_type(2)));
typedef double v2d_t __attribute__((ext_vector_type(2)));

template <int EPI>
__global__ void __launch_bounds__(kSpmvBlock) k_spmv2(const int4* __restrict__ desc, int nblk,
                                                       const int* __restrict__ ia, const int* __restrict__ ja,
                                                       const double* __restrict__ a, const double* __restrict__ x,
                                                       double* __restrict__ y, const double* __restrict__ e1,
                                                       double* __restrict__ partials) {
  __shared__ double prod[kSpmvTile + 2];
  __shared__ double red[kSpmvBlock][2];
  const int G = (int)gridDim.x;  // a multiple of 8
  const int b = (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8);
  if (b >= nblk) return;  // whole workgroup: no barrier is skipped by a part of it
  const int tid = (int)threadIdx.x;
  const int4 d = desc[b];
  const int r0 = d.x, r1 = d.y, k0 = d.z, k1 = d.w;
  double pv[2] = {0.0, 0.0};
  if (k1 - k0 <= kSpmvTile) {
    const int ka = k0 & ~1;
    const int np = (k1 - ka + 1) >> 1;
    // first row of this lane: bounds (and e1) requested before the tile.  Every load below is
    // unconditional (out-of-range lanes re-read a valid pair): no branch separates the requests,
    // so the compiler issues them all before the first wait.
    const int rf = r0 + tid;
    const int rc = rf < r1 ? rf : r1 - 1;
    int ib = ia[rc], ie = ia[rc + 1];
    double ef = 0.0;
    if (EPI != 0) ef = e1[rc];
    const int pmax = np > 0 ? np - 1 : 0;
    v2i_t jv[kSpmvPairs];
    v2d_t av[kSpmvPairs];
#pragma unroll
    for (int j = 0; j < kSpmvPairs; ++j) {
      const int p = min(tid + j * kSpmvBlock, pmax);
      jv[j] = __builtin_nontemporal_load(reinterpret_cast<const v2i_t*>(ja + ka) + p);
      av[j] = __builtin_nontemporal_load(reinterpret_cast<const v2d_t*>(a + ka) + p);
    }
    double xv0[kSpmvPairs], xv1[kSpmvPairs];
#pragma unroll
    for (int j = 0; j < kSpmvPairs; ++j) {
      xv0[j] = x[jv[j].x];
      xv1[j] = x[jv[j].y];
    }
#pragma unroll
    for (int j = 0; j < kSpmvPairs; ++j) {
      const int p = tid + j * kSpmvBlock;
      if (p < np) {
        prod[2 * p] = av[j].x * xv0[j];
        prod[2 * p + 1] = av[j].y * xv1[j];
      }
    }
    __syncthreads();
    for (int r = rf; r < r1; r += kSpmvBlock) {
      if (r != rf) {
        ib = ia[r];
        ie = ia[r + 1];
        if (EPI != 0) ef = e1[r];
      }
      double s = 0.0;
      for (int kk = ib; kk < ie; ++kk) s += prod[kk - ka];
      y[r] = s;
      if (EPI == 1) pv[0] += ef * s;
      if (EPI == 2) {
        pv[0] += s * ef;
        pv[1] += s * s;
      }
    }
  } else {  // a single row longer than the tile: chunks, summed in order by lane 0
    double s = 0.0;
    for (int c = k0; c < k1; c += kSpmvTile) {
      const int ce = (c + kSpmvTile < k1) ? c + kSpmvTile : k1;
      for (int k = c + tid; k < ce; k += kSpmvBlock) prod[k - c] = a[k] * x[ja[k]];
      __syncthreads();
      if (tid == 0)
        for (int k = c; k < ce; ++k) s += prod[k - c];
      __syncthreads();
    }
    if (tid == 0) {
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
    if (tid == 0) {
      partials[(size_t)b * 2 + 0] = pv[0];
      partials[(size_t)b * 2 + 1] = pv[1];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Level-scheduled sync-free factor and sweeps.  At sfac the host assigns every row its level in
// the dependency DAG of the lower (forward) or upper (backward) factor and lists the rows level by
// level, each level padded to whole chunks of 64 (padding = -1), so the 64 rows of a chunk never
// depend on each other.  A persistent grid of wavefronts takes chunks in list order from a ticket
// counter: every dependency of a chunk lies in a chunk handed out earlier, to a wavefront that is
// running, so waiting is deadlock-free.  Each lane computes one row; a row publishes its value as
// two self-validating 8-byte {epoch, half} granules (sweeps) or as agent-scope stores drained
// before an epoch flag (factor); waits re-poll with up to kBatch loads in flight, bounded.
__device__ __forceinline__ void backoff(unsigned& spins, bool progressed, unsigned* err, unsigned code, bool& give_up) {
  if (progressed) {
    spins = 0;
    return;
  }
  if (++spins > kSpinMax) {
    atomicOr(err, code);
    give_up = true;
    return;
  }
  __builtin_amdgcn_s_sleep(2);
}

// ILU numeric factor (scaler_ILU::factor, ILU_class.cpp:300-444).  Row i is zeroed, A's values
// loaded (amap, in storage order: a duplicate's last value wins, as the reference's row[] scatter
// does), then for every lower entry id in ascending order mult = row[id] / U(id,id) and
// row[idd] -= mult * U(id,idd) for the entries idd of row id's upper part that row i holds (two
// sorted lists merged).  The lane works on its own row with plain accesses and publishes it
// with agent-scope stores before the flag.
__global__ void __launch_bounds__(kSweepRows) k_ilu_factor(const int* __restrict__ ia, const int* __restrict__ ja,
                                                          const double* __restrict__ a, const int* __restrict__ amap,
                                                          const int* __restrict__ iaf, const int* __restrict__ jaf,
                                                          const int* __restrict__ dg, const int2* __restrict__ piv,
                                                          const int* __restrict__ perm, int nchunks, double* af,
                                                          unsigned* flags, unsigned epoch, unsigned* ticket,
                                                          unsigned* err) {
  const int lane = (int)threadIdx.x;
  bool give_up = false;
  while (!give_up) {
    const int t = take_ticket(ticket);
    if (t >= nchunks) break;
    const int i = perm[(size_t)t * kSweepRows + lane];
    const bool valid = i >= 0;
    int kc = 0, kd = 0, kb = 0, ke = 0;
    if (valid) {
      kb = iaf[i];
      kd = dg[i];
      ke = iaf[i + 1];
      for (int k = kb; k < ke; ++k) af[k] = 0.0;
      for (int ii = ia[i]; ii < ia[i + 1]; ++ii) af[amap[ii]] = a[ii];
      kc = kb;
    }
    // eliminate the lower entries in ascending order, each as soon as its pivot row is published
    // (rows finishing late are usually the last entries, so earlier ones overlap the wait); the
    // pivot-row range comes from piv (host-built) together with the flag poll
    int kk = kc;
    bool done = !valid;
    unsigned spins = 0;
    while (true) {
      bool fin = false, prog = false;
      if (!done) {
        while (kk < kd) {
          const int id = jaf[kk];
          const int2 pv = piv[kk];
          if (__hip_atomic_load(&flags[id], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) break;
          prog = true;
          const int ub = pv.x, uend = pv.y;
          const double pivot = ld_agent(&af[ub]);
          int jj[kFactorBatch];
          double uu[kFactorBatch];
          const int m0 = (uend - ub - 1 < kFactorBatch) ? uend - ub - 1 : kFactorBatch;
#pragma unroll
          for (int q = 0; q < kFactorBatch; ++q)
            if (q < m0) {
              jj[q] = jaf[ub + 1 + q];
              uu[q] = ld_agent(&af[ub + 1 + q]);
            }
          const double mult = af[kk] / pivot;
          af[kk] = mult;
          int p = kk + 1;
#pragma unroll
          for (int q = 0; q < kFactorBatch; ++q)
            if (q < m0) {
              const int idd = jj[q];
              while (p < ke && jaf[p] < idd) ++p;
              if (p < ke && jaf[p] == idd) af[p] = af[p] - mult * uu[q];
            }
          for (int c0 = ub + 1 + kFactorBatch; c0 < uend; c0 += kFactorBatch) {  // long pivot rows
#pragma unroll
            for (int q = 0; q < kFactorBatch; ++q)
              if (c0 + q < uend) {
                jj[q] = jaf[c0 + q];
                uu[q] = ld_agent(&af[c0 + q]);
              }
#pragma unroll
            for (int q = 0; q < kFactorBatch; ++q)
              if (c0 + q < uend) {
                const int idd = jj[q];
                while (p < ke && jaf[p] < idd) ++p;
                if (p < ke && jaf[p] == idd) af[p] = af[p] - mult * uu[q];
              }
          }
          ++kk;
        }
        fin = (kk == kd);
      }
      if (fin) {  // publish: agent-scope (write-through) stores, drained, then the flag
        for (int k = kb; k < ke; ++k) st_agent(&af[k], af[k]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&flags[i], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done = true;
      }
      if (__all(done)) break;
      backoff(spins, __ballot(fin || prog) != 0, err, 1u, give_up);
      if (give_up) break;
    }
  }
}

// The same factor with the lane's row held in LDS and the dependency waits batched.  Row i's
// kFacBatch next lower entries have their flags polled together (one round trip); for the ready
// prefix, every pivot and the first kFacU upper values of every pivot row are requested together
// (a second round trip), with the host-built positions tgt[] in row i that each upper value updates
// (-1: row i does not hold that column) -- no merge search.  Then the eliminations run in ascending
// order on the LDS image of the row (same operations, same order as k_ilu_factor: bit-identical).
// A 2D mesh row (<= 7 lower entries) waits two round trips instead of two per lower entry.
template <int B, int U>
__global__ void __launch_bounds__(kSweepRows) k_ilu_factor_lds(const int* __restrict__ ia, const double* __restrict__ a,
                                                              const int* __restrict__ amap, const int* __restrict__ iaf,
                                                              const int* __restrict__ jaf, const int* __restrict__ dg,
                                                              const int2* __restrict__ piv, const int* __restrict__ toff,
                                                              const signed char* __restrict__ tgt,
                                                              const int* __restrict__ perm, int nchunks, double* af,
                                                              unsigned* flags, unsigned epoch, unsigned* ticket,
                                                              unsigned* err) {
  __shared__ double rowv[kFacW * kSweepRows];
  const int lane = (int)threadIdx.x;
  double* my = rowv + lane;  // entry e of the lane's row at my[e * 64]
  bool give_up = false;
  while (!give_up) {
    const int t = take_ticket(ticket);
    if (t >= nchunks) break;
    const int i = perm[(size_t)t * kSweepRows + lane];
    const bool valid = i >= 0;
    int kb = 0, kd = 0, ke = 0;
    if (valid) {
      kb = iaf[i];
      kd = dg[i];
      ke = iaf[i + 1];
      for (int e = 0; e < ke - kb; ++e) my[e * kSweepRows] = 0.0;
      for (int ii = ia[i]; ii < ia[i + 1]; ++ii) my[(amap[ii] - kb) * kSweepRows] = a[ii];
    }
    int kk = kb;
    bool done = !valid;
    unsigned spins = 0;
    while (true) {
      bool fin = false, prog = false;
      if (!done && kk < kd) {
        const int nb = (kd - kk < B) ? kd - kk : B;
        int id[B], to[B];
        int2 pv[B];
        unsigned fl[B];
#pragma unroll
        for (int q = 0; q < B; ++q)
          if (q < nb) {
            id[q] = jaf[kk + q];
            pv[q] = piv[kk + q];
            to[q] = toff[kk + q];
          }
#pragma unroll
        for (int q = 0; q < B; ++q)
          if (q < nb) fl[q] = __hip_atomic_load(&flags[id[q]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int r = 0;
#pragma unroll
        for (int q = 0; q < B; ++q)
          if (q < nb && r == q && fl[q] == epoch) r = q + 1;
        if (r > 0) {
          prog = true;
          double pvt[B], uu[B][U];
          signed char tg[B][U];
#pragma unroll
          for (int q = 0; q < B; ++q)
            if (q < r) {
              pvt[q] = ld_agent(&af[pv[q].x]);
              const int m = pv[q].y - pv[q].x - 1;
#pragma unroll
              for (int u = 0; u < U; ++u)
                if (u < m) {
                  uu[q][u] = ld_agent(&af[pv[q].x + 1 + u]);
                  tg[q][u] = tgt[to[q] + u];
                }
            }
#pragma unroll
          for (int q = 0; q < B; ++q)
            if (q < r) {
              const int e0 = kk + q - kb;
              const double mult = my[e0 * kSweepRows] / pvt[q];
              my[e0 * kSweepRows] = mult;
              const int m = pv[q].y - pv[q].x - 1;
#pragma unroll
              for (int u = 0; u < U; ++u)
                if (u < m && tg[q][u] >= 0) my[tg[q][u] * kSweepRows] = my[tg[q][u] * kSweepRows] - mult * uu[q][u];
              for (int c0 = U; c0 < m; c0 += U) {  // long pivot rows
                double uc[U];
                signed char tc[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                  if (c0 + u < m) {
                    uc[u] = ld_agent(&af[pv[q].x + 1 + c0 + u]);
                    tc[u] = tgt[to[q] + c0 + u];
                  }
#pragma unroll
                for (int u = 0; u < U; ++u)
                  if (c0 + u < m && tc[u] >= 0) my[tc[u] * kSweepRows] = my[tc[u] * kSweepRows] - mult * uc[u];
              }
            }
          kk += r;
        }
      }
      if (!done && kk == kd) {  // publish: agent-scope (write-through) stores, drained, then the flag
        for (int e = 0; e < ke - kb; ++e) st_agent(&af[kb + e], my[e * kSweepRows]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&flags[i], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done = true;
        fin = true;
      }
      if (__all(done)) break;
      backoff(spins, __ballot(fin || prog) != 0, err, 1u, give_up);
      if (give_up) break;
    }
  }
}

// The same factor with one wavefront per row (rows wider than a lane can take in reasonable time:
// 3D mesh rows have up to 26 lower and 71 entries).  Each wavefront takes rows by ticket in
// forward level order, and requests its next ticket while the current row runs: the smallest
// ticket not yet finished is always some running wave's current row, whose pivots all carry
// smaller tickets, so the factor progresses with any number of resident waves (round 5 dealt rows
// round-robin to a grid assumed resident at once, which a concurrent kernel could break).  Per row: its image in LDS (entry e at w[e]); lane q polls
// the flag of lower entry q's pivot row until all are published; then, for every lower entry q,
// lane u holds U(j_q, .)'s u-th upper value and its position tgt[] in row i (-1: not held),
// requested together.  The eliminations run in ascending q: mult = w[q] / U(j_q, j_q), w[q] = mult,
// and every lane with a target subtracts mult * U at once (distinct targets; LDS in order within
// the wavefront) -- the operations of k_ilu_factor in the same order, so bit-identical.  NL: lower
// entries per row, at most; upper parts of at most 64 entries (host-checked).
template <int NL, bool GR, int WG = 4>
__global__ void __launch_bounds__(64 * WG) k_ilu_factor_wave(const int* __restrict__ ia, const double* __restrict__ a,
                                                         const int* __restrict__ amap, const int* __restrict__ iaf,
                                                         const int* __restrict__ dg, const int2* __restrict__ piv,
                                                         const int* __restrict__ jaf, const int* __restrict__ toff,
                                                         const signed char* __restrict__ tgt, const int* __restrict__ perm,
                                                         int nrows, int chunk, unsigned* ticket, double* af,
                                                         unsigned* flags, uint64_t* gF, unsigned epoch, unsigned* err) {
  __shared__ double s_row[WG][kFacW + 1];
  const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
  double* w = s_row[wv];
  // lane 0 takes the wave's tickets (the value is read only where it is needed: the next ticket's
  // round trip overlaps the current chunk).  A ticket is a chunk of `chunk` consecutive rows of the
  // order, done in order by the wave: one ticket per row made the single counter's device-scope
  // atomics (~7 ns each, serialised) the factor's bottleneck -- C4 11.2 -> 20.9 ms
  // one row: false when a dependency wait gave up
  auto row = [&](int x) -> bool {
    const int i = perm[x];
    const int kb = iaf[i], kd = dg[i], ke = iaf[i + 1];
    const int W = ke - kb, nl = kd - kb;
    for (int e = lane; e < W; e += 64) w[e] = 0.0;
    for (int ii = ia[i] + lane; ii < ia[i + 1]; ii += 64) w[amap[ii] - kb] = a[ii];
    // lane q: lower entry q's pivot row (flag, diagonal position, end of its upper part, targets)
    const bool low = lane < nl;
    const int pj = low ? jaf[kb + lane] : 0;
    const int2 pv = low ? piv[kb + lane] : make_int2(0, 0);
    const int to = low ? toff[kb + lane] : 0;
    unsigned spins = 0;
    bool ready = !low, give_up = false;
    double pvt = 1.0;
    while (true) {
      if (!ready) {
        if constexpr (GR)
          ready = load_granule(gF + 2 * (size_t)pv.x, epoch, pvt);  // the pivot's diagonal, self-validating
        else
          ready = __hip_atomic_load(&flags[pj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      }
      if (__all(ready)) break;
      backoff(spins, false, err, 4u, give_up);
      if (give_up) break;
    }
    if (give_up) return false;
    if constexpr (!GR) pvt = low ? ld_agent(&af[pv.x]) : 1.0;
    double uu[NL];
    int tg[NL];
    // GR: the upper values carry their own tags (stored in no particular order): all requested at
    // once, then the lane repeats its requests until every tag is this factor's (rare)
    bool okU = true;
    auto fetch_upper = [&](bool first) {
#pragma unroll
      for (int q = 0; q < NL; ++q) {
        if (first) {
          uu[q] = 0.0;
          tg[q] = -1;
        }
        if (q < nl) {
          const int px = __shfl(pv.x, q), m = __shfl(pv.y, q) - px - 1, tq = __shfl(to, q);  // (all lanes)
          if (lane < m) {
            if constexpr (GR) {
              const uint64_t* g = gF + 2 * ((size_t)px + 1 + lane);
              const uint64_t lo = __hip_atomic_load(const_cast<uint64_t*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const uint64_t hi = __hip_atomic_load(const_cast<uint64_t*>(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              okU = okU && (unsigned)(lo >> 32) == epoch && (unsigned)(hi >> 32) == epoch;
              uu[q] = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
            } else {
              uu[q] = ld_agent(&af[px + 1 + lane]);
            }
            if (first) tg[q] = tgt[tq + lane];
          }
        }
      }
    };
    fetch_upper(true);
    if constexpr (GR) {
      unsigned sp = 0;
      bool gu = false;
      while (!__all(okU)) {
        backoff(sp, false, err, 4u, gu);
        if (gu) return false;
        if (!okU) {
          okU = true;
          fetch_upper(false);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NL; ++q)
      if (q < nl) {
        const double mult = w[q] / __shfl(pvt, q);
        if (lane == 0) w[q] = mult;
        if (tg[q] >= 0) w[tg[q]] = w[tg[q]] - mult * uu[q];
      }
    if constexpr (GR) {
      // publish: the factor's values, and the diagonal + upper part as tagged granules (no drain)
      for (int e = lane; e < W; e += 64) af[kb + e] = w[e];
      for (int e = nl + lane; e < W; e += 64) store_granule(gF + 2 * ((size_t)kb + e), epoch, w[e]);
    } else {
      // publish: agent-scope (write-through) stores, drained, then the flag
      for (int e = lane; e < W; e += 64) st_agent(&af[kb + e], w[e]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(&flags[i], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
  };
  if (chunk > 0) {
    // per wave: lane 0 takes the wave's tickets (read only where needed: the next ticket's round
    // trip overlaps the current chunk); a ticket is `chunk` consecutive rows of the order, done in
    // order by the wave
    auto take = [&]() -> unsigned { return lane == 0 ? atomicAdd(ticket, 1u) : 0u; };
    unsigned tk = take();
    for (int x0 = (int)__shfl(tk, 0) * chunk; x0 < nrows; x0 = (int)__shfl(tk, 0) * chunk) {
      tk = take();  // the next chunk's ticket
      const int x1 = min(x0 + chunk, nrows);
      for (int x = x0; x < x1; ++x)
        if (!row(x)) return;
    }
  } else {
    // per workgroup (the default): a ticket is 4 consecutive rows of the order, one per wave, taken
    // by lane 0 of wave 0 one chunk ahead (a quarter of the device-scope atomics on the one counter:
    // at one per row they were the factor's bottleneck -- C4 20.9 ms against 11.2 ms without
    // tickets); the waves meet at a barrier per chunk
    __shared__ unsigned s_tk[2];
    __shared__ int s_bad;
    if (threadIdx.x == 0) {
      s_tk[0] = atomicAdd(ticket, 1u);
      s_bad = 0;
    }
    __syncthreads();
    int par = 0;
    for (unsigned t = s_tk[0]; (long long)t * WG < nrows; t = s_tk[par]) {
      if (threadIdx.x == 0) s_tk[par ^ 1] = atomicAdd(ticket, 1u);
      const int x = (int)t * WG + wv;
      if (x < nrows && !row(x) && lane == 0) s_bad = 1;
      __syncthreads();
      if (s_bad) return;
      par ^= 1;
    }
  }
}

// Triangular sweeps (scaler_ILU::solve, ILU_class.cpp:470-499).  Forward (unit L):
// y_i = b_i - sum_{k<diag} af_k y_jk; backward (U): x_i = (y_i - sum_{k>diag} af_k x_jk) / af_diag;
// the terms are subtracted one at a time in ascending column order.  The forward sweep fuses the
// CG-STAB prologue: pro 0 b = src; pro 1 pvec = res + beta*(pvec - omega*avbar)
// (accel_class.cpp:339-341); pro 2 svec = res - alpha*avbar (361-363), stored to p.
template <bool FWD, int PRO>
__global__ void __launch_bounds__(kSweepRows) k_sweep(const int* __restrict__ iaf, const int* __restrict__ jaf,
                                                     const int* __restrict__ dg, const double* __restrict__ af,
                                                     const int* __restrict__ perm, int nchunks,
                                                     const double* __restrict__ src, double* __restrict__ p,
                                                     const double* __restrict__ res, const double* __restrict__ avbar,
                                                     const CgsScalars* __restrict__ sc, const uint64_t* __restrict__ gin,
                                                     uint64_t* gout, double* __restrict__ out, unsigned epoch,
                                                     unsigned* ticket, unsigned* err) {
  const int lane = (int)threadIdx.x;
  bool give_up = false;
  while (!give_up) {
    const int t = take_ticket(ticket);
    if (t >= nchunks) break;
    const int i = perm[(size_t)t * kSweepRows + lane];
    const bool valid = i >= 0;
    double acc = 0.0;
    int k = 0, ke = 0, kd = 0;
    if (valid) {
      if (FWD) {
        if (PRO == 0) {
          acc = src[i];
        } else if (PRO == 1) {
          acc = res[i] + sc->beta * (p[i] - sc->omega * avbar[i]);
          p[i] = acc;
        } else {
          acc = res[i] - sc->alpha * avbar[i];
          p[i] = acc;
        }
      } else {
        acc = granule_value(gin + 2 * (size_t)i);
      }
      kd = dg[i];
      k = FWD ? iaf[i] : kd + 1;
      ke = FWD ? kd : iaf[i + 1];
    }
    bool done = !valid;
    unsigned spins = 0;
    while (true) {
      bool fin = false, prog = false;
      if (!done) {
        while (k < ke) {
          int jb[kBatch];
          const int m = (ke - k < kBatch) ? ke - k : kBatch;
#pragma unroll
          for (int q = 0; q < kBatch; ++q) jb[q] = (q < m) ? jaf[k + q] : 0;
          uint64_t lo[kBatch], hi[kBatch];
#pragma unroll
          for (int q = 0; q < kBatch; ++q)
            if (q < m) {
              lo[q] = __hip_atomic_load(gout + 2 * (size_t)jb[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              hi[q] = __hip_atomic_load(gout + 2 * (size_t)jb[q] + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          int c = 0;
          bool blocked = false;
#pragma unroll
          for (int q = 0; q < kBatch; ++q)
            if (q < m && !blocked) {
              if ((unsigned)(lo[q] >> 32) != epoch || (unsigned)(hi[q] >> 32) != epoch) {
                blocked = true;
              } else {
                acc -= af[k + q] * __longlong_as_double((long long)((hi[q] << 32) | (lo[q] & 0xffffffffull)));
                ++c;
              }
            }
          k += c;
          prog |= (c > 0);
          if (blocked) break;
        }
        fin = (k == ke);
      }
      if (fin) {
        if (!FWD) acc = acc / af[kd];
        if (!FWD) out[i] = acc;
        store_granule(gout + 2 * (size_t)i, epoch, acc);
        done = true;
      }
      if (__all(done)) break;
      backoff(spins, __ballot(fin || prog) != 0, err, FWD ? 2u : 4u, give_up);
      if (give_up) break;
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

// The forward sweeps' CG-STAB prologues as a vector pass (MMX_CGS_UNFUSE): MODE 1 p = res + beta
// (p - omega avbar), MODE 2 s = res - alpha avbar -- the operations of the fused forms in
// chain_sweep.hip / k_sweep, so the sweep that follows reads one operand
template <int MODE>
__global__ void __launch_bounds__(kVecBlock) k_cgs_pro(int n, const double* __restrict__ res,
                                                      const double* __restrict__ avbar, double* __restrict__ out,
                                                      const CgsScalars* __restrict__ sc) {
  const double beta = sc->beta, omega = sc->omega, alpha = sc->alpha;
  for (int i = blockIdx.x * kVecBlock + threadIdx.x; i < n; i += gridDim.x * kVecBlock) {
    if constexpr (MODE == 1)
      out[i] = res[i] + beta * (out[i] - omega * avbar[i]);
    else
      out[i] = res[i] - alpha * avbar[i];
  }
}

// a sweep's result from its granules {tag | lo, tag | hi} (every row publishes one)
__global__ void __launch_bounds__(kVecBlock) k_gran_extract(int n, const uint64_t* __restrict__ g, double* __restrict__ out) {
  for (int i = blockIdx.x * kVecBlock + threadIdx.x; i < n; i += gridDim.x * kVecBlock) {
    const uint64_t lo = g[2 * (size_t)i] & 0xffffffffull, hi = g[2 * (size_t)i + 1] & 0xffffffffull;
    out[i] = __longlong_as_double((long long)((hi << 32) | lo));
  }
}
void launch_gran_extract(int n, const uint64_t* g, double* out, hipStream_t st) {
  hipLaunchKernelGGL(k_gran_extract, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, n, g, out);
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

void launch_spmv2(int epi, int nblk, const int4* desc, const int* ia, const int* ja, const double* a, const double* x,
                  double* y, const double* e1, double* partials, hipStream_t st) {
  if (nblk <= 0) return;
  const dim3 g((unsigned)((nblk + 7) / 8 * 8)), bl(kSpmvBlock);
  if (epi == 0)
    hipLaunchKernelGGL(k_spmv2<0>, g, bl, 0, st, desc, nblk, ia, ja, a, x, y, e1, partials);
  else if (epi == 1)
    hipLaunchKernelGGL(k_spmv2<1>, g, bl, 0, st, desc, nblk, ia, ja, a, x, y, e1, partials);
  else
    hipLaunchKernelGGL(k_spmv2<2>, g, bl, 0, st, desc, nblk, ia, ja, a, x, y, e1, partials);
}

void launch_ilu_factor_lds(const int* ia, const double* a, const int* amap, const int* iaf, const int* jaf, const int* dg,
                           const int2* piv, const int* toff, const signed char* tgt, const int* perm, int nchunks,
                           double* af, unsigned* flags, unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st) {
  if (nchunks <= 0) return;
  const int grid = nchunks < sweep_grid() ? nchunks : sweep_grid();
  hipLaunchKernelGGL((k_ilu_factor_lds<8, 8>), dim3(grid), dim3(kSweepRows), 0, st, ia, a, amap, iaf, jaf, dg, piv, toff,
                     tgt, perm, nchunks, af, flags, epoch, ticket, err);
}

// tickets of the wave factor: 0 = per workgroup, 4 rows (one per wave); n > 0 = per wave, n
// consecutive rows (MMX_FAC_CHUNK overrides)
constexpr int kFacWaveChunk = 0;
// (the grid's size is a throughput choice only: the tickets need no co-residency)
static int factor_wg() {  // waves per workgroup of the wave factor (MMX_FAC_WG: 4 or 8)
  static const int v = [] {
    const char* e = getenv("MMX_FAC_WG");
    return (e && atoi(e) == 8) ? 8 : 4;
  }();
  return v;
}
int ilu_factor_wave_grid() {
  static int g = [] {
    int dev = 0, cus = 0, nb = 0, nb2 = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (factor_wg() == 8) {
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_ilu_factor_wave<kFacWaveNL, true, 8>, 512, 0);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb2, k_ilu_factor_wave<kFacWaveNL, false, 8>, 512, 0);
    } else {
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_ilu_factor_wave<kFacWaveNL, true>, 256, 0);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb2, k_ilu_factor_wave<kFacWaveNL, false>, 256, 0);
    }
    nb = nb < nb2 ? nb : nb2;
    nb = nb < 1 ? 1 : (nb > 8 ? 8 : nb);
    return (cus > 0 ? cus : 1) * nb;
  }();
  return g;
}

void launch_ilu_factor_wave(const int* ia, const double* a, const int* amap, const int* iaf, const int* dg,
                            const int2* piv, const int* jaf, const int* toff, const signed char* tgt, const int* perm,
                            int nrows, double* af, unsigned* flags, uint64_t* gF, unsigned epoch, unsigned* ticket,
                            unsigned* err, hipStream_t st) {
  if (nrows <= 0) return;
  // one CU's worth of waves per CU and occupancy slot; rows by ticket (*ticket zeroed by the caller),
  // MMX_FAC_CHUNK rows per ticket
  static const int chunk = [] {
    const char* e = getenv("MMX_FAC_CHUNK");
    return e ? std::max(0, atoi(e)) : kFacWaveChunk;
  }();
  const int wg = chunk > 0 ? 4 : factor_wg();
  const int per = wg * std::max(chunk, 1);  // rows a workgroup takes per round of tickets
  const int blocks = std::min(ilu_factor_wave_grid(), (nrows + per - 1) / per);
#define MMX_FACW(G, W)                                                                                           \
  hipLaunchKernelGGL((k_ilu_factor_wave<kFacWaveNL, G, W>), dim3(blocks), dim3(64 * W), 0, st, ia, a, amap, iaf, dg, \
                     piv, jaf, toff, tgt, perm, nrows, chunk, ticket, af, flags, gF, epoch, err)
  if (gF && wg == 8)
    MMX_FACW(true, 8);
  else if (gF)
    MMX_FACW(true, 4);
  else if (wg == 8)
    MMX_FACW(false, 8);
  else
    MMX_FACW(false, 4);
#undef MMX_FACW
}

// one wavefront per row (sparse.cpp sfac; the host loops this replaces): lane q takes lower entry q
// (and q + 64, ...): its pivot range; with toff / tgt its offset (rowTot[i] + an exclusive scan of
// the lower entries' pivot upper lengths across the lanes) and a merge walk of row i's sorted
// columns against the pivot row's upper part, as scaler_ILU::factor's target search
__global__ void __launch_bounds__(256) k_fac_prep(int n, const int* __restrict__ iaf, const int* __restrict__ jaf,
                                                  const int* __restrict__ dg, const long long* __restrict__ rowTot,
                                                  int2* __restrict__ piv, int* __restrict__ toff,
                                                  signed char* __restrict__ tgt) {
  const int i = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6), lane = (int)threadIdx.x & 63;
  if (i >= n) return;
  const int rb = iaf[i], re = iaf[i + 1], d = dg[i];
  for (int k = d + lane; k < re; k += 64) {  // diagonal and upper entries
    piv[k] = make_int2(0, 0);
    if (toff) toff[k] = 0;
  }
  long long base = rowTot[i];
  for (int k0 = rb; k0 < d; k0 += 64) {
    const int k = k0 + lane;
    const bool low = k < d;
    int dj = 0, ej = 0;
    if (low) {
      const int j = jaf[k];
      dj = dg[j];
      ej = iaf[j + 1];
      piv[k] = make_int2(dj, ej);
    }
    if (!toff) continue;
    const long long len = low ? (long long)(ej - dj - 1) : 0;
    long long inc = len;  // inclusive scan over the lanes
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const long long o = __shfl_up(inc, sh);
      if (lane >= sh) inc += o;
    }
    const long long t = base + inc - len;
    base += __shfl(inc, 63);
    if (!low) continue;
    toff[k] = (int)t;
    int f = rb;
    for (int pp = dj + 1; pp < ej; ++pp) {
      const int c = jaf[pp];
      while (f < re && jaf[f] < c) ++f;
      tgt[t + (pp - dj - 1)] = (f < re && jaf[f] == c) ? (signed char)(f - rb) : (signed char)-1;
    }
  }
}
void launch_fac_prep(int n, const int* iaf, const int* jaf, const int* dg, const long long* rowTot, int2* piv,
                     int* toff, signed char* tgt, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fac_prep, dim3((n + 3) / 4), dim3(256), 0, st, n, iaf, jaf, dg, rowTot, piv, toff, tgt);
}

// Test hook (mmx_occupy): `blocks` workgroups of 1024 lanes with 64 KB of LDS each that hold their
// CUs for `ms` milliseconds (the 100 MHz real-time counter; every wave leaves at the deadline) --
// a concurrent kernel that keeps part of the chip away from the solver's kernels.
__global__ void __launch_bounds__(1024) k_occupy(unsigned long long ticks, double* sink) {
  extern __shared__ double lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (double)threadIdx.x;
  double acc = 0.0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    acc += lds[(threadIdx.x * 7) & 1023];
  }
  if (acc < 0.0) sink[threadIdx.x] = acc;  // never true: keeps the loop's reads
}
void launch_occupy(int blocks, double ms, double* sink, hipStream_t st) {
  if (blocks <= 0 || !(ms > 0)) return;
  const unsigned long long ticks = (unsigned long long)(ms * 1e5);  // 100 MHz
  hipLaunchKernelGGL(k_occupy, dim3(blocks), dim3(1024), 64 * 1024, st, ticks, sink);
}

void launch_ilu_factor(const int* ia, const int* ja, const double* a, const int* amap, const int* iaf, const int* jaf,
                       const int* dg, const int2* piv, const int* perm, int nchunks, double* af, unsigned* flags,
                       unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st) {
  if (nchunks <= 0) return;
  const int grid = nchunks < sweep_grid() ? nchunks : sweep_grid();
  hipLaunchKernelGGL(k_ilu_factor, dim3(grid), dim3(kSweepRows), 0, st, ia, ja, a, amap, iaf, jaf, dg, piv, perm, nchunks,
                     af, flags, epoch, ticket, err);
}

void launch_sweep(bool fwd, int pro, const int* iaf, const int* jaf, const int* dg, const double* af, const int* perm,
                  int nchunks, const double* src, double* p, const double* res, const double* avbar, const CgsScalars* sc,
                  const uint64_t* gin, uint64_t* gout, double* out, unsigned epoch, unsigned* ticket, unsigned* err,
                  hipStream_t st) {
  if (nchunks <= 0) return;
  const dim3 g(nchunks < sweep_grid() ? nchunks : sweep_grid()), b(kSweepRows);
#define MMX_SWEEP(F, P)                                                                                              \
  hipLaunchKernelGGL((k_sweep<F, P>), g, b, 0, st, iaf, jaf, dg, af, perm, nchunks, src, p, res, avbar, sc, gin, gout, \
                     out, epoch, ticket, err)
  if (!fwd)
    MMX_SWEEP(false, 0);
  else if (pro == 0)
    MMX_SWEEP(true, 0);
  else if (pro == 1)
    MMX_SWEEP(true, 1);
  else
    MMX_SWEEP(true, 2);
#undef MMX_SWEEP
}

void launch_cgs_init(int mode, int n, const double* b, double* x, double* res, double* res0, double* p, double* avbar,
                     int copy_res0, double* partials, hipStream_t st) {
  hipLaunchKernelGGL(k_cgs_init, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, mode, n, b, x, res, res0, p, avbar,
                     copy_res0, partials);
}

void launch_dot_into(int n, const double* x, const double* y, double* partials, hipStream_t st) {
  hipLaunchKernelGGL(k_dot_into, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, n, x, y, partials);
}

void launch_cgs_pro(int mode, int n, const double* res, const double* avbar, double* out, const CgsScalars* sc,
                    hipStream_t st) {
  if (mode == 1)
    hipLaunchKernelGGL(k_cgs_pro<1>, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, n, res, avbar, out, sc);
  else
    hipLaunchKernelGGL(k_cgs_pro<2>, dim3(vec_grid(n)), dim3(kVecBlock), 0, st, n, res, avbar, out, sc);
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

// Streaming copy (measurement utility: the achievable HBM ceiling the bench reports beside the
// 8 TB/s spec), 16 B per lane per access.  Variant 0: grid-stride, 4 accesses in flight per lane,
// nontemporal hints, 8 workgroups per CU; 1: one 16-B element per lane, one pass (n2/256
// workgroups), default policy; 2: 4 consecutive-by-stride elements per lane, one pass, default
// policy.
template <int VAR>
__global__ void __launch_bounds__(256) k_stream_copy(long long n2, const v2d_t* __restrict__ src,
                                                     v2d_t* __restrict__ dst) {
  if constexpr (VAR == 0) {
    const long long stride = (long long)gridDim.x * 256;
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n2; i += 4 * stride) {
      v2d_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
      for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + i + u * stride);
    }
    for (; i < n2; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
  } else if constexpr (VAR == 1) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n2) dst[i] = src[i];
  } else if constexpr (VAR >= 3) {
    // counter calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are calibrated only for
    // 16-B streaming reads and stores): the access widths of the ADMM kernels over n = 2 n2 doubles,
    // one access group per lane; reads keep their value live through a store that never happens
    const double* sd = reinterpret_cast<const double*>(src);
    double* dd = reinterpret_cast<double*>(dst);
    const long long n = 2 * n2, i = (long long)blockIdx.x * 256 + threadIdx.x;
    double a = 0.0;
    if constexpr (VAR == 3) {  // 8 B per lane, coalesced (the 3D prox's Bkinv rows)
      if (i < n) a = sd[i];
    } else if constexpr (VAR == 4) {  // a 24-B record per lane as three 8-B loads (slot terms)
      if (i < n / 3) a = sd[3 * i] + sd[3 * i + 1] + sd[3 * i + 2];
    } else if constexpr (VAR == 5) {  // 16 B per lane, coalesced (the calibrated case)
      if (i < n2) {
        const v2d_t v = src[i];
        a = v.x + v.y;
      }
    } else if constexpr (VAR == 6) {  // 8-B stores per lane, coalesced
      if (i < n) dd[i] = (double)i;
    } else if constexpr (VAR == 7) {  // 8-B nontemporal stores per lane (the 3D prox's new Bkinv)
      if (i < n) __builtin_nontemporal_store((double)i, dd + i);
    } else {  // a random 24-B record per lane (the x-update's gathers at their worst)
      const long long nrec = n / 3;
      if (i < nrec) {
        const long long r = (long long)(((unsigned long long)i * 2654435761ull) % (unsigned long long)nrec);
        a = sd[3 * r] + sd[3 * r + 1] + sd[3 * r + 2];
      }
    }
    if (a == -7.25e300) dd[i] = a;
  } else {
    const long long base = (long long)blockIdx.x * 1024 + threadIdx.x;
    v2d_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (base + u * 256 < n2) v[u] = src[base + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (base + u * 256 < n2) dst[base + u * 256] = v[u];
  }
}

void launch_stream_copy(int variant, long long n2, const double* src, double* dst, hipStream_t st) {
  const v2d_t* s2 = reinterpret_cast<const v2d_t*>(src);
  v2d_t* d2 = reinterpret_cast<v2d_t*>(dst);
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_stream_copy<0>, dim3(256 * 8), dim3(256), 0, st, n2, s2, d2); break;
    case 1: hipLaunchKernelGGL(k_stream_copy<1>, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, st, n2, s2, d2); break;
    case 2: hipLaunchKernelGGL(k_stream_copy<2>, dim3((unsigned)((n2 + 1023) / 1024)), dim3(256), 0, st, n2, s2, d2); break;
    case 3: hipLaunchKernelGGL(k_stream_copy<3>, dim3((unsigned)((2 * n2 + 255) / 256)), dim3(256), 0, st, n2, s2, d2); break;
    case 4: hipLaunchKernelGGL(k_stream_copy<4>, dim3((unsigned)((2 * n2 / 3 + 255) / 256)), dim3(256), 0, st, n2, s2, d2); break;
    case 5: hipLaunchKernelGGL(k_stream_copy<5>, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, st, n2, s2, d2); break;
    case 6: hipLaunchKernelGGL(k_stream_copy<6>, dim3((unsigned)((2 * n2 + 255) / 256)), dim3(256), 0, st, n2, s2, d2); break;
    case 7: hipLaunchKernelGGL(k_stream_copy<7>, dim3((unsigned)((2 * n2 + 255) / 256)), dim3(256), 0, st, n2, s2, d2); break;
    default: hipLaunchKernelGGL(k_stream_copy<8>, dim3((unsigned)((2 * n2 / 3 + 255) / 256)), dim3(256), 0, st, n2, s2, d2); break;
  }
}

}  // namespace mmx

// the layout word this kernel object was compiled with (layout.h; checked by the host at create)
extern "C" unsigned mmx_layout_sparse(void) { return mmx::kLayoutWord; }
