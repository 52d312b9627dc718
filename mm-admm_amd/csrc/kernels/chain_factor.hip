// chain_factor.hip -- the numeric ILU(0) factor (scaler_ILU::factor, lib/LASolver/ILU_class.cpp:
// 300-527) on the chain/band schedule of the forward sweep (host/chain_sched.h,
// build_factor_schedule) for gfx950.
//
// One workgroup runs one band (64 chains, one per lane) at a time, four wavefronts: a compute
// wave; a loader DMA-ing each iteration's stage (the row's initial values, the LDS indices of its
// update and pivot values, its metadata) into LDS; a storer that writes the compute wave's finished
// rows (left in an LDS output buffer) to af and to the global granules; and an importer that copies
// the diagonal + upper part of rows of other bands (or rows too old for the ring) from their
// self-validating global granules into LDS import slots.  The storer's lanes take consecutive
// entries of a row, so a store instruction touches a few cache lines instead of one per lane
// (the compute wave storing its own rows spent ~80% of an iteration issuing them).
//
// Row i at iteration t, target by target (ascending column e): w_e = a_e, then for every lower
// entry q < e whose pivot row j_q holds column col(e) above its diagonal, in ascending q,
// w_e -= m_q * U(j_q, col e); a lower entry then becomes m_e = w_e / U(j_e, j_e).  Those are the
// reference's operations in the reference's order for every entry (IKJ: pivot q updates its targets
// before pivot q + 1 is divided), so the factor is bit-identical to k_ilu_factor_lds and to the
// reference.  The row's diagonal and upper part go to the lane's LDS ring (kFacWU cells per row)
// and to the global granules {epoch:32, half:32} x 2 for other bands; all entries to af.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparse_kernels.h"

#ifndef MMX_FAC_GRAN_B128
#define MMX_FAC_GRAN_B128 1  // the storer's granules as one 16-byte store each (n = 2 M factor 12.46 -> 11.4 ms; 0: two 8-byte atomic stores)
#endif
namespace mmx {
namespace {

#define MMX_LDS __attribute__((address_space(3)))

// = host/chain_sched.h
constexpr int kWF = 18, kNL = 9, kWU = 14, kNSC = 128, kImpRows = 384, kRMax = 4;
constexpr int fslot(int e, int q) { return (e <= kNL ? e * (e - 1) / 2 : kNL * (kNL - 1) / 2 + (e - kNL) * kNL) + q; }
constexpr int kNUpd = fslot(kWF, 0);
constexpr int DL = 2;                         // stages
constexpr int kValChunks = kWF / 2;           // 16-B chunks of a row's initial values
constexpr int kCodeChunks = kNSC / 8;         // 16-B chunks of its 16-bit LDS indices
constexpr int kDep = 1 + 64 * (kRMax + 1) * kWU + kImpRows * kWU;
constexpr unsigned kSpinMax = 1u << 22;
constexpr int NI = kValChunks + kCodeChunks + 3;  // DMA instructions per stage
constexpr int LAG = 1;
#ifndef MMX_FAC_IMP_Q
#define MMX_FAC_IMP_Q 1  // n = 2 M: 1 12.2 ms, 2 15.4 ms, 4 18.2 ms (the extra polls only add traffic)
#endif
constexpr int kFacImpQ = MMX_FAC_IMP_Q;  // imports each importer lane polls per round

template <typename T>
__device__ __forceinline__ unsigned lds_off(T* p) {
  return (unsigned)(size_t)(MMX_LDS T*)p;
}
__device__ __forceinline__ int lds_read(const int* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_off(p)) : "memory");
  return v;
}
__device__ __forceinline__ void lds_write(int* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_off(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void dma16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (MMX_LDS void*)lds_base, 16, 0, 0);
}
__device__ __forceinline__ void dma4(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (MMX_LDS void*)lds_base, 4, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ double join_words(uint32_t lo, uint32_t hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }
// MMX_FAC_FINE (timing experiment, dev builds only): per-phase cycles of band 0's row compute
#ifdef MMX_FAC_FINE
#define FAC_STAMP(k)                                          \
  do {                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
    const unsigned long long c_ = clk();                      \
    if (b == 0 && lane == 0) fine[k] += c_ - fineLast;        \
    fineLast = c_;                                            \
  } while (0)
#else
#define FAC_STAMP(k) \
  do {               \
  } while (0)
#endif
__device__ __forceinline__ bool aborted(unsigned* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ bool spin(unsigned& spins, unsigned* err, unsigned code) {
  if ((++spins & 255u) == 0 && aborted(err)) return false;
  if (spins > kSpinMax) {
    atomicOr(err, code);
    return false;
  }
  __builtin_amdgcn_s_sleep(1);
  return true;
}

__global__ void __launch_bounds__(256) k_chain_factor(FactorArgs fa, double* __restrict__ af, uint64_t* gU,
                                                      unsigned epoch, unsigned* ticket, unsigned* err) {
  __shared__ double s_val[DL * kWF * 64];     // [stage][chunk][lane][2]
  __shared__ uint16_t s_code[DL * kNSC * 64];  // [stage][chunk][lane][8]
  __shared__ int s_meta[DL * 3 * 64];          // [stage][meta | kb | impNeed][lane]
  __shared__ double s_dep[kDep];               // [0] = 0, lane rings, import slots
  __shared__ double s_out[2 * kWF * 64];      // [buffer][entry][lane]: the finished rows
  __shared__ int s_oinfo[2 * 2 * 64];          // [buffer][kb | W, nlow, flags][lane]
  __shared__ int s_tag[DL];
  __shared__ int s_prog, s_band, s_impDone, s_outDone;

  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int R = fa.R;
  const int impBase = 1 + 64 * (R + 1) * kWU;

  while (true) {
    if (tid == 0) {
      const unsigned tk = atomicAdd(ticket, 1u);
      s_band = tk < (unsigned)fa.nbands ? fa.bandOrder[tk] : fa.nbands;
      s_prog = 0;
      s_impDone = 0;
      s_outDone = 0;
      s_dep[0] = 0.0;
    }
    if (tid < DL) s_tag[tid] = -1;
    __syncthreads();
    const int b = s_band;
    if (b >= fa.nbands) break;
    const bool skip = aborted(err);
    const int sb = fa.bandSlot[b], T = fa.bandT[b];
    const int g = b * 64 + lane;
    int len = fa.laneLen[g], skew = fa.laneSkew[g];
    asm volatile("" : "+v"(len), "+v"(skew));

    if (skip) {
    } else if (wave == 0) {
      // ---------------- compute ----------------
      wait_vm<0>();
      bool ok = true;
      int seen = 0;
      const unsigned long long c0 = fa.prof ? clk() : 0;
      unsigned long long cst = 0, cim = 0;
#ifdef MMX_FAC_FINE
      unsigned long long fine[6] = {0, 0, 0, 0, 0, 0}, fineLast = 0;
#endif
      for (int t = 0; t < T && ok; ++t) {
        const int st = t & (DL - 1);
        {  // the stage
          unsigned spins = 0;
          const unsigned long long w0 = fa.prof ? clk() : 0;
          while (lds_read(&s_tag[st]) != t)
            if (!(ok = spin(spins, err, 8u))) break;
          if (fa.prof) cst += clk() - w0;
          if (!ok) break;
        }
        const int* sm = s_meta + st * 3 * 64;
        const int meta = sm[lane], kb = sm[64 + lane];
        const int need = __builtin_amdgcn_readfirstlane(sm[128 + lane]);
        if (need >= 0 && seen <= need) {  // imports this iteration reads
          unsigned spins = 0;
          const unsigned long long i0 = fa.prof ? clk() : 0;
          while ((seen = lds_read(&s_impDone)) <= need)
            if (!(ok = spin(spins, err, 16u))) break;
          if (fa.prof) cim += clk() - i0;
          if (!ok) break;
        }
        const int p = t - skew;
        if (t >= 2 && lds_read(&s_outDone) < t - 1) {  // the output buffer of iteration t - 2 drained
          unsigned spins = 0;
          while (lds_read(&s_outDone) < t - 1)
            if (!(ok = spin(spins, err, 128u))) break;
          if (!ok) break;
        }
        if (!(p >= 0 && p < len && (meta >> 16))) s_oinfo[((t & 1) * 2 + 1) * 64 + lane] = 0;
        if (p >= 0 && p < len && (meta >> 16)) {
#ifdef MMX_FAC_FINE
          fineLast = clk();
#endif
          const int W = meta & 0xFF, nlow = (meta >> 8) & 0xFF;
          const double* sv = s_val + st * kWF * 64;
          const uint16_t* sc = s_code + st * kNSC * 64;
          double a[kWF];
#pragma unroll
          for (int c = 0; c < kValChunks; ++c) {
            const double2 v = *reinterpret_cast<const double2*>(sv + (c * 64 + lane) * 2);
            a[2 * c] = v.x;
            a[2 * c + 1] = v.y;
          }
          uint16_t cd[kNSC];
#pragma unroll
          for (int c = 0; c < kCodeChunks; ++c) {
            const uint4 v = *reinterpret_cast<const uint4*>(sc + (c * 64 + lane) * 8);
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              cd[c * 8 + 2 * k] = (uint16_t)(w4[k] & 0xFFFFu);
              cd[c * 8 + 2 * k + 1] = (uint16_t)(w4[k] >> 16);
            }
          }
          // every gather issued before the arithmetic, in one batch (one wait instead of one per
          // value), and the updates branch-free: an absent update (code 0) reads the zero cell and
          // its result is discarded by a select, so no sum sees it
          FAC_STAMP(0);
          double piv[kNL], uv[kNUpd];
#pragma unroll
          for (int q = 0; q < kNL; ++q) piv[q] = s_dep[cd[kNUpd + q]];
#pragma unroll
          for (int k = 0; k < kNUpd; ++k) uv[k] = s_dep[cd[k]];
          FAC_STAMP(1);
          double m[kNL], res[kWF];
#pragma unroll
          for (int e = 0; e < kWF; ++e) {
            double acc = a[e];
#pragma unroll
            for (int q = 0; q < (e < kNL ? e : kNL); ++q) {
              const double t = acc - m[q] * uv[fslot(e, q)];
              acc = (cd[fslot(e, q)] != 0) ? t : acc;
            }
            if (e < kNL) {
              m[e] = acc / piv[e];  // used only when e is a lower entry (e < nlow)
              res[e] = (e < nlow) ? m[e] : acc;
            } else {
              res[e] = acc;
            }
          }
          FAC_STAMP(2);
          // the row: the diagonal + upper part to the ring; every entry to the output buffer, from
          // where the storer writes af and the granules
          const int rs = 1 + (lane * (R + 1) + (p & (R - 1))) * kWU;
#pragma unroll
          for (int e = 0; e < kWF; ++e)
            if (e < W && e >= nlow) s_dep[rs + e - nlow] = res[e];
          const int ob = t & 1;
#pragma unroll
          for (int e = 0; e < kWF; ++e) s_out[(ob * kWF + e) * 64 + lane] = res[e];
          s_oinfo[(ob * 2) * 64 + lane] = kb;
          s_oinfo[(ob * 2 + 1) * 64 + lane] = (meta & 0xFFFF) | (((meta >> 17) & 1) << 16) | (1 << 17);
          FAC_STAMP(3);
        }
        if (lane == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          lds_write(&s_prog, t + 1);
        }
      }
      if (fa.prof && lane == 0) {
        const unsigned long long tot = clk() - c0;
        atomicAdd(fa.prof + 0, tot);
        atomicAdd(fa.prof + 1, cst);
        atomicAdd(fa.prof + 2, cim);
        atomicAdd(fa.prof + 3, (unsigned long long)T);
        atomicAdd(fa.prof + 4, 1ull);
#ifdef MMX_FAC_FINE
        for (int k = 0; k < 4; ++k) atomicAdd(fa.prof + 6 + k, fine[k]);
#endif
        if (b < 16) {  // the first bands (2D: the grid-line bands, the critical path)
          atomicAdd(fa.prof + 320 + 4 * b, tot);
          atomicAdd(fa.prof + 321 + 4 * b, cst);
          atomicAdd(fa.prof + 322 + 4 * b, cim);
          atomicAdd(fa.prof + 323 + 4 * b, (unsigned long long)T);
        }
      }
    } else if (wave == 1) {
      // ---------------- loader (every stage) ----------------
      int nextPub = 0;
      bool ok = true;
      for (int t = 0; t < T && ok; ++t) {
        const int st = t & (DL - 1);
        if (lds_read(&s_prog) < t - DL + 1) {  // slot busy: publish what is in flight, then wait
          wait_vm<0>();
          for (; nextPub < t; ++nextPub)
            if (lane == 0) lds_write(&s_tag[nextPub & (DL - 1)], nextPub);
          unsigned spins = 0;
          while (lds_read(&s_prog) < t - DL + 1)
            if (!(ok = spin(spins, err, 32u))) break;
          if (!ok) break;
        }
        const size_t slot = (size_t)(sb + t);
        const double* gv = fa.val + slot * kWF * 64;
#pragma unroll
        for (int c = 0; c < kValChunks; ++c) dma16(gv + (c * 64 + lane) * 2, s_val + st * kWF * 64 + c * 128);
        const uint16_t* gc = fa.code + slot * kNSC * 64;
#pragma unroll
        for (int c = 0; c < kCodeChunks; ++c) dma16(gc + (c * 64 + lane) * 8, s_code + st * kNSC * 64 + c * 512);
        int* sm = s_meta + st * 3 * 64;
        dma4(fa.meta + slot * 64 + lane, sm);
        dma4(fa.rowStart + slot * 64 + lane, sm + 64);
        dma4(fa.impNeed + slot, sm + 128);  // the same word in every lane
        if (t - nextPub + 1 > LAG) {
          wait_vm<NI * LAG>();
          for (; nextPub <= t - LAG; ++nextPub)
            if (lane == 0) lds_write(&s_tag[nextPub & (DL - 1)], nextPub);
        }
      }
      wait_vm<0>();
      if (ok)
        for (; nextPub < T; ++nextPub)
          if (lane == 0) lds_write(&s_tag[nextPub & (DL - 1)], nextPub);
    } else if (wave == 2) {
      // ---------------- storer ----------------
      // iteration t's rows: 64 x kWF (row, entry) pairs, lane l of pass c taking pair c 64 + l
      // (row (c 64 + l) / kWF): consecutive lanes write consecutive entries of a row
      const uint64_t tag = (uint64_t)epoch << 32;
      // (byte offsets into gU: factor positions < 2^27)
      const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(gU, 0, 0x7fffffff, 0x00020000);
      bool ok = true;
      for (int t = 0; t < T && ok; ++t) {
        unsigned spins = 0;
        while (lds_read(&s_prog) <= t)
          if (!(ok = spin(spins, err, 128u))) break;
        if (!ok) break;
        const int ob = t & 1;
#pragma unroll 3
        for (int c = 0; c < kWF; ++c) {
          const int v = c * 64 + lane, r = v / kWF, e = v - r * kWF;
          const int kb = s_oinfo[(ob * 2) * 64 + r], info = s_oinfo[(ob * 2 + 1) * 64 + r];
          const int W = info & 0xFF, nlow = (info >> 8) & 0xFF;
          if ((info >> 17) && e < W) {
            const double x = s_out[(ob * kWF + e) * 64 + r];
            af[kb + e] = x;
            if (e >= nlow && ((info >> 16) & 1)) {  // some band imports this row
              const uint64_t bits = (uint64_t)__double_as_longlong(x);
              if constexpr (MMX_FAC_GRAN_B128) {  // one 16-byte store, agent-scope policy (chain_sweep.hip)
                typedef unsigned v4u __attribute__((ext_vector_type(4)));
                const v4u d = {(unsigned)bits, epoch, (unsigned)(bits >> 32), epoch};
                __builtin_amdgcn_raw_buffer_store_b128(d, grs, (kb + e) * 16, 0, 16);
              } else {
                __hip_atomic_store(gU + 2 * (size_t)(kb + e), tag | (bits & 0xffffffffull), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(gU + 2 * (size_t)(kb + e) + 1, tag | (bits >> 32), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
              }
            }
          }
        }
        if (lane == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          lds_write(&s_outDone, t + 1);
        }
      }
    } else {
      // ---------------- importer ----------------
      // lane l delivers imports l, l + 64, ... in order, each the diagonal + upper part of one row
      // (up to kWU granules), polling its next kFacImpQ at once; the published count is the lowest
      // import still pending over the lanes
      constexpr int Q = kFacImpQ;
      const int ib = fa.bandImp[b], ni = fa.bandNImp[b];
      const unsigned long long m0 = fa.prof ? clk() : 0;
      int k = lane, published = 0;
      unsigned spins = 0;
      int wq[Q], pq[Q], cq[Q], sq[Q];
      bool fresh = true;
      while (ni > 0) {
        if (fresh) {  // the slot-free iterations, rows and slots of the lane's next Q imports
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int kq = k + 64 * q;
            wq[q] = kq < ni ? fa.impWait[ib + kq] : -1;
            pq[q] = kq < ni ? fa.impPos[ib + kq] : 0;
            cq[q] = kq < ni ? fa.impCnt[ib + kq] : 0;
            sq[q] = kq < ni ? fa.impSlot[ib + kq] : 0;
          }
          fresh = false;
        }
        const int progNow = (k < ni) ? lds_read(&s_prog) : 0;
        uint64_t lo[Q][kWU], hi[Q][kWU];
        bool req[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {  // a slot is free once its previous import's last reader has run
          req[q] = k + 64 * q < ni && progNow > wq[q];
#pragma unroll
          for (int u = 0; u < kWU; ++u) {
            lo[q][u] = hi[q][u] = 0;
            if (req[q] && u < cq[q]) {
              lo[q][u] = __hip_atomic_load(gU + 2 * (size_t)(pq[q] + u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              hi[q][u] = __hip_atomic_load(gU + 2 * (size_t)(pq[q] + u) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
        }
        int d = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {  // the ready prefix, in order
          bool ready = d == q && req[q];
#pragma unroll
          for (int u = 0; u < kWU; ++u)
            if (u < cq[q]) ready = ready && (unsigned)(lo[q][u] >> 32) == epoch && (unsigned)(hi[q][u] >> 32) == epoch;
          if (ready) {
#pragma unroll
            for (int u = 0; u < kWU; ++u)
              if (u < cq[q]) s_dep[impBase + sq[q] * kWU + u] = join_words((uint32_t)lo[q][u], (uint32_t)hi[q][u]);
            d = q + 1;
          }
        }
        const bool prog = d > 0;
        if (prog) {
          k += 64 * d;
          fresh = true;
        }
        int low = k < ni ? k : ni;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) low = min(low, __shfl_xor(low, o));
        if (low > published) {
          published = low;
          if (lane == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_write(&s_impDone, low);
          }
        }
        if (low >= ni) break;
        if (__any(prog)) {
          spins = 0;
        } else if (!spin(spins, err, 64u)) {
          break;
        }
      }
      if (fa.prof && lane == 0) atomicAdd(fa.prof + 5, clk() - m0);
    }
    __syncthreads();
  }
}

}  // namespace

void launch_chain_factor(const FactorArgs& fa, double* af, uint64_t* gU, unsigned epoch, unsigned* ticket,
                         unsigned* err, hipStream_t st) {
  if (fa.nbands <= 0) return;
  const dim3 grid(fa.nbands < 256 ? fa.nbands : 256), block(256);
  hipLaunchKernelGGL(k_chain_factor, grid, block, 0, st, fa, af, gU, epoch, ticket, err);
}

}  // namespace mmx
