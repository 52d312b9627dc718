// chain_sweep.hip -- band/chain-scheduled ILU triangular sweeps (scaler_ILU::solve,
// lib/LASolver/ILU_class.cpp:470-499) for gfx950.  Schedule: host/chain_sched.h.
//
// One workgroup runs one band (64 chains) at a time, four wavefronts:
//   wave 0  compute: lane l computes position t - skew[l] of its chain at iteration t; every
//           entry carries the LDS index of its value: the zero cell (pads), a lane's ring slot
//           (static schedule: written at an earlier iteration, not yet overwritten) or an import
//           slot (delivered once the importer's counter passes the iteration's impNeed);
//   wave 1,2 loaders: global -> LDS DMA (global_load_lds) of the matrix entries, their codes and
//           the right-hand-side operands of iteration t into stage t % DL (even / odd t), each
//           keeping several stages in flight against its own vmcnt;
//   wave 3  importer: polls the producers' global granules (agent scope) of the band's imports in
//           order of first use, stores each into its slot once the slot is free and publishes the
//           length of the delivered prefix.
// Every row is x_i = (b_i - sum_k a_k x_jk) [/ d_i] with the terms subtracted in ascending column
// order, exactly as the level-scheduled k_sweep and the reference.  SEG: a lane's rows take ns
// positions each (32 entries per position, the partial sum carried in a register), for triangles
// with rows wider than 48 entries; rows of 33..48 entries (the 3D backward triangle) take one
// position of a 48-entry stage (entry codes are 16-bit in every stage).  G = 2: a position computes
// two consecutive rows of the chain (rows of at most 16 entries, 2D), the second taking the first's
// value from the register, which halves the iterations on the critical path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sparse_kernels.h"

namespace mmx {
namespace {

#define MMX_LDS __attribute__((address_space(3)))

constexpr int kPad = -2147483647 - 1;
constexpr int kRingMax = 32;    // = kChainRingMax (host/chain_sched.h)
constexpr int kRingWide = 8;    // = kChainRingWide: the ring of the 48-entry stages
constexpr int kImpMax = 2048;   // = kChainImpMax
#ifndef MMX_IMP_Q
#define MMX_IMP_Q 4
#endif
constexpr int kImpQ = MMX_IMP_Q;  // imports each importer lane polls per round
#ifndef MMX_CHAIN_SPEC
#define MMX_CHAIN_SPEC 1  // compute loop bodies per entry-count class (no per-group branches)
#endif
constexpr unsigned kChainSpinMax = 1u << 22;

template <typename T>
__device__ __forceinline__ unsigned lds_off(T* p) {
  return (unsigned)(size_t)(MMX_LDS T*)p;
}
// LDS word access the compiler does not track: the loaders' tag stores must not wait for their
// own in-flight DMA (the compiler would insert vmcnt(0) before any tracked LDS access).
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
// s_waitcnt vmcnt(N) through the builtin, so the compiler's waitcnt pass knows the DMA has landed
// (an inline-asm wait is opaque to it and it would add vmcnt(0) before later LDS reads)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

__device__ __forceinline__ double join_words(uint32_t lo, uint32_t hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// stage geometry
template <int E>
struct Geo {
  static constexpr int DL = (E <= 16) ? 8 : 4;  // stages in the LDS ring
};
template <bool FWD, int PRO, int G>
struct AuxN {  // DMA instructions for the right-hand-side operands of one stage (+1: impNeed)
  static constexpr int n = G * (FWD ? (PRO == 0 ? 2 : PRO == 1 ? 6 : 4) : 2) + 1;  // bwd: y granule + diagonal
};
// per stage: the operands of each of the G rows of a position (<= 384 words each), then impNeed
// (64 copies)
template <int G>
struct Aux {
  static constexpr int need = 384 * G;
  static constexpr int words = need + 64;
};
// LDS cells of a lane ring of RM rows: [0] = +0.0, the rings, the import slots, the pairs' forwarded cell
template <int RM>
struct DepCells {
  static constexpr int n = 1 + 64 * (RM + 1) + kImpMax + 1;
};
// entry codes: 16-bit (32-bit in MMX_CHAIN_CODE16=0 builds, except the 48-entry stages)
template <int EE>
struct CodeOf {
  typedef typename std::conditional<chain_code16(EE), uint16_t, int>::type T;
};

// abort protocol: a bounded wait that gives up sets err; everyone polls err now and then
__device__ __forceinline__ bool aborted(unsigned* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
template <bool SLEEP = true>
__device__ __forceinline__ bool spin(unsigned& spins, unsigned* err, unsigned code) {
  if ((++spins & 255u) == 0 && aborted(err)) return false;
  if (spins > (SLEEP ? kChainSpinMax : kChainSpinMax * 16u)) {
    atomicOr(err, code);
    return false;
  }
  if constexpr (SLEEP) __builtin_amdgcn_s_sleep(1);
  return true;
}
#ifndef MMX_GRAN_B128
#define MMX_GRAN_B128 1  // a row's granule as one 16-byte store (n = 2 M sweeps 2.01 -> 1.88 ms, C4 1.69 -> 1.55 ms; 0: two 8-byte atomic stores)
#endif
#ifndef MMX_CHAIN_HOTSPIN
#define MMX_CHAIN_HOTSPIN 0  // 1: the compute wave polls its stage / import counters without s_sleep
#endif

// profiling counters (ca.prof, s_memtime cycles): 0 compute cycles, 1 compute waiting for stages,
// 2 compute waiting for imports, 3 compute iterations, 4 loader flush waits, 5 loader slot waits,
// 6 loader in-flight waits, 7 importer cycles, 8 bands; 16 + 4 i + {0 total, 1 stage wait,
// 2 import wait, 3 iterations} for the first 32 (i = b) and the last 32 bands (i = 64 + b - nbands)
__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ void prof_add(unsigned long long* prof, int i, unsigned long long v) {
  if (prof) atomicAdd(prof + i, v);
}

template <bool FWD, int PRO, int E, bool SEG, int G>
__global__ void __launch_bounds__(256) k_chain_sweep(ChainArgs ca, const double* __restrict__ src,
                                                     double* __restrict__ pvec, const double* __restrict__ res,
                                                     const double* __restrict__ avbar, const CgsScalars* __restrict__ sc,
                                                     const uint64_t* __restrict__ gin, uint64_t* gout,
                                                     double* __restrict__ out, unsigned epoch, unsigned* ticket,
                                                     unsigned* err) {
  static_assert(G == 1 || !SEG, "pairs of segmented rows");
  constexpr int EE = E * G;  // entry slots per position
  constexpr int DL = Geo<EE>::DL;
  constexpr int NAUX = AuxN<FWD, PRO, G>::n;
  constexpr int kAuxWords = Aux<G>::words;
  typedef typename CodeOf<EE>::T CodeT;
  constexpr int RM = EE > 32 ? kRingWide : kRingMax;
  // half-stage class: entry slots per row moved and read for a band using at most half of them
  constexpr int EH = (E / 2) % 4 == 0 && ((E / 2) * (int)sizeof(CodeT)) % 16 == 0 ? E / 2 : E;
  __shared__ __attribute__((aligned(16))) double s_val[DL * EE * 64];
  __shared__ __attribute__((aligned(16))) CodeT s_code[DL * EE * 64];
  __shared__ uint32_t s_aux[DL * kAuxWords];
  __shared__ double s_dep[DepCells<RM>::n];  // [0] = +0.0, lane rings, import slots
  __shared__ int s_tag[DL];
  __shared__ int s_prog, s_band, s_impDone;

  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int R = ca.R;
  // MMX_GRAN_B128: the granules written through a buffer resource (byte offsets: rows < 2^27)
  const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(gout, 0, 0x7fffffff, 0x00020000);
  const int impBase = 1 + 64 * (R + 1);
  const int fwdCell = impBase + ca.RI;  // G = 2: the entry whose value is the pair's first row
  double beta = 0.0, omega = 0.0, alpha = 0.0;
  if (FWD && PRO == 1) {
    beta = sc->beta;
    omega = sc->omega;
  }
  if (FWD && PRO == 2) alpha = sc->alpha;

  while (true) {
    if (tid == 0) {
      const unsigned tk = atomicAdd(ticket, 1u);
      s_band = tk < (unsigned)ca.nbands ? ca.bandOrder[tk] : ca.nbands;
      s_prog = 0;
      s_impDone = 0;
      s_dep[0] = 0.0;
    }
    if (tid < DL) s_tag[tid] = -1;
    __syncthreads();
    const int b = s_band;
    if (b >= ca.nbands) break;
    const bool skip = aborted(err);
    const int sb = ca.bandSlot[b], T = ca.bandT[b];
    const int g = b * 64 + lane;
    int cst = ca.laneStart[g], len = ca.laneLen[g], skew = ca.laneSkew[g], ns = SEG ? ca.laneNs[g] : 1;
    // launder the loaded lane values: inside the loops they must not count as pending loads, or the
    // waitcnt pass waits for every younger store/DMA (vmcnt(0)) at each iteration
    asm volatile("" : "+v"(cst), "+v"(len), "+v"(skew), "+v"(ns));

    const bool half = EH < E && ca.trim && ca.bandE[b] <= EH;
    if (skip) {
      // nothing: an earlier wait gave up; the host reports it
    } else if (wave == 0) {
      // ---------------- compute ----------------
      // iteration t + 1's stage (entries, addresses, operands) is read before iteration t is
      // computed, so an iteration costs one LDS round trip (its dependency values) plus the chain
      // 3D stages (E >= 32): the band's entry count selects the loop body at compile time (EB entry
      // slots per row, pads included: 0 * (+0.0) changes nothing), so the iteration has no
      // per-group branches (C4 sweeps 1.88 -> 1.80 ms).  2D stages keep one body with run-time
      // checks against bandE: two bodies measured slower there (2.68 -> 2.80 ms; the instruction
      // cache).  MMX_CHAIN_SPEC=0 (build option): one body everywhere.
      constexpr bool kSpec = MMX_CHAIN_SPEC && E >= 32;
      const int Eb = ca.bandE[b];
      auto compute = [&](auto ebc) {
        constexpr int EB = decltype(ebc)::value;
        wait_vm<0>();  // nothing in flight here; tells the waitcnt pass so the loop needs no vmcnt waits
        unsigned long long c0 = ca.prof ? clk() : 0, cstage = 0, cimp = 0;
        bool ok = true;
        struct Fetched {
          double a[EE];
          int c[EE];
          double init[G], diag[G];
          int need;
        };
        auto load_stage = [&](int st, Fetched& f) {
          const uint32_t* sa0 = s_aux + st * kAuxWords;
          f.need = (int)sa0[Aux<G>::need + lane];  // the same in every lane; made scalar where it is used
          const double* sv = s_val + st * EE * 64;
          const CodeT* scd = s_code + st * EE * 64;
#pragma unroll
          for (int g = 0; g < G; ++g)
#pragma unroll
            for (int e0 = 0; e0 < EB; e0 += 4)
              if (kSpec || e0 < Eb) {
                if constexpr (MMX_CHAIN_VEC) {
                  // stage image [g][e / 2][lane][2] (values), [g][e / 4][lane][4] (32-bit codes),
                  // [g][e / 8][lane][8] (16-bit codes): four entries of a lane in three LDS reads
                  const double2 a01 = *reinterpret_cast<const double2*>(sv + (g * E + e0) * 64 + lane * 2);
                  const double2 a23 = *reinterpret_cast<const double2*>(sv + (g * E + e0 + 2) * 64 + lane * 2);
                  f.a[g * E + e0] = a01.x;
                  f.a[g * E + e0 + 1] = a01.y;
                  f.a[g * E + e0 + 2] = a23.x;
                  f.a[g * E + e0 + 3] = a23.y;
                  if constexpr (sizeof(CodeT) == 4) {
                    const int4 c4 = *reinterpret_cast<const int4*>(scd + (g * E + e0) * 64 + lane * 4);
                    f.c[g * E + e0] = c4.x;
                    f.c[g * E + e0 + 1] = c4.y;
                    f.c[g * E + e0 + 2] = c4.z;
                    f.c[g * E + e0 + 3] = c4.w;
                  } else {
                    const ushort4 c4 =
                        *reinterpret_cast<const ushort4*>(scd + (g * E + (e0 & ~7)) * 64 + lane * 8 + (e0 & 4));
                    f.c[g * E + e0] = c4.x;
                    f.c[g * E + e0 + 1] = c4.y;
                    f.c[g * E + e0 + 2] = c4.z;
                    f.c[g * E + e0 + 3] = c4.w;
                  }
                } else {
#pragma unroll
                  for (int q = 0; q < 4; ++q) {
                    f.a[g * E + e0 + q] = sv[(g * E + e0 + q) * 64 + lane];
                    f.c[g * E + e0 + q] = scd[(g * E + e0 + q) * 64 + lane];
                  }
                }
              }
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const uint32_t* sa = sa0 + g * 384;
            if (FWD) {
              const double r0 = join_words(sa[lane], sa[64 + lane]);
              if (PRO == 0) {
                f.init[g] = r0;
              } else if (PRO == 1) {
                const double pv = join_words(sa[128 + lane], sa[192 + lane]);
                const double av = join_words(sa[256 + lane], sa[320 + lane]);
                f.init[g] = r0 + beta * (pv - omega * av);
              } else {
                const double av = join_words(sa[128 + lane], sa[192 + lane]);
                f.init[g] = r0 - alpha * av;
              }
              f.diag[g] = 1.0;
            } else {
              f.init[g] = join_words(sa[4 * lane], sa[4 * lane + 2]);  // granule {tag|lo, tag|hi}
              f.diag[g] = join_words(sa[256 + 2 * lane], sa[256 + 2 * lane + 1]);
            }
          }
        };
        auto fetch = [&](int t, Fetched& f) {  // blocking: wait for stage t, then read it
          const int st = t & (DL - 1);
          unsigned spins = 0;
          const unsigned long long w0 = ca.profIter ? clk() : 0;
          while (lds_read(&s_tag[st]) != t)
            if (!(ok = spin<!MMX_CHAIN_HOTSPIN>(spins, err, 8u))) break;
          if (ca.profIter) cstage += clk() - w0;
          load_stage(st, f);
        };
        // one iteration: a single batch of LDS reads -- this iteration's dependency values, the next
        // stage's tag, the import count, and the next stage's contents (valid when that tag, read
        // first and served first, says the stage has landed) -- then the chain
        int seen = 0;  // import count read by the previous batch
        double carry = 0.0;  // SEG: the partial sum of a row whose next segment comes at the next position
#ifdef MMX_CHAIN_FINE
        // probe (dev builds only): cycles of the step's segments, each closed by a full wait
        unsigned long long fq[5] = {0, 0, 0, 0, 0};
#define MMX_FINE_MARK(k)                                     \
    do {                                                       \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
      const unsigned long long _c = clk();                     \
      fq[k] += _c - fqt;                                       \
      fqt = _c;                                                \
    } while (0)
#else
#define MMX_FINE_MARK(k) \
    do {                   \
    } while (0)
#endif
        auto step = [&](int t, const Fetched& f, Fetched& nx) {
          const int need = __builtin_amdgcn_readfirstlane(f.need);
          if (need >= 0 && seen <= need) {  // imports this iteration reads: wait for their delivery
            unsigned spins = 0;
            const unsigned long long i0 = ca.profIter ? clk() : 0;
            while ((seen = lds_read(&s_impDone)) <= need)
              if (!(ok = spin<!MMX_CHAIN_HOTSPIN>(spins, err, 16u))) break;
            if (ca.profIter) cimp += clk() - i0;
            if (!ok) return;
          }
#ifdef MMX_CHAIN_FINE
          unsigned long long fqt = clk();
#endif
          double v[EE];
#pragma unroll
          for (int g = 0; g < G; ++g)
#pragma unroll
            for (int e0 = 0; e0 < EB; e0 += 4)
              if (kSpec || e0 < Eb) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[g * E + e0 + q] = s_dep[f.c[g * E + e0 + q]];
              }
          MMX_FINE_MARK(0);
          const bool hasNext = t + 1 < T;
          const int stn = (t + 1) & (DL - 1);
          const int tagN = __hip_atomic_load(&s_tag[stn], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int doneN = __hip_atomic_load(&s_impDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          asm volatile("" ::: "memory");  // keep the stage reads behind the tag read (LDS serves them in order)
          if (hasNext) load_stage(stn, nx);
          MMX_FINE_MARK(1);
          const int p = t - skew;
          double prev = 0.0;  // G = 2: the pair's first row
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const bool on = (G == 2) ? (p >= 0 && 2 * p + g < len) : (p >= 0 && p < len);
            if (on) {
              int ri = (G == 2) ? 2 * p + g : p, sg = 0;  // row of the chain, segment of the row
              if constexpr (SEG) {
                ri = p / ns;
                sg = p - ri * ns;
              }
              const int row = FWD ? cst + ri : cst - ri;
              // acc -= a_e * value_e in entry order; pads are 0 * (+0.0) and change nothing
              double acc = (SEG && sg != 0) ? carry : f.init[g];
#pragma unroll
              for (int e0 = 0; e0 < EB; e0 += 4)
                if (kSpec || e0 < Eb) {
#pragma unroll
                  for (int q = 0; q < 4; ++q) {
                    const int e = g * E + e0 + q;
                    const double val = (G == 2 && g == 1 && f.c[e] == fwdCell) ? prev : v[e];
                    acc -= f.a[e] * val;
                  }
                }
              if (SEG && sg != ns - 1) {
                carry = acc;  // the row goes on at the next position
              } else {
                if (!FWD) acc = acc / f.diag[g];
#ifdef MMX_CHAIN_FINE
                asm volatile("" ::"v"(acc));
                MMX_FINE_MARK(2);
#endif
                s_dep[1 + lane * (R + 1) + (((G == 2) ? ri : p) & (R - 1))] = acc;
                const uint64_t bits = (uint64_t)__double_as_longlong(acc), tag = (uint64_t)epoch << 32;
                if constexpr (MMX_GRAN_B128) {
                  // the granule {tag | lo, tag | hi} as one 16-byte store with the agent-scope (sc1)
                  // policy the two 8-byte atomic stores have; each 8-byte half is still written whole
                  typedef unsigned v4u __attribute__((ext_vector_type(4)));
                  const v4u d = {(unsigned)bits, epoch, (unsigned)(bits >> 32), epoch};
                  __builtin_amdgcn_raw_buffer_store_b128(d, grs, row * 16, 0, 16);
                } else {
                  __hip_atomic_store(gout + 2 * (size_t)row, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
                  __hip_atomic_store(gout + 2 * (size_t)row + 1, tag | (bits >> 32), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
                }
                if (!FWD && out) out[row] = acc;  // (out = nullptr: taken from the granules afterwards)
                if (FWD && PRO != 0) pvec[row] = f.init[g];
                prev = acc;
              }
            }
          }
          if (lane == 0) lds_write(&s_prog, t + 1);
          MMX_FINE_MARK(3);
          seen = doneN;
          if (hasNext && __builtin_amdgcn_readfirstlane(tagN) != t + 1) fetch(t + 1, nx);  // not landed yet
          MMX_FINE_MARK(4);
        };
        Fetched fa, fb;
        if (T > 0) fetch(0, fa);
        for (int t = 0; t < T && ok; t += 2) {
          step(t, fa, fb);
          if (t + 1 >= T || !ok) break;
          step(t + 1, fb, fa);
        }
        if (ca.prof && lane == 0) {
          const unsigned long long tot = clk() - c0;
          prof_add(ca.prof, 0, tot);
          prof_add(ca.prof, 1, cstage);
          prof_add(ca.prof, 2, cimp);
          prof_add(ca.prof, 3, (unsigned long long)T);
          prof_add(ca.prof, 8, 1ull);
#ifdef MMX_CHAIN_FINE
          for (int k = 0; k < 5; ++k) prof_add(ca.prof, 9 + k, fq[k]);
#endif
          const int pi = b < 32 ? b : (b >= ca.nbands - 32 ? 64 + b - ca.nbands : -1);
          if (pi >= 0) {
            prof_add(ca.prof, 16 + 4 * pi, tot);
            prof_add(ca.prof, 16 + 4 * pi + 1, cstage);
            prof_add(ca.prof, 16 + 4 * pi + 2, cimp);
            prof_add(ca.prof, 16 + 4 * pi + 3, (unsigned long long)T);
          }
        }
      };
      if constexpr (kSpec) {
        if (half)
          compute(std::integral_constant<int, EH>());
        else
          compute(std::integral_constant<int, E>());
      } else {
        compute(std::integral_constant<int, E>());
      }
    } else if (wave <= 2) {
      // ---------------- loaders (stages t = w, w+2, ...) ----------------
      // A band whose rows use at most half the stage's entry slots (bandE; e.g. the 2D grid-line
      // bands: <= 5 of 16) has only those moved: fewer DMA instructions per stage, so more stages
      // fit the 6-bit vmcnt window in flight.  The compute wave reads entries < bandE only.
      auto loader = [&](auto ebc) {
        constexpr int EB = decltype(ebc)::value;  // entry slots moved per row
        constexpr int NVb = EB / 2, NCb = EB * (int)sizeof(CodeT) / 16;
        constexpr int NIb = G * (NVb + NCb) + NAUX;
        constexpr int LAGb0 = 63 / NIb < 1 ? 1 : 63 / NIb;
        constexpr int LAGb = LAGb0 < DL / 2 ? LAGb0 : DL / 2;
        static_assert(EB <= E && EB % 4 == 0 && (EB * (int)sizeof(CodeT)) % 16 == 0, "stage entry slots");
        const int w = wave - 1;
        int nextPub = w;
        bool ok = true;
        unsigned long long cfl = 0, csl = 0, cin = 0;
        for (int t = w; t < T && ok; t += 2) {
          const int st = t & (DL - 1);
          if (lds_read(&s_prog) < t - DL + 1) {  // slot busy: publish what is in flight, then wait
            const unsigned long long f0 = ca.prof ? clk() : 0;
            wait_vm<0>();
            if (ca.prof) cfl += clk() - f0;
            for (; nextPub < t; nextPub += 2)
              if (lane == 0) lds_write(&s_tag[nextPub & (DL - 1)], nextPub);
            unsigned spins = 0;
            const unsigned long long s0 = ca.prof ? clk() : 0;
            while (lds_read(&s_prog) < t - DL + 1)
              if (!(ok = spin(spins, err, 32u))) break;
            if (ca.prof) csl += clk() - s0;
            if (!ok) break;
          }
          const size_t slot = (size_t)(sb + t);
          const double* gv = ca.val + slot * EE * 64;
          const char* gc = (const char*)ca.code + slot * EE * 64 * sizeof(CodeT);
#pragma unroll
          for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int i = 0; i < NVb; ++i)
              dma16(gv + (g * E / 2 + i) * 128 + lane * 2, s_val + st * EE * 64 + (g * E / 2 + i) * 128);
            constexpr int gcs = E * (int)sizeof(CodeT) / 16;  // code instructions per row block
#pragma unroll
            for (int i = 0; i < NCb; ++i)
              dma16(gc + (g * gcs + i) * 1024 + lane * 16, (char*)(s_code + st * EE * 64) + (g * gcs + i) * 1024);
          }
          const int p = t - skew;
          uint32_t* sa0 = s_aux + st * kAuxWords;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            // the row's operands (at each of its segments; a missing second row of a pair: row 0)
            const int ri = (G == 2) ? 2 * p + g : (SEG ? p / ns : p);
            const bool on = (G == 2) ? (p >= 0 && ri < len) : (p >= 0 && p < len);
            const int row = on ? (FWD ? cst + ri : cst - ri) : 0;
            uint32_t* sa = sa0 + g * 384;
            if (FWD) {
              const double* v0 = (PRO == 0) ? src : res;
              dma4((const char*)(v0 + row), sa);
              dma4((const char*)(v0 + row) + 4, sa + 64);
              if (PRO == 1) {
                dma4((const char*)(pvec + row), sa + 128);
                dma4((const char*)(pvec + row) + 4, sa + 192);
                dma4((const char*)(avbar + row), sa + 256);
                dma4((const char*)(avbar + row) + 4, sa + 320);
              } else if (PRO == 2) {
                dma4((const char*)(avbar + row), sa + 128);
                dma4((const char*)(avbar + row) + 4, sa + 192);
              }
            } else {
              dma16(gin + 2 * (size_t)row, sa);  // 64 x 16 B: words 0..255
              if (lane < 32) dma16(ca.dval + (slot * G + g) * 64 + lane * 2, sa + 256);  // 64 diagonals: words 256..383
            }
          }
          dma4(ca.impNeed + slot, sa0 + Aux<G>::need);  // the same word in every lane
          if ((t - nextPub) / 2 + 1 > LAGb) {
            const unsigned long long l0 = ca.prof ? clk() : 0;
            wait_vm<NIb * LAGb>();
            if (ca.prof) cin += clk() - l0;
            for (; nextPub <= t - 2 * LAGb; nextPub += 2)
              if (lane == 0) lds_write(&s_tag[nextPub & (DL - 1)], nextPub);
          }
        }
        wait_vm<0>();
        if (ok)
          for (; nextPub < T; nextPub += 2)
            if (lane == 0) lds_write(&s_tag[nextPub & (DL - 1)], nextPub);
        if (ca.prof && lane == 0) {
          prof_add(ca.prof, 4, cfl);
          prof_add(ca.prof, 5, csl);
          prof_add(ca.prof, 6, cin);
        }
      };
      if (half)
        loader(std::integral_constant<int, EH>());
      else
        loader(std::integral_constant<int, E>());
    } else {
      // ---------------- importer ----------------
      // lane l delivers imports l, l + 64, l + 128, ... in order, polling its next kImpQ at once:
      // a band of long chains below the cell-centre rows imports ~4 values per row (256 per
      // iteration), so one import per lane per round trip would set the pace; the published count
      // is the lowest import still pending over the lanes (all below it are in their slots)
      constexpr int Q = kImpQ;
      const int ib = ca.bandImp[b], ni = ca.bandNImp[b];
      const unsigned long long m0 = ca.prof ? clk() : 0;
      int k = lane;
      int published = 0;
      unsigned spins = 0;
      int jq[Q], nq[Q], sq[Q];
      bool fresh = true;
      while (ni > 0) {
        if (fresh) {  // the rows and slot-free iterations of the lane's next Q imports
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int kq = k + 64 * q;
            jq[q] = kq < ni ? ca.impRow[ib + kq] : 0;
            nq[q] = kq < ni ? ca.impWait[ib + kq] : -1;
            sq[q] = kq < ni ? ca.impSlot[ib + kq] : 0;
          }
          fresh = false;
        }
        const int progNow = (k < ni) ? lds_read(&s_prog) : 0;
        uint64_t lo[Q], hi[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {  // a slot is free once its previous import's last reader has run
          lo[q] = hi[q] = 0;
          if (k + 64 * q < ni && progNow > nq[q]) {
            lo[q] = __hip_atomic_load(gout + 2 * (size_t)jq[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hi[q] = __hip_atomic_load(gout + 2 * (size_t)jq[q] + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        int d = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {  // the ready prefix, in order
          if (d == q && k + 64 * q < ni && (unsigned)(lo[q] >> 32) == epoch && (unsigned)(hi[q] >> 32) == epoch) {
            s_dep[impBase + sq[q]] = join_words((uint32_t)lo[q], (uint32_t)hi[q]);
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
        if (low > published) {  // values are written before the count, same wavefront
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
      if (ca.prof && lane == 0) prof_add(ca.prof, 7, clk() - m0);
    }
    __syncthreads();
  }
}

}  // namespace

void launch_chain_sweep(bool fwd, int pro, int E, const ChainArgs& ca, const double* src, double* p, const double* res,
                        const double* avbar, const CgsScalars* sc, const uint64_t* gin, uint64_t* gout, double* out,
                        unsigned epoch, unsigned* ticket, unsigned* err, hipStream_t st) {
  if (ca.nbands <= 0) return;
  const dim3 grid(ca.nbands < 256 ? ca.nbands : 256), block(256);
#define MMX_CHAIN(F, P, EE, SG, GG)                                                                            \
  hipLaunchKernelGGL((k_chain_sweep<F, P, EE, SG, GG>), grid, block, 0, st, ca, src, p, res, avbar, sc, gin, gout, \
                     out, epoch, ticket, err)
#define MMX_CHAIN_E(F, P)                \
  do {                                   \
    if (ca.seg)                          \
      MMX_CHAIN(F, P, 32, true, 1);      \
    else if (ca.G == 2 && E == 8)        \
      MMX_CHAIN(F, P, 8, false, 2);      \
    else if (ca.G == 2)                  \
      MMX_CHAIN(F, P, 16, false, 2);     \
    else if (E == 8)                     \
      MMX_CHAIN(F, P, 8, false, 1);      \
    else if (E == 16)                    \
      MMX_CHAIN(F, P, 16, false, 1);     \
    else if (E == 48)                    \
      MMX_CHAIN(F, P, 48, false, 1);     \
    else                                 \
      MMX_CHAIN(F, P, 32, false, 1);     \
  } while (0)
  if (!fwd)
    MMX_CHAIN_E(false, 0);
  else if (pro == 0)
    MMX_CHAIN_E(true, 0);
  else if (pro == 1)
    MMX_CHAIN_E(true, 1);
  else
    MMX_CHAIN_E(true, 2);
#undef MMX_CHAIN_E
#undef MMX_CHAIN
}

__global__ void k_chain_fill(long long n, const int* __restrict__ srcIdx, const double* __restrict__ af,
                             double* __restrict__ val, double padValue) {
  const long long x = (long long)blockIdx.x * 256 + threadIdx.x;
  if (x < n) {
    const int s = srcIdx[x];
    val[x] = s >= 0 ? af[s] : padValue;
  }
}

__global__ void k_scatter_a(long long nnz, const int* __restrict__ amap, const double* __restrict__ a,
                            double* __restrict__ af) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k < nnz) af[amap[k]] = a[k];
}

void launch_scatter_a(long long nnz, const int* amap, const double* a, double* af, hipStream_t st) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(k_scatter_a, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, st, nnz, amap, a, af);
}

void launch_chain_fill(long long n, const int* srcIdx, const double* af, double* val, double padValue,
                       hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_chain_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, srcIdx, af, val, padValue);
}

}  // namespace mmx

// the layout word this kernel object was compiled with (layout.h; checked by the host at create)
extern "C" unsigned mmx_layout_chain(void) { return mmx::kLayoutWord; }
