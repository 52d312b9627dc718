// sparse.cpp -- host side of the LASolver replacement (include/mmx_sparse.h): MatrixStruc
// packing, the symbolic ILU (level of fill, natural order) and the device-resident MatrixIter
// whose numeric factor, sweeps, SpMV and CG-STAB run as HIP kernels (kernels/sparse_kernels.hip).
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <queue>
#include <vector>

#include "../../../include/mmx_sparse.h"
#include "../kernels/sparse_kernels.h"
#include "chain_sched.h"
#include "common.h"

namespace mmx {
namespace {

// MatrixStruc (lib/LASolver/MatrixIter.cpp:88-257): per-row column lists; pack() sorts each row
// ascending and removes duplicates; the diagonal is present unless no_diag.
// MMX_SCHED_PROF=1: phase times of the host set-up on stderr
struct PhaseTimer {
  bool on;
  const char* who;
  std::chrono::steady_clock::time_point t;
  explicit PhaseTimer(const char* w) : on(getenv("MMX_SCHED_PROF") != nullptr), who(w), t(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[sched] %s %s %.3f s\n", who, what, std::chrono::duration<double>(now - t).count());
    t = now;
  }
};

struct Struc {
  int n = 0;
  bool packed = false;
  bool diag = false;  // every row holds its diagonal (MatrixStruc(n), no_diag = 0): implicit until pack
  std::vector<std::vector<int>> rows;  // entries set one at a time (set_entry)
  // entries of mesh_pattern in bulk, as a CSR whose rows are sorted and duplicate-free (no
  // per-row allocations: 1.5 M rows at C4)
  std::vector<int> bia, bja;
  std::vector<int> ia, ja;

  void pack() {
    if (packed) throw Error(MMADMM_ERR_INVALID, "error: data structure already packed");
    ia.assign(n + 1, 0);
    const bool bulk = !bia.empty();
    // row i = sorted union of {i} (diag), rows[i] and bulk row i: sizes first, then the entries
    std::vector<int> cnt(n, 0);
    auto merged = [&](int i, int* out) {  // writes the row (out != nullptr) and returns its length
      std::vector<int>& r = rows[i];
      if (!std::is_sorted(r.begin(), r.end())) std::sort(r.begin(), r.end());
      r.erase(std::unique(r.begin(), r.end()), r.end());
      const int* b = bulk ? bja.data() + bia[i] : nullptr;
      const int* be = bulk ? bja.data() + bia[i + 1] : nullptr;
      const int* a = r.data();
      const int* ae = r.data() + r.size();
      bool dpend = diag;
      int len = 0, last = -1;
      while (true) {
        int v = INT32_MAX;
        if (a != ae) v = std::min(v, *a);
        if (b != be) v = std::min(v, *b);
        if (dpend) v = std::min(v, i);
        if (v == INT32_MAX) break;
        if (a != ae && *a == v) ++a;
        if (b != be && *b == v) ++b;
        if (dpend && v == i) dpend = false;
        if (v != last) {
          if (out) out[len] = v;
          ++len;
          last = v;
        }
      }
      return len;
    };
#pragma omp parallel for schedule(dynamic, 4096)
    for (int i = 0; i < n; ++i) cnt[i] = merged(i, nullptr);
    for (int i = 0; i < n; ++i) ia[i + 1] = ia[i] + cnt[i];
    ja.resize(ia[n]);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int i = 0; i < n; ++i) {
      merged(i, ja.data() + ia[i]);
      std::vector<int>().swap(rows[i]);
    }
    rows.clear();
    std::vector<int>().swap(bia);
    std::vector<int>().swap(bja);
    packed = true;
  }
};

// Symbolic ILU by level of fill (scaler_ILU::sfac2 + merge2, lib/LASolver/ILU_class.cpp:17-295),
// natural ordering.  Rows must be duplicate-free and hold their diagonal (as pack() makes them).
}  // namespace
void symbolic_ilu(int n, const std::vector<int>& ia, const std::vector<int>& ja, int level, std::vector<int>& iaf,
                  std::vector<int>& jaf, std::vector<int>& dgRel) {
  if (level == 0) {  // no fill can reach level 0 (levnew >= 1): the pattern of A, rows sorted
    iaf.assign(ia.begin(), ia.begin() + n + 1);
    jaf.assign(ja.begin(), ja.begin() + ia[n]);
    dgRel.assign(n, -1);
    // rows in parallel; the first bad row (lowest index) is reported, as the sequential loop would
    int bad = n, why = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(min : bad)
    for (int i = 0; i < n; ++i) {
      int* b = jaf.data() + iaf[i];
      int* e = jaf.data() + iaf[i + 1];
      if (b == e) {
        bad = std::min(bad, i);
        continue;
      }
      std::sort(b, e);
      bool dup = false;
      for (int* q = b + 1; q < e; ++q) dup |= (*q == q[-1]);
      int* d = std::lower_bound(b, e, i);
      if (dup || d == e || *d != i) {
        bad = std::min(bad, i);
        continue;
      }
      dgRel[i] = (int)(d - b);
    }
    if (bad < n) {
      const int* b = jaf.data() + iaf[bad];
      const int* e = jaf.data() + iaf[bad + 1];
      bool dup = false;
      for (const int* q = b + 1; q < e; ++q) dup |= (*q == q[-1]);
      why = (b == e) ? 0 : dup ? 1 : 2;
      throw Error(MMADMM_ERR_INVALID, "row " + std::to_string(bad) +
                                          (why == 0 ? " is empty (no diagonal)" : why == 1 ? " has duplicate columns"
                                                                                           : " has no diagonal entry"));
    }
    return;
  }
  // Level of fill, row by row (IKJ order): a row starts from its pattern at level 0; its pivots k < i
  // are taken in ascending order -- fill columns below i join them as they appear, always above the
  // pivot that creates them, so a min-heap delivers every pivot after all pivots that can change
  // its level -- and each pivot's upper entries j propose level lev(i, k) + lev(k, j) + 1: an
  // existing entry keeps the smaller level, a new one enters when the proposal is at most `level`
  // (the fill rule of scaler_ILU::sfac2 / merge2, lib/LASolver/ILU_class.cpp:17-90)
  constexpr int kAbsent = INT32_MAX;
  std::vector<std::vector<int>> rj(n), rl(n);
  std::vector<int> lev(n, kAbsent), cols;
  dgRel.assign(n, -1);
  for (int i = 0; i < n; ++i) {
    cols.assign(ja.begin() + ia[i], ja.begin() + ia[i + 1]);
    if (cols.empty()) throw Error(MMADMM_ERR_INVALID, "row " + std::to_string(i) + " is empty (no diagonal)");
    std::sort(cols.begin(), cols.end());
    if (std::adjacent_find(cols.begin(), cols.end()) != cols.end())
      throw Error(MMADMM_ERR_INVALID, "row " + std::to_string(i) + " has duplicate columns");
    std::priority_queue<int, std::vector<int>, std::greater<int>> pivots;
    for (int c : cols) {
      lev[c] = 0;
      if (c < i) pivots.push(c);
    }
    while (!pivots.empty()) {
      const int k = pivots.top();
      pivots.pop();
      const int lk = lev[k];
      const std::vector<int>& J = rj[k];
      const std::vector<int>& Lv = rl[k];
      for (size_t q = (size_t)dgRel[k] + 1; q < J.size(); ++q) {
        const int j = J[q], cand = lk + Lv[q] + 1;
        if (lev[j] != kAbsent) {
          lev[j] = std::min(lev[j], cand);
        } else if (cand <= level) {
          lev[j] = cand;
          cols.push_back(j);
          if (j < i) pivots.push(j);
        }
      }
    }
    std::sort(cols.begin(), cols.end());
    rj[i] = cols;
    rl[i].resize(cols.size());
    for (size_t q = 0; q < cols.size(); ++q) {
      if (cols[q] == i) dgRel[i] = (int)q;
      rl[i][q] = lev[cols[q]];
      lev[cols[q]] = kAbsent;
    }
    if (dgRel[i] < 0) throw Error(MMADMM_ERR_INVALID, "row " + std::to_string(i) + " has no diagonal entry");
  }
  iaf.assign(n + 1, 0);
  for (int i = 0; i < n; ++i) iaf[i + 1] = iaf[i] + (int)rj[i].size();
  jaf.resize(iaf[n]);
  for (int i = 0; i < n; ++i) std::copy(rj[i].begin(), rj[i].end(), jaf.begin() + iaf[i]);
}

namespace {

// SpMV kernel: 2 = k_spmv2 (default), 1 = k_spmv (MMX_SPMV=1; kept for A/B measurements)
int spmv_version() {
  static int v = [] {
    const char* e = getenv("MMX_SPMV");
    return (e && atoi(e) == 1) ? 1 : 2;
  }();
  return v;
}

void check_params(const mmx_param_iter& p) {
  if (p.order != 0) throw Error(MMADMM_ERR_INVALID, "unsupported ParamIter.order (only natural ordering, 0)");
  if (p.drop_ilu != 0) throw Error(MMADMM_ERR_INVALID, "unsupported ParamIter.drop_ilu (only level-of-fill ILU, 0)");
  if (p.iscal != 0) throw Error(MMADMM_ERR_INVALID, "unsupported ParamIter.iscal (only no scaling, 0)");
  if (p.ipiv != 0) throw Error(MMADMM_ERR_INVALID, "unsupported ParamIter.ipiv (only no pivoting, 0)");
  if (p.iaccel != 0) throw Error(MMADMM_ERR_INVALID, "unsupported ParamIter.iaccel (only CG-STAB, 0)");
  if (p.level < 0) throw Error(MMADMM_ERR_INVALID, "ParamIter.level must be >= 0");
}

struct Timer {
  hipEvent_t a = nullptr, b = nullptr;
  bool armed = false;
  void init() {
    if (!a) {
      // timing only: no system-scope fence at the records (engine.cpp nextEvent)
      MMX_HIP(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
      MMX_HIP(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    }
  }
  ~Timer() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
  }
};

}  // namespace

struct SparseMatrix {
  int device = 0;
  hipStream_t st = nullptr;
  int n = 0;
  long long nnz = 0;
  std::vector<int> ia, ja;
  DevBuf<int> d_ia, d_ja, d_rowblk;
  DevBuf<int4> d_desc;  // SpMV block descriptors {r0, r1, k0, k1}
  int nblk = 0;
  DevBuf<double> d_a, d_b, d_tol;
  bool tolSet = false;
  // symbolic + numeric ILU
  bool symbolic = false;
  int level = -1;
  std::vector<int> iaf, jaf, dgRel;
  DevBuf<int> d_iaf, d_jaf, d_dg, d_amap, d_permf, d_permb;
  DevBuf<int2> d_piv;
  DevBuf<int> d_toff;           // factor in LDS: per lower entry, its offset into d_tgt
  DevBuf<signed char> d_tgt;    // per (lower entry, pivot-row upper entry): position updated in the row, or -1
  bool facLds = false;
  int nchf = 0, nchb = 0, nlevf = 0, nlevb = 0;
  DevBuf<double> d_af;
  DevBuf<unsigned> d_flags, d_ctl;  // ctl: 8 tickets, err, pad (16-byte multiple)
  DevBuf<uint64_t> d_gy, d_gx;
  unsigned epoch = 0, fepoch = 0;
  // chain/band-scheduled sweeps (host/chain_sched.h); level-scheduled when a schedule is not
  // possible or MMX_SWEEP=level (rows wider than 32 entries: segmented schedule, chain_sched.h)
  struct ChainDir {
    int E = 0;
    long long nent = 0, nslot = 0;
    DevBuf<int> bandSlot, bandT, bandImp, bandNImp, bandE, bandOrder, laneStart, laneLen, laneSkew, laneNs, code, src, dsrc,
        impRow, impSlot, impWait, impNeed;
    DevBuf<uint16_t> code16;  // the codes of a 48-entry schedule (16-bit)
    DevBuf<double> val, dval;
    ChainArgs args{};
  };
  ChainDir chf, chb;
  bool useChain = false;
  // the numeric factor on the forward chain/band schedule (chain_factor.hip, 2D rows); the
  // level schedule otherwise or with MMX_FACTOR=level
  struct FactorDir {
    DevBuf<int> bandSlot, bandT, laneLen, laneSkew, bandOrder, bandImp, bandNImp, impPos, impCnt, impSlot, impWait,
        impNeed, meta, rowStart, vsrc;
    DevBuf<uint16_t> code;
    DevBuf<double> val, af0;
    DevBuf<uint64_t> gU;
    FactorArgs args{};
  } chfac;
  bool useChainFactor = false;
  bool facWave = false;     // k_ilu_factor_wave (one wavefront per row) over d_permw
  DevBuf<int> d_permw;
  DevBuf<uint64_t> d_gF;    // the wave factor's granules (MMX_FACTOR_GRAN=0: flags + drained stores)
  DevBuf<unsigned long long> d_cprof;  // MMX_CHAIN_PROF: 2 x 512 counters (forward, backward)
  // numeric factor cache: the ILU of unchanged values is the same, so a solve re-factors only
  // after set_values / sfac (the reference re-factors in every solve, MatrixIter.cpp:684)
  long long valVersion = 0, factVersion = -1;
  // CG-STAB vectors
  DevBuf<double> d_res, d_res0, d_p, d_vbar, d_avbar, d_s, d_z, d_t, d_x, d_part, d_tmp;
  DevBuf<CgsScalars> d_sc;
  CgsScalars* h_sc = nullptr;
  bool timing = false;
  mmx_sparse_stats stats{};
  Timer tm[4];  // spmv, sweeps, factor, whole solve

  SparseMatrix(int dev, int n_, const int* ia_, const int* ja_) : device(dev), n(n_) {
    if (n <= 0) throw Error(MMADMM_ERR_INVALID, "matrix size must be positive");
    if (ia_[0] != 0) throw Error(MMADMM_ERR_INVALID, "ia[0] must be 0");
    for (int i = 0; i < n; ++i)
      if (ia_[i + 1] < ia_[i]) throw Error(MMADMM_ERR_INVALID, "ia must be non-decreasing");
    nnz = ia_[n];
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(max : bad)
    for (long long k = 0; k < nnz; ++k)
      if (ja_[k] < 0 || ja_[k] >= n) bad = 1;
    if (bad) throw Error(MMADMM_ERR_INVALID, "column index out of range");
    ia.assign(ia_, ia_ + n + 1);
    ja.resize(nnz);
#pragma omp parallel for schedule(static)
    for (long long k = 0; k < nnz; ++k) ja[k] = ja_[k];
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) throw Error(MMADMM_ERR_HIP, "no HIP device available");
    MMX_HIP(hipSetDevice(device));
    MMX_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    d_ia.upload(ia.data(), ia.size(), st);
    // 2 padding entries: launch_spmv2 reads whole aligned pairs
    d_ja.alloc((size_t)nnz + 2);
    if (nnz * sizeof(int) >= ((size_t)16 << 20))
      upload_staged(d_ja.p, ja.data(), (size_t)nnz * sizeof(int), st);
    else if (nnz)
      MMX_HIP(hipMemcpyAsync(d_ja.p, ja.data(), (size_t)nnz * sizeof(int), hipMemcpyHostToDevice, st));
    MMX_HIP(hipMemsetAsync(d_ja.p + nnz, 0, 2 * sizeof(int), st));
    d_a.alloc(nnz + 2);
    MMX_HIP(hipMemsetAsync(d_a.p, 0, sizeof(double) * (nnz + 2), st));
    d_b.alloc(n);
    MMX_HIP(hipMemsetAsync(d_b.p, 0, sizeof(double) * n, st));
    // SpMV row blocks: greedy runs of rows with <= kSpmvTile nonzeros (a longer row alone)
    std::vector<int> rb{0};
    int r0 = 0;
    while (r0 < n) {
      int r = r0 + 1;
      while (r < n && ia[r + 1] - ia[r0] <= kSpmvTile && r - r0 < 4 * kSpmvBlock) ++r;
      rb.push_back(r);
      r0 = r;
    }
    nblk = (int)rb.size() - 1;
    d_rowblk.upload(rb.data(), rb.size(), st);
    std::vector<int4> desc(nblk);
    for (int b = 0; b < nblk; ++b) desc[b] = make_int4(rb[b], rb[b + 1], ia[rb[b]], ia[rb[b + 1]]);
    d_desc.upload(desc.data(), desc.size(), st);
    MMX_HIP(hipStreamSynchronize(st));
    for (DevBuf<double>* v : {&d_res, &d_res0, &d_p, &d_vbar, &d_avbar, &d_s, &d_z, &d_t, &d_x, &d_tmp}) v->alloc(n);
    d_part.alloc((size_t)std::max(nblk, vec_grid(n)) * 3);
    d_sc.alloc(1);
    MMX_HIP(hipMemsetAsync(d_sc.p, 0, sizeof(CgsScalars), st));
    MMX_HIP(hipHostMalloc((void**)&h_sc, sizeof(CgsScalars), hipHostMallocDefault));
    d_ctl.alloc(16);
    MMX_HIP(hipMemsetAsync(d_ctl.p, 0, 16 * sizeof(unsigned), st));
    d_gy.alloc(2 * (size_t)n);
    d_gx.alloc(2 * (size_t)n);
    MMX_HIP(hipMemsetAsync(d_gy.p, 0, 16 * (size_t)n, st));
    MMX_HIP(hipMemsetAsync(d_gx.p, 0, 16 * (size_t)n, st));
    d_flags.alloc(n);
    MMX_HIP(hipMemsetAsync(d_flags.p, 0, sizeof(unsigned) * n, st));
    stats.spmv_bytes = 12.0 * (double)nnz + 4.0 * (n + 1) + 16.0 * n;
    MMX_HIP(hipStreamSynchronize(st));
  }
  ~SparseMatrix() {
    if (st) (void)hipStreamSynchronize(st);
    if (evSpin) (void)hipEventDestroy(evSpin);
    if (h_sc) (void)hipHostFree(h_sc);
    if (st) (void)hipStreamDestroy(st);
  }

  // the stream's work so far has completed, waited for by polling an event: the per-iteration
  // convergence readback of CG-STAB waits in a spin, not in the blocking stream wait, whose wake-up
  // latency varied by milliseconds on a loaded host (a backward-Euler step 24-34 ms over runs of the
  // same kernels); MMX_SPIN=0: the stream wait
  hipEvent_t evSpin = nullptr;
  void spin_sync() {
    static const bool spin = [] {
      const char* e = getenv("MMX_SPIN");
      return !(e && atoi(e) == 0);
    }();
    if (!spin) {
      MMX_HIP(hipStreamSynchronize(st));
      return;
    }
    if (!evSpin) MMX_HIP(hipEventCreateWithFlags(&evSpin, hipEventDisableTiming));
    MMX_HIP(hipEventRecord(evSpin, st));
    hipError_t r;
    while ((r = hipEventQuery(evSpin)) == hipErrorNotReady) __builtin_ia32_pause();
    MMX_HIP(r);
  }

  unsigned* tickets() { return d_ctl.p; }
  unsigned* errw() { return d_ctl.p + 8; }

  void sfac(const mmx_param_iter& p) {
    check_params(p);
    PhaseTimer pt("sfac");
    symbolic_ilu(n, ia, ja, p.level, iaf, jaf, dgRel);
    pt.mark("symbolic");
    level = p.level;
    std::vector<int> dg(n), amap(nnz);
    for (int i = 0; i < n; ++i) dg[i] = iaf[i] + dgRel[i];
    // the sweep and factor schedules (the bulk of the host set-up: DESIGN.md §7b) depend only on the
    // factor's pattern: built on helper threads while this one prepares the rest
    const char* smode = getenv("MMX_SWEEP");
    const bool tryChain = !(smode && std::strcmp(smode, "level") == 0);
    const char* fmode = getenv("MMX_FACTOR");
    const bool tryChainFactor = !(fmode && (std::strcmp(fmode, "level") == 0 || std::strcmp(fmode, "global") == 0));
    ChainSchedule Fs, Bs;
    FactorSchedule FS;
    std::vector<std::thread> helpers;
    std::exception_ptr helperErr[3];
    const int nt = std::max(1, omp_get_max_threads());
    auto helper = [&](int slot, auto fn) {
      helpers.emplace_back([&, slot, fn, nt] {
        try {
          omp_set_num_threads(std::max(1, nt / 2));
          fn();
        } catch (...) {
          helperErr[slot] = std::current_exception();
        }
      });
    };
    // each sweep schedule is uploaded by its helper as soon as it is built (2D: under the factor
    // schedule, the longest of the three); a failed one leaves useChain off below
    const char* pe = getenv("MMX_CHAIN_PROF");
    if (tryChain && pe && atoi(pe) && !d_cprof.p) {
      d_cprof.alloc(1024);
      MMX_HIP(hipMemsetAsync(d_cprof.p, 0, 1024 * sizeof(unsigned long long), st));
    }
    bool upF = false, upB = false;
    if (tryChain) {
      helper(0, [&] {
        Bs = build_chain_schedule(n, iaf, jaf, dg, false);
        if (Bs.ok) {
          upload_chain(Bs, chb);
          upB = true;
          release(Bs);
        }
      });
      if (tryChainFactor) helper(1, [&] { FS = build_factor_schedule(n, iaf, jaf, dg); });
      helper(2, [&] {
        Fs = build_chain_schedule(n, iaf, jaf, dg, true);
        if (Fs.ok) {
          upload_chain(Fs, chf);
          upF = true;
          release(Fs);
        }
      });
    }
    struct Joiner {  // the helpers reference this frame: joined on every way out of it
      std::vector<std::thread>& h;
      ~Joiner() {
        for (auto& t : h)
          if (t.joinable()) t.join();
      }
    } joiner{helpers};
#pragma omp parallel for schedule(dynamic, 4096)
    for (int i = 0; i < n; ++i) {
      const int* b = jaf.data() + iaf[i];
      const int* e = jaf.data() + iaf[i + 1];
      for (int k = ia[i]; k < ia[i + 1]; ++k) amap[k] = (int)(std::lower_bound(b, e, ja[k]) - jaf.data());
    }
    d_iaf.upload(iaf.data(), iaf.size(), st);
    d_jaf.upload(jaf.data(), jaf.size(), st);
    d_dg.upload(dg.data(), dg.size(), st);
    d_amap.upload(amap.data(), std::max<size_t>(amap.size(), 1), st);
    d_af.alloc(std::max<size_t>(jaf.size(), 1));
    factVersion = -1;
    pt.mark("amap + uploads");
    {
      // per row: its width and its lower entries' pivot upper lengths, summed, then a scan of rows --
      // the offsets into the update-target table.  The pivot ranges, offsets and targets themselves
      // are formed on the device from the factor pattern just uploaded (launch_fac_prep): at C4 they
      // are ~1.3 GB that a pageable upload took ~0.4 s to move
      int maxW = 0;
      std::vector<long long> rowTot(n + 1, 0);
#pragma omp parallel for schedule(dynamic, 4096) reduction(max : maxW)
      for (int i = 0; i < n; ++i) {
        maxW = std::max(maxW, iaf[i + 1] - iaf[i]);
        long long t = 0;
        for (int k = iaf[i]; k < dg[i]; ++k) t += iaf[jaf[k] + 1] - dg[jaf[k]] - 1;
        rowTot[i + 1] = t;
      }
      for (int i = 0; i < n; ++i) rowTot[i + 1] += rowTot[i];
      const long long tot = rowTot[n];
      const char* fm = getenv("MMX_FACTOR");
      facLds = maxW <= kFacW && tot < (1ll << 31) && !(fm && std::strcmp(fm, "global") == 0);
      DevBuf<long long> d_rowTot;
      d_rowTot.upload(rowTot.data(), rowTot.size(), st);
      d_piv.alloc(std::max<size_t>(jaf.size(), 1));
      if (facLds) {
        d_toff.alloc(std::max<size_t>(jaf.size(), 1));
        d_tgt.alloc((size_t)std::max<long long>(tot, 1));
        MMX_HIP(hipMemsetAsync(d_tgt.p, 0xFF, d_tgt.n, st));  // (-1: only a zero-size table keeps it)
      }
      launch_fac_prep(n, d_iaf.p, d_jaf.p, d_dg.p, d_rowTot.p, d_piv.p, facLds ? d_toff.p : nullptr,
                      facLds ? d_tgt.p : nullptr, st);
      MMX_HIP(hipStreamSynchronize(st));  // (d_rowTot and rowTot go out of scope)
      pt.mark("pivot ranges + update targets (device)");
    }
    // level schedules of the lower (forward sweep, factor) and upper (backward sweep) factor: the
    // two concurrently; the forward levels are kept for the wave factor's row order
    std::vector<int> levF(n), levB(n);
    auto schedule = [&](bool fwd, DevBuf<int>& out, int& nch, int& nlev) {
      std::vector<int>& lev = fwd ? levF : levB;
      int maxl = 0;
      for (int t = 0; t < n; ++t) {
        const int i = fwd ? t : n - 1 - t;
        int l = 0;
        const int kb = fwd ? iaf[i] : dg[i] + 1, ke = fwd ? dg[i] : iaf[i + 1];
        for (int k = kb; k < ke; ++k) l = std::max(l, lev[jaf[k]] + 1);
        lev[i] = l;
        maxl = std::max(maxl, l);
      }
      nlev = maxl + 1;
      std::vector<int> cnt(nlev + 1, 0);
      for (int i = 0; i < n; ++i) cnt[lev[i] + 1]++;
      std::vector<int> start(nlev + 1, 0);  // padded chunk offsets
      for (int l = 0; l < nlev; ++l) start[l + 1] = start[l] + (cnt[l + 1] + kSweepRows - 1) / kSweepRows * kSweepRows;
      std::vector<int> perm(start[nlev], -1), fill(start.begin(), start.end() - 1);
      for (int t = 0; t < n; ++t) {
        const int i = fwd ? t : n - 1 - t;
        perm[fill[lev[i]]++] = i;
      }
      nch = start[nlev] / kSweepRows;
      return perm;
    };
    std::vector<int> permF, permB;
#pragma omp parallel sections num_threads(2)
    {
#pragma omp section
      permF = schedule(true, d_permf, nchf, nlevf);
#pragma omp section
      permB = schedule(false, d_permb, nchb, nlevb);
    }
    d_permf.upload(permF.data(), permF.size(), st);
    d_permb.upload(permB.data(), permB.size(), st);
    pt.mark("level schedules");
    useChain = false;
    if (tryChain) {
      for (auto& h : helpers) h.join();
      for (auto& e : helperErr)
        if (e) std::rethrow_exception(e);
      pt.mark("chain + factor schedules, sweep uploads (joined)");
      // (the sweeps address their granules through 32-bit byte offsets: rows < 2^27)
      useChain = upF && upB && n < (1 << 27);
    }
    useChainFactor = false;
    facWave = false;
    {
      // default where the rows fit its layout (2D): bit-identical to the level schedule and
      // 12.3 ms against 25.0 ms at n = 2 M (profiles/r03/chain_factor/);
      // MMX_FACTOR=level (or global) keeps the level-scheduled factor
      const char* fm = fmode;
      if (useChain && tryChainFactor && jaf.size() < ((size_t)1 << 27)) {  // (32-bit granule byte offsets)
        if (FS.ok && !(fm && std::strcmp(fm, "wave") == 0)) {
          upload_factor(FS, dg);
          useChainFactor = true;
        }
      }
      // otherwise one wavefront per row (3D rows: 45 ms -> see DESIGN.md §7) where the rows fit it;
      // MMX_FACTOR=level keeps the level-scheduled lane-per-row factor
      if (!useChainFactor && facLds && !(fm && (std::strcmp(fm, "level") == 0 || std::strcmp(fm, "global") == 0))) {
        // the row image is scattered by all lanes at once: no two entries of A onto one factor slot
        // (rows in parallel; a row's amap is increasing when its columns are, else sorted here)
        int fitsAll = 1;
#pragma omp parallel for schedule(dynamic, 4096) reduction(min : fitsAll)
        for (int i = 0; i < n; ++i) {
          int ok = (dg[i] - iaf[i] <= kFacWaveNL && iaf[i + 1] - dg[i] - 1 <= 64) ? 1 : 0;
          bool inc = true;
          for (int k = ia[i] + 1; k < ia[i + 1] && inc; ++k) inc = amap[k] > amap[k - 1];
          if (ok && !inc) {
            std::vector<int> v(amap.begin() + ia[i], amap.begin() + ia[i + 1]);
            std::sort(v.begin(), v.end());
            ok = std::adjacent_find(v.begin(), v.end()) == v.end() ? 1 : 0;
          }
          fitsAll = std::min(fitsAll, ok);
        }
        const bool fits = fitsAll != 0;
        if (fits) {  // every row once, in forward level order (the forward sweep's levels)
          const std::vector<int>& lv = levF;
          std::vector<int> cnt;
          const int nl = nlevf;
          cnt.assign(nl + 1, 0);
          for (int i = 0; i < n; ++i) cnt[lv[i] + 1]++;
          for (int l = 0; l < nl; ++l) cnt[l + 1] += cnt[l];
          std::vector<int> pw(n);
          for (int i = 0; i < n; ++i) pw[cnt[lv[i]]++] = i;
          d_permw.upload(pw.data(), pw.size(), st);
          facWave = true;
          // MMX_FACTOR_GRAN=1: publish through tagged granules instead of drained stores + a flag
          // (measured: C4 factor 11.1 -> 12.0 ms, 2D 13.4 -> 13.5 ms; profiles/r05/experiments/
          // lasolver3d/factor_gran_ab.jsonl)
          const char* fg = getenv("MMX_FACTOR_GRAN");
          if (fg && atoi(fg) == 1) {
            d_gF.alloc(2 * jaf.size());
            MMX_HIP(hipMemsetAsync(d_gF.p, 0, d_gF.n * sizeof(uint64_t), st));
          } else {
            d_gF.alloc(0);
          }
        }
      }
    }
    MMX_HIP(hipStreamSynchronize(st));
    pt.mark("factor set-up + uploads");
    release(FS);
    symbolic = true;
  }

  // the schedules' host images (GBs at C4) are freed where they are done with: the sweep schedules
  // by their helper threads, under the factor schedule's build.  (Freed on a detached thread
  // instead, their page-table teardown went on into the work that followed and slowed it: a 2D
  // backward-Euler step after the C4-pattern solve 24.0 -> 29-35 ms.)
  template <class T>
  static void release(T& obj) {
    obj = T();
  }

  static int chain_trim() {
    const char* e = getenv("MMX_CHAIN_TRIM");
    return (e && atoi(e) == 0) ? 0 : 1;
  }
  void upload_chain(const ChainSchedule& S, ChainDir& c) {
    auto up = [&](DevBuf<int>& d, const auto& h) {
      if (h.empty()) {
        const int z = 0;
        d.upload(&z, 1, st);
      } else {
        d.upload(h.data(), h.size(), st);
      }
    };
    up(c.bandSlot, S.bandSlot);
    up(c.bandT, S.bandT);
    up(c.bandImp, S.bandImp);
    up(c.bandNImp, S.bandNImp);
    up(c.laneStart, S.laneStart);
    up(c.laneLen, S.laneLen);
    up(c.laneSkew, S.laneSkew);
    up(c.laneNs, S.laneNs);
    // the stage images as the kernel reads them (MMX_CHAIN_VEC, chain_sweep.hip): within each
    // [slot][g] block of E entries x 64 lanes, values [e / 2][lane][2] and codes [e / W][lane][W]
    // (W = 4 for 32-bit codes, 8 for 16-bit) instead of [e][lane]; the DMA instructions move the
    // same entry ranges either way
    const int EEs = S.E * S.G;
    const size_t blocks = S.code.size() / ((size_t)S.E * kChainLanes);
    auto permute = [&](const BigVec& lg, int W) {
      BigVec ph;
      if (!MMX_CHAIN_VEC) {
        ph = lg;
        return ph;
      }
      ph.resize(lg.size());  // uninitialised: every element is written below
      const int E = S.E, L = kChainLanes;
#pragma omp parallel for schedule(static)
      for (long long bk = 0; bk < (long long)blocks; ++bk) {
        const size_t base = (size_t)bk * E * L;
        for (int e = 0; e < E; ++e)
          for (int l = 0; l < L; ++l) ph[base + (size_t)(e / W) * W * L + (size_t)l * W + (e % W)] = lg[base + (size_t)e * L + l];
      }
      return ph;
    };
    (void)EEs;
    const void* codePtr;
    const bool c16on = chain_code16(S.E * S.G);
    const BigVec pcode = permute(S.code, c16on ? 8 : 4), psrc = permute(S.src, 2);
    std::vector<uint16_t> c16;
    if (S.E > 32 && (S.seg || S.G != 1 || S.R > kChainRingWide))
      throw Error(MMADMM_ERR_INVALID, "wide chain stage layout");
    if (c16on) {  // 16-bit codes (validate_chain_schedule: every index fits)
      c16.resize(pcode.size());
#pragma omp parallel for schedule(static)
      for (size_t x = 0; x < pcode.size(); ++x) c16[x] = (uint16_t)pcode[x];
      c.code16.upload(c16.data(), std::max<size_t>(c16.size(), 1), st);
      codePtr = c.code16.p;
    } else {
      up(c.code, pcode);
      codePtr = c.code.p;
    }
    up(c.src, psrc);
    MMX_HIP(hipStreamSynchronize(st));  // (the host images above go out of scope)
    up(c.dsrc, S.dsrc);
    up(c.impRow, S.impRow);
    up(c.impSlot, S.impSlot);
    up(c.impWait, S.impWait);
    up(c.impNeed, S.impNeed);
    up(c.bandE, S.bandE);
    up(c.bandOrder, S.bandOrder);
    c.E = S.E;
    c.nent = (long long)S.code.size();
    c.nslot = (long long)S.dsrc.size();
    c.val.alloc(std::max<long long>(c.nent, 1));
    c.dval.alloc(std::max<long long>(c.nslot, 1));
    const char* pe = getenv("MMX_CHAIN_PROF");
    c.args = ChainArgs{c.bandSlot.p, c.bandT.p, c.bandImp.p, c.bandNImp.p, c.laneStart.p, c.laneLen.p, c.laneSkew.p,
                       c.laneNs.p, c.bandE.p, c.val.p, codePtr, c.dval.p, c.impRow.p, c.impSlot.p, c.impWait.p, c.impNeed.p,
                       c.bandOrder.p, S.nbands, S.R, S.RI, S.seg ? 1 : 0, S.G,
                       d_cprof.p ? d_cprof.p + (S.fwd ? 0 : 512) : nullptr, (pe && atoi(pe) >= 2) ? 1 : 0,
                       chain_trim()};
  }

  void upload_factor(const FactorSchedule& F, const std::vector<int>& dg) {
    auto up = [&](DevBuf<int>& d, const auto& h) {
      if (h.empty()) {
        const int z = 0;
        d.upload(&z, 1, st);
      } else {
        d.upload(h.data(), h.size(), st);
      }
    };
    FactorDir& c = chfac;
    const ChainSchedule& S = F.geo;
    up(c.bandSlot, S.bandSlot);
    up(c.bandT, S.bandT);
    up(c.laneLen, S.laneLen);
    up(c.laneSkew, S.laneSkew);
    up(c.bandOrder, S.bandOrder);
    up(c.bandImp, F.bandImp);
    up(c.bandNImp, F.bandNImp);
    std::vector<int> pos(F.impRow.size()), cnt(F.impRow.size());
    for (size_t k = 0; k < F.impRow.size(); ++k) {
      const int j = F.impRow[k];
      pos[k] = dg[j];
      cnt[k] = iaf[j + 1] - dg[j];
    }
    up(c.impPos, pos);
    up(c.impCnt, cnt);
    up(c.impSlot, F.impSlot);
    up(c.impWait, F.impWait);
    up(c.impNeed, F.impNeed);
    up(c.meta, F.meta);
    up(c.rowStart, F.rowStart);
    up(c.vsrc, F.vsrc);
    c.code.upload(F.code.data(), F.code.size(), st);
    c.val.alloc(std::max<size_t>(F.vsrc.size(), 1));
    c.af0.alloc(std::max<size_t>(jaf.size(), 1));
    c.gU.alloc(2 * std::max<size_t>(jaf.size(), 1));
    MMX_HIP(hipMemsetAsync(c.gU.p, 0, c.gU.n * sizeof(uint64_t), st));
    c.args = FactorArgs{c.bandSlot.p, c.bandT.p, c.laneLen.p, c.laneSkew.p, c.bandOrder.p, c.bandImp.p, c.bandNImp.p,
                        c.impPos.p, c.impCnt.p, c.impSlot.p, c.impWait.p, c.impNeed.p, c.val.p, c.code.p, c.meta.p,
                        c.rowStart.p, S.nbands, F.R, d_cprof.p ? d_cprof.p + 480 : nullptr};
  }

  void begin(int t) {
    if (!timing) return;
    tm[t].init();
    MMX_HIP(hipEventRecord(tm[t].a, st));
  }
  float end(int t) {
    if (!timing) return 0.f;
    MMX_HIP(hipEventRecord(tm[t].b, st));
    MMX_HIP(hipEventSynchronize(tm[t].b));
    float ms = 0.f;
    MMX_HIP(hipEventElapsedTime(&ms, tm[t].a, tm[t].b));
    return ms;
  }

  void check_err() {
    unsigned e = 0;
    MMX_HIP(hipMemcpyAsync(&e, errw(), sizeof(unsigned), hipMemcpyDeviceToHost, st));
    MMX_HIP(hipStreamSynchronize(st));
    if (e) {
      factVersion = -1;
      MMX_HIP(hipMemsetAsync(errw(), 0, sizeof(unsigned), st));
      throw Error(MMADMM_ERR_HIP, "sync-free ILU dependency wait gave up (code " + std::to_string(e) + ")");
    }
  }

  void factor(bool force = true) {
    if (!symbolic) throw Error(MMADMM_ERR_INVALID, "error: solve called with no symbolic ILU");
    if (!force && factVersion == valVersion) return;
    factVersion = valVersion;
    MMX_HIP(hipMemsetAsync(tickets(), 0, 8 * sizeof(unsigned), st));
    if (++fepoch == 0) {
      MMX_HIP(hipMemsetAsync(d_flags.p, 0, sizeof(unsigned) * n, st));
      if (useChainFactor) MMX_HIP(hipMemsetAsync(chfac.gU.p, 0, chfac.gU.n * sizeof(uint64_t), st));
      if (d_gF.n) MMX_HIP(hipMemsetAsync(d_gF.p, 0, d_gF.n * sizeof(uint64_t), st));
      fepoch = 1;
    }
    begin(2);
    if (useChainFactor) {  // A into the factor pattern, the rows' values in schedule order, the factor
      MMX_HIP(hipMemsetAsync(chfac.af0.p, 0, chfac.af0.n * sizeof(double), st));
      launch_scatter_a((long long)nnz, d_amap.p, d_a.p, chfac.af0.p, st);
      launch_chain_fill((long long)chfac.vsrc.n, chfac.vsrc.p, chfac.af0.p, chfac.val.p, 0.0, st);
      launch_chain_factor(chfac.args, d_af.p, chfac.gU.p, fepoch, tickets(), errw(), st);
    } else if (facWave) {
      launch_ilu_factor_wave(d_ia.p, d_a.p, d_amap.p, d_iaf.p, d_dg.p, d_piv.p, d_jaf.p, d_toff.p, d_tgt.p, d_permw.p, n,
                             d_af.p, d_flags.p, d_gF.n ? d_gF.p : nullptr, fepoch, tickets(), errw(), st);
    } else if (facLds)
      launch_ilu_factor_lds(d_ia.p, d_a.p, d_amap.p, d_iaf.p, d_jaf.p, d_dg.p, d_piv.p, d_toff.p, d_tgt.p, d_permf.p, nchf,
                            d_af.p, d_flags.p, fepoch, tickets(), errw(), st);
    else
      launch_ilu_factor(d_ia.p, d_ja.p, d_a.p, d_amap.p, d_iaf.p, d_jaf.p, d_dg.p, d_piv.p, d_permf.p, nchf, d_af.p,
                        d_flags.p, fepoch, tickets(), errw(), st);
    if (useChain) {  // the sweeps read the factor's entries in schedule order
      launch_chain_fill(chf.nent, chf.src.p, d_af.p, chf.val.p, 0.0, st);
      launch_chain_fill(chb.nent, chb.src.p, d_af.p, chb.val.p, 0.0, st);
      launch_chain_fill(chb.nslot, chb.dsrc.p, d_af.p, chb.dval.p, 1.0, st);
    }
    MMX_HIP(hipGetLastError());
    const float ms = end(2);
    stats.factors++;
    if (timing) {
      stats.t_factor_ms += ms;
      stats.n_factor_timed++;
    }
  }

  unsigned next_epoch() {
    if (++epoch == 0) {  // wrapped: clear every granule tag
      MMX_HIP(hipMemsetAsync(d_gy.p, 0, 16 * (size_t)n, st));
      MMX_HIP(hipMemsetAsync(d_gx.p, 0, 16 * (size_t)n, st));
      epoch = 1;
    }
    return epoch;
  }

  // scaler_ILU::solve: out = (LU)^-1 src, or with the CG-STAB prologues (pro 1: p, pro 2: s)
  void ilu_apply(int pro, const double* src, double* p, double* out, unsigned* tk) {
    begin(1);
    const unsigned ey = next_epoch();
    if (useChain)
      launch_chain_sweep(true, pro, chf.E, chf.args, src, p, d_res.p, d_avbar.p, d_sc.p, nullptr, d_gy.p, nullptr, ey,
                         tk, errw(), st);
    else
      launch_sweep(true, pro, d_iaf.p, d_jaf.p, d_dg.p, d_af.p, d_permf.p, nchf, src, p, d_res.p, d_avbar.p, d_sc.p,
                   nullptr, d_gy.p, nullptr, ey, tk, errw(), st);
    const unsigned ex = next_epoch();
    // the backward sweep's result taken from the granules it publishes for every row anyway, by a
    // vector pass after it: one store less per row on the compute wave (n = 2 M: sweeps 2.14-2.17 ->
    // 2.02 ms, solve 47.7-48.2 -> 45.8-46.0 ms; MMX_BWD_GRAN=0: the sweep stores it)
    const char* bg = getenv("MMX_BWD_GRAN");
    const bool fromGran = !(bg && atoi(bg) == 0);
    if (useChain) {
      launch_chain_sweep(false, 0, chb.E, chb.args, nullptr, nullptr, nullptr, nullptr, nullptr, d_gy.p, d_gx.p,
                         fromGran ? nullptr : out, ex, tk + 1, errw(), st);
      if (fromGran) launch_gran_extract(n, d_gx.p, out, st);
    } else
      launch_sweep(false, 0, d_iaf.p, d_jaf.p, d_dg.p, d_af.p, d_permb.p, nchb, nullptr, nullptr, nullptr, nullptr,
                   nullptr, d_gy.p, d_gx.p, out, ex, tk + 1, errw(), st);
    MMX_HIP(hipGetLastError());
    const float ms = end(1);
    stats.sweeps += 2;
    if (timing) {
      stats.t_sweep_ms += ms;
      stats.n_sweep_timed += 2;
    }
  }

  void spmv(int epi, const double* x, double* y, const double* e1) {
    begin(0);
    if (spmv_version() == 1)
      launch_spmv(epi, nblk, d_rowblk.p, d_ia.p, d_ja.p, d_a.p, x, y, e1, d_part.p, st);
    else
      launch_spmv2(epi, nblk, d_desc.p, d_ia.p, d_ja.p, d_a.p, x, y, e1, d_part.p, st);
    MMX_HIP(hipGetLastError());
    const float ms = end(0);
    stats.spmvs++;
    if (timing) {
      stats.t_spmv_ms += ms;
      stats.n_spmv_timed++;
    }
  }

  // MatrixIter::solve (lib/LASolver/MatrixIter.cpp:635-819) with scaler_cgstab.
  void solve(const mmx_param_iter& p, double* d_xout, int& nitr, int initial_guess) {
    check_params(p);
    if (!symbolic) throw Error(MMADMM_ERR_INVALID, "error: solve called with no symbolic ILU");
    if (p.level != level) throw Error(MMADMM_ERR_INVALID, "ParamIter.level differs from the one given to sfac");
    hipEvent_t t0 = nullptr;
    if (timing) {
      tm[3].init();
      MMX_HIP(hipEventRecord(tm[3].a, st));
    }
    factor(false);
    const int gv = vec_grid(n);
    if (initial_guess == 0) {
      launch_cgs_init(0, n, d_b.p, d_xout, d_res.p, d_res0.p, d_p.p, d_avbar.p, p.new_rhat == 0, d_part.p, st);
    } else {
      spmv(0, d_xout, d_res.p, nullptr);
      launch_cgs_init(1, n, d_b.p, d_xout, d_res.p, d_res0.p, d_p.p, d_avbar.p, p.new_rhat == 0, d_part.p, st);
    }
    if (p.new_rhat != 0) {  // scaler_cgstab(n, res, ilu): res0 = (LU)^-1 res  (accel_class.h:87-94)
      MMX_HIP(hipMemsetAsync(tickets(), 0, 8 * sizeof(unsigned), st));
      ilu_apply(0, d_res.p, nullptr, d_res0.p, tickets());
      launch_dot_into(n, d_res0.p, d_res.p, d_part.p, st);
    }
    const double ctol = p.resid_reduc;
    MMX_HIP(hipMemcpyAsync(&d_sc.p->ctol, &ctol, sizeof(double), hipMemcpyHostToDevice, st));
    launch_cgs_fin(0, d_part.p, gv, d_sc.p, st);
    const double* tol = tolSet ? d_tol.p : nullptr;
    // the forward sweeps' CG-STAB prologues (p and s updates) as vector passes before them, so the
    // sweeps read one operand and store nothing but their results (n = 2 M: average sweep 2.61 ->
    // 2.16-2.20 ms, solve 55.6 -> 48.5-49.0 ms; MMX_CGS_UNFUSE=0: fused into the forward sweeps)
    const char* uf = getenv("MMX_CGS_UNFUSE");
    const bool unfuse = !(uf && atoi(uf) == 0);
    int conv = 0, it = 0;
    for (int iter = 1; iter <= p.nitmax; ++iter) {
      ++it;
      MMX_HIP(hipMemsetAsync(tickets(), 0, 8 * sizeof(unsigned), st));
      if (unfuse) {  // the prologues as vector passes, the forward sweeps reading one operand
        launch_cgs_pro(1, n, d_res.p, d_avbar.p, d_p.p, d_sc.p, st);
        ilu_apply(0, d_p.p, nullptr, d_vbar.p, tickets());
      } else {
        ilu_apply(1, nullptr, d_p.p, d_vbar.p, tickets());          // p update; vbar = (LU)^-1 p
      }
      spmv(1, d_vbar.p, d_avbar.p, d_res0.p);                      // avbar = A vbar; (res0, avbar)
      launch_cgs_fin(1, d_part.p, nblk, d_sc.p, st);               // alpha
      if (unfuse) {
        launch_cgs_pro(2, n, d_res.p, d_avbar.p, d_s.p, d_sc.p, st);
        ilu_apply(0, d_s.p, nullptr, d_z.p, tickets() + 2);
      } else {
        ilu_apply(2, nullptr, d_s.p, d_z.p, tickets() + 2);          // s = res - alpha avbar; z = (LU)^-1 s
      }
      spmv(2, d_z.p, d_t.p, d_s.p);                                // t = A z; (t, s), (t, t)
      launch_cgs_fin(2, d_part.p, nblk, d_sc.p, st);               // omega
      launch_cgs_update(n, d_vbar.p, d_z.p, d_s.p, d_t.p, d_res0.p, tol, d_xout, d_res.p, d_sc.p, d_part.p, st);
      launch_cgs_fin(3, d_part.p, gv, d_sc.p, st);
      MMX_HIP(hipGetLastError());
      MMX_HIP(hipMemcpyAsync(h_sc, d_sc.p, sizeof(CgsScalars), hipMemcpyDeviceToHost, st));
      spin_sync();
      stats.iterations++;
      if (h_sc->conv) {
        conv = 1;
        break;
      }
    }
    if (p.nitmax <= 0) {  // the reference's loop body never runs; report non-convergence
      MMX_HIP(hipMemcpyAsync(h_sc, d_sc.p, sizeof(CgsScalars), hipMemcpyDeviceToHost, st));
      MMX_HIP(hipStreamSynchronize(st));
    }
    check_err();
    nitr = conv ? it : -1;
    stats.solves++;
    stats.last_rms = h_sc->rms;
    stats.rmsi = h_sc->rmsi;
    if (timing) {
      MMX_HIP(hipEventRecord(tm[3].b, st));
      MMX_HIP(hipEventSynchronize(tm[3].b));
      float ms = 0.f;
      MMX_HIP(hipEventElapsedTime(&ms, tm[3].a, tm[3].b));
      stats.t_solve_ms += ms;
    }
    (void)t0;
  }
};

struct StrucHandle {
  Struc s;
};

}  // namespace mmx

struct mmx_struc_s {
  mmx::Struc s;
};
struct mmx_matrix_s {
  mmx::SparseMatrix* m;
};

using mmx::Error;
using mmx::guarded;

extern "C" {

void mmx_param_iter_default(mmx_param_iter* p) {  // ParamIter() (MatrixIter.h:155-168)
  if (!p) return;
  p->order = 1;
  p->level = 1;
  p->drop_ilu = 0;
  p->iscal = 1;
  p->nitmax = 30;
  p->resid_reduc = 1.e-6;
  p->drop_tol = 1.e-3;
  p->info = 1;
  p->new_rhat = 0;
  p->iaccel = 0;
  p->north = 10;
  p->ipiv = 0;
}

void mmx_param_iter_mesh(mmx_param_iter* p) {  // src/Mesh.cpp:264-304
  if (!p) return;
  mmx_param_iter_default(p);
  p->order = 0;
  p->level = 0;
  p->drop_ilu = 0;
  p->iscal = 0;
  p->nitmax = 10000;
  p->ipiv = 0;
  p->resid_reduc = 1.e-6;
  p->info = 0;
  p->drop_tol = 1.e-3;
  p->new_rhat = 0;
  p->iaccel = 0;
  p->north = 10;
}

int mmx_struc_create(int n, int no_diag, mmx_struc* out) {
  return guarded([&] {
    if (!out || n <= 0) throw Error(MMADMM_ERR_INVALID, "mmx_struc_create: bad arguments");
    auto* h = new mmx_struc_s;
    h->s.n = n;
    h->s.rows.resize(n);
    h->s.diag = (no_diag == 0);  // (implicit until pack: no n one-entry allocations)
    *out = h;
  });
}

int mmx_struc_set_entry(mmx_struc s, int row, int col) {
  return guarded([&] {
    if (!s) throw Error(MMADMM_ERR_INVALID, "null structure");
    if (s->s.packed) throw Error(MMADMM_ERR_INVALID, "error: data structure already compressed");
    if (row < 0 || row >= s->s.n) throw Error(MMADMM_ERR_INVALID, "invalid row entry in set_entry");
    if (col < 0 || col >= s->s.n) throw Error(MMADMM_ERR_INVALID, "invalid column entry in set_entry");
    s->s.rows[row].push_back(col);
  });
}

int mmx_struc_set_entries(mmx_struc s, long long count, const int32_t* rows, const int32_t* cols) {
  return guarded([&] {
    if (!s || (count > 0 && (!rows || !cols))) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    if (s->s.packed) throw Error(MMADMM_ERR_INVALID, "error: data structure already compressed");
    for (long long e = 0; e < count; ++e) {
      if (rows[e] < 0 || rows[e] >= s->s.n) throw Error(MMADMM_ERR_INVALID, "invalid row entry in set_entry");
      if (cols[e] < 0 || cols[e] >= s->s.n) throw Error(MMADMM_ERR_INVALID, "invalid column entry in set_entry");
      s->s.rows[rows[e]].push_back(cols[e]);
    }
  });
}

int mmx_struc_mesh_pattern(mmx_struc s, int dim, int nF, const int32_t* F) {
  return guarded([&] {
    if (!s || (dim != 2 && dim != 3) || nF < 0 || (nF > 0 && !F)) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    if (s->s.packed) throw Error(MMADMM_ERR_INVALID, "error: data structure already compressed");
    const int D = dim, nP = s->s.n / D;
    if (nP * D != s->s.n) throw Error(MMADMM_ERR_INVALID, "structure size is not dim * nodes");
    // node adjacency first (every vertex pair of every simplex, flat CSR), then D x D blocks
    // (counts and fills in parallel: a node's list is sorted below, so the order it is filled in
    // does not matter)
    std::vector<int> cnt(nP + 1, 0);
    int badv = 0;
#pragma omp parallel for schedule(static) reduction(max : badv)
    for (long long k = 0; k < (long long)nF * (D + 1); ++k) {
      const int va = F[k];
      if (va < 0 || va >= nP) {
        badv = 1;
        continue;
      }
      __atomic_fetch_add(&cnt[va + 1], D + 1, __ATOMIC_RELAXED);
    }
    if (badv) throw Error(MMADMM_ERR_INVALID, "simplex vertex out of range");
    for (int v = 0; v < nP; ++v) cnt[v + 1] += cnt[v];
    std::vector<int> nb(cnt[nP]), fill(cnt.begin(), cnt.end() - 1);
#pragma omp parallel for schedule(static)
    for (int t = 0; t < nF; ++t)
      for (int a = 0; a <= D; ++a) {
        const int va = F[(size_t)t * (D + 1) + a];
        const int o = __atomic_fetch_add(&fill[va], D + 1, __ATOMIC_RELAXED);
        for (int b = 0; b <= D; ++b) nb[o + b] = F[(size_t)t * (D + 1) + b];
      }
    std::vector<int> nu(nP);  // distinct neighbours (itself included) of every node
#pragma omp parallel for schedule(dynamic, 4096)
    for (int v = 0; v < nP; ++v) {
      int* b = nb.data() + cnt[v];
      std::sort(b, nb.data() + cnt[v + 1]);
      nu[v] = (int)(std::unique(b, nb.data() + cnt[v + 1]) - b);
    }
    auto& S = s->s;
    if (!S.bia.empty()) {  // a second mesh pattern (rare): into the per-row lists
      for (int v = 0; v < nP; ++v)
        for (int d = 0; d < D; ++d) {
          auto& r = S.rows[v * D + d];
          for (int q = 0; q < nu[v]; ++q)
            for (int c = 0; c < D; ++c) r.push_back(nb[cnt[v] + q] * D + c);
        }
      return;
    }
    // the bulk CSR: row v D + d holds (u D + c) for the neighbours u (ascending) and c < D
    S.bia.assign((size_t)S.n + 1, 0);
    for (int v = 0; v < nP; ++v)
      for (int d = 0; d < D; ++d) S.bia[(size_t)v * D + d + 1] = nu[v] * D;
    for (int i = 0; i < S.n; ++i) S.bia[i + 1] += S.bia[i];
    S.bja.resize(S.bia[S.n]);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int v = 0; v < nP; ++v)
      for (int d = 0; d < D; ++d) {
        int* o = S.bja.data() + S.bia[(size_t)v * D + d];
        for (int q = 0; q < nu[v]; ++q)
          for (int c = 0; c < D; ++c) *o++ = nb[cnt[v] + q] * D + c;
      }
  });
}

int mmx_struc_pack(mmx_struc s) {
  return guarded([&] {
    if (!s) throw Error(MMADMM_ERR_INVALID, "null structure");
    s->s.pack();
  });
}

int mmx_struc_get(mmx_struc s, int* n, long long* nnz, int32_t* ia, int32_t* ja) {
  return guarded([&] {
    if (!s) throw Error(MMADMM_ERR_INVALID, "null structure");
    if (!s->s.packed) s->s.pack();  // getia/getja pack on demand (MatrixIter.cpp:146-148)
    if (n) *n = s->s.n;
    if (nnz) *nnz = s->s.ia[s->s.n];
    if (ia) std::memcpy(ia, s->s.ia.data(), sizeof(int) * (s->s.n + 1));
    if (ja) std::memcpy(ja, s->s.ja.data(), sizeof(int) * s->s.ja.size());
  });
}

int mmx_struc_destroy(mmx_struc s) {
  delete s;
  return MMADMM_OK;
}

int mmx_matrix_create(int device, int n, const int32_t* ia, const int32_t* ja, mmx_matrix* out) {
  return guarded([&] {
    mmx::check_kernel_layout(mmx::kLayoutWord);
    if (!out || !ia || (n > 0 && !ja && ia[n] > 0)) throw Error(MMADMM_ERR_INVALID, "mmx_matrix_create: bad arguments");
    *out = nullptr;
    auto* h = new mmx_matrix_s;
    try {
      h->m = new mmx::SparseMatrix(device, n, ia, ja);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int mmx_matrix_create_from_struc(int device, mmx_struc s, mmx_matrix* out) {
  return guarded([&] {
    mmx::check_kernel_layout(mmx::kLayoutWord);
    if (!s || !out) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    if (!s->s.packed) s->s.pack();
    *out = nullptr;
    auto* h = new mmx_matrix_s;
    try {
      h->m = new mmx::SparseMatrix(device, s->s.n, s->s.ia.data(), s->s.ja.data());
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

#define MMX_M(m)                                                    \
  if (!(m) || !(m)->m) throw Error(MMADMM_ERR_INVALID, "null matrix"); \
  mmx::SparseMatrix& M = *(m)->m;                                   \
  MMX_HIP(hipSetDevice(M.device))

int mmx_matrix_sizes(mmx_matrix m, int* n, long long* nnz) {
  return guarded([&] {
    MMX_M(m);
    if (n) *n = M.n;
    if (nnz) *nnz = M.nnz;
  });
}

int mmx_matrix_stream(mmx_matrix m, void** s) {
  return guarded([&] {
    MMX_M(m);
    if (s) *s = (void*)M.st;
  });
}

int mmx_matrix_set_values(mmx_matrix m, const double* a) {
  return guarded([&] {
    MMX_M(m);
    if (!a && M.nnz) throw Error(MMADMM_ERR_INVALID, "null values");
    MMX_HIP(hipMemcpyAsync(M.d_a.p, a, sizeof(double) * M.nnz, hipMemcpyHostToDevice, M.st));
    M.valVersion++;
    MMX_HIP(hipStreamSynchronize(M.st));
  });
}

int mmx_matrix_set_values_device(mmx_matrix m, const double* d_a) {
  return guarded([&] {
    MMX_M(m);
    if (!d_a && M.nnz) throw Error(MMADMM_ERR_INVALID, "null values");
    MMX_HIP(hipMemcpyAsync(M.d_a.p, d_a, sizeof(double) * M.nnz, hipMemcpyDeviceToDevice, M.st));
    M.valVersion++;
  });
}

int mmx_matrix_set_rhs(mmx_matrix m, const double* b) {
  return guarded([&] {
    MMX_M(m);
    if (!b) throw Error(MMADMM_ERR_INVALID, "null rhs");
    MMX_HIP(hipMemcpyAsync(M.d_b.p, b, sizeof(double) * M.n, hipMemcpyHostToDevice, M.st));
    MMX_HIP(hipStreamSynchronize(M.st));
  });
}

int mmx_matrix_set_rhs_device(mmx_matrix m, const double* d_b) {
  return guarded([&] {
    MMX_M(m);
    if (!d_b) throw Error(MMADMM_ERR_INVALID, "null rhs");
    MMX_HIP(hipMemcpyAsync(M.d_b.p, d_b, sizeof(double) * M.n, hipMemcpyDeviceToDevice, M.st));
  });
}

int mmx_matrix_set_toler(mmx_matrix m, const double* tol) {
  return guarded([&] {
    MMX_M(m);
    if (!tol) throw Error(MMADMM_ERR_INVALID, "null tolerance vector");
    bool allZero = true;
    for (int i = 0; i < M.n; ++i) allZero &= (tol[i] == 0.0);
    if (allZero) {  // the reference's default (MatrixIter.cpp:394-398) and src/Mesh.cpp's setting
      M.tolSet = false;
      return;
    }
    M.d_tol.upload(tol, M.n, M.st);
    MMX_HIP(hipStreamSynchronize(M.st));
    M.tolSet = true;
  });
}

int mmx_matrix_sfac(mmx_matrix m, const mmx_param_iter* p) {
  return guarded([&] {
    MMX_M(m);
    if (!p) throw Error(MMADMM_ERR_INVALID, "null parameters");
    M.sfac(*p);
  });
}

int mmx_matrix_solve_device(mmx_matrix m, const mmx_param_iter* p, double* d_x, int* nitr, int initial_guess) {
  return guarded([&] {
    MMX_M(m);
    if (!p || !d_x || !nitr) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    M.solve(*p, d_x, *nitr, initial_guess);
  });
}

int mmx_matrix_solve(mmx_matrix m, const mmx_param_iter* p, double* x, int* nitr, int initial_guess) {
  return guarded([&] {
    MMX_M(m);
    if (!p || !x || !nitr) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    if (initial_guess) MMX_HIP(hipMemcpyAsync(M.d_x.p, x, sizeof(double) * M.n, hipMemcpyHostToDevice, M.st));
    M.solve(*p, M.d_x.p, *nitr, initial_guess);
    MMX_HIP(hipMemcpyAsync(x, M.d_x.p, sizeof(double) * M.n, hipMemcpyDeviceToHost, M.st));
    MMX_HIP(hipStreamSynchronize(M.st));
  });
}

int mmx_matrix_matmult_device(mmx_matrix m, const double* d_x, double* d_y) {
  return guarded([&] {
    MMX_M(m);
    if (!d_x || !d_y) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    M.spmv(0, d_x, d_y, nullptr);
  });
}

int mmx_matrix_matmult(mmx_matrix m, const double* x, double* y) {
  return guarded([&] {
    MMX_M(m);
    if (!x || !y) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    MMX_HIP(hipMemcpyAsync(M.d_tmp.p, x, sizeof(double) * M.n, hipMemcpyHostToDevice, M.st));
    M.spmv(0, M.d_tmp.p, M.d_t.p, nullptr);
    MMX_HIP(hipMemcpyAsync(y, M.d_t.p, sizeof(double) * M.n, hipMemcpyDeviceToHost, M.st));
    MMX_HIP(hipStreamSynchronize(M.st));
  });
}

int mmx_matrix_factor(mmx_matrix m) {
  return guarded([&] {
    MMX_M(m);
    M.factor();
    M.check_err();
  });
}

int mmx_matrix_ilu_solve_device(mmx_matrix m, const double* d_b, double* d_x) {
  return guarded([&] {
    MMX_M(m);
    if (!d_b || !d_x) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    if (!M.symbolic || M.fepoch == 0) throw Error(MMADMM_ERR_INVALID, "error: solve called with no factor");
    MMX_HIP(hipMemsetAsync(M.tickets(), 0, 8 * sizeof(unsigned), M.st));
    M.ilu_apply(0, d_b, nullptr, d_x, M.tickets());
  });
}

int mmx_matrix_ilu_solve(mmx_matrix m, const double* b, double* x) {
  return guarded([&] {
    MMX_M(m);
    if (!b || !x) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    if (!M.symbolic || M.fepoch == 0) throw Error(MMADMM_ERR_INVALID, "error: solve called with no factor");
    MMX_HIP(hipMemcpyAsync(M.d_tmp.p, b, sizeof(double) * M.n, hipMemcpyHostToDevice, M.st));
    MMX_HIP(hipMemsetAsync(M.tickets(), 0, 8 * sizeof(unsigned), M.st));
    M.ilu_apply(0, M.d_tmp.p, nullptr, M.d_t.p, M.tickets());
    MMX_HIP(hipMemcpyAsync(x, M.d_t.p, sizeof(double) * M.n, hipMemcpyDeviceToHost, M.st));
    MMX_HIP(hipStreamSynchronize(M.st));
    M.check_err();
  });
}

int mmx_matrix_factor_nnz(mmx_matrix m, long long* nnzf) {
  return guarded([&] {
    MMX_M(m);
    if (!M.symbolic) throw Error(MMADMM_ERR_INVALID, "no symbolic factor (call mmx_matrix_sfac)");
    if (nnzf) *nnzf = (long long)M.jaf.size();
  });
}

int mmx_matrix_get_factor(mmx_matrix m, int32_t* iaf, int32_t* jaf, double* af, int32_t* diag) {
  return guarded([&] {
    MMX_M(m);
    if (!M.symbolic) throw Error(MMADMM_ERR_INVALID, "no symbolic factor (call mmx_matrix_sfac)");
    if (iaf) std::memcpy(iaf, M.iaf.data(), sizeof(int) * (M.n + 1));
    if (jaf) std::memcpy(jaf, M.jaf.data(), sizeof(int) * M.jaf.size());
    if (diag) std::memcpy(diag, M.dgRel.data(), sizeof(int) * M.n);
    if (af) {
      MMX_HIP(hipMemcpyAsync(af, M.d_af.p, sizeof(double) * M.jaf.size(), hipMemcpyDeviceToHost, M.st));
      MMX_HIP(hipStreamSynchronize(M.st));
    }
  });
}

int mmx_matrix_set_timing(mmx_matrix m, int on) {
  return guarded([&] {
    MMX_M(m);
    M.timing = on != 0;
  });
}

int mmx_matrix_stats_get(mmx_matrix m, mmx_sparse_stats* out) {
  return guarded([&] {
    MMX_M(m);
    if (out) {
      *out = M.stats;
      out->sweep_mode = M.useChain ? 1 : 0;
      out->factor_mode = M.useChainFactor ? 1 : M.facWave ? 2 : 0;
      out->sweep_e = M.useChain ? M.chf.E : 0;
      out->sweep_e_bwd = M.useChain ? M.chb.E : 0;
    }
  });
}

int mmx_matrix_chain_prof(mmx_matrix m, unsigned long long* out, int reset) {
  return guarded([&] {
    MMX_M(m);
    if (!M.d_cprof.p) throw Error(MMADMM_ERR_INVALID, "chain profiling off (set MMX_CHAIN_PROF=1 before sfac)");
    if (out)
      MMX_HIP(hipMemcpyAsync(out, M.d_cprof.p, 1024 * sizeof(unsigned long long), hipMemcpyDeviceToHost, M.st));
    if (reset) MMX_HIP(hipMemsetAsync(M.d_cprof.p, 0, 1024 * sizeof(unsigned long long), M.st));
    MMX_HIP(hipStreamSynchronize(M.st));
  });
}

int mmx_matrix_stats_reset(mmx_matrix m) {
  return guarded([&] {
    MMX_M(m);
    const double bytes = M.stats.spmv_bytes;
    M.stats = mmx_sparse_stats{};
    M.stats.spmv_bytes = bytes;
  });
}

int mmx_ilu_symbolic(int n, const int32_t* ia, const int32_t* ja, int level, long long* nnzf, int32_t* iaf,
                     int32_t* jaf, int32_t* diag) {
  return guarded([&] {
    if (n <= 0 || !ia || !ja || level < 0) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    std::vector<int> via(ia, ia + n + 1), vja(ja, ja + ia[n]), fia, fja, dg;
    mmx::symbolic_ilu(n, via, vja, level, fia, fja, dg);
    if (nnzf) *nnzf = (long long)fja.size();
    if (iaf) std::memcpy(iaf, fia.data(), sizeof(int) * (n + 1));
    if (jaf) std::memcpy(jaf, fja.data(), sizeof(int) * fja.size());
    if (diag) std::memcpy(diag, dg.data(), sizeof(int) * n);
  });
}

int mmx_sweep_schedule_info(int n, const int32_t* ia, const int32_t* ja, int level, int fwd, long long* info) {
  return guarded([&] {
    if (n <= 0 || !ia || !ja || level < 0 || !info) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    std::vector<int> via(ia, ia + n + 1), vja(ja, ja + ia[n]), fia, fja, dgRel;
    mmx::symbolic_ilu(n, via, vja, level, fia, fja, dgRel);
    std::vector<int> dg(n);
    for (int i = 0; i < n; ++i) dg[i] = fia[i] + dgRel[i];
    const mmx::ChainSchedule S = mmx::build_chain_schedule(n, fia, fja, dg, fwd != 0);
    int nlev = 0;
    {
      std::vector<int> lev(n, 0);
      for (int t = 0; t < n; ++t) {
        const int i = fwd ? t : n - 1 - t;
        int l = 0;
        const int kb = fwd ? fia[i] : dg[i] + 1, ke = fwd ? dg[i] : fia[i + 1];
        for (int k = kb; k < ke; ++k) l = std::max(l, lev[fja[k]] + 1);
        lev[i] = l;
        nlev = std::max(nlev, l + 1);
      }
    }
    const std::string bad = S.ok ? mmx::validate_chain_schedule(S, n, fia, fja, dg) : std::string();
    if (!bad.empty()) throw Error(MMADMM_ERR_INVALID, "chain schedule invalid: " + bad);
    const long long v[16] = {S.ok ? 1 : 0, S.E, S.R, S.RI, S.nbands, S.nchains, S.maxLen, S.maxSkew,
                             S.maxT, S.slots, S.nImports, S.estIters, nlev, 0, 0, 0};
    std::memcpy(info, v, sizeof(v));
  });
}

int mmx_factor_schedule_info(int n, const int32_t* ia, const int32_t* ja, int level, long long* info) {
  return guarded([&] {
    if (n <= 0 || !ia || !ja || level < 0 || !info) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    std::vector<int> via(ia, ia + n + 1), vja(ja, ja + ia[n]), fia, fja, dgRel;
    mmx::symbolic_ilu(n, via, vja, level, fia, fja, dgRel);
    std::vector<int> dg(n);
    for (int i = 0; i < n; ++i) dg[i] = fia[i] + dgRel[i];
    const mmx::FactorSchedule F = mmx::build_factor_schedule(n, fia, fja, dg);
    int nlev = 0;
    {
      std::vector<int> lev(n, 0);
      for (int i = 0; i < n; ++i) {
        int l = 0;
        for (int k = fia[i]; k < dg[i]; ++k) l = std::max(l, lev[fja[k]] + 1);
        lev[i] = l;
        nlev = std::max(nlev, l + 1);
      }
    }
    const std::string bad = F.ok ? mmx::validate_factor_schedule(F, n, fia, fja, dg) : std::string();
    if (!bad.empty()) throw Error(MMADMM_ERR_INVALID, "factor schedule invalid: " + bad);
    const long long v[8] = {F.ok ? 1 : 0, F.geo.nbands, F.slots, F.R, F.nImports, F.maxImpSlots, F.geo.estIters, nlev};
    std::memcpy(info, v, sizeof(v));
  });
}

int mmx_stream_copy(int device, const double* d_src, double* d_dst, long long n, int reps, int variant, double* ms) {
  return guarded([&] {
    if (!d_src || !d_dst || n <= 0 || (n & 1) || reps <= 0 || !ms) throw Error(MMADMM_ERR_INVALID, "bad arguments");
    MMX_HIP(hipSetDevice(device));
    hipStream_t st;
    MMX_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    mmx::Timer t;
    t.init();
    mmx::launch_stream_copy(variant, n / 2, d_src, d_dst, st);  // warm-up
    MMX_HIP(hipEventRecord(t.a, st));
    for (int r = 0; r < reps; ++r) mmx::launch_stream_copy(variant, n / 2, d_src, d_dst, st);
    MMX_HIP(hipEventRecord(t.b, st));
    MMX_HIP(hipEventSynchronize(t.b));
    float el = 0.f;
    MMX_HIP(hipEventElapsedTime(&el, t.a, t.b));
    MMX_HIP(hipStreamDestroy(st));
    *ms = (double)el / reps;
  });
}

// test hook: a kernel on a stream of its own that holds `blocks` workgroups' CUs for ms milliseconds
// (asynchronous; mmx_occupy_wait joins it) -- e.g. the wave factor must complete beside it
static hipStream_t g_occSt = nullptr;
static mmx::DevBuf<double>* g_occSink = nullptr;
int mmx_occupy(int device, int blocks, double ms) {
  return guarded([&] {
    if (blocks < 1 || blocks > 65536 || !(ms > 0) || ms > 10000) throw Error(MMADMM_ERR_INVALID, "mmx_occupy: bad arguments");
    MMX_HIP(hipSetDevice(device));
    if (!g_occSt) MMX_HIP(hipStreamCreateWithFlags(&g_occSt, hipStreamNonBlocking));
    if (!g_occSink) {
      g_occSink = new mmx::DevBuf<double>();
      g_occSink->alloc(1024);
    }
    mmx::launch_occupy(blocks, ms, g_occSink->p, g_occSt);
    MMX_HIP(hipGetLastError());
  });
}
int mmx_occupy_wait(void) {
  return guarded([&] {
    if (g_occSt) MMX_HIP(hipStreamSynchronize(g_occSt));
  });
}

int mmx_matrix_destroy(mmx_matrix m) {
  if (!m) return MMADMM_OK;
  delete m->m;
  delete m;
  return MMADMM_OK;
}

}  // extern "C"
