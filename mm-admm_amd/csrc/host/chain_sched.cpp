// chain_sched.cpp -- see chain_sched.h.
#include "chain_sched.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <queue>
#include <unordered_map>
#include <cstdint>

namespace mmx {

namespace {
// MMX_SCHED_PROF=1: the builders' phase times on stderr (host set-up of the first backward-Euler step)
struct PhaseClock {
  bool on;
  const char* who;
  std::chrono::steady_clock::time_point t;
  explicit PhaseClock(const char* w) : on(getenv("MMX_SCHED_PROF") != nullptr), who(w), t(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[sched] %s %s %.3f s\n", who, what, std::chrono::duration<double>(n - t).count());
    t = n;
  }
};
constexpr int kChainLenCap = 1 << 20;  // longest chain (positions fit the schedule's ints)
// iterations a global value takes to reach another band (model; MMX_CHAIN_LAT overrides)
static int import_latency() {
  static int v = [] {
    const char* e = getenv("MMX_CHAIN_LAT");
    return e ? std::max(0, atoi(e)) : 8;
  }();
  return v;
}
int pow2_at_least(int v) {
  int r = 1;
  while (r < v) r <<= 1;
  return r;
}
// Import slots for imports in order of first use (first[ord[q]] ascending): every one of the RI
// slots is used once before any is taken again, and then the slot whose last reader passed
// longest ago is taken (it waits for the compute wave to pass that reader): the importer may run
// as far ahead as the slots allow, and a band needs at most as many slots as it has imports live
// at once.  False when RI slots are too few.
bool assign_import_slots(const std::vector<int>& first, const std::vector<int>& last, const std::vector<int>& ord,
                         int RI, std::vector<int>& slotOf, std::vector<int>& waitOf, int& used) {
  typedef std::pair<int, int> P;  // (last use, slot)
  std::priority_queue<P, std::vector<P>, std::greater<P>> busy;
  std::queue<int> freed;  // slots whose last reader has passed, in the order they were freed
  std::vector<int> slotLast;
  slotOf.assign(ord.size(), 0);
  waitOf.assign(ord.size(), -1);
  for (size_t q = 0; q < ord.size(); ++q) {
    const int f = first[ord[q]];
    while (!busy.empty() && busy.top().first < f) {
      freed.push(busy.top().second);
      busy.pop();
    }
    int sl;
    if ((int)slotLast.size() < RI) {
      sl = (int)slotLast.size();
      slotLast.push_back(-1);
    } else if (!freed.empty()) {
      sl = freed.front();
      freed.pop();
    } else {
      return false;
    }
    slotOf[q] = sl;
    waitOf[q] = slotLast[sl];
    slotLast[sl] = last[ord[q]];
    busy.push({last[ord[q]], sl});
  }
  used = (int)slotLast.size();
  return true;
}
}  // namespace

void big_fill(BigVec& v, size_t n, int x) {
  BigVec().swap(v);
  v.resize(n);  // uninitialised (NoInitAlloc)
  int* p = v.data();
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; ++i) p[i] = x;
}

ChainSchedule build_chain_schedule(int n, const std::vector<int>& iaf, const std::vector<int>& jaf,
                                   const std::vector<int>& dg, bool fwd, int forceG, bool codes) {
  ChainSchedule S;
  S.fwd = fwd;
  PhaseClock pc(fwd ? "fwd" : "bwd");
  auto rb = [&](int i) { return fwd ? iaf[i] : dg[i] + 1; };
  auto re = [&](int i) { return fwd ? dg[i] : iaf[i + 1]; };
  int emax = 0;
  for (int i = 0; i < n; ++i) emax = std::max(emax, re(i) - rb(i));
  // rows wider than 32 entries (3D) are split into segments of E = 32 entries computed at
  // consecutive positions of their lane (the partial sum carried in a register, so the order of
  // the subtractions is unchanged); every row of a chain takes the chain's segment count ns.
  // Narrower rows (2D) are computed two per position (G = 2): the chain's next row takes the
  // first one's value straight from the register (MMX_CHAIN_PAIR=0: one row per position).
  {
    const char* we = getenv("MMX_CHAIN_E48");
    const bool wide = emax > 32 && emax <= kChainWideE && !(we && atoi(we) == 0);
    S.E = emax <= 8 ? 8 : emax <= 16 ? 16 : emax <= 32 ? 32 : wide ? kChainWideE : 32;
    S.seg = emax > 32 && !wide;
  }
  if (emax > kChainSegMax * 32) {
    S.why = "a row has more than " + std::to_string(kChainSegMax * 32) + " entries in the triangle";
    return S;
  }
  {
    const char* pe = getenv("MMX_CHAIN_PAIR");
    S.G = (!S.seg && S.E <= 16 && !(pe && atoi(pe) == 0)) ? 2 : 1;
    if (forceG == 1 || (forceG == 2 && !S.seg && S.E <= 16)) S.G = forceG;
  }
  const int G = S.G, E = S.E, EE = E * G;
  auto nsRow = [&](int i) { return S.seg ? std::max(1, (re(i) - rb(i) + E - 1) / E) : 1; };
  // chains in processing order (forward: ascending rows; backward: descending); a chain also ends
  // where the segment count changes, so no row pays for a wider neighbour's segments
  std::vector<int> chainOf(n), rowIdx(n), cStart, cRows, cNs;
  for (int t = 0; t < n; ++t) {
    const int i = fwd ? t : n - 1 - t;
    const int b = rb(i), e = re(i), ns = nsRow(i);
    const bool cont = t > 0 && cRows.back() < kChainLenCap && cNs.back() == ns &&
                      (fwd ? (e > b && jaf[e - 1] == i - 1) : (e > b && jaf[b] == i + 1));
    if (!cont) {
      cStart.push_back(i);
      cRows.push_back(0);
      cNs.push_back(ns);
    }
    chainOf[i] = (int)cStart.size() - 1;
    rowIdx[i] = cRows.back()++;
  }
  const int C = (int)cStart.size();
  pc.mark("chains");
  // positions: a row's value is final at posOf (its last segment / its pair's position); ringOf
  // is the row's sequence number in its lane's LDS ring
  std::vector<int> cLen(C), posOf(n), ringOf(n);
  for (int c = 0; c < C; ++c) cLen[c] = (G == 2) ? (cRows[c] + 1) / 2 : cRows[c] * cNs[c];
  for (int i = 0; i < n; ++i) {
    const int c = chainOf[i];
    posOf[i] = (G == 2) ? rowIdx[i] / 2 : rowIdx[i] * cNs[c] + cNs[c] - 1;
    ringOf[i] = (G == 2) ? rowIdx[i] : posOf[i];
  }
  S.nchains = C;
  S.nbands = (C + kChainLanes - 1) / kChainLanes;
  const int L = kChainLanes;
  S.laneStart.assign((size_t)S.nbands * L, 0);
  S.laneLen.assign((size_t)S.nbands * L, 0);
  S.laneSkew.assign((size_t)S.nbands * L, 0);
  S.laneNs.assign((size_t)S.nbands * L, 1);
  S.bandSlot.assign(S.nbands, 0);
  S.bandT.assign(S.nbands, 0);
  S.bandImp.assign(S.nbands, 0);
  S.bandNImp.assign(S.nbands, 0);
  // part g of position p of chain c: its row (-1: none) and segment q, entries [kb, ke)
  auto part = [&](int c, int p, int g, int& q, int& kb, int& ke) {
    int ri;
    if (G == 2) {
      ri = 2 * p + g;
      q = 0;
      if (ri >= cRows[c]) return -1;
    } else {
      if (g > 0) return -1;
      ri = p / cNs[c];
      q = p % cNs[c];
    }
    const int i = fwd ? cStart[c] + ri : cStart[c] - ri;
    kb = rb(i) + q * E;
    ke = std::min(re(i), kb + E);
    return i;
  };

  // pass 1: skews and band lengths, with a model of the critical path: band b starts at iteration
  // offset[b] (not before band b - 1), a row is published at offset + position + skew + 1 and an
  // import reaches another band kImportLatency iterations later.  Plain skews satisfy only the
  // band's own dependencies (the band then waits for late imports); aligned skews also delay each
  // lane until its imports are due (3D: a band's chains span planes whose imports arrive at very
  // different times).  MMX_CHAIN_ALIGN=0/1 forces one; by default the shorter modelled path wins.
  struct Pass1 {  // one modelled schedule: lane skews, band lengths and offsets
    std::vector<int> laneSkew, bandT;
    std::vector<long long> doneAt, offset;
    long long est = 0;
  };
  auto pass1 = [&](bool align, Pass1& P) {
    P.laneSkew.assign((size_t)S.nbands * L, 0);
    P.bandT.assign(S.nbands, 0);
    P.doneAt.assign(n, -1);
    P.offset.assign(S.nbands, 0);
    std::vector<int>& laneSkew = P.laneSkew;
    std::vector<long long>& doneAt = P.doneAt;
    std::vector<long long>& offset = P.offset;
    long long est = 0;
    for (int b = 0; b < S.nbands; ++b) {
      const int c0 = b * L, nl = std::min(L, C - c0);
      const long long off0 = b > 0 ? offset[b - 1] : 0;
      long long off = off0;
      int T = 0, minSk = INT32_MAX;
      for (int l = 0; l < nl; ++l) {
        const int c = c0 + l;
        long long sk = 0;
        for (int p = 0; p < cLen[c]; ++p)
          for (int g = 0; g < G; ++g) {
            int q, kb, ke;
            if (part(c, p, g, q, kb, ke) < 0) continue;
            for (int k = kb; k < ke; ++k) {
              const int j = jaf[k], cj = chainOf[j];
              if (cj >= c0 && cj < c) {
                sk = std::max<long long>(sk, laneSkew[(size_t)b * L + (cj - c0)] + posOf[j] - p + 1);
              } else if (align && cj < c0 && doneAt[j] >= 0) {
                sk = std::max<long long>(sk, doneAt[j] + import_latency() - off0 - p);
              }
            }
          }
        if (sk > kChainLenCap) sk = kChainLenCap;
        laneSkew[(size_t)b * L + l] = (int)sk;
        minSk = std::min(minSk, (int)sk);
      }
      if (align && nl > 0 && minSk > 0) {  // start the band later rather than idle its lanes
        for (int l = 0; l < nl; ++l) laneSkew[(size_t)b * L + l] -= minSk;
        off += minSk;
      }
      for (int l = 0; l < nl; ++l) {
        const int c = c0 + l, sk = laneSkew[(size_t)b * L + l];
        T = std::max(T, sk + cLen[c]);
        if (!align)  // the band waits for its late imports
          for (int p = 0; p < cLen[c]; ++p)
            for (int g = 0; g < G; ++g) {
              int q, kb, ke;
              if (part(c, p, g, q, kb, ke) < 0) continue;
              for (int k = kb; k < ke; ++k) {
                const int j = jaf[k];
                if (chainOf[j] < c0 && doneAt[j] >= 0) off = std::max(off, doneAt[j] + import_latency() - (p + sk));
              }
            }
      }
      offset[b] = off;
      for (int l = 0; l < nl; ++l) {
        const int c = c0 + l, sk = laneSkew[(size_t)b * L + l];
        for (int r = 0; r < cRows[c]; ++r) {
          const int i = fwd ? cStart[c] + r : cStart[c] - r;
          doneAt[i] = off + posOf[i] + sk + 1;
        }
      }
      P.bandT[b] = T;
      est = std::max(est, off + T);
    }
    P.est = est;
  };
  {
    // MMX_CHAIN_ALIGN=0/1 forces one; by default both are modelled (concurrently) and the shorter
    // critical path wins
    const char* ae = getenv("MMX_CHAIN_ALIGN");
    const int mode = ae ? atoi(ae) : -1;
    Pass1 P0, P1;
    if (mode >= 0) {
      pass1(mode != 0, P0);
      S.aligned = mode != 0;
    } else {
#pragma omp parallel sections num_threads(2)
      {
#pragma omp section
        pass1(false, P0);
#pragma omp section
        pass1(true, P1);
      }
      S.aligned = P1.est < P0.est;
      if (S.aligned) std::swap(P0, P1);
    }
    S.estIters = P0.est;
    S.laneSkew.swap(P0.laneSkew);
    S.bandT.swap(P0.bandT);
  }
  pc.mark("pass1");
  // lane arrays, slots, ring distances (a ring slot of a lane is written again R / G positions
  // after it is written); a value further back than the ring holds is imported
  int maxDist = 1;
  const int ringCap = E > 32 ? kChainRingWide : kChainRingMax;
  for (int b = 0; b < S.nbands; ++b) {
    const int c0 = b * L, nl = std::min(L, C - c0);
    for (int l = 0; l < nl; ++l) {
      const int c = c0 + l, sk = S.laneSkew[(size_t)b * L + l];
      S.laneStart[(size_t)b * L + l] = cStart[c];
      S.laneLen[(size_t)b * L + l] = (G == 2) ? cRows[c] : cLen[c];  // pairs: rows; else positions
      S.laneNs[(size_t)b * L + l] = cNs[c];
      S.maxSkew = std::max(S.maxSkew, sk);
      S.maxLen = std::max(S.maxLen, cLen[c]);
    }
    for (int l = 0; l < nl; ++l) {
      const int c = c0 + l, skl = S.laneSkew[(size_t)b * L + l];
      for (int p = 0; p < cLen[c]; ++p)
        for (int g = 0; g < G; ++g) {
          int q, kb, ke;
          if (part(c, p, g, q, kb, ke) < 0) continue;
          for (int k = kb; k < ke; ++k) {
            const int j = jaf[k], cj = chainOf[j];
            if (cj < c0 || cj > c) continue;
            const int d = (p + skl) - (posOf[j] + S.laneSkew[(size_t)b * L + (cj - c0)]);
            if (d >= 1 && d * G <= ringCap) maxDist = std::max(maxDist, d * G);
          }
        }
    }
    S.bandSlot[b] = (int)S.slots;
    S.slots += S.bandT[b];
    S.maxT = std::max(S.maxT, S.bandT[b]);
  }
  if (S.slots * L * EE > (long long)INT32_MAX) {
    S.why = "schedule too large";
    return S;
  }
  S.R = std::max(2 * G, pow2_at_least(maxDist));
  const int R = S.R;
  pc.mark("ring");

  // pass 2: codes, value sources, imports
  const size_t ne = codes ? (size_t)S.slots * L * EE : 0;
  big_fill(S.code, ne, kChainPad);
  S.impNeed.assign(codes ? (size_t)S.slots : 0, -1);
  S.bandE.assign(S.nbands, 4);
  big_fill(S.src, ne, -1);
  if (!fwd && codes) S.dsrc.assign((size_t)S.slots * G * L, -1);
  pc.mark("alloc");
  std::vector<std::vector<int>> srcBands(S.nbands);  // bands each band imports from
  // the importer runs at most RI imports ahead of the compute wave: it takes the whole ring (a
  // band importing hundreds of values per iteration needs many iterations of run-ahead)
  const int RI = kChainImpMax;
  struct BandOut {  // per band: its imports in order of first use, or why it failed
    std::vector<int> row, free, slot, wait;
    int used = 0;
    bool bad = false;
  };
  std::vector<BandOut> bout(S.nbands);
  // bands are independent here (disjoint slots of the code / source arrays, their own imports):
  // in parallel, each thread with its own row -> import map; the imports are listed in band order
  // after the loop, exactly as a sequential walk lists them
#pragma omp parallel
  {
    std::vector<int> impOf(n, -1), first, last, rows;
#pragma omp for schedule(dynamic, 8)
    for (int b = 0; b < S.nbands; ++b) {
      const int c0 = b * L, nl = std::min(L, C - c0);
      first.clear();
      last.clear();
      rows.clear();
      struct Use {
        size_t slot;
        int row;
      };
      std::vector<Use> impUses;
      for (int l = 0; l < nl; ++l) {
        const int c = c0 + l, skl = S.laneSkew[(size_t)b * L + l];
        for (int p = 0; p < cLen[c]; ++p)
          for (int g = 0; g < G; ++g) {
            int q, kb, ke;
            const int i = part(c, p, g, q, kb, ke);
            if (i < 0) continue;
            const int t = p + skl;
            const size_t base = ((size_t)(S.bandSlot[b] + t) * EE + (size_t)g * E) * L + l;  // [slot][g][e][lane]
            if (codes && !fwd && q == cNs[c] - 1) S.dsrc[((size_t)(S.bandSlot[b] + t) * G + g) * L + l] = dg[i];
            int e = 0;
            S.bandE[b] = std::max(S.bandE[b], (std::max(ke - kb, 0) + 3) / 4 * 4);
            for (int k = kb; k < ke; ++k, ++e) {
              const int j = jaf[k], cj = chainOf[j];
              const size_t x = base + (size_t)e * L;
              if (codes) S.src[x] = k;
              bool ring = false;
              if (cj == c && posOf[j] == p) {  // the pair's first row, taken from the register
                if (codes) S.code[x] = kChainFwd;
                ring = true;
              } else if (cj >= c0 && cj <= c) {
                const int lj = cj - c0;
                const int d = t - (posOf[j] + S.laneSkew[(size_t)b * L + lj]);
                if (d * G <= R) {
                  if (codes) S.code[x] = lj * (R + 1) + (ringOf[j] & (R - 1));
                  ring = true;
                }
              }
              if (!ring) {
                int& id = impOf[j];
                if (id < 0) {
                  id = (int)rows.size();
                  rows.push_back(j);
                  first.push_back(t);
                  last.push_back(t);
                }
                first[id] = std::min(first[id], t);
                last[id] = std::max(last[id], t);
                if (codes) impUses.push_back({x, j});
              }
            }
          }
      }
      // imports in order of first use
      std::vector<int> ord(rows.size());
      for (size_t q = 0; q < ord.size(); ++q) ord[q] = (int)q;
      std::sort(ord.begin(), ord.end(), [&](int a, int c) {
        return first[a] != first[c] ? first[a] < first[c] : rows[a] < rows[c];
      });
      std::vector<int> rank(rows.size());
      for (size_t q = 0; q < ord.size(); ++q) rank[ord[q]] = (int)q;
      std::vector<int> slotOf, waitOf;
      BandOut& bo = bout[b];
      bo.bad = !assign_import_slots(first, last, ord, RI, slotOf, waitOf, bo.used);
      if (!bo.bad) {
        for (const Use& u : impUses) {
          const int k = rank[impOf[u.row]];
          S.code[u.slot] = -(slotOf[k] + 1);
          const size_t it = u.slot / ((size_t)EE * L);  // slot (iteration) of the use
          S.impNeed[it] = std::max(S.impNeed[it], k);
        }
        for (int j : rows) srcBands[b].push_back(chainOf[j] / L);
        std::sort(srcBands[b].begin(), srcBands[b].end());
        srcBands[b].erase(std::unique(srcBands[b].begin(), srcBands[b].end()), srcBands[b].end());
        for (size_t q = 0; q < ord.size(); ++q) {
          const int id = ord[q];
          bo.row.push_back(rows[id]);
          bo.free.push_back(last[id]);
          bo.slot.push_back(slotOf[q]);
          bo.wait.push_back(waitOf[q]);
        }
      }
      for (int j : rows) impOf[j] = -1;
    }
  }
  for (int b = 0; b < S.nbands; ++b) {
    const BandOut& bo = bout[b];
    if (bo.bad) {
      S.why = "import ring too small for band " + std::to_string(b);
      return S;
    }
    S.maxImpSlots = std::max(S.maxImpSlots, bo.used);
    S.bandImp[b] = (int)S.impRow.size();
    S.bandNImp[b] = (int)bo.row.size();
    S.impRow.insert(S.impRow.end(), bo.row.begin(), bo.row.end());
    S.impFree.insert(S.impFree.end(), bo.free.begin(), bo.free.end());
    S.impSlot.insert(S.impSlot.end(), bo.slot.begin(), bo.slot.end());
    S.impWait.insert(S.impWait.end(), bo.wait.begin(), bo.wait.end());
  }
  S.RI = RI;
  S.nImports = (long long)S.impRow.size();
  pc.mark("pass2");
  // ticket order: a band becomes available once every band it imports from has a ticket; among the
  // available bands the longest (most iterations) goes first, then the lowest index.  The long
  // bands carry the critical path (in the backward sweep they come last by index, behind thousands
  // of one-iteration bands they barely depend on).
  {
    std::vector<std::vector<int>> users(S.nbands);
    std::vector<int> pending(S.nbands, 0);
    for (int b = 0; b < S.nbands; ++b)
      for (int a : srcBands[b])
        if (a != b) {
          users[a].push_back(b);
          ++pending[b];
        }
    auto later = [&](int a, int c) { return S.bandT[a] != S.bandT[c] ? S.bandT[a] < S.bandT[c] : a > c; };
    std::priority_queue<int, std::vector<int>, decltype(later)> avail(later);
    for (int b = 0; b < S.nbands; ++b)
      if (pending[b] == 0) avail.push(b);
    S.bandOrder.clear();
    while (!avail.empty()) {
      const int b = avail.top();
      avail.pop();
      S.bandOrder.push_back(b);
      for (int c : users[b])
        if (--pending[c] == 0) avail.push(c);
    }
    if ((int)S.bandOrder.size() != S.nbands) {
      S.why = "band import cycle";
      return S;
    }
  }
  // codes -> LDS indices: 0 zero cell, 1 + ring index, 1 + 64 (R + 1) + import slot; the pair's
  // forwarded entry: the cell after the import slots (never read: the kernel takes the register)
  const int impBase = 1 + L * (R + 1);
#pragma omp parallel for schedule(static)
  for (size_t x = 0; x < S.code.size(); ++x) {
    int& c = S.code[x];
    c = (c == kChainPad) ? 0 : (c == kChainFwd) ? impBase + RI : (c >= 0 ? 1 + c : impBase + (-c - 1));
  }
  pc.mark("order+codes");
  S.ok = true;
  return S;
}

std::string validate_chain_schedule(const ChainSchedule& S, int n, const std::vector<int>& iaf,
                                    const std::vector<int>& jaf, const std::vector<int>& dg) {
  if (!S.ok) return "schedule not built: " + S.why;
  const int L = kChainLanes, E = S.E, R = S.R, G = S.G, EE = E * G;
  const bool fwd = S.fwd;
  if (G != 1 && G != 2) return "bad rows per position";
  if (G == 2 && S.seg) return "pairs of segmented rows";
  if (E != 8 && E != 16 && E != 32 && E != kChainWideE) return "no kernel for this stage width";
  if (R < 1 || (R & (R - 1)) || R > (E > 32 ? kChainRingWide : kChainRingMax)) return "ring larger than the kernel's";
  if (E > 32 && (S.seg || G != 1)) return "wide stages with segments or pairs";
  if (1 + L * (R + 1) + S.RI >= 65536) return "stage codes do not fit 16 bits";  // (the kernel's codes are 16-bit)
  // where every row is computed: band, lane, position of its final value, ring sequence number,
  // part (pair half), segments
  std::vector<int> bandOf(n, -1), laneOf(n, -1), posOf(n, -1), ringOf(n, -1), partOf(n, 0), iterOf(n, -1),
      nsOf(n, 1);
  if (S.laneNs.size() != S.laneLen.size()) return "segment counts missing";
  for (int b = 0; b < S.nbands; ++b)
    for (int l = 0; l < L; ++l) {
      const size_t g = (size_t)b * L + l;
      const int ns = S.laneNs[g];
      if (ns < 1 || ns > kChainSegMax || (ns > 1 && !S.seg)) return "bad segment count";
      if (G == 1 && S.laneLen[g] % ns) return "lane length not a whole number of rows";
      const int nrows = (G == 2) ? S.laneLen[g] : S.laneLen[g] / ns;
      for (int r = 0; r < nrows; ++r) {
        const int i = fwd ? S.laneStart[g] + r : S.laneStart[g] - r;
        if (i < 0 || i >= n) return "row out of range";
        if (bandOf[i] >= 0) return "row " + std::to_string(i) + " scheduled twice";
        bandOf[i] = b;
        laneOf[i] = l;
        posOf[i] = (G == 2) ? r / 2 : r * ns + ns - 1;
        ringOf[i] = (G == 2) ? r : posOf[i];
        partOf[i] = (G == 2) ? r % 2 : 0;
        nsOf[i] = ns;
        iterOf[i] = posOf[i] + S.laneSkew[g];
        if (iterOf[i] >= S.bandT[b]) return "row beyond its band's iterations";
      }
    }
  for (int i = 0; i < n; ++i)
    if (bandOf[i] < 0) return "row " + std::to_string(i) + " never scheduled";
  // tickets: every band once, after every band it imports from (the importers never wait on a band
  // that has no workgroup yet)
  if ((int)S.bandOrder.size() != S.nbands) return "band order size";
  std::vector<int> ticketOf(S.nbands, -1);
  for (int q = 0; q < S.nbands; ++q) {
    const int b = S.bandOrder[q];
    if (b < 0 || b >= S.nbands || ticketOf[b] >= 0) return "band order is not a permutation";
    ticketOf[b] = q;
  }
  for (int b = 0; b < S.nbands; ++b)
    for (int q = 0; q < S.bandNImp[b]; ++q) {
      const int j = S.impRow[(size_t)S.bandImp[b] + q];
      if (bandOf[j] != b && ticketOf[bandOf[j]] > ticketOf[b]) return "band imports from a later ticket";
    }
  // per band: import index of each imported row; per import: the next import of its slot
  std::vector<std::unordered_map<int, int>> impOfRow(S.nbands);
  std::vector<int> nextInSlot(S.impRow.size(), -1);
  if (S.impSlot.size() != S.impRow.size() || S.impWait.size() != S.impRow.size()) return "import slots missing";
  for (int b = 0; b < S.nbands; ++b) {
    std::unordered_map<int, int> lastInSlot;
    for (int q = 0; q < S.bandNImp[b]; ++q) {
      const size_t g = (size_t)S.bandImp[b] + q;
      if (!impOfRow[b].emplace(S.impRow[g], q).second) return "row imported twice by one band";
      auto ls = lastInSlot.find(S.impSlot[g]);
      if (ls != lastInSlot.end()) {
        nextInSlot[(size_t)S.bandImp[b] + ls->second] = q;
        if (S.impWait[g] != S.impFree[(size_t)S.bandImp[b] + ls->second]) return "import does not wait for its slot";
      } else if (S.impWait[g] != -1) {
        return "first import of a slot waits";
      }
      lastInSlot[S.impSlot[g]] = q;
    }
  }
  const int impBase = 1 + L * (R + 1), fwdCell = impBase + S.RI;
  for (int i = 0; i < n; ++i) {
    const int b = bandOf[i], l = laneOf[i], ns = nsOf[i], gp = partOf[i];
    const int kb0 = fwd ? iaf[i] : dg[i] + 1, ke0 = fwd ? dg[i] : iaf[i + 1];
    if (ke0 - kb0 > E * ns) return "row wider than its segments";
    for (int sg = 0; sg < ns; ++sg) {
      const int t = iterOf[i] - (ns - 1) + sg;  // segment sg of the row
      const size_t base = ((size_t)(S.bandSlot[b] + t) * EE + (size_t)gp * E) * L + l;
      const int kb = kb0 + sg * E, ke = std::min(ke0, kb + E);
      if (!fwd && S.dsrc[((size_t)(S.bandSlot[b] + t) * G + gp) * L + l] != (sg == ns - 1 ? dg[i] : -1))
        return "diagonal source";
      for (int e = 0; e < E; ++e) {
        const size_t x = base + (size_t)e * L;
        const int k = kb + e;
        if (k >= ke) {
          if (S.code[x] != 0 || S.src[x] != -1) return "pad slot in use";
          continue;
        }
        if (e >= S.bandE[b]) return "entry beyond the band's entry count";
        if (S.src[x] != k) return "entry order differs from the reference";
        const int j = jaf[k], c = S.code[x];
        if (c <= 0) return "missing entry";
        if (c == fwdCell) {  // the pair's first row, from the register
          if (gp != 1 || bandOf[j] != b || laneOf[j] != l || posOf[j] != posOf[i] || partOf[j] != 0)
            return "forwarded entry is not the pair's first row";
        } else if (c < impBase) {
          const int r = c - 1, lp = r / (R + 1), slot = r % (R + 1);
          if (bandOf[j] != b || laneOf[j] != lp || (ringOf[j] & (R - 1)) != slot) return "ring slot of another row";
          if (iterOf[j] >= t) return "ring value read before it is written";
          // the slot is written again by the lane's row with ring number ringOf[j] + R, at its
          // position; a read in that same iteration comes first
          const size_t gl = (size_t)b * L + lp;
          const int over = ringOf[j] + R;
          const int overPos = (G == 2) ? over / 2 : over;
          const int lenRows = (G == 2) ? S.laneLen[gl] : S.laneLen[gl];
          if (over < lenRows && overPos + S.laneSkew[gl] < t) return "ring value overwritten before it is read";
        } else {
          // the import: the one of this band whose slot matches and whose row is j
          const int slot = c - impBase;
          if (slot >= S.RI) return "import slot out of range";
          auto it = impOfRow[b].find(j);
          if (it == impOfRow[b].end()) return "import of a row the band does not import";
          const int k2 = it->second;
          const size_t q = (size_t)S.bandImp[b] + k2;
          if (S.impSlot[q] != slot) return "import read from another slot";
          if (S.impNeed[(size_t)S.bandSlot[b] + t] < k2) return "iteration does not wait for its import";
          if (S.impFree[q] < t) return "import read after its slot is released";
          // no deadlock: every use (the first included) comes after the import's wait, and imports
          // are in order of first use, so every import iteration t waits for is deliverable by then
          if (S.impWait[q] >= t) return "import delivered only after it is read";
          const int nx = nextInSlot[q];  // the slot's next import is delivered after this read
          if (nx >= 0 && S.impWait[(size_t)S.bandImp[b] + nx] < t) return "import read after its slot is taken again";
          if (bandOf[j] == b && iterOf[j] >= t) return "import read before it is written";
        }
      }
    }
  }
  return "";
}

FactorSchedule build_factor_schedule(int n, const std::vector<int>& iaf, const std::vector<int>& jaf,
                                     const std::vector<int>& dg) {
  FactorSchedule F;
  for (int i = 0; i < n; ++i) {
    const int W = iaf[i + 1] - iaf[i], nl = dg[i] - iaf[i];
    if (W > kFacWF || nl > kFacNL || W - nl > kFacWU) {
      F.why = "row " + std::to_string(i) + " wider than the factor's row layout";
      return F;
    }
  }
  PhaseClock pc("factor");
  F.geo = build_chain_schedule(n, iaf, jaf, dg, true, 1, false);  // its geometry (no stage codes)
  pc.mark("geometry");
  ChainSchedule& S = F.geo;
  if (!S.ok) {
    F.why = "forward chain schedule: " + S.why;
    return F;
  }
  if (S.seg || S.G != 1) {
    F.why = "segmented schedule";
    return F;
  }
  const int L = kChainLanes;
  const char* fr = getenv("MMX_FAC_R");
  const int R = std::min(std::min(S.R, kFacRMax), fr ? atoi(fr) : kFacRMax);  // ring slots per lane (rows)
  if (R != 1 && R != 2 && R != 4) {  // the ring is indexed p & (R - 1): a power of two, at most kFacRMax
    F.why = "factor ring size " + std::to_string(R) + " not in {1, 2, 4}";
    return F;
  }
  F.R = R;
  F.slots = S.slots;
  // where every row is: band, lane, position, iteration
  std::vector<int> bandOf(n, -1), laneOf(n, -1), posOf(n, -1);
  for (int b = 0; b < S.nbands; ++b)
    for (int l = 0; l < L; ++l) {
      const size_t g = (size_t)b * L + l;
      for (int p = 0; p < S.laneLen[g]; ++p) {
        const int i = S.laneStart[g] + p;
        bandOf[i] = b;
        laneOf[i] = l;
        posOf[i] = p;
      }
    }
  const size_t nslot = (size_t)S.slots;
  pc.mark("positions");
  {
    const size_t nc = nslot * kFacNSC * L;
    F.code.resize(nc);  // uninitialised, then zeroed in parallel
    uint16_t* cp = F.code.data();
#pragma omp parallel for schedule(static)
    for (size_t x = 0; x < nc; ++x) cp[x] = 0;
  }
  big_fill(F.vsrc, nslot * kFacWF * L, -1);
  F.meta.assign(nslot * L, 0);
  F.rowStart.assign(nslot * L, 0);
  F.impNeed.assign(nslot, -1);
  F.bandImp.assign(S.nbands, 0);
  F.bandNImp.assign(S.nbands, 0);
  const char* fri = getenv("MMX_FAC_RI");
  const int RI = fri ? std::max(1, std::min(atoi(fri), kFacImpRows)) : kFacImpRows;  // s_dep holds kFacImpRows
  F.RI = RI;
  const int impBase = 1 + L * (R + 1) * kFacWU;
  struct Use {
    size_t cell;
    int id, u;  // import, offset in the row's diagonal + upper part
  };
  struct BandOut {  // per band: its imports in order, or why it failed
    std::vector<int> row, free, slot, wait;
    int slots = 0;
    bool bad = false;
  };
  std::vector<BandOut> out(S.nbands);
  pc.mark("alloc");
  // bands are independent (disjoint slots of the code arrays; imports per band): in parallel
#pragma omp parallel
  {
  std::vector<int> impOf(n, -1);  // imported row -> import id (this thread's current band)
#pragma omp for schedule(dynamic, 16)
  for (int b = 0; b < S.nbands; ++b) {
    std::vector<int> rows, first, last;  // per import id: row, first and last use
    std::vector<Use> uses;
    BandOut& bo = out[b];
    for (int l = 0; l < L; ++l) {
      const size_t g = (size_t)b * L + l;
      const int skl = S.laneSkew[g];
      for (int p = 0; p < S.laneLen[g]; ++p) {
        const int i = S.laneStart[g] + p, t = p + skl;
        const size_t slot = (size_t)S.bandSlot[b] + t;
        const int kb = iaf[i], W = iaf[i + 1] - kb, nl = dg[i] - kb;
        F.meta[slot * L + l] = W | (nl << 8) | (1 << 16);
        F.rowStart[slot * L + l] = kb;
        for (int e = 0; e < W; ++e) F.vsrc[fac_vidx(slot, e, l)] = kb + e;
        // the LDS index of U(j, .) at factor position pos (the caller found it) for the row at
        // iteration t
        auto value = [&](int j, int pos, size_t cell) {
          if (bandOf[j] == b && laneOf[j] <= l) {
            const size_t gj = (size_t)b * L + laneOf[j];
            const int d = t - (posOf[j] + S.laneSkew[gj]);
            if (d >= 1 && d <= R) {
              F.code[cell] = (uint16_t)(1 + (laneOf[j] * (R + 1) + (posOf[j] & (R - 1))) * kFacWU + (pos - dg[j]));
              return;
            }
          }
          int& id = impOf[j];
          if (id < 0) {
            id = (int)rows.size();
            rows.push_back(j);
            first.push_back(t);
            last.push_back(t);
          }
          first[id] = std::min(first[id], t);
          last[id] = std::max(last[id], t);
          uses.push_back({cell, id, pos - dg[j]});
        };
        for (int q = 0; q < nl; ++q) {
          const int j = jaf[kb + q];
          value(j, dg[j], fac_cidx(slot, kFacNUpd + q, l));  // the pivot U(j, j)
          // the targets of pivot q: entries e > q whose column lies in row j's upper part (both
          // column lists ascending: one merge walk)
          const int* f = jaf.data() + dg[j] + 1;
          const int* ue = jaf.data() + iaf[j + 1];
          for (int e = q + 1; e < W && f != ue; ++e) {
            const int c = jaf[kb + e];
            if (c <= j) continue;
            while (f != ue && *f < c) ++f;
            if (f != ue && *f == c) value(j, (int)(f - jaf.data()), fac_cidx(slot, fac_slot(e, q), l));
          }
        }
      }
    }
    // imports in order of first use, slots as in build_chain_schedule
    std::vector<int> ord(rows.size());
    for (size_t q = 0; q < ord.size(); ++q) ord[q] = (int)q;
    std::sort(ord.begin(), ord.end(), [&](int a, int c) { return first[a] != first[c] ? first[a] < first[c] : rows[a] < rows[c]; });
    std::vector<int> rank(rows.size()), slotOf, waitOf;
    for (size_t q = 0; q < ord.size(); ++q) rank[ord[q]] = (int)q;
    int used = 0;
    bo.bad = !assign_import_slots(first, last, ord, RI, slotOf, waitOf, used);
    if (bo.bad) {
      for (int j : rows) impOf[j] = -1;
      continue;
    }
    bo.slots = used;
    for (const Use& u : uses) {
      const int k = rank[u.id];
      F.code[u.cell] = (uint16_t)(impBase + slotOf[k] * kFacWU + u.u);
      const size_t it = u.cell / ((size_t)kFacNSC * L);
      F.impNeed[it] = std::max(F.impNeed[it], k);
    }
    for (size_t q = 0; q < ord.size(); ++q) {
      bo.row.push_back(rows[ord[q]]);
      bo.free.push_back(last[ord[q]]);
      bo.slot.push_back(slotOf[q]);
      bo.wait.push_back(waitOf[q]);
    }
    for (int j : rows) impOf[j] = -1;
  }
  }
  pc.mark("bands");
  for (int b = 0; b < S.nbands; ++b) {
    const BandOut& bo = out[b];
    if (bo.bad) {
      F.why = "import slots too few for band " + std::to_string(b);
      return F;
    }
    F.maxImpSlots = std::max(F.maxImpSlots, bo.slots);
    F.bandImp[b] = (int)F.impRow.size();
    F.bandNImp[b] = (int)bo.row.size();
    F.impRow.insert(F.impRow.end(), bo.row.begin(), bo.row.end());
    F.impFree.insert(F.impFree.end(), bo.free.begin(), bo.free.end());
    F.impSlot.insert(F.impSlot.end(), bo.slot.begin(), bo.slot.end());
    F.impWait.insert(F.impWait.end(), bo.wait.begin(), bo.wait.end());
  }
  if (impBase + RI * kFacWU >= 65536) {
    F.why = "LDS indices exceed 16 bits";
    return F;
  }
  // a band imports only from bands with earlier tickets (the forward sweep's order already puts
  // every band after the bands its rows depend on, which are the bands its imports come from)
  {
    std::vector<int> ticketOf(S.nbands);
    for (int q = 0; q < S.nbands; ++q) ticketOf[S.bandOrder[q]] = q;
    for (int b = 0; b < S.nbands; ++b)
      for (int q = 0; q < F.bandNImp[b]; ++q) {
        const int j = F.impRow[(size_t)F.bandImp[b] + q];
        if (bandOf[j] != b && ticketOf[bandOf[j]] > ticketOf[b]) {
          F.why = "factor band imports from a later ticket";
          return F;
        }
      }
  }
  F.nImports = (long long)F.impRow.size();
  // rows some band imports publish their diagonal + upper part as global granules (bit 17 of
  // meta); the others are read through the lane rings only and skip those stores
  {
    std::vector<char> exported(n, 0);
    for (int j : F.impRow) exported[j] = 1;
    for (int b = 0; b < S.nbands; ++b)
      for (int l = 0; l < L; ++l) {
        const size_t g = (size_t)b * L + l;
        for (int p = 0; p < S.laneLen[g]; ++p) {
          const int i = S.laneStart[g] + p;
          if (exported[i]) F.meta[((size_t)S.bandSlot[b] + p + S.laneSkew[g]) * L + l] |= 1 << 17;
        }
      }
  }
  pc.mark("exports");
  F.ok = true;
  return F;
}

std::string validate_factor_schedule(const FactorSchedule& F, int n, const std::vector<int>& iaf,
                                     const std::vector<int>& jaf, const std::vector<int>& dg) {
  if (!F.ok) return "factor schedule not built: " + F.why;
  const ChainSchedule& S = F.geo;
  const int L = kChainLanes, R = F.R;
  const int impBase = 1 + L * (R + 1) * kFacWU;
  std::vector<int> bandOf(n, -1), laneOf(n, -1), posOf(n, -1), iterOf(n, -1);
  for (int b = 0; b < S.nbands; ++b)
    for (int l = 0; l < L; ++l) {
      const size_t g = (size_t)b * L + l;
      for (int p = 0; p < S.laneLen[g]; ++p) {
        const int i = S.laneStart[g] + p;
        if (i < 0 || i >= n || bandOf[i] >= 0) return "row scheduled twice or out of range";
        bandOf[i] = b;
        laneOf[i] = l;
        posOf[i] = p;
        iterOf[i] = p + S.laneSkew[g];
      }
    }
  for (int i = 0; i < n; ++i)
    if (bandOf[i] < 0) return "row never scheduled";
  std::vector<std::unordered_map<int, int>> impOfRow(S.nbands);
  std::vector<int> nextInSlot(F.impRow.size(), -1);
  for (int b = 0; b < S.nbands; ++b) {
    std::unordered_map<int, int> lastInSlot;
    for (int q = 0; q < F.bandNImp[b]; ++q) {
      const size_t g = (size_t)F.bandImp[b] + q;
      if (!impOfRow[b].emplace(F.impRow[g], q).second) return "row imported twice by one band";
      auto ls = lastInSlot.find(F.impSlot[g]);
      if (ls != lastInSlot.end()) {
        nextInSlot[(size_t)F.bandImp[b] + ls->second] = q;
        if (F.impWait[g] != F.impFree[(size_t)F.bandImp[b] + ls->second]) return "import does not wait for its slot";
      } else if (F.impWait[g] != -1) {
        return "first import of a slot waits";
      }
      lastInSlot[F.impSlot[g]] = q;
    }
  }
  // the cell that must hold U(j, c) for a reader at (band b, lane l, iteration t)
  auto check = [&](int j, int c, int b, int l, int t, int cell) -> std::string {
    const int* ub = jaf.data() + dg[j];
    const int* ue = jaf.data() + iaf[j + 1];
    const int* f = std::lower_bound(ub, ue, c);
    if (f == ue || *f != c) return "value of an entry the pivot row does not hold";
    const int pos = (int)(f - jaf.data());
    if (cell <= 0) return "missing value";
    if (cell < impBase) {
      const int r = (cell - 1) / kFacWU, u = (cell - 1) % kFacWU, lp = r / (R + 1), sl = r % (R + 1);
      if (bandOf[j] != b || laneOf[j] != lp || (posOf[j] & (R - 1)) != sl || u != pos - dg[j]) return "ring cell of another value";
      if (iterOf[j] >= t) return "ring value read before it is written";
      const size_t gl = (size_t)b * L + lp;
      const int over = posOf[j] + R;
      if (over < S.laneLen[gl] && over + S.laneSkew[gl] < t) return "ring value overwritten before it is read";
      return "";
    }
    const int slot = (cell - impBase) / kFacWU, u = (cell - impBase) % kFacWU;
    if (slot >= F.RI) return "import slot out of range";
    auto it = impOfRow[b].find(j);
    if (it == impOfRow[b].end()) return "import of a row the band does not import";
    const size_t q = (size_t)F.bandImp[b] + it->second;
    if (F.impSlot[q] != slot || u != pos - dg[j]) return "import read from another slot";
    if (F.impNeed[(size_t)S.bandSlot[b] + t] < it->second) return "iteration does not wait for its import";
    if (F.impFree[q] < t) return "import read after its slot is released";
    if (F.impWait[q] >= t) return "import delivered only after it is read";
    const int nx = nextInSlot[q];
    if (nx >= 0 && F.impWait[(size_t)F.bandImp[b] + nx] < t) return "import read after its slot is taken again";
    if (bandOf[j] == b && iterOf[j] >= t) return "import read before it is written";
    return "";
  };
  for (int i = 0; i < n; ++i) {
    const int b = bandOf[i], l = laneOf[i], t = iterOf[i];
    const size_t slot = (size_t)S.bandSlot[b] + t;
    const int kb = iaf[i], W = iaf[i + 1] - kb, nl = dg[i] - kb;
    if ((F.meta[slot * L + l] & 0x1FFFF) != (W | (nl << 8) | (1 << 16))) return "row metadata";
    for (int e = 0; e < kFacWF; ++e)
      if (F.vsrc[fac_vidx(slot, e, l)] != (e < W ? kb + e : -1)) return "row values";
    for (int q = 0; q < kFacNL; ++q) {
      const int cell = F.code[fac_cidx(slot, kFacNUpd + q, l)];
      if (q >= nl) {
        if (cell) return "pivot beyond the lower entries";
        continue;
      }
      const std::string r = check(jaf[kb + q], jaf[kb + q], b, l, t, cell);
      if (!r.empty()) return "pivot: " + r;
    }
    for (int e = 1; e < kFacWF; ++e)
      for (int q = 0; q < std::min(e, kFacNL); ++q) {
        const int cell = F.code[fac_cidx(slot, fac_slot(e, q), l)];
        bool upd = false;
        if (e < W && q < nl) {  // the reference updates entry e from pivot q iff row j_q holds col(e) above j_q
          const int j = jaf[kb + q], c = jaf[kb + e];
          if (c > j) upd = std::binary_search(jaf.begin() + dg[j] + 1, jaf.begin() + iaf[j + 1], c);
        }
        if (!upd) {
          if (cell) return "update the reference does not make";
          continue;
        }
        const std::string r = check(jaf[kb + q], jaf[kb + e], b, l, t, cell);
        if (!r.empty()) return "update: " + r;
      }
  }
  return "";
}

}  // namespace mmx
