// chain_sched.cpp -- see chain_sched.h.
#include "chain_sched.h"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <queue>
#include <unordered_map>
#include <cstdint>

namespace mmx {

namespace {
constexpr int kChainLenCap = 1 << 20;  // longest chain (positions fit the schedule's ints)
constexpr int kImportLatency = 8;      // iterations a global value takes to reach another band (model)
int pow2_at_least(int v) {
  int r = 1;
  while (r < v) r <<= 1;
  return r;
}
}  // namespace

ChainSchedule build_chain_schedule(int n, const std::vector<int>& iaf, const std::vector<int>& jaf,
                                   const std::vector<int>& dg, bool fwd) {
  ChainSchedule S;
  S.fwd = fwd;
  auto rb = [&](int i) { return fwd ? iaf[i] : dg[i] + 1; };
  auto re = [&](int i) { return fwd ? dg[i] : iaf[i + 1]; };
  int emax = 0;
  for (int i = 0; i < n; ++i) emax = std::max(emax, re(i) - rb(i));
  // rows wider than 32 entries (3D) are split into segments of E = 32 entries computed at
  // consecutive positions of their lane (the partial sum carried in a register, so the order of
  // the subtractions is unchanged); every row of a chain takes the chain's segment count ns
  S.E = emax <= 8 ? 8 : emax <= 16 ? 16 : 32;
  S.seg = emax > 32;
  if (emax > kChainSegMax * 32) {
    S.why = "a row has more than " + std::to_string(kChainSegMax * 32) + " entries in the triangle";
    return S;
  }
  auto nsRow = [&](int i) { return std::max(1, (re(i) - rb(i) + S.E - 1) / S.E); };
  // chains in processing order (forward: ascending rows; backward: descending); a chain also ends
  // where the segment count changes, so no row pays for a wider neighbour's segments
  std::vector<int> chainOf(n), posOf(n), cStart, cLen, cNs;
  for (int t = 0; t < n; ++t) {
    const int i = fwd ? t : n - 1 - t;
    const int b = rb(i), e = re(i), ns = nsRow(i);
    const bool cont = t > 0 && cLen.back() < kChainLenCap && cNs.back() == ns &&
                      (fwd ? (e > b && jaf[e - 1] == i - 1) : (e > b && jaf[b] == i + 1));
    if (!cont) {
      cStart.push_back(i);
      cLen.push_back(0);
      cNs.push_back(ns);
    }
    chainOf[i] = (int)cStart.size() - 1;
    posOf[i] = cLen.back() + ns - 1;  // the row's value is ready after its last segment
    cLen.back() += ns;
  }
  const int C = (int)cStart.size();
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
  // row and segment at position p of chain c
  auto rowAt = [&](int c, int p) { return fwd ? cStart[c] + p / cNs[c] : cStart[c] - p / cNs[c]; };

  // pass 1: skews and band lengths, with a model of the critical path: band b starts at iteration
  // offset[b] (not before band b - 1), a row is published at offset + position + skew + 1 and an
  // import reaches another band kImportLatency iterations later.  Plain skews satisfy only the
  // band's own dependencies (the band then waits for late imports); aligned skews also delay each
  // lane until its imports are due (3D: a band's chains span planes whose imports arrive at very
  // different times).  MMX_CHAIN_ALIGN=0/1 forces one; by default the shorter modelled path wins.
  std::vector<long long> doneAt(n, -1), offset(S.nbands, 0);
  auto pass1 = [&](bool align) {
    std::fill(doneAt.begin(), doneAt.end(), -1);
    long long est = 0;
    for (int b = 0; b < S.nbands; ++b) {
      const int c0 = b * L, nl = std::min(L, C - c0);
      const long long off0 = b > 0 ? offset[b - 1] : 0;
      long long off = off0;
      int T = 0, minSk = INT32_MAX;
      for (int l = 0; l < nl; ++l) {
        const int c = c0 + l;
        long long sk = 0;
        for (int p = 0; p < cLen[c]; ++p) {
          const int i = rowAt(c, p), q = p % cNs[c];
          const int kb = rb(i) + q * S.E, ke = std::min(re(i), kb + S.E);
          for (int k = kb; k < ke; ++k) {
            const int j = jaf[k], cj = chainOf[j];
            if (cj >= c0 && cj < c) {
              sk = std::max<long long>(sk, S.laneSkew[(size_t)b * L + (cj - c0)] + posOf[j] - p + 1);
            } else if (align && cj < c0 && doneAt[j] >= 0) {
              sk = std::max<long long>(sk, doneAt[j] + kImportLatency - off0 - p);
            }
          }
        }
        if (sk > kChainLenCap) sk = kChainLenCap;
        S.laneSkew[(size_t)b * L + l] = (int)sk;
        minSk = std::min(minSk, (int)sk);
      }
      if (align && nl > 0 && minSk > 0) {  // start the band later rather than idle its lanes
        for (int l = 0; l < nl; ++l) S.laneSkew[(size_t)b * L + l] -= minSk;
        off += minSk;
      }
      for (int l = 0; l < nl; ++l) {
        const int c = c0 + l, sk = S.laneSkew[(size_t)b * L + l];
        T = std::max(T, sk + cLen[c]);
        if (!align)  // the band waits for its late imports
          for (int p = 0; p < cLen[c]; ++p) {
            const int i = rowAt(c, p), q = p % cNs[c];
            const int kb = rb(i) + q * S.E, ke = std::min(re(i), kb + S.E);
            for (int k = kb; k < ke; ++k) {
              const int j = jaf[k];
              if (chainOf[j] < c0 && doneAt[j] >= 0) off = std::max(off, doneAt[j] + kImportLatency - (p + sk));
            }
          }
      }
      offset[b] = off;
      for (int l = 0; l < nl; ++l) {
        const int c = c0 + l, sk = S.laneSkew[(size_t)b * L + l];
        for (int p = cNs[c] - 1; p < cLen[c]; p += cNs[c]) doneAt[rowAt(c, p)] = off + p + sk + 1;
      }
      S.bandT[b] = T;
      est = std::max(est, off + T);
    }
    return est;
  };
  {
    const char* ae = getenv("MMX_CHAIN_ALIGN");
    const int mode = ae ? atoi(ae) : -1;
    long long est;
    if (mode >= 0) {
      est = pass1(mode != 0);
      S.aligned = mode != 0;
    } else {
      const long long e0 = pass1(false), e1 = pass1(true);
      S.aligned = e1 < e0;
      est = S.aligned ? e1 : pass1(false);
    }
    S.estIters = est;
  }
  // lane arrays, slots, ring distances
  int maxDist = 1;
  for (int b = 0; b < S.nbands; ++b) {
    const int c0 = b * L, nl = std::min(L, C - c0);
    for (int l = 0; l < nl; ++l) {
      const int c = c0 + l, sk = S.laneSkew[(size_t)b * L + l];
      S.laneStart[(size_t)b * L + l] = cStart[c];
      S.laneLen[(size_t)b * L + l] = cLen[c];
      S.laneNs[(size_t)b * L + l] = cNs[c];
      S.maxSkew = std::max(S.maxSkew, sk);
      S.maxLen = std::max(S.maxLen, cLen[c]);
    }
    for (int l = 0; l < nl; ++l) {
      const int c = c0 + l, skl = S.laneSkew[(size_t)b * L + l];
      for (int p = 0; p < cLen[c]; ++p) {
        const int i = rowAt(c, p), q = p % cNs[c];
        const int kb = rb(i) + q * S.E, ke = std::min(re(i), kb + S.E);
        for (int k = kb; k < ke; ++k) {
          const int cj = chainOf[jaf[k]];
          if (cj < c0 || cj > c) continue;
          const int d = (p + skl) - (posOf[jaf[k]] + S.laneSkew[(size_t)b * L + (cj - c0)]);
          if (d <= kChainRingMax) maxDist = std::max(maxDist, d);
        }
      }
    }
    S.bandSlot[b] = (int)S.slots;
    S.slots += S.bandT[b];
    S.maxT = std::max(S.maxT, S.bandT[b]);
  }
  if (S.slots * L * S.E > (long long)INT32_MAX) {
    S.why = "schedule too large";
    return S;
  }
  S.R = std::max(2, pow2_at_least(maxDist));
  const int R = S.R;

  // pass 2: codes, value sources, imports
  const size_t ne = (size_t)S.slots * L * S.E;
  S.code.assign(ne, kChainPad);
  S.impNeed.assign((size_t)S.slots, -1);
  S.bandE.assign(S.nbands, 4);
  S.src.assign(ne, -1);
  if (!fwd) S.dsrc.assign((size_t)S.slots * L, -1);
  std::vector<int> impOf(n, -1), first, last, rows;
  std::vector<std::vector<int>> srcBands(S.nbands);  // bands each band imports from
  // the importer runs at most RI imports ahead of the compute wave: it takes the whole ring (a
  // band importing hundreds of values per iteration needs many iterations of run-ahead)
  const int RI = kChainImpMax;
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
      for (int p = 0; p < cLen[c]; ++p) {
        const int i = rowAt(c, p), t = p + skl, q = p % cNs[c];
        const size_t base = ((size_t)(S.bandSlot[b] + t) * S.E) * L + l;  // [slot][e][lane]
        if (!fwd && q == cNs[c] - 1) S.dsrc[(size_t)(S.bandSlot[b] + t) * L + l] = dg[i];
        const int kb = rb(i) + q * S.E, ke = std::min(re(i), kb + S.E);
        int e = 0;
        S.bandE[b] = std::max(S.bandE[b], (std::max(ke - kb, 0) + 3) / 4 * 4);
        for (int k = kb; k < ke; ++k, ++e) {
          const int j = jaf[k], cj = chainOf[j];
          const size_t x = base + (size_t)e * L;
          S.src[x] = k;
          bool ring = false;
          if (cj >= c0 && cj <= c) {
            const int lj = cj - c0, qj = posOf[j];
            const int d = t - (qj + S.laneSkew[(size_t)b * L + lj]);
            if (d <= R) {
              S.code[x] = lj * (R + 1) + (qj & (R - 1));
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
            impUses.push_back({x, j});
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
    // import slots by interval colouring in order of first use: an import takes the lowest slot
    // whose previous import's last use has passed (and waits for the compute wave to pass it), so
    // the slots needed are the most imports live at once
    std::vector<int> slotOf(ord.size()), waitOf(ord.size()), slotLast;
    {
      typedef std::pair<int, int> P;  // (last use, slot)
      std::priority_queue<P, std::vector<P>, std::greater<P>> busy;
      std::priority_queue<int, std::vector<int>, std::greater<int>> freeSlots;
      for (size_t q = 0; q < ord.size(); ++q) {
        const int f = first[ord[q]];
        while (!busy.empty() && busy.top().first < f) {
          freeSlots.push(busy.top().second);
          busy.pop();
        }
        int sl;
        if (!freeSlots.empty()) {
          sl = freeSlots.top();
          freeSlots.pop();
        } else {
          sl = (int)slotLast.size();
          if (sl == RI) {
            S.why = "import ring too small for band " + std::to_string(b);
            return S;
          }
          slotLast.push_back(-1);
        }
        slotOf[q] = sl;
        waitOf[q] = slotLast[sl];
        slotLast[sl] = last[ord[q]];
        busy.push({last[ord[q]], sl});
      }
    }
    S.maxImpSlots = std::max(S.maxImpSlots, (int)slotLast.size());
    for (const Use& u : impUses) {
      const int k = rank[impOf[u.row]];
      S.code[u.slot] = -(slotOf[k] + 1);
      const size_t it = u.slot / ((size_t)S.E * L);  // slot (iteration) of the use
      S.impNeed[it] = std::max(S.impNeed[it], k);
    }
    S.bandImp[b] = (int)S.impRow.size();
    S.bandNImp[b] = (int)ord.size();
    for (int j : rows) srcBands[b].push_back(chainOf[j] / L);
    std::sort(srcBands[b].begin(), srcBands[b].end());
    srcBands[b].erase(std::unique(srcBands[b].begin(), srcBands[b].end()), srcBands[b].end());
    for (size_t q = 0; q < ord.size(); ++q) {
      const int id = ord[q];
      S.impRow.push_back(rows[id]);
      S.impFree.push_back(last[id]);
      S.impSlot.push_back(slotOf[q]);
      S.impWait.push_back(waitOf[q]);
    }
    for (int j : rows) impOf[j] = -1;
  }
  S.RI = RI;
  S.nImports = (long long)S.impRow.size();
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
  // codes -> LDS indices: 0 zero cell, 1 + ring index, 1 + 64 (R + 1) + import slot
  const int impBase = 1 + L * (R + 1);
  for (int& c : S.code) c = (c == kChainPad) ? 0 : (c >= 0 ? 1 + c : impBase + (-c - 1));
  S.ok = true;
  return S;
}

std::string validate_chain_schedule(const ChainSchedule& S, int n, const std::vector<int>& iaf,
                                    const std::vector<int>& jaf, const std::vector<int>& dg) {
  if (!S.ok) return "schedule not built: " + S.why;
  const int L = kChainLanes, E = S.E, R = S.R;
  const bool fwd = S.fwd;
  // where every row is computed: band, lane, position of its last segment, iteration
  std::vector<int> bandOf(n, -1), laneOf(n, -1), posOf(n, -1), iterOf(n, -1), nsOf(n, 1);
  if (S.laneNs.size() != S.laneLen.size()) return "segment counts missing";
  for (int b = 0; b < S.nbands; ++b)
    for (int l = 0; l < L; ++l) {
      const size_t g = (size_t)b * L + l;
      const int ns = S.laneNs[g];
      if (ns < 1 || ns > kChainSegMax || (ns > 1 && !S.seg)) return "bad segment count";
      if (S.laneLen[g] % ns) return "lane length not a whole number of rows";
      for (int p = ns - 1; p < S.laneLen[g]; p += ns) {
        const int i = fwd ? S.laneStart[g] + p / ns : S.laneStart[g] - p / ns;
        if (i < 0 || i >= n) return "row out of range";
        if (bandOf[i] >= 0) return "row " + std::to_string(i) + " scheduled twice";
        bandOf[i] = b;
        laneOf[i] = l;
        posOf[i] = p;
        nsOf[i] = ns;
        iterOf[i] = p + S.laneSkew[g];
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
  for (int i = 0; i < n; ++i) {
    const int b = bandOf[i], l = laneOf[i], ns = nsOf[i];
    const int kb0 = fwd ? iaf[i] : dg[i] + 1, ke0 = fwd ? dg[i] : iaf[i + 1];
    if (ke0 - kb0 > E * ns) return "row wider than its segments";
    for (int sg = 0; sg < ns; ++sg) {
      const int t = iterOf[i] - (ns - 1) + sg;  // segment sg of the row
      const size_t base = ((size_t)(S.bandSlot[b] + t) * E) * L + l;
      const int kb = kb0 + sg * E, ke = std::min(ke0, kb + E);
      if (!fwd && S.dsrc[(size_t)(S.bandSlot[b] + t) * L + l] != (sg == ns - 1 ? dg[i] : -1)) return "diagonal source";
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
        const int impBase = 1 + L * (R + 1);
        if (c <= 0) return "missing entry";
        if (c < impBase) {
          const int r = c - 1, lp = r / (R + 1), slot = r % (R + 1);
          if (bandOf[j] != b || laneOf[j] != lp || (posOf[j] & (R - 1)) != slot) return "ring slot of another row";
          if (iterOf[j] >= t) return "ring value read before it is written";
          const size_t gp = (size_t)b * L + lp;
          const int over = posOf[j] + R;  // next write to the same slot
          if (over < S.laneLen[gp] && over + S.laneSkew[gp] < t) return "ring value overwritten before it is read";
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

}  // namespace mmx
