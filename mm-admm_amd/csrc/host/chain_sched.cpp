// chain_sched.cpp -- see chain_sched.h.
#include "chain_sched.h"

#include <algorithm>
#include <queue>
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
  S.E = emax <= 8 ? 8 : emax <= 16 ? 16 : emax <= 32 ? 32 : 0;
  if (!S.E) {
    S.why = "a row has more than 32 entries in the triangle";
    return S;
  }
  // chains in processing order (forward: ascending rows; backward: descending)
  std::vector<int> chainOf(n), posOf(n), cStart, cLen;
  for (int t = 0; t < n; ++t) {
    const int i = fwd ? t : n - 1 - t;
    const int b = rb(i), e = re(i);
    const bool cont = t > 0 && cLen.back() < kChainLenCap &&
                      (fwd ? (e > b && jaf[e - 1] == i - 1) : (e > b && jaf[b] == i + 1));
    if (!cont) {
      cStart.push_back(i);
      cLen.push_back(0);
    }
    chainOf[i] = (int)cStart.size() - 1;
    posOf[i] = cLen.back()++;
  }
  const int C = (int)cStart.size();
  S.nchains = C;
  S.nbands = (C + kChainLanes - 1) / kChainLanes;
  const int L = kChainLanes;
  S.laneStart.assign((size_t)S.nbands * L, 0);
  S.laneLen.assign((size_t)S.nbands * L, 0);
  S.laneSkew.assign((size_t)S.nbands * L, 0);
  S.bandSlot.assign(S.nbands, 0);
  S.bandT.assign(S.nbands, 0);
  S.bandImp.assign(S.nbands, 0);
  S.bandNImp.assign(S.nbands, 0);
  auto rowAt = [&](int c, int p) { return fwd ? cStart[c] + p : cStart[c] - p; };

  // pass 1: skews, band lengths, ring distances
  int maxDist = 1;
  for (int b = 0; b < S.nbands; ++b) {
    const int c0 = b * L, nl = std::min(L, C - c0);
    int T = 0;
    for (int l = 0; l < nl; ++l) {
      const int c = c0 + l;
      int sk = 0;
      for (int p = 0; p < cLen[c]; ++p) {
        const int i = rowAt(c, p);
        for (int k = rb(i); k < re(i); ++k) {
          const int cj = chainOf[jaf[k]];
          if (cj >= c0 && cj < c) sk = std::max(sk, S.laneSkew[(size_t)b * L + (cj - c0)] + posOf[jaf[k]] - p + 1);
        }
      }
      S.laneStart[(size_t)b * L + l] = cStart[c];
      S.laneLen[(size_t)b * L + l] = cLen[c];
      S.laneSkew[(size_t)b * L + l] = sk;
      S.maxSkew = std::max(S.maxSkew, sk);
      S.maxLen = std::max(S.maxLen, cLen[c]);
      T = std::max(T, sk + cLen[c]);
    }
    for (int l = 0; l < nl; ++l) {
      const int c = c0 + l, skl = S.laneSkew[(size_t)b * L + l];
      for (int p = 0; p < cLen[c]; ++p) {
        const int i = rowAt(c, p);
        for (int k = rb(i); k < re(i); ++k) {
          const int cj = chainOf[jaf[k]];
          if (cj < c0 || cj > c) continue;
          const int d = (p + skl) - (posOf[jaf[k]] + S.laneSkew[(size_t)b * L + (cj - c0)]);
          if (d <= kChainRingMax) maxDist = std::max(maxDist, d);
        }
      }
    }
    S.bandT[b] = T;
    S.bandSlot[b] = (int)S.slots;
    S.slots += T;
    S.maxT = std::max(S.maxT, T);
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
  std::vector<long long> doneAt(n, 0);  // iteration (band-relative + offset) a row is published
  std::vector<long long> offset(S.nbands, 0);
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
        const int i = rowAt(c, p), t = p + skl;
        const size_t base = ((size_t)(S.bandSlot[b] + t) * S.E) * L + l;  // [slot][e][lane]
        if (!fwd) S.dsrc[(size_t)(S.bandSlot[b] + t) * L + l] = dg[i];
        int e = 0;
        S.bandE[b] = std::max(S.bandE[b], (re(i) - rb(i) + 3) / 4 * 4);
        for (int k = rb(i); k < re(i); ++k, ++e) {
          const int j = jaf[k], cj = chainOf[j];
          const size_t x = base + (size_t)e * L;
          S.src[x] = k;
          bool ring = false;
          if (cj >= c0 && cj <= c) {
            const int lj = cj - c0, q = posOf[j];
            const int d = t - (q + S.laneSkew[(size_t)b * L + lj]);
            if (d <= R) {
              S.code[x] = lj * (R + 1) + (q & (R - 1));
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
    for (const Use& u : impUses) {
      const int k = rank[impOf[u.row]];
      S.code[u.slot] = -(k + 1);
      const size_t it = u.slot / ((size_t)S.E * L);  // slot (iteration) of the use
      S.impNeed[it] = std::max(S.impNeed[it], k);
    }
    // a slot is reused by import k + RI once import k's last use has passed
    auto fits = [&](int ri) {
      for (size_t q = (size_t)ri; q < ord.size(); ++q)
        if (first[ord[q]] <= last[ord[q - ri]]) return false;
      return true;
    };
    if (!fits(RI)) {
      S.why = "import ring too small for band " + std::to_string(b);
      return S;
    }
    S.bandImp[b] = (int)S.impRow.size();
    S.bandNImp[b] = (int)ord.size();
    for (int j : rows) srcBands[b].push_back(chainOf[j] / L);
    std::sort(srcBands[b].begin(), srcBands[b].end());
    srcBands[b].erase(std::unique(srcBands[b].begin(), srcBands[b].end()), srcBands[b].end());
    long long off = 0;
    for (size_t q = 0; q < ord.size(); ++q) {
      const int id = ord[q];
      S.impRow.push_back(rows[id]);
      S.impFree.push_back(last[id]);
      const int j = rows[id], cj = chainOf[j];
      if (cj < c0) off = std::max(off, doneAt[j] + kImportLatency - first[id]);
    }
    if (b > 0) off = std::max(off, offset[b - 1]);
    offset[b] = off;
    for (int l = 0; l < nl; ++l) {
      const int c = c0 + l, skl = S.laneSkew[(size_t)b * L + l];
      for (int p = 0; p < cLen[c]; ++p) doneAt[rowAt(c, p)] = off + p + skl + 1;
    }
    S.estIters = std::max(S.estIters, off + S.bandT[b]);
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
  for (int& c : S.code) c = (c == kChainPad) ? 0 : (c >= 0 ? 1 + c : impBase + ((-c - 1) & (RI - 1)));
  S.ok = true;
  return S;
}

std::string validate_chain_schedule(const ChainSchedule& S, int n, const std::vector<int>& iaf,
                                    const std::vector<int>& jaf, const std::vector<int>& dg) {
  if (!S.ok) return "schedule not built: " + S.why;
  const int L = kChainLanes, E = S.E, R = S.R;
  const bool fwd = S.fwd;
  // where every row is computed: band, lane, position, iteration
  std::vector<int> bandOf(n, -1), laneOf(n, -1), posOf(n, -1), iterOf(n, -1);
  for (int b = 0; b < S.nbands; ++b)
    for (int l = 0; l < L; ++l) {
      const size_t g = (size_t)b * L + l;
      for (int p = 0; p < S.laneLen[g]; ++p) {
        const int i = fwd ? S.laneStart[g] + p : S.laneStart[g] - p;
        if (i < 0 || i >= n) return "row out of range";
        if (bandOf[i] >= 0) return "row " + std::to_string(i) + " scheduled twice";
        bandOf[i] = b;
        laneOf[i] = l;
        posOf[i] = p;
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
  for (int i = 0; i < n; ++i) {
    const int b = bandOf[i], l = laneOf[i], t = iterOf[i];
    const size_t base = ((size_t)(S.bandSlot[b] + t) * E) * L + l;
    const int kb = fwd ? iaf[i] : dg[i] + 1, ke = fwd ? dg[i] : iaf[i + 1];
    if (ke - kb > E) return "row wider than E";
    if (!fwd && S.dsrc[(size_t)(S.bandSlot[b] + t) * L + l] != dg[i]) return "diagonal source";
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
        int k2 = -1;
        for (int q = slot; q < S.bandNImp[b]; q += S.RI)
          if (S.impRow[(size_t)S.bandImp[b] + q] == j) k2 = q;
        if (k2 < 0) return "import of another row";
        const size_t q = (size_t)S.bandImp[b] + k2;
        if (S.impNeed[(size_t)S.bandSlot[b] + t] < k2) return "iteration does not wait for its import";
        if (S.impFree[q] < t) return "import read after its slot is released";
        if (k2 >= S.RI && S.impFree[q - S.RI] >= t) return "import read before its slot is free";
        if (bandOf[j] == b && iterOf[j] >= t) return "import read before it is written";
        // every import up to impNeed[t] is free to be delivered by iteration t (no deadlock)
        const int need = S.impNeed[(size_t)S.bandSlot[b] + t];
        if (need >= S.RI && S.impFree[(size_t)S.bandImp[b] + need - S.RI] >= t) return "import delivery would deadlock";
      }
    }
  }
  return "";
}

}  // namespace mmx
