// partition.cpp -- see partition.h.
#include "partition.h"

#include <algorithm>
#include <cmath>
#include <string>

#include "common.h"

namespace mmx {

std::vector<int> partition_owners(int D, int nP, const double* Xp, int nF, const int32_t* F, int nranks, int method) {
  const int V = D + 1;
  std::vector<int> owner(nF, 0);
  if (nranks == 1) return owner;
  if (method == kPartRanges) {
    for (int q = 0; q < nranks; ++q)
      for (long long s = (long long)q * nF / nranks; s < (long long)(q + 1) * nF / nranks; ++s) owner[s] = q;
    return owner;
  }
  if (method != kPartRCB) throw Error(MMADMM_ERR_INVALID, "unknown partition method");
  if (!Xp) throw Error(MMADMM_ERR_INVALID, "RCB partition needs the node positions");
  (void)nP;
  // centroids, and the largest extent of a simplex along each axis
  std::vector<double> cen((size_t)nF * D);
  double ext[3] = {0.0, 0.0, 0.0};
#pragma omp parallel for reduction(max : ext[:3]) schedule(static)
  for (long long s = 0; s < (long long)nF; ++s)
    for (int a = 0; a < D; ++a) {
      double c = 0.0, lo = INFINITY, hi = -INFINITY;
      for (int n = 0; n < V; ++n) {
        const double x = Xp[(size_t)F[s * V + n] * D + a];
        c += x;
        lo = std::min(lo, x);
        hi = std::max(hi, x);
      }
      cen[s * D + a] = c / V;
      ext[a] = std::max(ext[a], hi - lo);
    }
  std::vector<int> ids(nF);
  for (int s = 0; s < nF; ++s) ids[s] = s;
  struct Part {
    int b, e, r0, nr;
  };
  std::vector<Part> todo{{0, nF, 0, nranks}};
  std::vector<std::pair<double, int>> key;
  while (!todo.empty()) {
    const Part P = todo.back();
    todo.pop_back();
    if (P.nr == 1 || P.e - P.b <= 1) {
      for (int i = P.b; i < P.e; ++i) owner[ids[i]] = P.r0;
      continue;
    }
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = P.b; i < P.e; ++i)
      for (int a = 0; a < D; ++a) {
        const double c = cen[(size_t)ids[i] * D + a];
        lo[a] = std::min(lo[a], c);
        hi[a] = std::max(hi[a], c);
      }
    int axis = 0;
    for (int a = 1; a < D; ++a)
      if (hi[a] - lo[a] > hi[axis] - lo[axis]) axis = a;
    const int nlo = P.nr / 2;
    int cut = P.b + (int)((long long)(P.e - P.b) * nlo / P.nr);
    key.resize(P.e - P.b);
    for (int i = P.b; i < P.e; ++i) key[i - P.b] = {cen[(size_t)ids[i] * D + axis], ids[i]};
    std::nth_element(key.begin(), key.begin() + (cut - P.b), key.end());
    // The cut plane: among the vertex coordinates nearest the proportional centroid (kCand below
    // and above it, within half a window of 4 simplex extents), the one that the fewest
    // simplices straddle, within 2% of the proportional split.  On a structured mesh the cut then
    // runs between two layers of cells instead of through one (which would replicate about three
    // planes of nodes).  Only simplices whose centroid lies in the window can supply a candidate
    // or straddle one; the others are wholly on one side of every candidate.
    const double target = key[cut - P.b].first, win = 4.0 * ext[axis];
    constexpr int kCand = 8;
    std::vector<double> below, above;  // nearest distinct coordinates < target / >= target
    double worstB = -INFINITY, worstA = INFINITY;  // admission thresholds once a list is full
    auto offer = [&](std::vector<double>& v, double& worst, double c, bool lower) {
      if ((int)v.size() == kCand && (lower ? c <= worst : c >= worst)) return;
      for (double x : v)
        if (x == c) return;
      if ((int)v.size() < kCand) {
        v.push_back(c);
      } else {
        auto w = lower ? std::min_element(v.begin(), v.end()) : std::max_element(v.begin(), v.end());
        *w = c;
      }
      if ((int)v.size() == kCand) worst = lower ? *std::min_element(v.begin(), v.end()) : *std::max_element(v.begin(), v.end());
    };
    std::vector<int> near;
    for (const auto& k : key)
      if (std::fabs(k.first - target) <= win) near.push_back(k.second);
    for (int sN : near)
      for (int n = 0; n < V; ++n) {
        const double c = Xp[(size_t)F[(size_t)sN * V + n] * D + axis];
        if (std::fabs(c - target) > 0.5 * win) continue;
        if (c < target) offer(below, worstB, c, true);
        else offer(above, worstA, c, false);
      }
    std::vector<double> cand(below);
    cand.insert(cand.end(), above.begin(), above.end());
    std::sort(cand.begin(), cand.end());
    std::vector<long long> strad(cand.size(), 0), left(cand.size(), 0);
    long long allLeft = 0;
    for (const auto& k : key)
      if (k.first < target - win) ++allLeft;
    for (int sN : near) {
      double slo = INFINITY, shi = -INFINITY;
      for (int n = 0; n < V; ++n) {
        const double c = Xp[(size_t)F[(size_t)sN * V + n] * D + axis];
        slo = std::min(slo, c);
        shi = std::max(shi, c);
      }
      const double cs = cen[(size_t)sN * D + axis];
      for (size_t j = 0; j < cand.size(); ++j) {
        strad[j] += (slo < cand[j] && cand[j] < shi) ? 1 : 0;
        left[j] += (cs < cand[j]) ? 1 : 0;
      }
    }
    for (auto& l : left) l += allLeft;
    const long long want = cut - P.b, tolr = std::max<long long>(1, (P.e - P.b) / 50);
    int pick = -1;
    for (size_t j = 0; j < cand.size(); ++j) {
      // each side keeps at least one simplex per rank it goes to (the proportional cut does too,
      // since every part holds at least as many simplices as ranks), so no rank ends up empty
      if (left[j] < nlo || (P.e - P.b) - left[j] < P.nr - nlo || std::llabs(left[j] - want) > tolr) continue;
      if (pick < 0 || strad[j] < strad[pick] ||
          (strad[j] == strad[pick] && std::llabs(left[j] - want) < std::llabs(left[pick] - want)))
        pick = (int)j;
    }
    if (pick >= 0) {
      const double plane = cand[pick];
      std::partition(key.begin(), key.end(), [&](const std::pair<double, int>& k) { return k.first < plane; });
      cut = P.b + (int)left[pick];
    }
    for (int i = P.b; i < P.e; ++i) ids[i] = key[i - P.b].second;  // the two sets are order-independent
    todo.push_back({cut, P.e, P.r0 + nlo, P.nr - nlo});
    todo.push_back({P.b, cut, P.r0, nlo});
  }
  return owner;
}

PartitionPlan make_partition_plan(int D, int nP, const double* Xp, int nF, const int32_t* F, int nranks, int rank,
                                  int method) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(MMADMM_ERR_INVALID, "bad rank / nranks");
  if (nranks > 64) throw Error(MMADMM_ERR_INVALID, "element partition: at most 64 ranks");
  if ((long long)nranks > (long long)nF && nF > 0)
    throw Error(MMADMM_ERR_INVALID, "more ranks than simplices");
  const int V = D + 1, K = D * (D + 1);
  PartitionPlan P;
  P.nranks = nranks;
  P.rank = rank;
  P.method = method;
  P.nF = nF;
  P.nP = nP;
  const std::vector<int> owner = partition_owners(D, nP, Xp, nF, F, nranks, method);
  // the ranks touching each node, and each node's owner (the rank of its lowest incident simplex)
  std::vector<uint64_t> touch(nP, 0);
  P.nodeOwner.assign(nP, -1);
  for (size_t s = 0; s < (size_t)nF; ++s)
    for (int n = 0; n < V; ++n) {
      const int v = F[s * V + n];
      touch[v] |= 1ull << owner[s];
      if (P.nodeOwner[v] < 0) P.nodeOwner[v] = owner[s];
    }
  for (int v = 0; v < nP; ++v)
    if (P.nodeOwner[v] < 0) P.nodeOwner[v] = 0;
  const uint64_t me = 1ull << rank;
  // local simplices (ascending global id) and local nodes (+ isolated nodes on rank 0)
  std::vector<int> g2l(nP, -1);
  for (int v = 0; v < nP; ++v)
    if ((touch[v] & me) || (touch[v] == 0 && rank == 0)) {
      g2l[v] = (int)P.localNodes.size();
      P.localNodes.push_back(v);
      if (touch[v] & ~me) P.interfaceNodes++;
    }
  for (int s = 0; s < nF; ++s)
    if (owner[s] == rank) P.localSimplices.push_back(s);
  const int nfl = (int)P.localSimplices.size();
  P.Flocal.resize((size_t)nfl * V);
  for (int ls = 0; ls < nfl; ++ls)
    for (int n = 0; n < V; ++n) P.Flocal[(size_t)ls * V + n] = g2l[F[(size_t)P.localSimplices[ls] * V + n]];
  // neighbours: every other rank touching one of our nodes.  Send list to q: our slots on nodes
  // q touches, (s, n) ascending; q's list to us is its slots on nodes we touch, in the same order
  uint64_t nb = 0;
  for (int v : P.localNodes) nb |= touch[v];
  nb &= ~me;
  std::vector<int> recvCount(nranks, 0), recvOff(nranks, 0), seen(nranks, 0);
  for (size_t s = 0; s < (size_t)nF; ++s) {
    const int q = owner[s];
    if (q == rank) continue;
    for (int n = 0; n < V; ++n)
      if (touch[F[s * V + n]] & me) recvCount[q]++;
  }
  for (int q = 0; q < nranks; ++q) {
    if (!((nb >> q) & 1)) continue;
    HaloPeer h;
    h.rank = q;
    h.sendOff = (int)P.sendOff.size();
    const uint64_t bq = 1ull << q;
    for (int ls = 0; ls < nfl; ++ls)
      for (int n = 0; n < V; ++n)
        if (touch[F[(size_t)P.localSimplices[ls] * V + n]] & bq) P.sendOff.push_back(ls * K + n * D);
    h.sendCount = (int)P.sendOff.size() - h.sendOff;
    h.recvOff = P.recvRows;
    h.recvCount = recvCount[q];
    recvOff[q] = h.recvOff;
    P.recvRows += h.recvCount;
    P.peers.push_back(h);
  }
  // global incidence of the local nodes, ascending simplex id
  const int nl = (int)P.localNodes.size();
  P.incPtr.assign(nl + 1, 0);
  for (size_t s = 0; s < (size_t)nF; ++s)
    for (int n = 0; n < V; ++n) {
      const int l = g2l[F[s * V + n]];
      if (l >= 0) P.incPtr[l + 1]++;
    }
  for (int l = 0; l < nl; ++l) P.incPtr[l + 1] += P.incPtr[l];
  P.incSrc.resize(P.incPtr[nl]);
  P.valence.resize(nl);
  for (int l = 0; l < nl; ++l) P.valence[l] = P.incPtr[l + 1] - P.incPtr[l];
  std::vector<int> fill(P.incPtr.begin(), P.incPtr.end() - 1);
  int ls = 0;
  for (size_t s = 0; s < (size_t)nF; ++s) {
    const int q = owner[s];
    for (int n = 0; n < V; ++n) {
      const int l = g2l[F[s * V + n]];
      if (l < 0) continue;
      int src;
      if (q == rank) {
        src = ls * K + n * D;
      } else {
        if (!((touch[F[s * V + n]] >> rank) & 1)) throw Error(MMADMM_ERR_INVALID, "partition plan: remote slot");
        src = -1 - (recvOff[q] + seen[q]++);
      }
      P.incSrc[fill[l]++] = src;
    }
    if (q == rank) ++ls;
  }
  for (const HaloPeer& h : P.peers)
    if (seen[h.rank] != h.recvCount) throw Error(MMADMM_ERR_INVALID, "partition plan: receive count mismatch");
  return P;
}

}  // namespace mmx

// ---- C-ABI: the plan on its own, for host-side tests of the exchange (no GPU needed) ----
struct mmadmm_plan_s {
  mmx::PartitionPlan p;
};

extern "C" {

int mmadmm_plan_create(int dim, int nP, const double* Xp, int nF, const int32_t* F, int nranks, int rank, int method,
                       mmadmm_plan* out) {
  return mmx::guarded([&] {
    if (!out || !F || (dim != 2 && dim != 3) || nP <= 0 || nF <= 0)
      throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_plan_create: bad arguments");
    for (long long i = 0; i < (long long)nF * (dim + 1); ++i)
      if (F[i] < 0 || F[i] >= nP) throw mmx::Error(MMADMM_ERR_INVALID, "simplex vertex id out of range");
    auto* h = new mmadmm_plan_s;
    try {
      h->p = mmx::make_partition_plan(dim, nP, Xp, nF, F, nranks, rank, method);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int mmadmm_plan_sizes(mmadmm_plan h, int* nLocalNodes, int* nLocalSimplices, int* nSources, int* nSend, int* nRecv,
                      int* nPeers, int* nInterface) {
  return mmx::guarded([&] {
    if (!h) throw mmx::Error(MMADMM_ERR_INVALID, "null plan");
    const auto& p = h->p;
    if (nLocalNodes) *nLocalNodes = (int)p.localNodes.size();
    if (nLocalSimplices) *nLocalSimplices = (int)p.localSimplices.size();
    if (nSources) *nSources = (int)p.incSrc.size();
    if (nSend) *nSend = (int)p.sendOff.size();
    if (nRecv) *nRecv = p.recvRows;
    if (nPeers) *nPeers = (int)p.peers.size();
    if (nInterface) *nInterface = p.interfaceNodes;
  });
}

int mmadmm_plan_get(mmadmm_plan h, int32_t* localNodes, int32_t* localSimplices, int32_t* incPtr, int32_t* incSrc,
                    int32_t* sendOff, int32_t* peers) {
  return mmx::guarded([&] {
    if (!h) throw mmx::Error(MMADMM_ERR_INVALID, "null plan");
    const auto& p = h->p;
    if (localNodes) std::copy(p.localNodes.begin(), p.localNodes.end(), localNodes);
    if (localSimplices) std::copy(p.localSimplices.begin(), p.localSimplices.end(), localSimplices);
    if (incPtr) std::copy(p.incPtr.begin(), p.incPtr.end(), incPtr);
    if (incSrc) std::copy(p.incSrc.begin(), p.incSrc.end(), incSrc);
    if (sendOff) std::copy(p.sendOff.begin(), p.sendOff.end(), sendOff);
    if (peers)
      for (size_t i = 0; i < p.peers.size(); ++i) {
        peers[i * 3 + 0] = p.peers[i].rank;
        peers[i * 3 + 1] = p.peers[i].sendCount;
        peers[i * 3 + 2] = p.peers[i].recvCount;
      }
  });
}

int mmadmm_plan_destroy(mmadmm_plan h) {
  delete h;
  return MMADMM_OK;
}

}  // extern "C"
