// partition.cpp -- see partition.h.
#include "partition.h"

#include <algorithm>
#include <string>

#include "common.h"

namespace mmx {

PartitionPlan make_partition_plan(int D, int nP, int nF, const int32_t* F, int nranks, int rank) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(MMADMM_ERR_INVALID, "bad rank / nranks");
  if ((long long)nranks > (long long)nF && nF > 0)
    throw Error(MMADMM_ERR_INVALID, "more ranks than simplices");
  const int V = D + 1, K = D * (D + 1);
  PartitionPlan P;
  P.nranks = nranks;
  P.rank = rank;
  P.nF = nF;
  P.nP = nP;
  P.sbeg.resize(nranks + 1);
  for (int q = 0; q <= nranks; ++q) P.sbeg[q] = (long long)q * nF / nranks;
  P.s0 = (int)P.sbeg[rank];
  P.s1 = (int)P.sbeg[rank + 1];
  // which ranks touch each node: first toucher and a "shared" flag
  std::vector<int> first(nP, -1);
  std::vector<uint8_t> shared(nP, 0);
  for (int q = 0; q < nranks; ++q)
    for (long long s = P.sbeg[q]; s < P.sbeg[q + 1]; ++s)
      for (int n = 0; n < V; ++n) {
        const int v = F[s * V + n];
        if (first[v] < 0)
          first[v] = q;
        else if (first[v] != q)
          shared[v] = 1;
      }
  // export index of every slot of a shared node, per owning rank, in (s, n) order
  std::vector<int> slotExp((size_t)nF * V, -1);
  std::vector<int> nexp(nranks, 0);
  for (int q = 0; q < nranks; ++q)
    for (long long s = P.sbeg[q]; s < P.sbeg[q + 1]; ++s)
      for (int n = 0; n < V; ++n)
        if (shared[F[s * V + n]]) slotExp[(size_t)s * V + n] = nexp[q]++;
  P.maxExport = nranks > 1 ? *std::max_element(nexp.begin(), nexp.end()) : 0;
  for (long long s = P.s0; s < P.s1; ++s)
    for (int n = 0; n < V; ++n)
      if (shared[F[s * V + n]]) P.exportOff.push_back((int)((s - P.s0) * K + n * D));
  // local nodes: nodes of local simplices (+ isolated nodes on rank 0), ascending global id
  std::vector<int> g2l(nP, -1);
  for (int v = 0; v < nP; ++v)
    if ((first[v] < 0 && rank == 0) || first[v] == rank) g2l[v] = 0;
  for (long long s = P.s0; s < P.s1; ++s)
    for (int n = 0; n < V; ++n) g2l[F[s * V + n]] = 0;
  for (int v = 0; v < nP; ++v)
    if (g2l[v] == 0) {
      g2l[v] = (int)P.localNodes.size();
      P.localNodes.push_back(v);
    }
  P.Flocal.resize((size_t)(P.s1 - P.s0) * V);
  for (long long s = P.s0; s < P.s1; ++s)
    for (int n = 0; n < V; ++n) P.Flocal[(size_t)(s - P.s0) * V + n] = g2l[F[s * V + n]];
  // global incidence of the local nodes, ascending simplex id
  const int nl = (int)P.localNodes.size();
  P.incPtr.assign(nl + 1, 0);
  for (int s = 0; s < nF; ++s)
    for (int n = 0; n < V; ++n) {
      const int l = g2l[F[(size_t)s * V + n]];
      if (l >= 0) P.incPtr[l + 1]++;
    }
  for (int l = 0; l < nl; ++l) P.incPtr[l + 1] += P.incPtr[l];
  P.incSrc.resize(P.incPtr[nl]);
  P.valence.resize(nl);
  for (int l = 0; l < nl; ++l) P.valence[l] = P.incPtr[l + 1] - P.incPtr[l];
  std::vector<int> fill(P.incPtr.begin(), P.incPtr.end() - 1);
  int q = 0;
  for (int s = 0; s < nF; ++s) {
    while (s >= P.sbeg[q + 1]) ++q;
    for (int n = 0; n < V; ++n) {
      const int l = g2l[F[(size_t)s * V + n]];
      if (l < 0) continue;
      int src;
      if (q == rank) {
        src = (int)((s - P.s0) * K + n * D);
      } else {
        const int e = slotExp[(size_t)s * V + n];
        if (e < 0) throw Error(MMADMM_ERR_INVALID, "partition plan: remote slot without export index");
        src = -1 - (q * P.maxExport + e);
      }
      P.incSrc[fill[l]++] = src;
    }
  }
  return P;
}

}  // namespace mmx

// ---- C-ABI: the plan on its own, for host-side tests of the exchange (no GPU needed) ----
struct mmadmm_plan_s {
  mmx::PartitionPlan p;
};

extern "C" {

int mmadmm_plan_create(int dim, int nP, int nF, const int32_t* F, int nranks, int rank, mmadmm_plan* out) {
  return mmx::guarded([&] {
    if (!out || !F || (dim != 2 && dim != 3) || nP <= 0 || nF <= 0)
      throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_plan_create: bad arguments");
    for (long long i = 0; i < (long long)nF * (dim + 1); ++i)
      if (F[i] < 0 || F[i] >= nP) throw mmx::Error(MMADMM_ERR_INVALID, "simplex vertex id out of range");
    auto* h = new mmadmm_plan_s;
    h->p = mmx::make_partition_plan(dim, nP, nF, F, nranks, rank);
    *out = h;
  });
}

int mmadmm_plan_sizes(mmadmm_plan h, int* nLocalNodes, int* nLocalSimplices, int* simplexBegin, int* nSources,
                      int* nExport, int* maxExport) {
  return mmx::guarded([&] {
    if (!h) throw mmx::Error(MMADMM_ERR_INVALID, "null plan");
    const auto& p = h->p;
    if (nLocalNodes) *nLocalNodes = (int)p.localNodes.size();
    if (nLocalSimplices) *nLocalSimplices = p.s1 - p.s0;
    if (simplexBegin) *simplexBegin = p.s0;
    if (nSources) *nSources = (int)p.incSrc.size();
    if (nExport) *nExport = (int)p.exportOff.size();
    if (maxExport) *maxExport = p.maxExport;
  });
}

int mmadmm_plan_get(mmadmm_plan h, int32_t* localNodes, int32_t* incPtr, int32_t* incSrc, int32_t* exportOff) {
  return mmx::guarded([&] {
    if (!h) throw mmx::Error(MMADMM_ERR_INVALID, "null plan");
    const auto& p = h->p;
    if (localNodes) std::copy(p.localNodes.begin(), p.localNodes.end(), localNodes);
    if (incPtr) std::copy(p.incPtr.begin(), p.incPtr.end(), incPtr);
    if (incSrc) std::copy(p.incSrc.begin(), p.incSrc.end(), incSrc);
    if (exportOff) std::copy(p.exportOff.begin(), p.exportOff.end(), exportOff);
  });
}

int mmadmm_plan_destroy(mmadmm_plan h) {
  delete h;
  return MMADMM_OK;
}

}  // extern "C"
