// partition.h -- element partition of the ADMM path across ranks (DESIGN.md
// §Multi-GPU).  Rank r owns the contiguous simplex range [sbeg[r], sbeg[r+1]) (generator order
// gives strips/slabs), its z, u, Bkinv and the nodes of its simplices; interface nodes are
// replicated.  The only coupling is the per-node sum over incident slots in the x-update and the
// gradient predictor: the sum runs over the node's incident slots in ascending GLOBAL simplex
// id, taking the other ranks' slots from an all-gathered buffer of interface-slot values, so
// every rank computes exactly the floating-point sums a single GPU does.
#pragma once
#include <cstdint>
#include <vector>

namespace mmx {

struct PartitionPlan {
  int nranks = 1, rank = 0;
  int nF = 0, nP = 0;              // global sizes
  std::vector<long long> sbeg;     // nranks+1 simplex boundaries
  int s0 = 0, s1 = 0;              // local simplex range
  std::vector<int> localNodes;     // global node ids, ascending (isolated nodes go to rank 0)
  std::vector<int> Flocal;         // local simplices, local node ids
  std::vector<int> incPtr;         // local node -> incident slot sources
  std::vector<int> incSrc;         // >= 0 local slot offset s*K + n*D; < 0: -1 - row of the remote buffer
  std::vector<int> valence;        // global number of incident slots per local node
  std::vector<int> exportOff;      // local slot offsets this rank exports, ascending (s, n)
  int maxExport = 0;               // rows per rank in the gathered buffer (padding)
};

// F: nF x (D+1) global node ids (already re-oriented).  Deterministic: every rank computes every
// rank's export order from the same global mesh, no communication needed.
PartitionPlan make_partition_plan(int D, int nP, int nF, const int32_t* F, int nranks, int rank);

}  // namespace mmx
