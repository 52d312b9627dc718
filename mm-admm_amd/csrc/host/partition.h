// partition.h -- element partition of the ADMM path across ranks (DESIGN.md
// §Multi-GPU).  Every simplex has one owner rank: by recursive coordinate bisection of the
// simplex centroids (default: compact parts, short interfaces, whatever the generator's
// numbering) or by contiguous ranges of global ids.  A rank owns its simplices' z, u, Bkinv and
// the nodes they touch; interface nodes are replicated.  The only coupling is the per-node sum
// over incident slots in the x-update and the gradient predictor: the sum runs over the node's
// incident slots in ascending GLOBAL simplex id, taking the other ranks' slots from a halo
// exchange with the neighbouring ranks only (each sends the values of its slots on the nodes it
// shares with that neighbour), so every rank computes exactly the floating-point sums a single
// GPU does.
#pragma once
#include <cstdint>
#include <vector>

namespace mmx {

enum PartitionMethod { kPartRCB = 0, kPartRanges = 1 };

// One neighbour of the halo exchange: rows of D doubles sent to / received from `rank`, at row
// offsets sendOff / recvOff of the send and receive buffers.
struct HaloPeer {
  int rank = 0;
  int sendOff = 0, sendCount = 0;
  int recvOff = 0, recvCount = 0;
};

struct PartitionPlan {
  int nranks = 1, rank = 0, method = kPartRCB;
  int nF = 0, nP = 0;                // global sizes
  std::vector<int> localSimplices;   // global simplex ids of this rank, ascending
  std::vector<int> localNodes;       // global node ids, ascending (isolated nodes go to rank 0)
  std::vector<int> Flocal;           // local simplices, local node ids
  std::vector<int> incPtr;           // local node -> incident slot sources
  std::vector<int> incSrc;           // >= 0 local slot offset s*K + n*D; < 0: -1 - row of the receive buffer
  std::vector<int> valence;          // global number of incident slots per local node
  std::vector<int> sendOff;          // local slot offsets sent, per peer in ascending peer rank, each (s, n) ascending
  std::vector<HaloPeer> peers;       // neighbour ranks, ascending
  int recvRows = 0;                  // rows of the receive buffer
  int interfaceNodes = 0;            // local nodes that some other rank also touches
  std::vector<int> nodeOwner;        // per global node: owner of its lowest incident simplex (0 if isolated)
};

// Owner rank of every simplex.  RCB: the centroids are bisected recursively along the longest
// extent of their bounding box, the ranks split in halves and the simplices in the same proportion
// -- the cut plane snapped to the vertex coordinate nearest the proportional centroid (a structured
// mesh is cut between cell layers), ties broken by global id.  Deterministic, so every rank
// computes the same owners.
std::vector<int> partition_owners(int D, int nP, const double* Xp, int nF, const int32_t* F, int nranks, int method);

// F: nF x (D+1) global node ids (already re-oriented); Xp: nP x D (needed by RCB).  Deterministic:
// every rank derives every rank's send order from the same global mesh, no communication needed.
PartitionPlan make_partition_plan(int D, int nP, const double* Xp, int nF, const int32_t* F, int nranks, int rank,
                                  int method = kPartRCB);

}  // namespace mmx
