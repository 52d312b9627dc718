// chain_sched.h -- chain/band schedule of the ILU triangular sweeps.
//
// The level-scheduled sweep pays one cross-CU hand-off (~2 us) per level of the dependency DAG.
// Mesh matrices in natural order are mostly chains: row i depends on row i-1 (forward) or i+1
// (backward), and that entry is the LAST lower (FIRST upper) entry of the row, so it can be
// resolved in LDS without changing the order of the subtractions.  The schedule:
//   * chains: maximal runs of rows where each row depends on its predecessor in processing order;
//   * bands: 64 consecutive chains, one per lane of a wavefront; lane l processes position
//     p = t - skew[l] of its chain at iteration t, with static skews that satisfy every
//     dependency inside the band, whose values pass through a per-lane LDS ring;
//   * segments: a row wider than 32 entries (3D) takes ns consecutive positions of its lane, 32
//     entries each, its partial sum carried in a register; every row of a chain has the same ns;
//   * imports: values from other bands (or too old for the ring) are copied from the global
//     granules into LDS import slots by a helper wavefront, in order of first use (slots assigned
//     by interval colouring: the slot whose previous import's last use has passed); it publishes
//     how many it has delivered, and iteration t waits for impNeed[t] (the highest it reads).
// Entries address one LDS array: [0] = +0.0 (pads: value 0 times +0.0 changes nothing, not even
// the sign of a zero), [1, 1 + 64 (R+1)) the lane rings, then RI import slots.
// Every row is computed by exactly the arithmetic of the level sweep (same entries, same order).
#pragma once
#include <string>
#include <vector>

namespace mmx {

constexpr int kChainLanes = 64;
constexpr int kChainRingMax = 32;    // LDS ring slots per lane (doubles) -- chain_sweep.hip kRingMax
constexpr int kChainImpMax = 2048;   // LDS import slots (16-byte granules) -- chain_sweep.hip kImpMax
constexpr int kChainPad = -2147483647 - 1;  // empty entry slot (schedule building only)
constexpr int kChainSegMax = 4;      // segments of E = 32 entries a row may take (rows up to 128 entries)

struct ChainSchedule {
  bool ok = false;
  std::string why;      // reason when !ok
  bool fwd = true;
  int E = 0;            // entry slots per row segment (8, 16 or 32)
  bool seg = false;     // rows wider than 32 entries: split into segments at consecutive positions
  int R = 0;            // ring slots per lane (power of two); ring stride R + 1
  int RI = 0;           // import slots (power of two)
  int nbands = 0, nchains = 0, maxLen = 0, maxSkew = 0, maxT = 0;
  long long slots = 0;      // sum over bands of their iteration counts
  long long nImports = 0;
  long long estIters = 0;   // simulated critical path (iterations)
  bool aligned = false;     // lane skews also wait for the lane's imports (chain_sched.cpp pass 1)
  std::vector<int> bandSlot, bandT, bandImp, bandNImp;  // per band
  std::vector<int> laneStart, laneLen, laneSkew;        // per band * 64 + lane (laneLen in positions)
  std::vector<int> laneNs;                              // per band * 64 + lane: segments per row
  std::vector<int> code;   // per (slot * E + e) * 64 + lane: LDS index of the value (0 for pads)
  std::vector<int> src;    // same shape: index of the value in the factor (af), -1 for pads
  std::vector<int> dsrc;   // backward: per slot * 64 + lane, index of the diagonal in af (-1 idle)
  std::vector<int> impRow, impFree;  // per import: producer row; last iteration it is read
  std::vector<int> impSlot, impWait; // per import: LDS slot; iterations to complete before it is
                                     // delivered (the slot's previous import's last use, -1 none)
  int maxImpSlots = 0;               // the most import slots a band uses
  std::vector<int> impNeed;          // per slot: highest import index read at that iteration (-1)
  std::vector<int> bandE;            // per band: entry slots in use (multiple of 4, <= E)
  std::vector<int> bandOrder;        // per ticket: the band taken (every band after the bands it
                                     // imports from; long bands as early as their sources allow)
};

// fwd: unit-lower sweep over the entries [iaf[i], dg[i]); !fwd: upper sweep over (dg[i], iaf[i+1]).
ChainSchedule build_chain_schedule(int n, const std::vector<int>& iaf, const std::vector<int>& jaf,
                                   const std::vector<int>& dg, bool fwd);

// Replays the lockstep execution of S: every row once, its entries in the reference's order, every
// ring read served by its producer's value written at an earlier iteration and not yet
// overwritten, every import the right row, read only while its slot holds it.  "" when valid.
std::string validate_chain_schedule(const ChainSchedule& S, int n, const std::vector<int>& iaf,
                                    const std::vector<int>& jaf, const std::vector<int>& dg);

}  // namespace mmx
