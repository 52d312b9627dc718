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
//   * pairs (G = 2, rows of at most 16 entries): a position computes two consecutive rows of the
//     chain, the second taking the first's value from the register (its entry's code is the cell
//     after the import slots, never read); the lane's ring holds R rows, R / 2 positions;
//   * imports: values from other bands (or too old for the ring) are copied from the global
//     granules into LDS import slots by a helper wavefront, in order of first use (every slot
//     once, then the slot whose previous import's last reader passed longest ago, delivered once
//     the compute wave has passed that reader); it publishes how many it has delivered, and
//     iteration t waits for impNeed[t] (the highest it reads).
// Entries address one LDS array: [0] = +0.0 (pads: value 0 times +0.0 changes nothing, not even
// the sign of a zero), [1, 1 + 64 (R+1)) the lane rings, then RI import slots.
// Every row is computed by exactly the arithmetic of the level sweep (same entries, same order).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace mmx {

// an allocator whose resize() leaves ints uninitialised: the schedule's entry arrays (GBs at C4)
// are then first touched by the parallel fills that set them, not by one thread's zeroing
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    if constexpr (sizeof...(A) == 0)
      ::new ((void*)p) U;
    else
      ::new ((void*)p) U(std::forward<A>(a)...);
  }
};
using BigVec = std::vector<int, NoInitAlloc<int>>;
// v = n copies of x, filled in parallel
void big_fill(BigVec& v, size_t n, int x);

constexpr int kChainLanes = 64;
constexpr int kChainRingMax = 32;    // LDS ring slots per lane (doubles) -- chain_sweep.hip kRingMax
constexpr int kChainImpMax = 2048;   // LDS import slots (16-byte granules) -- chain_sweep.hip kImpMax
constexpr int kChainPad = -2147483647 - 1;  // empty entry slot (schedule building only)
constexpr int kChainFwd = -2147483647;      // entry whose value is the pair's first row (building only)
constexpr int kChainSegMax = 4;      // segments of E = 32 entries a row may take (rows up to 128 entries)
// rows of 33..48 entries (the 3D backward triangle: up to 44) take one position of a 48-entry stage
// with 16-bit codes instead of two 32-entry segments; its LDS budget leaves a ring of 8 rows per lane
// (chain_sweep.hip kRingWide; values farther back are imported).  MMX_CHAIN_E48=0: segments.
constexpr int kChainWideE = 48;
constexpr int kChainRingWide = 8;

struct ChainSchedule {
  bool ok = false;
  std::string why;      // reason when !ok
  bool fwd = true;
  int E = 0;            // entry slots per row segment (8, 16 or 32)
  bool seg = false;     // rows wider than 32 entries: split into segments at consecutive positions
  int G = 1;            // rows per position (2: consecutive chain rows as a pair, narrow rows only)
  int R = 0;            // ring slots per lane (power of two); ring stride R + 1
  int RI = 0;           // import slots (power of two)
  int nbands = 0, nchains = 0, maxLen = 0, maxSkew = 0, maxT = 0;
  long long slots = 0;      // sum over bands of their iteration counts
  long long nImports = 0;
  long long estIters = 0;   // simulated critical path (iterations)
  bool aligned = false;     // lane skews also wait for the lane's imports (chain_sched.cpp pass 1)
  std::vector<int> bandSlot, bandT, bandImp, bandNImp;  // per band
  std::vector<int> laneStart, laneLen, laneSkew;        // per band * 64 + lane (laneLen: rows if G = 2, else positions)
  std::vector<int> laneNs;                              // per band * 64 + lane: segments per row
  BigVec code;   // per ((slot * G + g) * E + e) * 64 + lane: LDS index of the value (0 for pads)
  BigVec src;    // same shape: index of the value in the factor (af), -1 for pads
  std::vector<int> dsrc;   // backward: per (slot * G + g) * 64 + lane, index of the diagonal in af (-1 idle)
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
// forceG: rows per position (0: automatic).  codes = false: the geometry only (bands, lanes, skews,
// slots, ring size, ticket order) -- no entry codes, sources or import tables (the factor schedule's
// use: it lays its own stages over the forward geometry).
ChainSchedule build_chain_schedule(int n, const std::vector<int>& iaf, const std::vector<int>& jaf,
                                   const std::vector<int>& dg, bool fwd, int forceG = 0, bool codes = true);

// ---- the numeric ILU(0) factor on the same chain/band schedule (chain_factor.hip) ----------------
// Row i of the factor (scaler_ILU::factor, ILU_class.cpp:300-527, IKJ order) restated target by
// target: entry e of the row (ascending column) receives, for each lower entry q < e in ascending
// order whose pivot row j_q holds column col(e) above its diagonal, w_e -= m_q * U(j_q, col e);
// then a lower entry becomes m_e = w_e / U(j_e, j_e).  Every entry gets exactly the reference's
// operations in the reference's order.  The values U(j, c) come from the lane rings (a row's
// diagonal and upper part, kFacWU values per ring slot) or are imported one by one.
constexpr int kFacWF = 18;   // entries per row (2D mesh rows: <= 18)
constexpr int kFacNL = 9;    // lower entries per row
constexpr int kFacWU = 14;   // diagonal + upper entries per row
constexpr int kFacNSC = 128; // 16-bit codes per row: the (e, q) update slots, then the kFacNL pivots (padded)
constexpr int kFacImpRows = 384;  // LDS import slots (rows; 2D meshes need <= ~330 live at once)
constexpr int kFacRMax = 4;       // ring slots per lane (rows)
// update slot of (e, q), q < min(e, kFacNL): sum over e' < e of min(e', kFacNL), plus q
constexpr int fac_slot(int e, int q) { return (e <= kFacNL ? e * (e - 1) / 2 : kFacNL * (kFacNL - 1) / 2 + (e - kFacNL) * kFacNL) + q; }
constexpr int kFacNUpd = fac_slot(kFacWF, 0);  // 117
// layouts of the per-iteration arrays as the kernel DMA-s them: 16-byte chunks per lane
inline size_t fac_vidx(size_t slot, int e, int l) { return ((slot * (kFacWF / 2) + e / 2) * 64 + l) * 2 + e % 2; }
inline size_t fac_cidx(size_t slot, int k, int l) { return ((slot * (kFacNSC / 8) + k / 8) * 64 + l) * 8 + k % 8; }
static_assert(kFacNUpd + kFacNL <= kFacNSC, "factor codes per row");

struct FactorSchedule {
  bool ok = false;
  std::string why;
  ChainSchedule geo;               // bands, lanes, skews, ticket order (forward, one row per position)
  int R = 0, RI = 0;
  long long slots = 0;
  std::vector<uint16_t, NoInitAlloc<uint16_t>> code;  // [slot][kFacNSC][lane]: LDS index of each (e, q) value / pivot (0: none)
  BigVec vsrc;                     // [slot][kFacWF][lane]: factor position of the row's entry e (-1: pad)
  std::vector<int> meta;           // [slot][lane]: W | nlow << 8 | 1 << 16 for a row (| 1 << 17 when
                                   // another band imports it: it publishes granules), 0 idle
  std::vector<int> rowStart;       // [slot][lane]: factor position of the row's first entry
  // imports are whole rows (their diagonal + upper part, kFacWU cells per slot), otherwise as in
  // ChainSchedule
  std::vector<int> impRow, impFree, impSlot, impWait, impNeed, bandImp, bandNImp;
  long long nImports = 0;
  int maxImpSlots = 0;
};
FactorSchedule build_factor_schedule(int n, const std::vector<int>& iaf, const std::vector<int>& jaf,
                                     const std::vector<int>& dg);
// Replays the schedule: every row's update and pivot values are the reference's (ring cells of the
// right row, written before and not overwritten; imports of the right position, delivered in time).
std::string validate_factor_schedule(const FactorSchedule& F, int n, const std::vector<int>& iaf,
                                     const std::vector<int>& jaf, const std::vector<int>& dg);

// Replays the lockstep execution of S: every row once, its entries in the reference's order, every
// ring read served by its producer's value written at an earlier iteration and not yet
// overwritten, every import the right row, read only while its slot holds it.  "" when valid.
std::string validate_chain_schedule(const ChainSchedule& S, int n, const std::vector<int>& iaf,
                                    const std::vector<int>& jaf, const std::vector<int>& dg);

}  // namespace mmx
