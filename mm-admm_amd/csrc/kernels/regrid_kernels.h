// regrid_kernels.h -- launch interface of the device monitor-grid set-up (regrid_kernels.hip),
// the time-varying-monitor path (DESIGN.md §Time-varying monitors).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace mmx {

// uniform cell grid over the vertices' bounding box (the nearest-vertex search structure)
struct CellGrid {
  double lo[3];
  double inv[3];  // cells per unit length (0 for a degenerate axis)
  int n[3];       // cells per axis (n[2] = 1 in 2D)
  double hmin;    // smallest cell edge
};

// a box of grid rows in STORAGE coordinates (row = k (nx+1)(ny+1) + sy (nx+1) + sx), inclusive
// bounds; the full grid is {0,0,0} .. {nx, ny, nz} (nz = 0 in 2D)
struct GridBox {
  int lo[3];
  int hi[3];
};

// per-block partial bounding boxes: partials[b * 2D + d] = min_d, [b * 2D + D + d] = max_d
template <int D>
void launch_bbox(const double* X, int n, double* partials, int nblocks, hipStream_t st);
// per-block widest simplex per axis: partials[b * D + d] = max over the block's simplices of the
// extent of their vertices along axis d (F: local simplices, D+1 local vertex ids each)
template <int D>
void launch_extent(const double* X, const int* F, int nF, double* partials, int nblocks, hipStream_t st);
// counting sort of the vertices into cells: starts[ncell + 1] (exclusive scan of counts),
// cellNodes[n]; counts must hold ncell + 1 ints, fill ncell
template <int D>
void launch_bin(const double* X, int n, const CellGrid& cg, int* cellOfV, int* counts, int* starts, int* fill,
                int* cellNodes, void* scanTmp, size_t scanTmpBytes, hipStream_t st);
size_t bin_scan_bytes(int ncell);
// MonType 7 at the vertices, centre c[3] of the moving bump at the current time
template <int D>
void launch_monitor_tv(const double* X, int n, const double* c, double* monVals, hipStream_t st);
// candidates of a partitioned regrid: global ids (the tie rule) and the search box S they were
// gathered from; every grid point checks its nearest candidate is strictly nearer than S's
// boundary, else *fail is set (gid == nullptr: every vertex, indexed by global id)
struct NnCand {
  const int* gid;
  double slo[3], shi[3];
  int* fail;
};
// nearest vertex of the grid point of every row in `box` -> its monitor value (host layout: 3D
// rows swap x and y, src/MeshInterpolator.cpp:234); rows enumerated in storage order
template <int D>
void launch_nn_fill(const double* X, const CellGrid& cg, const int* starts, const int* cellNodes, const double* gx,
                    const double* gy, const double* gz, int nx, int ny, int nz, const double* monVals, double* vals,
                    const GridBox& box, hipStream_t st, const NnCand& cand = NnCand{nullptr, {0, 0, 0}, {0, 0, 0}, nullptr});
// partitioned regrid: owned vertices inside other ranks' search boxes (sboxes: nranks x {lo[D],
// hi[D]}) appended as rows {x[D], gid} to send block q (rows q*cap ..); counts[q] must start at 0
template <int D>
void launch_select_owned(const double* X, const int* ownLocal, const int* ownGid, int nOwned, int nranks, int rank,
                         const double* sboxes, int* counts, double* send, int cap, hipStream_t st);
// candidates = this rank's vertices (X, gidLocal) then the received rows {x[D], gid}
template <int D>
void launch_build_cand(const double* X, const int* gidLocal, int nLocal, const double* recv, int nRecv, double* cx,
                       int* cgid, hipStream_t st);
// one Jacobi smoothing pass in -> out over the rows of `box` (the others are not written)
template <int D>
void launch_smooth(const double* in, double* out, int nx, int ny, int nz, const GridBox& box, hipStream_t st);
// partitioned regrid: vals (and, 3D, the 10-double padded copy) = src inside `box`, NaN outside it
// (a monitor evaluation outside the rank's box turns into a NaN energy: reported, never silent)
template <int D>
void launch_box_commit(const double* src, double* vals, double* pad, int nx, int ny, int nz, const GridBox& box,
                       hipStream_t st);

// rows of D doubles: out[i] = in[idx[i]] (gather) / out[idx[i]] = in[i] for idx[i] >= 0 (scatter)
void launch_rows_gather(int D, const int* idx, int n, const double* in, double* out, hipStream_t st);
void launch_rows_scatter(int D, const int* idx, int n, const double* in, double* out, hipStream_t st);

}  // namespace mmx
