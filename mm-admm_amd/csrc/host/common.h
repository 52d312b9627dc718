// common.h -- host-side helpers shared by the libmmadmm translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/mmadmm.h"

namespace mmx {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);
// every kernel object's layout word equals the calling host TU's (kernels/layout.h kLayoutWord as
// that TU was compiled), else MMADMM_ERR_INVALID
void check_kernel_layout(unsigned hostWord);

#define MMX_HIP(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      throw ::mmx::Error(MMADMM_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Run f, translate exceptions to status codes (no exception crosses the C-ABI).
template <class Fn>
int guarded(Fn&& f) {
  try {
    f();
    return MMADMM_OK;
  } catch (const Error& e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error("out of host memory");
    return MMADMM_ERR_INVALID;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return MMADMM_ERR_INVALID;
  }
}

// dst <- src (bytes) on stream st through pinned staging buffers (staging.cpp); src may be freed
// when it returns
void upload_staged(void* dst, const void* src, size_t bytes, hipStream_t st);

// Owning device buffer (hipMalloc / hipFree).
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  void alloc(size_t count) {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = count;
    if (count) MMX_HIP(hipMalloc(&p, count * sizeof(T)));
  }
  void upload(const T* h, size_t count, hipStream_t st) {
    alloc(count);
    if (count * sizeof(T) >= ((size_t)16 << 20))  // large: pinned staging (~5x the pageable rate)
      upload_staged(p, h, count * sizeof(T), st);
    else if (count)
      MMX_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, st));
  }
};

// Built-in monitors (Experiments/TestMonitors/MEx*.h restated), by MonType
void builtin_monitor_eval(int dim, int monType, const double* x, double* M);

// Host mesh buffer behind mmadmm_mesh
struct MeshBuf {
  int dim = 2;
  std::vector<double> Vp;
  std::vector<int32_t> F;
  std::vector<int32_t> mask;
  std::vector<double> Vc;  // reference positions when they differ from Vp (Shoulder), else empty
  int nP() const { return (int)(Vp.size() / dim); }
  int nF() const { return (int)(F.size() / (dim + 1)); }
};

// Smoothed monitor grid (src/MeshInterpolator.cpp:68-130, 166-259, 366-404)
struct HostGrid {
  int nx = 0, ny = 0, nz = 0;
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};  // linspace end points (bounding box)
  std::vector<double> gx, gy, gz;
  std::vector<double> vals;  // rows x dim*dim
};
void build_monitor_grid(int dim, const double* X, int nP, mmadmm_monitor_fn fn, void* user,
                        HostGrid& g);
// grid size and linspace coordinates from the vertex count and bounding box (updateMesh,
// src/MeshInterpolator.cpp:68-130); vals is not touched
void grid_geometry(int dim, int nP, const double* lo, const double* hi, HostGrid& g);
// built-in monitor behind (fn, user) (MonType), or -1 for a user callback
int builtin_monitor_kind(mmadmm_monitor_fn fn, void* user);
// MonType 7's centre at time t
void moving_bump_centre(double t, double c[3]);

struct Comm;
Comm* comm_of(mmadmm_comm c);

}  // namespace mmx
