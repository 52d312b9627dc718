// staging.cpp -- large host-to-device uploads through pinned staging buffers (common.h
// upload_staged).  A hipMemcpyAsync from pageable memory moved the LASolver's set-up arrays at
// ~3-5 GB/s on the box (C4: ~1.5 GB of sweep stages and factor tables, ~0.4 s of the first
// backward-Euler step); here the source is copied into one of two pinned 32 MB buffers by the
// host threads while the other one's DMA runs.
#include <omp.h>

#include <algorithm>
#include <cstring>
#include <mutex>

#include "common.h"

namespace mmx {

void upload_staged(void* dst, const void* src, size_t bytes, hipStream_t st) {
  constexpr size_t kChunk = (size_t)32 << 20;
  static std::mutex mu;
  static char* buf[2] = {nullptr, nullptr};
  static hipEvent_t ev[2] = {nullptr, nullptr};
  static bool pending[2] = {false, false};
  std::lock_guard<std::mutex> lk(mu);
  if (!buf[0]) {
    for (int k = 0; k < 2; ++k) {
      MMX_HIP(hipHostMalloc((void**)&buf[k], kChunk, hipHostMallocDefault));
      MMX_HIP(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
    }
  }
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  int k = 0;
  for (size_t off = 0; off < bytes; off += kChunk, k ^= 1) {
    const size_t n = std::min(kChunk, bytes - off);
    if (pending[k]) MMX_HIP(hipEventSynchronize(ev[k]));  // the buffer's previous DMA has read it
    constexpr size_t kPiece = (size_t)1 << 20;
    const long long pieces = (long long)((n + kPiece - 1) / kPiece);
#pragma omp parallel for schedule(static)
    for (long long q = 0; q < pieces; ++q) {
      const size_t o = (size_t)q * kPiece;
      std::memcpy(buf[k] + o, s + off + o, std::min(kPiece, n - o));
    }
    MMX_HIP(hipMemcpyAsync(d + off, buf[k], n, hipMemcpyHostToDevice, st));
    MMX_HIP(hipEventRecord(ev[k], st));
    pending[k] = true;
  }
  // the source may be freed once this returns; the staging buffers are guarded by their events
}

}  // namespace mmx
