// staging.cpp -- large host-to-device uploads through pinned staging buffers (common.h
// upload_staged).  A hipMemcpyAsync from pageable memory moved the LASolver's set-up arrays at
// ~3-5 GB/s on the box (C4: ~1.5 GB of sweep stages and factor tables, ~0.4 s of the first
// backward-Euler step); here the source is copied into one of two pinned 32 MB buffers by the
// host threads while the other one's DMA runs.  Pairs of buffers are pooled per concurrent caller.
#include <omp.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

namespace mmx {

namespace {
// a pair of pinned chunks with the events of their last DMAs; pairs are pooled, so uploads from
// several host threads (the LASolver's schedule helpers) run concurrently
struct Staging {
  static constexpr size_t kChunk = (size_t)32 << 20;
  char* buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool pending[2] = {false, false};
};
std::mutex g_mu;
std::vector<Staging*> g_free;

Staging* acquire() {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_free.empty()) {
      Staging* s = g_free.back();
      g_free.pop_back();
      return s;
    }
  }
  auto* s = new Staging;
  for (int k = 0; k < 2; ++k) {
    MMX_HIP(hipHostMalloc((void**)&s->buf[k], Staging::kChunk, hipHostMallocDefault));
    MMX_HIP(hipEventCreateWithFlags(&s->ev[k], hipEventDisableTiming));
  }
  return s;
}
void give_back(Staging* s) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_free.push_back(s);
}
}  // namespace

void upload_staged(void* dst, const void* src, size_t bytes, hipStream_t st) {
  constexpr size_t kChunk = Staging::kChunk;
  Staging* sg = acquire();
  struct Back {  // the pair goes back to the pool on every way out (its events guard its chunks)
    Staging* s;
    ~Back() { give_back(s); }
  } back{sg};
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  int k = 0;
  for (size_t off = 0; off < bytes; off += kChunk, k ^= 1) {
    const size_t n = std::min(kChunk, bytes - off);
    if (sg->pending[k]) MMX_HIP(hipEventSynchronize(sg->ev[k]));  // the chunk's previous DMA has read it
    constexpr size_t kPiece = (size_t)1 << 20;
    const long long pieces = (long long)((n + kPiece - 1) / kPiece);
    char* b = sg->buf[k];
#pragma omp parallel for schedule(static)
    for (long long q = 0; q < pieces; ++q) {
      const size_t o = (size_t)q * kPiece;
      std::memcpy(b + o, s + off + o, std::min(kPiece, n - o));
    }
    MMX_HIP(hipMemcpyAsync(d + off, b, n, hipMemcpyHostToDevice, st));
    MMX_HIP(hipEventRecord(sg->ev[k], st));
    sg->pending[k] = true;
  }
  // the source may be freed once this returns; the staging chunks are guarded by their events
}

}  // namespace mmx
