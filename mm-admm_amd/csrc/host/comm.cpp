// comm.cpp -- see comm.h.
#include "comm.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "common.h"

namespace mmx {
namespace {

#define MMX_NCCL(expr)                                                                              \
  do {                                                                                              \
    ncclResult_t r_ = (expr);                                                                       \
    if (r_ != ncclSuccess)                                                                          \
      throw ::mmx::Error(MMADMM_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_));      \
  } while (0)

struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;
  RcclComm(int n, int rank, const void* uid, int device) {
    nranks = n;
    MMX_HIP(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    MMX_NCCL(ncclCommInitRank(&comm, n, id, rank));
  }
  ~RcclComm() override {
    if (comm) (void)ncclCommDestroy(comm);
  }
  int transport_ranks() override {
    int n = 0;
    MMX_NCCL(ncclCommCount(comm, &n));
    return n;
  }
  void allgather(int, const double* dsend, double* drecv, size_t count, hipStream_t st) override {
    MMX_NCCL(ncclAllGather(dsend, drecv, count, ncclDouble, comm, st));
  }
  void exchange(int, const double* dsend, double* drecv, const std::vector<HaloPeer>& peers, int rowLen,
                hipStream_t st) override {
    if (peers.empty()) return;
    MMX_NCCL(ncclGroupStart());
    for (const HaloPeer& p : peers) {
      if (p.sendCount)
        MMX_NCCL(ncclSend(dsend + (size_t)p.sendOff * rowLen, (size_t)p.sendCount * rowLen, ncclDouble, p.rank, comm, st));
      if (p.recvCount)
        MMX_NCCL(ncclRecv(drecv + (size_t)p.recvOff * rowLen, (size_t)p.recvCount * rowLen, ncclDouble, p.rank, comm, st));
    }
    MMX_NCCL(ncclGroupEnd());
  }
};

// Threads of one process, one per rank, all on the same or on different devices.
struct LoopbackComm final : Comm {
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long long generation = 0;
  std::vector<std::vector<double>> slots;
  std::vector<std::vector<std::vector<double>>> mail;  // mail[from][to]
  explicit LoopbackComm(int n) : slots(n), mail(n, std::vector<std::vector<double>>(n)) { nranks = n; }
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const long long g = generation;
    if (++arrived == nranks) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != g; });
    }
  }
  void allgather(int rank, const double* dsend, double* drecv, size_t count, hipStream_t st) override {
    slots[rank].resize(count);
    if (count) MMX_HIP(hipMemcpyAsync(slots[rank].data(), dsend, count * sizeof(double), hipMemcpyDeviceToHost, st));
    MMX_HIP(hipStreamSynchronize(st));
    barrier();
    for (int q = 0; q < nranks; ++q)
      if (count)
        MMX_HIP(hipMemcpyAsync(drecv + (size_t)q * count, slots[q].data(), count * sizeof(double),
                               hipMemcpyHostToDevice, st));
    MMX_HIP(hipStreamSynchronize(st));
    barrier();
  }
  void exchange(int rank, const double* dsend, double* drecv, const std::vector<HaloPeer>& peers, int rowLen,
                hipStream_t st) override {
    for (const HaloPeer& p : peers) {
      auto& box = mail[rank][p.rank];
      box.resize((size_t)p.sendCount * rowLen);
      if (!box.empty())
        MMX_HIP(hipMemcpyAsync(box.data(), dsend + (size_t)p.sendOff * rowLen, box.size() * sizeof(double),
                               hipMemcpyDeviceToHost, st));
    }
    MMX_HIP(hipStreamSynchronize(st));
    barrier();
    for (const HaloPeer& p : peers) {
      const auto& box = mail[p.rank][rank];
      if (box.size() != (size_t)p.recvCount * rowLen) throw Error(MMADMM_ERR_INVALID, "loopback exchange: size mismatch");
      if (!box.empty())
        MMX_HIP(hipMemcpyAsync(drecv + (size_t)p.recvOff * rowLen, box.data(), box.size() * sizeof(double),
                               hipMemcpyHostToDevice, st));
    }
    MMX_HIP(hipStreamSynchronize(st));
    barrier();
  }
};

// Transfers done by the caller (e.g. torch.distributed over gloo, or MPI, in the host process of
// each rank): device blocks are staged through pinned host buffers and handed to the callbacks.
// Every rank makes the same sequence of allgather / exchange calls (the engine's schedule), so the
// callbacks can match their messages by call order.
struct HostComm final : Comm {
  int rank = 0;
  mmadmm_allgather_fn ag;
  mmadmm_exchange_fn ex;
  void* user;
  double* hs = nullptr;
  double* hr = nullptr;
  size_t cs = 0, cr = 0;
  HostComm(int n, int r, mmadmm_allgather_fn a, mmadmm_exchange_fn e, void* u) : rank(r), ag(a), ex(e), user(u) {
    nranks = n;
  }
  ~HostComm() override {
    if (hs) (void)hipHostFree(hs);
    if (hr) (void)hipHostFree(hr);
  }
  void reserve(size_t ns, size_t nr) {
    if (ns > cs) {
      if (hs) MMX_HIP(hipHostFree(hs));
      hs = nullptr;
      MMX_HIP(hipHostMalloc((void**)&hs, ns * sizeof(double), hipHostMallocDefault));
      cs = ns;
    }
    if (nr > cr) {
      if (hr) MMX_HIP(hipHostFree(hr));
      hr = nullptr;
      MMX_HIP(hipHostMalloc((void**)&hr, nr * sizeof(double), hipHostMallocDefault));
      cr = nr;
    }
  }
  void allgather(int, const double* dsend, double* drecv, size_t count, hipStream_t st) override {
    reserve(std::max<size_t>(count, 1), std::max<size_t>(count * nranks, 1));
    if (count) MMX_HIP(hipMemcpyAsync(hs, dsend, count * sizeof(double), hipMemcpyDeviceToHost, st));
    MMX_HIP(hipStreamSynchronize(st));
    if (ag(user, hs, hr, (long long)count) != 0) throw Error(MMADMM_ERR_RCCL, "host transport: allgather failed");
    if (count) MMX_HIP(hipMemcpyAsync(drecv, hr, count * nranks * sizeof(double), hipMemcpyHostToDevice, st));
    MMX_HIP(hipStreamSynchronize(st));
  }
  void exchange(int, const double* dsend, double* drecv, const std::vector<HaloPeer>& peers, int rowLen,
                hipStream_t st) override {
    const int np = (int)peers.size();
    std::vector<int> pr(np);
    std::vector<long long> so(np), sc(np), ro(np), rc(np);
    size_t ns = 1, nr = 1;
    for (int i = 0; i < np; ++i) {
      const HaloPeer& p = peers[i];
      pr[i] = p.rank;
      so[i] = (long long)p.sendOff * rowLen;
      sc[i] = (long long)p.sendCount * rowLen;
      ro[i] = (long long)p.recvOff * rowLen;
      rc[i] = (long long)p.recvCount * rowLen;
      ns = std::max(ns, (size_t)(so[i] + sc[i]));
      nr = std::max(nr, (size_t)(ro[i] + rc[i]));
    }
    reserve(ns, nr);
    for (int i = 0; i < np; ++i)
      if (sc[i])
        MMX_HIP(hipMemcpyAsync(hs + so[i], dsend + so[i], sc[i] * sizeof(double), hipMemcpyDeviceToHost, st));
    MMX_HIP(hipStreamSynchronize(st));
    // called on every exchange, also with no peers, so the callbacks see the same call sequence on all ranks
    if (ex(user, np, pr.data(), hs, so.data(), sc.data(), hr, ro.data(), rc.data()) != 0)
      throw Error(MMADMM_ERR_RCCL, "host transport: exchange failed");
    for (int i = 0; i < np; ++i)
      if (rc[i])
        MMX_HIP(hipMemcpyAsync(drecv + ro[i], hr + ro[i], rc[i] * sizeof(double), hipMemcpyHostToDevice, st));
    MMX_HIP(hipStreamSynchronize(st));
  }
};

}  // namespace

Comm* make_rccl_comm(int nranks, int rank, const void* uid, int device) {
  return new RcclComm(nranks, rank, uid, device);
}
Comm* make_loopback_comm(int nranks) { return new LoopbackComm(nranks); }
void rccl_unique_id(void* out128) {
  ncclUniqueId id;
  MMX_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof(id));
}

}  // namespace mmx

struct mmadmm_comm_s {
  mmx::Comm* c;
};

extern "C" {

int mmadmm_comm_unique_id(void* out, int len) {
  return mmx::guarded([&] {
    if (!out || len < MMADMM_UNIQUE_ID_BYTES) throw mmx::Error(MMADMM_ERR_INVALID, "unique id buffer too small");
    mmx::rccl_unique_id(out);
  });
}

int mmadmm_comm_create_rccl(int nranks, int rank, const void* uid, int device, mmadmm_comm* out) {
  return mmx::guarded([&] {
    if (!out || !uid || nranks < 1 || rank < 0 || rank >= nranks)
      throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_comm_create_rccl: bad arguments");
    *out = nullptr;
    auto* h = new mmadmm_comm_s{nullptr};
    try {
      h->c = mmx::make_rccl_comm(nranks, rank, uid, device);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int mmadmm_comm_create_loopback(int nranks, mmadmm_comm* out) {
  return mmx::guarded([&] {
    if (!out || nranks < 1) throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_comm_create_loopback: bad arguments");
    *out = new mmadmm_comm_s{mmx::make_loopback_comm(nranks)};
  });
}

int mmadmm_comm_create_host(int nranks, int rank, mmadmm_allgather_fn allgather, mmadmm_exchange_fn exchange,
                            void* user, mmadmm_comm* out) {
  return mmx::guarded([&] {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || !allgather || !exchange)
      throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_comm_create_host: bad arguments");
    *out = new mmadmm_comm_s{new mmx::HostComm(nranks, rank, allgather, exchange, user)};
  });
}

int mmadmm_comm_nranks(mmadmm_comm c, int* nranks) {
  return mmx::guarded([&] {
    if (!c || !c->c || !nranks) throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_comm_nranks: bad arguments");
    *nranks = c->c->transport_ranks();
  });
}

int mmadmm_comm_destroy(mmadmm_comm c) {
  if (!c) return MMADMM_OK;
  delete c->c;
  delete c;
  return MMADMM_OK;
}

}  // extern "C"

namespace mmx {
Comm* comm_of(mmadmm_comm c) { return c ? c->c : nullptr; }
}  // namespace mmx
