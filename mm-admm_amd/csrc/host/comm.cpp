// comm.cpp -- see comm.h.
#include "comm.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <string>

#include "comm_poll.h"
#include "common.h"

namespace mmx {
namespace {

#define MMX_NCCL(expr)                                                                              \
  do {                                                                                              \
    ncclResult_t r_ = (expr);                                                                       \
    if (r_ != ncclSuccess)                                                                          \
      throw ::mmx::Error(MMADMM_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_));      \
  } while (0)

// RCCL over xGMI, one process per GPU.  The communicator is non-blocking (config.blocking = 0):
// its creation and every call that reports ncclInProgress are polled against a deadline
// (comm_poll.h), and so is every stream wait of a partitioned step (wait()), so a rank that never
// joins or stops half-way ends the job with MMADMM_ERR_RCCL and a message naming the call, after
// ncclCommAbort -- not with a hang.
// The communicator's initialisation on a helper thread (RcclComm's constructor).  The helper owns
// the non-blocking group: it polls ncclCommGetAsyncError until the initialisation is complete
// before it exits (RCCL's asynchronous group job refers to the calling thread's thread-local group
// state: a helper that returned early left it dangling -- measured, a segfault at one rank).  The
// constructor, past its deadline, aborts the communicator itself while the helper is still
// blocked in ncclGroupEnd, or asks the polling helper to abort it; `mu` orders the two.
struct InitJob {
  std::mutex mu;
  int stage = 0;          // 1: handle known, 2: finished (res final)
  bool polling = false;   // the helper is past ncclGroupEnd
  bool aborted = false;   // ncclCommAbort was called (by either thread)
  bool abortReq = false;  // the constructor asks the polling helper to abort
  ncclComm_t comm = nullptr;
  ncclResult_t res = ncclSuccess;
  ncclUniqueId id;
  ncclConfig_t cfg;
};

struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;
  std::shared_ptr<InitJob> initJob_;
  int rank = 0;
  double timeout = 300.0;
  hipEvent_t ev = nullptr;
  RcclComm(int n, int r, const void* uid, int device, double timeout_s) {
    nranks = n;
    rank = r;
    timeout = timeout_s;
    MMX_HIP(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    // RCCL 2.27 blocks in the initialisation until every rank has joined even for a non-blocking
    // communicator (measured on the box with a rank that never comes: ncclCommInitRankConfig alone,
    // and ncclGroupEnd around it, never returned).  So it runs on a helper thread that hands over the
    // communicator's handle first; this thread waits for it against the deadline and, past it,
    // aborts the communicator (which ends the helper's wait) and reports MMADMM_ERR_RCCL.
    // the job (with the id and the config RCCL may still read after the call returns) lives as
    // long as this communicator, or as the helper thread if that outlives it
    auto job = std::make_shared<InitJob>();
    job->id = id;
    job->cfg = cfg;
    initJob_ = job;
    std::thread th([job, n, r, device]() {
      (void)hipSetDevice(device);
      ncclResult_t a = ncclGroupStart();
      ncclComm_t c = nullptr;
      if (a == ncclSuccess) a = ncclCommInitRankConfig(&c, n, job->id, r, &job->cfg);
      {
        std::lock_guard<std::mutex> lk(job->mu);
        job->comm = c;
        job->stage = 1;
      }
      const ncclResult_t b = ncclGroupEnd();
      ncclResult_t res = (a == ncclSuccess || a == ncclInProgress) ? b : a;
      {
        std::lock_guard<std::mutex> lk(job->mu);
        job->polling = true;
        if (job->aborted) {  // the constructor aborted while this thread was in ncclGroupEnd
          job->res = ncclInternalError;
          job->stage = 2;
          return;
        }
      }
      while (res == ncclInProgress) {
        {
          std::lock_guard<std::mutex> lk(job->mu);
          if (job->abortReq) {
            if (c) (void)ncclCommAbort(c);
            job->aborted = true;
            job->res = ncclInProgress;
            job->stage = 2;
            return;
          }
          ncclResult_t st = ncclInProgress;
          if (ncclCommGetAsyncError(c, &st) != ncclSuccess) st = ncclInternalError;
          res = st;
        }
        if (res == ncclInProgress) short_sleep();
      }
      std::lock_guard<std::mutex> lk(job->mu);
      job->res = res;
      job->stage = 2;
    });
    auto stage = [&] {
      std::lock_guard<std::mutex> lk(job->mu);
      return job->stage;
    };
    const int pr = poll_bounded([&] { return stage() == 2 ? kPollReady : kPollBusy; }, timeout, steady_seconds,
                                short_sleep, 100);
    if (pr == kPollOk) {
      th.join();
      if (dbg()) fprintf(stderr, "[mmx comm] rank %d: initialisation returned %d\n", rank, (int)job->res);
      if (job->res != ncclSuccess) {
        if (job->comm && !job->aborted) (void)ncclCommAbort(job->comm);
        throw Error(MMADMM_ERR_RCCL, "rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                                         ": ncclCommInitRankConfig: " + ncclGetErrorString(job->res));
      }
      comm = job->comm;
      return;
    }
    // past the deadline: abort -- here if the helper is blocked in ncclGroupEnd (the abort ends that
    // wait), else through the helper -- give it a little while to return, then report; a helper that
    // still does not return is left detached
    if (dbg()) fprintf(stderr, "[mmx comm] rank %d: initialisation past its deadline\n", rank);
    while (stage() < 1) short_sleep();  // the handle comes at once (the call queues in the group)
    {
      bool here = false;
      ncclComm_t c = nullptr;
      {
        std::lock_guard<std::mutex> lk(job->mu);
        if (job->stage < 2) {
          if (job->polling) {
            job->abortReq = true;
          } else {
            job->aborted = true;
            here = true;
            c = job->comm;
          }
        }
      }
      if (here && c) (void)ncclCommAbort(c);
    }
    const int pr2 = poll_bounded([&] { return stage() == 2 ? kPollReady : kPollBusy; }, 20.0, steady_seconds,
                                 short_sleep, 100);
    if (pr2 == kPollOk)
      th.join();
    else
      th.detach();
    comm = nullptr;
    throw Error(MMADMM_ERR_RCCL, "rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                                     ": ncclCommInitRankConfig (every rank must create its communicator): not complete "
                                     "after " + std::to_string(timeout) +
                                     " s (MMX_COMM_TIMEOUT_S) -- a peer rank is missing or stuck; communicator aborted");
  }
  ~RcclComm() override {
    if (ev) (void)hipEventDestroy(ev);
    if (!comm) return;
    // flush, then destroy; a peer that is gone makes the flush time out: abort instead
    ncclResult_t a = ncclCommFinalize(comm);
    if (a == ncclInProgress) a = settle_state();
    if (a == ncclSuccess)
      (void)ncclCommDestroy(comm);
    else
      (void)ncclCommAbort(comm);
  }
  // ncclCommGetAsyncError polled until it leaves ncclInProgress (or the deadline passes:
  // ncclInProgress is returned)
  ncclResult_t settle_state() {
    ncclResult_t last = ncclInProgress;
    const int pr = poll_bounded(
        [&] {
          ncclResult_t a = ncclInProgress;
          if (ncclCommGetAsyncError(comm, &a) != ncclSuccess) a = ncclInternalError;
          last = a;
          return a == ncclInProgress ? kPollBusy : a == ncclSuccess ? kPollReady : kPollFailed;
        },
        timeout, steady_seconds, short_sleep);
    return pr == kPollTimeout ? ncclInProgress : last;
  }
  static bool dbg() {
    static const bool on = getenv("MMX_COMM_DEBUG") != nullptr;
    return on;
  }
  [[noreturn]] void fail(const std::string& msg) {
    if (dbg()) fprintf(stderr, "[mmx comm] rank %d: %s -- aborting the communicator\n", rank, msg.c_str());
    if (comm) (void)ncclCommAbort(comm);
    if (dbg()) fprintf(stderr, "[mmx comm] rank %d: ncclCommAbort returned\n", rank);
    comm = nullptr;
    throw Error(MMADMM_ERR_RCCL, "rank " + std::to_string(rank) + " of " + std::to_string(nranks) + ": " + msg);
  }
  void check(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) r = settle_state();
    if (r == ncclInProgress)
      fail(std::string(what) + ": not complete after " + std::to_string(timeout) +
           " s (MMX_COMM_TIMEOUT_S) -- a peer rank is missing or stuck; communicator aborted");
    if (r != ncclSuccess) fail(std::string(what) + ": " + ncclGetErrorString(r));
  }
  void live(const char* what) {
    if (!comm) throw Error(MMADMM_ERR_RCCL, std::string(what) + ": the communicator was aborted by an earlier failure");
  }
  int transport_ranks() override {
    live("ncclCommCount");
    int n = 0;
    check(ncclCommCount(comm, &n), "ncclCommCount");
    return n;
  }
  void allgather(int, const double* dsend, double* drecv, size_t count, hipStream_t st) override {
    live("ncclAllGather");
    check(ncclAllGather(dsend, drecv, count, ncclDouble, comm, st), "ncclAllGather");
  }
  void exchange(int, const double* dsend, double* drecv, const std::vector<HaloPeer>& peers, int rowLen,
                hipStream_t st) override {
    if (peers.empty()) return;
    live("halo exchange");
    check(ncclGroupStart(), "ncclGroupStart");
    for (const HaloPeer& p : peers) {
      if (p.sendCount)
        check(ncclSend(dsend + (size_t)p.sendOff * rowLen, (size_t)p.sendCount * rowLen, ncclDouble, p.rank, comm, st),
              "ncclSend");
      if (p.recvCount)
        check(ncclRecv(drecv + (size_t)p.recvOff * rowLen, (size_t)p.recvCount * rowLen, ncclDouble, p.rank, comm, st),
              "ncclRecv");
    }
    check(ncclGroupEnd(), "ncclGroupEnd (halo send/recv)");
  }
  // the stream's work so far has completed, or the deadline passed (a peer's matching send/recv
  // never came) -- then the communicator is aborted, which also ends its kernels
  void wait(hipStream_t st) override {
    live("stream wait");
    if (!ev) MMX_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    MMX_HIP(hipEventRecord(ev, st));
    hipError_t herr = hipSuccess;
    ncclResult_t nerr = ncclSuccess;
    const int pr = poll_bounded(
        [&] {
          herr = hipEventQuery(ev);
          if (herr == hipSuccess) return kPollReady;
          if (herr != hipErrorNotReady) return kPollFailed;
          if (ncclCommGetAsyncError(comm, &nerr) == ncclSuccess && nerr != ncclSuccess && nerr != ncclInProgress)
            return kPollFailed;
          return kPollBusy;
        },
        timeout, steady_seconds, short_sleep, 20000);
    if (pr == kPollTimeout)
      fail("the partitioned step's stream did not complete within " + std::to_string(timeout) +
           " s (MMX_COMM_TIMEOUT_S) -- a peer rank is missing or stuck; communicator aborted");
    if (herr != hipSuccess && herr != hipErrorNotReady) MMX_HIP(herr);
    if (pr == kPollError) fail(std::string("asynchronous RCCL error: ") + ncclGetErrorString(nerr));
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

void Comm::throw_hip(hipError_t e) { throw Error(MMADMM_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e)); }

Comm* make_rccl_comm(int nranks, int rank, const void* uid, int device, double timeout_s) {
  return new RcclComm(nranks, rank, uid, device, timeout_s);
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
  return mmadmm_comm_create_rccl_timeout(nranks, rank, uid, device, mmx::comm_timeout_default(), out);
}

int mmadmm_comm_create_rccl_timeout(int nranks, int rank, const void* uid, int device, double timeout_s,
                                    mmadmm_comm* out) {
  return mmx::guarded([&] {
    if (!out || !uid || nranks < 1 || rank < 0 || rank >= nranks)
      throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_comm_create_rccl: bad arguments");
    *out = nullptr;
    auto* h = new mmadmm_comm_s{nullptr};
    try {
      h->c = mmx::make_rccl_comm(nranks, rank, uid, device, timeout_s);
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
