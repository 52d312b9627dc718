// comm.h -- the communication the element-partitioned ADMM path needs: a halo exchange of
// interface-slot values with the neighbouring ranks (x-update and predictor sums, once per ADMM
// iteration), and an all-gather of small fixed-size fp64 blocks (per-step scalar partials; the
// vertex positions of a time-varying monitor's grid rebuild).  RCCL over xGMI between processes
// (one per GPU); a host-staged loopback between threads of one process, which lets the
// partitioned path be tested on a single GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <mutex>
#include <vector>

#include "partition.h"

namespace mmx {

struct Comm {
  int nranks = 1;
  virtual ~Comm() = default;
  // the ranks the transport itself reports (RCCL: ncclCommCount)
  virtual int transport_ranks() { return nranks; }
  // recv[q*count .. (q+1)*count) = rank q's send block (device pointers, stream-ordered)
  virtual void allgather(int rank, const double* dsend, double* drecv, size_t count, hipStream_t st) = 0;
  // for every peer p: send rows [p.sendOff, p.sendOff + p.sendCount) of dsend to p.rank, receive
  // p.recvCount rows from p.rank into drecv at row p.recvOff (rows of rowLen doubles, device
  // pointers, stream-ordered)
  virtual void exchange(int rank, const double* dsend, double* drecv, const std::vector<HaloPeer>& peers, int rowLen,
                        hipStream_t st) = 0;
  // the stream's work so far has completed (RCCL: bounded by the communicator's deadline, then
  // MMADMM_ERR_RCCL after an abort -- comm_poll.h; the host transports complete their transfers
  // inside the calls above)
  virtual void wait(hipStream_t st) {
    const hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) throw_hip(e);
  }
  static void throw_hip(hipError_t e);
};

Comm* make_rccl_comm(int nranks, int rank, const void* uid, int device, double timeout_s);
Comm* make_loopback_comm(int nranks);
void rccl_unique_id(void* out128);

}  // namespace mmx
