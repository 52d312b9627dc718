// comm.h -- the one collective the element-partitioned ADMM path needs: an all-gather of
// fixed-size fp64 blocks (interface-slot values, per-iteration scalar partials).  RCCL over xGMI
// between processes (one per GPU); a host-staged loopback between threads of one process, which
// lets the partitioned path be tested on a single GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <mutex>
#include <vector>

namespace mmx {

struct Comm {
  int nranks = 1;
  virtual ~Comm() = default;
  // recv[q*count .. (q+1)*count) = rank q's send block (device pointers, stream-ordered)
  virtual void allgather(int rank, const double* dsend, double* drecv, size_t count, hipStream_t st) = 0;
};

Comm* make_rccl_comm(int nranks, int rank, const void* uid, int device);
Comm* make_loopback_comm(int nranks);
void rccl_unique_id(void* out128);

}  // namespace mmx
