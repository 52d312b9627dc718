// comm_poll.h -- bounded waits of the element-partitioned path (no HIP, no RCCL: unit-tested on
// the host by tests/cpp/comm_poll_check.cpp).
//
// A rank that never joins, or stops half-way, must end the run with a status code and a message,
// never with a silent hang: RCCL's communicator is created non-blocking (ncclCommInitRankConfig,
// config.blocking = 0) and every call that reports ncclInProgress -- the creation, a grouped
// send/recv, an all-gather -- and every stream wait of a partitioned step is polled here against
// a deadline; on expiry the caller aborts the communicator (ncclCommAbort) and reports
// MMADMM_ERR_RCCL.  The reference has no multi-process axis (its only parallelism is OpenMP over
// simplices, src/Mesh.cpp:945-948); this is the failure handling of the element partition that
// replaces it.
#pragma once
#include <chrono>
#include <cstdlib>
#include <thread>

namespace mmx {

enum PollState { kPollReady = 0, kPollBusy = 1, kPollFailed = 2 };
enum PollResult { kPollOk = 0, kPollError = -1, kPollTimeout = -2 };

// Polls `state()` until it is no longer kPollBusy or `timeout_s` has passed on `now()` (seconds,
// monotonic).  Between polls: `spins` busy polls, then `pause()` (a short sleep) -- the first
// polls stay cheap for the common case of a wait that ends within microseconds.  timeout_s <= 0
// waits without a deadline.  `polls` (optional) counts the calls of state().
template <class State, class Now, class Pause>
int poll_bounded(State&& state, double timeout_s, Now&& now, Pause&& pause, int spins = 1000, long* polls = nullptr) {
  const double t0 = now();
  for (long i = 0;; ++i) {
    const int s = state();
    if (polls) ++*polls;
    if (s == kPollReady) return kPollOk;
    if (s == kPollFailed) return kPollError;
    if (timeout_s > 0 && now() - t0 >= timeout_s) return kPollTimeout;
    if (i >= spins) pause();
  }
}

inline double steady_seconds() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline void short_sleep() { std::this_thread::sleep_for(std::chrono::microseconds(50)); }

// the deadline of a communicator wait: MMX_COMM_TIMEOUT_S (seconds; 0 = none), default 300 s --
// longer than any step or rendezvous of the bench's workloads, short enough that a stuck rank ends
// the job well inside a driver's time limit
inline double comm_timeout_default() {
  const char* e = std::getenv("MMX_COMM_TIMEOUT_S");
  if (e && *e) return std::atof(e);
  return 300.0;
}

}  // namespace mmx
