// comm_poll_check.cpp -- host unit test of the bounded wait (mm-admm_amd/csrc/host/comm_poll.h)
// behind the RCCL communicator's timeouts: a fake clock and fake states, no GPU, no RCCL.
// Built and run by tests/test_comm_timeout.py; prints "ok" and exits 0 when every case holds.
#include <cstdio>
#include <cstdlib>

#include "../../mm-admm_amd/csrc/host/comm_poll.h"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAILED line %d: %s\n", __LINE__, #c);           \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

int main() {
  using namespace mmx;
  // a peer that never joins: the state stays busy; the fake clock advances 1 s per pause
  {
    double t = 0.0;
    long polls = 0, pauses = 0;
    const int r = poll_bounded([&] { return kPollBusy; }, 30.0, [&] { return t; },
                               [&] {
                                 ++pauses;
                                 t += 1.0;
                               },
                               5, &polls);
    CHECK(r == kPollTimeout);
    CHECK(t >= 30.0 && t <= 31.0);  // ended at the deadline, not later
    CHECK(pauses == 30);
    CHECK(polls == 6 + 30);  // the first `spins` + 1 polls without a pause
  }
  // the communicator becomes ready after a while: no timeout, the state's answer is returned
  {
    double t = 0.0;
    int n = 0;
    const int r = poll_bounded([&] { return ++n < 50 ? kPollBusy : kPollReady; }, 30.0, [&] { return t; },
                               [&] { t += 0.1; }, 10);
    CHECK(r == kPollOk);
    CHECK(n == 50);
  }
  // an asynchronous error ends the wait at once
  {
    double t = 0.0;
    int n = 0;
    const int r = poll_bounded([&] { return ++n < 3 ? kPollBusy : kPollFailed; }, 30.0, [&] { return t; },
                               [&] { t += 1.0; }, 0);
    CHECK(r == kPollError);
    CHECK(n == 3);
  }
  // timeout <= 0: no deadline (ends only when the state does)
  {
    double t = 0.0;
    int n = 0;
    const int r = poll_bounded([&] { return ++n < 1000 ? kPollBusy : kPollReady; }, 0.0, [&] { return t; },
                               [&] { t += 100.0; }, 0);
    CHECK(r == kPollOk);
    CHECK(t > 1000.0);
  }
  // ready on the first poll: no clock reads beyond the start, no pause
  {
    int pauses = 0;
    const int r = poll_bounded([&] { return kPollReady; }, 1.0, [&] { return 0.0; }, [&] { ++pauses; }, 0);
    CHECK(r == kPollOk && pauses == 0);
  }
  // the real clock: a busy state times out after ~0.2 s
  {
    const double t0 = steady_seconds();
    const int r = poll_bounded([&] { return kPollBusy; }, 0.2, steady_seconds, short_sleep, 100);
    const double el = steady_seconds() - t0;
    CHECK(r == kPollTimeout);
    CHECK(el >= 0.2 && el < 2.0);
  }
  std::printf("ok\n");
  return 0;
}
