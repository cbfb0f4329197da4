// comm_wait.h -- deadline polling for the RCCL communicators (comm.cpp).
//
// A first multi-GPU run that hangs inside RCCL (a communicator that never finishes
// connecting, a collective whose peer never arrives) must fail, not block: the bench's
// fallback chain (native RCCL -> torch over RCCL -> gloo) can only engage if every rank
// returns.  The communicators are created non-blocking (ncclConfig_t.blocking = 0) and
// every wait -- communicator setup, a collective's enqueue, its stream -- is a poll against
// one deadline; past it the caller aborts the communicators (ncclCommAbort) and reports
// the failure.  Header-only so the logic is unit-tested on the CPU
// (tests/test_comm_deadline_cpu.py builds a host program from it with g++).
#pragma once
#include <chrono>
#include <thread>

namespace h2g {
namespace commwait {

enum Poll { POLL_DONE = 1, POLL_PENDING = 0, POLL_ERROR = -1 };
enum Wait { WAIT_OK = 0, WAIT_ERROR = -1, WAIT_TIMEOUT = -2 };

struct SteadyClock {
  double operator()() const {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
};
struct SleepUs {
  void operator()(int us) const { std::this_thread::sleep_for(std::chrono::microseconds(us)); }
};

// poll() until it reports done or an error, or `timeout_s` (<= 0: no deadline) has passed
// on `now`.  Spins for the first ~50 us (collectives usually finish in tens of
// microseconds), then sleeps between polls with a growing interval capped at 1 ms.
template <class P, class Clock = SteadyClock, class Sleep = SleepUs>
int poll_until(P&& poll, double timeout_s, Clock now = Clock(), Sleep sleep = Sleep()) {
  const double t0 = now();
  int nap = 0;
  for (long it = 0;; it++) {
    const int r = poll();
    if (r == POLL_DONE) return WAIT_OK;
    if (r == POLL_ERROR) return WAIT_ERROR;
    if (timeout_s > 0 && now() - t0 > timeout_s) return WAIT_TIMEOUT;
    if (it >= 64) {
      nap = nap ? (2 * nap < 1000 ? 2 * nap : 1000) : 10;
      sleep(nap);
    }
  }
}

// A serving peer's loop (h2g_comm_serve, shard mode): rank 0's requests until its STOP.
// next(&op) waits for the next header -- against the serve loop's idle deadline, so a rank 0
// that aborted or died ends the loop with next's nonzero status instead of a wait that never
// returns; PING headers (rank 0's keep-alive while it idles) only renew that deadline;
// answer() serves one MSM request.  Returns 0 (and *served) after STOP, else the failing
// call's status.
enum Req { REQ_STOP = 0, REQ_MSM = 1, REQ_PING = 2 };
template <class Next, class Answer>
int serve_requests(Next&& next, Answer&& answer, unsigned long long* served) {
  unsigned long long count = 0;
  for (;;) {
    int op = REQ_STOP;
    const int rc = next(&op);
    if (rc != 0) return rc;
    if (op == REQ_STOP) break;
    if (op == REQ_PING) continue;
    const int ra = answer(op);
    if (ra != 0) return ra;
    count++;
  }
  if (served) *served = count;
  return 0;
}

}  // namespace commwait
}  // namespace h2g
