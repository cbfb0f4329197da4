"""The RCCL deadline logic (csrc/comm_wait.h) on the CPU: a host program built from the
header with g++ polls fake conditions against a fake clock.  The communicators in
csrc/comm.cpp wait only through poll_until, so these cases are the fail-soft behaviour of
a first multi-GPU run that hangs inside RCCL."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "yet-another-halo2-fork_amd", "csrc")

PROG = r"""
#include "comm_wait.h"
#include <cstdio>
using namespace h2g::commwait;
struct FakeClock { double* t; double operator()() const { return *t; } };
struct FakeSleep { double* t; long* naps; int* maxnap; void operator()(int us) const {
  *t += us * 1e-6; (*naps)++; if (us > *maxnap) *maxnap = us; } };
int main() {
  double t = 0; long naps = 0; int maxnap = 0, calls = 0;
  FakeClock clk{&t}; FakeSleep sl{&t, &naps, &maxnap};
  // 1. done after 5 polls
  int r = poll_until([&] { return ++calls >= 5 ? POLL_DONE : POLL_PENDING; }, 1.0, clk, sl);
  printf("done %d %d\n", r, calls);
  // 2. an error ends the wait at once
  calls = 0;
  r = poll_until([&] { return ++calls >= 3 ? POLL_ERROR : POLL_PENDING; }, 1.0, clk, sl);
  printf("error %d %d\n", r, calls);
  // 3. never done: times out once the (fake) clock passes the deadline
  t = 0; calls = 0; naps = 0; maxnap = 0;
  r = poll_until([&] { ++calls; return POLL_PENDING; }, 2.5, clk, sl);
  printf("timeout %d %.6f %ld %d\n", r, t, naps, maxnap);
  // 4. no deadline: waits as long as it takes
  t = 0; calls = 0;
  r = poll_until([&] { return ++calls >= 20000 ? POLL_DONE : POLL_PENDING; }, 0.0, clk, sl);
  printf("nodeadline %d %d %.1f\n", r, calls, t);
  return 0;
}
"""


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    d = tmp_path_factory.mktemp("commwait")
    src, exe = d / "t.cpp", d / "t"
    src.write_text(PROG)
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", CSRC, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {ln.split()[0]: ln.split()[1:] for ln in out.splitlines()}


def test_poll_until_done(prog):
    assert prog["done"] == ["0", "5"]


def test_poll_until_error_stops_at_once(prog):
    assert prog["error"] == ["-1", "3"]


def test_poll_until_times_out_past_the_deadline(prog):
    r, t, naps, maxnap = prog["timeout"]
    assert r == "-2"
    assert 2.5 < float(t) <= 2.502  # returns within one (capped, 1 ms) nap of the deadline
    assert int(maxnap) == 1000 and int(naps) > 0


def test_poll_until_without_deadline_waits(prog):
    r, calls, _ = prog["nodeadline"]
    assert r == "0" and calls == "20000"


SERVE = r"""
#include "comm_wait.h"
#include <cstdio>
#include <vector>
using namespace h2g::commwait;
struct FakeClock { double* t; double operator()() const { return *t; } };
struct FakeSleep { double* t; void operator()(int us) const { *t += us * 1e-6; } };
// rank 0's headers as (arrival time, op); the peer's serve loop waits for each against its
// idle deadline (h2g_comm_set_serve_timeout), as comm_next_request does
int run(const std::vector<std::pair<double, int>>& hdrs, double idle, unsigned long long* served, double* t_end,
        int* answered) {
  double t = 0;
  size_t i = 0;
  FakeClock clk{&t};
  FakeSleep sl{&t};
  *answered = 0;
  auto next = [&](int* op) -> int {
    const int w = poll_until([&] { return i < hdrs.size() && hdrs[i].first <= t ? POLL_DONE : POLL_PENDING; }, idle,
                             clk, sl);
    if (w != WAIT_OK) return 3;  // H2G_ERR_DEVICE: rank 0 gone, communicators aborted
    *op = hdrs[i++].second;
    return 0;
  };
  auto answer = [&](int op) -> int { return op == REQ_MSM ? ((*answered)++, 0) : 2; };
  const int rc = serve_requests(next, answer, served);
  *t_end = t;
  return rc;
}
int main() {
  unsigned long long served = 0;
  double t = 0;
  int ans = 0;
  // 1. three MSMs and STOP: served 3
  int rc = run({{0.1, REQ_MSM}, {0.2, REQ_MSM}, {0.3, REQ_MSM}, {0.4, REQ_STOP}}, 5.0, &served, &t, &ans);
  printf("stop %d %llu %d\n", rc, served, ans);
  // 2. rank 0 aborts after two MSMs (no more headers): the peer returns an error once the
  //    idle deadline has passed, instead of waiting forever
  served = 777;
  rc = run({{0.1, REQ_MSM}, {0.2, REQ_MSM}}, 5.0, &served, &t, &ans);
  printf("abort %d %llu %d %.3f\n", rc, served, ans, t);
  // 3. a long idle period kept alive by PINGs every 4 s (deadline 5 s), then an MSM and STOP
  std::vector<std::pair<double, int>> h = {{0.1, REQ_MSM}};
  for (int k = 1; k <= 10; k++) h.push_back({0.1 + 4.0 * k, REQ_PING});
  h.push_back({40.5, REQ_MSM});
  h.push_back({40.6, REQ_STOP});
  rc = run(h, 5.0, &served, &t, &ans);
  printf("keepalive %d %llu %d\n", rc, served, ans);
  // 4. the same idle period without PINGs: fails at the first gap longer than the deadline
  rc = run({{0.1, REQ_MSM}, {40.5, REQ_MSM}, {40.6, REQ_STOP}}, 5.0, &served, &t, &ans);
  printf("gap %d %d %.3f\n", rc, ans, t);
  // 5. a malformed request ends the loop with answer()'s status
  rc = run({{0.1, REQ_MSM}, {0.2, 9}}, 5.0, &served, &t, &ans);
  printf("malformed %d %d\n", rc, ans);
  return 0;
}
"""


@pytest.fixture(scope="module")
def serve(tmp_path_factory):
    d = tmp_path_factory.mktemp("serve")
    src, exe = d / "s.cpp", d / "s"
    src.write_text(SERVE)
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", CSRC, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {ln.split()[0]: ln.split()[1:] for ln in out.splitlines()}


def test_serve_loop_stops_on_stop(serve):
    assert serve["stop"] == ["0", "3", "3"]


def test_serve_loop_rank0_abort_returns_an_error(serve):
    """shard mode's fail-soft hole: rank 0 stops sending (aborted or
    dead); the peer's serve loop fails once its idle deadline passes"""
    rc, served, ans, t = serve["abort"]
    assert rc == "3" and ans == "2" and served == "777"  # *served untouched on failure
    assert 5.2 < float(t) <= 5.202


def test_serve_loop_keepalive_renews_the_deadline(serve):
    assert serve["keepalive"] == ["0", "2", "2"]


def test_serve_loop_gap_without_keepalive_fails(serve):
    rc, ans, t = serve["gap"]
    assert rc == "3" and ans == "1" and float(t) < 6.0


def test_serve_loop_malformed_request(serve):
    assert serve["malformed"] == ["2", "1"]
