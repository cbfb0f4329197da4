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
