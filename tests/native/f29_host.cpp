// f29_host.cpp -- the F29 primitives of csrc/f29.h driven on the host (test harness only).
//
// Built by tests/test_f29_host_cpu.py with hipcc for the host side only (the same
// H2G_HD functions the kernels inline).  Reads one operation per line from stdin,
// "op limbs...", every F29 value as 9 decimal 32-bit limbs (a point: X Y ZZ ZZZ, 36 limbs),
// and prints the result's limbs on one line.  Python picks the operands at the bounds
// tools/f29_bounds.py derives and checks the results with big integers.
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>

#include "f29.h"

using namespace h2g;

static bool rd(std::istringstream& in, F29& v) {
  for (int i = 0; i < 9; i++)
    if (!(in >> v.l[i])) return false;
  return true;
}
static bool rdp(std::istringstream& in, G1xyzz29& p) { return rd(in, p.X) && rd(in, p.Y) && rd(in, p.ZZ) && rd(in, p.ZZZ); }
static void wr(const F29& v) {
  for (int i = 0; i < 9; i++) printf("%s%u", i ? " " : "", v.l[i]);
}
static void wrp(const G1xyzz29& p) {
  wr(p.X), printf(" "), wr(p.Y), printf(" "), wr(p.ZZ), printf(" "), wr(p.ZZZ);
}

// every sub29<P, K, OFF> instantiation the kernels use (f29.h, msm.hip, ntt.hip, prover_kernels.hip)
#define SUB_CASES(X)                                                                                           \
  X(q, FqParams, 64, 29) X(q, FqParams, 32, 31) X(q, FqParams, 16, 29) X(q, FqParams, 4, 31) X(q, FqParams, 4, 29) \
  X(q, FqParams, 2, 29) X(r, FrParams, 64, 29) X(r, FrParams, 4, 29) X(r, FrParams, 8, 29) X(r, FrParams, 16, 29)  \
  X(r, FrParams, 32, 29) X(r, FrParams, 64, 29) X(r, FrParams, 128, 29)

static bool run(const std::string& op, std::istringstream& in) {
  F29 a, b, c, d;
  G1xyzz29 p, q;
  if (op == "mulq" || op == "mulr") {
    if (!rd(in, a) || !rd(in, b)) return false;
    wr(op == "mulq" ? mul29<FqParams>(a, b) : mul29<FrParams>(a, b));
  } else if (op == "sqrq" || op == "sqrr") {
    if (!rd(in, a)) return false;
    wr(op == "sqrq" ? sqr29<FqParams>(a) : sqr29<FrParams>(a));
  } else if (op == "mulx2q" || op == "mulx2r") {
    if (!rd(in, a) || !rd(in, b) || !rd(in, c) || !rd(in, d)) return false;
    wr(op == "mulx2q" ? mul29x2<FqParams>(a, b, c, d) : mul29x2<FrParams>(a, b, c, d));
  } else if (op == "redq" || op == "redr") {
    if (!rd(in, a)) return false;
    wr(op == "redq" ? reduce29<FqParams>(a) : reduce29<FrParams>(a));
  } else if (op == "iszq" || op == "iszr") {
    if (!rd(in, a)) return false;
    printf("%d", op == "iszq" ? (int)is_zero29<FqParams>(a) : (int)is_zero29<FrParams>(a));
  } else if (op == "norm") {
    if (!rd(in, a)) return false;
    wr(norm29(a));
  } else if (op == "madd") {
    if (!rdp(in, p) || !rd(in, a) || !rd(in, b)) return false;
    wrp(xyzz29_madd(p, a, b));
  } else if (op == "add") {
    if (!rdp(in, p) || !rdp(in, q)) return false;
    wrp(xyzz29_add(p, q));
  } else if (op == "dbl") {
    if (!rdp(in, p)) return false;
    wrp(xyzz29_dbl(p));
  }
#define SUB_OP(f, P, K, OFF)                                                                \
  else if (op == "sub" #f "_" #K "_" #OFF) {                                                \
    if (!rd(in, a) || !rd(in, b)) return false;                                             \
    wr(sub29<P, K, OFF>(a, b));                                                             \
  }
  SUB_CASES(SUB_OP)
#undef SUB_OP
  else {
    return false;
  }
  return true;
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string op;
    if (!(in >> op)) continue;
    if (!run(op, in)) {
      printf("ERR %s", op.c_str());
    }
    printf("\n");
  }
  return 0;
}
