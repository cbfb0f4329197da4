// g2.h -- host-side BN254 G2 (twist over Fq2 = Fq[u]/(u^2 + 1)) for the two G2 points
// of ParamsKZG (g2, s_g2 = [s] g2; poly/kzg/commitment.rs:24-27,122-123) and their
// RawBytes serialisation checks.  O(1) work per params object: plain host code.
//
// Layout = halo2curves' G2Affine: x = (c0, c1), y = (c0, c1), each an Fq in Montgomery
// form (4 x u64 LE) -> 16 u64 / 128 raw bytes; identity = all zero.
#pragma once
#include "bn254.h"

namespace h2g {

struct Fq2 {
  Fq c0, c1;
};
inline Fq2 fq2_add(const Fq2& a, const Fq2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
inline Fq2 fq2_sub(const Fq2& a, const Fq2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
inline Fq2 fq2_mul(const Fq2& a, const Fq2& b) {
  // (a0 + a1 u)(b0 + b1 u) = a0 b0 - a1 b1 + (a0 b1 + a1 b0) u
  return {a.c0 * b.c0 - a.c1 * b.c1, a.c0 * b.c1 + a.c1 * b.c0};
}
inline Fq2 fq2_sqr(const Fq2& a) { return fq2_mul(a, a); }
inline Fq2 fq2_dbl(const Fq2& a) { return fq2_add(a, a); }
inline bool fq2_is_zero(const Fq2& a) { return a.c0.is_zero() && a.c1.is_zero(); }
inline bool fq2_eq(const Fq2& a, const Fq2& b) { return a.c0 == b.c0 && a.c1 == b.c1; }
inline Fq2 fq2_inv(const Fq2& a) {
  const Fq t = inv(a.c0 * a.c0 + a.c1 * a.c1);  // 1 / (a0^2 + a1^2)
  return {a.c0 * t, (Fq::zero() - a.c1) * t};
}
// b' = 3 / (9 + u), the coefficient of the D-type twist y^2 = x^3 + b'
inline Fq2 g2_b() {
  const Fq2 nine_u{from_u64<FqParams>(9), Fq::one()};
  const Fq2 three{from_u64<FqParams>(3), Fq::zero()};
  return fq2_mul(three, fq2_inv(nine_u));
}

struct G2Affine {
  Fq2 x, y;
  bool is_identity() const { return fq2_is_zero(x) && fq2_is_zero(y); }
};
struct G2Jac {  // x = X / Z^2, y = Y / Z^3; identity Z = 0
  Fq2 X, Y, Z;
};

inline bool g2_on_curve(const G2Affine& p) {
  if (p.is_identity()) return true;
  const Fq2 rhs = fq2_add(fq2_mul(fq2_sqr(p.x), p.x), g2_b());
  return fq2_eq(fq2_sqr(p.y), rhs);
}

// standard BN254 G2 generator (halo2curves G2_GENERATOR_X / _Y), canonical limbs
inline G2Affine g2_generator() {
  auto fq = [](uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    Fq v;
    const uint64_t w[4] = {a, b, c, d};
    for (int i = 0; i < 4; i++) {
      v.l[2 * i] = (uint32_t)w[i];
      v.l[2 * i + 1] = (uint32_t)(w[i] >> 32);
    }
    return from_canonical(v);
  };
  G2Affine g;
  g.x.c0 = fq(0x46debd5cd992f6edull, 0x674322d4f75edaddull, 0x426a00665e5c4479ull, 0x1800deef121f1e76ull);
  g.x.c1 = fq(0x97e485b7aef312c2ull, 0xf1aa493335a9e712ull, 0x7260bfb731fb5d25ull, 0x198e9393920d483aull);
  g.y.c0 = fq(0x4ce6cc0166fa7daaull, 0xe3d1e7690c43d37bull, 0x4aab71808dcb408full, 0x12c85ea5db8c6debull);
  g.y.c1 = fq(0x55acdadcd122975bull, 0xbc4b313370b38ef3ull, 0xec9e99ad690c3395ull, 0x090689d0585ff075ull);
  return g;
}

inline G2Jac g2_dbl(const G2Jac& p) {  // dbl-2009-l (a = 0)
  if (fq2_is_zero(p.Z)) return p;
  const Fq2 A = fq2_sqr(p.X), B = fq2_sqr(p.Y), C = fq2_sqr(B);
  const Fq2 D = fq2_dbl(fq2_sub(fq2_sub(fq2_sqr(fq2_add(p.X, B)), A), C));
  const Fq2 E = fq2_add(fq2_dbl(A), A), F = fq2_sqr(E);
  G2Jac r;
  r.X = fq2_sub(F, fq2_dbl(D));
  r.Y = fq2_sub(fq2_mul(E, fq2_sub(D, r.X)), fq2_dbl(fq2_dbl(fq2_dbl(C))));
  r.Z = fq2_dbl(fq2_mul(p.Y, p.Z));
  return r;
}
inline G2Jac g2_add_affine(const G2Jac& p, const G2Affine& q) {  // madd-2007-bl
  if (q.is_identity()) return p;
  if (fq2_is_zero(p.Z)) return {q.x, q.y, {Fq::one(), Fq::zero()}};
  const Fq2 Z1Z1 = fq2_sqr(p.Z);
  const Fq2 U2 = fq2_mul(q.x, Z1Z1), S2 = fq2_mul(fq2_mul(q.y, p.Z), Z1Z1);
  const Fq2 H = fq2_sub(U2, p.X), rr = fq2_dbl(fq2_sub(S2, p.Y));
  if (fq2_is_zero(H)) {
    if (fq2_is_zero(rr)) return g2_dbl({q.x, q.y, {Fq::one(), Fq::zero()}});
    return {{Fq::one(), Fq::zero()}, {Fq::one(), Fq::zero()}, {Fq::zero(), Fq::zero()}};
  }
  const Fq2 HH = fq2_sqr(H), I = fq2_dbl(fq2_dbl(HH)), J = fq2_mul(H, I), V = fq2_mul(p.X, I);
  G2Jac r;
  r.X = fq2_sub(fq2_sub(fq2_sqr(rr), J), fq2_dbl(V));
  r.Y = fq2_sub(fq2_mul(rr, fq2_sub(V, r.X)), fq2_dbl(fq2_mul(p.Y, J)));
  r.Z = fq2_sub(fq2_sub(fq2_sqr(fq2_add(p.Z, H)), Z1Z1), HH);
  return r;
}
inline G2Affine g2_to_affine(const G2Jac& p) {
  if (fq2_is_zero(p.Z)) return G2Affine{{Fq::zero(), Fq::zero()}, {Fq::zero(), Fq::zero()}};
  const Fq2 zi = fq2_inv(p.Z), zi2 = fq2_sqr(zi);
  return {fq2_mul(p.X, zi2), fq2_mul(fq2_mul(p.Y, zi2), zi)};
}
// [s] P for a canonical scalar s (8 LE u32 limbs), MSB-first double-and-add
inline G2Affine g2_mul(const G2Affine& p, const uint32_t s[8]) {
  G2Jac acc{{Fq::one(), Fq::zero()}, {Fq::one(), Fq::zero()}, {Fq::zero(), Fq::zero()}};
  for (int i = 7; i >= 0; i--)
    for (int b = 31; b >= 0; b--) {
      acc = g2_dbl(acc);
      if ((s[i] >> b) & 1) acc = g2_add_affine(acc, p);
    }
  return g2_to_affine(acc);
}

}  // namespace h2g
