// g2.h -- host-side BN254 G2 (twist over Fq2 = Fq[u]/(u^2 + 1)) for the two G2 points
// of ParamsKZG (g2, s_g2 = [s] g2; poly/kzg/commitment.rs:24-27,122-123) and their
// RawBytes serialisation checks.  O(1) work per params object: plain host code.
//
// Layout = halo2curves' G2Affine: x = (c0, c1), y = (c0, c1), each an Fq in Montgomery
// form (4 x u64 LE) -> 16 u64 / 128 raw bytes; identity = all zero.
#pragma once
#include <cstring>

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

// ---- SerdeFormat::Processed for G2 (GroupEncoding over Fq2: x = c0 || c1 canonical LE,
// bit 7 of byte 63 = parity of canonical y.c0, identity = 64 zero bytes)
inline Fq2 fq2_pow(const Fq2& a, const uint32_t e[8]) {
  Fq2 acc{Fq::one(), Fq::zero()};
  for (int i = 7; i >= 0; i--)
    for (int b = 31; b >= 0; b--) {
      acc = fq2_sqr(acc);
      if ((e[i] >> b) & 1) acc = fq2_mul(acc, a);
    }
  return acc;
}
// a square root in Fq2 for p = 3 mod 4 (Adj & Rodriguez-Henriquez, eprint 2012/685,
// Algorithm 9); false if a is a non-residue.  Which of the two roots comes back does not
// matter: the decoder picks the one whose parity matches the sign bit.
inline bool fq2_sqrt(const Fq2& a, Fq2* out) {
  static constexpr uint32_t P34[8] = {0xb61f3f51u, 0x4f082305u, 0x5a1c72a3u, 0x65e05aa4u,
                                      0xa0605617u, 0x6e14116du, 0xb84c680au, 0x0c19139cu};  // (p-3)/4
  static constexpr uint32_t P12[8] = {0x6c3e7ea3u, 0x9e10460bu, 0xb438e546u, 0xcbc0b548u,
                                      0x40c0ac2eu, 0xdc2822dbu, 0x7098d014u, 0x18322739u};  // (p-1)/2
  if (fq2_is_zero(a)) {
    *out = a;
    return true;
  }
  const Fq2 a1 = fq2_pow(a, P34);
  const Fq2 alpha = fq2_mul(fq2_sqr(a1), a);
  const Fq2 x0 = fq2_mul(a1, a);
  const Fq2 minus_one{Fq::zero() - Fq::one(), Fq::zero()};
  Fq2 x;
  if (fq2_eq(alpha, minus_one)) {
    x = {Fq::zero() - x0.c1, x0.c0};  // u * x0
  } else {
    const Fq2 b = fq2_pow(fq2_add(alpha, {Fq::one(), Fq::zero()}), P12);
    x = fq2_mul(b, x0);
  }
  if (!fq2_eq(fq2_sqr(x), a)) return false;
  *out = x;
  return true;
}
inline void g2_compress(const G2Affine& p, uint8_t out[64]) {
  std::memset(out, 0, 64);
  if (p.is_identity()) return;
  const Fq x0 = to_canonical(p.x.c0), x1 = to_canonical(p.x.c1);
  std::memcpy(out, x0.l, 32);
  std::memcpy(out + 32, x1.l, 32);
  out[63] |= (uint8_t)((to_canonical(p.y.c0).l[0] & 1u) << 7);
}
inline bool g2_decompress(const uint8_t in[64], G2Affine* out) {
  Fq x0, x1;
  std::memcpy(x0.l, in, 32);
  std::memcpy(x1.l, in + 32, 32);
  const uint32_t ysign = x1.l[7] >> 31;
  x1.l[7] &= 0x7fffffffu;
  auto below = [](const Fq& v) {
    unsigned br = 0;
    for (int i = 0; i < 8; i++) (void)__builtin_subc(v.l[i], FqParams::M[i], br, &br);
    return br != 0;
  };
  if (!below(x0) || !below(x1)) return false;
  if (x0.is_zero() && x1.is_zero() && !ysign) {
    *out = G2Affine{{Fq::zero(), Fq::zero()}, {Fq::zero(), Fq::zero()}};
    return true;
  }
  const Fq2 x{from_canonical(x0), from_canonical(x1)};
  Fq2 y;
  if (!fq2_sqrt(fq2_add(fq2_mul(fq2_sqr(x), x), g2_b()), &y)) return false;
  if ((to_canonical(y.c0).l[0] & 1u) != ysign) y = {Fq::zero() - y.c0, Fq::zero() - y.c1};
  *out = G2Affine{x, y};
  return true;
}

}  // namespace h2g
