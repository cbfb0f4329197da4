// f29.h -- BN254 field elements in 9 unsaturated 29-bit limbs (Montgomery, R = 2^261).
//
// Why: the 8 x 32-bit FIPS product of bn254.h spends one v_addc_co_u32 per
// v_mad_u64_u32 to catch the 64-bit column accumulator's carry-out.  With 29-bit limbs a
// 32x32->64 product is < 2^60 and one column (<= 9 a.b terms + <= 9 m.M terms) stays far
// below 2^64, so every product term is a lone v_mad_u64_u32 (no carry handling) and a
// column ends with one 64-bit shift: 162 mads + ~30 other ops against 128 mads + 128
// addcs + ~24 for the 32-bit form.
//
// Representation.  A value v is 9 limbs l[0..8], v = sum l[i] 2^(29 i); limbs 0..7 are
// kept < 2^29 ("normalised"); the top limb may hold a few more bits.  v represents the
// field element v * 2^-261 mod M.  The storage form used everywhere else (bn254.h:
// a * 2^256 mod M in 8 x 32-bit limbs, fully reduced) converts exactly by a shift: x * 32
// represents the same element here (x * 2^256 * 2^5 = x' * 2^261), so to29() is a
// repacking, not a product.  Values are not reduced: they carry multiples of M, bounded by
// the caller's data flow (see mul29's bound), and a zero test is a test modulo M.
#pragma once
#include "bn254.h"

namespace h2g {

static constexpr uint32_t F29_MASK = (1u << 29) - 1;

// 29-bit limb i of (x << sh) for a 256-bit constant x given as 8 LE 32-bit limbs
H2G_HD constexpr uint32_t limb29_of(const uint32_t* x, int i, int sh) {
  const int b = 29 * i - sh;  // bit offset in x
  if (b < 0) return (x[0] << (-b)) & F29_MASK;
  const int w = b >> 5, s = b & 31;
  const uint64_t lo = w < 8 ? x[w] : 0;
  const uint64_t hi = w + 1 < 8 ? x[w + 1] : 0;
  return (uint32_t)(((hi << 32) | lo) >> s) & F29_MASK;
}
template <class P>
struct C29 {
  static constexpr uint32_t M[9] = {limb29_of(P::M, 0, 0), limb29_of(P::M, 1, 0), limb29_of(P::M, 2, 0),
                                    limb29_of(P::M, 3, 0), limb29_of(P::M, 4, 0), limb29_of(P::M, 5, 0),
                                    limb29_of(P::M, 6, 0), limb29_of(P::M, 7, 0), limb29_of(P::M, 8, 0)};
  static constexpr uint32_t INV = P::INV & F29_MASK;  // -M^-1 mod 2^29
  // 2^256 mod M (= P::ONE) in 29-bit limbs: REDC(v * ONE) = v * 2^-5 mod M, the storage form
  static constexpr uint32_t ONE256[9] = {limb29_of(P::ONE, 0, 0), limb29_of(P::ONE, 1, 0), limb29_of(P::ONE, 2, 0),
                                         limb29_of(P::ONE, 3, 0), limb29_of(P::ONE, 4, 0), limb29_of(P::ONE, 5, 0),
                                         limb29_of(P::ONE, 6, 0), limb29_of(P::ONE, 7, 0), limb29_of(P::ONE, 8, 0)};
};

struct F29 {
  uint32_t l[9];
};

// ---- constants as 9-limb arrays (compile time)
struct Limbs9 {
  uint32_t v[9];
};
// k * M in normalised 29-bit limbs (k M < 2^264)
template <class P>
constexpr Limbs9 kmul_norm(uint32_t k) {
  Limbs9 r{};
  uint64_t c = 0;
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)limb29_of(P::M, i, 0) * k + c;
    r.v[i] = i < 8 ? (uint32_t)(t & F29_MASK) : (uint32_t)t;
    c = t >> 29;
  }
  return r;
}
// limb i of k * M in "borrow-safe" form: limbs 0..7 raised by 2^off (the top limb lowered to
// compensate), so that c - b never borrows in a limb for any b whose limbs 0..7 are below
// 2^off and whose top limb is below the top limb of the result (same value k M)
template <class P>
constexpr uint32_t kmul_safe(uint32_t k, int off, int i) {
  const Limbs9 n = kmul_norm<P>(k);
  const uint32_t unit = 1u << (off - 29);
  if (i == 0) return n.v[0] + (1u << off);
  if (i < 8) return n.v[i] + (1u << off) - unit;
  return n.v[8] - unit;
}
template <class P, uint32_t K, int OFF>
struct KM29 {
  static constexpr uint32_t L[9] = {kmul_safe<P>(K, OFF, 0), kmul_safe<P>(K, OFF, 1), kmul_safe<P>(K, OFF, 2),
                                    kmul_safe<P>(K, OFF, 3), kmul_safe<P>(K, OFF, 4), kmul_safe<P>(K, OFF, 5),
                                    kmul_safe<P>(K, OFF, 6), kmul_safe<P>(K, OFF, 7), kmul_safe<P>(K, OFF, 8)};
};
// 2^261 mod M (the element 1), reduced: 32 * (2^256 mod M) minus the multiple of M it holds
template <class P>
constexpr Limbs9 one29() {
  Limbs9 r{};
  for (int i = 0; i < 9; i++) r.v[i] = limb29_of(P::ONE, i, 5);
  for (int it = 0; it < 40; it++) {  // while r >= M: r -= M
    bool ge = true;
    for (int i = 8; i >= 0; i--) {
      const uint32_t m = limb29_of(P::M, i, 0);
      if (r.v[i] != m) {
        ge = r.v[i] > m;
        break;
      }
    }
    if (!ge) break;
    int64_t br = 0;
    for (int i = 0; i < 9; i++) {
      int64_t t = (int64_t)r.v[i] - limb29_of(P::M, i, 0) + br;
      br = t < 0 ? -1 : 0;
      r.v[i] = (uint32_t)(t & F29_MASK);
    }
  }
  return r;
}
template <class P>
struct One29 {
  static constexpr Limbs9 v = one29<P>();
  static constexpr uint32_t L[9] = {v.v[0], v.v[1], v.v[2], v.v[3], v.v[4], v.v[5], v.v[6], v.v[7], v.v[8]};
};

// storage (Montgomery 2^256, 8 x 32-bit limbs, value < 2^256) -> F29 of the same element:
// the integer x * 32 < 2^261, repacked into 29-bit limbs
template <class P>
H2G_HD F29 to29(const Fe<P>& x) {
  F29 r;
  r.l[0] = (x.l[0] << 5) & F29_MASK;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    const int b = 29 * i - 5, w = b >> 5, s = b & 31;
    const uint64_t lo = x.l[w];
    const uint64_t hi = w + 1 < 8 ? x.l[w + 1] : 0;
    r.l[i] = (uint32_t)(((hi << 32) | lo) >> s) & F29_MASK;
  }
  return r;
}

// Montgomery product REDC(a b) = a b 2^-261 mod M, as an unreduced value < a b / 2^261 + M.
// Column bound: with limbs of a and b < 2^30 (top limbs < 2^31) every column sum stays
// < 2^64, so inputs may be one unnormalised limb-wise add away from normalised values.
// Output limbs 0..7 normalised; the top limb is the rest (< 2^32 for outputs < 2^264).
#ifndef H2G_MUL29_SPLIT  // 1: the a b and m M terms of a column in two accumulators (NTT -4 %, MSM neutral)
#define H2G_MUL29_SPLIT 1
#endif
template <class P>
H2G_HD F29 mul29(const F29& a, const F29& b) {
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
  if constexpr (H2G_MUL29_SPLIT) {
    // two dependent chains per column instead of one (the column's a b terms and its m M
    // terms), joined before m_k and the carry -- half the chain depth, 17 more adds
#pragma unroll
    for (int k = 0; k < 9; k++) {
      uint64_t acc2 = 0;
#pragma unroll
      for (int i = 0; i <= k; i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
      for (int i = 0; i < k; i++) acc2 += (uint64_t)m[i] * C29<P>::M[k - i];
      acc += acc2;
      m[k] = ((uint32_t)acc * C29<P>::INV) & F29_MASK;
      acc += (uint64_t)m[k] * C29<P>::M[0];
      acc >>= 29;
    }
#pragma unroll
    for (int k = 9; k < 17; k++) {
      uint64_t acc2 = 0;
#pragma unroll
      for (int i = k - 8; i < 9; i++) {
        acc += (uint64_t)a.l[i] * b.l[k - i];
        acc2 += (uint64_t)m[i] * C29<P>::M[k - i];
      }
      acc += acc2;
      r.l[k - 9] = (uint32_t)acc & F29_MASK;
      acc >>= 29;
    }
    r.l[8] = (uint32_t)acc;
    return r;
  }
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * C29<P>::M[k - i];
    m[k] = ((uint32_t)acc * C29<P>::INV) & F29_MASK;
    acc += (uint64_t)m[k] * C29<P>::M[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; i < 9; i++) {
      acc += (uint64_t)a.l[i] * b.l[k - i];
      acc += (uint64_t)m[i] * C29<P>::M[k - i];
    }
    r.l[k - 9] = (uint32_t)acc & F29_MASK;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// REDC(a^2): the 36 cross products once, against the doubled limbs (2 a_i < 2^30 for a
// normalised a, so each term stays < 2^59), plus the 9 squares -- 45 + 81 mads instead of
// 81 + 81.  Same output bound as mul29(a, a).
template <class P>
H2G_HD F29 sqr29(const F29& a) {
  uint32_t m[9], d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.l[i] << 1;
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; i++) acc += (uint64_t)d[i] * a.l[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
    if (k < 9) {
#pragma unroll
      for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * C29<P>::M[k - i];
      m[k] = ((uint32_t)acc * C29<P>::INV) & F29_MASK;
      acc += (uint64_t)m[k] * C29<P>::M[0];
    } else {
#pragma unroll
      for (int i = k - 8; i < 9; i++) acc += (uint64_t)m[i] * C29<P>::M[k - i];
      r.l[k - 9] = (uint32_t)acc & F29_MASK;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// F29 -> storage form, fully reduced: REDC(v * (2^256 mod M)) = v 2^-5 mod M (< 2M for
// v < 2^261, i.e. a normalised top limb), one conditional subtraction, repacked into 32-bit limbs
template <class P>
H2G_HD Fe<P> from29(const F29& v) {
  F29 k;
#pragma unroll
  for (int i = 0; i < 9; i++) k.l[i] = C29<P>::ONE256[i];
  const F29 t = mul29<P>(v, k);
  Fe<P> r;
  uint64_t acc = 0;
  int have = 0, w = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)t.l[i] << have;
    have += 29;
    if (have >= 32 && w < 8) {
      r.l[w++] = (uint32_t)acc;
      acc >>= 32;
      have -= 32;
    }
  }
  if (w < 8) r.l[w] = (uint32_t)acc;
  return reduce_once(r);
}


// ---- limb-wise add / subtract, normalisation
H2G_HD F29 add29(const F29& a, const F29& b) {  // no carries: limbs grow by one bit
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + b.l[i];
  return r;
}
// a - b + K M, limb-wise without borrows (b's limbs 0..7 below 2^OFF, see kmul_safe); the
// result is unnormalised (limbs 0..7 below 2^(OFF+1) + 2^29)
template <class P, uint32_t K, int OFF>
H2G_HD F29 sub29(const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = (a.l[i] + KM29<P, K, OFF>::L[i]) - b.l[i];
  return r;
}
// carries of limbs 0..7 into the next limb (limbs are non-negative)
H2G_HD F29 norm29(F29 a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.l[i + 1] += a.l[i] >> 29;
    a.l[i] &= F29_MASK;
  }
  return a;
}

// REDC(a b + c d): two products under one Montgomery reduction (the m M terms are shared).
// Column bound: a, c normalised and b, d limbs below 1.5 * 2^30 keep every column < 2^64.
template <class P>
H2G_HD F29 mul29x2(const F29& a, const F29& b, const F29& c, const F29& d) {
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) {
      acc += (uint64_t)a.l[i] * b.l[k - i];
      acc += (uint64_t)c.l[i] * d.l[k - i];
    }
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * C29<P>::M[k - i];
    m[k] = ((uint32_t)acc * C29<P>::INV) & F29_MASK;
    acc += (uint64_t)m[k] * C29<P>::M[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; i < 9; i++) {
      acc += (uint64_t)a.l[i] * b.l[k - i];
      acc += (uint64_t)c.l[i] * d.l[k - i];
      acc += (uint64_t)m[i] * C29<P>::M[k - i];
    }
    r.l[k - 9] = (uint32_t)acc & F29_MASK;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// a == 0 mod M for a normalised a < 2^(29*8+32): a = k M with k < 2^29 has low limb
// k M_0 mod 2^29, so k = a_0 M^-1 mod 2^29 is the only candidate (a cheap filter; the exact
// comparison runs only when k is small enough to be real)
template <class P>
H2G_HD bool is_zero29(const F29& a) {
  constexpr uint32_t minv = (0u - C29<P>::INV) & F29_MASK;  // M^-1 mod 2^29
  const uint32_t k = (a.l[0] * minv) & F29_MASK;
  if (k > 1024) return false;
  uint64_t c = 0;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)C29<P>::M[i] * k + c;
    const uint32_t limb = i < 8 ? (uint32_t)(t & F29_MASK) : (uint32_t)t;
    c = t >> 29;
    diff |= limb ^ a.l[i];
  }
  return diff == 0;
}
template <class P>
H2G_HD F29 one29v() {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = One29<P>::L[i];
  return r;
}

// ---- G1 (XYZZ) over Fq in F29 limbs: the MSM bucket accumulation's arithmetic
// identity <=> ZZ is exactly zero (only ever created explicitly: a product of two nonzero
// elements is a nonzero element, hence never the integer 0)
struct G1xyzz29 {
  F29 X, Y, ZZ, ZZZ;
};
H2G_HD G1xyzz29 xyzz29_identity() {
  G1xyzz29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.X.l[i] = r.Y.l[i] = r.ZZ.l[i] = r.ZZZ.l[i] = 0;
  return r;
}
H2G_HD bool xyzz29_is_identity(const G1xyzz29& p) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) z |= p.ZZ.l[i];
  return z == 0;
}
// storage-form XYZZ (canonical 32-bit limbs) of a raw F29 accumulator
template <class P = FqParams>
H2G_HD G1xyzz xyzz_from29(const G1xyzz29& p) {
  G1xyzz r;
  r.X = from29<FqParams>(p.X);
  r.Y = from29<FqParams>(p.Y);
  r.ZZ = from29<FqParams>(p.ZZ);
  r.ZZZ = from29<FqParams>(p.ZZZ);
  return r;
}
// canonical storage form in; each coordinate reduced below 1.2 M (REDC(32 v * one))
template <class P>
H2G_HD F29 to29_reduced(const Fe<P>& v) {
  return mul29<P>(to29(v), one29v<P>());
}
H2G_HD G1xyzz29 xyzz29_from_xyzz(const G1xyzz& p) {
  G1xyzz29 r;
  r.X = to29_reduced(p.X);
  r.Y = to29_reduced(p.Y);
  r.ZZ = to29_reduced(p.ZZ);
  r.ZZZ = to29_reduced(p.ZZZ);
  return r;
}

// p + q for an affine q given as F29 coordinates of its canonical storage form (to29:
// values 32 x < 32 M), madd-2008-s.  Value bounds (tools/f29_bounds.py iterates this data
// flow from a fresh point to its fixpoint): every coordinate of p stays < 2^259.5, every
// intermediate < 2^259.9, so the subtraction constants below (64 M, 32 M, 64 M, 16 M)
// exceed what they subtract and every product's columns stay < 2^64.
// DBL = false drops the rare p == q branch (the doubling of q): *dbl is set instead and the
// result is meaningless.  The accumulation's hot loop uses that form -- the doubling's
// temporaries cost it 25 VGPRs, 3 waves per SIMD instead of 4 -- and redoes a chunk that
// hit the case with the full form (msm_acc_repair_kernel).
template <bool DBL = true>
H2G_HD G1xyzz29 xyzz29_madd(const G1xyzz29& p, const F29& qx, const F29& qy, bool* dbl = nullptr) {
  using P = FqParams;
  if (xyzz29_is_identity(p)) {
    G1xyzz29 r;
    r.X = qx;
    r.Y = qy;
    r.ZZ = one29v<P>();
    r.ZZZ = r.ZZ;
    return r;
  }
  const F29 U2 = mul29<P>(qx, p.ZZ);
  const F29 S2 = mul29<P>(qy, p.ZZZ);
  const F29 Pp = norm29(sub29<P, 64, 29>(U2, p.X));
  const F29 R = norm29(sub29<P, 64, 29>(S2, p.Y));
  if (is_zero29<P>(Pp)) {
    if (is_zero29<P>(R)) {  // p == q: double q (storage form, rare)
      if constexpr (DBL) {
        G1Affine a;
        a.x = from29<P>(qx);
        a.y = from29<P>(qy);
        return xyzz29_from_xyzz(xyzz_mdbl(a));
      } else {
        *dbl = true;
      }
    }
    return xyzz29_identity();  // p == -q
  }
  const F29 PP = sqr29<P>(Pp);
  const F29 PPP = mul29<P>(Pp, PP);
  const F29 Q = mul29<P>(p.X, PP);
  const F29 R2 = sqr29<P>(R);
  G1xyzz29 r;
  r.X = norm29(sub29<P, 32, 31>(R2, add29(add29(PPP, Q), Q)));  // R^2 - PPP - 2Q
  r.Y = mul29x2<P>(R, sub29<P, 64, 29>(Q, r.X), p.Y, sub29<P, 16, 29>(F29{}, PPP));  // R (Q - X3) - Y PPP
  r.ZZ = mul29<P>(p.ZZ, PP);
  r.ZZZ = mul29<P>(p.ZZZ, PPP);
  return r;
}


// ---- linear maps on storage-form data (the NTT): for a map that is linear over Fr, the
// storage integers x (x = e 2^256 mod M) can be taken as F29 values directly -- read as F29
// they stand for e 2^-5 -- and every constant (twiddle, coset power, scale) as a proper F29
// element (c 2^261 mod M).  Each product then carries the 2^-5 along, the outputs read as
// F29 stand for f 2^-5, i.e. they ARE the storage integers of the results f.  So data moves
// in and out by repacking 8 x 32 <-> 9 x 29 bits, with no conversion products.
template <class P>
H2G_HD F29 raw29(const Fe<P>& x) {  // the same integer in 29-bit limbs (x < 2^256)
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int b = 29 * i, w = b >> 5, s = b & 31;
    const uint64_t lo = x.l[w];
    const uint64_t hi = w + 1 < 8 ? x.l[w + 1] : 0;
    r.l[i] = (uint32_t)(((hi << 32) | lo) >> s) & F29_MASK;
  }
  return r;
}
template <class P>
H2G_HD Fe<P> pack29(const F29& v) {  // normalised v < 2^256 into 8 x 32-bit limbs
  Fe<P> r;
  uint64_t acc = 0;
  int have = 0, w = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)v.l[i] << have;
    have += 29;
    if (have >= 32 && w < 8) {
      r.l[w++] = (uint32_t)acc;
      acc >>= 32;
      have -= 32;
    }
  }
  if (w < 8) r.l[w] = (uint32_t)acc;
  return r;
}
// v - M if v >= M, for a normalised v (limbs 0..7 < 2^29): signed borrow chain, one select
template <class P>
H2G_HD F29 sub_m_if_ge29(const F29& v) {
  F29 d;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int32_t t = (int32_t)v.l[i] - (int32_t)C29<P>::M[i] + br;
    if (i < 8) {
      d.l[i] = (uint32_t)t & F29_MASK;
      br = t >> 29;
    } else {
      d.l[i] = (uint32_t)t;
      br = t >> 31;
    }
  }
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = br ? v.l[i] : d.l[i];
  return r;
}
// the F29 element of a storage-form constant, reduced to [0, M) and packed in 8 x 32 bits
// (twiddle tables: loaded with raw29, no product)
template <class P>
H2G_HD Fe<P> storage_to_f29_packed(const Fe<P>& s) {
  return pack29<P>(sub_m_if_ge29<P>(mul29<P>(to29(s), one29v<P>())));  // REDC(32 s one) < 1.2 M
}
template <class P>
H2G_HD F29 storage_to_f29(const Fe<P>& s) {
  return sub_m_if_ge29<P>(mul29<P>(to29(s), one29v<P>()));
}


// ---- the MSM back-end's XYZZ arithmetic (fixup, bucket reduction) in F29 ---------------
// The back-end works on a tighter class than the accumulation: every coordinate < 1.2 M.
// reduce29 brings the accumulation's values (< 2^259.5) into it once, and the full
// addition and the doubling reduce their one subtracted output (X3) the same way, so the
// subtraction constants stay small (2 M, 4 M) and no product's column comes near 2^64
// (tools/f29_bounds.py checks the class is closed under both).

// v - q M with q = floor(v_8 / (M_8 + 1)) (v normalised: limbs 0..7 < 2^29): the result is
// >= 0 and < M + (q + 2) 2^232 < 1.001 M -- the top limb's share of v removed, ~40 VALU ops
template <class P>
H2G_HD F29 reduce29(const F29& v) {
  constexpr uint32_t mt = C29<P>::M[8] + 1;
  const uint32_t q = v.l[8] / mt;
  F29 r;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int64_t t = (int64_t)v.l[i] - (int64_t)((uint64_t)q * C29<P>::M[i]) + br;
    if (i < 8) {
      r.l[i] = (uint32_t)t & F29_MASK;
      br = t >> 29;
    } else {
      r.l[i] = (uint32_t)t;
    }
  }
  return r;
}
H2G_HD G1xyzz29 xyzz29_reduce(const G1xyzz29& p) {
  G1xyzz29 r;
  r.X = reduce29<FqParams>(p.X);
  r.Y = reduce29<FqParams>(p.Y);
  r.ZZ = reduce29<FqParams>(p.ZZ);
  r.ZZZ = reduce29<FqParams>(p.ZZZ);
  return r;
}

// dbl-2008-s-1 on the back-end class
H2G_HD G1xyzz29 xyzz29_dbl(const G1xyzz29& p) {
  using P = FqParams;
  if (xyzz29_is_identity(p)) return p;
  const F29 U = norm29(add29(p.Y, p.Y));
  const F29 V = sqr29<P>(U);
  const F29 W = mul29<P>(U, V);
  const F29 S = mul29<P>(p.X, V);
  const F29 X2 = sqr29<P>(p.X);
  const F29 Mm = norm29(add29(add29(X2, X2), X2));
  G1xyzz29 r;
  r.X = reduce29<P>(norm29(sub29<P, 4, 31>(sqr29<P>(Mm), add29(S, S))));          // M^2 - 2S
  r.Y = mul29x2<P>(Mm, sub29<P, 4, 29>(S, r.X), p.Y, sub29<P, 2, 29>(F29{}, W));  // M (S - X3) - W Y
  r.ZZ = mul29<P>(V, p.ZZ);
  r.ZZZ = mul29<P>(W, p.ZZZ);
  return r;
}

// add-2008-s on the back-end class
H2G_HD G1xyzz29 xyzz29_add(const G1xyzz29& p, const G1xyzz29& q) {
  using P = FqParams;
  if (xyzz29_is_identity(q)) return p;
  if (xyzz29_is_identity(p)) return q;
  const F29 U1 = mul29<P>(p.X, q.ZZ);
  const F29 U2 = mul29<P>(q.X, p.ZZ);
  const F29 S1 = mul29<P>(p.Y, q.ZZZ);
  const F29 S2 = mul29<P>(q.Y, p.ZZZ);
  const F29 Pp = norm29(sub29<P, 2, 29>(U2, U1));
  const F29 R = norm29(sub29<P, 2, 29>(S2, S1));
  if (is_zero29<P>(Pp)) {
    if (is_zero29<P>(R)) return xyzz29_dbl(p);
    return xyzz29_identity();
  }
  const F29 PP = sqr29<P>(Pp);
  const F29 PPP = mul29<P>(Pp, PP);
  const F29 Q = mul29<P>(U1, PP);
  G1xyzz29 r;
  r.X = reduce29<P>(norm29(sub29<P, 4, 31>(sqr29<P>(R), add29(add29(PPP, Q), Q))));  // R^2 - PPP - 2Q
  r.Y = mul29x2<P>(R, sub29<P, 4, 29>(Q, r.X), S1, sub29<P, 2, 29>(F29{}, PPP));     // R (Q - X3) - S1 PPP
  r.ZZ = mul29<P>(mul29<P>(p.ZZ, q.ZZ), PP);
  r.ZZZ = mul29<P>(mul29<P>(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// [k] p for a small k (double-and-add, MSB first)
H2G_HD G1xyzz29 xyzz29_mul_u32(const G1xyzz29& p, uint32_t k) {
  if (k == 0) return xyzz29_identity();
  int top = 31;
  while (!((k >> top) & 1)) top--;
  G1xyzz29 acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = xyzz29_dbl(acc);
    if ((k >> b) & 1) acc = xyzz29_add(acc, p);
  }
  return acc;
}

}  // namespace h2g
