// bn254.h -- BN254 Fr/Fq Montgomery arithmetic and G1 group law for gfx950.
//
// 8 x 32-bit little-endian limbs, Montgomery form with R = 2^256: bit-for-bit
// the halo2curves 0.6 in-memory layout (4 x u64 LE limbs), so host slices of
// Fr / G1Affine are consumed and produced with no conversion pass.
// All values are kept fully reduced (< modulus); equality is limb equality.
//
// The same code compiles for the host (used only for O(1) glue such as
// combining per-GPU MSM partials and constants) and for the device.
//
// Limb arithmetic is written for the CDNA4 VALU: 32x32->64 products map onto
// v_mad_u64_u32, carry chains onto v_add_co_u32 / v_addc_co_u32.  No MFMA is
// involved (integer modular arithmetic, not a floating-point contraction).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H2G_HD __host__ __device__ __forceinline__

namespace h2g {

struct FrParams {
  static constexpr uint32_t M[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xefffffffu;  // -M^-1 mod 2^32
  static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                      0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr uint32_t R3[8] = {0xb4bf0040u, 0x5e94d8e1u, 0x1cfbb6b8u, 0x2a489cbeu,
                                     0xa19fcfedu, 0x893cc664u, 0x7fcc657cu, 0x0cf8594bu};
};
struct FqParams {
  static constexpr uint32_t M[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xe4866389u;
  static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                      0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
  static constexpr uint32_t R3[8] = {0xda1530dfu, 0xb1cd6dafu, 0xa7283db6u, 0x62f210e6u,
                                     0x0ada0afbu, 0xef7f0b0cu, 0x2d592544u, 0x20fd6e90u};
};

template <class P>
struct Fe {
  uint32_t l[8];

  H2G_HD static Fe zero() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = 0;
    return r;
  }
  H2G_HD static Fe one() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = P::ONE[i];
    return r;
  }
  H2G_HD bool is_zero() const {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= l[i];
    return x == 0;
  }
  H2G_HD bool operator==(const Fe& o) const {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= l[i] ^ o.l[i];
    return x == 0;
  }
  H2G_HD bool operator!=(const Fe& o) const { return !(*this == o); }
};

using Fr = Fe<FrParams>;
using Fq = Fe<FqParams>;

// ---------------------------------------------------------------- add / sub
// Carry chains through clang's __builtin_addc / __builtin_subc: on gfx950 each
// limb is one v_add_co/v_addc_co (v_sub_co/v_subb_co) and the reduction one
// v_cndmask -- 24 VALU ops per add or sub (a 64-bit signed emulation of the
// borrow compiled to ~5 ops per limb).
template <class P>
H2G_HD Fe<P> operator+(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> s, d;
  unsigned c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s.l[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
  // a + b < 2M < 2^255: no carry out; subtract M, keep if no borrow
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = __builtin_subc(s.l[i], P::M[i], br, &br);
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = br ? s.l[i] : d.l[i];
  return d;
}

template <class P>
H2G_HD Fe<P> operator-(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> d, s;
  unsigned br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
#pragma unroll
  for (int i = 0; i < 8; i++) s.l[i] = __builtin_addc(d.l[i], P::M[i], c, &c);
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = br ? s.l[i] : d.l[i];
  return d;
}

// r - M if r >= M (r < 2M)
template <class P>
H2G_HD Fe<P> reduce_once(const Fe<P>& r) {
  Fe<P> d;
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = __builtin_subc(r.l[i], P::M[i], br, &br);
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = br ? r.l[i] : d.l[i];
  return d;
}

template <class P>
H2G_HD Fe<P> neg(const Fe<P>& a) {
  return Fe<P>::zero() - a;
}
template <class P>
H2G_HD Fe<P> dbl(const Fe<P>& a) {
  return a + a;
}

// ---------------------------------------------------------------- Montgomery multiply
// Device: FIPS (finely integrated product scanning) Montgomery multiplication.
// A 96-bit column accumulator (lo64:hi32) takes every 32x32 product through one
// v_mad_u64_u32 whose carry-out (vcc) feeds one v_addc_co_u32: 128 mads + 128
// addcs + 8 mul_lo per product, no register shuffling (the compiler's own
// lowering of the CIOS loop spends ~2/3 of its instructions on v_mov/64-bit
// shifts: 86 vs 125 Gmodmul/s measured on MI355X, tools/microbench).
// One inline-asm block per product: hipcc pads each block boundary with an
// s_nop, but grouping a whole column per block measured
// slower (118 vs 125 Gmodmul/s) -- the compiler interleaves small blocks better.
// Not `volatile`: the scheduler may interleave the mac chains of independent
// products (a volatile asm statement is a scheduling barrier, which serialises
// e.g. the 4 independent butterflies of an NTT stage into one latency chain).
__device__ __forceinline__ void h2g_mac(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
               : "+v"(lo), "+v"(hi)
               : "v"(a), "v"(b)
               : "vcc");
}

// Montgomery product without the final conditional subtraction: for inputs
// a, b < 2M the result is < (4M^2 + 2^256 M) / 2^256 < 2M (both BN254 moduli are
// < 2^254, so 4M < 2^256).  Used by the "lazy" [0, 2M) arithmetic below.
template <class P>
__device__ __forceinline__ Fe<P> mont_mul_lazy(const Fe<P>& A, const Fe<P>& B) {
  const uint32_t* a = A.l;
  const uint32_t* b = B.l;
  uint32_t m[8];
  Fe<P> r;
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      h2g_mac(lo, hi, a[i], b[k - i]);
      h2g_mac(lo, hi, m[i], P::M[k - i]);
    }
    h2g_mac(lo, hi, a[k], b[0]);
    m[k] = (uint32_t)lo * P::INV;
    h2g_mac(lo, hi, m[k], P::M[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int i = k - 7; i < 8; i++) {
      h2g_mac(lo, hi, a[i], b[k - i]);
      h2g_mac(lo, hi, m[i], P::M[k - i]);
    }
    r.l[k - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r.l[7] = (uint32_t)lo;
  return r;
}

template <class P>
__device__ __forceinline__ Fe<P> operator*(const Fe<P>& A, const Fe<P>& B) {
  return reduce_once(mont_mul_lazy(A, B));  // fully reduced inputs: result < 2M
}
// Host: CIOS with the "no final carry" shortcut (top modulus limb < 2^63 - 1 for both
// BN254 moduli) over 64-bit limbs (~4x fewer multiplies than 32-bit limbs: the prover's
// host side -- commitment sums, SHPLONK's coefficients -- is latency-bound on these).
// Returns a*b*2^-256 mod M, fully reduced.
template <class P>
__host__ constexpr uint64_t host_inv64() {  // -M^-1 mod 2^64 from P::INV = -M^-1 mod 2^32
  const uint64_t m0 = (uint64_t)P::M[0] | (uint64_t)P::M[1] << 32;
  uint64_t x = (uint64_t)(0u - P::INV);  // M^-1 mod 2^32
  x = x * (2 - m0 * x);                  // Newton: M^-1 mod 2^64
  return 0 - x;
}
template <class P>
__host__ inline Fe<P> operator*(const Fe<P>& a, const Fe<P>& b) {
  using u128 = unsigned __int128;
  constexpr uint64_t inv = host_inv64<P>();
  uint64_t A[4], B[4], M[4], t[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    A[i] = (uint64_t)a.l[2 * i] | (uint64_t)a.l[2 * i + 1] << 32;
    B[i] = (uint64_t)b.l[2 * i] | (uint64_t)b.l[2 * i + 1] << 32;
    M[i] = (uint64_t)P::M[2 * i] | (uint64_t)P::M[2 * i + 1] << 32;
  }
  for (int i = 0; i < 4; i++) {
    u128 x = (u128)A[0] * B[i] + t[0];
    uint64_t hi = (uint64_t)(x >> 64);
    const uint64_t t0 = (uint64_t)x;
    const uint64_t m = t0 * inv;
    u128 y = (u128)m * M[0] + t0;
    uint64_t c = (uint64_t)(y >> 64);
    for (int j = 1; j < 4; j++) {
      x = (u128)A[j] * B[i] + t[j] + hi;
      hi = (uint64_t)(x >> 64);
      y = (u128)m * M[j] + (uint64_t)x + c;
      c = (uint64_t)(y >> 64);
      t[j - 1] = (uint64_t)y;
    }
    t[3] = c + hi;
  }
  Fe<P> r;
  for (int i = 0; i < 4; i++) {
    r.l[2 * i] = (uint32_t)t[i];
    r.l[2 * i + 1] = (uint32_t)(t[i] >> 32);
  }
  return reduce_once(r);
}

template <class P>
H2G_HD Fe<P> sqr(const Fe<P>& a) {
  return a * a;
}

// Montgomery -> canonical integer (little-endian limbs): a * 1 * 2^-256.
template <class P>
H2G_HD Fe<P> to_canonical(const Fe<P>& a) {
  Fe<P> one = Fe<P>::zero();
  one.l[0] = 1;
  return a * one;
}
template <class P>
H2G_HD Fe<P> from_canonical(const Fe<P>& a) {
  Fe<P> r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.l[i] = P::R2[i];
  return a * r2;
}
template <class P>
H2G_HD Fe<P> from_u64(uint64_t v) {
  Fe<P> c = Fe<P>::zero();
  c.l[0] = (uint32_t)v;
  c.l[1] = (uint32_t)(v >> 32);
  return from_canonical(c);
}

// a^e, e given as 8 little-endian 32-bit limbs (vartime in e; e is public).
template <class P>
H2G_HD Fe<P> pow_limbs(const Fe<P>& a, const uint32_t e[8]) {
  Fe<P> acc = Fe<P>::one();
  for (int i = 7; i >= 0; i--)
    for (int b = 31; b >= 0; b--) {
      acc = sqr(acc);
      if ((e[i] >> b) & 1) acc = acc * a;
    }
  return acc;
}
template <class P>
H2G_HD Fe<P> pow_u64(const Fe<P>& a, uint64_t e) {
  // from the top set bit of e: the skipped steps only square one (products are fully
  // reduced, so the result's bits do not change) -- a serial chain of log2(e) steps, not 64
  Fe<P> acc = Fe<P>::one();
  if (e == 0) return acc;
  for (int b = 63 - __builtin_clzll(e); b >= 0; b--) {
    acc = sqr(acc);
    if ((e >> b) & 1) acc = acc * a;
  }
  return acc;
}
// Fermat inversion a^(M-2); inv_fermat(0) = 0.
template <class P>
H2G_HD Fe<P> inv_fermat(const Fe<P>& a) {
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = P::M[i];
  e[0] -= 2;
  return pow_limbs(a, e);
}

// Inversion by the binary extended Euclidean algorithm; inv(0) = 0 (matches ff's
// invert().unwrap_or(ZERO) use in batch_invert).  Variable time -- nothing the prover
// inverts is secret from the device.  ~500 halvings and ~350 subtractions of 8-limb
// integers (add/sub/shift only, no multiplies): on a lone wave its dependent chain is
// ~4x shorter than Fermat's 380 Montgomery products, which is what bounds a batch
// inversion (one inversion per thread at the end of a serial prefix product).
// The Montgomery limbs x = aR are inverted as an integer, y = (aR)^-1, and one
// Montgomery product by R^3 gives a^-1 R.
template <class P>
H2G_HD void bgcd_half_mod(uint32_t x[8]) {  // x / 2 mod M, x < M
  uint32_t s[8];
  unsigned c = 0;
  const uint32_t odd = 0u - (x[0] & 1u);
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = __builtin_addc(x[i], P::M[i] & odd, c, &c);  // < 2^255
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = (s[i] >> 1) | (s[i + 1] << 31);
  x[7] = s[7] >> 1;
}
H2G_HD void bgcd_shr1(uint32_t u[8]) {
#pragma unroll
  for (int i = 0; i < 7; i++) u[i] = (u[i] >> 1) | (u[i + 1] << 31);
  u[7] >>= 1;
}
template <class P>
H2G_HD void bgcd_sub_mod(uint32_t x[8], const uint32_t y[8]) {  // x - y mod M
  unsigned br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = __builtin_subc(x[i], y[i], br, &br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = __builtin_addc(x[i], P::M[i] & mask, c, &c);
}
H2G_HD bool bgcd_is_one(const uint32_t u[8]) {
  uint32_t o = u[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 8; i++) o |= u[i];
  return o == 0;
}
template <class P>
H2G_HD Fe<P> inv(const Fe<P>& a) {
  if (a.is_zero()) return a;
  uint32_t u[8], v[8], x1[8], x2[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u[i] = a.l[i];
    v[i] = P::M[i];
    x1[i] = 0;
    x2[i] = 0;
  }
  x1[0] = 1;  // invariants: x1 * a = u, x2 * a = v (mod M)
  while (!bgcd_is_one(u) && !bgcd_is_one(v)) {
    while (!(u[0] & 1u)) {
      bgcd_shr1(u);
      bgcd_half_mod<P>(x1);
    }
    while (!(v[0] & 1u)) {
      bgcd_shr1(v);
      bgcd_half_mod<P>(x2);
    }
    uint32_t d[8];
    unsigned br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = __builtin_subc(u[i], v[i], br, &br);
    if (!br) {  // u >= v
#pragma unroll
      for (int i = 0; i < 8; i++) u[i] = d[i];
      bgcd_sub_mod<P>(x1, x2);
    } else {
      unsigned b2 = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = __builtin_subc(v[i], u[i], b2, &b2);
      bgcd_sub_mod<P>(x2, x1);
    }
  }
  Fe<P> y, r3;
  const bool uo = bgcd_is_one(u);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    y.l[i] = uo ? x1[i] : x2[i];
    r3.l[i] = P::R3[i];  // R^3 mod M
  }
  return y * r3;
}

// Inversion by Bernstein-Yang divsteps (the "safegcd" algorithm, "Fast constant-time gcd
// computation and modular inversion", 2019), in the signed 30-bit-limb form of its 32-bit
// formulation: 20 rounds of 30 branch-free divsteps on the low words give a 2x2 transition
// matrix, applied to (f, g) and to the Bezout pair (d, e) modulo M.  Every lane runs the
// same instructions -- the binary-GCD `inv` above diverges across a wave's lanes (each
// lane its own number of halvings and subtractions), which made one batch inversion's
// middle level ~250-400 us of one wave on gfx950; this is ~15 K uniform ops.  Same
// result as inv (a^-1 in Montgomery form; 0 -> 0).  600 divsteps >= the 590 that 256-bit
// inputs need.
struct By30 {
  int32_t v[9];
};
__device__ __forceinline__ By30 by30_from_limbs(const uint32_t x[8]) {
  By30 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int b = 30 * i, w = b >> 5, s = b & 31;
    uint64_t lo = x[w];
    if (w + 1 < 8) lo |= (uint64_t)x[w + 1] << 32;
    r.v[i] = (int32_t)((lo >> s) & (i < 8 ? 0x3fffffffull : 0xffffffffull));
  }
  return r;
}
__device__ __forceinline__ void by30_to_limbs(const By30& a, uint32_t x[8]) {  // limbs in [0, 2^30), value < 2^256
  uint64_t acc = 0;
  int have = 0, w = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)(uint32_t)a.v[i] << have;
    have += 30;
    if (have >= 32 && w < 8) {
      x[w++] = (uint32_t)acc;
      acc >>= 32;
      have -= 32;
    }
  }
  if (w < 8) x[w] = (uint32_t)acc;
}
// 30 divsteps on the low words: returns the new zeta; t = (u, v, q, r) scaled by 2^30
__device__ __forceinline__ int32_t by30_divsteps(int32_t zeta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    uint32_t m1 = (uint32_t)(zeta >> 31);
    const uint32_t m2 = 0u - (g & 1u);
    const uint32_t x = (f ^ m1) - m1, y = (u ^ m1) - m1, z = (v ^ m1) - m1;
    g += x & m2;
    q += y & m2;
    r += z & m2;
    m1 &= m2;
    zeta = (zeta ^ (int32_t)m1) - 1;
    f += g & m1;
    u += q & m1;
    v += r & m1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return zeta;
}
template <class P>
__device__ __forceinline__ Fe<P> inv_by(const Fe<P>& a) {
  if (a.is_zero()) return a;
  constexpr int32_t M30 = 0x3fffffff;
  const By30 mod = by30_from_limbs(P::M);
  const uint32_t inv30 = (0u - P::INV) & (uint32_t)M30;  // M^-1 mod 2^30 (P::INV = -M^-1 mod 2^32)
  By30 d = {}, e = {}, f = mod, g = by30_from_limbs(a.l);
  e.v[0] = 1;
  int32_t zeta = -1;
  for (int it = 0; it < 20; it++) {
    int32_t t[4];
    zeta = by30_divsteps(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
    // (d, e) <- (t [d, e] + M [md, me]) / 2^30, md / me chosen so the low 30 bits vanish
    {
      const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
      int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
      int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
      int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
      md -= (int32_t)((inv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
      me -= (int32_t)((inv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
      cd += (int64_t)mod.v[0] * md;
      ce += (int64_t)mod.v[0] * me;
      cd >>= 30;
      ce >>= 30;
#pragma unroll
      for (int i = 1; i < 9; i++) {
        cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)mod.v[i] * md;
        ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)mod.v[i] * me;
        d.v[i - 1] = (int32_t)cd & M30;
        e.v[i - 1] = (int32_t)ce & M30;
        cd >>= 30;
        ce >>= 30;
      }
      d.v[8] = (int32_t)cd;
      e.v[8] = (int32_t)ce;
    }
    // (f, g) <- t [f, g] / 2^30
    {
      int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
      int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
      cf >>= 30;
      cg >>= 30;
#pragma unroll
      for (int i = 1; i < 9; i++) {
        cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
        cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
        f.v[i - 1] = (int32_t)cf & M30;
        g.v[i - 1] = (int32_t)cg & M30;
        cf >>= 30;
        cg >>= 30;
      }
      f.v[8] = (int32_t)cf;
      g.v[8] = (int32_t)cg;
    }
  }
  // f = +-1 now; d = +-a^-1 in (-2M, M): into [0, M) with f's sign
  const int32_t neg = f.v[8] >> 31;
  int32_t c = d.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) d.v[i] += mod.v[i] & c;
#pragma unroll
  for (int i = 0; i < 9; i++) d.v[i] = (d.v[i] ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= M30;
  }
  c = d.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) d.v[i] += mod.v[i] & c;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    d.v[i + 1] += d.v[i] >> 30;
    d.v[i] &= M30;
  }
  Fe<P> y, r3;
  by30_to_limbs(d, y.l);
#pragma unroll
  for (int i = 0; i < 8; i++) r3.l[i] = P::R3[i];  // (aR)^-1 R^3 R^-1 = a^-1 R
  return y * r3;
}

// ---------------------------------------------------------------- G1 (y^2 = x^3 + 3 over Fq)

struct G1Affine {  // halo2curves layout; identity = (0, 0)
  Fq x, y;
  H2G_HD bool is_identity() const { return x.is_zero() && y.is_zero(); }
};

// Extended Jacobian "XYZZ": x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2; identity: ZZ = 0.
struct G1xyzz {
  Fq X, Y, ZZ, ZZZ;
  H2G_HD static G1xyzz identity() {
    G1xyzz r;
    r.X = Fq::one();
    r.Y = Fq::one();
    r.ZZ = Fq::zero();
    r.ZZZ = Fq::zero();
    return r;
  }
  H2G_HD bool is_identity() const { return ZZ.is_zero(); }
  H2G_HD static G1xyzz from_affine(const G1Affine& a) {
    if (a.is_identity()) return identity();
    G1xyzz r;
    r.X = a.x;
    r.Y = a.y;
    r.ZZ = Fq::one();
    r.ZZZ = Fq::one();
    return r;
  }
};

// dbl-2008-s-1 (a = 0)
H2G_HD G1xyzz xyzz_dbl(const G1xyzz& p) {
  if (p.is_identity()) return p;
  const Fq U = dbl(p.Y);
  const Fq V = sqr(U);
  const Fq W = U * V;
  const Fq S = p.X * V;
  const Fq X2 = sqr(p.X);
  const Fq M = X2 + dbl(X2);
  G1xyzz r;
  r.X = sqr(M) - dbl(S);
  r.Y = M * (S - r.X) - W * p.Y;
  r.ZZ = V * p.ZZ;
  r.ZZZ = W * p.ZZZ;
  return r;
}

// mdbl-2008-s-1: double an affine point (not identity)
H2G_HD G1xyzz xyzz_mdbl(const G1Affine& a) {
  const Fq U = dbl(a.y);
  const Fq V = sqr(U);
  const Fq W = U * V;
  const Fq S = a.x * V;
  const Fq X2 = sqr(a.x);
  const Fq M = X2 + dbl(X2);
  G1xyzz r;
  r.X = sqr(M) - dbl(S);
  r.Y = M * (S - r.X) - W * a.y;
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// madd-2008-s: p + affine q
H2G_HD G1xyzz xyzz_madd(const G1xyzz& p, const G1Affine& q) {
  if (q.is_identity()) return p;
  if (p.is_identity()) return G1xyzz::from_affine(q);
  const Fq U2 = q.x * p.ZZ;
  const Fq S2 = q.y * p.ZZZ;
  const Fq Pp = U2 - p.X;
  const Fq R = S2 - p.Y;
  if (Pp.is_zero()) {
    if (R.is_zero()) return xyzz_mdbl(q);
    return G1xyzz::identity();
  }
  const Fq PP = sqr(Pp);
  const Fq PPP = Pp * PP;
  const Fq Q = p.X * PP;
  G1xyzz r;
  r.X = sqr(R) - PPP - dbl(Q);
  r.Y = R * (Q - r.X) - p.Y * PPP;
  r.ZZ = p.ZZ * PP;
  r.ZZZ = p.ZZZ * PPP;
  return r;
}

// add-2008-s: p + q
H2G_HD G1xyzz xyzz_add(const G1xyzz& p, const G1xyzz& q) {
  if (q.is_identity()) return p;
  if (p.is_identity()) return q;
  const Fq U1 = p.X * q.ZZ;
  const Fq U2 = q.X * p.ZZ;
  const Fq S1 = p.Y * q.ZZZ;
  const Fq S2 = q.Y * p.ZZZ;
  const Fq Pp = U2 - U1;
  const Fq R = S2 - S1;
  if (Pp.is_zero()) {
    if (R.is_zero()) return xyzz_dbl(p);
    return G1xyzz::identity();
  }
  const Fq PP = sqr(Pp);
  const Fq PPP = Pp * PP;
  const Fq Q = U1 * PP;
  G1xyzz r;
  r.X = sqr(R) - PPP - dbl(Q);
  r.Y = R * (Q - r.X) - S1 * PPP;
  r.ZZ = p.ZZ * q.ZZ * PP;
  r.ZZZ = p.ZZZ * q.ZZZ * PPP;
  return r;
}

H2G_HD G1xyzz xyzz_neg(const G1xyzz& p) {
  G1xyzz r = p;
  r.Y = neg(p.Y);
  return r;
}

H2G_HD G1Affine affine_neg(const G1Affine& a) {
  G1Affine r = a;
  if (!a.is_identity()) r.y = neg(a.y);
  return r;
}

H2G_HD G1Affine xyzz_to_affine(const G1xyzz& p) {
  G1Affine r;
  if (p.is_identity()) {
    r.x = Fq::zero();
    r.y = Fq::zero();
    return r;
  }
  const Fq i = inv(p.ZZ * p.ZZZ);  // 1/(ZZ*ZZZ)
  const Fq izz = i * p.ZZZ;        // 1/ZZ
  const Fq izzz = i * p.ZZ;        // 1/ZZZ
  r.x = p.X * izz;
  r.y = p.Y * izzz;
  return r;
}
// host: m points at once with one inversion (Montgomery's trick over the ZZ * ZZZ
// products; a host inversion costs ~80 host products), for a stage's commitments
inline void xyzz_to_affine_batch(const G1xyzz* p, G1Affine* out, int m) {
  Fq* pre = new Fq[m > 0 ? m : 1];
  Fq acc = Fq::one();
  for (int i = 0; i < m; i++) {
    pre[i] = acc;
    if (!p[i].is_identity()) acc = acc * (p[i].ZZ * p[i].ZZZ);
  }
  Fq ia = inv(acc);  // 1 / prod of the non-identity points' ZZ ZZZ
  for (int i = m - 1; i >= 0; i--) {
    if (p[i].is_identity()) {
      out[i].x = Fq::zero();
      out[i].y = Fq::zero();
      continue;
    }
    const Fq d = p[i].ZZ * p[i].ZZZ;
    const Fq id = ia * pre[i];  // 1 / (ZZ ZZZ) of point i
    ia = ia * d;
    out[i].x = p[i].X * (id * p[i].ZZZ);
    out[i].y = p[i].Y * (id * p[i].ZZ);
  }
  delete[] pre;
}
// the same with the wave-uniform divsteps inversion (kernels converting many points:
// fixed-base tables, SRS, prefix bases)
__device__ __forceinline__ G1Affine xyzz_to_affine_by(const G1xyzz& p) {
  G1Affine r;
  if (p.is_identity()) {
    r.x = Fq::zero();
    r.y = Fq::zero();
    return r;
  }
  const Fq i = inv_by(p.ZZ * p.ZZZ);
  r.x = p.X * (i * p.ZZZ);
  r.y = p.Y * (i * p.ZZ);
  return r;
}

// ---------------------------------------------------------------- lazy [0, 2M) arithmetic (device)
// For long chains of group additions that never leave the device (the MSM bucket
// accumulation): values live in [0, 2M), so a Montgomery product skips its final
// conditional subtraction (mont_mul_lazy); add/sub reduce modulo 2M; zero tests
// accept both representatives 0 and M.  canon2 maps back to [0, M) before a value
// is stored for code that assumes fully reduced limbs.
template <class P>
__device__ __forceinline__ uint32_t two_m_limb(int i) {
  return (P::M[i] << 1) | (i ? P::M[i - 1] >> 31 : 0u);
}
template <class P>
__device__ __forceinline__ Fe<P> add2(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> s, d;
  unsigned c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s.l[i] = __builtin_addc(a.l[i], b.l[i], c, &c);  // < 4M < 2^256
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = __builtin_subc(s.l[i], two_m_limb<P>(i), br, &br);
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = br ? s.l[i] : d.l[i];
  return d;
}
template <class P>
__device__ __forceinline__ Fe<P> sub2(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> d, s;
  unsigned br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
  // a - b in (-2M, 2M): add 2M back on borrow (mod 2^256)
#pragma unroll
  for (int i = 0; i < 8; i++) s.l[i] = __builtin_addc(d.l[i], two_m_limb<P>(i), c, &c);
#pragma unroll
  for (int i = 0; i < 8; i++) d.l[i] = br ? s.l[i] : d.l[i];
  return d;
}
template <class P>
__device__ __forceinline__ bool is_zero2(const Fe<P>& a) {
  uint32_t z = 0, m = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    z |= a.l[i];
    m |= a.l[i] ^ P::M[i];
  }
  return z == 0 || m == 0;
}
template <class P>
__device__ __forceinline__ Fe<P> canon2(const Fe<P>& a) {
  return reduce_once(a);
}
__device__ __forceinline__ G1xyzz xyzz_canon2(const G1xyzz& p) {
  G1xyzz r;
  r.X = canon2(p.X);
  r.Y = canon2(p.Y);
  r.ZZ = canon2(p.ZZ);
  r.ZZZ = canon2(p.ZZZ);
  return r;
}
// madd-2008-s on [0, 2M) coordinates (p lazy or the identity, q canonical affine);
// the same formula and special cases as xyzz_madd.
__device__ __forceinline__ G1xyzz xyzz_madd_lazy(const G1xyzz& p, const G1Affine& q) {
  if (q.is_identity()) return p;
  if (is_zero2(p.ZZ)) return G1xyzz::from_affine(q);
  const Fq U2 = mont_mul_lazy(q.x, p.ZZ);
  const Fq S2 = mont_mul_lazy(q.y, p.ZZZ);
  const Fq Pp = sub2(U2, p.X);
  const Fq R = sub2(S2, p.Y);
  if (is_zero2(Pp)) {
    if (is_zero2(R)) return xyzz_mdbl(q);
    return G1xyzz::identity();
  }
  const Fq PP = mont_mul_lazy(Pp, Pp);
  const Fq PPP = mont_mul_lazy(Pp, PP);
  const Fq Q = mont_mul_lazy(p.X, PP);
  G1xyzz r;
  r.X = sub2(sub2(mont_mul_lazy(R, R), PPP), add2(Q, Q));
  r.Y = sub2(mont_mul_lazy(R, sub2(Q, r.X)), mont_mul_lazy(p.Y, PPP));
  r.ZZ = mont_mul_lazy(p.ZZ, PP);
  r.ZZZ = mont_mul_lazy(p.ZZZ, PPP);
  return r;
}

// [k] P for a small unsigned k (double-and-add, MSB first)
H2G_HD G1xyzz xyzz_mul_u32(const G1xyzz& p, uint32_t k) {
  if (k == 0) return G1xyzz::identity();
  int top = 31;
  while (!((k >> top) & 1)) top--;
  G1xyzz acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = xyzz_dbl(acc);
    if ((k >> b) & 1) acc = xyzz_add(acc, p);
  }
  return acc;
}

// [s] P for a full canonical scalar s (8 LE limbs)
H2G_HD G1xyzz xyzz_mul_canonical(const G1xyzz& p, const uint32_t s[8]) {
  G1xyzz acc = G1xyzz::identity();
  for (int i = 7; i >= 0; i--)
    for (int b = 31; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      if ((s[i] >> b) & 1) acc = xyzz_add(acc, p);
    }
  return acc;
}

}  // namespace h2g
