// ntt.hip -- register-resident radix-2^m NTT over BN254 Fr for gfx950.
//
// Computes exactly what halo2curves' best_fft computes (natural order in,
// natural order out, y_k = sum_i a_i w^(ik)), as called by
// EvaluationDomain (halo2_backend/src/poly/domain.rs:220, 238, 275, 344),
// plus the fused pre/post maps of coeff_to_extended / extended_to_coeff /
// lagrange_to_coeff (domain.rs:216-293).
//
// Decomposition: N = N_0 * N_1 * ... * N_{P-1}, every N_p = 2^m_p with
// 3 <= m_p <= 6 and the last pass 2^6.  With i = i_low + (L_p/N_p) i_p, pass p
// runs the size-N_p DFT over i_p, then multiplies by w^{(N/L_p) i_low k_p}, in
// place; the last pass reads contiguous runs and writes natural order (digit
// reversal folded into its store).  Each pass touches HBM once (64 B/element).
//
// One wavefront owns CPW = 64 / 2^(m-3) adjacent columns; every lane holds 8
// elements of one column in registers.  A 2^m-point DIF = one in-register
// radix-8 round on the top 3 index bits, (m-3) lane<->register bit swaps by
// __shfl_xor (no LDS staging, no barriers), and a second in-register round on
// the low m-3 bits.  Global accesses are runs of >= 8 x 32 B across the lanes
// of one instruction.  Inter-pass twiddles come from a 2-level table
// w^E = lo[E mod 2^b] * hi[E >> b] (both L2-resident).
#include <algorithm>
#include <type_traits>

#include "ntt.h"
#include "f29.h"

namespace h2g {

static constexpr int NTT_WAVES = 4;  // waves per block (independent; no block barriers after the table)
static constexpr int NTT_THREADS = 64 * NTT_WAVES;
#ifndef NTT_MIN_WAVES
#define NTT_MIN_WAVES 2  // waves per SIMD the register allocation must admit
#endif
// 2^6 passes fit 168 VGPRs without spilling -> 3 waves per SIMD (512 / 168);
// the smaller passes would spill at 168 and stay at 2.
template <int M>
struct NttPassWaves {
  static constexpr int value = M == 6 ? 3 : NTT_MIN_WAVES;
};

__device__ __forceinline__ Fr ld_fr(const Fr* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  Fr r;
  r.l[0] = a.x; r.l[1] = a.y; r.l[2] = a.z; r.l[3] = a.w;
  r.l[4] = b.x; r.l[5] = b.y; r.l[6] = b.z; r.l[7] = b.w;
  return r;
}
__device__ __forceinline__ void st_fr(Fr* p, const Fr& v) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
  q[1] = make_uint4(v.l[4], v.l[5], v.l[6], v.l[7]);
}

__device__ __forceinline__ Fr twiddle(const NttTables& t, uint64_t e) {
  return t.lo[e & ((1ull << t.b) - 1)] * t.hi[e >> t.b];
}

__device__ __forceinline__ Fr shfl_xor_fr(const Fr& v, int mask) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (uint32_t)__shfl_xor((int)v.l[i], mask);
  return r;
}

__device__ __forceinline__ Fr fr_select(int c, const Fr& a, const Fr& b) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// y mod 3 for 64-bit y with 32-bit arithmetic (2^32 = 1 mod 3)
__device__ __forceinline__ uint32_t mod3(uint64_t y) {
  return ((uint32_t)(y >> 32) % 3u + (uint32_t)y % 3u) % 3u;
}

__device__ __forceinline__ uint32_t brev_bits(uint32_t x, int m) { return __brev(x) >> (32 - m); }

// Butterfly arithmetic on lazily reduced values (bn254.h's [0, 2M) arithmetic): the
// passes keep their data in [0, 2M) -- sums reduce modulo 2M, a difference headed for a
// product is a - b + 2M in (0, 4M) without any select, and the products skip their final
// subtraction (an input < 4M times a twiddle < M gives < 2M); only the last pass's stores
// reduce to [0, M).  ~24 VALU ops fewer per multiplied butterfly.
#ifndef H2G_NTT_LAZY  // A/B builds: 0 = fully reduced butterflies
#define H2G_NTT_LAZY 1
#endif
__device__ __forceinline__ Fr bf_add(const Fr& a, const Fr& b) {
  if constexpr (H2G_NTT_LAZY) return add2(a, b);
  else return a + b;
}
__device__ __forceinline__ Fr bf_sub(const Fr& a, const Fr& b) {  // a difference kept as is
  if constexpr (H2G_NTT_LAZY) return sub2(a, b);
  else return a - b;
}
__device__ __forceinline__ Fr bf_sub_mul(const Fr& a, const Fr& b, const Fr& w) {  // (a - b) w
  if constexpr (H2G_NTT_LAZY) {
    Fr d;
    unsigned br = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d.l[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; i++) d.l[i] = __builtin_addc(d.l[i], two_m_limb<FrParams>(i), c, &c);  // (0, 4M)
    return mont_mul_lazy(d, w);
  } else {
    return (a - b) * w;
  }
}
__device__ __forceinline__ Fr bf_mul(const Fr& x, const Fr& w) {  // x < 2M, w < M
  if constexpr (H2G_NTT_LAZY) return mont_mul_lazy(x, w);
  else return x * w;
}
__device__ __forceinline__ Fr bf_out(const Fr& x) {  // to [0, M) for the stored result
  if constexpr (H2G_NTT_LAZY) return reduce_once(x);
  else return x;
}

// In-register DIF of 2^M-point columns.  Lane = c + CPW * rg; register q of the
// lane initially holds row r = rg + LPC * q.  `w[j] = w_{2^M}^j`, j < 2^(M-1).
// After run(), register q holds DIF position rpos(q, rg) (output index
// k = bitrev_M(rpos)).
template <int M>
struct WaveDif {
  static constexpr int LPC = 1 << (M - 3);  // lanes per column
  static constexpr int CPW = 64 / LPC;      // columns per wave

  __device__ static __forceinline__ void run(Fr x[8], const Fr* w, int rg) {
    // round A: row bits M-1..M-3 live in the register index
#pragma unroll
    for (int t = 2; t >= 0; t--) {
      const int htlog = (M - 3) + t;
#pragma unroll
      for (int p = 0; p < 4; p++) {
        const int q = ((p >> t) << (t + 1)) | (p & ((1 << t) - 1));
        const int j = rg + (p & ((1 << t) - 1)) * LPC;
        const Fr a = x[q], b = x[q + (1 << t)];
        x[q] = bf_add(a, b);
        x[q + (1 << t)] = bf_sub_mul(a, b, w[j << (M - 1 - htlog)]);
      }
    }
    // swap register bit b <-> lane bit b (lane index bit log2(CPW) + b), b < M-3
#pragma unroll
    for (int b = 0; b < M - 3; b++) {
      const int lb = (rg >> b) & 1;
#pragma unroll
      for (int p = 0; p < 4; p++) {
        const int q = ((p >> b) << (b + 1)) | (p & ((1 << b) - 1));
        // value selects only (a data-dependent register index would spill x[] to scratch)
        const Fr lo_v = x[q], hi_v = x[q | (1 << b)];
        const Fr recv = shfl_xor_fr(fr_select(lb, lo_v, hi_v), CPW << b);
        x[q] = fr_select(lb, recv, lo_v);
        x[q | (1 << b)] = fr_select(lb, hi_v, recv);
      }
    }
    // round B: row bits M-4..0 now live in register bits M-4..0
#pragma unroll
    for (int t = M - 4; t >= 0; t--) {
#pragma unroll
      for (int p = 0; p < 4; p++) {
        const int q = ((p >> t) << (t + 1)) | (p & ((1 << t) - 1));
        const int j = q & ((1 << t) - 1);  // compile-time after unrolling
        const Fr a = x[q], b = x[q + (1 << t)];
        x[q] = bf_add(a, b);
        // w^0 = 1 exactly (Montgomery one, fully reduced): skip the product --
        // every butterfly of the t = 0 stage, half of t = 1, a quarter of t = 2
        x[q + (1 << t)] = j == 0 ? bf_sub(a, b) : bf_sub_mul(a, b, w[j << (M - 1 - t)]);
      }
    }
  }

  // DIF position held by register q of lane rg after run()
  __device__ static __forceinline__ uint32_t rpos(int q, int rg) {
    constexpr int LB = M - 3;
    const uint32_t lowmask = (1u << LB) - 1;
    const uint32_t lo = (uint32_t)q & lowmask;                              // row bits < LB
    const uint32_t mid = (uint32_t)rg & lowmask;                            // row bits LB..2LB-1
    const uint32_t hi = ((uint32_t)q >> LB) << LB;                          // untouched register bits
    return lo + ((mid | hi) << LB);
  }
};

// ---------------------------------------------------------------------------
// Generic (non-last) pass, 2^M-point sub-transforms, in place on `data`.
//   L_p = 2^lrem (remaining length including this pass), S = L_p / 2^M.
//   Pass 0 reads `in` (n_in valid elements, zero padding beyond) and, if
//   `distribute`, multiplies element i by zeta^(i mod 3) (domain.rs:325-341).
template <int M>
__global__ void __launch_bounds__(NTT_THREADS, NttPassWaves<M>::value)
ntt_pass_kernel(Fr* data, NttIo io, int first, uint64_t n_in, NttTables tab, const Fr* __restrict__ ptw, int L,
                int lrem, int distribute, Fr z1, Fr z2) {
  using D = WaveDif<M>;
  data += (uint64_t)blockIdx.y << L;  // transform blockIdx.y of a batch
  const Fr* in = first ? io.src[blockIdx.y] : nullptr;
  __shared__ Fr w[1 << (M - 1)];
  for (int j = threadIdx.x; j < (1 << (M - 1)); j += blockDim.x) w[j] = twiddle(tab, (uint64_t)j << (L - M));
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * NTT_WAVES + (threadIdx.x >> 6);
  if (wave >= (1ull << L) / ((1ull << M) * D::CPW)) return;
  const uint64_t S = 1ull << (lrem - M);
  const uint64_t groups = S / D::CPW;
  const uint64_t q = wave / groups;
  const uint64_t g = wave % groups;
  const uint64_t base = (q << lrem) + g * D::CPW;
  const int c = lane % D::CPW, rg = lane / D::CPW;
  Fr x[8];
#pragma unroll
  for (int qq = 0; qq < 8; qq++) {
    const uint64_t pos = base + c + (uint64_t)(rg + D::LPC * qq) * S;
    if (in) {
      if (pos < n_in) {
        Fr v = ld_fr(in + pos);
        if (distribute) {
          const uint32_t md = mod3(pos);
          v = v * fr_select(md == 1, z1, fr_select(md == 2, z2, Fr::one()));
        }
        x[qq] = v;
      } else {
        x[qq] = Fr::zero();
      }
    } else {
      x[qq] = ld_fr(data + pos);
    }
  }
  D::run(x, w, rg);
  const uint64_t ilow = g * D::CPW + c;
#pragma unroll
  for (int qq = 0; qq < 8; qq++) {
    const uint32_t k = brev_bits(D::rpos(qq, rg), M);
    // w^((N / L_p) i_low k) from the precomputed pass table (one load instead of a
    // table product + multiplication)
    const Fr v = bf_mul(x[qq], ld_fr(ptw + (uint64_t)k * S + ilow));
    st_fr(data + base + c + (uint64_t)k * S, v);
  }
}

// ---------------------------------------------------------------------------
// Last pass (2^6-point columns): contiguous runs, output in natural order.
//   pos = k_0 (N/N_0) + m_idx 2^6 + i ;  y = k_0 + mid_nat(m_idx) + (N/2^6) k
//   Epilogue: multiply by `scale` and, if `distribute`, by the zeta power of
//   y mod 3; drop y >= out_len (truncation, domain.rs:288-290).
__global__ void __launch_bounds__(NTT_THREADS, NTT_MIN_WAVES)
ntt_last_kernel(const Fr* data, NttIo io, uint64_t out_len, NttTables tab, int L, NttPlanLg plan, int has_mul,
                Fr mul0, Fr mul1, Fr mul2) {
  constexpr int M = 6;
  data += (uint64_t)blockIdx.y << L;
  Fr* out = io.dst[blockIdx.y];
  using D = WaveDif<M>;
  __shared__ Fr w[1 << (M - 1)];
  for (int j = threadIdx.x; j < (1 << (M - 1)); j += blockDim.x) w[j] = twiddle(tab, (uint64_t)j << (L - M));
  __syncthreads();
  const int* lgs = plan.lg;
  const int P = plan.p;
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * NTT_WAVES + (threadIdx.x >> 6);
  if (wave >= (1ull << L) / ((1ull << M) * D::CPW)) return;
  const int l0 = lgs[0];
  const uint64_t groups = (1ull << l0) / D::CPW;
  const uint64_t midx = wave / groups;
  const uint64_t g = wave % groups;
  // m_idx = k_1 (N_2..N_{P-2}) + ... + k_{P-2}  ->  natural weight of k_p is N_0..N_{p-1}
  uint64_t mid_nat = 0;
  {
    uint64_t rem = midx;
    int wbits_tail = L - M;  // bits of k_0..k_{P-2}
#pragma unroll
    for (int p = NTT_MAX_PASSES - 2; p >= 1; p--) {  // constant indices into plan.lg (no scratch copy)
      if (p > P - 2) continue;
      const int lgp = lgs[p];
      const uint64_t dig = rem & ((1ull << lgp) - 1);
      rem >>= lgp;
      wbits_tail -= lgp;
      mid_nat |= dig << wbits_tail;
    }
  }
  const int c = lane % D::CPW, rg = lane / D::CPW;
  const uint64_t k0 = g * D::CPW + c;
  const uint64_t colbase = k0 * (1ull << (L - l0)) + (midx << M);
  Fr x[8];
#pragma unroll
  for (int qq = 0; qq < 8; qq++) x[qq] = ld_fr(data + colbase + rg + D::LPC * qq);
  D::run(x, w, rg);
  const uint64_t kstride = 1ull << (L - M);
#pragma unroll
  for (int qq = 0; qq < 8; qq++) {
    const uint32_t k = brev_bits(D::rpos(qq, rg), M);
    const uint64_t y = k0 + mid_nat + (uint64_t)k * kstride;
    if (y >= out_len) continue;
    Fr v = x[qq];
    if (has_mul) {  // ifft divisor and/or zeta power, one product (host folds them)
      const uint32_t md = mod3(y);
      v = v * fr_select(md == 1, mul1, fr_select(md == 2, mul2, mul0));  // < 2M in, reduced out
    } else {
      v = bf_out(v);
    }
    st_fr(out + y, v);
  }
}

// ---------------------------------------------------------------------------
// The passes in 9 x 29-bit limbs (f29.h), H2G_NTT29.  The transform is linear, so the
// stored integers move in and out by repacking only (f29.h: raw29 / pack29) and the
// constants -- twiddles, coset powers, scales -- are F29 elements (the pass tables are
// built in that form, storage_to_f29_packed).  Products are f29.h's carry-free REDC.
// Value bounds (tools/f29_bounds.py, "ntt"): stored values < 3 M; stage s of a pass
// subtracts with K_s = 2^(s+2) M (>= the stage's input bound with a top-limb margin), so
// after 6 stages every value is < 254 M < 2^262 and the closing product (pass twiddle or
// epilogue constant, < M) brings it back below 2.6 M; the last pass reduces to [0, M).
#ifndef H2G_NTT29  // A/B builds: 0 = the 8 x 32-bit FIPS passes above
#define H2G_NTT29 1
#endif

__device__ __forceinline__ F29 ld29(const Fr* p) { return raw29(ld_fr(p)); }
__device__ __forceinline__ void st29(Fr* p, const F29& v) { st_fr(p, pack29<FrParams>(v)); }
__device__ __forceinline__ F29 shfl_xor29(const F29& v, int mask) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = (uint32_t)__shfl_xor((int)v.l[i], mask);
  return r;
}
__device__ __forceinline__ F29 sel29(int c, const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}
// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N) -- for loops over
// whole products, which `#pragma unroll` may leave rolled (x[] is then indexed at run time
// and moves to scratch)
template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// a - b + K_s M for stage s: K_s = 2^(s+2)
template <int S>
__device__ __forceinline__ F29 nsub29(const F29& a, const F29& b) {
  return sub29<FrParams, (4u << S), 29>(a, b);
}

// The same butterfly schedule as WaveDif<M>::run (lane / register layout, rpos), its
// stages as templates: unrolled loops over whole products were left rolled by the
// compiler, and a rolled stage loop indexes x[] at run time (x[] then lives in scratch).
template <int M>
struct WaveDif29 {
  static constexpr int LPC = 1 << (M - 3);
  static constexpr int CPW = 64 / LPC;
  template <int T>  // round A, row bit M-3+T (stage 2 - T)
  __device__ static __forceinline__ void stage_a(F29 x[8], const F29* w, int rg) {
    constexpr int htlog = (M - 3) + T;
#pragma unroll
    for (int p = 0; p < 4; p++) {
      const int q = ((p >> T) << (T + 1)) | (p & ((1 << T) - 1));
      const int j = rg + (p & ((1 << T) - 1)) * LPC;
      const F29 a = x[q], b = x[q + (1 << T)];
      x[q] = norm29(add29(a, b));
      x[q + (1 << T)] = mul29<FrParams>(nsub29<2 - T>(a, b), w[j << (M - 1 - htlog)]);
    }
    if constexpr (T > 0) stage_a<T - 1>(x, w, rg);
  }
  template <int B>  // register bit B <-> lane bit
  __device__ static __forceinline__ void swap_bits(F29 x[8], int rg) {
    if constexpr (B < M - 3) {
      const int lb = (rg >> B) & 1;
#pragma unroll
      for (int p = 0; p < 4; p++) {
        const int q = ((p >> B) << (B + 1)) | (p & ((1 << B) - 1));
        const F29 lo_v = x[q], hi_v = x[q | (1 << B)];
        const F29 recv = shfl_xor29(sel29(lb, lo_v, hi_v), CPW << B);
        x[q] = sel29(lb, recv, lo_v);
        x[q | (1 << B)] = sel29(lb, hi_v, recv);
      }
      swap_bits<B + 1>(x, rg);
    }
  }
  template <int T>  // round B, row bit T (stage 3 + M - 4 - T)
  __device__ static __forceinline__ void stage_b(F29 x[8], const F29* w) {
    if constexpr (T >= 0) {
      constexpr int S = 3 + (M - 4 - T);
#pragma unroll
      for (int p = 0; p < 4; p++) {
        const int q = ((p >> T) << (T + 1)) | (p & ((1 << T) - 1));
        const int j = q & ((1 << T) - 1);
        const F29 a = x[q], b = x[q + (1 << T)];
        x[q] = norm29(add29(a, b));
        x[q + (1 << T)] = j == 0 ? norm29(nsub29<S>(a, b)) : mul29<FrParams>(nsub29<S>(a, b), w[j << (M - 1 - T)]);
      }
      stage_b<T - 1>(x, w);
    }
  }
  __device__ static __forceinline__ void run(F29 x[8], const F29* w, int rg) {
    stage_a<2>(x, w, rg);
    swap_bits<0>(x, rg);
    stage_b<M - 4>(x, w);
  }
};

// the constants of one launch in F29 form (host-converted)
struct NttConst29 {
  F29 z1, z2;      // input coset powers (pass 0)
  F29 mul[3];      // epilogue multiplier per y mod 3 (last pass), one29 when none
};

// inter-pass twiddles formed in the pass from the two-level table (one product and two
// L2-resident loads per element) instead of streamed from pass_tw (32 B of HBM per element):
// 1 = the first pass only (its table is N entries), 2 = every non-last pass, 0 = none
#ifndef H2G_NTT_TW_LIVE
#define H2G_NTT_TW_LIVE 0
#endif

template <int M>
__global__ void __launch_bounds__(NTT_THREADS, NttPassWaves<M>::value)
ntt_pass29_kernel(Fr* data, NttIo io, int first, uint64_t n_in, NttTables tab, const Fr* __restrict__ ptw, int L,
                  int lrem, int distribute, NttConst29 k29) {
  using D = WaveDif29<M>;
  data += (uint64_t)blockIdx.y << L;
  const Fr* in = first ? io.src[blockIdx.y] : nullptr;
  __shared__ F29 w[1 << (M - 1)];
  for (int j = threadIdx.x; j < (1 << (M - 1)); j += blockDim.x) w[j] = ld29(tab.root64 + (j << (6 - M)));
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * NTT_WAVES + (threadIdx.x >> 6);
  if (wave >= (1ull << L) / ((1ull << M) * D::CPW)) return;
  const uint64_t S = 1ull << (lrem - M);
  const uint64_t groups = S / D::CPW;
  const uint64_t q = wave / groups;
  const uint64_t g = wave % groups;
  const uint64_t base = (q << lrem) + g * D::CPW;
  const int c = lane % D::CPW, rg = lane / D::CPW;
  F29 x[8];
  sfor<0, 8>([&](auto qc) {
    constexpr int qq = decltype(qc)::value;
    const uint64_t pos = base + c + (uint64_t)(rg + D::LPC * qq) * S;
    if (in) {
      F29 v;
#pragma unroll
      for (int i = 0; i < 9; i++) v.l[i] = 0;
      if (pos < n_in) {
        v = ld29(in + pos);
        if (distribute) {
          const uint32_t md = mod3(pos);
          if (md) v = mul29<FrParams>(v, sel29(md == 1, k29.z1, k29.z2));
        }
      }
      x[qq] = v;
    } else {
      x[qq] = ld29(data + pos);
    }
  });
  D::run(x, w, rg);
  const uint64_t ilow = g * D::CPW + c;
  const bool live = H2G_NTT_TW_LIVE == 2 || (H2G_NTT_TW_LIVE == 1 && first);
  sfor<0, 8>([&](auto qc) {
    constexpr int qq = decltype(qc)::value;
    const uint32_t k = brev_bits(WaveDif<M>::rpos(qq, rg), M);
    F29 tw;
    if (live) {  // w^((N / L_p) i_low k) = lo[e mod 2^b] hi[e >> b], < 1.01 M
      const uint64_t e = (ilow * k) << (L - lrem);
      tw = mul29<FrParams>(ld29(tab.lo29 + (e & ((1ull << tab.b) - 1))), ld29(tab.hi29 + (e >> tab.b)));
    } else {
      tw = ld29(ptw + (uint64_t)k * S + ilow);
    }
    st29(data + base + c + (uint64_t)k * S, mul29<FrParams>(x[qq], tw));
  });
}

// Persistent variant of ntt_pass29_kernel for the passes after the first (H2G_NTT_PIPE): a wave walks column groups
// item, item + stride, ... and loads the next group's elements before it transforms the
// current one, so a SIMD's VALU work is not held up by its waves' loads all arriving at
// once (one launch round of the plain kernel loads, then computes, then stores).
#ifndef H2G_NTT_PIPE
#define H2G_NTT_PIPE 1
#endif
template <int M>
__global__ void __launch_bounds__(NTT_THREADS, 2)
ntt_pass29p_kernel(Fr* data, NttTables tab, const Fr* __restrict__ ptw, int L, int lrem, uint64_t items) {
  using D = WaveDif29<M>;
  data += (uint64_t)blockIdx.y << L;
  __shared__ F29 w[1 << (M - 1)];
  for (int j = threadIdx.x; j < (1 << (M - 1)); j += blockDim.x) w[j] = ld29(tab.root64 + (j << (6 - M)));
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint64_t stride = (uint64_t)gridDim.x * NTT_WAVES;
  uint64_t item = (uint64_t)blockIdx.x * NTT_WAVES + (threadIdx.x >> 6);
  if (item >= items) return;
  const uint64_t S = 1ull << (lrem - M);
  const uint64_t groups = S / D::CPW;
  const int c = lane % D::CPW, rg = lane / D::CPW;
  Fr nx[8];
  auto fetch = [&](uint64_t it) {
    const uint64_t b = ((it / groups) << lrem) + (it % groups) * D::CPW;
    sfor<0, 8>([&](auto qc) {
      constexpr int qq = decltype(qc)::value;
      const uint64_t pos = b + c + (uint64_t)(rg + D::LPC * qq) * S;
      nx[qq] = ld_fr(data + pos);
    });
  };
  fetch(item);
  for (;;) {
    const uint64_t cur = item;
    const uint64_t base = ((cur / groups) << lrem) + (cur % groups) * D::CPW;
    F29 x[8];
    sfor<0, 8>([&](auto qc) {
      constexpr int qq = decltype(qc)::value;
      x[qq] = raw29(nx[qq]);
    });
    item += stride;
    const bool more = item < items;
    if (more) fetch(item);
    __builtin_amdgcn_sched_barrier(0);  // the prefetch issues before the transform, the twiddle loads after it
    D::run(x, w, rg);
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t ilow = (cur % groups) * D::CPW + c;
    sfor<0, 8>([&](auto qc) {
      constexpr int qq = decltype(qc)::value;
      const uint32_t k = brev_bits(WaveDif<M>::rpos(qq, rg), M);
      st29(data + base + c + (uint64_t)k * S, mul29<FrParams>(x[qq], ld29(ptw + (uint64_t)k * S + ilow)));
    });
    if (!more) break;
  }
}

// First pass of 2^3 points when at most the first two of every column's eight inputs are
// nonzero (n_in <= N / 4: a coset extension by 4 or more, coeff_to_extended of a degree-5
// circuit): y_k = x_0 + w_8^k x_1 (w_8^(k+4) = -w_8^k), two loads and three products per
// column instead of eight loads and the twelve products of the 8-point DIF.  One lane per
// column; outputs < 1.04 M.
#ifndef H2G_NTT_SPARSE
#define H2G_NTT_SPARSE 1
#endif
__global__ void __launch_bounds__(NTT_THREADS)
ntt_first_sparse29_kernel(Fr* data, NttIo io, uint64_t n_in, NttTables tab, const Fr* __restrict__ ptw, int L,
                          int distribute, NttConst29 k29) {
  data += (uint64_t)blockIdx.y << L;
  const Fr* in = io.src[blockIdx.y];
  const uint64_t S = 1ull << (L - 3);
  const uint64_t col = (uint64_t)blockIdx.x * NTT_THREADS + threadIdx.x;
  if (col >= S) return;
  F29 x[2];
  sfor<0, 2>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const uint64_t pos = col + (uint64_t)j * S;
    F29 v;
#pragma unroll
    for (int i = 0; i < 9; i++) v.l[i] = 0;
    if (pos < n_in) {
      v = ld29(in + pos);
      if (distribute) {
        const uint32_t md = mod3(pos);
        if (md) v = mul29<FrParams>(v, sel29(md == 1, k29.z1, k29.z2));
      }
    }
    x[j] = v;
  });
  F29 y[8];
  sfor<0, 4>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const F29 pj = j == 0 ? x[1] : mul29<FrParams>(x[1], ld29(tab.root64 + 8 * j));
    y[j] = norm29(add29(x[0], pj));
    y[j + 4] = sub29<FrParams, 4, 29>(x[0], pj);
  });
  sfor<0, 8>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    st29(data + col + (uint64_t)k * S, mul29<FrParams>(y[k], ld29(ptw + (uint64_t)k * S + col)));
  });
}

static int ntt_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                   hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

#ifndef NTT_LAST_WAVES  // waves per SIMD of the untruncated last pass (142 VGPRs: 3 without spilling)
#define NTT_LAST_WAVES 3
#endif
// TRUNC: out_len < N (extended_to_coeff's truncation) -- the stores are predicated per
// element; without it every element is stored and the epilogue has no branches
// ONE: the epilogue constant is one for every y (no scale left, no output distribution) --
// the values (< 256 M) are brought to [0, M) by reduce29 and one conditional subtraction
// instead of a product
template <bool TRUNC, bool ONE>
__global__ void __launch_bounds__(NTT_THREADS, TRUNC ? NTT_MIN_WAVES : NTT_LAST_WAVES)
ntt_last29_kernel(const Fr* data, NttIo io, uint64_t out_len, NttTables tab, int L, NttPlanLg plan,
                  NttConst29 k29) {
  constexpr int M = 6;
  data += (uint64_t)blockIdx.y << L;
  Fr* out = io.dst[blockIdx.y];
  using D = WaveDif29<M>;
  __shared__ F29 w[1 << (M - 1)];
  for (int j = threadIdx.x; j < (1 << (M - 1)); j += blockDim.x) w[j] = ld29(tab.root64 + (j << (6 - M)));
  __syncthreads();
  const int* lgs = plan.lg;
  const int P = plan.p;
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * NTT_WAVES + (threadIdx.x >> 6);
  if (wave >= (1ull << L) / ((1ull << M) * D::CPW)) return;
  const int l0 = lgs[0];
  const uint64_t groups = (1ull << l0) / D::CPW;
  const uint64_t midx = wave / groups;
  const uint64_t g = wave % groups;
  uint64_t mid_nat = 0;
  {
    uint64_t rem = midx;
    int wbits_tail = L - M;
#pragma unroll
    for (int p = NTT_MAX_PASSES - 2; p >= 1; p--) {
      if (p > P - 2) continue;
      const int lgp = lgs[p];
      const uint64_t dig = rem & ((1ull << lgp) - 1);
      rem >>= lgp;
      wbits_tail -= lgp;
      mid_nat |= dig << wbits_tail;
    }
  }
  const int c = lane % D::CPW, rg = lane / D::CPW;
  const uint64_t k0 = g * D::CPW + c;
  const uint64_t colbase = k0 * (1ull << (L - l0)) + (midx << M);
  F29 x[8];
  sfor<0, 8>([&](auto qc) {
    constexpr int qq = decltype(qc)::value;
    x[qq] = ld29(data + colbase + rg + D::LPC * qq);
  });
  D::run(x, w, rg);
  const uint64_t kstride = 1ull << (L - M);
  sfor<0, 8>([&](auto qc) {
    constexpr int qq = decltype(qc)::value;
    const uint32_t k = brev_bits(WaveDif<M>::rpos(qq, rg), M);
    const uint64_t y = k0 + mid_nat + (uint64_t)k * kstride;
    if (!TRUNC || y < out_len) {
      if constexpr (ONE) {
        st29(out + y, sub_m_if_ge29<FrParams>(reduce29<FrParams>(x[qq])));
      } else {
        const uint32_t md = mod3(y);
        // the epilogue constant (scale and / or zeta power) also brings the value below
        // 2.6 M; two conditional subtractions reach [0, M)
        const F29 v = mul29<FrParams>(x[qq], sel29(md == 1, k29.mul[1], sel29(md == 2, k29.mul[2], k29.mul[0])));
        st29(out + y, sub_m_if_ge29<FrParams>(sub_m_if_ge29<FrParams>(v)));
      }
    }
  });
}

// ---------------------------------------------------------------------------
// Whole transform in one block (N <= 2^NTT_SMALL_MAX_LOG), radix-2 DIF in LDS.
__global__ void __launch_bounds__(256)
ntt_small_kernel(NttIo io, uint64_t n_in, uint64_t out_len, NttTables tab, int L,
                 int in_distribute, Fr iz1, Fr iz2, int has_scale, Fr scale, int out_distribute,
                 Fr oz1, Fr oz2) {
  const Fr* src = io.src[blockIdx.x];
  Fr* out = io.dst[blockIdx.x];
  extern __shared__ __align__(16) unsigned char smem_raw[];
  Fr* s = reinterpret_cast<Fr*>(smem_raw);
  const int N = 1 << L;
  Fr* w = s + N;
  for (int j = threadIdx.x; j < N / 2; j += blockDim.x) w[j] = twiddle(tab, (uint64_t)j);
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    Fr v = Fr::zero();
    if ((uint64_t)i < n_in) {
      v = ld_fr(src + i);
      if (in_distribute) {
        const int md = i % 3;
        if (md == 1) v = v * iz1;
        else if (md == 2) v = v * iz2;
      }
    }
    s[i] = v;
  }
  __syncthreads();
  for (int hlog = L - 1; hlog >= 0; hlog--) {
    const int h = 1 << hlog;
    for (int t = threadIdx.x; t < N / 2; t += blockDim.x) {
      const int j = t & (h - 1);
      const int i = ((t >> hlog) << (hlog + 1)) + j;
      const Fr a = s[i], b = s[i + h];
      s[i] = a + b;
      s[i + h] = (a - b) * w[j << (L - 1 - hlog)];
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    if ((uint64_t)k >= out_len) continue;
    Fr v = s[L > 0 ? brev_bits((uint32_t)k, L) : 0];
    if (has_scale) v = v * scale;
    if (out_distribute) {
      const int md = k % 3;
      if (md == 1) v = v * oz1;
      else if (md == 2) v = v * oz2;
    }
    st_fr(out + k, v);
  }
}

// ---------------------------------------------------------------------------
// Twiddle tables: lo[j] = w^j (j < 2^b), hi[j] = w^(j 2^b) (j < 2^(L-b)).
__global__ void ntt_tables_kernel(Fr* lo, Fr* hi, Fr w, int b, int L) {
  const uint64_t nlo = 1ull << b, nhi = 1ull << (L - b);
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t < nlo) lo[t] = pow_u64(w, t);
  if (t < nhi) {
    Fr wb = w;
    for (int i = 0; i < b; i++) wb = sqr(wb);
    hi[t] = pow_u64(wb, t);
  }
}

// w_64^j = w^(j 2^(L - 6)), j < 32, as packed F29 elements (the F29 passes' LDS twiddles)
__global__ void ntt_root64_kernel(Fr* out, NttTables tab, int L) {
  const int j = threadIdx.x;
  if (j < 32) out[j] = storage_to_f29_packed<FrParams>(twiddle(tab, (uint64_t)j << (L - 6)));
}

// lo / hi as packed F29 elements
__global__ void ntt_tables29_kernel(Fr* lo29, Fr* hi29, const Fr* lo, const Fr* hi, uint64_t nlo, uint64_t nhi) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t < nlo) lo29[t] = storage_to_f29_packed<FrParams>(lo[t]);
  if (t < nhi) hi29[t] = storage_to_f29_packed<FrParams>(hi[t]);
}

// pass table: t = k * S + i_low over [0, 2^lrem): w^(i_low k 2^(L - lrem))
__global__ void ntt_pass_tw_kernel(Fr* out, NttTables tab, int L, int lrem, int M, int fold) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= (1ull << lrem)) return;
  const uint64_t S = 1ull << (lrem - M);
  const uint64_t k = t / S, ilow = t % S;
  Fr v = twiddle(tab, (ilow * k) << (L - lrem));
  if (fold) v = v * tab.fold;  // the first pass carries the transform's scale
  out[t] = H2G_NTT29 ? storage_to_f29_packed<FrParams>(v) : v;  // the passes' form
}

// ---------------------------------------------------------------------------
// Host side

void ntt_split(int L, int* P, int lg[NTT_MAX_PASSES]) {
  if (L <= NTT_SMALL_MAX_LOG) {
    *P = 1;
    lg[0] = L;
    return;
  }
  int p = (L + 5) / 6;
  const int R = L - 6 * (p - 1);
  int i = 0;
#ifndef H2G_NTT_SPLIT  // A/B: 0 = the short pass first, 1 = second, 2 = two 5-bit passes for a 4-bit one
#define H2G_NTT_SPLIT 0
#endif
  if (H2G_NTT_SPLIT == 2 && R == 4 && p >= 3) {
    lg[i++] = 5;
    lg[i++] = 5;
  } else if (R >= 3) {
    if (H2G_NTT_SPLIT == 1 && p >= 3) lg[i++] = 6;
    lg[i++] = R;
  } else {  // borrow 3 bits so every pass has 3..6 bits
    lg[i++] = 3;
    lg[i++] = R + 3;
  }
  while (i < p) lg[i++] = 6;
  *P = p;
}

hipError_t ntt_build_tables(NttTables* t, const Fr& omega, int L, hipStream_t st, const Fr& fold) {
  t->L = L;
  t->fold = fold;
  t->fold_inv = inv(fold);
  t->b = (L + 1) / 2;
  if (t->b < 1) t->b = 1;
  const uint64_t nlo = 1ull << t->b, nhi = 1ull << (L > t->b ? L - t->b : 0);
  hipError_t e = hipMalloc(&t->lo, nlo * sizeof(Fr));
  if (e != hipSuccess) return e;
  e = hipMalloc(&t->hi, (nhi > 0 ? nhi : 1) * sizeof(Fr));
  if (e != hipSuccess) return e;
  const uint64_t mx = nlo > nhi ? nlo : nhi;
  const int bs = 256;
  hipLaunchKernelGGL(ntt_tables_kernel, dim3((unsigned)((mx + bs - 1) / bs)), dim3(bs), 0, st, t->lo, t->hi,
                     omega, t->b, L < t->b ? t->b : L);
  e = hipGetLastError();
  if (e != hipSuccess || L <= NTT_SMALL_MAX_LOG) return e;
  int P, lg[NTT_MAX_PASSES];
  ntt_split(L, &P, lg);
  uint64_t total = 0;
  int lrem = L;
  for (int p = 0; p < P - 1; p++) {
    t->pass_off[p] = total;
    total += 1ull << lrem;
    lrem -= lg[p];
  }
  e = hipMalloc(&t->pass_tw, (total ? total : 1) * sizeof(Fr));
  if (e != hipSuccess) return e;
  e = hipMalloc(&t->root64, 32 * sizeof(Fr));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ntt_root64_kernel, dim3(1), dim3(32), 0, st, t->root64, *t, L);
  e = hipMalloc(&t->lo29, nlo * sizeof(Fr));
  if (e != hipSuccess) return e;
  e = hipMalloc(&t->hi29, (nhi > 0 ? nhi : 1) * sizeof(Fr));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ntt_tables29_kernel, dim3((unsigned)((mx + bs - 1) / bs)), dim3(bs), 0, st, t->lo29, t->hi29,
                     t->lo, t->hi, nlo, nhi);
  lrem = L;
  for (int p = 0; p < P - 1; p++) {
    const uint64_t cnt = 1ull << lrem;
    hipLaunchKernelGGL(ntt_pass_tw_kernel, dim3((unsigned)((cnt + bs - 1) / bs)), dim3(bs), 0, st,
                       t->pass_tw + t->pass_off[p], *t, L, lrem, lg[p], p == 0 ? 1 : 0);
    lrem -= lg[p];
  }
  return hipGetLastError();
}

void ntt_free_tables(NttTables* t) {
  if (t->lo) (void)hipFree(t->lo);
  if (t->hi) (void)hipFree(t->hi);
  if (t->pass_tw) (void)hipFree(t->pass_tw);
  if (t->root64) (void)hipFree(t->root64);
  if (t->lo29) (void)hipFree(t->lo29);
  if (t->hi29) (void)hipFree(t->hi29);
  t->lo = t->hi = t->pass_tw = t->root64 = t->lo29 = t->hi29 = nullptr;
}

hipError_t ntt_init_attributes() {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(&ntt_small_kernel),
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int M>
static void launch_pass(const NttArgs& a, const NttIo& io, int B, int p, int first, uint64_t n_in, int L, int lrem,
                        int dist, const NttConst29& k29, hipStream_t st) {
  const uint64_t N = 1ull << L;
  const uint64_t waves = N / ((1ull << M) * WaveDif<M>::CPW);
  const unsigned blocks = (unsigned)((waves + NTT_WAVES - 1) / NTT_WAVES);
  if (H2G_NTT29 && H2G_NTT_SPARSE && M == 3 && first && n_in <= (N >> 2)) {
    const uint64_t S = N >> 3;
    hipLaunchKernelGGL(ntt_first_sparse29_kernel, dim3((unsigned)((S + NTT_THREADS - 1) / NTT_THREADS), (unsigned)B),
                       dim3(NTT_THREADS), 0, st, a.work, io, n_in, a.tab,
                       (const Fr*)(a.tab.pass_tw + a.tab.pass_off[p]), L, dist, k29);
    return;
  }
  if (H2G_NTT29 && H2G_NTT_PIPE && !first) {  // two 4-wave blocks per CU over the whole batch, every wave several groups
    const uint64_t want = (uint64_t)ntt_cus() * 2 / (uint64_t)B;
    const unsigned pb = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks, want));
    hipLaunchKernelGGL(ntt_pass29p_kernel<M>, dim3(pb, (unsigned)B), dim3(NTT_THREADS), 0, st, a.work, a.tab,
                       (const Fr*)(a.tab.pass_tw + a.tab.pass_off[p]), L, lrem, waves);
    return;
  }
  if (H2G_NTT29)
    hipLaunchKernelGGL(ntt_pass29_kernel<M>, dim3(blocks, (unsigned)B), dim3(NTT_THREADS), 0, st, a.work, io, first,
                       n_in, a.tab, (const Fr*)(a.tab.pass_tw + a.tab.pass_off[p]), L, lrem, dist, k29);
  else
    hipLaunchKernelGGL(ntt_pass_kernel<M>, dim3(blocks, (unsigned)B), dim3(NTT_THREADS), 0, st, a.work, io, first,
                       n_in, a.tab, (const Fr*)(a.tab.pass_tw + a.tab.pass_off[p]), L, lrem, dist, a.in_z1, a.in_z2);
}

hipError_t ntt_run(const NttArgs& a, hipStream_t st) {
  const int L = a.tab.L;
  const uint64_t N = 1ull << L;
  const uint64_t out_len = a.out_len ? a.out_len : N;
  const int B = a.count < 1 ? 1 : a.count;
  if (B > NTT_MAX_BATCH) return hipErrorInvalidValue;
  NttIo io = {};
  for (int b = 0; b < B; b++) {
    io.src[b] = B == 1 ? a.src : a.srcs[b];
    io.dst[b] = B == 1 ? a.dst : a.dsts[b];
  }
  NttPlanLg plan;
  ntt_split(L, &plan.p, plan.lg);
  const int P = plan.p;
  const int* lg = plan.lg;
  if (P == 1) {
    const size_t sm = (N + N / 2 + 1) * sizeof(Fr);
    hipLaunchKernelGGL(ntt_small_kernel, dim3((unsigned)B), dim3(256), sm, st, io, a.n_in, out_len, a.tab, L,
                       a.in_distribute, a.in_z1, a.in_z2, a.has_scale, a.scale, a.out_distribute, a.out_z1,
                       a.out_z2);
    return hipGetLastError();
  }
  if (P > NTT_MAX_PASSES || lg[P - 1] != 6 || !a.tab.pass_tw) return hipErrorInvalidValue;
  // epilogue multiplier per (y mod 3): scale * zeta-power / the scale folded into the
  // first pass's table, on the host
  Fr mul[3];
  bool one = true;
  for (int r = 0; r < 3; r++) {
    Fr m = (a.has_scale ? a.scale : Fr::one()) * a.tab.fold_inv;
    if (a.out_distribute && r == 1) m = m * a.out_z1;
    if (a.out_distribute && r == 2) m = m * a.out_z2;
    mul[r] = m;
    one = one && m == Fr::one();
  }
  const int has_mul = !one;
  NttConst29 k29;  // the F29 passes' constants
  k29.z1 = storage_to_f29<FrParams>(a.in_z1);
  k29.z2 = storage_to_f29<FrParams>(a.in_z2);
  for (int r = 0; r < 3; r++) k29.mul[r] = storage_to_f29<FrParams>(mul[r]);
  // N / N_0 and every middle S are multiples of 64 >= CPW: waves divide evenly.
  // pass 0: src -> work (out of place), passes 1..P-2 in place on work,
  // last pass: work -> dst in natural order.
  int lrem = L;
  for (int p = 0; p < P - 1; p++) {
    const int first = p == 0;
    const uint64_t nin = first ? a.n_in : 0;
    const int dist = first ? a.in_distribute : 0;
    switch (lg[p]) {
      case 3: launch_pass<3>(a, io, B, p, first, nin, L, lrem, dist, k29, st); break;
      case 4: launch_pass<4>(a, io, B, p, first, nin, L, lrem, dist, k29, st); break;
      case 5: launch_pass<5>(a, io, B, p, first, nin, L, lrem, dist, k29, st); break;
      case 6: launch_pass<6>(a, io, B, p, first, nin, L, lrem, dist, k29, st); break;
      default: return hipErrorInvalidValue;
    }
    lrem -= lg[p];
  }
  {
    const uint64_t waves = N / (64ull * WaveDif<6>::CPW);
    const unsigned blocks = (unsigned)((waves + NTT_WAVES - 1) / NTT_WAVES);
    const dim3 g(blocks, (unsigned)B), b(NTT_THREADS);
    const bool tr = out_len < N;
    if (H2G_NTT29 && tr && one)
      hipLaunchKernelGGL((ntt_last29_kernel<true, true>), g, b, 0, st, (const Fr*)a.work, io, out_len, a.tab, L, plan,
                         k29);
    else if (H2G_NTT29 && tr)
      hipLaunchKernelGGL((ntt_last29_kernel<true, false>), g, b, 0, st, (const Fr*)a.work, io, out_len, a.tab, L,
                         plan, k29);
    else if (H2G_NTT29 && one)
      hipLaunchKernelGGL((ntt_last29_kernel<false, true>), g, b, 0, st, (const Fr*)a.work, io, out_len, a.tab, L,
                         plan, k29);
    else if (H2G_NTT29)
      hipLaunchKernelGGL((ntt_last29_kernel<false, false>), g, b, 0, st, (const Fr*)a.work, io, out_len, a.tab, L,
                         plan, k29);
    else
      hipLaunchKernelGGL(ntt_last_kernel, dim3(blocks, (unsigned)B), dim3(NTT_THREADS), 0, st, (const Fr*)a.work,
                         io, out_len, a.tab, L, plan, has_mul, mul[0], mul[1], mul[2]);
  }
  return hipGetLastError();
}

}  // namespace h2g
