// ntt.hip -- radix-2^m LDS-tiled NTT over BN254 Fr for gfx950.
//
// Computes exactly what halo2curves' best_fft computes (natural order in,
// natural order out, y_k = sum_i a_i w^(ik)), as called by
// EvaluationDomain (halo2_backend/src/poly/domain.rs:220, 238, 275, 344),
// plus the fused pre/post maps of coeff_to_extended / extended_to_coeff /
// lagrange_to_coeff (domain.rs:216-293).
//
// Algorithm: N = N_1 * ... * N_P (each N_p <= 2^8).  With i = i_low + (L_p/N_p) i_p
// the pass-p DFT runs over i_p in LDS, then multiplies by w^{(N/L_p) i_low k_p}
// (in place).  The last pass reads contiguous runs and writes natural order
// (digit reversal folded into its store).  Every pass touches HBM once:
// 64 B/element/pass of algorithmic traffic, reads and writes in >= 256 B runs
// (G = 8 adjacent columns of 32-B elements).  Twiddles come from a 2-level
// table w^E = lo[E mod 2^b] * hi[E >> b] (both L2-resident).
#include "ntt.h"

namespace h2g {

static constexpr int NTT_G = 8;        // columns per block (8 x 32 B = 256 B runs)
static constexpr int NTT_THREADS = 256;

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

// In-LDS radix-2 DIF over `cols` columns of length 2^m (column c at s[c*len]).
// Input natural order, output bit-reversed.  `w` holds w_len^j, j < len/2.
__device__ __forceinline__ void lds_dif(Fr* s, const Fr* w, int m, int cols) {
  const int len = 1 << m;
  const int nbf = cols * (len >> 1);
  for (int hlog = m - 1; hlog >= 0; hlog--) {
    const int h = 1 << hlog;
    for (int t = threadIdx.x; t < nbf; t += blockDim.x) {
      const int c = t >> (m - 1);
      const int r = t & ((len >> 1) - 1);
      const int j = r & (h - 1);
      const int i = ((r >> hlog) << (hlog + 1)) + j;
      Fr* col = s + c * len;
      const Fr u = col[i];
      const Fr v = col[i + h];
      col[i] = u + v;
      const Fr d = u - v;
      col[i + h] = (hlog == m - 1) ? d * w[j] : d * w[j << (m - 1 - hlog)];
    }
    __syncthreads();
  }
}

__device__ __forceinline__ int brev(int x, int m) { return (int)(__brev((unsigned)x) >> (32 - m)); }

// ---------------------------------------------------------------------------
// Generic (non-last) pass, in place.  grid = N / (N_p * G) blocks.
//   L_p = 2^lrem (remaining length including this pass), S = L_p / N_p.
//   Optional input map on pass 0 (coset extend): read `in` (length n_in) with
//   zero padding and multiply by zeta powers (domain.rs:325-341).
__global__ void __launch_bounds__(NTT_THREADS)
ntt_pass_kernel(Fr* data, const Fr* in, uint64_t n_in, NttTables tab, int L, int m, int lrem,
                int distribute, Fr z1, Fr z2) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  Fr* s = reinterpret_cast<Fr*>(smem_raw);
  const int Np = 1 << m;
  Fr* w = s + NTT_G * Np;
  const uint64_t S = 1ull << (lrem - m);
  const uint64_t groups = S / NTT_G;
  const uint64_t q = blockIdx.x / groups;
  const uint64_t g = blockIdx.x % groups;
  const uint64_t base = (q << lrem) + g * NTT_G;
  // inner twiddles w_{Np}^j = w^{(N/Np) j}
  for (int j = threadIdx.x; j < Np / 2; j += blockDim.x) w[j] = twiddle(tab, (uint64_t)j << (L - m));
  for (int t = threadIdx.x; t < NTT_G * Np; t += blockDim.x) {
    const int c = t % NTT_G, r = t / NTT_G;
    const uint64_t pos = base + c + (uint64_t)r * S;
    Fr v;
    if (in) {
      if (pos < n_in) {
        v = ld_fr(in + pos);
        if (distribute) {
          const uint32_t md = (uint32_t)(pos % 3);
          if (md == 1) v = v * z1;
          else if (md == 2) v = v * z2;
        }
      } else {
        v = Fr::zero();
      }
    } else {
      v = ld_fr(data + pos);
    }
    s[c * Np + r] = v;
  }
  __syncthreads();
  lds_dif(s, w, m, NTT_G);
  const uint64_t stride_prefix = (uint64_t)1 << (L - lrem);  // N / L_p
  for (int t = threadIdx.x; t < NTT_G * Np; t += blockDim.x) {
    const int c = t % NTT_G, k = t / NTT_G;
    Fr v = s[c * Np + brev(k, m)];
    const uint64_t ilow = g * NTT_G + c;
    const uint64_t e = (stride_prefix * ilow * (uint64_t)k) & ((1ull << L) - 1);
    if (e) v = v * twiddle(tab, e);
    st_fr(data + base + c + (uint64_t)k * S, v);
  }
}

// ---------------------------------------------------------------------------
// Last pass: contiguous runs of N_P, output in natural order.
//   pos = k1 (N/N1) + m_idx N_P + i_P ;  y = k1 + N1 * mid_nat(m_idx) + (N/N_P) k_P
//   digits of m_idx (position order, least significant = k_{P-1}) are given by
//   lg[1..P-2].  Epilogue: multiply by `scale` and, if `distribute`, by the
//   zeta power of y mod 3; drop y >= out_len (truncation, domain.rs:288-290).
__global__ void __launch_bounds__(NTT_THREADS)
ntt_last_kernel(const Fr* data, Fr* out, uint64_t out_len, NttTables tab, int L, int P, int4 lg,
                int has_scale, Fr scale, int distribute, Fr z1, Fr z2) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  Fr* s = reinterpret_cast<Fr*>(smem_raw);
  const int lgs[4] = {lg.x, lg.y, lg.z, lg.w};
  const int m = lgs[P - 1];
  const int Np = 1 << m;
  const int l1 = lgs[0];
  Fr* w = s + NTT_G * Np;
  const uint64_t N1 = 1ull << l1;
  const uint64_t groups = N1 / NTT_G;
  const uint64_t midx = blockIdx.x / groups;
  const uint64_t g = blockIdx.x % groups;
  // decode middle digits: m_idx = k2 * (N3..N_{P-1}) + ... + k_{P-1}
  uint64_t mid_nat = 0;
  {
    uint64_t rem = midx;
    int lsum_before = L - lgs[P - 1];  // bits of k1..k_{P-1}
    // natural weight of k_p is N1*..*N_{p-1}
    for (int p = P - 2; p >= 1; p--) {
      const uint64_t dig = rem & ((1ull << lgs[p]) - 1);
      rem >>= lgs[p];
      int wbits = 0;
      for (int qq = 0; qq < p; qq++) wbits += lgs[qq];
      mid_nat |= dig << wbits;
    }
    (void)lsum_before;
  }
  for (int j = threadIdx.x; j < Np / 2; j += blockDim.x) w[j] = twiddle(tab, (uint64_t)j << (L - m));
  const uint64_t colstride = 1ull << (L - l1);  // N / N1
  for (int t = threadIdx.x; t < NTT_G * Np; t += blockDim.x) {
    const int c = t / Np, i = t % Np;
    const uint64_t pos = (g * NTT_G + c) * colstride + (midx << m) + i;
    s[c * Np + i] = ld_fr(data + pos);
  }
  __syncthreads();
  lds_dif(s, w, m, NTT_G);
  const uint64_t kstride = 1ull << (L - m);  // N / N_P
  for (int t = threadIdx.x; t < NTT_G * Np; t += blockDim.x) {
    const int c = t % NTT_G, k = t / NTT_G;
    const uint64_t y = (g * NTT_G + c) + mid_nat + (uint64_t)k * kstride;
    if (y >= out_len) continue;
    Fr v = s[c * Np + brev(k, m)];
    if (has_scale) v = v * scale;
    if (distribute) {
      const uint32_t md = (uint32_t)(y % 3);
      if (md == 1) v = v * z1;
      else if (md == 2) v = v * z2;
    }
    st_fr(out + y, v);
  }
}

// ---------------------------------------------------------------------------
// Whole transform in one block (N <= 2^11): same maps as above.
__global__ void __launch_bounds__(1024)
ntt_small_kernel(const Fr* src, uint64_t n_in, Fr* out, uint64_t out_len, NttTables tab, int L,
                 int in_distribute, Fr iz1, Fr iz2, int has_scale, Fr scale, int out_distribute,
                 Fr oz1, Fr oz2) {
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
  if (L > 0) lds_dif(s, w, L, 1);
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    if ((uint64_t)k >= out_len) continue;
    Fr v = s[L > 0 ? brev(k, L) : 0];
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

// ---------------------------------------------------------------------------
// Host side

void ntt_split(int L, int* P, int lg[4]) {
  if (L <= NTT_SMALL_MAX_LOG) { *P = 1; lg[0] = L; return; }
  int p = (L + NTT_MAX_PASS_LOG - 1) / NTT_MAX_PASS_LOG;
  if (p < 2) p = 2;
  int base = L / p, extra = L % p;
  for (int i = 0; i < p; i++) lg[i] = base + (i < extra ? 1 : 0);
  *P = p;
}

hipError_t ntt_build_tables(NttTables* t, const Fr& omega, int L, hipStream_t st) {
  t->L = L;
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
  return hipGetLastError();
}

void ntt_free_tables(NttTables* t) {
  if (t->lo) (void)hipFree(t->lo);
  if (t->hi) (void)hipFree(t->hi);
  t->lo = t->hi = nullptr;
}

hipError_t ntt_init_attributes() {
  hipError_t e;
  const int big = 160 * 1024;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ntt_pass_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, big);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ntt_last_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, big);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(&ntt_small_kernel),
                             hipFuncAttributeMaxDynamicSharedMemorySize, big);
}

hipError_t ntt_run(const NttArgs& a, hipStream_t st) {
  const int L = a.tab.L;
  const uint64_t N = 1ull << L;
  const uint64_t out_len = a.out_len ? a.out_len : N;
  int P, lg[4] = {0, 0, 0, 0};
  ntt_split(L, &P, lg);
  if (P == 1) {
    const size_t sm = (N + N / 2 + 1) * sizeof(Fr);
    const int threads = N >= 1024 ? 1024 : (N >= 64 ? (int)N : 64);
    hipLaunchKernelGGL(ntt_small_kernel, dim3(1), dim3(threads), sm, st, a.src, a.n_in, a.dst, out_len, a.tab,
                       L, a.in_distribute, a.in_z1, a.in_z2, a.has_scale, a.scale, a.out_distribute, a.out_z1,
                       a.out_z2);
    return hipGetLastError();
  }
  // pass 0: src -> work (out of place), passes 1..P-2 in place on work,
  // last pass: work -> dst in natural order.
  int lrem = L;
  for (int p = 0; p < P - 1; p++) {
    const int m = lg[p];
    const uint64_t blocks = N / ((1ull << m) * NTT_G);
    const size_t sm = (NTT_G * (1ull << m) + (1ull << m) / 2) * sizeof(Fr);
    hipLaunchKernelGGL(ntt_pass_kernel, dim3((unsigned)blocks), dim3(NTT_THREADS), sm, st, a.work,
                       p == 0 ? a.src : (const Fr*)nullptr, p == 0 ? a.n_in : 0, a.tab, L, m, lrem,
                       p == 0 ? a.in_distribute : 0, a.in_z1, a.in_z2);
    lrem -= m;
  }
  {
    const int m = lg[P - 1];
    const uint64_t blocks = N / ((1ull << m) * NTT_G);
    const size_t sm = (NTT_G * (1ull << m) + (1ull << m) / 2) * sizeof(Fr);
    hipLaunchKernelGGL(ntt_last_kernel, dim3((unsigned)blocks), dim3(NTT_THREADS), sm, st, (const Fr*)a.work,
                       a.dst, out_len, a.tab, L, P, make_int4(lg[0], lg[1], lg[2], lg[3]), a.has_scale, a.scale,
                       a.out_distribute, a.out_z1, a.out_z2);
  }
  return hipGetLastError();
}

}  // namespace h2g
