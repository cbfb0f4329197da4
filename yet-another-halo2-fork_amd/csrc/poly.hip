// poly.hip -- HBM-streaming elementwise kernels and Fr scans for gfx950.
//
// Elementwise ops restate halo2_backend/src/poly.rs:200-276 (Add, Sub, Mul<F>,
// Sub<F>) and domain.rs:297-316 (divide_by_vanishing_poly); every element is
// 32 B read per input and 32 B written, 16-B vector accesses, grid-stride loops.
// Scans restate ff::BatchInvert (permutation/prover.rs:124, lookup/prover.rs:225,
// shuffle/prover.rs:150) and the grand-product recurrences
// (permutation/prover.rs:160-166, lookup/prover.rs:254-265, shuffle/prover.rs:161-172).
#include "poly.h"
#include "fr_io.h"

#include <stdlib.h>

#include <algorithm>

namespace h2g {

static constexpr int PT = 256;

static unsigned grid_for(size_t n) {
  size_t g = (n + PT - 1) / PT;
  const size_t cap = 256 * 16;  // 256 CUs x 16 blocks, grid-stride beyond
  return (unsigned)(g < cap ? (g ? g : 1) : cap);
}

template <int OP>
__global__ void __launch_bounds__(PT) binop_kernel(const Fr* __restrict__ a, const Fr* __restrict__ b,
                                                   const Fr c, Fr* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const Fr x = ldf(a + i);
    Fr r;
    if (OP == POLY_ADD) r = x + ldf(b + i);
    else if (OP == POLY_SUB) r = x - ldf(b + i);
    else if (OP == POLY_MUL) r = x * ldf(b + i);
    else if (OP == POLY_SCALE) r = x * c;
    else if (OP == POLY_SUB_CONST) r = x - c;
    else if (OP == POLY_ADD_CONST) r = x + c;
    else r = x * c + ldf(b + i);
    stf(out + i, r);
  }
}

hipError_t poly_binop(int op, const Fr* a, const Fr* b, const Fr& c, Fr* out, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const dim3 g(grid_for(n)), blk(PT);
  switch (op) {
    case POLY_ADD: hipLaunchKernelGGL(binop_kernel<POLY_ADD>, g, blk, 0, st, a, b, c, out, n); break;
    case POLY_SUB: hipLaunchKernelGGL(binop_kernel<POLY_SUB>, g, blk, 0, st, a, b, c, out, n); break;
    case POLY_MUL: hipLaunchKernelGGL(binop_kernel<POLY_MUL>, g, blk, 0, st, a, b, c, out, n); break;
    case POLY_SCALE: hipLaunchKernelGGL(binop_kernel<POLY_SCALE>, g, blk, 0, st, a, b, c, out, n); break;
    case POLY_SUB_CONST: hipLaunchKernelGGL(binop_kernel<POLY_SUB_CONST>, g, blk, 0, st, a, b, c, out, n); break;
    case POLY_ADD_CONST: hipLaunchKernelGGL(binop_kernel<POLY_ADD_CONST>, g, blk, 0, st, a, b, c, out, n); break;
    case POLY_AXPY: hipLaunchKernelGGL(binop_kernel<POLY_AXPY>, g, blk, 0, st, a, b, c, out, n); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

__global__ void __launch_bounds__(PT) mul_cyclic_kernel(Fr* __restrict__ a, size_t n, const Fr* __restrict__ t,
                                                         size_t mask) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(a + i, ldf(a + i) * t[i & mask]);
}

hipError_t poly_mul_cyclic(Fr* a, size_t n, const Fr* t, size_t t_len, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (t_len == 0 || (t_len & (t_len - 1))) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mul_cyclic_kernel, dim3(grid_for(n)), dim3(PT), 0, st, a, n, t, t_len - 1);
  return hipGetLastError();
}

// ---------------------------------------------------------------- batch inversion
// Montgomery's trick in three levels, so the inversion (Bernstein-Yang divsteps, inv_by in bn254.h;
// ≈ 15 K uniform ops, ≈ 100 µs of one wave on gfx950) is paid once per ≈ 256 elements while
// the element passes keep 2^18+ threads in flight:
//   1. inv_fwd: thread t walks its strided subset {t + kT}, storing the running product
//      before each element (the prefix; 1 for k = 0, so slot t of the scratch is free and
//      takes the thread's total P_t);
//   2. inv_regs: the totals P_t (scratch[0..T)) inverted in place, INV_REG per thread with
//      the prefixes in registers and one inversion per thread;
//   3. inv_bwd: from 1/P_t back down the subset: 1/x_i = (1/P) * prefix_i, 1/P *= x_i.
// Zeros are skipped and stay zero (ff's invert().unwrap_or(ZERO)).  3 products per element
// plus 3 per INV_PER1 elements for level 2.  Arrays of one launch (blockIdx.y) are
// independent inversions (e.g. every lookup's product denominators at once).
struct InvBatch {
  Fr* a[POLY_INV_MAX_BATCH];
  Fr* pref[POLY_INV_MAX_BATCH];
};
static constexpr int INV_REG = 16;
// the middle level's inversion: Bernstein-Yang divsteps (inv_by, uniform across the wave's
// lanes) or the binary extended Euclid (inv, divergent); A/B builds -DH2G_INV_BY=0
#ifndef H2G_INV_BY
#define H2G_INV_BY 1
#endif

__global__ void __launch_bounds__(PT) inv_fwd_kernel(InvBatch bt, size_t n, size_t T) {
  const Fr* __restrict__ a = bt.a[blockIdx.y];
  Fr* __restrict__ pref = bt.pref[blockIdx.y];
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  Fr acc = Fr::one();
  {
    const Fr x = ldf(a + t);
    if (!x.is_zero()) acc = x;
  }
  for (size_t i = t + T; i < n; i += T) {
    stf(pref + i, acc);
    const Fr x = ldf(a + i);
    if (!x.is_zero()) acc = acc * x;
  }
  stf(pref + t, acc);
}

// in place over a[0..m) of each array (nonzero entries), no scratch
__global__ void __launch_bounds__(PT) inv_regs_kernel(InvBatch bt, size_t m) {
  Fr* __restrict__ a = bt.pref[blockIdx.y];
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  Fr v[INV_REG], pre[INV_REG];
  Fr acc = Fr::one();
#pragma unroll
  for (int k = 0; k < INV_REG; k++) {
    const size_t i = t + k * T;
    v[k] = i < m ? ldf(a + i) : Fr::zero();
    pre[k] = acc;
    if (!v[k].is_zero()) acc = acc * v[k];
  }
  Fr iv = H2G_INV_BY ? inv_by(acc) : inv(acc);
#pragma unroll
  for (int k = INV_REG - 1; k >= 0; k--) {
    const size_t i = t + k * T;
    if (!v[k].is_zero()) {
      stf(a + i, iv * pre[k]);
      iv = iv * v[k];
    }
  }
}

__global__ void __launch_bounds__(PT) inv_bwd_kernel(InvBatch bt, size_t n, size_t T) {
  Fr* __restrict__ a = bt.a[blockIdx.y];
  const Fr* __restrict__ pref = bt.pref[blockIdx.y];
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  Fr iv = ldf(pref + t);
  size_t last = t;
  while (last + T < n) last += T;
  for (size_t i = last; i > t; i -= T) {
    const Fr x = ldf(a + i);
    if (!x.is_zero()) {
      const Fr r = iv * ldf(pref + i);
      iv = iv * x;
      stf(a + i, r);
    }
  }
  if (!ldf(a + t).is_zero()) stf(a + t, iv);
}

hipError_t poly_batch_invert_multi(Fr* const* a, Fr* const* scratch, int count, size_t n, hipStream_t st) {
  if (n == 0 || count <= 0) return hipSuccess;
  // level-1 elements per thread: 16 once the arrays give 2^18 threads, fewer below
  size_t per = 16;
  while (per > 2 && (n * (size_t)count) / per < ((size_t)1 << 18)) per >>= 1;
  const size_t T = (n + per - 1) / per;
  const unsigned blk1 = (unsigned)((T + PT - 1) / PT);
  const size_t T2 = (T + INV_REG - 1) / INV_REG;
  const unsigned blk2 = (unsigned)((T2 + PT - 1) / PT);
  for (int b0 = 0; b0 < count; b0 += POLY_INV_MAX_BATCH) {
    const int m = std::min(POLY_INV_MAX_BATCH, count - b0);
    InvBatch bt = {};
    for (int i = 0; i < m; i++) {
      bt.a[i] = a[b0 + i];
      bt.pref[i] = scratch[b0 + i];
    }
    hipLaunchKernelGGL(inv_fwd_kernel, dim3(blk1, (unsigned)m), dim3(PT), 0, st, bt, n, T);
    hipLaunchKernelGGL(inv_regs_kernel, dim3(blk2, (unsigned)m), dim3(PT), 0, st, bt, T);
    hipLaunchKernelGGL(inv_bwd_kernel, dim3(blk1, (unsigned)m), dim3(PT), 0, st, bt, n, T);
  }
  return hipGetLastError();
}

hipError_t poly_batch_invert(Fr* a, size_t n, Fr* scratch, hipStream_t st) {
  return poly_batch_invert_multi(&a, &scratch, 1, n, st);
}

// ---------------------------------------------------------------- prefix product
// Tile = PT threads x K contiguous elements.  Phase 1: tile products; phase 2:
// exclusive scan of tile products (one block); phase 3: rescan with offsets.
static constexpr int PK = 8;
static constexpr size_t PTILE = (size_t)PT * PK;

__device__ Fr block_exclusive_scan_mul(Fr v, Fr* sh, Fr* total) {
  // Hillis-Steele inclusive scan in LDS, then shift.
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int off = 1; off < PT; off <<= 1) {
    Fr x = sh[t];
    if (t >= off) x = sh[t - off] * x;
    __syncthreads();
    sh[t] = x;
    __syncthreads();
  }
  const Fr incl = sh[t];
  const Fr excl = t ? sh[t - 1] : Fr::one();
  if (total) *total = sh[PT - 1];
  __syncthreads();
  (void)incl;
  return excl;
}

// Arrays of one launch (blockIdx.y) are independent scans (every lookup's product at once);
// array y's tile products live at scratch[y * (m + 1)].
struct PrefBatch {
  const Fr* a[POLY_INV_MAX_BATCH];
  Fr* out[POLY_INV_MAX_BATCH];
};

__global__ void __launch_bounds__(PT) prefix_phase1(PrefBatch pb, size_t n, Fr* __restrict__ tile_prod, size_t m) {
  __shared__ Fr sh[PT];
  const Fr* __restrict__ a = pb.a[blockIdx.y];
  const size_t base = blockIdx.x * PTILE + (size_t)threadIdx.x * PK;
  Fr p = Fr::one();
  for (int k = 0; k < PK; k++)
    if (base + k < n) p = p * ldf(a + base + k);
  Fr total;
  block_exclusive_scan_mul(p, sh, &total);
  if (threadIdx.x == 0) tile_prod[blockIdx.y * (m + 1) + blockIdx.x] = total;
}

// one block per array: exclusive scan of its m tile products, in place
__global__ void __launch_bounds__(PT) prefix_phase2(Fr* __restrict__ tile_prod, size_t m) {
  __shared__ Fr sh[PT];
  Fr* __restrict__ tp = tile_prod + blockIdx.x * (m + 1);
  const size_t per = (m + PT - 1) / PT;
  const size_t lo = threadIdx.x * per;
  Fr p = Fr::one();
  for (size_t i = lo; i < lo + per && i < m; i++) p = p * tp[i];
  Fr run = block_exclusive_scan_mul(p, sh, nullptr);
  for (size_t i = lo; i < lo + per && i < m; i++) {
    const Fr x = tp[i];
    tp[i] = run;
    run = run * x;
  }
}

// out may alias a (each thread reads its own elements before writing them)
__global__ void __launch_bounds__(PT) prefix_phase3(PrefBatch pb, size_t n, const Fr* __restrict__ tile_excl,
                                                    size_t m) {
  __shared__ Fr sh[PT];
  const Fr* a = pb.a[blockIdx.y];
  Fr* out = pb.out[blockIdx.y];
  const size_t base = blockIdx.x * PTILE + (size_t)threadIdx.x * PK;
  Fr x[PK];
  Fr p = Fr::one();
#pragma unroll
  for (int k = 0; k < PK; k++) {
    x[k] = base + k < n ? ldf(a + base + k) : Fr::one();
    p = p * x[k];
  }
  Fr run = block_exclusive_scan_mul(p, sh, nullptr);
  run = tile_excl[blockIdx.y * (m + 1) + blockIdx.x] * run;
#pragma unroll
  for (int k = 0; k < PK; k++)
    if (base + k < n) {
      run = run * x[k];
      stf(out + base + k, run);
    }
}

size_t poly_prefix_scratch_len(size_t n) { return (n + PTILE - 1) / PTILE + 1; }

hipError_t poly_prefix_product_multi(const Fr* const* a, Fr* const* out, int count, size_t n, Fr* scratch,
                                     size_t scratch_len, hipStream_t st) {
  if (n == 0 || count <= 0) return hipSuccess;
  const size_t m = (n + PTILE - 1) / PTILE;
  for (int b0 = 0; b0 < count; b0 += POLY_INV_MAX_BATCH) {
    const int c = std::min(POLY_INV_MAX_BATCH, count - b0);
    if (scratch_len < (size_t)c * (m + 1)) return hipErrorInvalidValue;
    PrefBatch pb = {};
    for (int i = 0; i < c; i++) {
      pb.a[i] = a[b0 + i];
      pb.out[i] = out[b0 + i];
    }
    hipLaunchKernelGGL(prefix_phase1, dim3((unsigned)m, (unsigned)c), dim3(PT), 0, st, pb, n, scratch, m);
    hipLaunchKernelGGL(prefix_phase2, dim3((unsigned)c), dim3(PT), 0, st, scratch, m);
    hipLaunchKernelGGL(prefix_phase3, dim3((unsigned)m, (unsigned)c), dim3(PT), 0, st, pb, n, (const Fr*)scratch, m);
  }
  return hipGetLastError();
}

hipError_t poly_prefix_product(const Fr* a, Fr* out, size_t n, Fr* scratch, size_t scratch_len, hipStream_t st) {
  return poly_prefix_product_multi(&a, &out, 1, n, scratch, scratch_len, st);
}

}  // namespace h2g
