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
// Montgomery's trick over the strided subset {i = t (mod T)} of each thread:
// 3 multiplications per element + one inversion per thread (bn254.h inv: binary
// extended Euclid, whose short dependent chain bounds the kernel's latency).
// Arrays of one launch (blockIdx.y): independent batch inversions share the latency of
// the per-thread inversion (e.g. every lookup's product denominators at once).
struct InvBatch {
  Fr* a[POLY_INV_MAX_BATCH];
  Fr* pref[POLY_INV_MAX_BATCH];
};

__global__ void __launch_bounds__(PT) batch_invert_kernel(InvBatch bt, size_t n) {
  Fr* __restrict__ a = bt.a[blockIdx.y];
  Fr* __restrict__ pref = bt.pref[blockIdx.y];
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= n) return;
  Fr acc = Fr::one();
  size_t last = t;
  for (size_t i = t; i < n; i += T) {
    stf(pref + i, acc);
    const Fr x = ldf(a + i);
    if (!x.is_zero()) acc = acc * x;
    last = i;
  }
  Fr iv = inv(acc);
  for (size_t i = last;; i -= T) {
    const Fr x = ldf(a + i);
    if (!x.is_zero()) {
      const Fr r = iv * ldf(pref + i);
      iv = iv * x;
      stf(a + i, r);
    }
    if (i < T) break;
  }
}

hipError_t poly_batch_invert_multi(Fr* const* a, Fr* const* scratch, int count, size_t n, hipStream_t st) {
  if (n == 0 || count <= 0) return hipSuccess;
  // elements per thread: the serial chain is ~3 per products + one inversion, the
  // inversions' total work n / per of them -- measured on MI355X, 4 at 2^18 (keccak-style
  // proof) and 32 at 2^22 (C3) are best: about 2^16 threads per array
  static const long env_per = [] {
    const char* e = getenv("H2G_BINV_PER");
    return e ? atol(e) : 0L;
  }();
  size_t per = env_per > 0 ? (size_t)env_per : std::min<size_t>(32, std::max<size_t>(4, n >> 16));
  size_t threads = (n + per - 1) / per;  // elements per thread amortise the inversion
  if (threads < 1) threads = 1;
  const unsigned blocks = (unsigned)((threads + PT - 1) / PT);
  for (int b0 = 0; b0 < count; b0 += POLY_INV_MAX_BATCH) {
    const int m = std::min(POLY_INV_MAX_BATCH, count - b0);
    InvBatch bt = {};
    for (int i = 0; i < m; i++) {
      bt.a[i] = a[b0 + i];
      bt.pref[i] = scratch[b0 + i];
    }
    hipLaunchKernelGGL(batch_invert_kernel, dim3(blocks, (unsigned)m), dim3(PT), 0, st, bt, n);
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

__global__ void __launch_bounds__(PT) prefix_phase1(const Fr* __restrict__ a, size_t n, Fr* __restrict__ tile_prod) {
  __shared__ Fr sh[PT];
  const size_t base = blockIdx.x * PTILE + (size_t)threadIdx.x * PK;
  Fr p = Fr::one();
  for (int k = 0; k < PK; k++)
    if (base + k < n) p = p * ldf(a + base + k);
  Fr total;
  block_exclusive_scan_mul(p, sh, &total);
  if (threadIdx.x == 0) tile_prod[blockIdx.x] = total;
}

// single block: exclusive scan of m tile products, in place
__global__ void __launch_bounds__(PT) prefix_phase2(Fr* __restrict__ tp, size_t m) {
  __shared__ Fr sh[PT];
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

__global__ void __launch_bounds__(PT) prefix_phase3(const Fr* __restrict__ a, Fr* __restrict__ out, size_t n,
                                                    const Fr* __restrict__ tile_excl) {
  __shared__ Fr sh[PT];
  const size_t base = blockIdx.x * PTILE + (size_t)threadIdx.x * PK;
  Fr p = Fr::one();
  for (int k = 0; k < PK; k++)
    if (base + k < n) p = p * ldf(a + base + k);
  Fr run = block_exclusive_scan_mul(p, sh, nullptr);
  run = tile_excl[blockIdx.x] * run;
  for (int k = 0; k < PK; k++)
    if (base + k < n) {
      run = run * ldf(a + base + k);
      stf(out + base + k, run);
    }
}

size_t poly_prefix_scratch_len(size_t n) { return (n + PTILE - 1) / PTILE + 1; }

hipError_t poly_prefix_product(const Fr* a, Fr* out, size_t n, Fr* scratch, size_t scratch_len, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t m = (n + PTILE - 1) / PTILE;
  if (scratch_len < m) return hipErrorInvalidValue;
  hipLaunchKernelGGL(prefix_phase1, dim3((unsigned)m), dim3(PT), 0, st, a, n, scratch);
  hipLaunchKernelGGL(prefix_phase2, dim3(1), dim3(PT), 0, st, scratch, m);
  hipLaunchKernelGGL(prefix_phase3, dim3((unsigned)m), dim3(PT), 0, st, a, out, n, (const Fr*)scratch);
  return hipGetLastError();
}

}  // namespace h2g
