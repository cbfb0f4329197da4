// radix.hip -- LSD radix sort of (u64 key, u32 value) pairs for gfx950, and the stream
// compaction the lookup argument needs (see radix.h).
//
// permute_expression_pair (halo2_backend/src/plonk/lookup/prover.rs:410-494) sorts each
// lookup's compressed input and table columns by value.  All of a proof's columns go
// through ONE sort: segment s's keys carry s above their key bits, so the composite keys
// order the columns one after another and each column's rows come out contiguous and
// sorted -- a few launches per 8-bit digit for the whole proof instead of a library sort
// (and its launches) per column.
//
// Per 8-bit digit pass, tiles of RX_TILE = 256 threads x 16 rows:
//   radix_hist_kernel    per-tile digit histogram (LDS), digit-major counts[d][tile]
//   scan (3 kernels)     exclusive scan of the counts = every (digit, tile)'s output base
//   radix_scatter_kernel stable scatter: a row's rank among the tile's earlier rows with
//                        its digit from 8 wave ballots (lanes with equal digits) plus the
//                        earlier waves' and rows' counts in LDS
// Stability makes the passes compose (least significant digit first).
#include "radix.h"

namespace h2g {

static constexpr int RX_T = 256;
static constexpr int RX_ROWS = 16;
static constexpr uint32_t RX_TILE = (uint32_t)RX_T * RX_ROWS;

__global__ void __launch_bounds__(RX_T) radix_hist_kernel(const uint64_t* __restrict__ keys, uint32_t n, int shift,
                                                         uint32_t ntiles, uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[256];
  const uint32_t t = threadIdx.x;
  h[t] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RX_TILE;
#pragma unroll 4
  for (int i = 0; i < RX_ROWS; i++) {
    const uint32_t e = base + (uint32_t)i * RX_T + t;
    if (e < n) atomicAdd(&h[(uint32_t)(keys[e] >> shift) & 255u], 1u);
  }
  __syncthreads();
  counts[(size_t)t * ntiles + blockIdx.x] = h[t];
}

__global__ void __launch_bounds__(RX_T) radix_scatter_kernel(const uint64_t* __restrict__ kin,
                                                            const uint32_t* __restrict__ vin, uint64_t* __restrict__ kout,
                                                            uint32_t* __restrict__ vout, uint32_t n, int shift,
                                                            uint32_t ntiles, const uint32_t* __restrict__ offs) {
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[RX_T / 64][256];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  base[t] = offs[(size_t)t * ntiles + blockIdx.x];
#pragma unroll
  for (int q = 0; q < RX_T / 64; q++) wcnt[q][t] = 0;
  __syncthreads();
  const uint32_t tile = blockIdx.x * RX_TILE;
  const uint64_t below = (1ull << lane) - 1;
  for (int i = 0; i < RX_ROWS; i++) {
    const uint32_t e = tile + (uint32_t)i * RX_T + t;
    const bool valid = e < n;
    const uint64_t k = valid ? kin[e] : 0;
    const uint32_t v = valid ? vin[e] : 0;
    const uint32_t d = (uint32_t)(k >> shift) & 255u;
    uint64_t m = __ballot(valid);  // the wave's lanes holding this lane's digit
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t bb = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t rk = (uint32_t)__popcll(m & below);
    if (valid && rk == 0) wcnt[w][d] = (uint32_t)__popcll(m);
    __syncthreads();
    if (valid) {
      uint32_t pos = base[d] + rk;
      for (uint32_t q = 0; q < w; q++) pos += wcnt[q][d];
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int q = 0; q < RX_T / 64; q++) {
      add += wcnt[q][t];
      wcnt[q][t] = 0;
    }
    base[t] += add;
    __syncthreads();
  }
}

// exclusive scan of u32: 4096-element blocks (1024 threads x 4); the block sums are
// scanned by one block when they fit (<= 4096 blocks, len <= 2^24), else by the same
// routine recursively; then added back
static constexpr uint32_t SC_T = 1024, SC_PER = 4, SC_BLK = SC_T * SC_PER;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (uint32_t d = 1; d < SC_T; d <<= 1) {
    const uint32_t x = t >= d ? sh[t - d] : 0;
    __syncthreads();
    sh[t] += x;
    __syncthreads();
  }
  const uint32_t incl = sh[t];
  if (total) *total = sh[SC_T - 1];
  __syncthreads();
  return incl - v;
}

// in and out may alias (each thread reads its elements before the block scan's barriers)
__global__ void __launch_bounds__(SC_T) scan_blocks_kernel(const uint32_t* in, uint32_t* out, uint32_t len,
                                                          uint32_t* __restrict__ bsum) {
  __shared__ uint32_t sh[SC_T];
  const uint32_t lo = blockIdx.x * SC_BLK + threadIdx.x * SC_PER;
  uint32_t v[SC_PER], s = 0;
#pragma unroll
  for (uint32_t i = 0; i < SC_PER; i++) {
    v[i] = lo + i < len ? in[lo + i] : 0;
    s += v[i];
  }
  uint32_t tot;
  uint32_t run = block_excl_scan(s, sh, &tot);
#pragma unroll
  for (uint32_t i = 0; i < SC_PER; i++) {
    if (lo + i < len) out[lo + i] = run;
    run += v[i];
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SC_T) scan_sums_kernel(uint32_t* __restrict__ bsum, uint32_t nb) {
  __shared__ uint32_t sh[SC_T];
  const uint32_t lo = threadIdx.x * SC_PER;
  uint32_t v[SC_PER], s = 0;
#pragma unroll
  for (uint32_t i = 0; i < SC_PER; i++) {
    v[i] = lo + i < nb ? bsum[lo + i] : 0;
    s += v[i];
  }
  uint32_t run = block_excl_scan(s, sh, nullptr);
#pragma unroll
  for (uint32_t i = 0; i < SC_PER; i++) {
    if (lo + i < nb) bsum[lo + i] = run;
    run += v[i];
  }
}

__global__ void __launch_bounds__(SC_T) scan_add_kernel(uint32_t* __restrict__ out, uint32_t len,
                                                       const uint32_t* __restrict__ bsum) {
  const uint32_t lo = blockIdx.x * SC_BLK + threadIdx.x * SC_PER, add = bsum[blockIdx.x];
#pragma unroll
  for (uint32_t i = 0; i < SC_PER; i++)
    if (lo + i < len) out[lo + i] += add;
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t scan_u32_scratch_bytes(size_t len) {
  const size_t nb = (len + SC_BLK - 1) / SC_BLK;
  return align256((nb + 1) * 4) + (nb > SC_BLK ? scan_u32_scratch_bytes(nb) : 0);
}

hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, size_t len, void* scratch, hipStream_t st) {
  if (len == 0) return hipSuccess;
  if (len >= 0xffffffffull) return hipErrorInvalidValue;
  const uint32_t nb = (uint32_t)((len + SC_BLK - 1) / SC_BLK);
  uint32_t* bsum = static_cast<uint32_t*>(scratch);
  hipLaunchKernelGGL(scan_blocks_kernel, dim3(nb), dim3(SC_T), 0, st, in, out, (uint32_t)len, bsum);
  if (nb <= SC_BLK) {
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(SC_T), 0, st, bsum, nb);
  } else {  // more than 4096 blocks: the block sums in place, recursively
    const hipError_t e =
        exclusive_scan_u32(bsum, bsum, nb, static_cast<char*>(scratch) + align256(((size_t)nb + 1) * 4), st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(scan_add_kernel, dim3(nb), dim3(SC_T), 0, st, out, (uint32_t)len, (const uint32_t*)bsum);
  return hipGetLastError();
}

size_t radix_sort_scratch_bytes(size_t n) {
  const size_t ntiles = (n + RX_TILE - 1) / RX_TILE;
  const size_t nc = 256 * (ntiles ? ntiles : 1);
  return 2 * align256(nc * 4) + scan_u32_scratch_bytes(nc);
}

hipError_t radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt, size_t n,
                            int lo_bit, int hi_bit, void* scratch, hipStream_t st, bool* in_alt) {
  *in_alt = false;
  if (n == 0 || hi_bit <= lo_bit) return hipSuccess;
  if (n >= 0xffffffffull) return hipErrorInvalidValue;
  const uint32_t ntiles = (uint32_t)((n + RX_TILE - 1) / RX_TILE);
  const size_t nc = 256 * (size_t)ntiles;
  uint32_t* counts = static_cast<uint32_t*>(scratch);
  uint32_t* offs = reinterpret_cast<uint32_t*>(static_cast<char*>(scratch) + align256(nc * 4));
  void* sscr = static_cast<char*>(scratch) + 2 * align256(nc * 4);
  uint64_t *ka = keys, *kb = keys_alt;
  uint32_t *va = vals, *vb = vals_alt;
  for (int shift = lo_bit; shift < hi_bit; shift += 8) {
    hipLaunchKernelGGL(radix_hist_kernel, dim3(ntiles), dim3(RX_T), 0, st, (const uint64_t*)ka, (uint32_t)n, shift,
                       ntiles, counts);
    hipError_t e = exclusive_scan_u32(counts, offs, nc, sscr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(ntiles), dim3(RX_T), 0, st, (const uint64_t*)ka,
                       (const uint32_t*)va, kb, vb, (uint32_t)n, shift, ntiles, (const uint32_t*)offs);
    std::swap(ka, kb);
    std::swap(va, vb);
    *in_alt = !*in_alt;
  }
  return hipGetLastError();
}

// ---- helpers of the full (256-bit) sort: identity permutation, limb keys by permutation
__global__ void __launch_bounds__(256) iota_kernel(uint32_t* __restrict__ o, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) o[i] = i;
}
hipError_t iota_u32(uint32_t* out, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(iota_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, (uint32_t)n);
  return hipGetLastError();
}
__global__ void __launch_bounds__(256) limb_keys_kernel(const CanonKey* __restrict__ c, const uint32_t* __restrict__ idx,
                                                       uint32_t n, int limb, uint64_t* __restrict__ key) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const CanonKey& v = c[idx[i]];
  key[i] = (uint64_t)v.l[2 * limb] | ((uint64_t)v.l[2 * limb + 1] << 32);
}
hipError_t canon_limb_keys(const CanonKey* canon, const uint32_t* idx, size_t n, int limb, uint64_t* key,
                           hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(limb_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, canon, idx, (uint32_t)n,
                     limb, key);
  return hipGetLastError();
}

// ---- stream compaction: out[j] = in[i] for the j-th i with flag[i] != 0 (order kept)
__global__ void __launch_bounds__(256) flags_to_u32_kernel(const uint8_t* __restrict__ f, uint32_t* __restrict__ o,
                                                          uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) o[i] = f[i] ? 1u : 0u;
}
template <class T>
__global__ void __launch_bounds__(256) compact_kernel(const T* __restrict__ in, const uint8_t* __restrict__ f,
                                                     const uint32_t* __restrict__ pos, uint32_t n, T* __restrict__ out,
                                                     uint32_t* __restrict__ count) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (f[i]) out[pos[i]] = in ? in[i] : T{};
  if (i == n - 1) *count = pos[i] + (f[i] ? 1u : 0u);
}
// index variant: out[j] = i
__global__ void __launch_bounds__(256) compact_index_kernel(const uint8_t* __restrict__ f,
                                                           const uint32_t* __restrict__ pos, uint32_t n,
                                                           uint32_t* __restrict__ out, uint32_t* __restrict__ count) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (f[i]) out[pos[i]] = i;
  if (i == n - 1) *count = pos[i] + (f[i] ? 1u : 0u);
}

size_t compact_scratch_bytes(size_t n) { return 2 * align256(n * 4) + scan_u32_scratch_bytes(n); }

static hipError_t compact_prepare(const uint8_t* flags, size_t n, void* scratch, hipStream_t st, uint32_t** pos) {
  uint32_t* f32 = static_cast<uint32_t*>(scratch);
  *pos = reinterpret_cast<uint32_t*>(static_cast<char*>(scratch) + align256(n * 4));
  void* sscr = static_cast<char*>(scratch) + 2 * align256(n * 4);
  hipLaunchKernelGGL(flags_to_u32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, flags, f32, (uint32_t)n);
  return exclusive_scan_u32(f32, *pos, n, sscr, st);
}

hipError_t compact_canon(const CanonKey* in, const uint8_t* flags, size_t n, CanonKey* out, uint32_t* d_count,
                         void* scratch, hipStream_t st) {
  if (n == 0) return hipMemsetAsync(d_count, 0, 4, st);
  uint32_t* pos;
  hipError_t e = compact_prepare(flags, n, scratch, st, &pos);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(compact_kernel<CanonKey>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, flags,
                     (const uint32_t*)pos, (uint32_t)n, out, d_count);
  return hipGetLastError();
}

hipError_t compact_index(const uint8_t* flags, size_t n, uint32_t* out, uint32_t* d_count, void* scratch,
                         hipStream_t st) {
  if (n == 0) return hipMemsetAsync(d_count, 0, 4, st);
  uint32_t* pos;
  hipError_t e = compact_prepare(flags, n, scratch, st, &pos);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(compact_index_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, flags,
                     (const uint32_t*)pos, (uint32_t)n, out, d_count);
  return hipGetLastError();
}

}  // namespace h2g
