// msm_part.hip -- the bucket partition of the MSM pipeline (msm.hip step 2) for gfx950:
// signed digits straight from the scalars into coarse bins, then keys inside the bins.
// Its own translation unit: none of it is elliptic-curve arithmetic, so it builds in
// seconds while msm.hip's point kernels take minutes.
#include <stdlib.h>

#include "msm_part.h"

namespace h2g {

// 1. signed digits: key = window * NB + |d| - 1 (generic mode), value = point index.
// Fixed-base mode (bases pre-multiplied per window, table[w * stride + i] = [2^(c w)] P_i):
// every window shares one set of NB buckets, key = |d| - 1, value = w * stride + i.
// Batched fixed-base mode (blockIdx.y = b of nbatch MSMs over the same windows): MSM b
// owns bucket set b, key = b * NB + |d| - 1, so one partition / accumulation / reduction
// serves them all.  Negative digits set bit 31 of the value.
// 2. bucket partition of the entries ------------------------------------------------
// The accumulation needs each bucket's entries contiguous, not sorted: a two-round
// counting partition replaces the radix sort.  Round 1 splits by the key's high bits
// (coarse bins) straight from the scalars, round 2 by the low FB bits inside each coarse
// bin (a bin's region is a few hundred KB, so its scattered writes stay in L2).  Zero
// digits produce no entry at all.  Order inside a bucket is arbitrary (the sum is exact).
#ifndef H2G_MSM_PT
#define H2G_MSM_PT 512
#endif
#ifndef H2G_MSM_FPER  // entries per fine-kernel thread: 8 (2048-entry tiles) measured best at 10 fine bits
#define H2G_MSM_FPER 8
#endif
static constexpr int PT = H2G_MSM_PT;      // threads of the coarse kernels (one scalar each)
static constexpr int PWG = 16;             // windows per coarse-kernel thread (grid.z groups)
static constexpr int FT = 256;             // threads of the fine kernels
static constexpr int FPER = H2G_MSM_FPER;  // entries per fine-kernel thread
static constexpr uint32_t FTILE = (uint32_t)FT * FPER;


// the signed digits of scalar i (batch bi) for windows [w0, w0 + PWG): fn(slot, key, val)
// for each nonzero digit (same key / value encoding as msm_digits_kernel); fixed-base
// windows take their balanced widths (fb_width), generic ones c bits each
template <class Fn>
__device__ __forceinline__ void scalar_digits(const MsmScalarList& list, size_t n, int c, int W, uint32_t NB,
                                              int fixed, size_t stride, uint32_t bi, size_t i, int w0, Fn fn) {
  const uint4* q = reinterpret_cast<const uint4*>(list.p[bi] + i);
  uint4 a = q[0], b = q[1];
  Fr s;
  s.l[0] = a.x; s.l[1] = a.y; s.l[2] = a.z; s.l[3] = a.w;
  s.l[4] = b.x; s.l[5] = b.y; s.l[6] = b.z; s.l[7] = b.w;
  Fr v = to_canonical(s);
  uint32_t carry = 0;
  const int wend = w0 + PWG < W ? w0 + PWG : W;
  for (int w = 0; w < wend; w++) {
    const int cw = fixed ? fb_width(W, w) : c;
    const uint32_t mask = (1u << cw) - 1;
    const uint32_t half = 1u << (cw - 1);
    const uint32_t d = (v.l[0] & mask) + carry;
#pragma unroll
    for (int k = 0; k < 7; k++) v.l[k] = (v.l[k] >> cw) | (v.l[k + 1] << (32 - cw));
    v.l[7] >>= cw;
    uint32_t mag, sign;
    if (d > half) {  // negative digit d - 2^cw (d == 2^cw gives digit 0, carry 1)
      mag = (1u << cw) - d;
      carry = 1;
      sign = 0x80000000u;
    } else {
      mag = d;
      carry = 0;
      sign = 0;
    }
    if (w < w0 || mag == 0) continue;
    uint32_t k = mag - 1;
    if (list.kn) {  // bucket range: keep [klo, klo + kn), rebased
      if (k - list.klo >= list.kn) continue;
      k -= list.klo;
    }
    const uint32_t koff = fixed ? bi * NB : (uint32_t)w * NB;
    const uint32_t val = (fixed ? (uint32_t)((size_t)w * stride + i) : (uint32_t)i) | sign;
    fn(w - w0, koff + k, val);
  }
}


// round 1a: coarse histogram (LDS per block, one global atomic per bin and block)
__global__ void __launch_bounds__(PT)
msm_coarse_hist_kernel(MsmScalarList list, size_t n, int c, int W, uint32_t NB, int fixed, size_t stride, int fb,
                       uint32_t ncoarse, uint32_t* __restrict__ ccount, MsmZero z) {
  __shared__ uint32_t h[COARSE_MAX];
  {  // the pipeline's other per-MSM zeroing (no separate fills)
    const size_t nthr = (size_t)gridDim.x * gridDim.y * gridDim.z * PT;
    const size_t tid = (((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * PT + threadIdx.x;
    for (size_t i = tid; i < z.nb; i += nthr) {
      z.bstart[i] = 0;
      z.bend[i] = 0;
    }
    if (tid < 2) z.counters[tid] = 0;
    if (tid < z.nrd) z.rdone[tid] = 0;
  }
  for (uint32_t t = threadIdx.x; t < ncoarse; t += PT) h[t] = 0;
  __syncthreads();
  const size_t i = blockIdx.x * (size_t)PT + threadIdx.x;
  if (i < n)
    scalar_digits(list, n, c, W, NB, fixed, stride, blockIdx.y, i, blockIdx.z * PWG,
                  [&](int, uint32_t key, uint32_t) { atomicAdd(&h[key >> fb], 1u); });
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < ncoarse; t += PT)
    if (h[t]) atomicAdd(&ccount[t], h[t]);
}

// exclusive scan of cnt[0, len) (one block, len <= 1024 * 64): off[] = cursor[] =
// prefix; *total = sum; clear: cnt[] is zeroed after use (the counts start at zero for
// the next MSM without a fill)
__global__ void __launch_bounds__(1024)
msm_scan_kernel(uint32_t* __restrict__ cnt, uint32_t len, uint32_t* __restrict__ off,
                uint32_t* __restrict__ cursor, uint32_t* __restrict__ total, bool clear) {
  __shared__ uint32_t part[1024];
  const uint32_t per = (len + 1023) / 1024;
  const uint32_t lo = threadIdx.x * per, hi = lo + per < len ? lo + per : len;
  uint32_t s = 0;
  for (uint32_t i = lo; i < hi; i++) s += cnt[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (uint32_t i = lo; i < hi; i++) {
    off[i] = run;
    if (cursor) cursor[i] = run;
    run += cnt[i];
    if (clear) cnt[i] = 0;
  }
  if (threadIdx.x == 1023 && total) *total = part[1023];
}

// large scans (the per-key counts): 1024-element blocks scanned locally, block sums
// scanned by msm_scan_kernel, then added back
__global__ void __launch_bounds__(1024)
msm_scan_block_kernel(uint32_t* __restrict__ cnt, uint32_t len, uint32_t* __restrict__ off,
                      uint32_t* __restrict__ bsum) {
  __shared__ uint32_t part[1024];
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t v0 = i < len ? cnt[i] : 0;
  if (i < len) cnt[i] = 0;  // zero for the next MSM (cnt is read only here)
  part[threadIdx.x] = v0;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint32_t v = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  if (i < len) off[i] = part[threadIdx.x] - v0;
  if (threadIdx.x == 1023) bsum[blockIdx.x] = part[1023];
}
__global__ void __launch_bounds__(1024)
msm_scan_add_kernel(uint32_t* __restrict__ off, uint32_t len, const uint32_t* __restrict__ boff,
                    uint32_t* __restrict__ cursor) {
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  if (i >= len) return;
  const uint32_t v = off[i] + boff[blockIdx.x];
  off[i] = v;
  cursor[i] = v;
}

// round 1b: entries written into their coarse bins (ranks from LDS atomics, one global
// reservation per bin and block)
__global__ void __launch_bounds__(PT)
msm_coarse_scatter_kernel(MsmScalarList list, size_t n, int c, int W, uint32_t NB, int fixed, size_t stride, int fb,
                          uint32_t ncoarse, uint32_t* __restrict__ ccursor, uint64_t* __restrict__ out) {
  __shared__ uint32_t cnt[COARSE_MAX], base[COARSE_MAX];
  for (uint32_t t = threadIdx.x; t < ncoarse; t += PT) cnt[t] = 0;
  __syncthreads();
  uint64_t ent[PWG];
  uint32_t rk[PWG];
#pragma unroll
  for (int k = 0; k < PWG; k++) rk[k] = ~0u;
  const size_t i = blockIdx.x * (size_t)PT + threadIdx.x;
  if (i < n)
    scalar_digits(list, n, c, W, NB, fixed, stride, blockIdx.y, i, blockIdx.z * PWG,
                  [&](int slot, uint32_t key, uint32_t val) {
#pragma unroll
                    for (int k = 0; k < PWG; k++)
                      if (k == slot) {
                        ent[k] = ((uint64_t)key << 32) | val;
                        rk[k] = atomicAdd(&cnt[key >> fb], 1u);
                      }
                  });
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < ncoarse; t += PT)
    if (cnt[t]) base[t] = atomicAdd(&ccursor[t], cnt[t]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PWG; k++)
    if (rk[k] != ~0u) out[base[(uint32_t)(ent[k] >> 32) >> fb] + rk[k]] = ent[k];
}

// round 2a: per-key counts inside coarse bins: tiles of FTILE entries; entries of the
// tile's first bin go through an LDS histogram, others (tiles straddling bins) directly
__global__ void __launch_bounds__(FT)
msm_fine_hist_kernel(const uint64_t* __restrict__ in, const uint32_t* __restrict__ d_total, int fb,
                     uint32_t* __restrict__ kcount) {
  __shared__ uint32_t h[1 << FB_MAX];
  const uint32_t total = *d_total;
  const uint32_t lo = blockIdx.x * FTILE;
  if (lo >= total) return;
  const uint32_t nf = 1u << fb;
  for (uint32_t t = threadIdx.x; t < nf; t += FT) h[t] = 0;
  const uint32_t bin0 = (uint32_t)(in[lo] >> 32) >> fb;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < FPER; k++) {
    const uint32_t p = lo + k * FT + threadIdx.x;
    if (p >= total) break;
    const uint32_t key = (uint32_t)(in[p] >> 32);
    if ((key >> fb) == bin0) atomicAdd(&h[key & (nf - 1)], 1u);
    else atomicAdd(&kcount[key], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nf; t += FT)
    if (h[t]) atomicAdd(&kcount[(bin0 << fb) + t], h[t]);
}

// round 2b: the same tiles scattered to their keys' positions
__global__ void __launch_bounds__(FT)
msm_fine_scatter_kernel(const uint64_t* __restrict__ in, const uint32_t* __restrict__ d_total, int fb,
                        uint32_t* __restrict__ kcursor, uint64_t* __restrict__ out) {
  __shared__ uint32_t cnt[1 << FB_MAX], base[1 << FB_MAX];
  const uint32_t total = *d_total;
  const uint32_t lo = blockIdx.x * FTILE;
  if (lo >= total) return;
  const uint32_t nf = 1u << fb;
  for (uint32_t t = threadIdx.x; t < nf; t += FT) cnt[t] = 0;
  const uint32_t bin0 = (uint32_t)(in[lo] >> 32) >> fb;
  __syncthreads();
  uint64_t ent[FPER];
  uint32_t rk[FPER];
#pragma unroll
  for (int k = 0; k < FPER; k++) {
    const uint32_t p = lo + k * FT + threadIdx.x;
    rk[k] = ~0u;
    ent[k] = 0;
    if (p < total) {
      ent[k] = in[p];
      const uint32_t key = (uint32_t)(ent[k] >> 32);
      if ((key >> fb) == bin0) rk[k] = atomicAdd(&cnt[key & (nf - 1)], 1u);
      else out[atomicAdd(&kcursor[key], 1u)] = ent[k];
    }
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nf; t += FT)
    if (cnt[t]) base[t] = atomicAdd(&kcursor[(bin0 << fb) + t], cnt[t]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < FPER; k++)
    if (rk[k] != ~0u) out[base[(uint32_t)(ent[k] >> 32) & (nf - 1)] + rk[k]] = ent[k];
}

// round 2, staged form: tiles of SW_T threads x SW_PER entries (8192) whose keys inside a
// local window of SW_LK keys (the tile's first coarse bin and the next) are counted and
// ranked in LDS, reserved with one global atomic per (tile, key), then written through an
// LDS copy of the tile in key order -- so a wave's stores are runs of each key's share of
// the tile (~8 entries at 10 fine bits) instead of 64 scattered 8-B writes, and the per-key
// global atomics drop 4x with the larger tile.  Keys outside the window (tiles straddling
// more than two bins: small bins) take a global atomic each, as in the unstaged kernels.
static constexpr int SW_T = 512;
static constexpr int SW_PER = 16;
static constexpr uint32_t SW_TILE = (uint32_t)SW_T * SW_PER;
static constexpr uint32_t SW_LK = 2048;

// exclusive block scan of one value per thread (TPB threads); *total = the block's sum
template <int TPB>
__device__ __forceinline__ uint32_t sw_block_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int q = 0; q < TPB / 64; q++) {
    const uint32_t s = wsum[q];
    if (q < (int)wv) before += s;
    all += s;
  }
  *total = all;
  return before + x - v;
}

__global__ void __launch_bounds__(SW_T)
msm_fine_hist_staged_kernel(const uint64_t* __restrict__ in, const uint32_t* __restrict__ d_total, int fb,
                            uint32_t* __restrict__ kcount) {
  __shared__ uint32_t h[SW_LK];
  const uint32_t total = *d_total;
  const uint32_t lo = blockIdx.x * SW_TILE;
  if (lo >= total) return;
  const uint32_t kbase = ((uint32_t)(in[lo] >> 32) >> fb) << fb;
  for (uint32_t t = threadIdx.x; t < SW_LK; t += SW_T) h[t] = 0;
  __syncthreads();
#pragma unroll 4
  for (int k = 0; k < SW_PER; k++) {
    const uint32_t p = lo + k * SW_T + threadIdx.x;
    if (p >= total) break;
    const uint32_t key = (uint32_t)(in[p] >> 32);
    if (key - kbase < SW_LK) atomicAdd(&h[key - kbase], 1u);
    else atomicAdd(&kcount[key], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < SW_LK; t += SW_T)
    if (h[t]) atomicAdd(&kcount[kbase + t], h[t]);
}

__global__ void __launch_bounds__(SW_T)
msm_fine_scatter_staged_kernel(const uint64_t* __restrict__ in, const uint32_t* __restrict__ d_total, int fb,
                               uint32_t* __restrict__ kcursor, uint64_t* __restrict__ out) {
  __shared__ uint64_t stage[SW_TILE];
  __shared__ uint32_t cnt[SW_LK], loff[SW_LK], gb[SW_LK];
  __shared__ uint32_t wsum[SW_T / 64];
  const uint32_t total = *d_total;
  const uint32_t lo = blockIdx.x * SW_TILE;
  if (lo >= total) return;
  const uint32_t kbase = ((uint32_t)(in[lo] >> 32) >> fb) << fb;
  for (uint32_t t = threadIdx.x; t < SW_LK; t += SW_T) cnt[t] = 0;
  __syncthreads();
  uint64_t ent[SW_PER];
  uint32_t rk[SW_PER];
#pragma unroll
  for (int k = 0; k < SW_PER; k++) {
    const uint32_t p = lo + k * SW_T + threadIdx.x;
    rk[k] = ~0u;
    ent[k] = 0;
    if (p < total) {
      ent[k] = in[p];
      const uint32_t key = (uint32_t)(ent[k] >> 32);
      if (key - kbase < SW_LK) rk[k] = atomicAdd(&cnt[key - kbase], 1u);
      else out[atomicAdd(&kcursor[key], 1u)] = ent[k];
    }
  }
  __syncthreads();
  // per-key tile offsets (each thread scans SW_LK / SW_T consecutive keys) and the global
  // reservations
  constexpr uint32_t KPT = SW_LK / SW_T;
  const uint32_t k0 = threadIdx.x * KPT;
  uint32_t c[KPT], s = 0;
#pragma unroll
  for (uint32_t i = 0; i < KPT; i++) {
    c[i] = cnt[k0 + i];
    s += c[i];
  }
  uint32_t m;
  uint32_t run = sw_block_scan<SW_T>(s, wsum, &m);
#pragma unroll
  for (uint32_t i = 0; i < KPT; i++) {
    loff[k0 + i] = run;
    run += c[i];
    if (c[i]) gb[k0 + i] = atomicAdd(&kcursor[kbase + k0 + i], c[i]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SW_PER; k++)
    if (rk[k] != ~0u) stage[loff[(uint32_t)(ent[k] >> 32) - kbase] + rk[k]] = ent[k];
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < m; j += SW_T) {
    const uint64_t e = stage[j];
    const uint32_t kk = (uint32_t)(e >> 32) - kbase;
    out[gb[kk] + (j - loff[kk])] = e;
  }
}

hipError_t msm_partition(const MsmPartArgs& a, hipStream_t st, MsmPhaseEvents* prof) {
  // staged fine pass below 2^25 entries (MSMs up to 2^21 points: fine pass 0.108 -> 0.084 ms
  // at 2^19, 0.356 -> 0.30 ms at 2^21); at 2^22 (54.5 M entries) it is no faster (0.61 vs
  // 0.60 ms).  H2G_MSM_FSTAGE=0 / 1 forces it (A/B).
  static const int fstage_env = [] {
    const char* e = getenv("H2G_MSM_FSTAGE");
    return e ? atoi(e) : -1;
  }();
  const bool fstage = fstage_env >= 0 ? fstage_env != 0 : a.total < (1ull << 25);
  {  // round 1: coarse bins straight from the scalars
    const dim3 g((unsigned)((a.n + PT - 1) / PT), (unsigned)a.nbatch, (unsigned)((a.W + PWG - 1) / PWG));
    hipLaunchKernelGGL(msm_coarse_hist_kernel, g, dim3(PT), 0, st, a.list, a.n, a.c, a.W, a.NB, a.fixed, a.stride,
                       a.fb, a.ncoarse, a.ccount, a.z);
    hipLaunchKernelGGL(msm_scan_kernel, dim3(1), dim3(1024), 0, st, a.ccount, a.ncoarse, a.coff, a.ccursor,
                       a.d_total, true);
    hipLaunchKernelGGL(msm_coarse_scatter_kernel, g, dim3(PT), 0, st, a.list, a.n, a.c, a.W, a.NB, a.fixed, a.stride,
                       a.fb, a.ncoarse, a.ccursor, a.keys_in);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (prof) {
    hipError_t e = hipEventRecord(prof->ev[1], st);
    if (e == hipSuccess && prof->entries) e = hipMemcpyAsync(prof->entries, a.d_total, 4, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return e;
  }
  {  // round 2: keys inside the coarse bins
    const unsigned tiles = (unsigned)((a.total + FTILE - 1) / FTILE);
    const unsigned stiles = (unsigned)((a.total + SW_TILE - 1) / SW_TILE);
    if (fstage)
      hipLaunchKernelGGL(msm_fine_hist_staged_kernel, dim3(stiles), dim3(SW_T), 0, st, (const uint64_t*)a.keys_in,
                         (const uint32_t*)a.d_total, a.fb, a.kcount);
    else
      hipLaunchKernelGGL(msm_fine_hist_kernel, dim3(tiles), dim3(FT), 0, st, (const uint64_t*)a.keys_in,
                         (const uint32_t*)a.d_total, a.fb, a.kcount);
    hipLaunchKernelGGL(msm_scan_block_kernel, dim3(a.kblocks), dim3(1024), 0, st, a.kcount, a.nbt, a.koff, a.kbsum);
    hipLaunchKernelGGL(msm_scan_kernel, dim3(1), dim3(1024), 0, st, a.kbsum, a.kblocks, a.kboff, (uint32_t*)nullptr,
                       (uint32_t*)nullptr, false);
    hipLaunchKernelGGL(msm_scan_add_kernel, dim3(a.kblocks), dim3(1024), 0, st, a.koff, a.nbt,
                       (const uint32_t*)a.kboff, a.kcursor);
    if (fstage)
      hipLaunchKernelGGL(msm_fine_scatter_staged_kernel, dim3(stiles), dim3(SW_T), 0, st, (const uint64_t*)a.keys_in,
                         (const uint32_t*)a.d_total, a.fb, a.kcursor, a.keys_out);
    else
      hipLaunchKernelGGL(msm_fine_scatter_kernel, dim3(tiles), dim3(FT), 0, st, (const uint64_t*)a.keys_in,
                         (const uint32_t*)a.d_total, a.fb, a.kcursor, a.keys_out);
  }
  return hipGetLastError();
}

}  // namespace h2g
