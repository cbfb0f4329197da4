// msm_part.hip -- the bucket partition of the MSM pipeline (msm.hip step 2) for gfx950:
// signed digits straight from the scalars into coarse bins, then keys inside the bins.
// Its own translation unit: none of it is elliptic-curve arithmetic, so it builds in
// seconds while msm.hip's point kernels take minutes.
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
// counting partition replaces a sort.  Round 1 splits by the key's high bits (coarse
// bins) straight from the scalars (u64 entries, key << 32 | value), round 2 by the low
// fb bits inside each coarse bin, in tiles of FTILE entries; it writes only the u32
// values, bucket k being [koff[k], koff[k + 1]) of them.  Round 2's tiles are ordered so
// that each XCD takes a contiguous range of them (workgroups go round-robin over the 8
// XCDs): a bin's scattered writes then come from one XCD's L2, where the partial lines
// merge.  (One workgroup per coarse bin instead -- LDS histogram, no global atomics --
// measured slower, 0.82 vs 0.58 ms at 2^22, and its long-lived 1024-thread workgroups
// starved the other MSM stream's accumulation inside the proof: 107 vs 90 ms.)  Zero
// digits produce no entry.  Order inside a bucket is arbitrary (the sum is exact).
static constexpr int PT = 512;     // threads of the coarse kernels (one scalar each)
static constexpr int PWG = 16;     // windows per coarse-kernel thread (grid.z groups)
static constexpr int FT = 256;     // threads of the fine kernels
static constexpr int FPER = 8;     // entries per fine-kernel thread: 8 (2048-entry tiles) measured best at 10 fine bits
static constexpr uint32_t FTILE = (uint32_t)FT * FPER;

// the signed digits of scalar i (batch bi) for windows [w0, w0 + PWG): fn(slot, key, val)
// for each nonzero digit; fixed-base windows take their balanced widths (fb_width),
// generic ones c bits each
template <class Fn>
__device__ __forceinline__ void scalar_digits(const MsmScalarList& list, int c, int W, uint32_t NB, int fixed,
                                              size_t stride, uint32_t bi, size_t i, int w0, Fn fn) {
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
    const uint32_t koff = fixed ? bi * NB : (uint32_t)w * NB;
    const uint32_t val = (fixed ? (uint32_t)((size_t)w * stride + i) : (uint32_t)i) | sign;
    fn(w - w0, koff + mag - 1, val);
  }
}

// round 1a: coarse histogram (LDS per block, one global atomic per bin and block)
__global__ void __launch_bounds__(PT)
msm_coarse_hist_kernel(MsmScalarList list, size_t n, int c, int W, uint32_t NB, int fixed, size_t stride, int fb,
                       uint32_t ncoarse, uint32_t* __restrict__ ccount, MsmZero z) {
  H2G_SETPRIO(H2G_PRIO_PART);
  __shared__ uint32_t h[COARSE_MAX];
  {  // the pipeline's other per-MSM zeroing (no separate fills)
    const size_t tid = (((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * PT + threadIdx.x;
    if (tid < 2) z.counters[tid] = 0;
    if (tid == 2) z.counters[4] = 0;  // the accumulation's repair count (msm_accumulate)
    if (tid < z.nrd) z.rdone[tid] = 0;
  }
  for (uint32_t t = threadIdx.x; t < ncoarse; t += PT) h[t] = 0;
  __syncthreads();
  const size_t i = blockIdx.x * (size_t)PT + threadIdx.x;
  if (i < n)
    scalar_digits(list, c, W, NB, fixed, stride, blockIdx.y, i, blockIdx.z * PWG,
                  [&](int, uint32_t key, uint32_t) { atomicAdd(&h[key >> fb], 1u); });
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < ncoarse; t += PT)
    if (h[t]) atomicAdd(&ccount[t], h[t]);
}

// exclusive scan of cnt[0, len) (one block, len <= 1024 * 64): off[] (and cursor[] if
// given) = prefix; *total = sum; clear: cnt[] is zeroed after use (the counts start at
// zero for the next MSM without a fill)
__global__ void __launch_bounds__(1024)
msm_scan_kernel(uint32_t* __restrict__ cnt, uint32_t len, uint32_t* __restrict__ off,
                uint32_t* __restrict__ cursor, uint32_t* __restrict__ total, bool clear) {
  H2G_SETPRIO(H2G_PRIO_PART);
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
  H2G_SETPRIO(H2G_PRIO_PART);
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
// off[i] += block offset (= koff, the first position of key i's run), cursor = the same;
// off[len] = the entry count, d_total[1] = the accumulation's chunk length (msm_chunk_len_dev)
__global__ void __launch_bounds__(1024)
msm_scan_add_kernel(uint32_t* __restrict__ off, uint32_t len, const uint32_t* __restrict__ boff,
                    uint32_t* __restrict__ cursor, uint32_t* __restrict__ d_total, MsmChunkRule rule) {
  H2G_SETPRIO(H2G_PRIO_PART);
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  if (i == 0) {
    const uint32_t tot = d_total[0];
    off[len] = tot;
    d_total[1] = msm_chunk_len_dev(tot, rule);
  }
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
  H2G_SETPRIO(H2G_PRIO_PART);
  __shared__ uint32_t cnt[COARSE_MAX], base[COARSE_MAX];
  for (uint32_t t = threadIdx.x; t < ncoarse; t += PT) cnt[t] = 0;
  __syncthreads();
  uint64_t ent[PWG];
  uint32_t rk[PWG];
#pragma unroll
  for (int k = 0; k < PWG; k++) rk[k] = ~0u;
  const size_t i = blockIdx.x * (size_t)PT + threadIdx.x;
  if (i < n)
    scalar_digits(list, c, W, NB, fixed, stride, blockIdx.y, i, blockIdx.z * PWG,
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

// round 2's tile of block b: XCD x (= b mod 8, workgroups dispatch round-robin over the
// XCDs) takes tiles [x T / 8, (x + 1) T / 8) in order, so a coarse bin's tiles -- and its
// scattered output writes -- stay on one XCD
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t T) {
  const uint32_t x = b & 7, q = b >> 3;
  const uint32_t per = T >> 3, extra = T & 7;  // XCDs x < extra take per + 1 tiles
  return x * per + (x < extra ? x : extra) + q;
}

// round 2a: per-key counts inside coarse bins: tiles of FTILE entries; entries of the
// tile's first bin go through an LDS histogram, others (tiles straddling bins) directly
__global__ void __launch_bounds__(FT)
msm_fine_hist_kernel(const uint64_t* __restrict__ in, const uint32_t* __restrict__ d_total, int fb, uint32_t tiles,
                     uint32_t* __restrict__ kcount) {
  H2G_SETPRIO(H2G_PRIO_PART);
  __shared__ uint32_t h[1 << FB_MAX];
  const uint32_t total = *d_total;
  const uint32_t lo = xcd_tile(blockIdx.x, tiles) * FTILE;
  if (lo >= total) return;
  const uint32_t* key32 = reinterpret_cast<const uint32_t*>(in) + 1;  // the keys (high words)
  const uint32_t nf = 1u << fb;
  for (uint32_t t = threadIdx.x; t < nf; t += FT) h[t] = 0;
  const uint32_t bin0 = key32[2 * (size_t)lo] >> fb;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < FPER; k++) {
    const uint32_t p = lo + k * FT + threadIdx.x;
    if (p >= total) break;
    const uint32_t key = key32[2 * (size_t)p];
    if ((key >> fb) == bin0) atomicAdd(&h[key & (nf - 1)], 1u);
    else atomicAdd(&kcount[key], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nf; t += FT)
    if (h[t]) atomicAdd(&kcount[(bin0 << fb) + t], h[t]);
}

// round 2b: the same tiles scattered to their keys' positions (values only)
__global__ void __launch_bounds__(FT)
msm_fine_scatter_kernel(const uint64_t* __restrict__ in, const uint32_t* __restrict__ d_total, int fb,
                        uint32_t tiles, uint32_t* __restrict__ kcursor, uint32_t* __restrict__ out) {
  H2G_SETPRIO(H2G_PRIO_PART);
  __shared__ uint32_t cnt[1 << FB_MAX], base[1 << FB_MAX];
  const uint32_t total = *d_total;
  const uint32_t lo = xcd_tile(blockIdx.x, tiles) * FTILE;
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
      else out[atomicAdd(&kcursor[key], 1u)] = (uint32_t)ent[k];
    }
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nf; t += FT)
    if (cnt[t]) base[t] = atomicAdd(&kcursor[(bin0 << fb) + t], cnt[t]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < FPER; k++)
    if (rk[k] != ~0u) out[base[(uint32_t)(ent[k] >> 32) & (nf - 1)] + rk[k]] = (uint32_t)ent[k];
}

// round 2, staged form (MSMs below 2^25 entries, the slabs of sharded proofs: 2^19
// points 0.108 -> 0.084 ms, 2^21 0.356 -> 0.30 ms; at 2^22 no faster, 0.61 vs 0.60 ms):
// tiles of SW_T threads x SW_PER entries (8192) whose keys inside a local window of SW_LK
// keys (the tile's first coarse bin and the next) are counted and ranked in LDS, reserved
// with one global atomic per (tile, key), then written through an LDS copy of the tile in
// key order -- a wave's stores are runs of each key's share of the tile instead of 64
// scattered writes, and the per-key global atomics drop 4x with the larger tile.  Keys
// outside the window (tiles straddling more than two bins) take a global atomic each.
#ifndef H2G_FSTAGE_MAX
#define H2G_FSTAGE_MAX (1ull << 25)
#endif
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
                            uint32_t tiles, uint32_t* __restrict__ kcount) {
  H2G_SETPRIO(H2G_PRIO_PART);
  __shared__ uint32_t h[SW_LK];
  const uint32_t total = *d_total;
  const uint32_t lo = xcd_tile(blockIdx.x, tiles) * SW_TILE;
  if (lo >= total) return;
  const uint32_t* key32 = reinterpret_cast<const uint32_t*>(in) + 1;
  const uint32_t kbase = (key32[2 * (size_t)lo] >> fb) << fb;
  for (uint32_t t = threadIdx.x; t < SW_LK; t += SW_T) h[t] = 0;
  __syncthreads();
#pragma unroll 4
  for (int k = 0; k < SW_PER; k++) {
    const uint32_t p = lo + k * SW_T + threadIdx.x;
    if (p >= total) break;
    const uint32_t key = key32[2 * (size_t)p];
    if (key - kbase < SW_LK) atomicAdd(&h[key - kbase], 1u);
    else atomicAdd(&kcount[key], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < SW_LK; t += SW_T)
    if (h[t]) atomicAdd(&kcount[kbase + t], h[t]);
}

__global__ void __launch_bounds__(SW_T)
msm_fine_scatter_staged_kernel(const uint64_t* __restrict__ in, const uint32_t* __restrict__ d_total, int fb,
                               uint32_t tiles, uint32_t* __restrict__ kcursor, uint32_t* __restrict__ out) {
  H2G_SETPRIO(H2G_PRIO_PART);
  __shared__ uint64_t stage[SW_TILE];
  __shared__ uint32_t cnt[SW_LK], loff[SW_LK], gb[SW_LK];
  __shared__ uint32_t wsum[SW_T / 64];
  const uint32_t total = *d_total;
  const uint32_t lo = xcd_tile(blockIdx.x, tiles) * SW_TILE;
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
      else out[atomicAdd(&kcursor[key], 1u)] = (uint32_t)ent[k];
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
    out[gb[kk] + (j - loff[kk])] = (uint32_t)e;
  }
}

hipError_t msm_partition(const MsmPartArgs& a, hipStream_t st, MsmPhaseEvents* prof) {
  const bool fstage = a.total < (uint64_t)H2G_FSTAGE_MAX;  // the staged fine pass (above)
  {  // round 1: coarse bins straight from the scalars
    const dim3 g((unsigned)((a.n + PT - 1) / PT), (unsigned)a.nbatch, (unsigned)((a.W + PWG - 1) / PWG));
    hipLaunchKernelGGL(msm_coarse_hist_kernel, g, dim3(PT), 0, st, a.list, a.n, a.c, a.W, a.NB, a.fixed, a.stride,
                       a.fb, a.ncoarse, a.ccount, a.z);
    hipLaunchKernelGGL(msm_scan_kernel, dim3(1), dim3(1024), 0, st, a.ccount, a.ncoarse, a.coff, a.ccursor,
                       a.d_total, true);
    hipLaunchKernelGGL(msm_coarse_scatter_kernel, g, dim3(PT), 0, st, a.list, a.n, a.c, a.W, a.NB, a.fixed, a.stride,
                       a.fb, a.ncoarse, a.ccursor, a.ent);
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
      hipLaunchKernelGGL(msm_fine_hist_staged_kernel, dim3(stiles), dim3(SW_T), 0, st, (const uint64_t*)a.ent,
                         (const uint32_t*)a.d_total, a.fb, stiles, a.kcount);
    else
      hipLaunchKernelGGL(msm_fine_hist_kernel, dim3(tiles), dim3(FT), 0, st, (const uint64_t*)a.ent,
                         (const uint32_t*)a.d_total, a.fb, tiles, a.kcount);
    hipLaunchKernelGGL(msm_scan_block_kernel, dim3(a.kblocks), dim3(1024), 0, st, a.kcount, a.nbt, a.koff, a.kbsum);
    hipLaunchKernelGGL(msm_scan_kernel, dim3(1), dim3(1024), 0, st, a.kbsum, a.kblocks, a.kboff, (uint32_t*)nullptr,
                       (uint32_t*)nullptr, false);
    hipLaunchKernelGGL(msm_scan_add_kernel, dim3(a.kblocks), dim3(1024), 0, st, a.koff, a.nbt,
                       (const uint32_t*)a.kboff, a.kcursor, a.d_total, a.rule);
    if (fstage)
      hipLaunchKernelGGL(msm_fine_scatter_staged_kernel, dim3(stiles), dim3(SW_T), 0, st, (const uint64_t*)a.ent,
                         (const uint32_t*)a.d_total, a.fb, stiles, a.kcursor, a.out);
    else
      hipLaunchKernelGGL(msm_fine_scatter_kernel, dim3(tiles), dim3(FT), 0, st, (const uint64_t*)a.ent,
                         (const uint32_t*)a.d_total, a.fb, tiles, a.kcursor, a.out);
  }
  return hipGetLastError();
}

}  // namespace h2g
