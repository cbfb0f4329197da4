// msm_part.h -- the MSM pipeline's stages in their own translation units (the bucket
// partition, msm_part.hip; the accumulation, msm_acc.hip), shared with msm.hip.
#pragma once
#include <algorithm>
#include "msm.h"
#include "f29.h"

namespace h2g {

static constexpr int FB_MAX = 11;        // fine bits (keys per coarse bin <= 2^FB_MAX)
static constexpr int COARSE_MAX = 2048;  // coarse bins

// Wave priorities (s_setprio) of the MSM's short phases.  Inside a proof the two MSM
// streams overlap: one MSM's partition, fixup and reduction share the SIMDs with the
// other's accumulation, a VALU-bound kernel that keeps every SIMD's issue port busy.  The
// reduction and fixup are latency-bound chains (one wave per SIMD, dependent point
// additions) and the partition waits on memory; raised priority lets their few
// instructions issue first while the accumulation's waves fill the remaining cycles.
#ifndef H2G_PRIO_RED
#define H2G_PRIO_RED 3
#endif
#ifndef H2G_PRIO_PART
#define H2G_PRIO_PART 2
#endif
#define H2G_SETPRIO(p) \
  do {                  \
    if ((p) > 0) __builtin_amdgcn_s_setprio(p); \
  } while (0)

// Fixed-base windows have balanced widths: W = ceil(255 / c) windows covering the 255
// bits signed digits need, the first 255 % W of them one bit wider (<= c).  Uniform
// c-bit windows leave a short top window (255 - c (W - 1) bits: 7 at c = 19, W = 14)
// whose digits pile n entries into a few buckets -- the big-bucket path, ~0.2-0.5 ms.
__host__ __device__ __forceinline__ int fb_width(int W, int w) { return 255 / W + (w < 255 % W ? 1 : 0); }

// zeroed by the coarse histogram kernel for the later phases: the big-item counters, the
// plane reduction's finished-block counts
struct MsmZero {
  uint32_t* counters;
  uint32_t* rdone;
  uint32_t nrd;
};

// The accumulation's chunk length L (entries per thread).  The host picks it from the
// entry bound n W nbatch (msm_chunk_len); the entries that exist are known only on the
// device, after the partition, and small or sparse scalars leave far fewer: a batch of
// 4-bit witness columns fills one window of 15 (1/15 of the bound), the lookup columns'
// prefix-basis differences a few hundred entries per column.  With the host's L those
// MSMs ran on a few waves per chip, each a long dependent chain of mixed additions
// (keccak-style k = 18: 1.1-1.4 ms accumulations of 0.1-8 M entries).  So once the count
// is known the partition's last scan picks L again (msm_chunk_len_dev): the host's L when
// at least half the bound exists (dense scalars: unchanged), otherwise enough chunks for
// 2^18 threads (4 waves per SIMD), never below 8 or above the host's L.  Every later
// kernel reads L from d_total[1]; grids and boundary slots are sized for the most chunks
// either choice can make (msm_chunk_cap).
struct MsmChunkRule {
  uint32_t Lh;      // the host's chunk length
  uint32_t adapt;   // 0: keep Lh (an explicit item_len)
  uint64_t bound;   // entry bound n W nbatch
  uint64_t nb_eff;  // buckets the windows can reach (the host rule's quarter-bucket floor)
};
static constexpr int MSM_ADAPT_LG = 18;  // threads the device choice aims for (2^18)
__host__ __device__ __forceinline__ uint32_t msm_chunk_len_dev(uint64_t actual, const MsmChunkRule& r) {
  if (!r.adapt || 2 * actual > r.bound) return r.Lh;
  uint64_t L = actual >> MSM_ADAPT_LG;
  const uint64_t quarter = r.nb_eff ? actual / (4 * r.nb_eff) : 0;
  if (L < quarter) L = quarter;
  if (L < 8) L = 8;
  if (L > r.Lh) L = r.Lh;
  return (uint32_t)L;
}
// the most chunks msm_chunk_len_dev can make: the host's count, or ceil(a / L) with
// L >= max(8, a >> 18), below 2^18 (1 + 1/8) + 1
__host__ __forceinline__ size_t msm_chunk_cap(const MsmChunkRule& r) {
  const size_t host = (size_t)((r.bound + r.Lh - 1) / r.Lh);
  if (!r.adapt) return host;
  const size_t dev = (size_t)std::min<uint64_t>((r.bound + 7) / 8, ((1ull << MSM_ADAPT_LG) * 9) / 8 + 1);
  return host > dev ? host : dev;
}

// One partition of the MSM pipeline's entries: round 1 (coarse bins straight from the
// scalars, into ent), phase event 1, round 2 (keys inside the bins: the values in bucket
// order into out, koff[k] = the first position of key k's run, koff[nbt] = the entry
// count).  The scratch arrays are msm_pipeline's (zero counts on entry, left zero).
struct MsmPartArgs {
  MsmScalarList list;
  int nbatch;
  size_t n;
  int c, W;
  uint32_t NB;
  int fixed;
  size_t stride;
  size_t total;  // upper bound of the entries (n W nbatch)
  int fb;
  uint32_t ncoarse, nbt, kblocks;
  uint32_t *ccount, *coff, *ccursor, *d_total, *kbsum, *kboff, *kcount, *koff, *kcursor;
  uint64_t* ent;
  uint32_t* out;
  MsmZero z;
  MsmChunkRule rule;  // d_total[1] = the accumulation's chunk length
};
hipError_t msm_partition(const MsmPartArgs& a, hipStream_t st, MsmPhaseEvents* prof);

// The accumulation's arithmetic: 1 = F29 (f29.h: 9 x 29-bit limbs, no carry ops in the
// products); its buckets and boundary slots are then raw G1xyzz29 accumulators (144 B),
// converted to canonical G1xyzz by the fixup.  0 = the 8 x 32-bit FIPS arithmetic of
// bn254.h writing G1xyzz directly (A/B builds: tools/build_variant.py TAG --src
// msm_acc.hip,msm.hip -DH2G_ACC29=0).
#ifndef H2G_ACC29
#define H2G_ACC29 1
#endif
#if H2G_ACC29
using AccPoint = G1xyzz29;
using RedPoint = G1xyzz29;  // the fixup's and the reduction's points (f29.h's back-end class)
#else
using AccPoint = G1xyzz;
using RedPoint = G1xyzz;
#endif

// raw 16-B moves of the accumulators (G1xyzz29 is 9 x 16 B)
__device__ __forceinline__ void st_acc(G1xyzz29* dst, const G1xyzz29& v) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = make_uint4(s[4 * i], s[4 * i + 1], s[4 * i + 2], s[4 * i + 3]);
}
__device__ __forceinline__ G1xyzz29 ld_acc(const G1xyzz29* src) {
  G1xyzz29 v;
  uint32_t* d = reinterpret_cast<uint32_t*>(&v);
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint4 q = s[i];
    d[4 * i] = q.x;
    d[4 * i + 1] = q.y;
    d[4 * i + 2] = q.z;
    d[4 * i + 3] = q.w;
  }
  return v;
}
__device__ __forceinline__ G1xyzz acc_to_xyzz(const G1xyzz29& v) { return xyzz_from29(v); }
__device__ __forceinline__ G1xyzz acc_to_xyzz(const G1xyzz& v) { return v; }
__device__ __forceinline__ AccPoint ld_accp(const AccPoint* p) {
#if H2G_ACC29
  return ld_acc(p);
#else
  return *p;
#endif
}

// step 3 of the pipeline (msm_acc.hip): XYZZ accumulation of the bucket-sorted values in
// chunks of L = d_total[1] (d_total[0]: the entries), one thread per chunk (a grid for
// nchunks_cap); bucket k's run is [koff[k], koff[k + 1]).  Whole buckets
// go to buckets[k], runs crossing a chunk boundary to the chunk's slots bnd[2 t + 0/1].
// rep (1 + MSM_REPAIR_CAP words, rep[0] zeroed by the partition): the chunks whose mixed
// additions met p == q, redone by a second launch with the doubling branch
static constexpr uint32_t MSM_REPAIR_CAP = 4096;
static constexpr int MSM_REPAIR_BLOCKS = 64;
hipError_t msm_accumulate(const G1Affine* bases, const uint32_t* vals, const uint32_t* koff, uint32_t nbt,
                          const uint32_t* d_total, size_t nchunks_cap, AccPoint* buckets, AccPoint* bnd,
                          uint32_t* rep, hipStream_t st);

}  // namespace h2g
