// msm_part.h -- the MSM pipeline's stages in their own translation units (the bucket
// partition, msm_part.hip; the accumulation, msm_acc.hip), shared with msm.hip.
#pragma once
#include "msm.h"

namespace h2g {

static constexpr int FB_MAX = 11;        // fine bits
static constexpr int COARSE_MAX = 2048;  // coarse bins (keys < 2^22)

// Fixed-base windows have balanced widths: W = ceil(255 / c) windows covering the 255
// bits signed digits need, the first 255 % W of them one bit wider (<= c).  Uniform
// c-bit windows leave a short top window (255 - c (W - 1) bits: 7 at c = 19, W = 14)
// whose digits pile n entries into a few buckets -- the big-bucket path, ~0.2-0.5 ms.
__host__ __device__ __forceinline__ int fb_width(int W, int w) { return 255 / W + (w < 255 % W ? 1 : 0); }

// zeroed by the coarse histogram kernel for the later phases: bucket [start, end) (empty
// buckets keep 0, 0), the big-item counters, the plane reduction's finished-block counts
struct MsmZero {
  uint32_t* bstart;
  uint32_t* bend;
  size_t nb;
  uint32_t* counters;
  uint32_t* rdone;
  uint32_t nrd;
};

// One partition of the MSM pipeline's entries: round 1 (coarse bins straight from the
// scalars, into keys_in), phase event 1, round 2 (keys inside the bins, into keys_out).
// The scratch arrays are msm_pipeline's (zero counts on entry, left zero).
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
  uint64_t *keys_in, *keys_out;
  MsmZero z;
};
hipError_t msm_partition(const MsmPartArgs& a, hipStream_t st, MsmPhaseEvents* prof);

// step 3 of the pipeline (msm_acc.hip): XYZZ accumulation of the bucket-sorted entries in
// chunks of L, one thread per chunk
hipError_t msm_accumulate(const G1Affine* bases, const uint64_t* ent, const uint32_t* d_total, uint32_t sentinel,
                          uint32_t L, size_t nchunks, G1xyzz* buckets, G1xyzz* bnd, uint32_t* bstart, uint32_t* bend,
                          hipStream_t st);

}  // namespace h2g
