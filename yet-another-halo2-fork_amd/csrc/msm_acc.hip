// msm_acc.hip -- step 3 of the MSM pipeline (msm.hip) for gfx950: the bucket accumulation,
// the dominant kernel of create_proof.  Its own translation unit so that A/B builds of it
// (tools/build_variant.py) recompile one kernel, not the reduction's dozen.
#include "msm_part.h"

namespace h2g {

static constexpr int MSM_THREADS = 256;

__device__ __forceinline__ G1Affine ld_aff(const G1Affine* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1], c = q[2], d = q[3];
  G1Affine r;
  r.x.l[0] = a.x; r.x.l[1] = a.y; r.x.l[2] = a.z; r.x.l[3] = a.w;
  r.x.l[4] = b.x; r.x.l[5] = b.y; r.x.l[6] = b.z; r.x.l[7] = b.w;
  r.y.l[0] = c.x; r.y.l[1] = c.y; r.y.l[2] = c.z; r.y.l[3] = c.w;
  r.y.l[4] = d.x; r.y.l[5] = d.y; r.y.l[6] = d.z; r.y.l[7] = d.w;
  return r;
}

// 3-4. accumulation straight from the bucket-sorted values ---------------------------
// The sorted array is cut into chunks of L entries, one thread per chunk.  Bucket k
// occupies [koff[k], koff[k + 1]); a chunk finds the bucket of its first entry by binary
// search over koff (~19 L2-resident loads, ~1 % of a chunk's time) and walks the later run
// ends from there.  A chunk's run of one bucket
// is the whole bucket iff the bucket starts and ends inside the chunk: such buckets are
// written directly, a run that crosses a chunk boundary goes to the chunk's boundary
// slot (slot 0 = its first run, slot 1 = its last run) for the fixup.
// H2G_ACC29: the accumulator is F29 (f29.h) and is stored raw -- a run end is a handful of
// stores, not a conversion: some lane of a wave ends a run on most steps, so anything
// costlier there would be paid by the whole wave nearly every step.
__device__ __forceinline__ void msm_emit(uint32_t key, const AccPoint& acc, bool first, bool from_prev, bool to_next,
                                         uint32_t t, AccPoint* __restrict__ buckets, AccPoint* __restrict__ bnd) {
  AccPoint* dst = (!from_prev && !to_next) ? buckets + key : bnd + 2 * (size_t)t + (first ? 0 : 1);
#if H2G_ACC29
  st_acc(dst, acc);
#else
  *dst = xyzz_canon2(acc);  // lazy [0, 2M) -> fully reduced for the later kernels
#endif
}

__device__ __forceinline__ AccPoint acc_identity() {
#if H2G_ACC29
  return xyzz29_identity();
#else
  return G1xyzz::identity();
#endif
}
template <bool SAFE>
__device__ __forceinline__ AccPoint acc_madd(const AccPoint& acc, const G1Affine& pt, bool* dbl) {
#if H2G_ACC29
  if (pt.is_identity()) return acc;
  return xyzz29_madd<SAFE>(acc, to29(pt.x), to29(pt.y), dbl);
#else
  (void)dbl;
  return xyzz_madd_lazy(acc, pt);
#endif
}

// one chunk [t L, t L + L) of the sorted values: the runs it holds to their buckets or to
// its boundary slots.  SAFE = false: the mixed addition without its doubling branch (the
// hot loop at 4 waves per SIMD); returns true when a run met p == q, and the chunk must be
// redone with SAFE = true -- its writes go to the same places, every one of them rewritten.
// The next entry's base point is loaded before the current mixed addition (software-
// pipelined gather), so its latency hides behind ~3000 VALU ops.
template <bool SAFE>
__device__ __forceinline__ bool acc_chunk(uint32_t t, const G1Affine* __restrict__ bases,
                                          const uint32_t* __restrict__ vals, const uint32_t* __restrict__ koff,
                                          uint32_t nbt, uint32_t total, uint32_t L, AccPoint* __restrict__ buckets,
                                          AccPoint* __restrict__ bnd) {
  const uint32_t lo = t * L;
  if (lo >= total) return false;
  const uint32_t hi = lo + L < total ? lo + L : total;
  // the bucket holding position lo: the largest k with koff[k] <= lo (an empty key shares
  // its offset with the next one, so the largest is the non-empty bucket; koff[nbt] = total)
  uint32_t key = 0, kh = nbt;
  while (kh - key > 1) {
    const uint32_t mid = (key + kh) >> 1;
    if (koff[mid] <= lo) key = mid;
    else kh = mid;
  }
  const bool prev_same = koff[key] < lo;
  uint32_t kend = koff[key + 1];
  bool first = true, dbl = false;
  AccPoint acc = acc_identity();
  uint32_t v = vals[lo];
  G1Affine pt = ld_aff(bases + (v & 0x7fffffffu));
  for (uint32_t p = lo; p < hi; p++) {
    const uint32_t v_next = vals[p + 1 < hi ? p + 1 : p];
    const G1Affine pt_next = ld_aff(bases + (v_next & 0x7fffffffu));
    if (p == kend) {  // the run of `key` ended at p: the next non-empty bucket starts here
      msm_emit(key, acc, first, first && prev_same, false, t, buckets, bnd);
      first = false;
      // the largest k with koff[k] <= p (koff[key + 1] == p): usually key + 1; empty
      // buckets in between (concentrated digits leave long empty ranges) are crossed by
      // galloping, then bisection
      uint32_t a = key + 1, b = a + 1, step = 1;
      while (b < nbt && koff[b] <= p) {
        a = b;
        step <<= 1;
        b = a + step;
      }
      if (b > nbt) b = nbt;
      while (b - a > 1) {
        const uint32_t mid = (a + b) >> 1;
        if (koff[mid] <= p) a = mid;
        else b = mid;
      }
      key = a;
      kend = koff[key + 1];
      acc = acc_identity();
    }
    if (v >> 31) pt = affine_neg(pt);
    acc = acc_madd<SAFE>(acc, pt, &dbl);
    v = v_next;
    pt = pt_next;
  }
  msm_emit(key, acc, first, first && prev_same, kend > hi, t, buckets, bnd);
  return dbl;
}

#ifndef H2G_ACC_FAST  // 0: the doubling branch inside the hot loop (152 VGPRs, 3 waves per SIMD; A/B)
#define H2G_ACC_FAST 1
#endif
// the chunks whose runs met p == q (same point twice in a row of one bucket: repeated bases
// of a generic MSM; never for distinct SRS points), recorded for the repair pass:
// rep[0] = count, rep[1 ..] = chunk ids (up to MSM_REPAIR_CAP; beyond it every chunk is redone)
__global__ void __launch_bounds__(MSM_THREADS)
msm_acc_kernel(const G1Affine* __restrict__ bases, const uint32_t* __restrict__ vals,
               const uint32_t* __restrict__ koff, uint32_t nbt, const uint32_t* __restrict__ d_total,
               AccPoint* __restrict__ buckets, AccPoint* __restrict__ bnd, uint32_t* __restrict__ rep) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (acc_chunk<!H2G_ACC29 || !H2G_ACC_FAST>(t, bases, vals, koff, nbt, d_total[0], d_total[1], buckets, bnd)) {
    const uint32_t i = atomicAdd(rep, 1u);
    if (i < MSM_REPAIR_CAP) rep[1 + i] = t;
  }
}

// the flagged chunks again, with the doubling branch (a handful of threads; most launches
// find no chunk and return at once)
__global__ void __launch_bounds__(MSM_THREADS)
msm_acc_repair_kernel(const G1Affine* __restrict__ bases, const uint32_t* __restrict__ vals,
                      const uint32_t* __restrict__ koff, uint32_t nbt, const uint32_t* __restrict__ d_total,
                      AccPoint* __restrict__ buckets, AccPoint* __restrict__ bnd, const uint32_t* __restrict__ rep) {
  const uint32_t cnt = rep[0];
  if (cnt == 0) return;
  const uint32_t total = d_total[0], L = d_total[1], nchunks = (total + L - 1) / L;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
  if (cnt <= MSM_REPAIR_CAP) {
    for (uint32_t i = g; i < cnt; i += stride) (void)acc_chunk<true>(rep[1 + i], bases, vals, koff, nbt, total, L,
                                                                      buckets, bnd);
  } else {
    for (uint32_t t = g; t < nchunks; t += stride) (void)acc_chunk<true>(t, bases, vals, koff, nbt, total, L, buckets,
                                                                         bnd);
  }
}

hipError_t msm_accumulate(const G1Affine* bases, const uint32_t* vals, const uint32_t* koff, uint32_t nbt,
                          const uint32_t* d_total, size_t nchunks_cap, AccPoint* buckets, AccPoint* bnd,
                          uint32_t* rep, hipStream_t st) {
  const int T = MSM_THREADS;
  const unsigned cgrid = (unsigned)((nchunks_cap + T - 1) / T);
  hipLaunchKernelGGL(msm_acc_kernel, dim3(cgrid), dim3(T), 0, st, bases, vals, koff, nbt, d_total, buckets, bnd, rep);
  if (H2G_ACC29)
    hipLaunchKernelGGL(msm_acc_repair_kernel, dim3(MSM_REPAIR_BLOCKS), dim3(T), 0, st, bases, vals, koff, nbt,
                       d_total, buckets, bnd, (const uint32_t*)rep);
  return hipGetLastError();
}

}  // namespace h2g
