// msm_acc.hip -- step 3 of the MSM pipeline (msm.hip) for gfx950: the bucket accumulation,
// the dominant kernel of create_proof.  Its own translation unit so that A/B builds of it
// (tools/build_variant.py) recompile one kernel, not the reduction's dozen.
#include <stdlib.h>

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

// 3-4. accumulation straight from the sorted entries -------------------------------
// The sorted array is cut into chunks of L entries, one thread per chunk.  A chunk's
// run of one bucket is the whole bucket iff it neither continues from the previous
// chunk nor into the next (two neighbour reads; no separate bounds pass): such
// buckets are written directly, a run that crosses a chunk boundary goes to the
// chunk's boundary slot (slot 0 = its first run, slot 1 = its last run).  The run
// that begins a bucket records its start, the run that ends it its end (for the
// fixup).  The sentinel entries (zero digits) sort last and end a chunk.
__device__ __forceinline__ uint32_t ent_key(uint64_t e) { return (uint32_t)(e >> 32); }

__device__ __forceinline__ void msm_emit(uint32_t key, const G1xyzz& acc, bool first, bool from_prev, bool to_next,
                                         uint32_t a, uint32_t b, uint32_t t, G1xyzz* __restrict__ buckets,
                                         G1xyzz* __restrict__ bnd, uint32_t* __restrict__ start,
                                         uint32_t* __restrict__ end) {
  const G1xyzz v = xyzz_canon2(acc);  // lazy [0, 2M) -> fully reduced for the later kernels
  if (!from_prev) start[key] = a;
  if (!to_next) end[key] = b;
  if (!from_prev && !to_next) buckets[key] = v;
  else bnd[2 * (size_t)t + (first ? 0 : 1)] = v;
}

// PF: software-pipelined gather -- the next entry's base point is loaded before
// the current mixed addition, so its latency hides behind ~3000 VALU ops (costs
// 16 VGPRs).
#ifdef H2G_ACC_WAVES  // A/B builds: waves per SIMD the register allocation must admit
#define H2G_ACC_ATTR __attribute__((amdgpu_waves_per_eu(H2G_ACC_WAVES, H2G_ACC_WAVES)))
#else
#define H2G_ACC_ATTR
#endif
template <bool PF>
__global__ void __launch_bounds__(MSM_THREADS) H2G_ACC_ATTR
msm_acc_kernel(const G1Affine* __restrict__ bases, const uint64_t* __restrict__ ent,
               const uint32_t* __restrict__ d_total, uint32_t sentinel, uint32_t L, G1xyzz* __restrict__ buckets,
               G1xyzz* __restrict__ bnd, uint32_t* __restrict__ start, uint32_t* __restrict__ end) {
  const uint32_t total = *d_total;  // entries (nonzero digits) of the partition
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lo = t * L;
  if (lo >= total) return;
  const uint32_t hi = lo + L < total ? lo + L : total;
  uint64_t e = ent[lo];
  uint32_t key = ent_key(e);
  if (key == sentinel) return;
  const bool prev_same = lo > 0 && ent_key(ent[lo - 1]) == key;
  bool first = true;
  uint32_t run_lo = lo;
  G1xyzz acc = G1xyzz::identity();
  G1Affine pt;
  if (PF) pt = ld_aff(bases + ((uint32_t)e & 0x7fffffffu));
  uint32_t p = lo;
  for (; p < hi; p++) {
    uint64_t e_next = 0;
    G1Affine pt_next;
    if (PF) {
      e_next = ent[p + 1 < hi ? p + 1 : p];
      pt_next = ld_aff(bases + ((uint32_t)e_next & 0x7fffffffu));
    } else {
      e = ent[p];
#ifdef H2G_MSM_TIMING_GATHER_MASK  // timing-only A/B build: gather from a small (L2-resident) table
      pt = ld_aff(bases + ((uint32_t)e & H2G_MSM_TIMING_GATHER_MASK));
#else
      pt = ld_aff(bases + ((uint32_t)e & 0x7fffffffu));
#endif
    }
    const uint32_t k2 = ent_key(e);
    if (k2 == sentinel) break;
    const uint32_t v = (uint32_t)e;
    if (k2 != key) {
      msm_emit(key, acc, first, first && prev_same, false, run_lo, p, t, buckets, bnd, start, end);
      first = false;
      run_lo = p;
      key = k2;
      acc = G1xyzz::identity();
    }
    if (v >> 31) pt = affine_neg(pt);
    acc = xyzz_madd_lazy(acc, pt);
    if (PF) {
      e = e_next;
      pt = pt_next;
    }
  }
  const bool to_next = p == hi && hi < total && ent_key(ent[hi]) == key;
  msm_emit(key, acc, first, first && prev_same, to_next, run_lo, p, t, buckets, bnd, start, end);
}

hipError_t msm_accumulate(const G1Affine* bases, const uint64_t* ent, const uint32_t* d_total, uint32_t sentinel,
                          uint32_t L, size_t nchunks, G1xyzz* buckets, G1xyzz* bnd, uint32_t* bstart, uint32_t* bend,
                          hipStream_t st) {
  const int T = MSM_THREADS;
  static const bool prefetch = [] {  // H2G_MSM_PREFETCH=0: gather inside the loop (A/B)
    const char* e = getenv("H2G_MSM_PREFETCH");
    return e ? atoi(e) != 0 : true;
  }();
  const unsigned cgrid = (unsigned)((nchunks + T - 1) / T);
  if (prefetch)
    hipLaunchKernelGGL(msm_acc_kernel<true>, dim3(cgrid), dim3(T), 0, st, bases, ent, d_total, sentinel, L, buckets,
                       bnd, bstart, bend);
  else
    hipLaunchKernelGGL(msm_acc_kernel<false>, dim3(cgrid), dim3(T), 0, st, bases, ent, d_total, sentinel, L, buckets,
                       bnd, bstart, bend);
  return hipGetLastError();
}

}  // namespace h2g
