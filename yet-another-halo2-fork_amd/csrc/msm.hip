// msm.hip -- Pippenger multi-scalar multiplication over BN254 G1 for gfx950.
//
// Computes MsmAccel::msm(coeffs, bases) = sum_i coeffs[i] * bases[i]
// (halo2_middleware/src/zal.rs:58; CPU reference halo2curves best_multiexp,
// zal.rs:136-138) for the commitment call sites listed in SURVEY 8a-1.
//
// Pipeline (one stream, no host round trips):
//   1. digits     : Montgomery -> canonical, signed c-bit windows (|d| <= 2^(c-1)),
//                   key = window*NB + |d|-1, value = point index | sign << 31; zero
//                   digits dropped
//   2. partition  : two counting rounds group the values by key (coarse bins from the
//                   scalars directly, then one workgroup per bin orders its keys in LDS)
//                   -- the accumulation needs buckets contiguous, not sorted; bucket k
//                   is [koff[k], koff[k + 1]) of the u32 value array
//   3. accumulate : the sorted array is cut into fixed chunks of L entries, one
//                   thread per chunk (every thread does exactly L mixed additions,
//                   whatever the bucket sizes -> no load imbalance, also for skewed
//                   scalars).  XYZZ += affine (madd-2008-s) on lazily reduced
//                   [0, 2p) coordinates, bases gathered by sorted index.  A run that
//                   neither continues from the previous chunk nor into the next is a
//                   whole bucket and is written directly; otherwise it goes to the
//                   chunk's boundary slot.
//   4. fixup      : buckets spanning chunks sum their boundary slots (one thread,
//                   or items of 64 pieces for buckets spanning more chunks)
//   5. reduction  : sum_j (j+1) B_j per bucket set: group running sums, then bit planes
//                   (or per-group scalar multiplications for c = 22 sets) and trees
//   6. final      : Horner over windows (c doublings each), to affine -- on the
//                   host for host-returning entry points (a single-lane chain of
//                   ~250 doublings is latency-bound on the GPU), else one device lane.
// The result is the unique affine point, so it is bit-identical to any other
// correct MSM (e.g. the CPU restatement in oracle/) regardless of summation order.
#include <algorithm>

#include "msm_part.h"

namespace h2g {

// Diagnostic build only (tools/build_variant.py ... -DH2G_RED_TIMING): wall-clock stamps
// (s_memrealtime, 100 MHz) at the phase boundaries of the reduction kernels, read back
// with h2g_dbg_red_ts (tools/red_timing.py)
#ifdef H2G_RED_TIMING
__device__ unsigned long long g_red_ts[64];
#define RED_TS(cond, i)                                  \
  do {                                                   \
    if ((cond) && threadIdx.x == 0) g_red_ts[i] = wall_clock64(); \
  } while (0)
#else
#define RED_TS(cond, i) \
  do {                  \
  } while (0)
#endif


static constexpr int MSM_THREADS = 256;
static constexpr uint32_t MSM_SMALL = 8;  // fixup: max chunk pieces summed by one thread

int msm_windows_for(int c) { return (255 + c - 1) / c; }

int msm_choose_c(size_t n) {
  if (n < 4) return 2;
  int best_c = 2;
  double best = 1e300;
  for (int c = 2; c <= 22; c++) {
    const double W = msm_windows_for(c);
    const double cost = W * ((double)n + 2.8 * (double)(1ull << (c - 1)));
    if (cost < best) {
      best = cost;
      best_c = c;
    }
  }
  return best_c;
}

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

// Quad-cooperative XYZZ arithmetic for the latency-bound reduction kernels ----------
// With one wave per SIMD an XYZZ addition is issue-bound at ~13 us (14 Montgomery
// products in sequence).  Its products fall into 4 dependent levels (a doubling's 10
// into 3): the 4 lanes of a quad hold the same operands, each lane computes one product
// of a level, and DPP quad_perm broadcasts hand the results to the quad.  ~3x less
// latency per operation for 1.3x the issue slots -- used where a kernel has too few
// threads to fill the SIMDs.  Every lane of a quad must be active with equal operands.
template <int K>
__device__ __forceinline__ Fq quad_bcast(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++)
    r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], K | (K << 2) | (K << 4) | (K << 6), 0xf, 0xf, false);
  return r;
}
__device__ __forceinline__ Fq quad_sel(int s, const Fq& a, const Fq& b, const Fq& c, const Fq& d) {
  // masks: a ternary chain here became an indexed load from a stack copy (scratch)
  const uint32_t m0 = 0u - (uint32_t)(s == 0), m1 = 0u - (uint32_t)(s == 1), m2 = 0u - (uint32_t)(s == 2),
                 m3 = 0u - (uint32_t)(s == 3);
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (a.l[i] & m0) | (b.l[i] & m1) | (c.l[i] & m2) | (d.l[i] & m3);
  return r;
}

// dbl-2008-s-1 (= xyzz_dbl): levels {V, X^2}, {W, S, ZZ', M^2}, {ZZZ', W Y, M (S - X')}
__device__ G1xyzz xyzz_dbl_q4(const G1xyzz& p) {
  if (p.is_identity()) return p;
  const int s = threadIdx.x & 3;
  const Fq U = dbl(p.Y);
  const Fq a1 = (s & 1) ? p.X : U;
  Fq m = a1 * a1;
  const Fq V = quad_bcast<0>(m), X2 = quad_bcast<1>(m);
  const Fq M = X2 + dbl(X2);
  m = quad_sel(s, U, p.X, V, M) * quad_sel(s, V, V, p.ZZ, M);
  const Fq W = quad_bcast<0>(m), S = quad_bcast<1>(m), ZZ3 = quad_bcast<2>(m), MM = quad_bcast<3>(m);
  G1xyzz r;
  r.X = MM - dbl(S);
  m = quad_sel(s, W, W, M, W) * quad_sel(s, p.ZZZ, p.Y, S - r.X, p.ZZZ);
  r.Y = quad_bcast<2>(m) - quad_bcast<1>(m);
  r.ZZ = ZZ3;
  r.ZZZ = quad_bcast<0>(m);
  return r;
}

// add-2008-s (= xyzz_add): levels {U1, U2, S1, S2}, {P^2, R^2, ZZ1 ZZ2, ZZZ1 ZZZ2},
// {PPP, Q, ZZ'}, {R (Q - X'), S1 PPP, ZZZ'}
__device__ G1xyzz xyzz_add_q4(const G1xyzz& p, const G1xyzz& q) {
  if (q.is_identity()) return p;
  if (p.is_identity()) return q;
  const int s = threadIdx.x & 3;
  Fq m = quad_sel(s, p.X, q.X, p.Y, q.Y) * quad_sel(s, q.ZZ, p.ZZ, q.ZZZ, p.ZZZ);
  const Fq U1 = quad_bcast<0>(m), U2 = quad_bcast<1>(m), S1 = quad_bcast<2>(m), S2 = quad_bcast<3>(m);
  const Fq Pp = U2 - U1;
  const Fq R = S2 - S1;
  if (Pp.is_zero()) {
    if (R.is_zero()) return xyzz_dbl_q4(p);
    return G1xyzz::identity();
  }
  m = quad_sel(s, Pp, R, p.ZZ, p.ZZZ) * quad_sel(s, Pp, R, q.ZZ, q.ZZZ);
  const Fq PP = quad_bcast<0>(m), RR = quad_bcast<1>(m), ZZ12 = quad_bcast<2>(m), ZZZ12 = quad_bcast<3>(m);
  m = quad_sel(s, Pp, U1, ZZ12, Pp) * PP;
  const Fq PPP = quad_bcast<0>(m), Q = quad_bcast<1>(m);
  G1xyzz r;
  r.ZZ = quad_bcast<2>(m);
  r.X = RR - PPP - dbl(Q);
  m = quad_sel(s, R, S1, ZZZ12, R) * quad_sel(s, Q - r.X, PPP, PPP, PPP);
  r.Y = quad_bcast<0>(m) - quad_bcast<1>(m);
  r.ZZZ = quad_bcast<2>(m);
  return r;
}

__device__ G1xyzz xyzz_mul_u32_q4(const G1xyzz& p, uint32_t k) {
  if (k == 0) return G1xyzz::identity();
  int top = 31;
  while (!((k >> top) & 1)) top--;
  G1xyzz acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = xyzz_dbl_q4(acc);
    if ((k >> b) & 1) acc = xyzz_add_q4(acc, p);
  }
  return acc;
}

#if H2G_ACC29
// the same quad-cooperative levels in F29 (f29.h; the back-end class, coordinates < 1.2 M)
template <int K>
__device__ __forceinline__ F29 quad_bcast29(const F29& a) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++)
    r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], K | (K << 2) | (K << 4) | (K << 6), 0xf, 0xf, false);
  return r;
}
// masks, not a ternary chain: the compiler turns a 4-way select on a lane index into an
// indexed load from a stack copy of the four operands (scratch traffic in every product)
__device__ __forceinline__ F29 quad_sel29(int s, const F29& a, const F29& b, const F29& c, const F29& d) {
  const uint32_t m0 = 0u - (uint32_t)(s == 0), m1 = 0u - (uint32_t)(s == 1), m2 = 0u - (uint32_t)(s == 2),
                 m3 = 0u - (uint32_t)(s == 3);
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = (a.l[i] & m0) | (b.l[i] & m1) | (c.l[i] & m2) | (d.l[i] & m3);
  return r;
}
// limb-wise select (a ternary on whole structs can become a select of their stack copies)
__device__ __forceinline__ F29 pick29(bool c, const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}
// levels {V, X^2}, {W, S, ZZ', M^2}, {ZZZ', M (S - X') - W Y (one merged reduction)}
__device__ __forceinline__ G1xyzz29 xyzz29_dbl_q4(const G1xyzz29& p) {
  using P = FqParams;
  if (xyzz29_is_identity(p)) return p;
  const int s = threadIdx.x & 3;
  const F29 U = norm29(add29(p.Y, p.Y));
  const F29 a1 = pick29(s & 1, p.X, U);
  F29 m = sqr29<P>(a1);
  const F29 V = quad_bcast29<0>(m), X2 = quad_bcast29<1>(m);
  const F29 Mm = norm29(add29(add29(X2, X2), X2));
  m = mul29<P>(quad_sel29(s, U, p.X, V, Mm), quad_sel29(s, V, V, p.ZZ, Mm));
  const F29 W = quad_bcast29<0>(m), S = quad_bcast29<1>(m), ZZ3 = quad_bcast29<2>(m), MM = quad_bcast29<3>(m);
  G1xyzz29 r;
  r.X = reduce29<P>(norm29(sub29<P, 4, 31>(MM, add29(S, S))));
  const F29 z = F29{};
  const bool s0 = s == 0;
  m = mul29x2<P>(pick29(s0, W, Mm), pick29(s0, p.ZZZ, sub29<P, 4, 29>(S, r.X)), pick29(s0, z, p.Y),
                 pick29(s0, z, sub29<P, 2, 29>(z, W)));
  r.ZZZ = quad_bcast29<0>(m);
  r.Y = quad_bcast29<1>(m);
  r.ZZ = ZZ3;
  return r;
}
// levels {U1, U2, S1, S2}, {P^2, R^2, ZZ1 ZZ2, ZZZ1 ZZZ2}, {PPP, Q, ZZ'}, {R (Q - X') - S1 PPP, ZZZ'}
__device__ __forceinline__ G1xyzz29 xyzz29_add_q4(const G1xyzz29& p, const G1xyzz29& q) {
  using P = FqParams;
  if (xyzz29_is_identity(q)) return p;
  if (xyzz29_is_identity(p)) return q;
  const int s = threadIdx.x & 3;
  F29 m = mul29<P>(quad_sel29(s, p.X, q.X, p.Y, q.Y), quad_sel29(s, q.ZZ, p.ZZ, q.ZZZ, p.ZZZ));
  const F29 U1 = quad_bcast29<0>(m), U2 = quad_bcast29<1>(m), S1 = quad_bcast29<2>(m), S2 = quad_bcast29<3>(m);
  const F29 Pp = norm29(sub29<P, 2, 29>(U2, U1));
  const F29 R = norm29(sub29<P, 2, 29>(S2, S1));
  if (is_zero29<P>(Pp)) {
    if (is_zero29<P>(R)) return xyzz29_dbl_q4(p);
    return xyzz29_identity();
  }
  m = mul29<P>(quad_sel29(s, Pp, R, p.ZZ, p.ZZZ), quad_sel29(s, Pp, R, q.ZZ, q.ZZZ));
  const F29 PP = quad_bcast29<0>(m), RR = quad_bcast29<1>(m), ZZ12 = quad_bcast29<2>(m), ZZZ12 = quad_bcast29<3>(m);
  m = mul29<P>(quad_sel29(s, Pp, U1, ZZ12, Pp), PP);
  const F29 PPP = quad_bcast29<0>(m), Q = quad_bcast29<1>(m);
  G1xyzz29 r;
  r.ZZ = quad_bcast29<2>(m);
  r.X = reduce29<P>(norm29(sub29<P, 4, 31>(RR, add29(add29(PPP, Q), Q))));
  const F29 z = F29{};
  const bool s0 = s == 0;
  m = mul29x2<P>(pick29(s0, R, ZZZ12), pick29(s0, sub29<P, 4, 29>(Q, r.X), PPP), pick29(s0, S1, z),
                 pick29(s0, sub29<P, 2, 29>(z, PPP), z));
  r.Y = quad_bcast29<0>(m);
  r.ZZZ = quad_bcast29<1>(m);
  return r;
}
__device__ G1xyzz29 xyzz29_mul_u32_q4(const G1xyzz29& p, uint32_t k) {
  if (k == 0) return xyzz29_identity();
  int top = 31;
  while (!((k >> top) & 1)) top--;
  G1xyzz29 acc = p;
  for (int b = top - 1; b >= 0; b--) {
    acc = xyzz29_dbl_q4(acc);
    if ((k >> b) & 1) acc = xyzz29_add_q4(acc, p);
  }
  return acc;
}
#endif

// The back-end's point type (msm_part.h RedPoint) and its operations: F29 accumulators in
// the back-end class with H2G_ACC29, canonical G1xyzz otherwise
__device__ __forceinline__ RedPoint rp_identity() {
#if H2G_ACC29
  return xyzz29_identity();
#else
  return G1xyzz::identity();
#endif
}
#if H2G_ACC29
__device__ __forceinline__ RedPoint rp_add(const RedPoint& a, const RedPoint& b) { return xyzz29_add(a, b); }
__device__ __forceinline__ RedPoint rp_dbl(const RedPoint& a) { return xyzz29_dbl(a); }
__device__ __forceinline__ RedPoint rp_add_q4(const RedPoint& a, const RedPoint& b) { return xyzz29_add_q4(a, b); }
__device__ __forceinline__ RedPoint rp_dbl_q4(const RedPoint& a) { return xyzz29_dbl_q4(a); }
__device__ __forceinline__ RedPoint rp_mul_u32(const RedPoint& a, uint32_t k) { return xyzz29_mul_u32(a, k); }
__device__ __forceinline__ RedPoint rp_mul_u32_q4(const RedPoint& a, uint32_t k) { return xyzz29_mul_u32_q4(a, k); }
__device__ __forceinline__ G1xyzz rp_to_xyzz(const RedPoint& a) { return xyzz_from29(a); }
// an accumulation output (bucket or boundary slot) into the back-end class
__device__ __forceinline__ RedPoint rp_from_acc(const AccPoint& a) { return xyzz29_reduce(a); }
#else
__device__ __forceinline__ RedPoint rp_add(const RedPoint& a, const RedPoint& b) { return xyzz_add(a, b); }
__device__ __forceinline__ RedPoint rp_dbl(const RedPoint& a) { return xyzz_dbl(a); }
__device__ __forceinline__ RedPoint rp_add_q4(const RedPoint& a, const RedPoint& b) { return xyzz_add_q4(a, b); }
__device__ __forceinline__ RedPoint rp_dbl_q4(const RedPoint& a) { return xyzz_dbl_q4(a); }
__device__ __forceinline__ RedPoint rp_mul_u32(const RedPoint& a, uint32_t k) { return xyzz_mul_u32(a, k); }
__device__ __forceinline__ RedPoint rp_mul_u32_q4(const RedPoint& a, uint32_t k) { return xyzz_mul_u32_q4(a, k); }
__device__ __forceinline__ G1xyzz rp_to_xyzz(const RedPoint& a) { return a; }
__device__ __forceinline__ RedPoint rp_from_acc(const AccPoint& a) { return a; }
#endif
// 16-B moves of back-end points in global memory
__device__ __forceinline__ RedPoint ld_rp(const RedPoint* p) {
#if H2G_ACC29
  return ld_acc(p);
#else
  return *p;
#endif
}
__device__ __forceinline__ void st_rp(RedPoint* p, const RedPoint& v) {
#if H2G_ACC29
  st_acc(p, v);
#else
  *p = v;
#endif
}

// Buckets spanning chunks, one thread per bucket: the piece in its first chunk t0 is
// that chunk's last run (slot 1) unless the bucket starts the chunk (slot 0); every
// later chunk holds it as its first run (slot 0).  Buckets over more than MSM_SMALL
// chunks are cut into items of at most MSM_ITEM pieces (msm_big_item_kernel), whose
// partial sums a second pass combines per bucket (msm_big_combine_kernel): the depth
// stays logarithmic however the scalars concentrate (fixed-base top windows: n / 2^12
// entries per bucket at c = 22; a column of equal values: n entries per bucket).
// (H2G_ACC29: the slots hold raw F29 accumulators, brought into the back-end class here)
__device__ __forceinline__ RedPoint msm_piece(const AccPoint* bnd, uint32_t t, uint32_t t0, uint32_t bs, uint32_t L) {
  return rp_from_acc(ld_accp(bnd + 2 * (size_t)t + ((t == t0 && bs != t0 * L) ? 1 : 0)));
}

static constexpr uint32_t MSM_GROUP = 16;            // lanes per item
static constexpr uint32_t MSM_ITEM = MSM_GROUP * 4;  // pieces per item (4 per lane)
static constexpr unsigned MSM_BIG_BLOCKS = 512;      // persistent grids below

// big-bucket work item: pieces [tb, te) of bucket b; slot = the item's index into the
// partial sums when the bucket has several items, ~0u when it is the bucket's only one
struct MsmBigItem {
  uint32_t b, tb, te, slot;
};

// upper bounds of the item lists (sizing): a bucket over np > MSM_SMALL chunks takes
// ceil(np / MSM_ITEM) items, and the buckets' piece counts sum to < 2 nchunks
static size_t msm_big_items_cap(size_t nchunks) { return 2 * nchunks / MSM_ITEM + 2 * nchunks / MSM_SMALL + 2; }
static size_t msm_big_multi_cap(size_t nchunks) { return 2 * nchunks / MSM_ITEM + 2; }

// The item lists are reserved with one atomic per wave (a wave-level scan of the lanes'
// item counts), not one per bucket.  Q = 4: a quad per bucket (xyzz_add_q4, ~3x less
// latency per addition) summing up to MSM_SMALL_Q4 pieces itself -- for small bucket
// sets (<= 2^15), whose buckets span up to ~10 chunks of the minimum chunk length (2^16
// points at c = 15: 9 pieces each, all of which took the big-item path: fixup 0.30 ->
// 0.11 ms; at 2^16 buckets the quads' issue cost loses, 0.097 -> 0.142 ms).
static constexpr uint32_t MSM_SMALL_Q4 = 32;

template <int Q>
__global__ void __launch_bounds__(MSM_THREADS)
msm_fixup_kernel(const AccPoint* __restrict__ bnd, const uint32_t* __restrict__ koff, uint32_t nbt,
                 const uint32_t* __restrict__ d_total, const AccPoint* __restrict__ whole, RedPoint* __restrict__ buckets,
                 MsmBigItem* __restrict__ items, uint4* __restrict__ multi, uint32_t* __restrict__ counters) {
  H2G_SETPRIO(H2G_PRIO_RED);
  const uint32_t L = d_total[1];  // the accumulation's chunk length (msm_chunk_len_dev)
  const uint32_t b = (blockIdx.x * blockDim.x + threadIdx.x) / Q;
  const uint32_t lane = threadIdx.x & 63;
  const bool lead = (threadIdx.x % Q) == 0;
  RED_TS(blockIdx.x == 0, 20);
  RED_TS(blockIdx.x == gridDim.x - 1, 22);
  uint32_t bs = 0, be = 0;
  if (b < nbt) {
    bs = koff[b];
    be = koff[b + 1];
  }
  // np pieces (0: empty bucket, or written by the accumulation kernel)
  const uint32_t t0 = bs / L, t1 = be > bs ? (be - 1) / L : t0;
  const uint32_t np = be > bs && t1 > t0 ? t1 - t0 + 1 : 0;
  const uint32_t small = Q == 4 ? MSM_SMALL_Q4 : MSM_SMALL;
  const uint32_t cnt = lead && np > small ? (np + MSM_ITEM - 1) / MSM_ITEM : 0;
  // every lane of the wave reaches the scan (no early returns above)
  uint32_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += v;
  }
  const uint32_t wtot = __shfl(incl, 63, 64);
  const uint64_t mm = __ballot(cnt > 1);
  uint32_t ibase = 0, mbase = 0;
  if (lane == 0) {
    if (wtot) ibase = atomicAdd(&counters[0], wtot);
    if (mm) mbase = atomicAdd(&counters[1], (uint32_t)__popcll(mm));
  }
  ibase = __shfl(ibase, 0, 64);
  mbase = __shfl(mbase, 0, 64);
  if (b < nbt && be <= bs && lead) st_rp(buckets + b, rp_identity());  // empty (no fill of buckets[])
#if H2G_ACC29
  // a bucket the accumulation wrote whole: its raw accumulator, into the back-end class
  if (b < nbt && be > bs && np == 0 && lead) st_rp(buckets + b, rp_from_acc(ld_accp(whole + b)));
#endif
  if (np == 0) return;
  if (np > small) {
    if (!cnt) return;  // the quad's other lanes
    const uint32_t base = ibase + incl - cnt;
    for (uint32_t i = 0; i < cnt; i++) {
      MsmBigItem it;
      it.b = b;
      it.tb = t0 + i * MSM_ITEM;
      it.te = min(t0 + (i + 1) * MSM_ITEM, t1 + 1);
      it.slot = cnt > 1 ? base + i : ~0u;
      items[base + i] = it;
    }
    if (cnt > 1) multi[mbase + (uint32_t)__popcll(mm & ((1ull << lane) - 1))] = make_uint4(b, base, cnt, 0);
    return;
  }
  RedPoint acc = msm_piece(bnd, t0, t0, bs, L);
  for (uint32_t t = t0 + 1; t <= t1; t++) {
    if constexpr (Q == 4) acc = rp_add_q4(acc, msm_piece(bnd, t, t0, bs, L));
    else acc = rp_add(acc, msm_piece(bnd, t, t0, bs, L));
  }
  if (lead) st_rp(buckets + b, acc);
}

// MSM_GROUP lanes per item (4 items per wave, persistent grid): each lane sums up to
// 4 strided pieces, then a log2(MSM_GROUP)-level tree in the wave's LDS slice.
__global__ void __launch_bounds__(MSM_THREADS)
msm_big_item_kernel(const AccPoint* __restrict__ bnd, const uint32_t* __restrict__ koff,
                    const uint32_t* __restrict__ d_total, const MsmBigItem* __restrict__ items,
                    const uint32_t* __restrict__ counters, RedPoint* __restrict__ partial,
                    RedPoint* __restrict__ buckets) {
  H2G_SETPRIO(H2G_PRIO_RED);
  const uint32_t L = d_total[1];
  __shared__ RedPoint sh[MSM_THREADS];
  const uint32_t nitems = counters[0];
  const uint32_t lane = threadIdx.x & 63, g = lane & (MSM_GROUP - 1);
  RedPoint* w = sh + (threadIdx.x & ~(MSM_GROUP - 1));
  constexpr uint32_t per_wave = 64 / MSM_GROUP;
  const uint32_t stride = gridDim.x * (MSM_THREADS / 64) * per_wave;
  // uniform trip count per wave (all lanes reach the wave barriers)
  for (uint32_t q0 = (blockIdx.x * (MSM_THREADS / 64) + (threadIdx.x >> 6)) * per_wave; q0 < nitems;
       q0 += stride) {
    const uint32_t q = q0 + lane / MSM_GROUP;
    RedPoint acc = rp_identity();
    MsmBigItem it = {0, 0, 0, 0};
    if (q < nitems) {
      it = items[q];
      const uint32_t bs = koff[it.b], t0 = bs / L;
      for (uint32_t t = it.tb + g; t < it.te; t += MSM_GROUP) acc = rp_add(acc, msm_piece(bnd, t, t0, bs, L));
    }
    w[g] = acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
    for (uint32_t h = MSM_GROUP / 2; h > 0; h >>= 1) {
      if (g < h) w[g] = rp_add(w[g], w[g + h]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (g == 0 && q < nitems) {
      if (it.slot == ~0u) buckets[it.b] = w[0];
      else partial[it.slot] = w[0];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// buckets with several items: the sum of their items' partial sums -- one lane per bucket
// of at most COMBINE_LANE items (a short sequential sum; skewed inputs -- a lookup's
// permuted column holds a few hundred distinct values -- make thousands of such buckets,
// where a wave per bucket left 63 lanes idle: 0.8 ms per keccak-style batch), one
// wavefront and a tree per larger bucket
static constexpr uint32_t COMBINE_LANE = 8;
__global__ void __launch_bounds__(MSM_THREADS)
msm_big_combine_kernel(const uint4* __restrict__ multi, const uint32_t* __restrict__ counters,
                       const RedPoint* __restrict__ partial, RedPoint* __restrict__ buckets) {
  H2G_SETPRIO(H2G_PRIO_RED);
  __shared__ RedPoint sh[MSM_THREADS];
  const uint32_t nm = counters[1];
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t q = blockIdx.x * MSM_THREADS + threadIdx.x; q < nm; q += gridDim.x * MSM_THREADS) {
    const uint4 m = multi[q];  // (bucket, first item, items)
    if (m.z > COMBINE_LANE) continue;
    RedPoint acc = partial[m.y];
    for (uint32_t i = 1; i < m.z; i++) acc = rp_add(acc, partial[m.y + i]);
    buckets[m.x] = acc;
  }
  RedPoint* w = sh + (threadIdx.x & ~63u);
  const uint32_t nwaves = gridDim.x * (MSM_THREADS / 64);
  for (uint32_t q = blockIdx.x * (MSM_THREADS / 64) + (threadIdx.x >> 6); q < nm; q += nwaves) {
    const uint4 m = multi[q];  // (bucket, first item, items)
    if (m.z <= COMBINE_LANE) continue;  // uniform across the wave
    RedPoint acc = rp_identity();
    for (uint32_t i = lane; i < m.z; i += 64) acc = rp_add(acc, partial[m.y + i]);
    w[lane] = acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
    for (uint32_t h = 32; h > 0; h >>= 1) {
      if (lane < h) w[lane] = rp_add(w[lane], w[lane + h]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) buckets[m.x] = w[0];
    __builtin_amdgcn_wave_barrier();
  }
}

// 6a. bucket reduction (default): F = sum_j (j+1) B_j per window, shallow ------------------
// A serial chain of XYZZ additions costs ~12 us on the GPU at low occupancy, so the
// reduction minimises dependent depth, not only work:
//   rgroup : groups of RG buckets: S_g = sum_t (t+1) B_{RG g+t}, R_g = sum_t B_{RG g+t}
//   then F = sum_g (S_g + [RG g] R_g) by bit planes (6a', up to 2^16 groups), or
//   rscale : V_g = S_g + [RG g] R_g (one scalar multiplication per group), block sums of V
//   rfinal : sum of the block sums
// (rscale's depth ~ 2 RG + (log2(RG m) dbl + adds) + 2 x 8 tree steps).
#ifndef H2G_MSM_RG
#define H2G_MSM_RG 8
#endif
static constexpr int RG = H2G_MSM_RG;

__global__ void __launch_bounds__(MSM_THREADS)
msm_rgroup_kernel(const RedPoint* __restrict__ B, uint32_t NB, uint32_t m1, RedPoint* __restrict__ S,
                  RedPoint* __restrict__ R) {
  H2G_SETPRIO(H2G_PRIO_RED);
  const uint32_t w = blockIdx.y;
  const uint32_t g = blockIdx.x * MSM_THREADS + threadIdx.x;
  if (g >= m1) return;
  const RedPoint* b = B + (size_t)w * NB;
  RedPoint racc = rp_identity(), sacc = rp_identity();
  for (int t = RG - 1; t >= 0; t--) {
    const uint32_t j = g * RG + t;
    if (j < NB) racc = rp_add(racc, b[j]);
    sacc = rp_add(sacc, racc);
  }
  S[(size_t)w * m1 + g] = sacc;
  R[(size_t)w * m1 + g] = racc;
}

__global__ void __launch_bounds__(MSM_THREADS)
msm_rscale_kernel(const RedPoint* __restrict__ S, const RedPoint* __restrict__ R, uint32_t m1,
                  RedPoint* __restrict__ part, uint32_t nblk) {
  H2G_SETPRIO(H2G_PRIO_RED);
  __shared__ RedPoint sh[MSM_THREADS];
  const uint32_t w = blockIdx.y;
  const uint32_t g = blockIdx.x * MSM_THREADS + threadIdx.x;
  RedPoint v = rp_identity();
  if (g < m1) {
    v = S[(size_t)w * m1 + g];
    if (g) v = rp_add(v, rp_mul_u32(R[(size_t)w * m1 + g], g * RG));
  }
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int h = MSM_THREADS / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) sh[threadIdx.x] = rp_add(sh[threadIdx.x], sh[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)w * nblk + blockIdx.x] = sh[0];
}

// the same three kernels with one quad per thread above (xyzz_*_q4): a quad per group,
// 64 groups per block; taken when the groups cannot fill the SIMDs (small MSMs, e.g. the
// 2^19-2^20-point slabs of a sharded proof), and always for the final tree
__global__ void __launch_bounds__(MSM_THREADS)
msm_rgroup_q4_kernel(const RedPoint* __restrict__ B, uint32_t NB, uint32_t m1, RedPoint* __restrict__ S,
                     RedPoint* __restrict__ R) {
  H2G_SETPRIO(H2G_PRIO_RED);
  const uint32_t w = blockIdx.y;
  const uint32_t g = (blockIdx.x * MSM_THREADS + threadIdx.x) >> 2;
  if (g >= m1) return;  // the whole quad
  const RedPoint* b = B + (size_t)w * NB;
  RedPoint racc = rp_identity(), sacc = rp_identity();
  for (int t = RG - 1; t >= 0; t--) {
    const uint32_t j = g * RG + t;
    if (j < NB) racc = rp_add_q4(racc, b[j]);
    sacc = rp_add_q4(sacc, racc);
  }
  if ((threadIdx.x & 3) == 0) {
    S[(size_t)w * m1 + g] = sacc;
    R[(size_t)w * m1 + g] = racc;
  }
}

static constexpr uint32_t Q4_GROUPS = MSM_THREADS / 4;  // quads per block

__global__ void __launch_bounds__(MSM_THREADS)
msm_rscale_q4_kernel(const RedPoint* __restrict__ S, const RedPoint* __restrict__ R, uint32_t m1,
                     RedPoint* __restrict__ part, uint32_t nblk) {
  H2G_SETPRIO(H2G_PRIO_RED);
  __shared__ RedPoint sh[Q4_GROUPS];
  const uint32_t w = blockIdx.y, qi = threadIdx.x >> 2;
  const uint32_t g = blockIdx.x * Q4_GROUPS + qi;
  RedPoint v = rp_identity();
  if (g < m1) {
    v = S[(size_t)w * m1 + g];
    if (g) v = rp_add_q4(v, rp_mul_u32_q4(R[(size_t)w * m1 + g], g * RG));
  }
  if ((threadIdx.x & 3) == 0) sh[qi] = v;
  __syncthreads();
  for (uint32_t h = Q4_GROUPS / 2; h > 0; h >>= 1) {
    if (qi < h) {  // sh[qi + h] is not written at this level
      const RedPoint t = rp_add_q4(sh[qi], sh[qi + h]);
      if ((threadIdx.x & 3) == 0) sh[qi] = t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)w * nblk + blockIdx.x] = sh[0];
}

__global__ void __launch_bounds__(MSM_THREADS)
msm_rfinal_q4_kernel(const RedPoint* __restrict__ part, uint32_t nblk, G1xyzz* __restrict__ windows) {
  H2G_SETPRIO(H2G_PRIO_RED);
  __shared__ RedPoint sh[Q4_GROUPS];
  const uint32_t w = blockIdx.x, qi = threadIdx.x >> 2;
  RedPoint acc = rp_identity();
  for (uint32_t i = qi; i < nblk; i += Q4_GROUPS) acc = rp_add_q4(acc, part[(size_t)w * nblk + i]);
  if ((threadIdx.x & 3) == 0) sh[qi] = acc;
  __syncthreads();
  for (uint32_t h = Q4_GROUPS / 2; h > 0; h >>= 1) {
    if (qi < h) {
      const RedPoint t = rp_add_q4(sh[qi], sh[qi + h]);
      if ((threadIdx.x & 3) == 0) sh[qi] = t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) windows[w] = rp_to_xyzz(sh[0]);  // the host finish reads G1xyzz
}

// 6a'. group weights by bit planes (default when the groups fit 2^16) ----------------------
// F = sum_g (S_g + 2^e g R_g) = sum_g S_g + sum_b 2^(b+e) U_b,  U_b = sum_{g : bit b of g} R_g.
// The plane sums need no scalar multiplication: a block of 256 groups folds its R_t in
// a binary tree whose nodes keep (T, L_0 .. L_{k-1}) -- the subtree total and the sums of
// the elements with bit b of t set; merging halves A | C of size 2^k costs k + 1 additions
// (T += T_C, L_b += L_b^C) and C's total becomes L_k in place.  ~2.5 point operations per
// group against ~30 for rscale's 19-bit double-and-add, depth 8.  The blocks' L_b are
// plain-summed across blocks (plane b < 8) and their totals folded once more by block
// index (planes 8..15); the last block to finish scales the 16 planes and adds them to
// sum S.  Two launches (rgroup fused into the first), lane-per-group (Q = 1, 256-group
// blocks) or quad-cooperative (Q = 4, 64-group blocks) like the group kernels above.

// The plane kernels' additions skip, wave-uniformly, when every lane adds the identity:
// sets of small or sparse scalars (a batch of 4-bit witness columns fills 15 buckets of
// 2^16 per set) are mostly empty groups, whose additions the identity test alone, taken
// per lane inside the formula, does not skip for the wave.  (A/B: H2G_RED_SKIP=0.)
#ifndef H2G_RED_SKIP
#define H2G_RED_SKIP 1
#endif
__device__ __forceinline__ bool rp_is_identity(const RedPoint& a) {
#if H2G_ACC29
  return xyzz29_is_identity(a);
#else
  return a.is_identity();
#endif
}
template <int Q>
__device__ __forceinline__ RedPoint padd(const RedPoint& a, const RedPoint& b) {
  if (H2G_RED_SKIP && !__any(!rp_is_identity(b))) return a;
  if constexpr (Q == 4) return rp_add_q4(a, b);
  else return rp_add(a, b);
}
template <int Q>
__device__ __forceinline__ RedPoint pdbl(const RedPoint& a) {
  if (H2G_RED_SKIP && !__any(!rp_is_identity(a))) return a;
  if constexpr (Q == 4) return rp_dbl_q4(a);
  else return rp_dbl(a);
}

// in LDS: T[0..len) holds one value per element, len = 2^K <= 512.  Afterwards T[0] is the
// total and T[2^b] (b < K) the sum over the elements with bit b of their index set.
// `workers`: the block's lanes (Q = 1) or quads (Q = 4); a level's items beyond them loop
template <int Q>
__device__ __forceinline__ void plane_fold(RedPoint* T, int K, uint32_t e, bool lead, uint32_t workers) {
  for (int k = 0; k < K; k++) {
    const uint32_t per = (uint32_t)k + 1, pairs = (1u << (K - 1 - k));
    for (uint32_t it = e; it < pairs * per; it += workers) {
      const uint32_t j = it / per, i = it % per;
      const uint32_t dst = (j << (k + 1)) + (i == 0 ? 0u : (1u << (i - 1))), src = dst + (1u << k);
      const RedPoint v = padd<Q>(T[dst], T[src]);
      if (lead) T[dst] = v;
    }
    __syncthreads();
  }
}

// level A, fused with rgroup: block b takes 2^LB groups g = 2^LB b + t, forms S_t, R_t like
// msm_rgroup_kernel, and writes planes[0][b] = sum S, planes[1 + p][b] = L_p (p < LB),
// planes[LB + 1][b] = T (the block's R total); planes[q] is (WB x nblk).  LB = 8 with a
// lane per group (full-size sets), LB = 6 with a quad per group (small sets: 4x the
// blocks, so the CUs fill)
// RGP: buckets per group (the dependent chain of 2 RGP additions before the planes); the
// planes then weight the groups by RGP g, hence e0 = log2(RGP) in the mid kernel
template <int Q, int LB, int RGP>
__global__ void __launch_bounds__((1 << LB) * Q)
msm_rgroup_plane_kernel(const RedPoint* __restrict__ B, uint32_t NB, uint32_t m1, uint32_t nblk,
                        RedPoint* __restrict__ planes) {
  H2G_SETPRIO(H2G_PRIO_RED);
  constexpr uint32_t BPL = 1u << LB;
  __shared__ RedPoint shT[BPL], shS[BPL];
  const uint32_t w = blockIdx.y, e = threadIdx.x / Q;
  const bool lead = (threadIdx.x % Q) == 0;
  const uint32_t g = blockIdx.x * BPL + e;
  const size_t ps = (size_t)gridDim.y * nblk;  // stride between planes
  const RedPoint* b = B + (size_t)w * NB;
  const bool b0 = blockIdx.x == 0 && blockIdx.y == 0, bl = blockIdx.x == gridDim.x - 1 && blockIdx.y == 0;
  RED_TS(b0, 0);
  RED_TS(bl, 4);
  RedPoint racc = rp_identity(), sacc = rp_identity();
  if (g < m1) {
#pragma unroll
    for (int t = RGP - 1; t >= 0; t--) {
      const uint32_t j = g * RGP + t;
      if (j < NB) racc = padd<Q>(racc, b[j]);
      sacc = t == RGP - 1 ? racc : padd<Q>(sacc, racc);
    }
  }
  if (lead) {
    shT[e] = racc;
    shS[e] = sacc;
  }
  __syncthreads();
  RED_TS(b0, 1);
  // the R tree and a plain S tree side by side: elements [0, 2^(LB-1-k)(k+1)) fold R at
  // level k, the next 2^(LB-1-k) fold S
  for (int k = 0; k < LB; k++) {
    const uint32_t per = (uint32_t)k + 1, pairs = 1u << (LB - 1 - k);
    if (e < pairs * per) {
      const uint32_t j = e / per, i = e % per;
      const uint32_t dst = (j << (k + 1)) + (i == 0 ? 0u : (1u << (i - 1))), src = dst + (1u << k);
      const RedPoint v = padd<Q>(shT[dst], shT[src]);
      if (lead) shT[dst] = v;
    } else if (e < pairs * (per + 1)) {
      const uint32_t j = e - pairs * per, dst = j << (k + 1);
      const RedPoint v = padd<Q>(shS[dst], shS[dst + (1u << k)]);
      if (lead) shS[dst] = v;
    }
    __syncthreads();
  }
  RED_TS(b0, 2);
  if (lead && e < LB + 2) {
    const RedPoint v = e == 0 ? shS[0] : (e <= LB ? shT[1u << (e - 1)] : shT[0]);
    planes[e * ps + (size_t)w * nblk + blockIdx.x] = v;
  }
  RED_TS(b0, 3);
  RED_TS(bl, 5);
}

// levels B and C, one launch (LB + 2 blocks per set): block q <= LB sums plane q over the
// nblk blocks; block LB + 1 folds the totals T by block index (nblk <= 2^RPK_MAX) --
// mid[q' * WB + w]: 0 = sum S, 1 + b = U_b (b < LB + K).  The last of a set's blocks to
// finish (device-scope counter, zeroed by the host) then scales U_b by 2^(b + e0), one
// quad per plane, and sums.
static constexpr int RPK_MAX = 9;  // block-index planes (LDS: 2^RPK_MAX points); above it (c = 22
                                   // sets) MSMs keep the rscale scheme
// threads per block: at 1024 the quad additions are held to 128 VGPRs and spill (136 B
// of scratch per lane in F29); at 512 they fit
#ifndef H2G_RPM_THREADS
#define H2G_RPM_THREADS 512
#endif
static constexpr uint32_t RPM_QUADS = H2G_RPM_THREADS / 4;
__global__ void __launch_bounds__(H2G_RPM_THREADS)
msm_rplane_mid_kernel(const RedPoint* __restrict__ planes, uint32_t nblk, int LB, int e0, RedPoint* __restrict__ mid,
                      uint32_t* __restrict__ done, G1xyzz* __restrict__ windows) {
  H2G_SETPRIO(H2G_PRIO_RED);
  __shared__ RedPoint sh[1 << RPK_MAX];
  __shared__ uint32_t last;
  const uint32_t q = blockIdx.x, w = blockIdx.y, e = threadIdx.x >> 2, WB = gridDim.y;
  const bool lead = (threadIdx.x & 3) == 0;
  const RedPoint* in = planes + (size_t)q * WB * nblk + (size_t)w * nblk;
  int K = 0;
  while ((1u << K) < nblk) K++;
  RED_TS(q == 0 && w == 0, 8);
  RED_TS(q == (uint32_t)LB + 1 && w == 0, 11);
  if (q <= (uint32_t)LB) {
    RedPoint acc = rp_identity();
    for (uint32_t i = e; i < nblk; i += RPM_QUADS) acc = padd<4>(acc, in[i]);
    if (lead) sh[e] = acc;
    __syncthreads();
    RED_TS(q == 0 && w == 0, 9);
    // the tree's levels above the filled entries would only add identities
    uint32_t h0 = 1;
    while (2 * h0 < (nblk < RPM_QUADS ? nblk : RPM_QUADS)) h0 <<= 1;
    for (uint32_t h = h0; h > 0; h >>= 1) {
      if (e < h) {
        const RedPoint v = padd<4>(sh[e], sh[e + h]);
        if (lead) sh[e] = v;
      }
      __syncthreads();
    }
    RED_TS(q == 0 && w == 0, 10);
    if (threadIdx.x == 0) mid[(size_t)q * WB + w] = sh[0];
  } else {
    for (uint32_t i = e; i < (1u << K); i += RPM_QUADS)
      if (lead) {
        if (i < nblk) sh[i] = ld_rp(in + i);
        else sh[i] = rp_identity();
      }
    __syncthreads();
    RED_TS(w == 0, 12);
    plane_fold<4>(sh, K, e, lead, RPM_QUADS);
    RED_TS(w == 0, 13);
    if (lead && e < (uint32_t)K) mid[(size_t)(1 + LB + e) * WB + w] = sh[1u << e];
    if (threadIdx.x == 0) mid[(size_t)(1 + LB + K) * WB + w] = sh[0];  // T
  }
  __syncthreads();  // this block's outputs are written
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&done[w], 1u) == (uint32_t)LB + 1u;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  RED_TS(w == 0, 14);
  const uint32_t np = (uint32_t)(LB + K);  // planes (<= 18)
  RedPoint x = rp_identity();
  if (e < np) {
    x = mid[(size_t)(1 + e) * WB + w];
    for (int i = 0; i < (int)e + e0; i++) x = pdbl<4>(x);
  } else if (e == np) {
    x = mid[w];
  }
  if (lead && e < 64) sh[e] = x;
  __syncthreads();
  RED_TS(w == 0, 15);
  uint32_t h0 = 1;  // np + 1 <= 2 h0 terms
  while (2 * h0 < np + 1) h0 <<= 1;
  for (uint32_t h = h0; h > 0; h >>= 1) {
    if (e < h) {
      const RedPoint v = padd<4>(sh[e], sh[e + h]);
      if (lead) sh[e] = v;
    }
    __syncthreads();
  }
  RED_TS(w == 0, 16);
  if (threadIdx.x == 0) windows[w] = rp_to_xyzz(sh[0]);  // the host finish reads G1xyzz
}

// fixed-base tables: table[w * stride + i] = [2^(offset of window w)] bases[i] -------
__global__ void __launch_bounds__(MSM_THREADS)
msm_precompute_kernel(const G1Affine* __restrict__ bases, size_t n, int W, size_t stride,
                      G1Affine* __restrict__ table) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1Affine p = bases[i];
  table[i] = p;
  G1xyzz x = G1xyzz::from_affine(p);
  for (int w = 1; w < W; w++) {
    for (int d = 0; d < fb_width(W, w - 1); d++) x = xyzz_dbl(x);
    table[(size_t)w * stride + i] = xyzz_to_affine_by(x);
  }
}

// 8. final Horner over windows -------------------------------------------------------
__host__ __device__ G1Affine msm_combine_windows(const G1xyzz* windows, int W, int c) {
  G1xyzz acc = windows[W - 1];
  for (int w = W - 2; w >= 0; w--) {
    for (int d = 0; d < c; d++) acc = xyzz_dbl(acc);
    acc = xyzz_add(acc, windows[w]);
  }
  return xyzz_to_affine(acc);
}

__global__ void msm_final_kernel(const G1xyzz* __restrict__ windows, int W, int c, G1Affine* out) {
  H2G_SETPRIO(H2G_PRIO_RED);
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  *out = msm_combine_windows(windows, W, c);
}

G1Affine msm_windows_host_finish(const G1xyzz* h_windows, int W, int c) {
  return msm_combine_windows(h_windows, W, c);
}

// ------------------------------------------------------------------------------------
static hipError_t grow(void** p, size_t bytes) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  return hipMalloc(p, bytes > 0 ? bytes : 16);
}

void msm_free(MsmWorkspace* ws) {
  void** ptrs[] = {&ws->ent, &ws->vals_out, &ws->item_off, &ws->item_bucket, &ws->partials,
                   &ws->buckets, &ws->segs, &ws->windows, &ws->result, &ws->total_items, &ws->sort_tmp};
  for (void** p : ptrs) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
  }
  for (auto& c : ws->cap) c = 0;
  ws->sort_tmp_bytes = 0;
  ws->sort_kcap = 0;
}

#define H2G_TRY(x)                      \
  do {                                  \
    hipError_t _e = (x);                \
    if (_e != hipSuccess) return _e;    \
  } while (0)

#ifndef H2G_MSM_ADAPT  // A/B builds: 0 = the host's chunk length always (msm_chunk_len_dev off)
#define H2G_MSM_ADAPT 1
#endif
uint32_t msm_chunk_len(size_t total, size_t nbt) {
  // ~4 resident waves per SIMD x 256 CUs x 64 lanes, several rounds deep ...
  uint64_t L = total / (256ull * 4 * 4 * 64 * 4);
  // ... but at least a quarter of the mean bucket, so that a bucket spans few chunks and
  // the fixup sums it in one thread (small MSMs: 2^19 points at c = 17 put ~120 entries
  // in each of 2^16 buckets; L = 8 sent every bucket through the big-item path, 0.74 ms),
  // while >= 2^17 threads remain
  const uint64_t quarter = nbt ? total / (4 * nbt) : 0;
  const uint64_t cap = total >> 17;
  if (L < quarter) L = quarter < cap ? quarter : (cap > L ? cap : L);
  if (L < 8) L = 8;
  if (L > 128) L = 128;
  return (uint32_t)L;
}

// quad-cooperative group kernels (rscale scheme) when the groups leave SIMDs idle: up to
// 32768 groups over all sets (MSMs up to 2^21 points).  At 65536 groups (2^22) the quad
// kernels lose even for a lone MSM: reduction 1.07 vs 0.72 ms, C3 k = 22 proof 94.1-94.3
// vs 90.2-90.3 ms (profiles/r02/ab_q4/).  Quad fixup up to 2^15 buckets (2^16, the
// 2^19-point slabs: the lane form is faster).
static constexpr size_t RED_Q4_MAX = 32768;
#ifndef H2G_PLANE_LB_SMALL  // A/B builds (tools/build_variant.py -DH2G_PLANE_LB_SMALL=8)
#define H2G_PLANE_LB_SMALL 6
#endif
static constexpr int kSmallLB = H2G_PLANE_LB_SMALL;
#ifndef H2G_PLANE_RGP_LARGE  // buckets per group of the lane-per-group plane kernel (large sets)
#define H2G_PLANE_RGP_LARGE 8
#endif
static constexpr int kLargeRGP = H2G_PLANE_RGP_LARGE;
static constexpr uint32_t FIXUP_Q4_MAX = 32768;

static hipError_t msm_pipeline(const MsmScalarList& list, int nbatch, const G1Affine* d_bases, size_t n, int c,
                               int W, int fixed, size_t stride, MsmWorkspace* ws, uint32_t item_len, G1Affine* d_out,
                               hipStream_t st, MsmPhaseEvents* prof) {
#define H2G_PHASE(i) \
  if (prof) H2G_TRY(hipEventRecord(prof->ev[i], st))
  const uint32_t NB = 1u << (c - 1);
  if (nbatch < 1 || nbatch > MSM_MAX_BATCH || (!fixed && nbatch != 1)) return hipErrorInvalidValue;
  const int WB = fixed ? nbatch : W;  // bucket sets
  const uint32_t nbt = (uint32_t)WB * NB;
  const size_t total = n * (size_t)W * nbatch;
  if (total >= 0x80000000ull) return hipErrorInvalidValue;  // u32 positions in the sorted array
  // buckets most windows can reach (fixed-base: 2^(base width - 1) of the balanced widths)
  const size_t nb_eff = (size_t)WB << ((fixed ? 255 / W : c) - 1);
  // the host's chunk length; the device may pick a shorter one once the entries are
  // counted (msm_chunk_len_dev), so everything chunk-sized takes the larger count
  const uint32_t L = item_len > 0 ? item_len : msm_chunk_len(total, nb_eff);
  const MsmChunkRule rule{L, item_len > 0 || !H2G_MSM_ADAPT ? 0u : 1u, (uint64_t)total, (uint64_t)nb_eff};
  const size_t nchunks = msm_chunk_cap(rule);
  const uint32_t m1 = (NB + RG - 1) / RG;
  const bool red_q4 = (size_t)m1 * WB <= RED_Q4_MAX;
  const uint32_t nblk = red_q4 ? (m1 + Q4_GROUPS - 1) / Q4_GROUPS : (m1 + MSM_THREADS - 1) / MSM_THREADS;
  // bit planes.  Small sets (<= 2^18 buckets over all sets, e.g. the 2^16 of a 2^19-point
  // slab): quad-cooperative, 256 groups per block, and the fewest buckets per group (rgp)
  // that keep the groups within 2^16 (4 waves per SIMD) -- latency-bound, the reduction
  // is a dependent chain of ~2 rgp + 8 + 9 + log2(NB) point operations, so the group chain
  // goes first (2^16 buckets: rgp = 1; 0.38 -> 0.33 ms at 2^19 points).  Larger sets: a
  // lane per group of 8 (the quads' 1.3x issue cost loses there: 0.62 -> 0.71 ms at 2^19
  // buckets; groups of 4: slower).
  // Small sets use blocks of 64 groups (256 threads, plane_lb = 6): a block's tree levels
  // are issue-bound on its CU (a level's quads all add at once), so 1024-thread blocks of
  // 256 groups left 4 waves per SIMD on few CUs (2^14 buckets: 64 CUs, ~13 us per level);
  // 4x the blocks spread the same levels over the chip.  The block index then needs 2 more
  // bits (<= RPK_MAX): at most 32768 groups per set.
  int rgp = 8, plane_q = 4, plane_lb = 8;
  if ((size_t)NB * WB <= (1u << 18)) {
    plane_lb = kSmallLB;
    for (rgp = 1; rgp < 8; rgp *= 2) {
      const size_t g = (NB + rgp - 1) / rgp;
      if (g * WB <= 65536 && g <= ((size_t)1 << (RPK_MAX + kSmallLB))) break;
    }
  } else {
    plane_q = 1;
    rgp = kLargeRGP;
  }
  const uint32_t m1p = (NB + rgp - 1) / rgp;                         // plane groups per set
  const uint32_t nblk_p = (m1p + (1u << plane_lb) - 1) >> plane_lb;  // plane kernels' blocks
  // bit planes unless the block index needs more than RPK_MAX bits (sets of > 2^17
  // groups, e.g. c = 22): those keep the rscale scheme
  const bool red_plane = nblk_p <= (1u << RPK_MAX);
  // grow-only workspace: MSMs of slightly different shapes (e.g. n and n - 1 points, so
  // another chunk length) reuse it instead of reallocating (~2 ms of host stall each)
  struct Need {
    void** p;
    size_t bytes;
  };
  const size_t icap = msm_big_items_cap(nchunks), mcap = msm_big_multi_cap(nchunks);
  // bucket partition geometry: keys < nbt, fine bits fb, coarse bins nbt >> fb.  Fine bits
  // (the fine pass's fan-out per tile): 10 -- 2x the coarse bins of 11 but half the
  // per-tile key runs; interleaved on one box the k = 22 proof took 86.5-86.8 ms vs
  // 86.8-87.3 ms at 11 (8, 9: slower coarse pass)
  int key_bits = 1;
  while ((1ull << key_bits) < (uint64_t)nbt) key_bits++;
  int fb = key_bits < 10 ? key_bits : 10;
  while (fb < FB_MAX && (((uint64_t)nbt + (1ull << fb) - 1) >> fb) > COARSE_MAX) fb++;
  // ent (the coarse-binned entries) is dead once the partition has run: with H2G_ACC29 it
  // holds the accumulation's whole buckets (raw F29) until the fixup converts them
  const size_t whole_bytes = H2G_ACC29 ? (size_t)nbt * sizeof(AccPoint) : 0;
  const Need need[10] = {{&ws->ent, std::max(total * 8, whole_bytes)},
                         {&ws->vals_out, total * 4},
                         {&ws->item_bucket, icap * sizeof(MsmBigItem)},    // big-bucket items
                         {&ws->partials, 2 * nchunks * sizeof(AccPoint)},  // boundary slots
                         {&ws->buckets, (size_t)nbt * sizeof(RedPoint)},
                         {&ws->segs, std::max<size_t>((size_t)2 * m1 + nblk, 10 * (size_t)nblk_p + 32) * WB *
                                         sizeof(RedPoint)},
                         {&ws->windows, (size_t)(W > WB ? W : WB) * sizeof(G1xyzz)},
                         // [0] items, [1] multi-item buckets, [4 ..] the accumulation's repair list
                         {&ws->result, 16 + 4 * (1 + (size_t)MSM_REPAIR_CAP)},
                         {&ws->item_off, mcap * sizeof(uint4)},          // multi-item buckets
                         {&ws->total_items, icap * sizeof(RedPoint)}};     // items' partial sums
  for (int b = 0; b < 10; b++)
    if (need[b].bytes > ws->cap[b]) {
      H2G_TRY(grow(need[b].p, need[b].bytes));
      ws->cap[b] = need[b].bytes;
    }
  ws->last_c = c;
  ws->last_W = WB;
  uint32_t* vals_out = (uint32_t*)ws->vals_out;
  uint32_t* counters = (uint32_t*)ws->result;
  MsmBigItem* items = (MsmBigItem*)ws->item_bucket;
  uint4* multi = (uint4*)ws->item_off;
  RedPoint* ipart = (RedPoint*)ws->total_items;
  RedPoint* buckets = (RedPoint*)ws->buckets;
  AccPoint* bnd = (AccPoint*)ws->partials;
  AccPoint* whole = H2G_ACC29 ? (AccPoint*)ws->ent : (AccPoint*)buckets;  // the accumulation's whole buckets
  RedPoint* rS = (RedPoint*)ws->segs;  // rscale scheme: group sums, group weights, block sums
  RedPoint* rR = rS + (size_t)WB * m1;
  RedPoint* rP = rR + (size_t)WB * m1;

  const uint32_t ncoarse = (uint32_t)(((uint64_t)nbt + (1ull << fb) - 1) >> fb);
  if (ncoarse > COARSE_MAX) return hipErrorInvalidValue;
  const uint32_t kblocks = (nbt + 1023) / 1024;
  constexpr int RDONE_MAX = 256;  // bucket sets: W <= 128 windows (c >= 2), or nbatch <= MSM_MAX_BATCH
  if (WB > RDONE_MAX) return hipErrorInvalidValue;
  // scratch (u32), laid out for a per-key capacity kcap >= nbt so that the counts stay at
  // fixed places: ccount | coff | ccursor | total | rdone | kbsum | kboff | kcount | koff
  // (kcap + 1) | kcursor.  Zeroed when allocated; the scans zero ccount / kcount after
  // reading them, so no MSM needs a fill.
  if ((size_t)nbt > ws->sort_kcap) {
    const size_t kcap = nbt, kbmax = (kcap + 1023) / 1024;
    const size_t words = 3 * (size_t)COARSE_MAX + 16 + RDONE_MAX + 2 * kbmax + 3 * kcap + 1;
    H2G_TRY(grow(&ws->sort_tmp, words * 4));
    H2G_TRY(hipMemsetAsync(ws->sort_tmp, 0, words * 4, st));
    ws->sort_tmp_bytes = words * 4;
    ws->sort_kcap = kcap;
  }
  const size_t kcap = ws->sort_kcap, kbmax = (kcap + 1023) / 1024;
  uint32_t* ccount = (uint32_t*)ws->sort_tmp;
  uint32_t* coff = ccount + COARSE_MAX;
  uint32_t* ccursor = coff + COARSE_MAX;
  uint32_t* d_total = ccursor + COARSE_MAX;
  uint32_t* rdone = d_total + 16;  // plane reduction: finished blocks per set
  uint32_t* kbsum = rdone + RDONE_MAX;
  uint32_t* kboff = kbsum + kbmax;
  uint32_t* kcount = kboff + kbmax;
  uint32_t* koff = kcount + kcap;
  uint32_t* kcursor = koff + kcap + 1;

  const int T = MSM_THREADS;
  H2G_PHASE(0);
  {  // rounds 1 and 2 (msm_part.hip); phase event 1 between them
    MsmPartArgs pa;
    pa.list = list;
    pa.nbatch = nbatch;
    pa.n = n;
    pa.c = c;
    pa.W = W;
    pa.NB = NB;
    pa.fixed = fixed;
    pa.stride = stride;
    pa.total = total;
    pa.fb = fb;
    pa.ncoarse = ncoarse;
    pa.nbt = nbt;
    pa.kblocks = kblocks;
    pa.ccount = ccount;
    pa.coff = coff;
    pa.ccursor = ccursor;
    pa.d_total = d_total;
    pa.kbsum = kbsum;
    pa.kboff = kboff;
    pa.kcount = kcount;
    pa.koff = koff;
    pa.kcursor = kcursor;
    pa.ent = (uint64_t*)ws->ent;
    pa.out = vals_out;
    pa.z = MsmZero{counters, rdone, (uint32_t)WB};
    pa.rule = rule;
    H2G_TRY(msm_partition(pa, st, prof));
  }
  H2G_PHASE(2);
  H2G_PHASE(3);
  H2G_TRY(msm_accumulate(d_bases, vals_out, koff, nbt, d_total, nchunks, whole, bnd, counters + 4, st));
  H2G_PHASE(4);
  if (nbt <= FIXUP_Q4_MAX)
    hipLaunchKernelGGL(msm_fixup_kernel<4>, dim3((unsigned)(((size_t)nbt * 4 + T - 1) / T)), dim3(T), 0, st,
                       (const AccPoint*)bnd, (const uint32_t*)koff, nbt, (const uint32_t*)d_total,
                       (const AccPoint*)whole, buckets, items, multi, counters);
  else
    hipLaunchKernelGGL(msm_fixup_kernel<1>, dim3((nbt + T - 1) / T), dim3(T), 0, st, (const AccPoint*)bnd,
                       (const uint32_t*)koff, nbt, (const uint32_t*)d_total, (const AccPoint*)whole, buckets, items,
                       multi, counters);
  hipLaunchKernelGGL(msm_big_item_kernel, dim3(MSM_BIG_BLOCKS), dim3(T), 0, st, (const AccPoint*)bnd,
                     (const uint32_t*)koff, (const uint32_t*)d_total, (const MsmBigItem*)items,
                     (const uint32_t*)counters, ipart, buckets);
  hipLaunchKernelGGL(msm_big_combine_kernel, dim3(MSM_BIG_BLOCKS / 4), dim3(T), 0, st, (const uint4*)multi,
                     (const uint32_t*)counters, (const RedPoint*)ipart, buckets);
  H2G_PHASE(5);
  if (red_plane) {  // bit planes (6a')
    RedPoint* planes = (RedPoint*)ws->segs;
    RedPoint* mid = planes + (size_t)(plane_lb + 2) * WB * nblk_p;
    int e0 = 0;
    while ((1 << e0) < rgp) e0++;
    const dim3 pg(nblk_p, (unsigned)WB), pb((unsigned)(plane_q << plane_lb));
    const RedPoint* bk = buckets;
    if (plane_q == 1)
      hipLaunchKernelGGL((msm_rgroup_plane_kernel<1, 8, kLargeRGP>), pg, pb, 0, st, bk, NB, m1p, nblk_p, planes);
    else if (rgp == 1)
      hipLaunchKernelGGL((msm_rgroup_plane_kernel<4, kSmallLB, 1>), pg, pb, 0, st, bk, NB, m1p, nblk_p, planes);
    else if (rgp == 2)
      hipLaunchKernelGGL((msm_rgroup_plane_kernel<4, kSmallLB, 2>), pg, pb, 0, st, bk, NB, m1p, nblk_p, planes);
    else if (rgp == 4)
      hipLaunchKernelGGL((msm_rgroup_plane_kernel<4, kSmallLB, 4>), pg, pb, 0, st, bk, NB, m1p, nblk_p, planes);
    else
      hipLaunchKernelGGL((msm_rgroup_plane_kernel<4, kSmallLB, 8>), pg, pb, 0, st, bk, NB, m1p, nblk_p, planes);
    hipLaunchKernelGGL(msm_rplane_mid_kernel, dim3((unsigned)plane_lb + 2, (unsigned)WB), dim3(H2G_RPM_THREADS), 0, st,
                       (const RedPoint*)planes, nblk_p, plane_lb, e0, mid, rdone, (G1xyzz*)ws->windows);
  } else {
    if (red_q4)
      hipLaunchKernelGGL(msm_rgroup_q4_kernel, dim3((unsigned)(((size_t)m1 * 4 + T - 1) / T), (unsigned)WB),
                         dim3(T), 0, st, (const RedPoint*)buckets, NB, m1, rS, rR);
    else
      hipLaunchKernelGGL(msm_rgroup_kernel, dim3((m1 + T - 1) / T, (unsigned)WB), dim3(T), 0, st,
                         (const RedPoint*)buckets, NB, m1, rS, rR);
    if (red_q4)
      hipLaunchKernelGGL(msm_rscale_q4_kernel, dim3(nblk, (unsigned)WB), dim3(T), 0, st, (const RedPoint*)rS,
                         (const RedPoint*)rR, m1, rP, nblk);
    else
      hipLaunchKernelGGL(msm_rscale_kernel, dim3(nblk, (unsigned)WB), dim3(T), 0, st, (const RedPoint*)rS,
                         (const RedPoint*)rR, m1, rP, nblk);
    hipLaunchKernelGGL(msm_rfinal_q4_kernel, dim3((unsigned)WB), dim3(T), 0, st, (const RedPoint*)rP, nblk,
                       (G1xyzz*)ws->windows);
  }
  if (d_out && nbatch == 1)
    hipLaunchKernelGGL(msm_final_kernel, dim3(1), dim3(64), 0, st, (const G1xyzz*)ws->windows, WB, c, d_out);
  H2G_TRY(hipGetLastError());
  H2G_PHASE(6);
#undef H2G_PHASE
  return hipSuccess;
}

#ifdef H2G_RED_TIMING
extern "C" int h2g_dbg_red_ts(unsigned long long* out) {  // read, then clear
  static const unsigned long long zero[64] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_red_ts), sizeof(g_red_ts)) != hipSuccess) return 1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_red_ts), zero, sizeof(zero)) == hipSuccess ? 0 : 1;
}
#endif

hipError_t msm_run(const Fr* d_scalars, const G1Affine* d_bases, size_t n, MsmWorkspace* ws,
                   const MsmConfig& cfg, G1Affine* d_out, hipStream_t st, MsmPhaseEvents* prof) {
  const int c = cfg.c > 0 ? cfg.c : msm_choose_c(n);
  MsmScalarList list;
  list.p[0] = d_scalars;
  return msm_pipeline(list, 1, d_bases, n, c, msm_windows_for(c), 0, 0, ws, (uint32_t)cfg.item_len, d_out, st, prof);
}

int msm_choose_c_fixed(size_t n) {
  // one shared bucket set: cost ~ n W (sort + accumulate) + a few adds per bucket
  if (n < 4) return 2;
  int best_c = 2;
  double best = 1e300;
  for (int c = 2; c <= 22; c++) {
    const double cost = (double)msm_windows_for(c) * (double)n + 3.0 * (double)(1ull << (c - 1));
    if (cost < best * 0.98) {  // prefer smaller tables unless clearly cheaper
      best = cost;
      best_c = c;
    }
  }
  return best_c;
}

hipError_t msm_fixed_base_build(const G1Affine* d_bases, size_t n, int c, MsmFixedBase* fb, hipStream_t st) {
  if (c <= 0) c = msm_choose_c_fixed(n);
  const int W = msm_windows_for(c);
  if ((size_t)W * n >= 0x80000000ull) return hipErrorInvalidValue;  // 31-bit table index
  msm_fixed_base_free(fb);
  H2G_TRY(hipMalloc(&fb->table, (size_t)W * n * sizeof(G1Affine)));
  fb->n = n;
  fb->c = c;
  fb->W = W;
  hipLaunchKernelGGL(msm_precompute_kernel, dim3((unsigned)((n + MSM_THREADS - 1) / MSM_THREADS)), dim3(MSM_THREADS),
                     0, st, d_bases, n, W, n, fb->table);
  return hipGetLastError();
}

// prefix sums of points (the lookup commitments' prefix basis, prover.cpp): chunk scans of
// PFX_C points per thread at two levels, a serial scan of the top level (<= 1024 sums at
// 2^22 points), and the offsets added back
static constexpr uint32_t PFX_C = 64;
__global__ void __launch_bounds__(MSM_THREADS)
msm_prefix_chunks_kernel(const G1Affine* __restrict__ in, const G1xyzz* __restrict__ inx, size_t n,
                         G1xyzz* __restrict__ run, G1xyzz* __restrict__ tot) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, lo = t * PFX_C;
  if (lo >= n) return;
  const size_t hi = lo + PFX_C < n ? lo + PFX_C : n;
  G1xyzz acc = G1xyzz::identity();
  for (size_t i = lo; i < hi; i++) {
    acc = inx ? xyzz_add(acc, inx[i]) : xyzz_madd(acc, in[i]);
    run[i] = acc;
  }
  tot[t] = acc;
}
__global__ void msm_prefix_serial_kernel(G1xyzz* a, size_t m) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (size_t i = 1; i < m; i++) a[i] = xyzz_add(a[i - 1], a[i]);
}
// run[i] += tot[i / PFX_C - 1] (tot inclusive over the chunks); to affine into out if given
__global__ void __launch_bounds__(MSM_THREADS)
msm_prefix_add_kernel(G1xyzz* __restrict__ run, size_t n, const G1xyzz* __restrict__ tot, G1Affine* __restrict__ out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1xyzz v = run[i];
  const size_t c = i / PFX_C;
  if (c) v = xyzz_add(v, tot[c - 1]);
  if (out) out[i] = xyzz_to_affine_by(v);
  else run[i] = v;
}
hipError_t msm_prefix_points(const G1Affine* in, size_t n, G1Affine* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t t1 = (n + PFX_C - 1) / PFX_C, t2 = (t1 + PFX_C - 1) / PFX_C;
  G1xyzz* buf = nullptr;
  H2G_TRY(hipMalloc(&buf, (n + 2 * t1 + t2) * sizeof(G1xyzz)));
  G1xyzz *run1 = buf, *tot1 = run1 + n, *run2 = tot1 + t1, *tot2 = run2 + t1;
  const unsigned T = MSM_THREADS;
  auto grid = [&](size_t m) { return dim3((unsigned)((m + T - 1) / T)); };
  hipLaunchKernelGGL(msm_prefix_chunks_kernel, grid(t1), dim3(T), 0, st, in, (const G1xyzz*)nullptr, n, run1, tot1);
  hipLaunchKernelGGL(msm_prefix_chunks_kernel, grid(t2), dim3(T), 0, st, (const G1Affine*)nullptr,
                     (const G1xyzz*)tot1, t1, run2, tot2);
  hipLaunchKernelGGL(msm_prefix_serial_kernel, dim3(1), dim3(64), 0, st, tot2, t2);
  hipLaunchKernelGGL(msm_prefix_add_kernel, grid(t1), dim3(T), 0, st, run2, t1, (const G1xyzz*)tot2, (G1Affine*)nullptr);
  hipLaunchKernelGGL(msm_prefix_add_kernel, grid(n), dim3(T), 0, st, run1, n, (const G1xyzz*)run2, out);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(buf);
  return e;
}

void msm_fixed_base_free(MsmFixedBase* fb) {
  if (fb->table) (void)hipFree(fb->table);
  fb->table = nullptr;
  fb->n = 0;
}

hipError_t msm_run_fixed(const Fr* d_scalars, const MsmFixedBase& fb, size_t off, size_t n, MsmWorkspace* ws,
                         G1Affine* d_out, hipStream_t st, MsmPhaseEvents* prof) {
  if (off + n > fb.n) return hipErrorInvalidValue;
  MsmScalarList list;
  list.p[0] = d_scalars;
  return msm_pipeline(list, 1, fb.table + off, n, fb.c, fb.W, 1, fb.n, ws, 0, d_out, st, prof);
}

hipError_t msm_run_fixed_batch(const MsmScalarList& list, int nbatch, const MsmFixedBase& fb, size_t off, size_t n,
                               MsmWorkspace* ws, hipStream_t st, MsmPhaseEvents* prof) {
  if (off + n > fb.n) return hipErrorInvalidValue;
  return msm_pipeline(list, nbatch, fb.table + off, n, fb.c, fb.W, 1, fb.n, ws, 0, nullptr, st, prof);
}

}  // namespace h2g
