// prover_kernels.hip -- the create_proof kernels beyond MSM / NTT, for gfx950.
//
//   perm_*               permutation_commit     halo2_backend/src/plonk/permutation/prover.rs:103-171
//   chacha_random_poly   vanishing commit       halo2_backend/src/plonk/vanishing/prover.rs:57-81
//   evaluate_h           Evaluator::evaluate_h  halo2_backend/src/plonk/evaluation.rs:317-620
//                        (+ divide_by_vanishing_poly domain.rs:297-316, fused)
//   poly_eval_batch      eval_polynomial        halo2_backend/src/arithmetic.rs:57-82
//   kate_division        kate_division          halo2_backend/src/arithmetic.rs:101-120
//   lincomb              Polynomial Add/Sub/Mul<F> folds (shplonk/prover.rs:157-276,
//                        vanishing/prover.rs:166-176)
//   sigma_from_mapping   permutation build_pk   halo2_backend/src/plonk/permutation/keygen.rs:139-170
//   srs_lagrange_*       ParamsKZG::setup       halo2_backend/src/poly/kzg/commitment.rs:92-131
//   compress / lookup_* / shuffle_*   lookup/prover.rs:64-494, shuffle/prover.rs:36-206
//
// Everything here is integer modular arithmetic on 32-byte Montgomery elements;
// elementwise kernels are HBM-streaming grid-stride loops with 16-byte accesses.
#include <algorithm>

#include "f29.h"
#include "fr_io.h"
#include "poly.h"
#include "prover_kernels.h"
#include "transcript.h"

namespace h2g {

static constexpr int KT = 256;

static unsigned grid_1d(size_t n, int per_block = KT) {
  size_t g = (n + per_block - 1) / per_block;
  const size_t cap = 256 * 16;
  return (unsigned)(g < cap ? (g ? g : 1) : cap);
}

__device__ __forceinline__ Fr pw(const PowTable& t, uint64_t i) {
  const uint64_t mask = (1ull << t.bits) - 1;
  return ldf(t.lo + (i & mask)) * ldf(t.hi + (i >> t.bits));
}

// ------------------------------------------------------------------ permutation
__global__ void __launch_bounds__(KT) perm_den_kernel(Fr* __restrict__ out, size_t n, PermCols c, Fr beta, Fr gamma,
                                                      int init) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    Fr acc = init ? Fr::one() : ldf(out + r);
    for (int j = 0; j < c.m; j++) acc = acc * (beta * ldf(c.sigma[j] + r) + gamma + ldf(c.v[j] + r));
    stf(out + r, acc);
  }
}

hipError_t perm_denominators(Fr* out, size_t n, const PermCols& c, const Fr& beta, const Fr& gamma, bool init,
                             hipStream_t st) {
  hipLaunchKernelGGL(perm_den_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, out, n, c, beta, gamma, init ? 1 : 0);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) perm_num_kernel(Fr* __restrict__ mod, size_t n, PermCols c, Fr gamma,
                                                      PowTable om, size_t r0) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    const Fr w = pw(om, r0 + r);
    Fr acc = ldf(mod + r);
    for (int j = 0; j < c.m; j++) acc = acc * (c.beta_delta[j] * w + gamma + ldf(c.v[j] + r));
    stf(mod + r, acc);
  }
}

hipError_t perm_numerators(Fr* mod, size_t n, const PermCols& c, const Fr& gamma, const PowTable& omega,
                           hipStream_t st, size_t r0) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(perm_num_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, mod, n, c, gamma, omega, r0);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) perm_z_kernel(Fr* __restrict__ z, size_t n, int bf, const Fr* __restrict__ pre,
                                                    const Fr* __restrict__ last_z, const Fr* __restrict__ blind,
                                                    size_t lo, size_t hi) {
  const Fr lz = ldf(last_z);
  const size_t u = n - (size_t)bf;
  for (size_t i = lo + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < hi; i += (size_t)gridDim.x * blockDim.x) {
    Fr v;
    if (i >= u) v = ldf(blind + (i - u));
    else if (i == lo) v = lz;
    else v = lz * ldf(pre + i - 1);
    stf(z + i, v);
  }
}

hipError_t perm_z_assemble(Fr* z, size_t n, int bf, const Fr* prefix, const Fr* last_z, const Fr* blind_rows,
                           hipStream_t st, size_t lo, size_t hi) {
  if (hi > n) hi = n;
  if (lo >= hi) return hipSuccess;
  hipLaunchKernelGGL(perm_z_kernel, dim3(grid_1d(hi - lo)), dim3(KT), 0, st, z, n, bf, prefix, last_z, blind_rows,
                     lo, hi);
  return hipGetLastError();
}

// ------------------------------------------------------------------ vanishing random poly
// Chunk t of the polynomial is filled by its own ChaCha20Rng(seed_t); each Fr::random
// consumes exactly one 64-byte block, so element j of the chunk is block j.
// Elements [lo, hi) only: the SPMD multi-open tail draws a rank's coefficient slab.
__global__ void __launch_bounds__(KT) chacha_poly_kernel(Fr* __restrict__ out, size_t lo_i, size_t hi_i,
                                                         const uint32_t* __restrict__ seeds,
                                                         const uint64_t* __restrict__ off, int chunks) {
  for (size_t i = lo_i + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < hi_i;
       i += (size_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = chunks - 1;  // last t with off[t] <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    uint32_t key[8], w[16];
#pragma unroll
    for (int k = 0; k < 8; k++) key[k] = seeds[8 * lo + k];
    chacha20_block(key, (uint64_t)(i - off[lo]), w);
    stf(out + i, fr_from_u512(w));
  }
}

hipError_t chacha_random_poly(Fr* out, size_t n, const uint32_t* d_seeds, const uint64_t* d_offsets, int chunks,
                              hipStream_t st, size_t lo, size_t hi) {
  if (hi > n) hi = n;
  if (lo >= hi) return hipSuccess;
  hipLaunchKernelGGL(chacha_poly_kernel, dim3(grid_1d(hi - lo)), dim3(KT), 0, st, out, lo, hi, d_seeds, d_offsets,
                     chunks);
  return hipGetLastError();
}

// ------------------------------------------------------------------ evaluate_h
// One wave per block; the gate program's value slots live in LDS as
// slot-major [slot][lane] 32-byte elements (conflict-free 16-byte accesses).
static constexpr int EH_T = 64;
static constexpr int EH_MAX_SLOTS = 24;
int evaluate_h_max_slots() { return EH_MAX_SLOTS; }

// run one program segment for row idx: Horner of its expression values with `factor`,
// starting from `acc`
__device__ __forceinline__ Fr run_prog(const int4* __restrict__ prog, int2 seg, const Fr* __restrict__ consts,
                                       const Fr* const* __restrict__ cols, const int* __restrict__ rots, uint64_t idx,
                                       uint64_t rot_scale, uint64_t mask, Fr factor, Fr* sl, int lane,
                                       Fr acc = Fr::zero()) {
  for (int pc = seg.x; pc < seg.x + seg.y; pc++) {
    const int4 in = prog[pc];
    Fr v;
    switch (in.x) {
      case G_LOAD: {
        const uint64_t j = (idx + (uint64_t)((int64_t)rots[in.z] * (int64_t)rot_scale)) & mask;
        v = ldf(cols[in.z] + j);
        break;
      }
      case G_CONST: v = ldf(consts + in.z); break;
      case G_ADD: v = sl[in.z * EH_T + lane] + sl[in.w * EH_T + lane]; break;
      case G_SUB: v = sl[in.z * EH_T + lane] - sl[in.w * EH_T + lane]; break;
      case G_MUL: v = sl[in.z * EH_T + lane] * sl[in.w * EH_T + lane]; break;
      case G_NEG: v = neg(sl[in.z * EH_T + lane]); break;
      default:  // G_HORNER
        acc = acc * factor + sl[in.z * EH_T + lane];
        continue;
    }
    sl[in.y * EH_T + lane] = v;
  }
  return acc;
}

__global__ void __launch_bounds__(EH_T) evaluate_h_kernel(EvalHArgs a) {
  extern __shared__ uint4 eh_lds[];
  Fr* sl = reinterpret_cast<Fr*>(eh_lds);
  const int lane = threadIdx.x;
  const uint64_t emask = a.ext - 1;
  const uint64_t rend = a.rows ? a.row0 + a.rows : a.ext;
  for (uint64_t idx = a.row0 + blockIdx.x * (uint64_t)EH_T + lane; idx < rend; idx += (uint64_t)gridDim.x * EH_T) {
    Fr acc = run_prog(a.prog, a.gates, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, a.y, sl, lane,
                      a.acc_in ? ldf(a.acc_in + idx) : Fr::zero());
    const Fr l0 = ldf(a.l0 + idx);
    const Fr ll = ldf(a.l_last + idx);
    const Fr la = ldf(a.l_active + idx);
    const uint64_t r_next = (idx + a.rot_scale) & emask;
    if (a.nsets > 0) {
      const uint64_t r_last = (idx + (uint64_t)((int64_t)a.last_rot * (int64_t)a.rot_scale)) & emask;
      // l_0(X) * (1 - z_0(X))
      acc = acc * a.y + (Fr::one() - ldf(a.z[0] + idx)) * l0;
      // l_last(X) * (z_l(X)^2 - z_l(X))
      {
        const Fr zl = ldf(a.z[a.nsets - 1] + idx);
        acc = acc * a.y + (zl * zl - zl) * ll;
      }
      // l_0(X) * (z_i(X) - z_{i-1}(omega^(last) X))
      for (int s = 1; s < a.nsets; s++) acc = acc * a.y + (ldf(a.z[s] + idx) - ldf(a.z[s - 1] + r_last)) * l0;
      // l_active(X) * (z_i(omega X) prod(p + beta sigma + gamma) - z_i(X) prod(p + delta^j beta X + gamma))
      Fr cur = a.delta_start * pw(a.ext_omega, idx);
      for (int s = 0; s < a.nsets; s++) {
        const int c0 = s * a.chunk_len;
        const int c1 = c0 + a.chunk_len < a.P ? c0 + a.chunk_len : a.P;
        Fr left = ldf(a.z[s] + r_next);
        Fr right = ldf(a.z[s] + idx);
        for (int c = c0; c < c1; c++) {
          const Fr v = ldf(a.perm_v[c] + idx);
          left = left * (v + a.beta * ldf(a.sigma[c] + idx) + a.gamma);
          right = right * (v + cur + a.gamma);
          cur = cur * a.delta;
        }
        acc = acc * a.y + (left - right) * la;
      }
    }
    if (a.nlookups + a.nshuffles > 0) {
      const uint64_t r_prev = (idx - a.rot_scale) & emask;
      for (int l = 0; l < a.nlookups; l++) {  // evaluation.rs:486-558
        const EvalLookup lk = a.lookups[l];
        const Fr ci = run_prog(a.prog, lk.in, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, a.theta,
                               sl, lane);
        const Fr ct = run_prog(a.prog, lk.tab, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, a.theta,
                               sl, lane);
        const Fr table_value = (ci + a.beta) * (ct + a.gamma);
        const Fr z = ldf(lk.z + idx), ap = ldf(lk.ap + idx), sp = ldf(lk.sp + idx);
        const Fr ams = ap - sp;
        acc = acc * a.y + (Fr::one() - z) * l0;
        acc = acc * a.y + (z * z - z) * ll;
        acc = acc * a.y + (ldf(lk.z + r_next) * (ap + a.beta) * (sp + a.gamma) - z * table_value) * la;
        acc = acc * a.y + ams * l0;
        acc = acc * a.y + ams * (ap - ldf(lk.ap + r_prev)) * la;
      }
      for (int s = 0; s < a.nshuffles; s++) {  // evaluation.rs:561-620
        const EvalShuffle sh = a.shuffles[s];
        const Fr ci = run_prog(a.prog, sh.in, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, a.theta,
                               sl, lane) + a.gamma;
        const Fr cs = run_prog(a.prog, sh.sh, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, a.theta,
                               sl, lane) + a.gamma;
        const Fr z = ldf(sh.z + idx);
        acc = acc * a.y + (Fr::one() - z) * l0;
        acc = acc * a.y + (z * z - z) * ll;
        acc = acc * a.y + la * (ldf(sh.z + r_next) * cs - z * ci);
      }
    }
    stf(a.out + idx, a.divide ? acc * ldf(a.t_evals + (idx & a.t_mask)) : acc);
  }
}

// ---- evaluate_h in F29 (f29.h), H2G_EVALH29 ---------------------------------------------
// Loads enter as to29 (the element, value < 32 M; a shift, no product), products are
// f29.h's carry-free REDC, every sum and difference is normalised and reduced (reduce29,
// < 1.001 M), so no value exceeds 64 M before a reduction and every product input is a
// load / constant (< 32 M), a product (< 7 M) or a reduced sum: the columns stay far below
// 2^64.  The row's result leaves with one product against the storage integer of t(X)^-1
// (REDC(acc 2^261 e * t 2^256) = the storage form of acc * t, no conversion product).
#ifndef H2G_EVALH29  // A/B builds: 0 = the 8 x 32-bit kernel above
#define H2G_EVALH29 1
#endif
struct EvalH29Scalars {
  F29 theta, beta, gamma, y, delta_start, delta, one;
};
__device__ __forceinline__ F29 eh_ld(const Fr* p) { return to29(ldf(p)); }
__device__ __forceinline__ F29 eh_add(const F29& a, const F29& b) { return reduce29<FrParams>(norm29(add29(a, b))); }
__device__ __forceinline__ F29 eh_add3(const F29& a, const F29& b, const F29& c) {
  return reduce29<FrParams>(norm29(add29(add29(a, b), c)));
}
__device__ __forceinline__ F29 eh_sub(const F29& a, const F29& b) {
  return reduce29<FrParams>(norm29(sub29<FrParams, 64, 29>(a, b)));
}
__device__ __forceinline__ F29 eh_mul(const F29& a, const F29& b) { return mul29<FrParams>(a, b); }
// the same without the reduction, where the result goes straight into one product with a
// load, a constant or a product (tools/f29_bounds.py "evaluate_h": every such operand stays
// below 96 M, and the product brings it back below 20 M)
__device__ __forceinline__ F29 eh_addn(const F29& a, const F29& b) { return norm29(add29(a, b)); }
__device__ __forceinline__ F29 eh_add3n(const F29& a, const F29& b, const F29& c) {
  return norm29(add29(add29(a, b), c));
}
__device__ __forceinline__ F29 eh_subn(const F29& a, const F29& b) { return norm29(sub29<FrParams, 64, 29>(a, b)); }
// acc * f + v
__device__ __forceinline__ F29 eh_horner(const F29& acc, const F29& f, const F29& v) {
  return eh_add(mul29<FrParams>(acc, f), v);
}

// slots in LDS limb-major: word (slot, limb, lane) -- nine conflict-free ds_read_b32 per value
__device__ __forceinline__ F29 eh_slot_ld(const uint32_t* sl, int slot, int lane) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = sl[(slot * 9 + i) * EH_T + lane];
  return r;
}
__device__ __forceinline__ void eh_slot_st(uint32_t* sl, int slot, int lane, const F29& v) {
#pragma unroll
  for (int i = 0; i < 9; i++) sl[(slot * 9 + i) * EH_T + lane] = v.l[i];
}

__device__ __forceinline__ F29 run_prog29(const int4* __restrict__ prog, int2 seg, const Fr* __restrict__ consts,
                                          const Fr* const* __restrict__ cols, const int* __restrict__ rots,
                                          uint64_t idx, uint64_t rot_scale, uint64_t mask, const F29& factor,
                                          uint32_t* sl, int lane, F29 acc) {
  for (int pc = seg.x; pc < seg.x + seg.y; pc++) {
    const int4 in = prog[pc];
    F29 v;
    switch (in.x) {
      case G_LOAD: {
        const uint64_t j = (idx + (uint64_t)((int64_t)rots[in.z] * (int64_t)rot_scale)) & mask;
        v = eh_ld(cols[in.z] + j);
        break;
      }
      case G_CONST: v = eh_ld(consts + in.z); break;
      case G_ADD: v = eh_add(eh_slot_ld(sl, in.z, lane), eh_slot_ld(sl, in.w, lane)); break;
      case G_SUB: v = eh_sub(eh_slot_ld(sl, in.z, lane), eh_slot_ld(sl, in.w, lane)); break;
      case G_MUL: v = eh_mul(eh_slot_ld(sl, in.z, lane), eh_slot_ld(sl, in.w, lane)); break;
      case G_NEG: v = eh_sub(F29{}, eh_slot_ld(sl, in.z, lane)); break;
      default:  // G_HORNER
        acc = eh_horner(acc, factor, eh_slot_ld(sl, in.z, lane));
        continue;
    }
    eh_slot_st(sl, in.y, lane, v);
  }
  return acc;
}

__global__ void __launch_bounds__(EH_T) evaluate_h29_kernel(EvalHArgs a, EvalH29Scalars k) {
  extern __shared__ uint4 eh_lds[];
  uint32_t* sl = reinterpret_cast<uint32_t*>(eh_lds);
  const int lane = threadIdx.x;
  const uint64_t emask = a.ext - 1;
  const uint64_t rend = a.rows ? a.row0 + a.rows : a.ext;
  const F29 zero29 = F29{};
  for (uint64_t idx = a.row0 + blockIdx.x * (uint64_t)EH_T + lane; idx < rend; idx += (uint64_t)gridDim.x * EH_T) {
    F29 acc = run_prog29(a.prog, a.gates, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, k.y, sl, lane,
                         a.acc_in ? reduce29<FrParams>(to29(ldf(a.acc_in + idx))) : zero29);
    const F29 l0 = eh_ld(a.l0 + idx);
    const F29 ll = eh_ld(a.l_last + idx);
    const F29 la = eh_ld(a.l_active + idx);
    const uint64_t r_next = (idx + a.rot_scale) & emask;
    if (a.nsets > 0) {
      const uint64_t r_last = (idx + (uint64_t)((int64_t)a.last_rot * (int64_t)a.rot_scale)) & emask;
      // l_0(X) * (1 - z_0(X))
      acc = eh_horner(acc, k.y, eh_mul(eh_subn(k.one, eh_ld(a.z[0] + idx)), l0));
      // l_last(X) * (z_l(X)^2 - z_l(X))
      {
        const F29 zl = eh_ld(a.z[a.nsets - 1] + idx);
        acc = eh_horner(acc, k.y, eh_mul(eh_subn(eh_mul(zl, zl), zl), ll));
      }
      // l_0(X) * (z_i(X) - z_{i-1}(omega^(last) X))
      for (int s = 1; s < a.nsets; s++)
        acc = eh_horner(acc, k.y, eh_mul(eh_subn(eh_ld(a.z[s] + idx), eh_ld(a.z[s - 1] + r_last)), l0));
      // l_active(X) * (z_i(omega X) prod(p + beta sigma + gamma) - z_i(X) prod(p + delta^j beta X + gamma))
      const uint64_t pmask = (1ull << a.ext_omega.bits) - 1;
      F29 cur = eh_mul(k.delta_start, eh_mul(eh_ld(a.ext_omega.lo + (idx & pmask)),
                                             eh_ld(a.ext_omega.hi + (idx >> a.ext_omega.bits))));
      for (int s = 0; s < a.nsets; s++) {
        const int c0 = s * a.chunk_len;
        const int c1 = c0 + a.chunk_len < a.P ? c0 + a.chunk_len : a.P;
        F29 left = eh_ld(a.z[s] + r_next);
        F29 right = eh_ld(a.z[s] + idx);
        for (int c = c0; c < c1; c++) {
          const F29 v = eh_ld(a.perm_v[c] + idx);
          left = eh_mul(left, eh_add3n(v, eh_mul(k.beta, eh_ld(a.sigma[c] + idx)), k.gamma));
          right = eh_mul(right, eh_add3n(v, cur, k.gamma));
          if (c + 1 < a.P) cur = eh_mul(cur, k.delta);  // delta^j beta X for the next column (none after the last)
        }
        acc = eh_horner(acc, k.y, eh_mul(eh_subn(left, right), la));
      }
    }
    if (a.nlookups + a.nshuffles > 0) {
      const uint64_t r_prev = (idx - a.rot_scale) & emask;
      for (int l = 0; l < a.nlookups; l++) {  // evaluation.rs:486-558
        const EvalLookup lk = a.lookups[l];
        const F29 ci = run_prog29(a.prog, lk.in, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, k.theta,
                                  sl, lane, zero29);
        const F29 ct = run_prog29(a.prog, lk.tab, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask, k.theta,
                                  sl, lane, zero29);
        const F29 table_value = eh_mul(eh_addn(ci, k.beta), eh_addn(ct, k.gamma));
        const F29 z = eh_ld(lk.z + idx), ap = eh_ld(lk.ap + idx), sp = eh_ld(lk.sp + idx);
        const F29 ams = eh_subn(ap, sp);
        acc = eh_horner(acc, k.y, eh_mul(eh_subn(k.one, z), l0));
        acc = eh_horner(acc, k.y, eh_mul(eh_subn(eh_mul(z, z), z), ll));
        acc = eh_horner(acc, k.y,
                        eh_mul(eh_subn(eh_mul(eh_mul(eh_ld(lk.z + r_next), eh_addn(ap, k.beta)), eh_addn(sp, k.gamma)),
                                       eh_mul(z, table_value)),
                               la));
        acc = eh_horner(acc, k.y, eh_mul(ams, l0));
        acc = eh_horner(acc, k.y, eh_mul(eh_mul(ams, eh_subn(ap, eh_ld(lk.ap + r_prev))), la));
      }
      for (int s = 0; s < a.nshuffles; s++) {  // evaluation.rs:561-620
        const EvalShuffle sh = a.shuffles[s];
        const F29 ci = eh_addn(run_prog29(a.prog, sh.in, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask,
                                         k.theta, sl, lane, zero29),
                              k.gamma);
        const F29 cs = eh_addn(run_prog29(a.prog, sh.sh, a.consts, a.query_col, a.query_rot, idx, a.rot_scale, emask,
                                         k.theta, sl, lane, zero29),
                              k.gamma);
        const F29 z = eh_ld(sh.z + idx);
        acc = eh_horner(acc, k.y, eh_mul(eh_subn(k.one, z), l0));
        acc = eh_horner(acc, k.y, eh_mul(eh_subn(eh_mul(z, z), z), ll));
        acc = eh_horner(acc, k.y, eh_mul(la, eh_subn(eh_mul(eh_ld(sh.z + r_next), cs), eh_mul(z, ci))));
      }
    }
    // out = storage(acc * t(X)^-1) (or storage(acc)): one REDC against the raw storage integer
    const Fr tv = a.divide ? ldf(a.t_evals + (idx & a.t_mask)) : Fr::one();
    stf(a.out + idx, pack29<FrParams>(sub_m_if_ge29<FrParams>(mul29<FrParams>(acc, raw29(tv)))));
  }
}

hipError_t evaluate_h(const EvalHArgs& a, hipStream_t st) {
  if (a.n_slots > EH_MAX_SLOTS) return hipErrorInvalidValue;
  size_t blocks = ((a.rows ? a.rows : a.ext) + EH_T - 1) / EH_T;
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (H2G_EVALH29) {
    const size_t lds = (size_t)(a.n_slots > 0 ? a.n_slots : 1) * EH_T * 9 * 4;
    EvalH29Scalars k;
    k.theta = storage_to_f29<FrParams>(a.theta);
    k.beta = storage_to_f29<FrParams>(a.beta);
    k.gamma = storage_to_f29<FrParams>(a.gamma);
    k.y = storage_to_f29<FrParams>(a.y);
    k.delta_start = storage_to_f29<FrParams>(a.delta_start);
    k.delta = storage_to_f29<FrParams>(a.delta);
    k.one = one29v<FrParams>();
    hipLaunchKernelGGL(evaluate_h29_kernel, dim3((unsigned)blocks), dim3(EH_T), lds, st, a, k);
  } else {
    const size_t lds = (size_t)(a.n_slots > 0 ? a.n_slots : 1) * EH_T * sizeof(Fr);
    hipLaunchKernelGGL(evaluate_h_kernel, dim3((unsigned)blocks), dim3(EH_T), lds, st, a);
  }
  return hipGetLastError();
}

__global__ void __launch_bounds__(EH_T) compress_kernel(CompressArgs a) {
  extern __shared__ uint4 eh_lds[];
  Fr* sl = reinterpret_cast<Fr*>(eh_lds);
  const int lane = threadIdx.x;
  const uint64_t mask = a.n - 1;
  for (uint64_t i = blockIdx.x * (uint64_t)EH_T + lane; i < a.n; i += (uint64_t)gridDim.x * EH_T)
    stf(a.out + i, run_prog(a.prog, a.seg, a.consts, a.load_col, a.load_rot, i, 1, mask, a.theta, sl, lane));
}

hipError_t compress_lagrange(const CompressArgs& a, hipStream_t st) {
  if (a.n_slots > EH_MAX_SLOTS) return hipErrorInvalidValue;
  const size_t lds = (size_t)(a.n_slots > 0 ? a.n_slots : 1) * EH_T * sizeof(Fr);
  size_t blocks = (a.n + EH_T - 1) / EH_T;
  if (blocks > 256 * 32) blocks = 256 * 32;
  hipLaunchKernelGGL(compress_kernel, dim3((unsigned)blocks), dim3(EH_T), lds, st, a);
  return hipGetLastError();
}

__global__ void __launch_bounds__(EH_T) compress_batch_kernel(CompressBatch a) {
  extern __shared__ uint4 eh_lds[];
  Fr* sl = reinterpret_cast<Fr*>(eh_lds);
  const int lane = threadIdx.x, b = blockIdx.y;
  const uint64_t mask = a.n - 1;
  for (uint64_t i = blockIdx.x * (uint64_t)EH_T + lane; i < a.n; i += (uint64_t)gridDim.x * EH_T)
    stf(a.out[b] + i, run_prog(a.prog, a.seg[b], a.consts, a.load_col[b], a.load_rot, i, 1, mask, a.theta, sl, lane));
}

hipError_t compress_lagrange_batch(const CompressBatch& a, hipStream_t st) {
  if (a.count <= 0) return hipSuccess;
  if (a.n_slots > EH_MAX_SLOTS || a.count > COMPRESS_BATCH_MAX) return hipErrorInvalidValue;
  const size_t lds = (size_t)(a.n_slots > 0 ? a.n_slots : 1) * EH_T * sizeof(Fr);
  size_t blocks = (a.n + EH_T - 1) / EH_T;
  if (blocks > 256 * 32) blocks = 256 * 32;
  hipLaunchKernelGGL(compress_batch_kernel, dim3((unsigned)blocks, (unsigned)a.count), dim3(EH_T), lds, st, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------ lookups / shuffles
__global__ void __launch_bounds__(KT) canon_kernel(const Fr* __restrict__ in, CanonKey* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const Fr c = to_canonical(ldf(in + i));
    CanonKey k;
#pragma unroll
    for (int j = 0; j < 8; j++) k.l[j] = c.l[j];
    out[i] = k;
  }
}
hipError_t fr_to_canon(const Fr* in, CanonKey* out, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(canon_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, in, out, n);
  return hipGetLastError();
}

// Radix keys: bits [s, s + 64) of the canonical value (bits past 255 read as zero) (monotone in the value while every
// value is below 2^(s + 64)); optionally the canonical values and the identity index;
// d_or[0..3] |= the values' 64-bit limbs (one atomic per limb per wave), from which the
// caller checks afterwards that the values fit the key window it chose.
__device__ __forceinline__ void lookup_keys_body(const Fr* __restrict__ in, size_t n, int s,
                                                 CanonKey* __restrict__ canon, uint64_t* __restrict__ key,
                                                 uint32_t* __restrict__ idx, unsigned long long* __restrict__ d_or,
                                                 uint64_t kmask, uint64_t tag) {
  uint64_t m[4] = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const Fr c = to_canonical(ldf(in + i));
    uint64_t v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[j] = (uint64_t)c.l[2 * j] | ((uint64_t)c.l[2 * j + 1] << 32);
      m[j] |= v[j];
    }
    const int w = s >> 6, b = s & 63;
    const uint64_t lo = w < 4 ? v[w] : 0, hi = w + 1 < 4 ? v[w + 1] : 0;
    if (key) key[i] = ((b ? (lo >> b) | (hi << (64 - b)) : lo) & kmask) | tag;
    if (idx) idx[i] = (uint32_t)i;
    if (canon) {
      CanonKey k;
#pragma unroll
      for (int j = 0; j < 8; j++) k.l[j] = c.l[j];
      canon[i] = k;
    }
  }
  // wave, then block reduction: one atomic per limb per block (same-address atomics
  // serialise at the memory side -- one per wave cost ~0.15 ms at 2^18)
  __shared__ uint64_t sm[KT / 64][4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m[j] |= __shfl_xor(m[j], o);
  }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int j = 0; j < 4; j++) sm[threadIdx.x >> 6][j] = m[j];
  __syncthreads();
  if (threadIdx.x < 4) {
    uint64_t v = 0;
#pragma unroll
    for (int w = 0; w < KT / 64; w++) v |= sm[w][threadIdx.x];
    if (v) atomicOr(&d_or[threadIdx.x], (unsigned long long)v);
  }
}
__global__ void __launch_bounds__(KT) lookup_keys_kernel(const Fr* __restrict__ in, size_t n, int s,
                                                         CanonKey* __restrict__ canon, uint64_t* __restrict__ key,
                                                         uint32_t* __restrict__ idx,
                                                         unsigned long long* __restrict__ d_or, uint64_t kmask,
                                                         uint64_t tag) {
  lookup_keys_body(in, n, s, canon, key, idx, d_or, kmask, tag);
}
// item b = blockIdx.y: column b.g[...] of the batch (canon / key / idx at g u, tag g << kbits)
__global__ void __launch_bounds__(KT) lookup_keys_batch_kernel(LookupKeysBatch b) {
  const int t = blockIdx.y;
  const size_t g = (size_t)b.g[t];
  lookup_keys_body(b.in[t], b.n, b.s[t], b.canon + g * b.n, b.key + g * b.n, b.idx + g * b.n, b.d_or[t], b.kmask,
                   (uint64_t)g << b.kbits);
}
hipError_t lookup_keys_batch(const LookupKeysBatch& b, hipStream_t st) {
  if (b.count <= 0 || b.n == 0) return hipSuccess;
  if (b.count > LOOKUP_KEYS_BATCH_MAX) return hipErrorInvalidValue;
  for (int t = 0; t < b.count; t++)
    if (b.s[t] < 0 || b.s[t] > 255) return hipErrorInvalidValue;
  const unsigned g = grid_1d(b.n) < 512 ? grid_1d(b.n) : 512;
  hipLaunchKernelGGL(lookup_keys_batch_kernel, dim3(g, (unsigned)b.count), dim3(KT), 0, st, b);
  return hipGetLastError();
}

hipError_t lookup_keys(const Fr* in, size_t n, int s, CanonKey* canon, uint64_t* key, uint32_t* idx,
                       unsigned long long* d_or, hipStream_t st, int kbits, uint64_t tag) {
  if (n == 0) return hipSuccess;
  if (s < 0 || s > 255 || kbits < 1 || kbits > 64) return hipErrorInvalidValue;
  const uint64_t kmask = kbits == 64 ? ~0ull : (1ull << kbits) - 1;
  // at most 512 blocks (grid-stride): 512 x 4 atomics
  const unsigned g = grid_1d(n) < 512 ? grid_1d(n) : 512;
  hipLaunchKernelGGL(lookup_keys_kernel, dim3(g), dim3(KT), 0, st, in, n, s, canon, key, idx, d_or, kmask, tag);
  return hipGetLastError();
}

// out[i] = canon[idx[i]]; *unsorted |= 1 where out[i + 1] < out[i] (the key window
// tied two different values out of order: the caller falls back to the full sort)
__global__ void __launch_bounds__(KT) lookup_gather_kernel(const CanonKey* __restrict__ canon,
                                                           const uint32_t* __restrict__ idx, size_t u,
                                                           CanonKey* __restrict__ out,
                                                           unsigned long long* __restrict__ unsorted) {
  const CanonLess less;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < u; i += (size_t)gridDim.x * blockDim.x) {
    const CanonKey v = canon[idx[i]];
    out[i] = v;
    if (i + 1 < u && less(canon[idx[i + 1]], v)) atomicOr(unsorted, 1ull);
  }
}
hipError_t lookup_gather(const CanonKey* canon, const uint32_t* idx, size_t u, CanonKey* out,
                         unsigned long long* unsorted, hipStream_t st) {
  if (u == 0) return hipSuccess;
  hipLaunchKernelGGL(lookup_gather_kernel, dim3(grid_1d(u)), dim3(KT), 0, st, canon, idx, u, out, unsorted);
  return hipGetLastError();
}
__global__ void __launch_bounds__(KT) key64_expand_kernel(const uint64_t* __restrict__ in, CanonKey* __restrict__ out,
                                                          size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t k = in[i];
    CanonKey c;
    c.l[0] = (uint32_t)k;
    c.l[1] = (uint32_t)(k >> 32);
#pragma unroll
    for (int j = 2; j < 8; j++) c.l[j] = 0;
    out[i] = c;
  }
}
hipError_t key64_expand(const uint64_t* in, CanonKey* out, size_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(key64_expand_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, in, out, n);
  return hipGetLastError();
}

__device__ __forceinline__ bool ck_eq(const CanonKey& a, const CanonKey& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.l[i] ^ b.l[i];
  return x == 0;
}

__global__ void __launch_bounds__(KT) lookup_mark_kernel(const CanonKey* __restrict__ a, const CanonKey* __restrict__ t,
                                                         size_t u, uint8_t* __restrict__ rep_flag,
                                                         uint8_t* __restrict__ left_flag, uint32_t* __restrict__ fail) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < u; r += (size_t)gridDim.x * blockDim.x) {
    const CanonKey v = a[r];
    const bool start = r == 0 || !ck_eq(v, a[r - 1]);
    rep_flag[r] = start ? 0 : 1;
    if (!start) continue;
    size_t lo = 0, hi = u;  // lower_bound
    const CanonLess less;
    while (lo < hi) {
      const size_t mid = (lo + hi) >> 1;
      if (less(t[mid], v)) lo = mid + 1;
      else hi = mid;
    }
    if (lo < u && ck_eq(t[lo], v)) left_flag[lo] = 0;
    else atomicAdd(fail, 1u);
  }
}
hipError_t lookup_mark(const CanonKey* a, const CanonKey* t, size_t u, uint8_t* rep_flag, uint8_t* left_flag,
                       uint32_t* fail, hipStream_t st) {
  if (u == 0) return hipSuccess;
  hipLaunchKernelGGL(lookup_mark_kernel, dim3(grid_1d(u)), dim3(KT), 0, st, a, t, u, rep_flag, left_flag, fail);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) lookup_assign_kernel(const CanonKey* __restrict__ a,
                                                           const uint8_t* __restrict__ rep_flag, size_t u,
                                                           Fr* __restrict__ ap, Fr* __restrict__ sp) {
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < u; r += (size_t)gridDim.x * blockDim.x) {
    Fr c;
#pragma unroll
    for (int j = 0; j < 8; j++) c.l[j] = a[r].l[j];
    const Fr m = from_canonical(c);
    stf(ap + r, m);
    if (!rep_flag[r]) stf(sp + r, m);
  }
}
hipError_t lookup_assign(const CanonKey* a, const uint8_t* rep_flag, size_t u, Fr* ap, Fr* sp, hipStream_t st) {
  if (u == 0) return hipSuccess;
  hipLaunchKernelGGL(lookup_assign_kernel, dim3(grid_1d(u)), dim3(KT), 0, st, a, rep_flag, u, ap, sp);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) lookup_scatter_kernel(const CanonKey* __restrict__ L,
                                                            const uint32_t* __restrict__ R,
                                                            const uint32_t* __restrict__ d_nrep, size_t cap,
                                                            Fr* __restrict__ sp) {
  const size_t nrep = *d_nrep;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrep && i < cap;
       i += (size_t)gridDim.x * blockDim.x) {
    Fr c;
#pragma unroll
    for (int j = 0; j < 8; j++) c.l[j] = L[i].l[j];
    stf(sp + R[nrep - 1 - i], from_canonical(c));
  }
}
hipError_t lookup_scatter(const CanonKey* L, const uint32_t* R, const uint32_t* d_nrep, size_t cap, Fr* sp,
                          hipStream_t st) {
  if (cap == 0) return hipSuccess;
  hipLaunchKernelGGL(lookup_scatter_kernel, dim3(grid_1d(cap)), dim3(KT), 0, st, L, R, d_nrep, cap, sp);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) lk_den_kernel(const Fr* __restrict__ ap, const Fr* __restrict__ sp, Fr beta,
                                                    Fr gamma, Fr* __restrict__ prod, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(prod + i, (beta + ldf(ap + i)) * (gamma + ldf(sp + i)));
}
__global__ void __launch_bounds__(KT) lk_num_kernel(const Fr* __restrict__ a, const Fr* __restrict__ s, Fr beta,
                                                    Fr gamma, Fr* __restrict__ prod, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(prod + i, ldf(prod + i) * (ldf(a + i) + beta) * (ldf(s + i) + gamma));
}
hipError_t lookup_prod_den(const Fr* ap, const Fr* sp, const Fr& beta, const Fr& gamma, Fr* prod, size_t n,
                           hipStream_t st) {
  hipLaunchKernelGGL(lk_den_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, ap, sp, beta, gamma, prod, n);
  return hipGetLastError();
}
hipError_t lookup_prod_num(const Fr* a, const Fr* s, const Fr& beta, const Fr& gamma, Fr* prod, size_t n,
                           hipStream_t st) {
  hipLaunchKernelGGL(lk_num_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, a, s, beta, gamma, prod, n);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) sh_den_kernel(const Fr* __restrict__ s, Fr gamma, Fr* __restrict__ prod,
                                                    size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(prod + i, gamma + ldf(s + i));
}
__global__ void __launch_bounds__(KT) sh_num_kernel(const Fr* __restrict__ a, Fr gamma, Fr* __restrict__ prod,
                                                    size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(prod + i, ldf(prod + i) * (gamma + ldf(a + i)));
}
hipError_t shuffle_prod_den(const Fr* s, const Fr& gamma, Fr* prod, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(sh_den_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, s, gamma, prod, n);
  return hipGetLastError();
}
hipError_t shuffle_prod_num(const Fr* a, const Fr& gamma, Fr* prod, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(sh_num_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, a, gamma, prod, n);
  return hipGetLastError();
}

// ------------------------------------------------------------------ block helpers
// sum over this block's threads of v_t * X^(t) with X_t = xs^t, where each thread's
// value already covers `per` consecutive elements: tree combine with xs^(per*2^l).
template <int NT>
__device__ Fr block_weighted_sum(Fr v, Fr step /* weight between consecutive threads */, Fr* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  Fr X = step;
  for (int s = 1; s < NT; s <<= 1) {
    if ((t & (2 * s - 1)) == 0) sh[t] = sh[t] + X * sh[t + s];
    X = X * X;
    __syncthreads();
  }
  const Fr r = sh[0];
  __syncthreads();
  return r;
}

// Suffix scan of affine maps f_t(c) = val_t + w_t * c over the block's threads.
// Returns, for thread t, the map F_{t+1} = f_{t+1} o ... o f_{NT-1} as (val, w)
// (identity (0, 1) for the last thread).
template <int NT>
__device__ void block_suffix_affine(Fr val, Fr w, Fr* shv, Fr* shw, Fr* out_val, Fr* out_w) {
  const int t = threadIdx.x;
  shv[t] = val;
  shw[t] = w;
  __syncthreads();
  for (int s = 1; s < NT; s <<= 1) {
    Fr v2 = shv[t], w2 = shw[t];
    if (t + s < NT) {
      // f_t..f_{t+s-1} composed with the next block of maps: (v, w) o (v', w') = (v + w v', w w')
      const Fr vn = shv[t + s], wn = shw[t + s];
      v2 = v2 + w2 * vn;
      w2 = w2 * wn;
    }
    __syncthreads();
    shv[t] = v2;
    shw[t] = w2;
    __syncthreads();
  }
  if (t + 1 < NT) {
    *out_val = shv[t + 1];
    *out_w = shw[t + 1];
  } else {
    *out_val = Fr::zero();
    *out_w = Fr::one();
  }
  __syncthreads();
}

// ------------------------------------------------------------------ polynomial evaluation
// H2G_HORNER29 = 1: the Horner chains of eval_level1 and kate_phase1/3 in F29 (f29.h): the
// recurrence is linear in the coefficients, so they enter as raw storage integers, the
// point as an F29 element, and the accumulator is reduced only where it is stored.
// 0: the 8 x 32-bit Montgomery chains (A/B builds).
#ifndef H2G_HORNER29
#define H2G_HORNER29 1
#endif
__device__ __forceinline__ Fr f29_to_storage(const F29& v) {  // v < 2^260 -> [0, M)
  return pack29<FrParams>(sub_m_if_ge29<FrParams>(reduce29<FrParams>(norm29(v))));
}

#ifndef H2G_EV_LS  // log2 of the coefficients per thread (4: 0.95 ms, 6: 0.69 ms for C3 k = 22's batch)
#define H2G_EV_LS 6
#endif
static constexpr int EV_T = 256;
static constexpr int EV_S = 1 << H2G_EV_LS;              // coefficients per thread
static constexpr uint64_t EV_BLK = (uint64_t)EV_T * EV_S;  // per block
static constexpr int EV_L = 8;                           // log2(EV_T)
static constexpr int EV_LB = EV_L + H2G_EV_LS;           // log2(EV_BLK)
static_assert((1 << EV_L) == EV_T && EV_BLK == (1ull << EV_LB), "eval_level2 raises x to EV_BLK = 2^EV_LB");

__global__ void __launch_bounds__(EV_T) eval_level1(const EvalReq* __restrict__ reqs, Fr* __restrict__ part,
                                                    uint64_t nbmax) {
  __shared__ Fr sh[EV_T];
  const EvalReq rq = reqs[blockIdx.y];
  const uint64_t base = blockIdx.x * EV_BLK;
  if (base >= rq.len) {
    if (threadIdx.x == 0) part[blockIdx.y * nbmax + blockIdx.x] = Fr::zero();
    return;
  }
  // coalesced: thread t takes the coefficients base + t + EV_T i (i < EV_S), a wave's loads
  // are 2 KB runs; acc_t = sum_i a_{t + EV_T i} (x^EV_T)^i, then sum_t acc_t x^t by a tree
  // with the level weights pw[l] = x^(2^l) (one thread's squaring chain, pw[EV_L] = x^EV_T).
  // (Four independent Horner chains per thread measured slower: 1.22 vs 0.97 ms for C3
  // k = 22's batch -- the unrolled loads and accumulators halve the waves per SIMD.)
  __shared__ Fr pw[EV_L + 1];
  __shared__ F29 x29;  // pw[EV_L] as an F29 element (H2G_HORNER29)
  const int t = threadIdx.x;
  if (t == 0) {
    Fr step = rq.x;
    for (int l = 0; l <= EV_L; l++) {
      pw[l] = step;
      step = step * step;
    }
    if (H2G_HORNER29) x29 = storage_to_f29<FrParams>(pw[EV_L]);
  }
  __syncthreads();
  const uint64_t lo = base + (uint64_t)t;
  Fr acc;
  if constexpr (H2G_HORNER29) {
    // F29 Horner (f29.h): storage integers enter raw, x^EV_T as an F29 element; the
    // accumulator stays unreduced (< 6.4 M, tools/f29_bounds.py) and is reduced once
    const F29 X = x29;
    F29 a29{};
    for (int i = EV_S - 1; i >= 0; i--) {
      const uint64_t j = lo + (uint64_t)i * EV_T;
      a29 = add29(mul29<FrParams>(a29, X), j < rq.len ? raw29(ldf(rq.poly + j)) : F29{});
    }
    acc = f29_to_storage(a29);
  } else {
    const Fr X = pw[EV_L];
    acc = Fr::zero();
    for (int i = EV_S - 1; i >= 0; i--) {
      const uint64_t j = lo + (uint64_t)i * EV_T;
      acc = acc * X + (j < rq.len ? ldf(rq.poly + j) : Fr::zero());
    }
  }
  sh[t] = acc;
  __syncthreads();
#pragma unroll
  for (int l = 0; l < EV_L; l++) {
    const int s = 1 << l;
    if ((t & (2 * s - 1)) == 0) sh[t] = sh[t] + pw[l] * sh[t + s];
    __syncthreads();
  }
  if (t == 0) part[blockIdx.y * nbmax + blockIdx.x] = sh[0];
}

__global__ void __launch_bounds__(EV_T) eval_level2(const EvalReq* __restrict__ reqs, const Fr* __restrict__ part,
                                                    uint64_t nbmax, Fr* __restrict__ out) {
  __shared__ Fr sh[EV_T];
  const EvalReq rq = reqs[blockIdx.x];
  const uint64_t nb = (rq.len + EV_BLK - 1) / EV_BLK;
  const uint64_t per = (nb + EV_T - 1) / EV_T;
  Fr xb = rq.x;
  for (int i = 0; i < EV_LB; i++) xb = xb * xb;  // x^EV_BLK
  const Fr* p = part + blockIdx.x * nbmax;
  const uint64_t lo = (uint64_t)threadIdx.x * per;
  Fr acc = Fr::zero();
  for (uint64_t i = per; i-- > 0;) {
    const uint64_t j = lo + i;
    acc = acc * xb + (j < nb ? p[j] : Fr::zero());
  }
  const Fr step = pow_u64(xb, per);
  const Fr r = block_weighted_sum<EV_T>(acc, step, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = r;
}

size_t poly_eval_scratch_len(int nreq, uint64_t max_len) {
  const uint64_t nb = (max_len + EV_BLK - 1) / EV_BLK;
  return (size_t)nreq * (nb ? nb : 1);
}

hipError_t poly_eval_batch(const EvalReq* d_reqs, int nreq, uint64_t max_len, Fr* d_out, Fr* scratch,
                           hipStream_t st) {
  if (nreq == 0) return hipSuccess;
  uint64_t nb = (max_len + EV_BLK - 1) / EV_BLK;
  if (nb == 0) nb = 1;
  hipLaunchKernelGGL(eval_level1, dim3((unsigned)nb, (unsigned)nreq), dim3(EV_T), 0, st, d_reqs, scratch, nb);
  hipLaunchKernelGGL(eval_level2, dim3((unsigned)nreq), dim3(EV_T), 0, st, d_reqs, (const Fr*)scratch, nb, d_out);
  return hipGetLastError();
}

// ------------------------------------------------------------------ kate division
// With a' = a[1..len) and M = len - 1: q[i] = sum_{j >= i} a'[j] b^(j - i), i.e. the
// suffix Horner of a' at b.  Phase 1: per-thread suffix sums over KD_S elements (kept for
// phase 3) and per-tile sums; phase 2: tile carries (one block, suffix scan of affine
// maps); phase 3: a weighted suffix scan of the kept per-thread sums (seeded with the
// tile's carry) gives each thread its carry, then the downward recurrence.  Every
// thread's map has the same slope b^KD_S, so both block scans need one product per level,
// with the level weights b^(KD_S 2^l) computed once on the host (KatePow).
// KD_S (elements per thread) is chosen per call: the largest power of two in
// [KD_S_MIN, KD_S_MAX] that still gives KD_MIN_BLOCKS tiles (longer chains amortise the
// block scans and the one-block phase 2; a short polynomial keeps its blocks).
#ifndef H2G_KD_S_MAX
#define H2G_KD_S_MAX 32
#endif
static constexpr int KD_T = 256;
static constexpr int KD_S_MIN = 8;
static constexpr int KD_S_MAX = H2G_KD_S_MAX;
static constexpr uint64_t KD_MIN_BLOCKS = 512;
static constexpr int KD_L = 8;  // log2(KD_T)
static_assert((1 << KD_L) == KD_T, "KD_L");
static_assert(KD_S_MAX >= KD_S_MIN && KD_S_MAX <= 64, "KD_S_MAX");

struct KatePow {
  Fr p[KD_L + 1];  // p[l] = b^(KD_S 2^l); p[KD_L] = b^KD_TILE
};

// Thread t's segment is KD_S consecutive coefficients, so a direct load by lane strides
// KD_S x 32 B between lanes (a wave touches 64 lines per load and uses 32 B of each).  The
// staged form (H2G_KATE_LDS) moves each segment's next KD_SUB coefficients for the whole
// block through LDS: every run of KD_SUB x 32 B = 128 B is loaded by 8 lanes with 16-B
// loads (whole lines), each thread then reads its own run from LDS -- rows padded to
// 144 B so the 16 lanes of a ds_read_b128 hit distinct banks.  Phase 3 stages its stored
// quotients (and, accumulating, the old ones) the same way.  Phase 3 only by default
// (H2G_KATE_LDS 1; 2 stages phase 1 too): at 2^22 phase 3 96 vs 135 us (136 vs 152 us
// accumulating); the read-only phase 1 was faster unstaged, 76 vs 85 us
// (profiles/r06/kate/).
#ifndef H2G_KATE_LDS
#define H2G_KATE_LDS 1
#endif
#ifndef H2G_KD_SUB
#define H2G_KD_SUB 4
#endif
static constexpr int KD_SUB = H2G_KD_SUB;          // coefficients per thread and stage
static constexpr int KD_ROW = 2 * KD_SUB + 1;      // uint4 per thread row (+1 pad)
struct KateStage {
  uint4 v[KD_T * KD_ROW];
};
// the block's run c (coefficients lo_t + KD_SUB c .. + KD_SUB of every thread t) -> st; the
// block's threads, 8 per run, each 16-B piece once; coefficients >= M read as zero
template <int KD_S>
__device__ __forceinline__ void kate_stage_load(KateStage& st, const Fr* __restrict__ src, uint64_t tile0, uint64_t M,
                                                int c) {
  constexpr int PER = 2 * KD_SUB;  // 16-B pieces per run
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int u = k * KD_T + threadIdx.x;  // piece u of the block's KD_T runs
    const int tt = u / PER, r = u % PER;
    const uint64_t j = tile0 + (uint64_t)tt * KD_S + (uint64_t)KD_SUB * c + (r >> 1);
    st.v[tt * KD_ROW + r] = j < M ? reinterpret_cast<const uint4*>(src + j)[r & 1] : make_uint4(0, 0, 0, 0);
  }
}
template <int KD_S>
__device__ __forceinline__ void kate_stage_store(const KateStage& st, Fr* __restrict__ dst, uint64_t tile0,
                                                 uint64_t M, int c) {
  constexpr int PER = 2 * KD_SUB;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int u = k * KD_T + threadIdx.x;
    const int tt = u / PER, r = u % PER;
    const uint64_t j = tile0 + (uint64_t)tt * KD_S + (uint64_t)KD_SUB * c + (r >> 1);
    if (j < M) reinterpret_cast<uint4*>(dst + j)[r & 1] = st.v[tt * KD_ROW + r];
  }
}
__device__ __forceinline__ Fr kate_stage_get(const KateStage& st, int t, int i) {
  const uint4 a = st.v[t * KD_ROW + 2 * i], b = st.v[t * KD_ROW + 2 * i + 1];
  Fr r;
  r.l[0] = a.x, r.l[1] = a.y, r.l[2] = a.z, r.l[3] = a.w;
  r.l[4] = b.x, r.l[5] = b.y, r.l[6] = b.z, r.l[7] = b.w;
  return r;
}
__device__ __forceinline__ void kate_stage_put(KateStage& st, int t, int i, const Fr& v) {
  st.v[t * KD_ROW + 2 * i] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
  st.v[t * KD_ROW + 2 * i + 1] = make_uint4(v.l[4], v.l[5], v.l[6], v.l[7]);
}

template <int KD_S>
__global__ void __launch_bounds__(KD_T) kate_phase1(const Fr* __restrict__ a1, uint64_t M, Fr b, F29 b29, KatePow pw,
                                                    Fr* __restrict__ tile_val, Fr* __restrict__ thr_val) {
  __shared__ Fr sh[KD_T];
  const int t = threadIdx.x;
  const uint64_t lo = blockIdx.x * (uint64_t)(KD_T * KD_S) + (uint64_t)t * KD_S;
  Fr acc;
  if constexpr (H2G_HORNER29 && H2G_KATE_LDS >= 2) {  // measured slower for phase 1 (85 vs 76 us at 2^22)
    __shared__ KateStage stg;
    const uint64_t tile0 = blockIdx.x * (uint64_t)(KD_T * KD_S);
    F29 a29{};
    for (int c = KD_S / KD_SUB - 1; c >= 0; c--) {
      __syncthreads();  // the previous run's reads are done
      kate_stage_load<KD_S>(stg, a1, tile0, M, c);
      __syncthreads();
#pragma unroll
      for (int i = KD_SUB - 1; i >= 0; i--) a29 = add29(mul29<FrParams>(a29, b29), raw29(kate_stage_get(stg, t, i)));
    }
    acc = f29_to_storage(a29);
  } else if constexpr (H2G_HORNER29) {
    F29 a29{};
#pragma unroll
    for (int i = KD_S - 1; i >= 0; i--) {
      const uint64_t j = lo + i;
      a29 = add29(mul29<FrParams>(a29, b29), j < M ? raw29(ldf(a1 + j)) : F29{});
    }
    acc = f29_to_storage(a29);
  } else {
    acc = Fr::zero();
#pragma unroll
    for (int i = KD_S - 1; i >= 0; i--) {
      const uint64_t j = lo + i;
      acc = acc * b + (j < M ? ldf(a1 + j) : Fr::zero());
    }
  }
  stf(thr_val + blockIdx.x * (uint64_t)KD_T + t, acc);
  // sum_t acc_t b^(KD_S t): tree with the level weights
  sh[t] = acc;
  __syncthreads();
#pragma unroll
  for (int l = 0; l < KD_L; l++) {
    const int s = 1 << l;
    if ((t & (2 * s - 1)) == 0) sh[t] = sh[t] + pw.p[l] * sh[t + s];
    __syncthreads();
  }
  if (t == 0) tile_val[blockIdx.x] = sh[0];
}

// one block: carry[c] = q[hi_c] = sum_{c' > c} V_c' B^(c' - c - 1), B = b^TILE
__global__ void __launch_bounds__(KD_T) kate_phase2(Fr* __restrict__ tile_val, uint64_t ntiles, Fr B) {
  __shared__ Fr shv[KD_T], shw[KD_T];
  const uint64_t per = (ntiles + KD_T - 1) / KD_T;
  const uint64_t lo = (uint64_t)threadIdx.x * per;
  const uint64_t hi = lo + per < ntiles ? lo + per : ntiles;
  // group map: f(c) = sum_{i in group} V_i B^(i - lo) + B^(cnt) c
  Fr val = Fr::zero(), w = Fr::one();
  for (uint64_t i = hi; i-- > lo;) {
    val = val * B + tile_val[i];
    w = w * B;
  }
  Fr cv, cw;
  block_suffix_affine<KD_T>(val, w, shv, shw, &cv, &cw);
  // carry above this group = F_{t+1}(0) = cv; walk down the group
  Fr carry = cv;
  for (uint64_t i = hi; i-- > lo;) {
    const Fr v = tile_val[i];
    tile_val[i] = carry;  // q at the top of tile i
    carry = v + B * carry;
  }
}

// q[j] (+)= the quotient; thread t's carry is the inclusive weighted suffix sum of
// x_t = (thread t+1's sum, or the tile's carry for the last thread)
template <int KD_S, bool ACC>
__global__ void __launch_bounds__(KD_T) kate_phase3(const Fr* __restrict__ a1, uint64_t M, Fr b, F29 b29, KatePow pw,
                                                    const Fr* __restrict__ tile_carry,
                                                    const Fr* __restrict__ thr_val, Fr* __restrict__ q) {
  __shared__ Fr sh[KD_T];
  const int t = threadIdx.x;
  const uint64_t g = blockIdx.x * (uint64_t)KD_T + t;
  Fr x = t + 1 < KD_T ? ldf(thr_val + g + 1) : tile_carry[blockIdx.x];
#pragma unroll
  for (int l = 0; l < KD_L; l++) {
    const int s = 1 << l;
    sh[t] = x;
    __syncthreads();
    if (t + s < KD_T) x = x + pw.p[l] * sh[t + s];
    __syncthreads();
  }
  const uint64_t lo = blockIdx.x * (uint64_t)(KD_T * KD_S) + (uint64_t)t * KD_S;
  if constexpr (H2G_HORNER29 && H2G_KATE_LDS) {
    // staged: run c's coefficients in, its quotients out (and the old ones in, ACC) through
    // LDS, every global access whole lines; the carried value stays unreduced (< 2.1 M)
    // (a thread reads and writes only its own row: without ACC the quotients overwrite the
    // coefficients they come from; with it the old quotients have a buffer of their own)
    __shared__ KateStage stg;
    KateStage* out = &stg;
    if constexpr (ACC) {
      __shared__ KateStage old;
      out = &old;
    }
    const uint64_t tile0 = blockIdx.x * (uint64_t)(KD_T * KD_S);
    F29 cur = raw29(x);
    for (int c = KD_S / KD_SUB - 1; c >= 0; c--) {
      __syncthreads();  // the previous run's reads and its coalesced stores are done
      kate_stage_load<KD_S>(stg, a1, tile0, M, c);
      if (ACC) kate_stage_load<KD_S>(*out, q, tile0, M, c);
      __syncthreads();
#pragma unroll
      for (int i = KD_SUB - 1; i >= 0; i--) {
        cur = add29(raw29(kate_stage_get(stg, t, i)), mul29<FrParams>(cur, b29));
        kate_stage_put(*out, t, i, f29_to_storage(ACC ? add29(raw29(kate_stage_get(*out, t, i)), cur) : cur));
      }
      __syncthreads();
      kate_stage_store<KD_S>(*out, q, tile0, M, c);
    }
    return;
  }
  if constexpr (H2G_HORNER29) {
    // the carried value stays unreduced (< 2.1 M); each stored quotient is reduced
    F29 cur = raw29(x);
    for (int i = KD_S - 1; i >= 0; i--) {
      const uint64_t j = lo + i;
      if (j < M) {
        cur = add29(raw29(ldf(a1 + j)), mul29<FrParams>(cur, b29));
        stf(q + j, f29_to_storage(ACC ? add29(raw29(ldf(q + j)), cur) : cur));
      }
    }
    return;
  }
  Fr cur = x;
  for (int i = KD_S - 1; i >= 0; i--) {
    const uint64_t j = lo + i;
    if (j < M) {
      cur = ldf(a1 + j) + b * cur;
      stf(q + j, ACC ? ldf(q + j) + cur : cur);
    }
  }
}

template <int S>
static void kate_launch(const Fr* a, uint64_t M, const Fr& b, const F29& b29, const KatePow& pw, Fr* tile, Fr* thr,
                        Fr* q, uint64_t nt, hipStream_t st, bool accumulate) {
  hipLaunchKernelGGL(kate_phase1<S>, dim3((unsigned)nt), dim3(KD_T), 0, st, a + 1, M, b, b29, pw, tile, thr);
  hipLaunchKernelGGL(kate_phase2, dim3(1), dim3(KD_T), 0, st, tile, nt, pw.p[KD_L]);
  if (accumulate)
    hipLaunchKernelGGL((kate_phase3<S, true>), dim3((unsigned)nt), dim3(KD_T), 0, st, a + 1, M, b, b29, pw,
                       (const Fr*)tile, (const Fr*)thr, q);
  else
    hipLaunchKernelGGL((kate_phase3<S, false>), dim3((unsigned)nt), dim3(KD_T), 0, st, a + 1, M, b, b29, pw,
                       (const Fr*)tile, (const Fr*)thr, q);
}

size_t kate_scratch_len(uint64_t len) {  // sized for the shortest tiles (KD_S_MIN)
  const uint64_t nt = (len + (uint64_t)KD_T * KD_S_MIN - 1) / ((uint64_t)KD_T * KD_S_MIN);
  return (size_t)(nt + 1 + nt * KD_T);
}

hipError_t kate_division(const Fr* a, uint64_t len, const Fr& b, Fr* q, Fr* scratch, hipStream_t st,
                         bool accumulate) {
  if (len < 2) return hipSuccess;
  const uint64_t M = len - 1;
  int S = KD_S_MIN;
  while (S < KD_S_MAX && (M + (uint64_t)KD_T * S * 2 - 1) / ((uint64_t)KD_T * S * 2) >= KD_MIN_BLOCKS) S <<= 1;
  const uint64_t tile_len = (uint64_t)KD_T * S;
  const uint64_t nt = (M + tile_len - 1) / tile_len;
  KatePow pw;
  Fr x = b;
  for (int i = 1; i < S; i <<= 1) x = x * x;
  for (int l = 0; l <= KD_L; l++) {
    pw.p[l] = x;
    x = x * x;
  }
  Fr* tile = scratch;
  Fr* thr = scratch + nt + 1;
  const F29 b29 = storage_to_f29<FrParams>(b);  // b as an F29 element (H2G_HORNER29)
  switch (S) {
    case 8: kate_launch<8>(a, M, b, b29, pw, tile, thr, q, nt, st, accumulate); break;
    case 16: kate_launch<16>(a, M, b, b29, pw, tile, thr, q, nt, st, accumulate); break;
    case 32: kate_launch<32>(a, M, b, b29, pw, tile, thr, q, nt, st, accumulate); break;
    default: kate_launch<64>(a, M, b, b29, pw, tile, thr, q, nt, st, accumulate); break;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------ linear combinations
__global__ void __launch_bounds__(KT) lincomb_kernel(Fr* __restrict__ out, uint64_t n, LinTerms t, int acc_in) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    Fr acc = acc_in ? ldf(out + i) : Fr::zero();
    for (int k = 0; k < t.k; k++)
      if (i < t.len[k]) acc = acc + t.coef[k] * ldf(t.p[k] + i);
    stf(out + i, acc);
  }
}

// The same in F29 (f29.h): the map is linear, so the storage integers of the columns enter
// raw, the coefficients as proper F29 elements, and two terms share one reduction
// (mul29x2); every pair's result is < 1.02 M, their sum (with the accumulated value) is
// brought to [0, M) by reduce29 and one subtraction.  H2G_LINCOMB29 = 0: the kernel above.
#ifndef H2G_LINCOMB29
#define H2G_LINCOMB29 1
#endif
struct LinTerms29 {
  const Fr* p[LIN_MAXT];
  uint64_t len[LIN_MAXT];
  F29 coef[LIN_MAXT];
  int k = 0;
};
__global__ void __launch_bounds__(KT) lincomb29_kernel(Fr* __restrict__ out, uint64_t n, LinTerms29 t, int acc_in) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    F29 acc = acc_in ? raw29(ldf(out + i)) : F29{};
    int k = 0;
    for (; k + 1 < t.k; k += 2) {
      const F29 a = i < t.len[k] ? raw29(ldf(t.p[k] + i)) : F29{};
      const F29 b = i < t.len[k + 1] ? raw29(ldf(t.p[k + 1] + i)) : F29{};
      acc = add29(acc, mul29x2<FrParams>(a, t.coef[k], b, t.coef[k + 1]));
    }
    if (k < t.k) {
      const F29 a = i < t.len[k] ? raw29(ldf(t.p[k] + i)) : F29{};
      acc = add29(acc, mul29<FrParams>(a, t.coef[k]));
    }
    stf(out + i, pack29<FrParams>(sub_m_if_ge29<FrParams>(reduce29<FrParams>(norm29(acc)))));
  }
}

hipError_t lincomb(Fr* out, uint64_t n, const LinTerms& t, bool accumulate, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (H2G_LINCOMB29) {
    LinTerms29 t29;
    t29.k = t.k;
    for (int k = 0; k < t.k; k++) {
      t29.p[k] = t.p[k];
      t29.len[k] = t.len[k];
      t29.coef[k] = storage_to_f29<FrParams>(t.coef[k]);
    }
    hipLaunchKernelGGL(lincomb29_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, out, n, t29, accumulate ? 1 : 0);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(lincomb_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, out, n, t, accumulate ? 1 : 0);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) scale_dev_kernel(Fr* __restrict__ out, const Fr* __restrict__ a, uint64_t n,
                                                       const Fr* __restrict__ s) {
  const Fr c = ldf(s);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    stf(out + i, ldf(a + i) * c);
}

hipError_t scale_by_dev(Fr* out, const Fr* a, uint64_t n, const Fr* scalar, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(scale_dev_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, out, a, n, scalar);
  return hipGetLastError();
}

// ------------------------------------------------------------------ sub-cosets (SPMD)
// The extended domain is 2^e cosets of the n-point subgroup: row y = t + 2^e m of the
// extended coset is point zeta w_ext^t w^m, so sub-coset t of a polynomial is an n-point
// NTT of c_j zeta^(j mod 3) w_ext^(t j) (the zeta powers are the NTT's input distribution)
__global__ void __launch_bounds__(KT) subcoset_twist_kernel(const Fr* __restrict__ src, Fr* __restrict__ dst,
                                                            size_t n, PowTable eo, uint64_t t, uint64_t ext_mask) {
  for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < n; j += (size_t)gridDim.x * blockDim.x)
    stf(dst + j, ldf(src + j) * pw(eo, (t * j) & ext_mask));
}
hipError_t subcoset_twist(const Fr* src, Fr* dst, size_t n, const PowTable& eo, uint64_t t, uint64_t ext_mask,
                          hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(subcoset_twist_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, src, dst, n, eo, t, ext_mask);
  return hipGetLastError();
}
// out[m] = full[t + (m << e)]: sub-coset t of a full extended-coset array (the key's cosets)
__global__ void __launch_bounds__(KT) subcoset_gather_kernel(const Fr* __restrict__ full, Fr* __restrict__ out,
                                                             size_t n, uint64_t t, int e) {
  for (size_t m = blockIdx.x * (size_t)blockDim.x + threadIdx.x; m < n; m += (size_t)gridDim.x * blockDim.x)
    stf(out + m, ldf(full + t + ((uint64_t)m << e)));
}
hipError_t subcoset_gather(const Fr* full, Fr* out, size_t n, uint64_t t, int e, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(subcoset_gather_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, full, out, n, t, e);
  return hipGetLastError();
}
// many device-to-device copies in one launch (SPMD pack / unpack of exchanged columns):
// segment blockIdx.y, its elements strided over blockIdx.x
__global__ void __launch_bounds__(KT) copy_segments_kernel(const CopySeg* __restrict__ segs) {
  const CopySeg g = segs[blockIdx.y];
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < g.len; i += (uint64_t)gridDim.x * blockDim.x)
    stf(g.dst + i, ldf(g.src + i));
}
hipError_t copy_segments(const CopySeg* d_segs, int nseg, uint64_t max_len, hipStream_t st) {
  if (nseg <= 0 || max_len == 0) return hipSuccess;
  const unsigned gx = (unsigned)std::min<uint64_t>((max_len + KT - 1) / KT, 256);
  for (int s0 = 0; s0 < nseg; s0 += 65535)
    hipLaunchKernelGGL(copy_segments_kernel, dim3(gx, (unsigned)std::min(65535, nseg - s0)), dim3(KT), 0, st,
                       d_segs + s0);
  return hipGetLastError();
}
// the witness columns into the prover's workspace: a streaming kernel (one read, one write
// per element) in place of per-column DMA copies, with the SPMD checksum on the same read
__device__ __forceinline__ uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}
// 16-byte chunks (lane-contiguous, fully coalesced), 4 per thread and iteration so that a
// wave has 4 loads in flight; the checksum mixes each chunk with its index
__device__ __forceinline__ uint64_t chunk_mix(size_t i, const uint4& v) {
  uint64_t h = fmix64((uint64_t)i * 0x9e3779b97f4a7c15ull + 0x2545f4914f6cdd1dull);
  h = fmix64(h ^ ((uint64_t)v.x | (uint64_t)v.y << 32));
  return fmix64(h ^ ((uint64_t)v.z | (uint64_t)v.w << 32));
}
template <bool SUM>
__global__ void __launch_bounds__(256) copy_columns_kernel(ColCopy b, size_t n2) {
  const uint4* __restrict__ s = reinterpret_cast<const uint4*>(b.src[blockIdx.y]);
  uint4* __restrict__ d = reinterpret_cast<uint4*>(b.dst[blockIdx.y]);
  uint64_t acc = 0;
  const size_t step = (size_t)gridDim.x * 1024;
  for (size_t i = blockIdx.x * (size_t)1024 + threadIdx.x; i < n2; i += step) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (i + 256 * k < n2) v[k] = s[i + 256 * k];
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (i + 256 * k < n2) {
        if (d) d[i + 256 * k] = v[k];
        if (SUM) acc += chunk_mix(i + 256 * k, v[k]);
      }
  }
  if (SUM) {
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    __shared__ uint64_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0 && b.sum[blockIdx.y])
      atomicAdd(b.sum[blockIdx.y], (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
  }
}
hipError_t copy_columns(const ColCopy& b, int m, size_t n, bool sums, hipStream_t st) {
  if (m <= 0 || n == 0) return hipSuccess;
  if (m > COPY_COLS_MAX) return hipErrorInvalidValue;
  const size_t n2 = 2 * n;  // 16-byte chunks of the 32-byte elements
  const size_t blocks = std::min<size_t>((n2 + 1023) / 1024, 1024);
  if (sums)
    hipLaunchKernelGGL(copy_columns_kernel<true>, dim3((unsigned)blocks, (unsigned)m), dim3(256), 0, st, b, n2);
  else
    hipLaunchKernelGGL(copy_columns_kernel<false>, dim3((unsigned)blocks, (unsigned)m), dim3(256), 0, st, b, n2);
  return hipGetLastError();
}
// ext[t + (m << e)] = subs[t n + m] for every t < 2^e: sub-coset slots back to row order
__global__ void __launch_bounds__(KT) subcoset_scatter_kernel(const Fr* __restrict__ subs, Fr* __restrict__ ext,
                                                              size_t n, int e) {
  const uint64_t total = (uint64_t)n << e, tmask = (1ull << e) - 1;
  for (uint64_t y = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; y < total; y += (uint64_t)gridDim.x * blockDim.x)
    stf(ext + y, ldf(subs + (y & tmask) * n + (y >> e)));
}
hipError_t subcoset_scatter(const Fr* subs, Fr* ext, size_t n, int e, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(subcoset_scatter_kernel, dim3(grid_1d((size_t)n << e)), dim3(KT), 0, st, subs, ext, n, e);
  return hipGetLastError();
}

// h(X)'s slab from the sub-coset owners' folded coefficients (SPMD, h2g_spmd_transport
// exchange): F_t[j] = sum_p h_{j+np} zeta^(np) rho^(t p) (rho = w_ext^n, t < E) for j in
// this rank's slab; h_{j+np} = sum_t coef[p E + t] F_t[j] with coef = zeta^(-np) rho^(-tp) / E
__global__ void __launch_bounds__(KT) h_slab_combine_kernel(HSlabArgs a) {
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < a.cnt; j += (uint64_t)gridDim.x * blockDim.x) {
    Fr f[HSLAB_MAX_E];
    for (int t = 0; t < a.E; t++) f[t] = ldf(a.recv + (uint64_t)a.idx[t] * a.cnt + j);
    for (int p = 0; p < a.np; p++) {
      Fr acc = Fr::zero();
      for (int t = 0; t < a.E; t++) acc = acc + ldf(a.coef + p * a.E + t) * f[t];
      stf(a.out + (uint64_t)p * a.n + a.lo + j, acc);
    }
  }
}
hipError_t h_slab_combine(const HSlabArgs& a, hipStream_t st) {
  if (a.cnt == 0 || a.np == 0) return hipSuccess;
  hipLaunchKernelGGL(h_slab_combine_kernel, dim3(grid_1d(a.cnt)), dim3(KT), 0, st, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------ keygen helpers
__global__ void __launch_bounds__(KT) sigma_kernel(Fr* __restrict__ sigma, const uint32_t* __restrict__ mc,
                                                   const uint32_t* __restrict__ mr, size_t n,
                                                   const Fr* __restrict__ dp, PowTable om) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(sigma + i, ldf(dp + mc[i]) * pw(om, mr[i]));
}

hipError_t sigma_from_mapping(Fr* sigma, const uint32_t* map_col, const uint32_t* map_row, size_t n,
                              const Fr* delta_pow, const PowTable& omega, hipStream_t st) {
  hipLaunchKernelGGL(sigma_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, sigma, map_col, map_row, n, delta_pow, omega);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) lag_den_kernel(Fr* __restrict__ d, size_t n, Fr s, PowTable om) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(d + i, s - pw(om, i));
}
__global__ void __launch_bounds__(KT) lag_num_kernel(Fr* __restrict__ d, size_t n, Fr mult, PowTable om) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    stf(d + i, ldf(d + i) * mult * pw(om, i));
}

hipError_t srs_lagrange_scalars(Fr* out, size_t n, const Fr& s, const Fr& mult, const PowTable& omega, Fr* scratch,
                                hipStream_t st) {
  hipLaunchKernelGGL(lag_den_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, out, n, s, omega);
  hipError_t e = poly_batch_invert(out, n, scratch, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(lag_num_kernel, dim3(grid_1d(n)), dim3(KT), 0, st, out, n, mult, omega);
  return hipGetLastError();
}

__global__ void __launch_bounds__(KT) gen_mul_kernel(const Fr* __restrict__ sc, size_t n, G1Affine* __restrict__ out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr e = to_canonical(ldf(sc + i));
  G1Affine g;
  g.x = Fq::one();
  g.y = from_u64<FqParams>(2);
  out[i] = xyzz_to_affine_by(xyzz_mul_canonical(G1xyzz::from_affine(g), e.l));
}

hipError_t g1_generator_mul(const Fr* scalars, size_t n, G1Affine* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gen_mul_kernel, dim3((unsigned)((n + KT - 1) / KT)), dim3(KT), 0, st, scalars, n, out);
  return hipGetLastError();
}

// ---- RawBytes checks ---------------------------------------------------------
template <class P>
__device__ __forceinline__ bool below_modulus(const Fe<P>& a) {
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)__builtin_subc(a.l[i], P::M[i], br, &br);
  return br != 0;  // a - M borrows <=> a < M
}
// one no-return atomic per wave that saw a bad element (bad inputs are the rare case)
__device__ __forceinline__ void count_bad(bool bad, uint32_t* out) {
  const uint64_t m = __ballot(bad);
  if (m && __lane_id() == (uint32_t)__builtin_ctzll(m)) atomicAdd(out, (uint32_t)__popcll(m));
}
__global__ void __launch_bounds__(KT) fr_unreduced_kernel(const Fr* __restrict__ a, size_t n, uint32_t* bad) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  count_bad(i < n && !below_modulus(a[i]), bad);
}
__global__ void __launch_bounds__(KT) g1_invalid_kernel(const G1Affine* __restrict__ p, size_t n, uint32_t* bad) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  bool b = false;
  if (i < n) {
    const G1Affine q = p[i];
    if (!below_modulus(q.x) || !below_modulus(q.y)) b = true;
    else if (!q.is_identity()) b = sqr(q.y) != sqr(q.x) * q.x + from_u64<FqParams>(3);
  }
  count_bad(b, bad);
}
hipError_t fr_count_unreduced(const Fr* a, size_t n, uint32_t* bad, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fr_unreduced_kernel, dim3((unsigned)((n + KT - 1) / KT)), dim3(KT), 0, st, a, n, bad);
  return hipGetLastError();
}
hipError_t g1_count_invalid(const G1Affine* p, size_t n, uint32_t* bad, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(g1_invalid_kernel, dim3((unsigned)((n + KT - 1) / KT)), dim3(KT), 0, st, p, n, bad);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) prefix_diff_kernel(PrefixDiff b, size_t n) {
  const Fr* __restrict__ a = b.a[blockIdx.y];
  Fr* __restrict__ e = b.e[blockIdx.y];
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    e[i] = i + 1 < n ? a[i] - a[i + 1] : a[i];
}
hipError_t prefix_diff(const PrefixDiff& b, int m, size_t n, hipStream_t st) {
  if (m <= 0 || n == 0) return hipSuccess;
  if (m > PREFIX_DIFF_MAX) return hipErrorInvalidValue;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(prefix_diff_kernel, dim3((unsigned)blocks, (unsigned)m), dim3(256), 0, st, b, n);
  return hipGetLastError();
}

}  // namespace h2g
