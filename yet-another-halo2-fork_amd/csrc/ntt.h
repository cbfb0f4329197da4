// ntt.h -- NTT plan/launch interface (see ntt.hip).
#pragma once
#include "bn254.h"

namespace h2g {

static constexpr int NTT_SMALL_MAX_LOG = 10;  // whole transform in one block up to 2^10
static constexpr int NTT_MAX_PASSES = 6;      // passes of 3..6 bits: N up to 2^28
static constexpr int NTT_MAX_BATCH = 8;       // transforms per batched launch (blockIdx.y)

// per-transform source / destination of a batched launch
struct NttIo {
  const Fr* src[NTT_MAX_BATCH];
  Fr* dst[NTT_MAX_BATCH];
};

struct NttPlanLg {
  int p = 0;
  int lg[NTT_MAX_PASSES] = {0, 0, 0, 0, 0, 0};
};

struct NttTables {
  int L = 0;  // log2 N
  int b = 0;  // split of the 2-level table
  Fr* lo = nullptr;
  Fr* hi = nullptr;
  // precomputed inter-pass twiddles of the non-last passes: pass p's table holds
  // w^((N/L_p) i_low k) at [k * S_p + i_low] (L_p entries; sum over passes ~ 1.1 N)
  Fr* pass_tw = nullptr;
  uint64_t pass_off[NTT_MAX_PASSES] = {0, 0, 0, 0, 0, 0};
  // the F29 passes' in-pass twiddles w_64^j, j < 32, as F29 elements packed in 8 x 32 bits
  // (a 2^m-point pass reads every 2^(6-m)-th); L >= 6
  Fr* root64 = nullptr;
  // lo / hi as packed F29 elements (passes that form their inter-pass twiddles from the
  // two-level table instead of streaming pass_tw, H2G_NTT_TW_LIVE)
  Fr* lo29 = nullptr;
  Fr* hi29 = nullptr;
  // the constant multiplied into the first pass's table (pass_tw; a transform's scale, so
  // its last pass needs no product) and its inverse (divided out of a call's epilogue)
  Fr fold = Fr::one();
  Fr fold_inv = Fr::one();
};

// One transform y = DFT_w(x) of size N = 2^tab.L with fused maps:
//   x_i = src[i] * (in_distribute ? zeta-power(i mod 3) : 1) for i < n_in, 0 beyond
//   dst[k] = y_k * (has_scale ? scale : 1) * (out_distribute ? zeta-power(k mod 3) : 1), k < out_len
// `work` is an N-element scratch buffer distinct from src and dst (src may alias dst).
// Batched: `count` > 1 independent transforms with the same maps, src / dst from
// `srcs` / `dsts`, `work` of count * N elements; one launch per pass serves them all
// (more waves in flight for the small transforms of many-column circuits).
struct NttArgs {
  const Fr* src = nullptr;
  uint64_t n_in = 0;
  Fr* work = nullptr;
  Fr* dst = nullptr;
  int count = 1;
  const Fr* srcs[NTT_MAX_BATCH] = {};
  Fr* dsts[NTT_MAX_BATCH] = {};
  uint64_t out_len = 0;
  NttTables tab;
  int in_distribute = 0;
  Fr in_z1, in_z2;
  int has_scale = 0;
  Fr scale;
  int out_distribute = 0;
  Fr out_z1, out_z2;
};

void ntt_split(int L, int* P, int lg[NTT_MAX_PASSES]);
hipError_t ntt_build_tables(NttTables* t, const Fr& omega, int L, hipStream_t st, const Fr& fold = Fr::one());
void ntt_free_tables(NttTables* t);
hipError_t ntt_run(const NttArgs& a, hipStream_t st);
hipError_t ntt_init_attributes();

}  // namespace h2g
