// prover_kernels.h -- device kernels of the create_proof pipeline beyond MSM/NTT
// (see prover_kernels.hip for the reference lines each one restates).
#pragma once
#include "bn254.h"

namespace h2g {

// Powers w^i of a fixed root for i < 2^L through two tables: w^i = lo[i & mask] * hi[i >> bits].
struct PowTable {
  const Fr* lo = nullptr;
  const Fr* hi = nullptr;
  int bits = 0;
};

// ---- permutation argument (permutation/prover.rs:103-171) ----
static constexpr int PERM_MAXC = 8;  // columns per kernel launch (sets are split into launches)
struct PermCols {
  const Fr* v[PERM_MAXC];      // column values (Lagrange)
  const Fr* sigma[PERM_MAXC];  // permutation polynomial values (Lagrange)
  Fr beta_delta[PERM_MAXC];    // beta * delta^(global column index)
  int m = 0;
};
// out[r] = (init ? 1 : out[r]) * prod_j (beta * sigma_j[r] + gamma + v_j[r])
hipError_t perm_denominators(Fr* out, size_t n, const PermCols& c, const Fr& beta, const Fr& gamma, bool init,
                             hipStream_t st);
// mod[r] *= prod_j (beta * delta^j * omega^(r0 + r) + gamma + v_j[r])  (r < n; r0: the rows' offset)
hipError_t perm_numerators(Fr* mod, size_t n, const PermCols& c, const Fr& gamma, const PowTable& omega,
                           hipStream_t st, size_t r0 = 0);
// z[0] = *last_z, z[i] = *last_z * prefix[i - 1] for 0 < i < n - bf; z[n-bf..n) = blind_rows[0..bf).
// Rows [lo, hi) only: z[lo] = *last_z (a slab's running product starts over: *last_z then
// carries the product of the rows below it), z[i] = *last_z * prefix[i - 1] above
hipError_t perm_z_assemble(Fr* z, size_t n, int bf, const Fr* prefix, const Fr* last_z, const Fr* blind_rows,
                           hipStream_t st, size_t lo = 0, size_t hi = ~(size_t)0);

// ---- vanishing argument: random polynomial (vanishing/prover.rs:57-81) ----
// out[i] = Fr::random(ChaCha20Rng(seed_t)) for the i - off[t]'th draw of chunk t, i in [lo, hi)
hipError_t chacha_random_poly(Fr* out, size_t n, const uint32_t* d_seeds, const uint64_t* d_offsets, int chunks,
                              hipStream_t st, size_t lo = 0, size_t hi = ~(size_t)0);

// ---- evaluate_h (evaluation.rs:317-620): expression programs + permutation + lookup +
// shuffle constraint blocks, fused with the division by t(X) ----
enum GateOp : int { G_LOAD = 0, G_CONST = 1, G_ADD = 2, G_SUB = 3, G_MUL = 4, G_NEG = 5, G_HORNER = 6 };
// instruction: {op, dst slot, a, b}; G_LOAD: a = load index; G_CONST: a = constant index;
// G_HORNER: acc = acc * factor + slot[a] (factor y for gates, theta for lookup/shuffle
// expression lists).  A program segment is int2 {offset, length} into the program array.
struct EvalLookup {
  int2 in, tab;  // compressed input / table expression programs
  const Fr* z;   // product coset
  const Fr* ap;  // permuted input coset
  const Fr* sp;  // permuted table coset
};
struct EvalShuffle {
  int2 in, sh;
  const Fr* z;
};
struct EvalHArgs {
  const int4* prog = nullptr;
  int2 gates = {0, 0};
  int n_slots = 0;
  Fr theta;
  int nlookups = 0, nshuffles = 0;
  const EvalLookup* lookups = nullptr;    // device arrays
  const EvalShuffle* shuffles = nullptr;
  const Fr* consts = nullptr;
  const Fr* const* query_col = nullptr;  // per query: column coset pointer
  const int* query_rot = nullptr;        // per query: rotation
  // permutation
  int nsets = 0, chunk_len = 0, P = 0;
  const Fr* const* z = nullptr;       // nsets
  const Fr* const* perm_v = nullptr;  // P column cosets
  const Fr* const* sigma = nullptr;   // P sigma cosets
  const Fr* l0 = nullptr;
  const Fr* l_last = nullptr;
  const Fr* l_active = nullptr;
  Fr beta, gamma, y, delta_start, delta;
  PowTable ext_omega;
  uint64_t ext = 0, rot_scale = 0;
  // rows [row0, row0 + rows) only (rows = 0: all ext rows); columns, l0 / l_last / l_active,
  // sigma, t_evals and out stay indexed by the row itself
  uint64_t row0 = 0, rows = 0;
  int last_rot = 0;
  const Fr* t_evals = nullptr;
  uint64_t t_mask = 0;
  // several circuits in one proof (evaluation.rs:367-620): circuit c > 0 continues the
  // Horner chain of the circuits before it from acc_in (the previous launch's output,
  // may alias out); only the last circuit's launch divides by t(X)
  const Fr* acc_in = nullptr;
  int divide = 1;
  Fr* out = nullptr;
};
hipError_t evaluate_h(const EvalHArgs& a, hipStream_t st);

// SPMD sub-coset split of the extended domain (prover_kernels.hip)
hipError_t subcoset_twist(const Fr* src, Fr* dst, size_t n, const PowTable& eo, uint64_t t, uint64_t ext_mask,
                          hipStream_t st);
hipError_t subcoset_gather(const Fr* full, Fr* out, size_t n, uint64_t t, int e, hipStream_t st);
hipError_t subcoset_scatter(const Fr* subs, Fr* ext, size_t n, int e, hipStream_t st);
// dst[i] = src[i] for i < len of every segment (device array of nseg), one launch
struct CopySeg {
  const Fr* src;
  Fr* dst;
  uint64_t len;
};
hipError_t copy_segments(const CopySeg* d_segs, int nseg, uint64_t max_len, hipStream_t st);
// dst[c][i] = src[c][i] (i < n) for up to COPY_COLS_MAX columns in one launch (dst[c] null:
// no copy); with sum[c], also an order-independent 64-bit checksum of the source column
// added into *sum[c] (every 16-byte chunk mixed with its index, summed mod 2^64: the SPMD witness
// digest, prover.cpp spmd_witness_fold)
static constexpr int COPY_COLS_MAX = 16;
struct ColCopy {
  const Fr* src[COPY_COLS_MAX];
  Fr* dst[COPY_COLS_MAX];
  unsigned long long* sum[COPY_COLS_MAX];
};
hipError_t copy_columns(const ColCopy& b, int m, size_t n, bool sums, hipStream_t st);

// e_i = a_i - a_{i+1} (e_{n-1} = a_{n-1}) for up to PREFIX_DIFF_MAX columns: the scalars of
// a commitment against the prefix-summed Lagrange basis (prover.cpp lookup commitments)
static constexpr int PREFIX_DIFF_MAX = 16;
struct PrefixDiff {
  const Fr* a[PREFIX_DIFF_MAX];
  Fr* e[PREFIX_DIFF_MAX];
};
hipError_t prefix_diff(const PrefixDiff& b, int m, size_t n, hipStream_t st);
int evaluate_h_max_slots();
// SPMD: this rank's slab [lo, lo + cnt) of the h pieces (out[p n + j], p < np) from the E
// sub-cosets' folded coefficients F_t (recv + idx[t] cnt); coef: np x E device matrix
static constexpr int HSLAB_MAX_E = 16;
struct HSlabArgs {
  const Fr* recv = nullptr;
  int idx[HSLAB_MAX_E] = {};
  int E = 0, np = 0;
  uint64_t cnt = 0, n = 0, lo = 0;
  const Fr* coef = nullptr;
  Fr* out = nullptr;
};
hipError_t h_slab_combine(const HSlabArgs& a, hipStream_t st);

// Lagrange-basis compression of an expression list (lookup/prover.rs:85-103,
// shuffle/prover.rs:45-66): out[i] = fold_e (acc * theta + e(row i)), rotations mod n
struct CompressArgs {
  const int4* prog = nullptr;
  int2 seg = {0, 0};
  int n_slots = 0;
  const Fr* consts = nullptr;
  const Fr* const* load_col = nullptr;  // Lagrange columns
  const int* load_rot = nullptr;
  uint64_t n = 0;
  Fr theta;
  Fr* out = nullptr;
};
hipError_t compress_lagrange(const CompressArgs& a, hipStream_t st);
// several compressions of one program table in one launch (blockIdx.y = item): a proof's
// lookup inputs and tables, two per lookup
static constexpr int COMPRESS_BATCH_MAX = 32;
struct CompressBatch {
  const int4* prog = nullptr;
  int n_slots = 0;
  const Fr* consts = nullptr;
  const int* load_rot = nullptr;
  uint64_t n = 0;
  Fr theta;
  int count = 0;
  int2 seg[COMPRESS_BATCH_MAX];
  const Fr* const* load_col[COMPRESS_BATCH_MAX];
  Fr* out[COMPRESS_BATCH_MAX];
};
hipError_t compress_lagrange_batch(const CompressBatch& a, hipStream_t st);

// ---- permute_expression_pair (lookup/prover.rs:410-494) building blocks ----
struct CanonKey {  // canonical (non-Montgomery) value: Ord on Fr
  uint32_t l[8];
};
struct CanonLess {
  __host__ __device__ bool operator()(const CanonKey& a, const CanonKey& b) const {
    for (int i = 7; i >= 0; i--)
      if (a.l[i] != b.l[i]) return a.l[i] < b.l[i];
    return false;
  }
};
hipError_t fr_to_canon(const Fr* in, CanonKey* out, size_t n, hipStream_t st);
// radix-sort keys key[i] = (bits [s, s + kbits) of canonical(in[i])) | tag (s < 256); key /
// canon / idx (optional) receive the keys, the canonical values and i; d_or[0..3] |= the
// values' 64-bit limbs
// the key step of several lookup columns in one launch (column t: in[t], window shift s[t],
// value-mask d_or[t]; its canon / key / idx regions at g[t] n of the batch buffers, its key
// tagged g[t] << kbits above the window; kmask = 2^kbits - 1)
static constexpr int LOOKUP_KEYS_BATCH_MAX = 32;
struct LookupKeysBatch {
  size_t n = 0;
  CanonKey* canon = nullptr;
  uint64_t* key = nullptr;
  uint32_t* idx = nullptr;
  uint64_t kmask = 0;
  int kbits = 48;
  int count = 0;
  const Fr* in[LOOKUP_KEYS_BATCH_MAX];
  int s[LOOKUP_KEYS_BATCH_MAX];
  int g[LOOKUP_KEYS_BATCH_MAX];
  unsigned long long* d_or[LOOKUP_KEYS_BATCH_MAX];
};
hipError_t lookup_keys_batch(const LookupKeysBatch& b, hipStream_t st);
hipError_t lookup_keys(const Fr* in, size_t n, int s, CanonKey* canon, uint64_t* key, uint32_t* idx,
                       unsigned long long* d_or, hipStream_t st, int kbits = 64, uint64_t tag = 0);
// out[i] = canon[idx[i]]; *unsorted |= 1 if out is not non-decreasing
hipError_t lookup_gather(const CanonKey* canon, const uint32_t* idx, size_t u, CanonKey* out,
                         unsigned long long* unsorted, hipStream_t st);
// canonical values below 2^64 from their low limbs
hipError_t key64_expand(const uint64_t* in, CanonKey* out, size_t n, hipStream_t st);
// run starts of the sorted input; each distinct input value marks its first occurrence in
// the sorted table (lower_bound); *fail counts input values missing from the table
hipError_t lookup_mark(const CanonKey* a, const CanonKey* t, size_t u, uint8_t* rep_flag, uint8_t* left_flag,
                       uint32_t* fail, hipStream_t st);
// Ap[r] = a[r]; Sp[r] = a[r] at run starts
hipError_t lookup_assign(const CanonKey* a, const uint8_t* rep_flag, size_t u, Fr* ap, Fr* sp, hipStream_t st);
// Sp[R[nrep - 1 - i]] = L[i]  (BTreeMap order, repeated rows popped from the end)
hipError_t lookup_scatter(const CanonKey* L, const uint32_t* R, const uint32_t* d_nrep, size_t cap, Fr* sp,
                          hipStream_t st);
// prod[i] = (beta + ap[i]) (gamma + sp[i])   and   prod[i] *= (a[i] + beta) (s[i] + gamma)
hipError_t lookup_prod_den(const Fr* ap, const Fr* sp, const Fr& beta, const Fr& gamma, Fr* prod, size_t n,
                           hipStream_t st);
hipError_t lookup_prod_num(const Fr* a, const Fr* s, const Fr& beta, const Fr& gamma, Fr* prod, size_t n,
                           hipStream_t st);
// shuffle: prod[i] = gamma + s[i]   and   prod[i] *= gamma + a[i]
hipError_t shuffle_prod_den(const Fr* s, const Fr& gamma, Fr* prod, size_t n, hipStream_t st);
hipError_t shuffle_prod_num(const Fr* a, const Fr& gamma, Fr* prod, size_t n, hipStream_t st);

// ---- polynomial evaluation (arithmetic.rs:57-82), batched ----
struct EvalReq {
  const Fr* poly;
  uint64_t len;
  Fr x;
};
// out[r] = sum_i reqs[r].poly[i] * reqs[r].x^i ; reqs/out in device memory; scratch >= eval_scratch_len
hipError_t poly_eval_batch(const EvalReq* d_reqs, int nreq, uint64_t max_len, Fr* d_out, Fr* scratch,
                           hipStream_t st);
size_t poly_eval_scratch_len(int nreq, uint64_t max_len);

// ---- kate_division (arithmetic.rs:101-120): q = (a - a(b)) / (X - b), len(q) = len(a) - 1 ----
// accumulate: q[0..len-1) += the quotient instead of =; scratch: kate_scratch_len(len)
hipError_t kate_division(const Fr* a, uint64_t len, const Fr& b, Fr* q, Fr* scratch, hipStream_t st,
                         bool accumulate = false);
size_t kate_scratch_len(uint64_t len);

// ---- linear combinations: out[i] = (acc ? out[i] : 0) + sum_k coef_k * p_k[i] (i < len_k) ----
static constexpr int LIN_MAXT = 12;
struct LinTerms {
  const Fr* p[LIN_MAXT];
  uint64_t len[LIN_MAXT];
  Fr coef[LIN_MAXT];
  int k = 0;
};
hipError_t lincomb(Fr* out, uint64_t n, const LinTerms& t, bool accumulate, hipStream_t st);
// out[i] = a[i] * (*scalar) (device scalar)
hipError_t scale_by_dev(Fr* out, const Fr* a, uint64_t n, const Fr* scalar, hipStream_t st);

// ---- keygen helpers ----
// sigma[r] = delta^col[r] * omega^row[r]  (permutation/keygen.rs:139-170)
hipError_t sigma_from_mapping(Fr* sigma, const uint32_t* map_col, const uint32_t* map_row, size_t n,
                              const Fr* delta_pow, const PowTable& omega, hipStream_t st);
// out[i] = [L_i(s)] G for the Lagrange SRS: L_i(s) = mult * w^i / (s - w^i) (kzg/commitment.rs:92-131)
hipError_t srs_lagrange_scalars(Fr* out, size_t n, const Fr& s, const Fr& mult, const PowTable& omega, Fr* scratch,
                                hipStream_t st);
hipError_t g1_generator_mul(const Fr* scalars, size_t n, G1Affine* out, hipStream_t st);

// ---- SerdeFormat::RawBytes checks (helpers.rs:40-48): *bad += count of elements not
// below the modulus (Fr arrays) / points with a coordinate >= p or off y^2 = x^3 + 3
// (identity (0, 0) allowed).  *bad must be zeroed by the caller.
hipError_t fr_count_unreduced(const Fr* a, size_t n, uint32_t* bad, hipStream_t st);
hipError_t g1_count_invalid(const G1Affine* p, size_t n, uint32_t* bad, hipStream_t st);

// ---- SerdeFormat::Processed (helpers.rs:36-100; serde.hip): 32-B compressed G1 points
// (GroupEncoding) and canonical field elements (to_repr / from_repr).  Decompression and
// from_repr add the number of invalid encodings to *bad (zeroed by the caller).
hipError_t g1_compress(const G1Affine* p, size_t n, uint8_t* out, hipStream_t st);
hipError_t g1_decompress(const uint8_t* in, size_t n, G1Affine* out, uint32_t* bad, hipStream_t st);
hipError_t fr_to_repr(const Fr* a, size_t n, Fr* out, hipStream_t st);
hipError_t fr_from_repr(Fr* a, size_t n, uint32_t* bad, hipStream_t st);

}  // namespace h2g
