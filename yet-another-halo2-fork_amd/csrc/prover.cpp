// prover.cpp -- keygen and create_proof on the device (BN254 / KZG / SHPLONK).
//
// Host orchestration of halo2_backend's prover, all polynomial data resident in HBM:
//   keygen_vk / keygen_pk          plonk/keygen.rs:43-190, circuit.rs:95-180,292-320
//   permutation Assembly/build_pk  plonk/permutation/keygen.rs:16-213
//   Prover::new_with_engine        plonk/prover.rs:174-305 (instances)
//   commit_phase                   plonk/prover.rs:309-494 (every advice phase, challenges after each)
//   create_proof                   plonk/prover.rs:512-899
//   permutation_commit/evaluate    plonk/permutation/prover.rs:50-333
//   vanishing commit/construct     plonk/vanishing/prover.rs:40-205
//   evaluate_h                     plonk/evaluation.rs:317-483
//   SHPLONK                        poly/kzg/multiopen/shplonk/prover.rs:121-305, shplonk.rs:48-140
// Host work is the transcript, the prover RNG's few hundred draws, query bookkeeping
// and O(#queries^2) interpolation; every length-n or extended-length operation is a
// kernel (MSM, NTT, prover_kernels.hip, poly.hip).  MSM results come back to the host
// (they enter the transcript), which is the only per-step synchronisation.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <functional>
#include <set>
#include <thread>

#include <unistd.h>

#include "comm.h"
#include "comm_wait.h"
#include "poly.h"
#include "radix.h"
#include "g2.h"
#include "prover_kernels.h"
#include "runtime.h"
#include "srs.h"
#include "transcript.h"

namespace h2g {
hipError_t link_delay(hipStream_t after, hipEvent_t done, double us);  // calib.hip
}

using namespace h2g;
using namespace h2g::rt;

namespace {

enum { COL_ADVICE = 0, COL_FIXED = 1, COL_INSTANCE = 2 };
enum { OP_CONST = 0, OP_QUERY = 1, OP_NEG = 2, OP_SUM = 3, OP_PROD = 4, OP_CHALLENGE = 5 };

struct Pool {  // owns device allocations of one params / pk object
  std::vector<void*> ptrs;
  hipError_t get(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  ~Pool() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};
#define PALLOC(pool, ptr, count) HIPCHK((pool).get((void**)&(ptr), (size_t)(count) * sizeof(*(ptr))))

struct Params {
  int device = 0;
  uint32_t k = 0;
  size_t n = 0;
  G1Affine* g = nullptr;
  G1Affine* gl = nullptr;
  MsmFixedBase fg, fgl;  // fixed-base MSM windows of g and g_lagrange (commit / commit_lagrange)
  // this rank's point slab [slab_lo, slab_hi) when one proof spans several GPUs: windows
  // sized for the slab length (h2g_params_set_slab)
  size_t slab_lo = 0, slab_hi = 0;
  MsmFixedBase sg, sgl;
  // windows of the prefix-summed Lagrange basis (params_prefix): built with the first key
  // that has lookups (keygen, outside any timed proof), for the whole basis (fgp) or -- once
  // a slab is set -- for the slab only (sgp), as sg / sgl are
  MsmFixedBase fgp, sgp;
  // the G2 half of ParamsKZG (g2, s_g2 = [s] g2; verifier side, serialised with the params)
  bool has_g2 = false;
  G2Affine g2, s_g2;
  Pool pool;
  ~Params() {
    msm_fixed_base_free(&fg);
    msm_fixed_base_free(&fgl);
    msm_fixed_base_free(&sg);
    msm_fixed_base_free(&sgl);
    msm_fixed_base_free(&fgp);
    msm_fixed_base_free(&sgp);
  }
  // windows and table offset serving the base range [off, off + n) of set 0 (g) / 1
  // (g_lagrange) / 2 (the Lagrange prefix sums: the slab's windows once built, else full)
  const MsmFixedBase& tables(int set, size_t off, size_t n, size_t* table_off) const {
    if (sg.table && off >= slab_lo && off + n <= slab_hi && (set != 2 || sgp.table)) {
      *table_off = off - slab_lo;
      return set == 0 ? sg : (set == 1 ? sgl : sgp);
    }
    if (set == 2) {
      *table_off = off;
      return fgp;
    }
    *table_off = off;
    return set == 0 ? fg : fgl;
  }
};

// The lookup commitments' basis.  A lookup's permuted columns A', S' are sorted into runs
// of equal values (permute_expression_pair), so with P_i = L_0 + ... + L_i,
//   sum_i a_i L_i = sum_i (a_i - a_{i+1}) P_i   (a_n = 0; the sum telescopes),
// the same commitment from scalars that are zero inside every run: the MSM's partition
// drops zero digits at the source, so its work follows the number of runs, not n.
// Windows of the prefix basis: for all n points (fgp; keygen builds them for keys with
// lookups, outside any proof) or for the rank's slab (sgp; built on the first set-2 MSM
// inside the slab, so a peer that only serves slabs never holds the full-size table).  Both
// need the prefix points of the whole basis (P_i sums every L_j below i), formed in scratch.
int params_prefix_build(Params& p, hipStream_t st, size_t lo, size_t hi, MsmFixedBase* out) {
  G1Affine* pre = nullptr;
  HIPCHK(hipMalloc(&pre, p.n * sizeof(G1Affine)));
  hipError_t e = msm_prefix_points(p.gl, p.n, pre, st);
  if (e == hipSuccess) e = msm_fixed_base_build(pre + lo, hi - lo, 0, out, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(pre);
  HIPCHK(e);
  return H2G_OK;
}
// before set-2 MSMs over [off, off + n): the slab's windows serve it if they exist, else the
// full windows, built here if nothing built them earlier (a fallback; normally a no-op)
int params_prefix(Params& p, hipStream_t st, size_t off = 0, size_t n = 0) {
  if (p.slab_hi > p.slab_lo && off >= p.slab_lo && off + n <= p.slab_hi && n > 0) {
    // inside this rank's slab: the slab's windows, built on first use (not in
    // h2g_params_set_slab, so params used without lookups never pay for them)
    if (!p.sgp.table) RCCHK(params_prefix_build(p, st, p.slab_lo, p.slab_hi, &p.sgp));
    return H2G_OK;
  }
  if (p.fgp.table) return H2G_OK;
  return params_prefix_build(p, st, 0, p.n, &p.fgp);
}

int params_finish(Params& p, hipStream_t st) {
  HIPCHK(msm_fixed_base_build(p.g, p.n, 0, &p.fg, st));
  HIPCHK(msm_fixed_base_build(p.gl, p.n, 0, &p.fgl, st));
  HIPCHK(hipStreamSynchronize(st));
  return H2G_OK;
}

struct Query {
  int type, index, rot;
  bool operator==(const Query& o) const { return type == o.type && index == o.index && rot == o.rot; }
};

// Per-circuit workspace of create_proof (one per circuit of a proof over several
// circuits, grown on demand and reused across proofs): the advice / instance columns,
// permutation, lookup and shuffle polynomials, and the device pointer tables that
// evaluate_h and the expression compressions read for this circuit.
struct CircuitWs {
  Pool pool;
  std::vector<Fr*> adv, adv_poly, adv_coset, inst_val, inst_poly, inst_coset, z, z_lag, z_coset;
  std::vector<Fr*> lk_a, lk_s, lk_ap, lk_sp, lk_ap_poly, lk_sp_poly, lk_z, lk_z_poly, lk_zc, lk_apc, lk_spc;
  std::vector<Fr*> sh_z, sh_z_poly, sh_zc;
  const Fr** d_load_col = nullptr;      // extended-coset columns (evaluate_h)
  const Fr** d_load_col_lag = nullptr;  // Lagrange columns (lookup / shuffle compression)
  const Fr** d_z = nullptr;
  const Fr** d_perm_v = nullptr;
  EvalLookup* d_lookups = nullptr;
  EvalShuffle* d_shuffles = nullptr;
  uint64_t* wit_pin = nullptr;  // advice staging of the witness source (num_advice x n Fr), pinned if possible
  bool wit_pin_pinned = false;
  // SPMD sub-coset split: per owned sub-coset i, the evaluate_h pointer tables with every
  // extended-coset column replaced by its sub-coset i (built for ProvingKey::sub_key)
  struct SubTables {
    const Fr** load_col = nullptr;
    const Fr** z = nullptr;
    const Fr** perm_v = nullptr;
    EvalLookup* lookups = nullptr;
    EvalShuffle* shuffles = nullptr;
  };
  std::vector<SubTables> sub;
  int64_t sub_key = -1;
  ~CircuitWs() {
    if (!wit_pin) return;
    if (wit_pin_pinned) (void)hipHostFree(wit_pin);
    else std::free(wit_pin);
  }
};

struct ProvingKey {
  int device = 0;
  uint64_t params = 0;
  uint32_t k = 0;
  size_t n = 0, ext = 0;
  uint64_t rot_scale = 0;
  int degree = 0, bf = 0, P = 0, nsets = 0, chunk_len = 0;
  int A = 0, F = 0, I = 0;
  std::vector<Query> adv_q, fix_q, ins_q;
  std::vector<std::pair<int, int>> perm_cols;
  std::vector<uint8_t> unblinded;
  // advice_column_phase, challenge_phase (ConstraintSystemMid); challenge values live in
  // consts[num_consts ..]
  std::vector<uint8_t> adv_phase, ch_phase;
  int num_consts = 0, max_phase = 0;
  Fr transcript_repr;
  // verifying-key commitments (fixed, permutation) of a key read from bytes; a key made
  // by keygen computes them when it is written (h2g_pk_write)
  std::vector<G1Affine> vk_fixed, vk_perm;
  // multi-open scheme of create_proof (the Prover type parameter, prover.rs:19-36):
  // 0 ProverSHPLONK, 1 ProverGWC; GWC witness polynomials, one per opening point
  int multiopen = 0;
  int transcript = 0;  // TRANSCRIPT_BLAKE2B / TRANSCRIPT_KECCAK256 (transcript.h)
  std::vector<Fr*> gwc_q;
  uint32_t* lk_cnt = nullptr;  // pinned per-(circuit, lookup) match counters (LKC each)
  size_t lk_cnt_len = 0;
  // per-(circuit, lookup) device counters and table-row flags of the match, so that one
  // memset each clears every lookup's and one copy brings all counters back
  static constexpr int LKC = 8;
  // the lookups' gathers and matches on LKS streams (lookup j's on stream j mod LKS), each
  // stream with its own scratch set; set 0 is the one above (ck_a2 ... rep_rows, lkb_scr)
  static constexpr int LKS = 4;
  hipStream_t lk_st[LKS] = {};
  hipEvent_t lk_ev[LKS + 1] = {};
  CanonKey *lks_a2[LKS] = {}, *lks_t2[LKS] = {}, *lks_left[LKS] = {};
  uint8_t* lks_rep[LKS] = {};
  uint32_t* lks_rows[LKS] = {};
  void* lks_scr[LKS] = {};
  size_t lks_n = 0;
  uint32_t* lk_counters = nullptr;
  uint8_t* lk_flags = nullptr;
  size_t lk_cf_n = 0, lk_cf_u = 0;
  Fr* lk_diff = nullptr;  // the lookup commitments' prefix-basis scalars (2 per lookup and circuit)
  size_t lk_diff_len = 0;
  // permute_expression_pair's sort, chosen per lookup from the value width lk_hb[l] (bit
  // length of the largest canonical value) seen by the previous proof: <= 64 bits: radix
  // sort of the values themselves; wider: radix sort of a 48-bit window of the top bits
  // with the row index, gather, and a sortedness check; 0: merge sort of the 256-bit
  // values.  lk_or_* (device / pinned, LKF per lookup): the limbs' OR and the check flag.
  static constexpr int LKF = 5;
  std::vector<int> lk_hb;
  unsigned long long *lk_or_d = nullptr, *lk_or_h = nullptr;
  size_t lk_or_len = 0;  // (circuit, lookup) entries of lk_or_*
  // SPMD witness checksums of an advice phase (copy_columns), device / pinned, and the event
  // that their copy to the host has landed (spmd_witness_fold)
  unsigned long long *wsum_d = nullptr, *wsum_h = nullptr;
  size_t wsum_len = 0;
  hipEvent_t wsum_ev = nullptr;
  // pinned staging of a proof's small host-to-device uploads (blinding rows, seeds, staged
  // scalars; pk_upload): from pageable memory a hipMemcpyAsync costs 8-60 us of host time
  // (a staged copy), which left the GPU idle between the keccak-style circuit's 32 advice
  // columns; from pinned memory the copy is queued at once.  Re-armed per proof
  uint8_t* up_h = nullptr;
  size_t up_len = 0, up_off = 0;
  Domain dom;
  Pool pool;
  // proving key (device)
  std::vector<Fr*> fixed_lag, fixed_poly, fixed_coset, sigma_lag, sigma_poly, sigma_coset;
  Fr *l0 = nullptr, *l_last = nullptr, *l_active = nullptr;
  PowTable om, eo;
  int4* prog = nullptr;
  int prog_len = 0, n_slots = 0;
  int2 seg_gates = {0, 0};
  std::vector<int2> seg_lk_in, seg_lk_tab, seg_sh_in, seg_sh_sh;  // expression-list programs
  // lookup l's table expressions equal lookup lk_trep[l]'s (the first such; l itself when
  // none): the proof sorts that table once (H2G_LK_SHARED_TABLES)
  std::vector<int> lk_trep;
  Fr* consts = nullptr;
  int n_loads = 0;
  std::vector<Query> loads;  // the programs' load table (column, rotation)
  int* d_load_rot = nullptr;
  const Fr** d_sigma = nullptr;
  int NL = 0, NS = 0;  // lookups, shuffles
  Fr *tmp_a = nullptr, *tmp_b = nullptr, *one = nullptr;
  CanonKey *ck_a2 = nullptr, *ck_t2 = nullptr, *ck_left = nullptr;
  uint8_t *rep_flag = nullptr, *left_flag = nullptr;
  uint32_t *rep_rows = nullptr, *counters = nullptr;
  // per-proof workspace (device), reused across proofs: per circuit, and shared
  std::vector<std::unique_ptr<CircuitWs>> cws;
  Fr *mod = nullptr, *pre = nullptr, *scr = nullptr, *random_poly = nullptr, *h_ext = nullptr, *h_coeff = nullptr;
  Fr *h_poly = nullptr, *nx = nullptr, *q1 = nullptr, *hx = nullptr, *lx = nullptr;
  Fr *small = nullptr, *last_z = nullptr, *evals = nullptr, *eval_scr = nullptr;
  // SPMD sub-coset split (h2g_spmd_transport.bcast): this rank's sub-cosets t = rank,
  // rank + world, ... < 2^e of the extended domain; the key's cosets cut to them (slot i
  // of each buffer = sub-coset sub_ts[i]), per-slot sigma tables, and the 2^e x n slots
  // the h evaluations are broadcast through
  int64_t sub_key = -1;  // (world * 65536 + rank) * 2 + pieces the cache holds
  std::vector<uint64_t> sub_ts;
  // more ranks than sub-cosets (world a multiple of 2^e, with the slab exchange): rank r
  // evaluates rows [sub_lo, sub_hi) of sub-coset r mod 2^e -- piece r / 2^e of world / 2^e
  // -- and holds its columns there with a halo of rotations [rot_lo, rot_hi]
  bool sub_pieces = false;
  uint64_t sub_lo = 0, sub_hi = 0;
  int rot_lo = -1, rot_hi = 1;
  Fr* cs_scr = nullptr;  // column ownership: the owned columns' 2^e sub-cosets
  size_t cs_scr_len = 0;
  Fr* perm_lz = nullptr;  // slab-wise grand products: z at each set's slab start
  size_t perm_lz_len = 0;
  std::vector<Fr*> sub_fixed, sub_sigma;
  Fr *sub_l0 = nullptr, *sub_ll = nullptr, *sub_la = nullptr;
  std::vector<const Fr**> d_sigma_sub;
  Fr* h_gather = nullptr;
  size_t scr_len = 0, eval_scr_len = 0;
  EvalReq* d_reqs = nullptr;
  int max_reqs = 0;
  // permute_expression_pair's batched sort: every lookup column's canonical values, keys
  // and row indices (ping-pong pairs), radix / compaction scratch
  CanonKey* lkb_canon = nullptr;
  uint64_t* lkb_key[2] = {nullptr, nullptr};
  uint32_t* lkb_idx[2] = {nullptr, nullptr};
  void* lkb_scr = nullptr;
  size_t lkb_len = 0;
  // SPMD coefficient slabs: per SHPLONK point a (slab + halo) combination buffer
  Fr* slab_buf = nullptr;
  size_t slab_buf_len = 0;
  // SPMD h(X) by slabs (h2g_spmd_transport.exchange): send / receive staging
  Fr *x_send = nullptr, *x_recv = nullptr;
  size_t x_send_len = 0, x_recv_len = 0;
  // SPMD column ownership: the pack / unpack copy lists (host lists live until the next
  // stage, after a stream synchronisation, so their asynchronous uploads have completed)
  CopySeg* d_segs = nullptr;
  size_t d_segs_len = 0;
  std::vector<CopySeg> h_segs[2];
  // overlapped column-ownership exchanges (h2g_set_spmd_exchange_async), in posting order:
  // each its own send / receive staging (grow-only, reused by the same position in the
  // next proof), completion event and unpack list, live from its post until xp_flush
  struct XPending {
    Fr *send = nullptr, *recv = nullptr;
    size_t send_len = 0, recv_len = 0;
    hipEvent_t done = nullptr;
    std::vector<CopySeg> unpack;
    bool live = false;
  };
  std::vector<XPending> xp;
  size_t xp_used = 0;
  // a stage's blinding rows, uploaded in one copy (upload_rows_batch)
  Fr* blind_d = nullptr;
  size_t blind_d_len = 0;
  uint32_t* d_seeds = nullptr;
  uint64_t* d_offsets = nullptr;
  int max_chunks = 0;
  // the keystream position of the vanishing argument's seed draws in the last proof with
  // the seeded RNG (the draws before them depend on the circuit's shape only), and its
  // thread count: the next proof generates and commits the random polynomial early
  int64_t van_pos = -1;
  uint32_t van_T = 0;
};

std::map<uint64_t, std::unique_ptr<Params>> g_params;
std::map<uint64_t, std::unique_ptr<ProvingKey>> g_pks;
std::vector<std::pair<const char*, double>> g_stages;
bool g_stage_sync = false;  // h2g_prover_stage_sync: stage times = GPU completion times
bool g_comm_overlap = false;  // h2g_comm_set_exchange_overlap: column exchanges on the second communicator

// ------------------------------------------------------------------ host field helpers
int fr_cmp(const Fr& a, const Fr& b) {  // Ord on Fr: canonical numeric order
  const Fr ca = to_canonical(a), cb = to_canonical(b);
  for (int i = 7; i >= 0; i--) {
    if (ca.l[i] < cb.l[i]) return -1;
    if (ca.l[i] > cb.l[i]) return 1;
  }
  return 0;
}
Fr fr_neg_one() { return Fr::zero() - Fr::one(); }

Fr rotate_omega(const Domain& d, const Fr& x, int rot) {
  return x * pow_u64(rot >= 0 ? d.omega : d.omega_inv, (uint64_t)(rot >= 0 ? rot : -rot));
}

// the Lagrange basis of the points: out[j] = coefficients of prod_{k != j} (X - p_k) / (p_j - p_k)
std::vector<std::vector<Fr>> lagrange_basis(const std::vector<Fr>& pts) {
  const size_t m = pts.size();
  std::vector<std::vector<Fr>> out(m);
  for (size_t j = 0; j < m; j++) {
    std::vector<Fr> num(1, Fr::one());
    Fr den = Fr::one();
    for (size_t k = 0; k < m; k++) {
      if (k == j) continue;
      std::vector<Fr> nn(num.size() + 1, Fr::zero());
      for (size_t i = 0; i < num.size(); i++) {
        nn[i + 1] = nn[i + 1] + num[i];
        nn[i] = nn[i] - pts[k] * num[i];
      }
      num.swap(nn);
      den = den * (pts[j] - pts[k]);
    }
    const Fr sc = inv(den);
    for (Fr& c : num) c = c * sc;
    out[j] = std::move(num);
  }
  return out;
}
Fr eval_host(const std::vector<Fr>& p, const Fr& x) {
  Fr acc = Fr::zero();
  for (size_t i = p.size(); i-- > 0;) acc = acc * x + p[i];
  return acc;
}

// two-level power table of w for exponents < 2^L
int build_pow_table(Pool& pool, const Fr& w, int L, PowTable* t, hipStream_t st) {
  const int bits = (L + 1) / 2;
  const size_t nlo = (size_t)1 << bits, nhi = (size_t)1 << (L - bits > 0 ? L - bits : 0);
  std::vector<Fr> lo(nlo), hi(nhi);
  lo[0] = Fr::one();
  for (size_t i = 1; i < nlo; i++) lo[i] = lo[i - 1] * w;
  const Fr wb = lo[nlo - 1] * w;  // w^(2^bits)
  hi[0] = Fr::one();
  for (size_t i = 1; i < nhi; i++) hi[i] = hi[i - 1] * wb;
  Fr *dlo, *dhi;
  PALLOC(pool, dlo, nlo);
  PALLOC(pool, dhi, nhi);
  HIPCHK(hipMemcpyAsync(dlo, lo.data(), nlo * sizeof(Fr), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dhi, hi.data(), nhi * sizeof(Fr), hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  t->lo = dlo;
  t->hi = dhi;
  t->bits = bits;
  return H2G_OK;
}

// Debug aid: a build with -DH2G_DUMP_DIR='"<dir>"' writes named intermediates (raw Fr
// arrays) of create_proof to <dir>/p<pid>/<name>.bin, one directory per process (rank); no
// run-time switch in the shipped library
void dump(const char* name, const Fr* dptr, size_t count, hipStream_t st, bool host = false) {
#ifndef H2G_DUMP_DIR
  (void)name, (void)dptr, (void)count, (void)st, (void)host;
  return;
#else
  const std::string dir = std::string(H2G_DUMP_DIR) + "/p" + std::to_string((long)getpid());
  std::vector<Fr> h(count);
  if (host) std::memcpy(h.data(), dptr, count * sizeof(Fr));
  else {
    (void)hipStreamSynchronize(st);
    (void)hipMemcpy(h.data(), dptr, count * sizeof(Fr), hipMemcpyDeviceToHost);
  }
  const std::string path = dir + "/" + name + ".bin";
  if (FILE* f = std::fopen(path.c_str(), "wb")) {
    std::fwrite(h.data(), sizeof(Fr), count, f);
    std::fclose(f);
  }
#endif
}

// ParamsKZG::commit / commit_lagrange (kzg/commitment.rs:305-317,354-366): MSM against a
// prefix of the resident SRS (fixed-base windows).  Launched asynchronously after the
// work queued on `st`; the affine result is collected when it enters the transcript.
// With a shard transport installed (h2g_set_shard_transport) the MSM is split into point
// slabs: this device takes slab 0, the peers the rest.
// SRS_LAGRANGE_PREFIX: prefix sums of the Lagrange basis, P_i = L_0 + ... + L_i (params_prefix)
enum { SRS_G = 0, SRS_LAGRANGE = 1, SRS_LAGRANGE_PREFIX = 2 };
h2g_shard_transport g_shard{nullptr, 1, nullptr, nullptr};
uint64_t g_shard_seq = 0;
// SPMD sharding (h2g_set_spmd_transport): every rank proves, rank r computes slab r
h2g_spmd_transport g_spmd{nullptr, 1, 0, nullptr, nullptr};
uint64_t g_spmd_seq = 0;
// row pieces: the advice transforms run in the permutation stage when every transform of
// the proof has a rank of its own (prove_impl); 0 keeps them in the advice stage (A/B)
#ifndef H2G_DEFER_ADV_XFORM
#define H2G_DEFER_ADV_XFORM 1
#endif
// Single-GPU proofs: the columns' transforms (lagrange_to_coeff, the coset extension) on a
// stream of their own (Device::xstream), joined before evaluate_h, their first reader.
// On the prover's stream they held back every later stage's kernels -- the lookups'
// sorts and grand products are chains of small launches that leave most of the chip idle,
// and ran only after the 2^20-point transforms ahead of them on the stream (keccak-style
// k = 18: the same 33.1 ms with every stage drained as without; 31.8-32.4 vs 33.3-34.3 ms
// on their own stream, profiles/r06/xs/ab_ordered_streams.log).  Only for circuits with
// lookups or shuffles: C3 (no lookups; its stages are MSM-bound, the chip already full)
// measured 76.1-77.3 vs 73.1-73.8 ms with it.  The stream is created by the first proof
// that uses it, after the MSM streams (the hardware-queue order matters, abi.cpp).  Stream
// priorities (transforms low, or MSMs high) measured slower (profiles/r06/xs/).  0: on the
// prover's stream.
#ifndef H2G_XFORM_STREAM
#define H2G_XFORM_STREAM 1
#endif
#ifndef H2G_LK_SHARED_TABLES  // A/B: 0 = every lookup sorts its own table column
#define H2G_LK_SHARED_TABLES 1
#endif
#ifndef H2G_XS_ALL  // A/B: 1 = the transform stream for circuits without lookups too
#define H2G_XS_ALL 0
#endif
// overlapped exchanges (h2g_set_spmd_exchange_async); NULL post: exchanges complete on return
h2g_spmd_exchange_post g_xpost = nullptr;
h2g_spmd_exchange_wait g_xwait = nullptr;
// time, calls and bytes (sent + received) inside the transport, per collective kind
// (h2g_spmd_stats): 0 MSM all-gathers, 1 host all-gathers, 2 exchanges, 3 broadcasts
struct SpmdStats {
  double ms[4] = {};
  uint64_t calls[4] = {}, bytes[4] = {};
};
SpmdStats g_spmd_stats;
template <class F>
int spmd_timed(int kind, uint64_t bytes, F&& f) {
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = f();
  g_spmd_stats.ms[kind] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  g_spmd_stats.calls[kind]++;
  g_spmd_stats.bytes[kind] += bytes;
  return rc;
}
int spmd_exchange(const void* d_send, const size_t* sb, void* d_recv, const size_t* rb) {
  uint64_t bytes = 0;
  for (int r = 0; r < g_spmd.world; r++) bytes += sb[r] + rb[r];
  return spmd_timed(2, bytes, [&] { return g_spmd.exchange(g_spmd.ctx, d_send, sb, d_recv, rb); });
}
// the running proof's transcript, RNG draws and witness, whose digest travels with every
// SPMD partial (H2G_SPMD_WORDS): ranks that diverged fail the proof instead of summing
// slabs of different polynomials.  The witness enters as a 64-bit checksum of every advice
// column, over the whole column on each rank, taken by the kernel that copies the column
// in (copy_columns; spmd_witness_fold): with the slabs summed, the commitments and
// evaluations alone would be the same on ranks fed different witnesses.  The checksums
// reach the host behind the stream and are folded in when the next collective needs the
// digest (spmd_witness_settle), so the check costs no synchronisation of its own.
struct SpmdCheck {
  const Transcript* tr = nullptr;
  const ProverRng* rng = nullptr;
  uint8_t wit[64] = {};
  const unsigned long long* pend = nullptr;  // pinned checksums still to fold (pend_n), ready at pend_ev
  int pend_n = 0;
  hipEvent_t pend_ev = nullptr;
};
SpmdCheck g_spmd_check;
void spmd_witness_settle() {
  SpmdCheck& c = g_spmd_check;
  if (!c.pend) return;
  (void)hipEventSynchronize(c.pend_ev);
  Blake2b h("h2g-spmd-witness");
  h.update(c.wit, 64);
  h.update(reinterpret_cast<const uint8_t*>(c.pend), (size_t)c.pend_n * sizeof(unsigned long long));
  h.digest(c.wit);
  c.pend = nullptr;
  c.pend_n = 0;
}
struct SpmdCheckScope {
  SpmdCheckScope(const Transcript* tr, const ProverRng* rng) {
    g_spmd_check = SpmdCheck{};
    g_spmd_check.tr = tr;
    g_spmd_check.rng = rng;
  }
  ~SpmdCheckScope() { g_spmd_check = SpmdCheck{}; }
};
void spmd_digest(uint64_t out[4]) {
  uint8_t a[64] = {}, b[64] = {}, d[64];
  spmd_witness_settle();
  if (g_spmd_check.tr) g_spmd_check.tr->state_digest(a);
  if (g_spmd_check.rng) g_spmd_check.rng->draws_digest(b);
  Blake2b h("h2g-spmd-check\0\0");
  h.update(a, 64);
  h.update(b, 64);
  h.update(g_spmd_check.wit, 64);
  h.digest(d);
  std::memcpy(out, d, 32);
}

hipError_t pk_upload(ProvingKey& pk, void* dst, const void* src, size_t bytes, hipStream_t st);

// SPMD column ownership of wide stages (h2g_spmd_set_column_owners; on by default)
bool g_spmd_colshard = true;
// ... from this world size up.  Ownership trades transform work for an all-to-all of the
// owned columns' sub-coset pieces: each rank sends (W - 1) / W of its 1 / W share of the
// extended-domain data, over W - 1 point-to-point xGMI links at once, i.e. ~D / W^2 per
// link for D bytes of cosets.  At W = 2 that is D / 4 on ONE link (keccak-style k = 18: D
// ~ 3 GB -> ~0.75 GB, ~12 ms at ~64 GB/s, against ~10 ms of transforms saved); at W = 4
// D / 16 and at W = 8 D / 64 (~50 MB per link, < 1 ms)
constexpr int kColshardMinWorld = 4;

// SPMD slab weights (h2g_spmd_set_weights): prefix sums, world + 1 entries; empty = uniform
std::vector<uint64_t> g_spmd_wprefix;

// slab r of an MSM of length n: the points [P r / world, P (r + 1) / world) of the
// params' P = 2^k, clipped to n (one partition for every MSM length, so each rank's
// slab windows cover all of its MSMs); SPMD with weights: [P S_r / S, P S_{r+1} / S)
size_t shard_lo(size_t P, size_t n, int world, int r) {
  size_t b;
  if (world > 1 && world == g_spmd.world && g_spmd_wprefix.size() == (size_t)world + 1)
    b = (size_t)((unsigned __int128)P * g_spmd_wprefix[(size_t)r] / g_spmd_wprefix[(size_t)world]);
  else
    b = (size_t)((unsigned __int128)P * (unsigned)r / (unsigned)world);
  return b < n ? b : n;
}

int commit_launch(Device* d, const Params& prm, const Fr* scalars, size_t n, int set, hipStream_t st, MsmTicket* t) {
  t->shard_seq = -1;
  size_t toff = 0;
  if (g_spmd.world > 1) {  // this rank's slab of its own copy of the scalars
    const size_t lo = shard_lo(prm.n, n, g_spmd.world, g_spmd.rank);
    const size_t hi = shard_lo(prm.n, n, g_spmd.world, g_spmd.rank + 1);
    const MsmFixedBase& tb = prm.tables(set, lo, hi - lo, &toff);
    RCCHK(msm_fixed_launch(d, scalars + lo, tb, toff, hi - lo, st, t));
    t->shard_seq = (int64_t)g_spmd_seq++;
    return H2G_OK;
  }
  if (g_shard.world <= 1) return msm_fixed_launch(d, scalars, prm.tables(set, 0, n, &toff), 0, n, st, t);
  const size_t n0 = shard_lo(prm.n, n, g_shard.world, 1);
  const MsmFixedBase& tb = prm.tables(set, 0, n0, &toff);
  RCCHK(msm_fixed_launch(d, scalars, tb, toff, n0, st, t));
  HIPCHK(hipStreamSynchronize(st));  // the transport reads the scalars right away
  const uint64_t seq = g_shard_seq++;
  if (g_shard.launch(g_shard.ctx, seq, set, n, scalars) != 0)
    return fail(H2G_ERR_STATE, "shard transport: launch of MSM " + std::to_string(seq) + " failed");
  t->shard_seq = (int64_t)seq;
  return H2G_OK;
}
int commit_collect(Device* d, MsmTicket* t, G1Affine* out) {
  if (t->remote) {  // owned by another rank: this rank's part of the sum is the identity
    std::memset(out, 0, sizeof(G1Affine));
    t->remote = false;
  } else {
    RCCHK(msm_collect(d, t, reinterpret_cast<uint64_t*>(out)));
  }
  if (t->shard_seq < 0) return H2G_OK;
  if (g_spmd.world > 1) {  // every rank's partial, summed in rank order (the same on every rank)
    const int W = g_spmd.world;
    constexpr int SW = H2G_SPMD_WORDS;
    uint64_t mine[SW];
    std::memcpy(mine, out, 64);
    mine[8] = out->is_identity() ? 1 : 0;
    spmd_digest(mine + 9);
    std::vector<uint64_t> all((size_t)W * SW);
    const int64_t seq = t->shard_seq;
    if (spmd_timed(0, (uint64_t)SW * 8 * (W + 1), [&] { return g_spmd.allgather(g_spmd.ctx, (uint64_t)seq, mine, all.data()); }) != 0)
      return fail(H2G_ERR_STATE, "spmd transport: all-gather of MSM " + std::to_string(seq) + " failed");
    t->shard_seq = -1;
    for (int r = 0; r < W; r++)
      if (std::memcmp(&all[(size_t)r * SW + 9], mine + 9, 32) != 0)
        return fail(H2G_ERR_STATE, "spmd: rank " + std::to_string(r) + " diverged from rank " +
                                       std::to_string(g_spmd.rank) + " before MSM " + std::to_string(seq) +
                                       " (different witness, instances, key or RNG draws on the ranks)");
    G1xyzz acc = G1xyzz::identity();
    for (int r = 0; r < W; r++) {
      if (all[(size_t)r * SW + 8]) continue;
      G1Affine p;
      std::memcpy(&p, &all[(size_t)r * SW], 64);
      acc = xyzz_madd(acc, p);
    }
    *out = xyzz_to_affine(acc);
    return H2G_OK;
  }
  const int peers = g_shard.world - 1;
  std::vector<G1Affine> part(peers);
  std::vector<int32_t> ids(peers, 0);
  if (g_shard.collect(g_shard.ctx, (uint64_t)t->shard_seq, reinterpret_cast<uint64_t*>(part.data()), ids.data()) != 0)
    return fail(H2G_ERR_STATE, "shard transport: collect of MSM " + std::to_string(t->shard_seq) + " failed");
  t->shard_seq = -1;
  G1xyzz acc = G1xyzz::identity();
  if (!out->is_identity()) acc = G1xyzz::from_affine(*out);
  for (int i = 0; i < peers; i++)
    if (!ids[i]) acc = xyzz_madd(acc, part[i]);
  *out = xyzz_to_affine(acc);
  return H2G_OK;
}
// The commitments of one stage together (the stage's MSMs were all launched before the
// first is needed): with SPMD and a host all-gather, every rank's partials of all of them
// travel in ONE all-gather (nb x H2G_SPMD_WORDS words per rank, one digest check), not one
// collective per MSM -- a many-column proof at 8 ranks made ~90 of them, each a host
// round trip of the ranks' streams.  The sums are the same, in rank order, as
// commit_collect's; the transcript writes follow in list order.
constexpr uint64_t kSpmdCommitTag = 0x54494d4d4f433248ull;  // "H2COMMIT"
int commit_collect_all(Device* d, MsmTicket* const* t, int nb, G1Affine* out) {
  bool spmd_all = g_spmd.world > 1 && g_spmd.allgather_host && nb > 1;
  bool local_all = nb > 1;  // plain single-GPU tickets
  for (int i = 0; i < nb; i++) {
    spmd_all &= t[i]->shard_seq >= 0;
    local_all &= t[i]->shard_seq < 0 && !t[i]->remote;
  }
  // the results leave the device in XYZZ form and go to affine together, one host inversion
  // per stage instead of one per commitment (~10 us each: ~0.3 ms a stage of 32)
  std::vector<G1xyzz> xz(nb > 0 ? nb : 1);
  if (local_all) {
    for (int i = 0; i < nb; i++) RCCHK(msm_collect_xyzz(d, t[i], &xz[i]));
    xyzz_to_affine_batch(xz.data(), out, nb);
    return H2G_OK;
  }
  if (!spmd_all) {
    for (int i = 0; i < nb; i++) RCCHK(commit_collect(d, t[i], &out[i]));
    return H2G_OK;
  }
  for (int i = 0; i < nb; i++) {
    if (t[i]->remote) {
      xz[i] = G1xyzz::identity();
      t[i]->remote = false;
    } else {
      RCCHK(msm_collect_xyzz(d, t[i], &xz[i]));
    }
  }
  xyzz_to_affine_batch(xz.data(), out, nb);
  const int W = g_spmd.world;
  constexpr int SW = H2G_SPMD_WORDS;
  // per rank: a 2-word header (tag, count -- lets a transport or a test harness recognise
  // a commitment batch), then nb records of H2G_SPMD_WORDS words as in commit_collect
  const size_t per = 2 + (size_t)nb * SW;
  std::vector<uint64_t> mine(per), all((size_t)W * per);
  mine[0] = kSpmdCommitTag;
  mine[1] = (uint64_t)nb;
  uint64_t dg[4];
  spmd_digest(dg);
  for (int i = 0; i < nb; i++) {
    uint64_t* m = &mine[2 + (size_t)i * SW];
    std::memcpy(m, &out[i], 64);
    m[8] = out[i].is_identity() ? 1 : 0;
    std::memcpy(m + 9, dg, 32);
  }
  const int64_t seq0 = t[0]->shard_seq;
  const size_t bytes = mine.size() * 8;
  if (spmd_timed(0, bytes * (W + 1), [&] { return g_spmd.allgather_host(g_spmd.ctx, mine.data(), bytes, all.data()); }) != 0)
    return fail(H2G_ERR_STATE, "spmd transport: all-gather of MSMs " + std::to_string(seq0) + ".. failed");
  for (int r = 0; r < W; r++)
    for (int i = 0; i < nb; i++)
      if (all[(size_t)r * per] != kSpmdCommitTag || all[(size_t)r * per + 1] != (uint64_t)nb ||
          std::memcmp(&all[(size_t)r * per + 2 + (size_t)i * SW + 9], dg, 32) != 0)
        return fail(H2G_ERR_STATE, "spmd: rank " + std::to_string(r) + " diverged from rank " +
                                       std::to_string(g_spmd.rank) + " before MSM " + std::to_string(seq0 + i) +
                                       " (different witness, instances, key or RNG draws on the ranks)");
  for (int i = 0; i < nb; i++) {
    t[i]->shard_seq = -1;
    G1xyzz acc = G1xyzz::identity();
    for (int r = 0; r < W; r++) {
      const uint64_t* a = &all[(size_t)r * per + 2 + (size_t)i * SW];
      if (a[8]) continue;
      G1Affine p;
      std::memcpy(&p, a, 64);
      acc = xyzz_madd(acc, p);
    }
    xz[i] = acc;
  }
  xyzz_to_affine_batch(xz.data(), out, nb);
  return H2G_OK;
}

#ifndef H2G_LOOKUP_PREFIX  // A/B builds: 0 = the lookup commitments against the Lagrange basis itself
#define H2G_LOOKUP_PREFIX 1
#endif

// Several commitments against one base set as batched MSMs (msm_run_fixed_batch): one
// sort, accumulation and reduction serve a group, so the latency-bound reduction is paid
// once per group instead of once per commitment -- what circuits with many columns at
// small k (C5) are dominated by (commit_batch_chunk); with a shard transport every MSM
// goes alone (point slabs).  SPMD ranks batch their slab MSMs the same way: a 2^19-point
// slab's reduction costs about what a 2^22 MSM's does.
// MSMs per batch for commitments of length n (1: no batching).  Batching pays where
// the reduction's latency is comparable to the accumulation: measured on MI355X, a
// keccak-style k = 18 proof (80 MSMs of 2^18) 127 -> 101 ms, while C3 at k = 22 (MSMs
// of 2^22, 13 x 2^22 entries each) is 0.6 ms better without -- so only MSMs of at most
// 2^25 sorted entries are batched, up to 2^27 entries per batch.
#ifndef H2G_MSM_BATCH_ENTRIES  // A/B builds (tools/build_variant.py --src prover.cpp -D...)
#define H2G_MSM_BATCH_ENTRIES (1ull << 27)
#endif
#ifndef H2G_MSM_BATCH_PER  // the largest MSM (sorted entries) that is batched
#define H2G_MSM_BATCH_PER (1ull << 25)
#endif
int commit_batch_chunk(const MsmFixedBase& tb, size_t n) {
  const uint64_t max_entries = H2G_MSM_BATCH_ENTRIES;
  if (g_shard.world > 1) return 1;
  const uint64_t per = (uint64_t)tb.W * (n ? n : 1);
  if (per > H2G_MSM_BATCH_PER) return 1;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(MSM_MAX_BATCH, max_entries / per));
}

// the points this rank's commitments of length n cover ([0, n), or its SPMD slab as in
// commit_launch) and the windows serving them
const MsmFixedBase& commit_tables(const Params& prm, size_t n, int set, size_t* lo, size_t* hi, size_t* toff) {
  *lo = 0;
  *hi = n;
  if (g_spmd.world > 1) {
    *lo = shard_lo(prm.n, n, g_spmd.world, g_spmd.rank);
    *hi = shard_lo(prm.n, n, g_spmd.world, g_spmd.rank + 1);
  }
  return prm.tables(set, *lo, *hi - *lo, toff);
}
int commit_batch_chunk(const Params& prm, size_t n, int set) {
  size_t lo, hi, toff;
  const MsmFixedBase& tb = commit_tables(prm, n, set, &lo, &hi, &toff);
  return commit_batch_chunk(tb, hi - lo);
}

int commit_launch_batch(Device* d, const Params& prm, const Fr* const* scalars, int nb, size_t n, int set,
                        hipStream_t st, MsmTicket* t) {
  size_t lo, hi, toff;
  const MsmFixedBase& tb = commit_tables(prm, n, set, &lo, &hi, &toff);
  const int chunk = commit_batch_chunk(tb, hi - lo);
  if (chunk < 2) {
    for (int b = 0; b < nb; b++) RCCHK(commit_launch(d, prm, scalars[b], n, set, st, &t[b]));
    return H2G_OK;
  }
  for (int b0 = 0; b0 < nb; b0 += chunk) {
    const int m = std::min(chunk, nb - b0);
    const Fr* sl[MSM_MAX_BATCH];
    for (int b = 0; b < m; b++) sl[b] = scalars[b0 + b] + lo;
    RCCHK(msm_fixed_launch_batch(d, reinterpret_cast<const void* const*>(sl), m, tb, toff, hi - lo, st, t + b0));
    // SPMD: every rank issues the same MSMs in the same order, so the sequence numbers agree
    for (int b = 0; b < m; b++) t[b0 + b].shard_seq = g_spmd.world > 1 ? (int64_t)g_spmd_seq++ : -1;
  }
  return H2G_OK;
}

// SPMD column ownership (wide stages): commitment i of the list is computed whole by rank
// owner[i] (its own ones batched, against the full windows), every other rank contributes
// the identity to its all-gather -- the sum is the owner's commitment, and the transcript
// and the sequence numbers stay the same on every rank.
int commit_launch_owned(Device* d, const Params& prm, const Fr* const* scalars, const int* owner, int nb, size_t n,
                        int set, hipStream_t st, MsmTicket* t) {
  std::vector<const Fr*> mine;
  std::vector<int> at;
  for (int i = 0; i < nb; i++)
    if (owner[i] == g_spmd.rank) {
      mine.push_back(scalars[i]);
      at.push_back(i);
    }
  const MsmFixedBase& tb = set == SRS_G ? prm.fg : (set == SRS_LAGRANGE ? prm.fgl : prm.fgp);
  const int chunk = std::max(1, commit_batch_chunk(tb, n));
  std::vector<MsmTicket> got(mine.size());
  for (size_t b0 = 0; b0 < mine.size(); b0 += (size_t)chunk) {
    const int m = (int)std::min<size_t>((size_t)chunk, mine.size() - b0);
    RCCHK(msm_fixed_launch_batch(d, reinterpret_cast<const void* const*>(mine.data() + b0), m, tb, 0, n, st,
                                 got.data() + b0));
  }
  for (size_t q = 0; q < at.size(); q++) t[at[q]] = got[q];
  for (int i = 0; i < nb; i++) {
    if (owner[i] != g_spmd.rank) {
      t[i] = MsmTicket{};
      t[i].remote = true;
    }
    t[i].shard_seq = (int64_t)g_spmd_seq++;
  }
  return H2G_OK;
}

int commit(Device* d, const Params& prm, const Fr* scalars, size_t n, int set, G1Affine* out, hipStream_t st) {
  MsmTicket t;
  RCCHK(commit_launch(d, prm, scalars, n, set, st, &t));
  return commit_collect(d, &t, out);
}

// ------------------------------------------------------------------ circuit analysis
struct CircuitView {
  const h2g_circuit* c;
  const int32_t* node(int i) const { return c->nodes + 4 * i; }
};

int node_degree(const CircuitView& v, int i, std::vector<int>& memo) {
  if (memo[i] >= 0) return memo[i];
  const int32_t* nd = v.node(i);
  int d = 0;
  switch (nd[0]) {
    case OP_CONST:
    case OP_CHALLENGE: d = 0; break;
    case OP_QUERY: d = 1; break;
    case OP_NEG: d = node_degree(v, nd[1], memo); break;
    case OP_SUM: d = std::max(node_degree(v, nd[1], memo), node_degree(v, nd[2], memo)); break;
    default: d = node_degree(v, nd[1], memo) + node_degree(v, nd[2], memo); break;
  }
  return memo[i] = d;
}

// structurally equal expressions (the same operations on the same queries, constants and
// challenges by index)
bool same_expr(const CircuitView& v, int a, int b) {
  if (a == b) return true;
  const int32_t* x = v.node(a);
  const int32_t* y = v.node(b);
  if (x[0] != y[0]) return false;
  switch (x[0]) {
    case OP_CONST:
    case OP_CHALLENGE: return x[1] == y[1];
    case OP_QUERY: return x[1] == y[1] && x[2] == y[2] && x[3] == y[3];
    case OP_NEG: return same_expr(v, x[1], y[1]);
    default: return same_expr(v, x[1], y[1]) && same_expr(v, x[2], y[2]);
  }
}

void add_query(std::vector<Query>& l, const Query& q) {
  if (std::find(l.begin(), l.end(), q) == l.end()) l.push_back(q);
}

void collect(const CircuitView& v, int i, ProvingKey& pk) {  // keygen.rs:217-249, lhs before rhs
  const int32_t* nd = v.node(i);
  switch (nd[0]) {
    case OP_CONST:
    case OP_CHALLENGE: return;
    case OP_QUERY: {
      const Query q{nd[1], nd[2], nd[3]};
      add_query(nd[1] == COL_ADVICE ? pk.adv_q : (nd[1] == COL_FIXED ? pk.fix_q : pk.ins_q), q);
      return;
    }
    case OP_NEG: collect(v, nd[1], pk); return;
    default:
      collect(v, nd[1], pk);
      collect(v, nd[2], pk);
      return;
  }
}

// Gate expressions -> straight-line program over LDS value slots (tree code
// generation, larger subtree first to bound live slots; a - b fused as SUB).
struct GateCompiler {
  const CircuitView& v;
  std::vector<int4> prog;
  std::vector<Query> loads;
  std::vector<int> free_slots;
  int n_slots = 0;
  std::vector<int> need;
  explicit GateCompiler(const CircuitView& cv) : v(cv), need(cv.c->num_nodes, -1) {}
  int alloc() {
    if (!free_slots.empty()) {
      const int s = free_slots.back();
      free_slots.pop_back();
      return s;
    }
    return n_slots++;
  }
  void release(int s) { free_slots.push_back(s); }
  int regs(int i) {  // Sethi-Ullman register need
    if (need[i] >= 0) return need[i];
    const int32_t* nd = v.node(i);
    int r = 1;
    if (nd[0] == OP_NEG) r = regs(nd[1]);
    else if (nd[0] == OP_SUM || nd[0] == OP_PROD) {
      const int a = regs(nd[1]), b = regs(nd[2]);
      r = a == b ? a + 1 : std::max(a, b);
    }
    return need[i] = r;
  }
  int load_index(const Query& q) {
    for (size_t i = 0; i < loads.size(); i++)
      if (loads[i] == q) return (int)i;
    loads.push_back(q);
    return (int)loads.size() - 1;
  }
  // program segment: Horner (acc = acc * factor + e) over the expressions `roots`
  int2 compile_list(const int32_t* roots, int m) {
    const int off = (int)prog.size();
    for (int i = 0; i < m; i++) {
      const int s = gen(roots[i]);
      prog.push_back(make_int4(G_HORNER, 0, s, 0));
      release(s);
    }
    return make_int2(off, (int)prog.size() - off);
  }
  int gen(int i) {
    const int32_t* nd = v.node(i);
    switch (nd[0]) {
      case OP_CONST: {
        const int s = alloc();
        prog.push_back(make_int4(G_CONST, s, nd[1], 0));
        return s;
      }
      case OP_CHALLENGE: {  // challenge values follow the constants in pk.consts
        const int s = alloc();
        prog.push_back(make_int4(G_CONST, s, (int)v.c->num_constants + nd[1], 0));
        return s;
      }
      case OP_QUERY: {
        const int s = alloc();
        prog.push_back(make_int4(G_LOAD, s, load_index(Query{nd[1], nd[2], nd[3]}), 0));
        return s;
      }
      case OP_NEG: {
        const int a = gen(nd[1]);
        release(a);
        const int s = alloc();
        prog.push_back(make_int4(G_NEG, s, a, 0));
        return s;
      }
      default: {
        int lhs = nd[1], rhs = nd[2];
        int op = nd[0] == OP_SUM ? G_ADD : G_MUL;
        if (nd[0] == OP_SUM && v.node(rhs)[0] == OP_NEG) {  // a + (-b) -> a - b
          op = G_SUB;
          rhs = v.node(rhs)[1];
        }
        int a, b;
        if (regs(rhs) > regs(lhs)) {
          b = gen(rhs);
          a = gen(lhs);
        } else {
          a = gen(lhs);
          b = gen(rhs);
        }
        release(a);
        release(b);
        const int s = alloc();
        prog.push_back(make_int4(op, s, a, b));
        return s;
      }
    }
  }
};

bool check_nodes(const h2g_circuit* c, std::string* why) {
  const int64_t n = 1ll << c->k;
  for (uint32_t i = 0; i < c->num_nodes; i++) {
    const int32_t* nd = c->nodes + 4 * i;
    switch (nd[0]) {
      case OP_CONST:
        if (nd[1] < 0 || (uint32_t)nd[1] >= c->num_constants) return *why = "constant index", false;
        break;
      case OP_QUERY: {
        const uint32_t lim = nd[1] == COL_ADVICE ? c->num_advice : nd[1] == COL_FIXED ? c->num_fixed
                                                                   : nd[1] == COL_INSTANCE ? c->num_instance : 0;
        if (nd[2] < 0 || (uint32_t)nd[2] >= lim) return *why = "query column", false;
        if (nd[3] <= -n || nd[3] >= n) return *why = "rotation", false;
        break;
      }
      case OP_NEG:
        if (nd[1] < 0 || (uint32_t)nd[1] >= i) return *why = "node child must precede its parent", false;
        break;
      case OP_SUM:
      case OP_PROD:
        if (nd[1] < 0 || nd[2] < 0 || (uint32_t)nd[1] >= i || (uint32_t)nd[2] >= i)
          return *why = "node child must precede its parent", false;
        break;
      case OP_CHALLENGE:
        if (nd[1] < 0 || (uint32_t)nd[1] >= c->num_challenges) return *why = "challenge index", false;
        break;
      default: return *why = "node op", false;
    }
  }
  for (uint32_t g = 0; g < c->num_gates; g++)
    if (c->gate_roots[g] < 0 || (uint32_t)c->gate_roots[g] >= c->num_nodes) return *why = "gate root", false;
  auto check_args = [&](uint32_t na, const uint32_t* sizes, const int32_t* roots, const char* what) -> bool {
    if (na && (!sizes || !roots)) return *why = std::string("null ") + what, false;
    size_t off = 0;
    for (uint32_t l = 0; l < na; l++) {
      if (sizes[l] == 0) return *why = std::string(what) + " without expressions", false;
      for (uint32_t i = 0; i < 2 * sizes[l]; i++)
        if (roots[off + i] < 0 || (uint32_t)roots[off + i] >= c->num_nodes)
          return *why = std::string(what) + " root", false;
      off += 2 * sizes[l];
    }
    return true;
  };
  return check_args(c->num_lookups, c->lookup_sizes, c->lookup_roots, "lookup") &&
         check_args(c->num_shuffles, c->shuffle_sizes, c->shuffle_roots, "shuffle");
}

// per-argument root lists: (inputs, tables) of lookup l / (inputs, shuffles) of shuffle l
struct ArgRoots {
  const int32_t* in;
  const int32_t* other;
  int m;
};
std::vector<ArgRoots> arg_roots(uint32_t na, const uint32_t* sizes, const int32_t* roots) {
  std::vector<ArgRoots> out;
  size_t off = 0;
  for (uint32_t l = 0; l < na; l++) {
    const int m = (int)sizes[l];
    out.push_back({roots + off, roots + off + m, m});
    off += 2 * (size_t)m;
  }
  return out;
}

// ------------------------------------------------------------------ keygen
// Proving-key arrays taken from a serialised ProvingKey (h2g_pk_read, plonk.rs:311-359)
// instead of being computed: host pointers into the file buffer, raw Montgomery Fr
// (SerdeFormat::RawBytes layout = the device layout), or canonical Fr (Processed: each
// array is converted with from_repr on the device right after its upload, elements >= r
// counted into *bad).
struct PkImage {
  std::vector<const uint8_t*> fixed_lag, fixed_poly, fixed_coset, sigma_lag, sigma_poly, sigma_coset;
  const uint8_t *l0 = nullptr, *l_last = nullptr, *l_active = nullptr;
  bool canonical = false;
  uint32_t* bad = nullptr;  // device counter, Processed only
  hipError_t upload(Fr* dst, const uint8_t* src, size_t cnt, hipStream_t st) const {
    hipError_t e = hipMemcpyAsync(dst, src, cnt * sizeof(Fr), hipMemcpyHostToDevice, st);
    if (e == hipSuccess && canonical) e = fr_from_repr(dst, cnt, bad, st);
    return e;
  }
};

// one more circuit workspace (create_proof over pk.cws.size() + 1 circuits)
int circuit_ws_add(ProvingKey& pk) {
  auto w = std::make_unique<CircuitWs>();
  const size_t n = pk.n, ext = pk.ext;
  auto vec_alloc = [&](std::vector<Fr*>& v, int cnt, size_t len) -> hipError_t {
    v.assign(cnt, nullptr);
    for (int i = 0; i < cnt; i++) {
      hipError_t e = w->pool.get((void**)&v[i], len * sizeof(Fr));
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  HIPCHK(vec_alloc(w->adv, pk.A, n));
  HIPCHK(vec_alloc(w->adv_poly, pk.A, n));
  HIPCHK(vec_alloc(w->adv_coset, pk.A, ext));
  HIPCHK(vec_alloc(w->inst_val, pk.I, n));
  HIPCHK(vec_alloc(w->inst_poly, pk.I, n));
  HIPCHK(vec_alloc(w->inst_coset, pk.I, ext));
  HIPCHK(vec_alloc(w->z, pk.nsets, n));
  HIPCHK(vec_alloc(w->z_lag, pk.nsets, n));
  HIPCHK(vec_alloc(w->z_coset, pk.nsets, ext));
  HIPCHK(vec_alloc(w->lk_a, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_s, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_ap, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_sp, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_ap_poly, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_sp_poly, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_z, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_z_poly, pk.NL, n));
  HIPCHK(vec_alloc(w->lk_zc, pk.NL, ext));
  HIPCHK(vec_alloc(w->lk_apc, pk.NL, ext));
  HIPCHK(vec_alloc(w->lk_spc, pk.NL, ext));
  HIPCHK(vec_alloc(w->sh_z, pk.NS, n));
  HIPCHK(vec_alloc(w->sh_z_poly, pk.NS, n));
  HIPCHK(vec_alloc(w->sh_zc, pk.NS, ext));
  // pointer tables: the load table's columns for this circuit (fixed columns are shared)
  auto col = [&](const Query& q, bool coset) -> const Fr* {
    if (q.type == COL_ADVICE) return coset ? w->adv_coset[q.index] : w->adv[q.index];
    if (q.type == COL_FIXED) return coset ? pk.fixed_coset[q.index] : pk.fixed_lag[q.index];
    return coset ? w->inst_coset[q.index] : w->inst_val[q.index];
  };
  std::vector<const Fr*> lc(pk.n_loads + 1, nullptr), ll(pk.n_loads + 1, nullptr);
  for (int i = 0; i < pk.n_loads; i++) {
    lc[i] = col(pk.loads[i], true);
    ll[i] = col(pk.loads[i], false);
  }
  std::vector<EvalLookup> el(pk.NL + 1);
  std::vector<EvalShuffle> es(pk.NS + 1);
  for (int l = 0; l < pk.NL; l++) el[l] = EvalLookup{pk.seg_lk_in[l], pk.seg_lk_tab[l], w->lk_zc[l], w->lk_apc[l], w->lk_spc[l]};
  for (int l = 0; l < pk.NS; l++) es[l] = EvalShuffle{pk.seg_sh_in[l], pk.seg_sh_sh[l], w->sh_zc[l]};
  std::vector<const Fr*> zt(pk.nsets + 1), pv(pk.P + 1);
  for (int s = 0; s < pk.nsets; s++) zt[s] = w->z_coset[s];
  for (int i = 0; i < pk.P; i++) pv[i] = col(Query{pk.perm_cols[i].first, pk.perm_cols[i].second, 0}, true);
  PALLOC(w->pool, w->d_load_col, lc.size());
  PALLOC(w->pool, w->d_load_col_lag, ll.size());
  PALLOC(w->pool, w->d_lookups, el.size());
  PALLOC(w->pool, w->d_shuffles, es.size());
  PALLOC(w->pool, w->d_z, zt.size());
  PALLOC(w->pool, w->d_perm_v, pv.size());
  HIPCHK(hipMemcpy(w->d_load_col, lc.data(), lc.size() * sizeof(Fr*), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(w->d_load_col_lag, ll.data(), ll.size() * sizeof(Fr*), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(w->d_lookups, el.data(), el.size() * sizeof(EvalLookup), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(w->d_shuffles, es.data(), es.size() * sizeof(EvalShuffle), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(w->d_z, zt.data(), zt.size() * sizeof(Fr*), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(w->d_perm_v, pv.data(), pv.size() * sizeof(Fr*), hipMemcpyHostToDevice));
  pk.cws.push_back(std::move(w));
  return H2G_OK;
}

// ------------------------------------------------------------------ SPMD sub-cosets
// Row y = t + 2^e m of the extended coset (e = extended_k - k) is the point
// zeta w_ext^t w^m, so sub-coset t of a column is an n-point NTT of its coefficients
// twisted by w_ext^(t j), and evaluate_h on rows of one sub-coset reads only sub-coset t of
// every column: rotations move rows by multiples of 2^e (evaluation.rs:317-620 evaluates
// the same expressions row by row; the row split does not change any value).
bool spmd_subcosets() { return g_spmd.world > 1 && g_spmd.bcast != nullptr; }

// ------------------------------------------------------------------ SPMD coefficient slabs
// With h2g_spmd_transport.allgather_host the evaluations and the SHPLONK multi-open run on
// coefficient slabs: rank r owns coefficients [lo, hi) of every length-n polynomial (the
// points of its MSM slabs, shard_lo) and computes one more (hi, the halo) where a kate
// division reads a[i + 1].  Partial evaluations and the divisions' carries between slabs
// are the only values that cross ranks (a few Fr per proof).
struct Slab {
  size_t lo = 0, hi = 0;  // owned coefficients
  size_t hi1 = 0;         // hi + 1 (the halo coefficient), clipped to n
};
Slab spmd_slab(size_t n, int r) {
  Slab s;
  s.lo = shard_lo(n, n, g_spmd.world, r);
  s.hi = shard_lo(n, n, g_spmd.world, r + 1);
  s.hi1 = std::min(s.hi + 1, n);
  return s;
}
// every rank's `mine` (same count on each), rank order
int spmd_allgather_fr(const std::vector<Fr>& mine, std::vector<Fr>* all) {
  const size_t W = (size_t)g_spmd.world, cnt = mine.size();
  all->assign(W * cnt, Fr::zero());
  if (!cnt) return H2G_OK;
  if (spmd_timed(1, cnt * sizeof(Fr) * (W + 1),
                 [&] { return g_spmd.allgather_host(g_spmd.ctx, mine.data(), cnt * sizeof(Fr), all->data()); }) != 0)
    return fail(H2G_ERR_STATE, "spmd transport: host all-gather failed");
  return H2G_OK;
}
// out[i] (+)= sum_k coef_k p_k[i] for i in [lo, hi) only (global indices; out, p_k full-length)
int lincomb_range(Fr* out, size_t lo, size_t hi, LinTerms t, bool accumulate, hipStream_t st) {
  if (hi <= lo) return H2G_OK;
  for (int k = 0; k < t.k; k++) {
    t.len[k] = t.len[k] > lo ? std::min<uint64_t>(t.len[k], hi) - lo : 0;
    t.p[k] = t.len[k] ? t.p[k] + lo : t.p[k];
  }
  HIPCHK(lincomb(out + lo, hi - lo, t, accumulate, st));
  return H2G_OK;
}
// The kate divisions' carries: for a_i (global indexing, valid on [lo, hi1)) and point b_i,
// carry[i] = q_i[hi'] = sum_{j >= hi'} a_i[j + 1] b_i^(j - hi') (hi' = min(hi, n - 1)), from
// every slab's partial Horner value E_s = sum_{j in [lo_s, hi'_s)} a_i[j + 1] b_i^(j - lo_s):
// C_{W-1} = 0, C_r = E_{r+1} + b^(hi'_{r+1} - lo_{r+1}) C_{r+1}.  One all-gather for all points.
template <class Buf>
int slab_carries(ProvingKey& pk, const Slab& sl, size_t n, const std::vector<Fr>& pts, Buf a, std::vector<Fr>* carry,
                 hipStream_t st) {
  const size_t np = pts.size();
  const size_t hq = std::min(sl.hi, n - 1);
  const uint64_t m = hq > sl.lo ? hq - sl.lo : 0;
  std::vector<EvalReq> reqs(np);
  for (size_t i = 0; i < np; i++) reqs[i] = EvalReq{a(i) + sl.lo + 1, m, pts[i]};
  if ((int)np > pk.max_reqs) {
    PALLOC(pk.pool, pk.d_reqs, np);
    PALLOC(pk.pool, pk.evals, np);
    pk.max_reqs = (int)np;
  }
  const size_t need = poly_eval_scratch_len((int)np, m ? m : 1);
  if (need > pk.eval_scr_len) {
    PALLOC(pk.pool, pk.eval_scr, need);
    pk.eval_scr_len = need;
  }
  HIPCHK(pk_upload(pk, pk.d_reqs, reqs.data(), np * sizeof(EvalReq), st));
  HIPCHK(poly_eval_batch(pk.d_reqs, (int)np, m ? m : 1, pk.evals, pk.eval_scr, st));
  std::vector<Fr> mine(np);
  HIPCHK(hipMemcpyAsync(mine.data(), pk.evals, np * sizeof(Fr), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  std::vector<Fr> all;
  RCCHK(spmd_allgather_fr(mine, &all));
  carry->assign(np, Fr::zero());
  for (size_t i = 0; i < np; i++) {
    Fr c = Fr::zero();
    for (int s = g_spmd.world - 1; s > g_spmd.rank; s--) {
      const Slab ss = spmd_slab(n, s);
      const size_t hs = std::min(ss.hi, n - 1);
      const uint64_t ms = hs > ss.lo ? hs - ss.lo : 0;
      c = all[(size_t)s * np + i] + pow_u64(pts[i], ms) * c;
    }
    (*carry)[i] = c;
  }
  return H2G_OK;
}

// the key's cosets cut to this rank's sub-cosets, once per (world, rank, pieces)
int sub_prepare(ProvingKey& pk, hipStream_t st, bool pieces) {
  const int64_t key = ((int64_t)g_spmd.world * 65536 + g_spmd.rank) * 2 + (pieces ? 1 : 0);
  if (pk.sub_key == key) return H2G_OK;
  const int e = (int)(pk.dom.ek - pk.dom.k);
  const uint64_t E = 1ull << e;
  const size_t n = pk.n;
  pk.sub_ts.clear();
  pk.sub_pieces = pieces;
  if (pieces) {  // world = G E: rank r takes piece r / E of sub-coset r mod E
    const uint64_t G = (uint64_t)g_spmd.world / E, p = (uint64_t)g_spmd.rank / E;
    pk.sub_ts.push_back((uint64_t)g_spmd.rank % E);
    pk.sub_lo = (uint64_t)n * p / G;
    pk.sub_hi = (uint64_t)n * (p + 1) / G;
  } else {
    for (uint64_t t = (uint64_t)g_spmd.rank; t < E; t += (uint64_t)g_spmd.world) pk.sub_ts.push_back(t);
    pk.sub_lo = 0;
    pk.sub_hi = n;
  }
  // the rows a piece reads around its own: every query rotation, z(omega X), z(omega^last X),
  // the lookups' A'(omega^-1 X)
  pk.rot_lo = std::min(-1, -(pk.bf + 1));
  pk.rot_hi = 1;
  for (const Query& q : pk.loads) {
    pk.rot_lo = std::min(pk.rot_lo, q.rot);
    pk.rot_hi = std::max(pk.rot_hi, q.rot);
  }
  const size_t nt = pk.sub_ts.size();
  auto cut = [&](const Fr* full, Fr** out) -> int {
    if (!*out) HIPCHK(pk.pool.get((void**)out, pk.ext * sizeof(Fr)));  // room for any rank's slots
    for (size_t i = 0; i < nt; i++) HIPCHK(subcoset_gather(full, *out + i * n, n, pk.sub_ts[i], e, st));
    return H2G_OK;
  };
  pk.sub_fixed.resize(pk.F, nullptr);
  pk.sub_sigma.resize(pk.P, nullptr);
  for (int f = 0; f < pk.F; f++) RCCHK(cut(pk.fixed_coset[f], &pk.sub_fixed[f]));
  for (int c = 0; c < pk.P; c++) RCCHK(cut(pk.sigma_coset[c], &pk.sub_sigma[c]));
  RCCHK(cut(pk.l0, &pk.sub_l0));
  RCCHK(cut(pk.l_last, &pk.sub_ll));
  RCCHK(cut(pk.l_active, &pk.sub_la));
  pk.d_sigma_sub.assign(nt, nullptr);
  for (size_t i = 0; i < nt; i++) {
    std::vector<const Fr*> sg(pk.P + 1, nullptr);
    for (int c = 0; c < pk.P; c++) sg[c] = pk.sub_sigma[c] + i * n;
    PALLOC(pk.pool, pk.d_sigma_sub[i], sg.size());
    HIPCHK(hipMemcpy(pk.d_sigma_sub[i], sg.data(), sg.size() * sizeof(Fr*), hipMemcpyHostToDevice));
  }
  if (!pk.h_gather) PALLOC(pk.pool, pk.h_gather, pk.ext);
  HIPCHK(hipStreamSynchronize(st));
  pk.sub_key = key;
  return H2G_OK;
}

// a circuit workspace's evaluate_h tables for each owned sub-coset (cf. circuit_ws_add)
int sub_ws_tables(const ProvingKey& pk, CircuitWs& w) {
  if (w.sub_key == pk.sub_key) return H2G_OK;
  const size_t n = pk.n, nt = pk.sub_ts.size();
  w.sub.assign(nt, CircuitWs::SubTables{});
  for (size_t i = 0; i < nt; i++) {
    const size_t off = i * n;
    auto col = [&](const Query& q) -> const Fr* {
      if (q.type == COL_ADVICE) return w.adv_coset[q.index] + off;
      if (q.type == COL_FIXED) return pk.sub_fixed[q.index] + off;
      return w.inst_coset[q.index] + off;
    };
    std::vector<const Fr*> lc(pk.n_loads + 1, nullptr);
    for (int j = 0; j < pk.n_loads; j++) lc[j] = col(pk.loads[j]);
    std::vector<EvalLookup> el(pk.NL + 1);
    std::vector<EvalShuffle> es(pk.NS + 1);
    for (int l = 0; l < pk.NL; l++)
      el[l] = EvalLookup{pk.seg_lk_in[l], pk.seg_lk_tab[l], w.lk_zc[l] + off, w.lk_apc[l] + off, w.lk_spc[l] + off};
    for (int l = 0; l < pk.NS; l++) es[l] = EvalShuffle{pk.seg_sh_in[l], pk.seg_sh_sh[l], w.sh_zc[l] + off};
    std::vector<const Fr*> zt(pk.nsets + 1, nullptr), pv(pk.P + 1, nullptr);
    for (int q = 0; q < pk.nsets; q++) zt[q] = w.z_coset[q] + off;
    for (int c = 0; c < pk.P; c++) pv[c] = col(Query{pk.perm_cols[c].first, pk.perm_cols[c].second, 0});
    CircuitWs::SubTables& S = w.sub[i];
    PALLOC(w.pool, S.load_col, lc.size());
    PALLOC(w.pool, S.lookups, el.size());
    PALLOC(w.pool, S.shuffles, es.size());
    PALLOC(w.pool, S.z, zt.size());
    PALLOC(w.pool, S.perm_v, pv.size());
    HIPCHK(hipMemcpy(S.load_col, lc.data(), lc.size() * sizeof(Fr*), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(S.lookups, el.data(), el.size() * sizeof(EvalLookup), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(S.shuffles, es.data(), es.size() * sizeof(EvalShuffle), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(S.z, zt.data(), zt.size() * sizeof(Fr*), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(S.perm_v, pv.data(), pv.size() * sizeof(Fr*), hipMemcpyHostToDevice));
  }
  w.sub_key = pk.sub_key;
  return H2G_OK;
}

// the extended-coset columns evaluate_h reads (coeff_to_extended, domain.rs:230-244):
// whole cosets, or under the SPMD sub-coset split this rank's sub-cosets (slot i of dst =
// sub-coset sub_ts[i]; a rank past 2^e owns none and computes nothing)
int ext_cosets(Device* d, const ProvingKey& pk, const Fr* const* src, Fr* const* dst, int count, hipStream_t st) {
  if (!spmd_subcosets()) return coeff_to_extended_batch(d, pk.dom, src, dst, count, st);
  const size_t n = pk.n, nt = pk.sub_ts.size();
  std::vector<const Fr*> s2;
  std::vector<Fr*> d2;
  for (int c = 0; c < count; c++)
    for (size_t i = 0; i < nt; i++) {
      Fr* o = dst[c] + i * n;
      HIPCHK(subcoset_twist(src[c], o, n, pk.eo, pk.sub_ts[i], pk.ext - 1, st));
      s2.push_back(o);
      d2.push_back(o);
    }
  const Fr one = Fr::one();
  for (size_t b0 = 0; b0 < s2.size(); b0 += NTT_MAX_BATCH)
    RCCHK(ntt_dev_impl_batch(d, s2.data() + b0, n, d2.data() + b0, (int)std::min<size_t>(NTT_MAX_BATCH, s2.size() - b0),
                             n, (int)pk.dom.k, pk.dom.omega, 1, pk.dom.g_coset, pk.dom.g_coset_inv, 0, one, 0, one,
                             one, st));
  return H2G_OK;
}

// SPMD h(X) by coefficient slabs (h2g_spmd_transport.exchange): the owner of sub-coset t
// holds h's evaluations H(zeta w_ext^t w^m) in h_gather slot t.  An n-point inverse NTT
// (1/n, times zeta^-j) and the twist w_ext^(-t j) give the folded coefficients
// F_t[j] = sum_p h_{j+np} zeta^(np) rho^(t p) (rho = w_ext^n); slab r of every F_t goes
// to rank r, which inverts the E-point transform over t for its coefficients:
// h_{j+np} = zeta^(-np) E^-1 sum_t rho^(-t p) F_t[j] (extended_to_coeff, domain.rs:271-293,
// split into pieces of n, vanishing/prover.rs:122-128).  Exact, so the pieces equal the
// single-GPU ones.
int h_by_slabs(Device* d, ProvingKey& pk, const Slab& sl, hipStream_t st) {
  const Domain& D = pk.dom;
  const size_t n = pk.n, ext = pk.ext;
  const int W = g_spmd.world, me = g_spmd.rank;
  const int e = (int)(D.ek - D.k);
  const int E = 1 << e;
  const int np = pk.degree - 1;
  if (E > HSLAB_MAX_E || np > E) return fail(H2G_ERR_ARG, "create_proof: too many sub-cosets for the h slab exchange");
  // the sub-cosets this rank interpolates (with row pieces: the leaders, ranks < E)
  std::vector<uint64_t> ts = pk.sub_ts;
  if (pk.sub_pieces && me >= E) ts.clear();
  const size_t nt = ts.size();
  // sizes: slab r of each owned sub-coset to rank r; every owner's blocks to me
  std::vector<size_t> sb(W), rb(W), soff(W + 1, 0);
  std::vector<Slab> slabs(W);
  for (int r = 0; r < W; r++) {
    slabs[r] = spmd_slab(n, r);
    sb[r] = nt * (slabs[r].hi1 - slabs[r].lo) * sizeof(Fr);
    soff[r + 1] = soff[r] + sb[r] / sizeof(Fr);
    int own = 0;
    for (int t = r; t < E; t += W) own++;
    rb[r] = (size_t)own * (sl.hi1 - sl.lo) * sizeof(Fr);
  }
  size_t rtot = 0;
  for (int r = 0; r < W; r++) rtot += rb[r] / sizeof(Fr);
  if (soff[W] > pk.x_send_len) {
    PALLOC(pk.pool, pk.x_send, soff[W]);
    pk.x_send_len = soff[W];
  }
  if (rtot > pk.x_recv_len) {
    PALLOC(pk.pool, pk.x_recv, rtot);
    pk.x_recv_len = rtot;
  }
  const Fr one = Fr::one();
  for (size_t i = 0; i < nt; i++) {
    const uint64_t t = ts[i];
    Fr* f = pk.h_coeff + i * n;  // scratch until the combine
    RCCHK(ntt_dev_impl(d, pk.h_gather + t * n, n, f, n, (int)D.k, D.omega_inv, 0, one, one, 1, D.ifft_div, 1,
                       D.g_coset_inv, D.g_coset, st));
    HIPCHK(subcoset_twist(f, f, n, pk.eo, (ext - t) & (ext - 1), ext - 1, st));
    for (int r = 0; r < W; r++) {
      const size_t cnt = slabs[r].hi1 - slabs[r].lo;
      if (cnt)
        HIPCHK(hipMemcpyAsync(pk.x_send + soff[r] + i * cnt, f + slabs[r].lo, cnt * sizeof(Fr), hipMemcpyDeviceToDevice,
                              st));
    }
  }
  // combine coefficients coef[p E + t] = zeta^(-n p) rho^(-t p) / E
  std::vector<Fr> coef((size_t)np * E);
  {
    Fr ef = Fr::zero();
    for (int i = 0; i < E; i++) ef = ef + one;
    const Fr einv = inv(ef);
    const Fr rho_inv = inv(pow_u64(D.ext_omega, n));
    const Fr zinv_n = pow_u64(inv(zeta()), n);
    Fr zp = einv;
    for (int p = 0; p < np; p++) {
      Fr w = zp;
      const Fr step = pow_u64(rho_inv, (uint64_t)p);
      for (int t = 0; t < E; t++) {
        coef[(size_t)p * E + t] = w;
        w = w * step;
      }
      zp = zp * zinv_n;
    }
  }
  HIPCHK(pk_upload(pk, pk.small, coef.data(), coef.size() * sizeof(Fr), st));
  HIPCHK(hipStreamSynchronize(st));  // the send staging is complete; coef (host) was read
  if (spmd_exchange(pk.x_send, sb.data(), pk.x_recv, rb.data()) != 0)
    return fail(H2G_ERR_STATE, "spmd transport: exchange of h slabs failed");
  HSlabArgs a;
  a.recv = pk.x_recv;
  int pos = 0;
  for (int o = 0; o < W; o++)
    for (int t = o; t < E; t += W) a.idx[t] = pos++;
  a.E = E;
  a.np = np;
  a.cnt = sl.hi1 - sl.lo;
  a.n = n;
  a.lo = sl.lo;
  a.coef = pk.small;
  a.out = pk.h_coeff;
  HIPCHK(h_slab_combine(a, st));
  return H2G_OK;
}

// SPMD with more ranks than sub-cosets (E = 2^e): ranks 0 .. E-1 own the sub-cosets and
// hold every coefficient column whole; ranks E.. skipped those iNTTs and receive their slab
// [lo, hi1) of each column (column c from owner c mod E), one all-to-all per proof.
int coef_exchange(ProvingKey& pk, const std::vector<Fr*>& cols, hipStream_t st) {
  const size_t n = pk.n;
  const int W = g_spmd.world, me = g_spmd.rank;
  const int E = 1 << (pk.dom.ek - pk.dom.k);
  const int nc = (int)cols.size();
  std::vector<Slab> slabs(W);
  for (int r = 0; r < W; r++) slabs[r] = spmd_slab(n, r);
  auto ncols_of = [&](int o) {  // columns owner o sends
    int c = 0;
    for (int i = o; i < nc; i += E) c++;
    return c;
  };
  std::vector<size_t> sb(W, 0), rb(W, 0);
  size_t stot = 0, rtot = 0;
  for (int r = 0; r < W; r++) {
    if (me < E && r >= E) sb[r] = (size_t)ncols_of(me) * (slabs[r].hi1 - slabs[r].lo) * sizeof(Fr);
    if (me >= E && r < E) rb[r] = (size_t)ncols_of(r) * (slabs[me].hi1 - slabs[me].lo) * sizeof(Fr);
    stot += sb[r] / sizeof(Fr);
    rtot += rb[r] / sizeof(Fr);
  }
  if (stot > pk.x_send_len) {
    PALLOC(pk.pool, pk.x_send, stot);
    pk.x_send_len = stot;
  }
  if (rtot > pk.x_recv_len) {
    PALLOC(pk.pool, pk.x_recv, rtot);
    pk.x_recv_len = rtot;
  }
  if (me < E) {  // pack: per destination, my columns' slabs
    size_t off = 0;
    for (int r = E; r < W; r++) {
      const size_t cnt = slabs[r].hi1 - slabs[r].lo;
      for (int c = me; c < nc; c += E) {
        if (cnt) HIPCHK(hipMemcpyAsync(pk.x_send + off, cols[c] + slabs[r].lo, cnt * sizeof(Fr),
                                       hipMemcpyDeviceToDevice, st));
        off += cnt;
      }
    }
  }
  HIPCHK(hipStreamSynchronize(st));
  if (spmd_exchange(pk.x_send, sb.data(), pk.x_recv, rb.data()) != 0)
    return fail(H2G_ERR_STATE, "spmd transport: exchange of coefficient slabs failed");
  if (me >= E) {  // unpack: owner by owner, its columns in order
    const size_t cnt = slabs[me].hi1 - slabs[me].lo;
    size_t off = 0;
    for (int o = 0; o < E; o++)
      for (int c = o; c < nc; c += E) {
        if (cnt) HIPCHK(hipMemcpyAsync(cols[c] + slabs[me].lo, pk.x_recv + off, cnt * sizeof(Fr),
                                       hipMemcpyDeviceToDevice, st));
        off += cnt;
      }
  }
  return H2G_OK;
}

// The rows of the extended domain rank r holds: (sub-coset t, its slot, first row a,
// count len; rows wrap mod n) -- whole sub-cosets t = r, r + world, ... when world <= 2^e,
// else its piece of sub-coset r mod 2^e with the halo of rotations around it
struct RowPiece {
  uint64_t t;
  int slot;
  uint64_t a, len;
};
std::vector<RowPiece> pieces_of(const ProvingKey& pk, int r) {
  const int W = g_spmd.world;
  const uint64_t E = 1ull << (pk.dom.ek - pk.dom.k), n = pk.n;
  std::vector<RowPiece> v;
  if (pk.sub_pieces) {
    const uint64_t G = (uint64_t)W / E, p = (uint64_t)r / E;
    const uint64_t lo = n * p / G, hi = n * (p + 1) / G;
    const uint64_t len = std::min<uint64_t>(n, hi - lo + (uint64_t)(pk.rot_hi - pk.rot_lo));
    const uint64_t a = (uint64_t)(((int64_t)lo + (int64_t)n + pk.rot_lo) % (int64_t)n);
    v.push_back({(uint64_t)r % E, 0, a, len});
  } else {
    int slot = 0;
    for (uint64_t t = (uint64_t)r; t < E; t += (uint64_t)W) v.push_back({t, slot++, 0, n});
  }
  return v;
}

// SPMD column ownership (SURVEY 8e's round-robin whole columns): column i of a stage is
// rank owner[i]'s, which alone forms its coefficients (the n-point iNTT, prover.rs:673-689 /
// lookup/prover.rs:131,311) and its E = 2^e sub-cosets (n-point NTTs of the twisted
// coefficients: the cosets of evaluation.rs:344-361) in its scratch.  One all-to-all then
// hands every rank the rows of every column it evaluates h on (pieces_of) and its
// coefficient slab [lo, hi1) (what the evaluations and SHPLONK read).  Message from o to r:
// per column of o in index order, r's pieces (in order, wrapped rows as two runs), then r's
// coefficient slab.  Used for wide stages (the owners also commit) and, with row pieces,
// for every stage (the transforms then never run twice).
int colshard_distribute(Device* d, ProvingKey& pk, const std::vector<const Fr*>& lag, const std::vector<Fr*>& poly,
                        const std::vector<Fr*>& coset, const std::vector<int>& owner, hipStream_t st) {
  const size_t n = pk.n;
  const int W = g_spmd.world, me = g_spmd.rank;
  const int E = 1 << (pk.dom.ek - pk.dom.k);
  const int M = (int)lag.size();
  std::vector<Slab> slabs(W);
  std::vector<std::vector<RowPiece>> pcs(W);
  for (int r = 0; r < W; r++) {
    slabs[r] = spmd_slab(n, r);
    pcs[r] = pieces_of(pk, r);
  }
  auto rows_of = [&](int r) {
    uint64_t w = 0;
    for (const RowPiece& pc : pcs[r]) w += pc.len;
    return w;
  };
  std::vector<int> mine;  // this rank's columns, index order
  for (int i = 0; i < M; i++)
    if (owner[i] == me) mine.push_back(i);
  std::vector<size_t> sb(W, 0), rb(W, 0), soff(W + 1, 0);
  for (int r = 0; r < W; r++) {
    if (r != me) {
      sb[r] = mine.size() * (rows_of(r) + (slabs[r].hi1 - slabs[r].lo)) * sizeof(Fr);
      size_t cols_r = 0;
      for (int i = 0; i < M; i++) cols_r += owner[i] == r;
      rb[r] = cols_r * (rows_of(me) + (slabs[me].hi1 - slabs[me].lo)) * sizeof(Fr);
    }
    soff[r + 1] = soff[r] + sb[r] / sizeof(Fr);
  }
  size_t rtot = 0;
  for (int r = 0; r < W; r++) rtot += rb[r] / sizeof(Fr);
  // overlapped: this exchange's own staging (the next stage packs while it is in flight);
  // otherwise the shared one
  ProvingKey::XPending* xp = nullptr;
  if (g_xpost) {
    if (pk.xp_used == pk.xp.size()) pk.xp.emplace_back();
    xp = &pk.xp[pk.xp_used];
    if (soff[W] > xp->send_len) {
      PALLOC(pk.pool, xp->send, soff[W]);
      xp->send_len = soff[W];
    }
    if (rtot > xp->recv_len) {
      PALLOC(pk.pool, xp->recv, rtot);
      xp->recv_len = rtot;
    }
    if (!xp->done) HIPCHK(hipEventCreateWithFlags(&xp->done, hipEventDisableTiming));
  } else {
    if (soff[W] > pk.x_send_len) {
      PALLOC(pk.pool, pk.x_send, soff[W]);
      pk.x_send_len = soff[W];
    }
    if (rtot > pk.x_recv_len) {
      PALLOC(pk.pool, pk.x_recv, rtot);
      pk.x_recv_len = rtot;
    }
  }
  Fr* const xs = xp ? xp->send : pk.x_send;
  Fr* const xr = xp ? xp->recv : pk.x_recv;
  const size_t scr = mine.size() * (size_t)E * n;
  if (scr > pk.cs_scr_len) {
    PALLOC(pk.pool, pk.cs_scr, scr);
    pk.cs_scr_len = scr;
  }
  auto run_segs = [&](std::vector<CopySeg>& v) -> int {  // one launch for a copy list
    if (v.empty()) return H2G_OK;
    if (v.size() > pk.d_segs_len) {
      PALLOC(pk.pool, pk.d_segs, v.size());
      pk.d_segs_len = v.size();
    }
    uint64_t mx = 0;
    for (const CopySeg& g : v) mx = std::max<uint64_t>(mx, g.len);
    HIPCHK(pk_upload(pk, pk.d_segs, v.data(), v.size() * sizeof(CopySeg), st));
    HIPCHK(copy_segments(pk.d_segs, (int)v.size(), mx, st));
    return H2G_OK;
  };
  // rows [a, a + len) mod n of one sub-coset: one or two runs
  auto runs = [&](const RowPiece& pc, auto&& fn) {
    const uint64_t first = std::min<uint64_t>(pc.len, n - pc.a);
    fn(pc.a, 0, first);
    if (pc.len > first) fn(0, first, pc.len - first);
  };
  // coefficients, then the twists and the n-point NTTs of every sub-coset of every column
  if (!mine.empty()) {
    std::vector<const Fr*> l2;
    std::vector<Fr*> p2, io;
    for (int i : mine) {
      l2.push_back(lag[i]);
      p2.push_back(poly[i]);
    }
    RCCHK(lagrange_to_coeff_batch(d, pk.dom, l2.data(), p2.data(), (int)l2.size(), st));
    for (size_t q = 0; q < mine.size(); q++)
      for (int t = 0; t < E; t++) {
        Fr* o = pk.cs_scr + (q * E + t) * n;
        HIPCHK(subcoset_twist(poly[mine[q]], o, n, pk.eo, (uint64_t)t, pk.ext - 1, st));
        io.push_back(o);
      }
    const Fr one = Fr::one();
    for (size_t b0 = 0; b0 < io.size(); b0 += NTT_MAX_BATCH)
      RCCHK(ntt_dev_impl_batch(d, (const Fr* const*)io.data() + b0, n, io.data() + b0,
                               (int)std::min<size_t>(NTT_MAX_BATCH, io.size() - b0), n, (int)pk.dom.k, pk.dom.omega, 1,
                               pk.dom.g_coset, pk.dom.g_coset_inv, 0, one, 0, one, one, st));
  }
  std::vector<CopySeg>& pack = pk.h_segs[0];
  std::vector<CopySeg>& unpack = pk.h_segs[1];
  pack.clear();
  unpack.clear();
  for (int r = 0; r < W; r++) {
    size_t pos = soff[r];
    for (size_t q = 0; q < mine.size(); q++) {
      const int i = mine[q];
      for (const RowPiece& pc : pcs[r]) {
        const Fr* src = pk.cs_scr + (q * E + pc.t) * n;
        runs(pc, [&](uint64_t row, uint64_t at, uint64_t cnt) {
          if (r == me) pack.push_back(CopySeg{src + row, coset[i] + (size_t)pc.slot * n + row, cnt});
          else pack.push_back(CopySeg{src + row, xs + pos + at, cnt});
        });
        if (r != me) pos += pc.len;
      }
      if (r == me) continue;
      const size_t cnt = slabs[r].hi1 - slabs[r].lo;
      if (cnt) pack.push_back(CopySeg{poly[i] + slabs[r].lo, xs + pos, cnt});
      pos += cnt;
    }
  }
  size_t off = 0;  // unpack, source by source
  const size_t mycnt = slabs[me].hi1 - slabs[me].lo;
  for (int o = 0; o < W; o++) {
    if (o == me) continue;
    for (int i = 0; i < M; i++) {
      if (owner[i] != o) continue;
      for (const RowPiece& pc : pcs[me]) {
        runs(pc, [&](uint64_t row, uint64_t at, uint64_t cnt) {
          unpack.push_back(CopySeg{xr + off + at, coset[i] + (size_t)pc.slot * n + row, cnt});
        });
        off += pc.len;
      }
      if (mycnt) unpack.push_back(CopySeg{xr + off, poly[i] + slabs[me].lo, mycnt});
      off += mycnt;
    }
  }
  RCCHK(run_segs(pack));
  if (xp) {  // behind the pack on the stream; the receiver's rows land before h(X) (xp_flush)
    uint64_t bytes = 0;
    for (int r = 0; r < W; r++) bytes += sb[r] + rb[r];
    if (spmd_timed(2, bytes, [&] { return g_xpost(g_spmd.ctx, xs, sb.data(), xr, rb.data(), st, xp->done); }) != 0)
      return fail(H2G_ERR_STATE, "spmd transport: exchange of column sub-cosets failed (post)");
    xp->unpack.swap(unpack);
    xp->live = true;
    pk.xp_used++;
    return H2G_OK;
  }
  HIPCHK(hipStreamSynchronize(st));
  if (spmd_exchange(xs, sb.data(), xr, rb.data()) != 0)
    return fail(H2G_ERR_STATE, "spmd transport: exchange of column sub-cosets failed");
  RCCHK(run_segs(unpack));
  return H2G_OK;
}

// the overlapped exchanges' received rows into their columns: every posted exchange waited
// for (the transport's deadline applies), the stream made to wait for its completion
// event, its unpack list queued -- before anything reads the cosets or the slabs
int xp_flush(ProvingKey& pk, hipStream_t st) {
  for (size_t k = 0; k < pk.xp_used; k++) {
    ProvingKey::XPending& x = pk.xp[k];
    if (!x.live) continue;
    x.live = false;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = g_xwait ? g_xwait(g_spmd.ctx, x.done) : (int)hipEventSynchronize(x.done);
    g_spmd_stats.ms[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc != 0) {
      pk.xp_used = 0;
      return fail(H2G_ERR_STATE, "spmd transport: exchange of column sub-cosets failed (wait)");
    }
    HIPCHK(hipStreamWaitEvent(st, x.done, 0));
    if (!x.unpack.empty()) {
      if (x.unpack.size() > pk.d_segs_len) {
        PALLOC(pk.pool, pk.d_segs, x.unpack.size());
        pk.d_segs_len = x.unpack.size();
      }
      uint64_t mx = 0;
      for (const CopySeg& g : x.unpack) mx = std::max<uint64_t>(mx, g.len);
      HIPCHK(pk_upload(pk, pk.d_segs, x.unpack.data(), x.unpack.size() * sizeof(CopySeg), st));
      HIPCHK(copy_segments(pk.d_segs, (int)x.unpack.size(), mx, st));
    }
  }
  pk.xp_used = 0;
  return H2G_OK;
}

// a failed proof's exchanges still in flight: wait for them before their staging is reused
// or freed -- one bound for all of them together (10 s), and an exchange still pending past
// it is abandoned, not reused: its staging and event are dropped (the key's pool releases
// the memory with the key) so that the next proof posts into fresh buffers a late transfer
// cannot write
void xp_drain(ProvingKey& pk) {
  const auto t0 = std::chrono::steady_clock::now();
  for (ProvingKey::XPending& x : pk.xp) {
    if (!x.live) continue;
    x.live = false;
    while (hipEventQuery(x.done) == hipErrorNotReady &&
           std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (hipEventQuery(x.done) == hipErrorNotReady) {
      x.send = x.recv = nullptr;
      x.send_len = x.recv_len = 0;
      x.done = nullptr;  // a new event for the next post (the pending one is left to the runtime)
      x.unpack.clear();
    }
  }
  pk.xp_used = 0;
}

// pieces: the leader of sub-coset t (rank t) receives the h rows of the sub-coset's other
// pieces (ranks t + 2^e p), which arrive in rank order -- the rows' own order -- straight
// into its h_gather slot
int h_gather_pieces(ProvingKey& pk, hipStream_t st) {
  const int W = g_spmd.world, me = g_spmd.rank;
  const int E = 1 << (pk.dom.ek - pk.dom.k);
  const size_t n = pk.n;
  const uint64_t t = (uint64_t)me % (uint64_t)E;
  std::vector<size_t> sb(W, 0), rb(W, 0);
  const int G = W / E;
  if (me >= E) sb[t] = (pk.sub_hi - pk.sub_lo) * sizeof(Fr);
  else
    for (int p = 1; p < G; p++) rb[me + E * p] = (size_t)(n * (p + 1) / G - n * p / G) * sizeof(Fr);
  Fr* slot = pk.h_gather + t * n;
  HIPCHK(hipStreamSynchronize(st));
  if (spmd_exchange(slot + pk.sub_lo, sb.data(), slot + n / G, rb.data()) != 0)
    return fail(H2G_ERR_STATE, "spmd transport: exchange of h pieces failed");
  return H2G_OK;
}

// column i's rows go from every rank's MSM slab [shard_lo(P, n, W, r), shard_lo(.., r + 1))
// to its owner owner[i] (which then holds the whole column): one exchange; message from r
// to o: the slab rows of every column o owns, index order
int gather_to_owners(ProvingKey& pk, const std::vector<Fr*>& cols, const std::vector<int>& owner, size_t P,
                     hipStream_t st) {
  const size_t n = pk.n;
  const int W = g_spmd.world, me = g_spmd.rank;
  const int M = (int)cols.size();
  std::vector<size_t> lo(W + 1);
  for (int r = 0; r <= W; r++) lo[r] = shard_lo(P, n, W, r);
  std::vector<size_t> sb(W, 0), rb(W, 0), soff(W + 1, 0);
  for (int r = 0; r < W; r++) {
    if (r != me) {
      size_t mine = 0, theirs = 0;
      for (int i = 0; i < M; i++) {
        mine += owner[i] == r;     // r's columns: I send my slab of each
        theirs += owner[i] == me;  // my columns: r sends its slab of each
      }
      sb[r] = mine * (lo[me + 1] - lo[me]) * sizeof(Fr);
      rb[r] = theirs * (lo[r + 1] - lo[r]) * sizeof(Fr);
    }
    soff[r + 1] = soff[r] + sb[r] / sizeof(Fr);
  }
  size_t rtot = 0;
  for (int r = 0; r < W; r++) rtot += rb[r] / sizeof(Fr);
  if (soff[W] > pk.x_send_len) {
    PALLOC(pk.pool, pk.x_send, soff[W]);
    pk.x_send_len = soff[W];
  }
  if (rtot > pk.x_recv_len) {
    PALLOC(pk.pool, pk.x_recv, rtot);
    pk.x_recv_len = rtot;
  }
  std::vector<CopySeg>& pack = pk.h_segs[0];
  std::vector<CopySeg>& unpack = pk.h_segs[1];
  pack.clear();
  unpack.clear();
  const size_t my = lo[me + 1] - lo[me];
  for (int r = 0; r < W; r++) {
    if (r == me || !my) continue;
    size_t pos = soff[r];
    for (int i = 0; i < M; i++)
      if (owner[i] == r) {
        pack.push_back(CopySeg{cols[i] + lo[me], pk.x_send + pos, my});
        pos += my;
      }
  }
  size_t off = 0;
  for (int r = 0; r < W; r++) {
    if (r == me) continue;
    const size_t cnt = lo[r + 1] - lo[r];
    for (int i = 0; i < M; i++)
      if (owner[i] == me && cnt) {
        unpack.push_back(CopySeg{pk.x_recv + off, cols[i] + lo[r], cnt});
        off += cnt;
      }
  }
  auto run = [&](std::vector<CopySeg>& v) -> int {
    if (v.empty()) return H2G_OK;
    if (v.size() > pk.d_segs_len) {
      PALLOC(pk.pool, pk.d_segs, v.size());
      pk.d_segs_len = v.size();
    }
    uint64_t mx = 0;
    for (const CopySeg& g : v) mx = std::max<uint64_t>(mx, g.len);
    HIPCHK(pk_upload(pk, pk.d_segs, v.data(), v.size() * sizeof(CopySeg), st));
    HIPCHK(copy_segments(pk.d_segs, (int)v.size(), mx, st));
    return H2G_OK;
  };
  RCCHK(run(pack));
  HIPCHK(hipStreamSynchronize(st));
  if (spmd_exchange(pk.x_send, sb.data(), pk.x_recv, rb.data()) != 0)
    return fail(H2G_ERR_STATE, "spmd transport: exchange of product slabs failed");
  RCCHK(run(unpack));
  return H2G_OK;
}

int keygen_impl(Device* d, Params& prm, const h2g_circuit* c, ProvingKey& pk, const PkImage* img = nullptr) {
  hipStream_t st = d->stream;
  std::string why;
  if (c->k != prm.k) return fail(H2G_ERR_ARG, "keygen: circuit k != params k");
  if (c->num_gates && (!c->gate_roots || !c->nodes)) return fail(H2G_ERR_ARG, "keygen: null gates");
  if (!check_nodes(c, &why)) return fail(H2G_ERR_ARG, "keygen: bad expression graph: " + why);
  if (!img && c->num_fixed && !c->fixed_values) return fail(H2G_ERR_ARG, "keygen: null fixed values");
  if (!c->transcript_repr) return fail(H2G_ERR_ARG, "keygen: null transcript_repr");
  const CircuitView cv{c};
  pk.device = d->id;
  pk.k = c->k;
  pk.n = (size_t)1 << c->k;
  pk.A = (int)c->num_advice;
  pk.F = (int)c->num_fixed;
  pk.I = (int)c->num_instance;
  pk.P = (int)c->num_perm_columns;
  pk.transcript_repr = fr_from_limbs(c->transcript_repr);
  pk.unblinded.assign(pk.A, 0);
  if (c->unblinded)
    for (int i = 0; i < pk.A; i++) pk.unblinded[i] = c->unblinded[i];
  pk.adv_phase.assign(pk.A, 0);
  if (c->advice_phase)
    for (int i = 0; i < pk.A; i++) pk.adv_phase[i] = c->advice_phase[i];
  pk.ch_phase.assign(c->num_challenges, 0);
  if (c->num_challenges && !c->challenge_phase) return fail(H2G_ERR_ARG, "keygen: null challenge_phase");
  for (uint32_t i = 0; i < c->num_challenges; i++) pk.ch_phase[i] = c->challenge_phase[i];
  pk.max_phase = 0;
  for (int i = 0; i < pk.A; i++) pk.max_phase = std::max(pk.max_phase, (int)pk.adv_phase[i]);
  for (uint8_t ph : pk.ch_phase)
    if ((int)ph > pk.max_phase) return fail(H2G_ERR_ARG, "keygen: challenge phase after the last advice phase");
  pk.num_consts = (int)c->num_constants;
  for (int i = 0; i < pk.P; i++) {
    const int t = c->perm_columns[2 * i], ix = c->perm_columns[2 * i + 1];
    const int lim = t == COL_ADVICE ? pk.A : t == COL_FIXED ? pk.F : t == COL_INSTANCE ? pk.I : 0;
    if (ix < 0 || ix >= lim) return fail(H2G_ERR_ARG, "keygen: permutation column out of range");
    pk.perm_cols.emplace_back(t, ix);
  }
  // degree, queries, blinding factors (circuit.rs:143-170,292-320; keygen.rs:191-260)
  std::vector<int> memo(c->num_nodes, -1);
  const std::vector<ArgRoots> lks = arg_roots(c->num_lookups, c->lookup_sizes, c->lookup_roots);
  const std::vector<ArgRoots> shs = arg_roots(c->num_shuffles, c->shuffle_sizes, c->shuffle_roots);
  pk.NL = (int)lks.size();
  pk.NS = (int)shs.size();
  pk.degree = 3;
  for (uint32_t g = 0; g < c->num_gates; g++) pk.degree = std::max(pk.degree, node_degree(cv, c->gate_roots[g], memo));
  for (const auto& a : lks) {  // lookup_argument_required_degree (circuit.rs:327-373)
    int di = 1, dt = 1;
    for (int i = 0; i < a.m; i++) {
      di = std::max(di, node_degree(cv, a.in[i], memo));
      dt = std::max(dt, node_degree(cv, a.other[i], memo));
    }
    pk.degree = std::max(pk.degree, std::max(4, 2 + di + dt));
  }
  for (const auto& a : shs) {  // shuffle_argument_required_degree (circuit.rs:375-389)
    int di = 1, ds = 1;
    for (int i = 0; i < a.m; i++) {
      di = std::max(di, node_degree(cv, a.in[i], memo));
      ds = std::max(ds, node_degree(cv, a.other[i], memo));
    }
    pk.degree = std::max(pk.degree, 2 + std::max(di, ds));
  }
  // queries: gates, lookups (inputs then tables), shuffles, permutation (keygen.rs:320-345)
  for (uint32_t g = 0; g < c->num_gates; g++) collect(cv, c->gate_roots[g], pk);
  for (const auto& a : lks) {
    for (int i = 0; i < a.m; i++) collect(cv, a.in[i], pk);
    for (int i = 0; i < a.m; i++) collect(cv, a.other[i], pk);
  }
  for (const auto& a : shs) {
    for (int i = 0; i < a.m; i++) collect(cv, a.in[i], pk);
    for (int i = 0; i < a.m; i++) collect(cv, a.other[i], pk);
  }
  for (auto& pc : pk.perm_cols)
    add_query(pc.first == COL_ADVICE ? pk.adv_q : (pc.first == COL_FIXED ? pk.fix_q : pk.ins_q),
              Query{pc.first, pc.second, 0});
  int maxq = 1;
  if (pk.A) {
    std::vector<int> cnt(pk.A, 0);
    for (auto& q : pk.adv_q) cnt[q.index]++;
    maxq = *std::max_element(cnt.begin(), cnt.end());
  }
  pk.bf = std::max(3, maxq) + 2;
  if ((int64_t)pk.n < pk.bf + 3) return fail(H2G_ERR_ARG, "keygen: not enough rows available");
  pk.chunk_len = pk.degree - 2;
  pk.nsets = (pk.P + pk.chunk_len - 1) / pk.chunk_len;
  RCCHK(domain_init(&pk.dom, (uint32_t)pk.degree, pk.k));
  pk.ext = (size_t)1 << pk.dom.ek;
  pk.rot_scale = 1ull << (pk.dom.ek - pk.k);
  const size_t n = pk.n, ext = pk.ext;
  Pool& pool = pk.pool;
  RCCHK(build_pow_table(pool, pk.dom.omega, (int)pk.k, &pk.om, st));
  RCCHK(build_pow_table(pool, pk.dom.ext_omega, (int)pk.dom.ek, &pk.eo, st));

  // workspace first (keygen uses some of it as scratch)
  auto falloc = [&](Fr** p, size_t cnt) { return pool.get((void**)p, cnt * sizeof(Fr)); };
  pk.scr_len = std::max(n + 64, kate_scratch_len(n) + poly_prefix_scratch_len(n) + 64);
  HIPCHK(falloc(&pk.mod, n));
  HIPCHK(falloc(&pk.pre, n));
  HIPCHK(falloc(&pk.scr, pk.scr_len));
  HIPCHK(falloc(&pk.random_poly, n));
  HIPCHK(falloc(&pk.h_ext, ext));
  HIPCHK(falloc(&pk.h_coeff, ext));
  HIPCHK(falloc(&pk.h_poly, n));
  HIPCHK(falloc(&pk.nx, n));
  HIPCHK(falloc(&pk.q1, n));
  HIPCHK(falloc(&pk.hx, n));
  HIPCHK(falloc(&pk.lx, n));
  HIPCHK(falloc(&pk.small, 4096));
  HIPCHK(falloc(&pk.last_z, 1));
  auto vec_alloc = [&](std::vector<Fr*>& v, int cnt, size_t len) -> hipError_t {
    v.assign(cnt, nullptr);
    for (int i = 0; i < cnt; i++) {
      hipError_t e = falloc(&v[i], len);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  HIPCHK(falloc(&pk.one, 1));
  {
    const Fr one = Fr::one();
    HIPCHK(hipMemcpy(pk.one, &one, sizeof(Fr), hipMemcpyHostToDevice));
  }
  if (pk.NL + pk.NS) {
    HIPCHK(falloc(&pk.tmp_a, n));
    HIPCHK(falloc(&pk.tmp_b, n));
  }
  if (pk.NL) {  // permute_expression_pair scratch (the batched sort's buffers grow per proof)
    PALLOC(pool, pk.ck_a2, n);
    PALLOC(pool, pk.ck_t2, n);
    PALLOC(pool, pk.ck_left, n);
    PALLOC(pool, pk.rep_flag, n);
    PALLOC(pool, pk.left_flag, n);
    PALLOC(pool, pk.rep_rows, n);
    PALLOC(pool, pk.counters, 8);
    pk.lk_hb.assign(pk.NL, 64);
  }

  // fixed columns
  HIPCHK(vec_alloc(pk.fixed_lag, pk.F, n));
  HIPCHK(vec_alloc(pk.fixed_poly, pk.F, n));
  HIPCHK(vec_alloc(pk.fixed_coset, pk.F, ext));
  for (int i = 0; i < pk.F; i++) {
    if (img) {
      HIPCHK(img->upload(pk.fixed_lag[i], img->fixed_lag[i], n, st));
      HIPCHK(img->upload(pk.fixed_poly[i], img->fixed_poly[i], n, st));
      HIPCHK(img->upload(pk.fixed_coset[i], img->fixed_coset[i], ext, st));
      continue;
    }
    HIPCHK(hipMemcpyAsync(pk.fixed_lag[i], c->fixed_values + 4 * n * i, n * sizeof(Fr), hipMemcpyHostToDevice, st));
    RCCHK(lagrange_to_coeff(d, pk.dom, pk.fixed_lag[i], pk.fixed_poly[i], st));
    RCCHK(coeff_to_extended(d, pk.dom, pk.fixed_poly[i], pk.fixed_coset[i], st));
  }
  // l_0, l_last, l_active (keygen.rs:147-175)
  HIPCHK(falloc(&pk.l0, ext));
  HIPCHK(falloc(&pk.l_last, ext));
  HIPCHK(falloc(&pk.l_active, ext));
  if (img) {
    HIPCHK(img->upload(pk.l0, img->l0, ext, st));
    HIPCHK(img->upload(pk.l_last, img->l_last, ext, st));
    HIPCHK(img->upload(pk.l_active, img->l_active, ext, st));
  } else {
    const Fr one = Fr::one();
    std::vector<Fr> ones(pk.bf, one);
    auto lagrange_unit = [&](size_t row0, int count, Fr* out) -> int {
      HIPCHK(hipMemsetAsync(pk.pre, 0, n * sizeof(Fr), st));
      HIPCHK(hipMemcpyAsync(pk.pre + row0, ones.data(), count * sizeof(Fr), hipMemcpyHostToDevice, st));
      RCCHK(lagrange_to_coeff(d, pk.dom, pk.pre, pk.mod, st));
      RCCHK(coeff_to_extended(d, pk.dom, pk.mod, out, st));
      HIPCHK(hipStreamSynchronize(st));
      return H2G_OK;
    };
    RCCHK(lagrange_unit(0, 1, pk.l0));
    RCCHK(lagrange_unit(n - pk.bf, pk.bf, pk.h_ext));  // l_blind
    RCCHK(lagrange_unit(n - pk.bf - 1, 1, pk.l_last));
    HIPCHK(poly_binop(POLY_ADD, pk.l_last, pk.h_ext, one, pk.l_active, ext, st));
    HIPCHK(poly_binop(POLY_SUB_CONST, pk.l_active, nullptr, one, pk.l_active, ext, st));
    HIPCHK(poly_binop(POLY_SCALE, pk.l_active, nullptr, fr_neg_one(), pk.l_active, ext, st));
  }
  // permutation: Assembly on the host, sigma polynomials on the device
  HIPCHK(vec_alloc(pk.sigma_lag, pk.P, n));
  HIPCHK(vec_alloc(pk.sigma_poly, pk.P, n));
  HIPCHK(vec_alloc(pk.sigma_coset, pk.P, ext));
  if (pk.P && img) {
    for (int i = 0; i < pk.P; i++) {
      HIPCHK(img->upload(pk.sigma_lag[i], img->sigma_lag[i], n, st));
      HIPCHK(img->upload(pk.sigma_poly[i], img->sigma_poly[i], n, st));
      HIPCHK(img->upload(pk.sigma_coset[i], img->sigma_coset[i], ext, st));
    }
    HIPCHK(hipStreamSynchronize(st));
  } else if (pk.P) {
    const size_t cells = (size_t)pk.P * n;
    std::vector<uint32_t> mcol(cells), mrow(cells), acol(cells), arow(cells);
    std::vector<uint64_t> sizes(cells, 1);
    for (int cI = 0; cI < pk.P; cI++)
      for (size_t r = 0; r < n; r++) {
        mcol[cI * n + r] = acol[cI * n + r] = (uint32_t)cI;
        mrow[cI * n + r] = arow[cI * n + r] = (uint32_t)r;
      }
    auto pos = [&](int t, int ix) -> int {
      for (int i = 0; i < pk.P; i++)
        if (pk.perm_cols[i].first == t && pk.perm_cols[i].second == ix) return i;
      return -1;
    };
    for (uint32_t ci = 0; ci < c->num_copies; ci++) {  // Assembly::copy (permutation/keygen.rs:59-97)
      const int32_t* cp = c->copies + 6 * ci;
      const int lc = pos(cp[0], cp[1]), rc = pos(cp[3], cp[4]);
      if (lc < 0 || rc < 0) return fail(H2G_ERR_ARG, "keygen: copy on a column not in the permutation");
      if (cp[2] < 0 || cp[5] < 0 || (size_t)cp[2] >= n || (size_t)cp[5] >= n)
        return fail(H2G_ERR_ARG, "keygen: copy row out of bounds");
      const size_t li = lc * n + cp[2], ri = rc * n + cp[5];
      size_t lcyc = acol[li] * n + arow[li], rcyc = acol[ri] * n + arow[ri];
      if (lcyc == rcyc) continue;
      if (sizes[lcyc] < sizes[rcyc]) std::swap(lcyc, rcyc);
      sizes[lcyc] += sizes[rcyc];
      size_t i = rcyc;
      for (;;) {
        acol[i] = (uint32_t)(lcyc / n);
        arow[i] = (uint32_t)(lcyc % n);
        i = (size_t)mcol[i] * n + mrow[i];
        if (i == rcyc) break;
      }
      std::swap(mcol[li], mcol[ri]);
      std::swap(mrow[li], mrow[ri]);
    }
    std::vector<Fr> dpow(pk.P + 1);
    dpow[0] = Fr::one();
    for (int i = 1; i <= pk.P; i++) dpow[i] = dpow[i - 1] * fr_delta();
    uint32_t *dmc, *dmr;
    Fr* ddp;
    HIPCHK(hipMalloc(&dmc, cells * 4));
    HIPCHK(hipMalloc(&dmr, cells * 4));
    HIPCHK(hipMalloc(&ddp, dpow.size() * sizeof(Fr)));
    HIPCHK(hipMemcpyAsync(dmc, mcol.data(), cells * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dmr, mrow.data(), cells * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(ddp, dpow.data(), dpow.size() * sizeof(Fr), hipMemcpyHostToDevice, st));
    for (int i = 0; i < pk.P; i++) {
      HIPCHK(sigma_from_mapping(pk.sigma_lag[i], dmc + i * n, dmr + i * n, n, ddp, pk.om, st));
      RCCHK(lagrange_to_coeff(d, pk.dom, pk.sigma_lag[i], pk.sigma_poly[i], st));
      RCCHK(coeff_to_extended(d, pk.dom, pk.sigma_poly[i], pk.sigma_coset[i], st));
    }
    HIPCHK(hipStreamSynchronize(st));
    (void)hipFree(dmc);
    (void)hipFree(dmr);
    (void)hipFree(ddp);
  }
  // expression programs: gates (Horner in y), then each lookup's / shuffle's expression
  // lists (Horner in theta), sharing one slot allocation and one load table
  {
    GateCompiler gc(cv);
    pk.seg_gates = gc.compile_list(c->gate_roots, (int)c->num_gates);
    for (const auto& a : lks) {
      pk.seg_lk_in.push_back(gc.compile_list(a.in, a.m));
      pk.seg_lk_tab.push_back(gc.compile_list(a.other, a.m));
    }
    pk.lk_trep.assign(lks.size(), 0);
    for (size_t l = 0; l < lks.size(); l++) {
      pk.lk_trep[l] = (int)l;
      for (size_t r = 0; r < l; r++) {
        bool same = lks[r].m == lks[l].m;
        for (int i = 0; same && i < lks[l].m; i++) same = same_expr(cv, lks[r].other[i], lks[l].other[i]);
        if (same) {
          pk.lk_trep[l] = (int)r;
          break;
        }
      }
    }
    for (const auto& a : shs) {
      pk.seg_sh_in.push_back(gc.compile_list(a.in, a.m));
      pk.seg_sh_sh.push_back(gc.compile_list(a.other, a.m));
    }
    if (gc.n_slots > evaluate_h_max_slots())
      return fail(H2G_ERR_ARG, "keygen: expressions need more than " + std::to_string(evaluate_h_max_slots()) +
                                   " live values");
    pk.prog_len = (int)gc.prog.size();
    pk.n_slots = gc.n_slots;
    PALLOC(pool, pk.prog, gc.prog.size() + 1);
    HIPCHK(hipMemcpy(pk.prog, gc.prog.data(), gc.prog.size() * sizeof(int4), hipMemcpyHostToDevice));
    PALLOC(pool, pk.consts, c->num_constants + c->num_challenges + 1);
    if (c->num_constants)
      HIPCHK(hipMemcpy(pk.consts, c->constants, c->num_constants * sizeof(Fr), hipMemcpyHostToDevice));
    pk.n_loads = (int)gc.loads.size();
    pk.loads = gc.loads;
    std::vector<int> lr(pk.n_loads + 1, 0);
    for (int i = 0; i < pk.n_loads; i++) lr[i] = gc.loads[i].rot;
    PALLOC(pool, pk.d_load_rot, lr.size());
    HIPCHK(hipMemcpy(pk.d_load_rot, lr.data(), lr.size() * sizeof(int), hipMemcpyHostToDevice));
    std::vector<const Fr*> sg(pk.P + 1);
    for (int i = 0; i < pk.P; i++) sg[i] = pk.sigma_coset[i];
    PALLOC(pool, pk.d_sigma, sg.size());
    HIPCHK(hipMemcpy(pk.d_sigma, sg.data(), sg.size() * sizeof(Fr*), hipMemcpyHostToDevice));
  }
  RCCHK(circuit_ws_add(pk));  // circuit 0's workspace
  HIPCHK(hipStreamSynchronize(st));
  return H2G_OK;
}

// ------------------------------------------------------------------ create_proof
// Synchronises a stream when it goes out of scope: declared after host staging buffers
// that asynchronous copies read, so that an early return cannot free them under a copy.
struct StreamSyncGuard {
  hipStream_t s;
  ~StreamSyncGuard() { (void)hipStreamSynchronize(s); }
};

// A proof that fails part-way leaves launched MSMs uncollected: their result ring entries
// would stay reserved.  Proofs run one at a time under the library lock and collect every
// MSM they launch, so on the way out the MSM streams are drained and the ring freed.
struct MsmRingGuard {
  Device* d;
  ~MsmRingGuard() {
    bool any = false;
    for (bool b : d->ring_busy) any = any || b;
    if (!any) return;
    for (hipStream_t s : d->mstream)
      if (s) (void)hipStreamSynchronize(s);
    for (bool& b : d->ring_busy) b = false;
  }
};

struct StageClock {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  hipStream_t st;
  bool sync_each;
  explicit StageClock(hipStream_t s, bool sync) : st(s), sync_each(sync) { g_stages.clear(); }
  void mark(const char* name) {
    if (sync_each) (void)hipStreamSynchronize(st);
    const auto t = std::chrono::steady_clock::now();
    g_stages.emplace_back(name, std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  }
};

struct PolyRef {  // a committed polynomial in coefficient form (SHPLONK's "commitment identity")
  const Fr* p;
  uint64_t len;
};

// SPMD: an advice phase's m column checksums (pk.wsum_d, filled by the copy_columns that
// brought the columns in) to the host behind the stream; folded into the consistency
// digest by the next collective (spmd_witness_settle) -- only when sharded
int spmd_witness_prepare(ProvingKey& pk, int m, hipStream_t st) {
  if (g_spmd.world <= 1 || m <= 0) return H2G_OK;
  spmd_witness_settle();  // an earlier phase's, before its pinned buffer is reused
  if ((size_t)m > pk.wsum_len) {
    if (pk.wsum_d) (void)hipFree(pk.wsum_d);
    if (pk.wsum_h) (void)hipHostFree(pk.wsum_h);
    pk.wsum_d = pk.wsum_h = nullptr;
    pk.wsum_len = 0;
    HIPCHK(hipMalloc((void**)&pk.wsum_d, (size_t)m * sizeof(unsigned long long)));
    HIPCHK(hipHostMalloc((void**)&pk.wsum_h, (size_t)m * sizeof(unsigned long long), hipHostMallocDefault));
    pk.wsum_len = (size_t)m;
  }
  if (!pk.wsum_ev) HIPCHK(hipEventCreateWithFlags(&pk.wsum_ev, hipEventDisableTiming));
  HIPCHK(hipMemsetAsync(pk.wsum_d, 0, (size_t)m * sizeof(unsigned long long), st));
  return H2G_OK;
}
int spmd_witness_fold(ProvingKey& pk, int m, hipStream_t st) {
  if (g_spmd.world <= 1 || m <= 0) return H2G_OK;
  HIPCHK(hipMemcpyAsync(pk.wsum_h, pk.wsum_d, (size_t)m * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIPCHK(hipEventRecord(pk.wsum_ev, st));
  g_spmd_check.pend = pk.wsum_h;
  g_spmd_check.pend_n = m;
  g_spmd_check.pend_ev = pk.wsum_ev;
  return H2G_OK;
}

// the proof's upload staging (ProvingKey::up_h): armed behind a sync of the prover's
// stream, so no copy of the previous proof still reads it
int pk_upload_arm(ProvingKey& pk, hipStream_t st) {
  HIPCHK(hipStreamSynchronize(st));
  if (!pk.up_h) {
    constexpr size_t kLen = 4u << 20;
    HIPCHK(hipHostMalloc((void**)&pk.up_h, kLen, hipHostMallocDefault));
    pk.up_len = kLen;
  }
  pk.up_off = 0;
  return H2G_OK;
}
// dst <- src (host, any) on st through the staging; past its end, the pageable copy
hipError_t pk_upload(ProvingKey& pk, void* dst, const void* src, size_t bytes, hipStream_t st) {
  const size_t a = (pk.up_off + 63) & ~(size_t)63;
  if (pk.up_h && a + bytes <= pk.up_len) {
    std::memcpy(pk.up_h + a, src, bytes);
    pk.up_off = a + bytes;
    return hipMemcpyAsync(dst, pk.up_h + a, bytes, hipMemcpyHostToDevice, st);
  }
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
}

// device staging for a batch of blinding rows (grow-only)
int blind_stage(ProvingKey& pk, size_t count) {
  if (count > pk.blind_d_len) {
    PALLOC(pk.pool, pk.blind_d, count);
    pk.blind_d_len = count;
  }
  return H2G_OK;
}
// several blocks of blinding rows in one upload and one copy launch: `host` (count Fr) lands
// in pk.blind_d, which `segs` read from.  Every small host-to-device copy is a ~6-us blit
// on the stream; a keccak-style proof made ~80 of them, one per column and lookup side
int upload_rows_batch(ProvingKey& pk, const Fr* host, size_t count, const std::vector<CopySeg>& segs,
                      hipStream_t st) {
  if (segs.empty()) return H2G_OK;
  HIPCHK(pk_upload(pk, pk.blind_d, host, count * sizeof(Fr), st));
  if (segs.size() > pk.d_segs_len) {
    PALLOC(pk.pool, pk.d_segs, segs.size());
    pk.d_segs_len = segs.size();
  }
  uint64_t mx = 0;
  for (const CopySeg& g : segs) mx = std::max<uint64_t>(mx, g.len);
  HIPCHK(pk_upload(pk, pk.d_segs, segs.data(), segs.size() * sizeof(CopySeg), st));
  HIPCHK(copy_segments(pk.d_segs, (int)segs.size(), mx, st));
  return H2G_OK;
}

std::vector<Fr> g_last_challenges;  // the challenges of the last proof (h2g_last_challenges)

// create_proof's inputs (halo2_proofs/src/plonk/prover.rs:19-36): per circuit the witness
// and the instances, the RNG, and the vanishing argument's thread count
struct ProveIn {
  int nc = 1;                                     // circuits
  const uint64_t* const* advice = nullptr;        // [nc] num_advice x n Fr (host, or device)
  bool adv_dev = false;
  const h2g_witness_source* src1 = nullptr;       // one circuit's per-phase witness source
  const h2g_witness_source_multi* src = nullptr;  // per-circuit per-phase witness source
  const uint64_t* const* instance = nullptr;      // [nc] num_instance x n Fr (zero padded)
  const uint32_t* const* inst_lens = nullptr;     // [nc] num_instance lengths
  ProverRng* rng = nullptr;
  uint32_t vthreads = 1;
};

int prove_impl(Device* d, Params& prm, ProvingKey& pk, const ProveIn& in, std::vector<uint8_t>* proof) {
  hipStream_t st = d->stream;
  xp_drain(pk);  // a failed proof's overlapped exchanges
  RCCHK(pk_upload_arm(pk, st));
  const size_t n = pk.n, ext = pk.ext;
  const int bf = pk.bf;
  const Domain& D = pk.dom;
  const int ncirc = in.nc;
  while ((int)pk.cws.size() < ncirc) RCCHK(circuit_ws_add(pk));  // workspaces grow once
  std::vector<CircuitWs*> W(ncirc);
  for (int c = 0; c < ncirc; c++) W[c] = pk.cws[c].get();
  // with the slab exchange and world a multiple of 2^e above it, every rank takes a row
  // piece of one sub-coset (sub_prepare)
  const int E_sub = 1 << (pk.dom.ek - pk.dom.k);
  const bool pieces = spmd_subcosets() && g_spmd.allgather_host && g_spmd.exchange && pk.multiopen == 0 &&
                      g_spmd_colshard && g_spmd.world >= kColshardMinWorld && g_spmd.world > E_sub &&
                      g_spmd.world % E_sub == 0;
  if (spmd_subcosets()) RCCHK(sub_prepare(pk, st, pieces));  // this rank's sub-cosets of the key's cosets
  MsmRingGuard ring_guard{d};
  StageClock clk(st, g_stage_sync);
  // SPMD coefficient slabs for the multi-open tail (SHPLONK only; GWC stays replicated)
  const bool slabs = g_spmd.world > 1 && g_spmd.allgather_host != nullptr && pk.multiopen == 0;
  Slab sl;
  sl.hi = sl.hi1 = n;
  if (slabs) sl = spmd_slab(n, g_spmd.rank);
  // SPMD with more ranks than sub-cosets: a rank that owns none needs the circuit's
  // coefficient columns only on its slab (evaluations, SHPLONK) -- the owners, which need
  // them whole for their cosets, send it (coef_exchange) and it skips their iNTTs
  const bool h_slabs = spmd_subcosets() && slabs && g_spmd.exchange != nullptr;
  const bool coef_recv = h_slabs && pk.sub_ts.empty();
  const bool coef_send = h_slabs && !pieces && !pk.sub_ts.empty() && g_spmd.world > (1 << (pk.dom.ek - pk.dom.k));
  // column ownership of wide stages (colshard_distribute): under the full split, a stage of
  // M columns goes to the ranks whole when M is a multiple of the ranks or at least 4x them
  // (balanced); fewer columns keep point slabs
  const int Wsp = g_spmd.world;
  auto wide = [&](int M) {
    return h_slabs && g_spmd_colshard && Wsp >= kColshardMinWorld && M >= Wsp && (M % Wsp == 0 || M >= 4 * Wsp);
  };
  // a stage's coefficient forms and extended-domain columns: with row pieces every stage's
  // transforms have one owner per column (round-robin across the stages, tr_next), a wide
  // stage's are its columns' owners (own); otherwise every sub-coset owner transforms
  // every column (the others receive coefficient slabs at the end, coef_exchange)
  // (with row pieces the rotation starts after the sub-cosets' leaders, ranks 0 .. E - 1,
  // which interpolate their sub-coset's h: C3 at 8 ranks puts its 6 column transforms on
  // ranks 2 .. 7 instead of stacking two roles on ranks 0 and 1)
  int tr_next = pieces ? E_sub : 0;
  // the transform stream (H2G_XFORM_STREAM): xs_begin orders it after the prover stream's
  // work so far (the inputs), xs_end marks its last transform, and the prover stream waits
  // for that mark before evaluate_h -- and at the end of the proof whatever its outcome
  // (XformJoin), so that the next proof's uploads never overtake a transform still reading
  const bool xsplit =
      H2G_XFORM_STREAM && g_spmd.world <= 1 && !spmd_subcosets() && (H2G_XS_ALL || pk.NL + pk.NS > 0);
  if (xsplit && !d->xstream) {  // after the MSM streams (h2g_init): the hardware-queue order, abi.cpp
    HIPCHK(hipStreamCreateWithFlags(&d->xstream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&d->xev_in, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->xev_done, hipEventDisableTiming));
  }
  const hipStream_t xst = xsplit ? d->xstream : st;
  struct XformJoin {
    Device* d;
    hipStream_t st;
    bool pending = false;
    hipError_t join() {
      if (!pending) return hipSuccess;
      pending = false;
      return hipStreamWaitEvent(st, d->xev_done, 0);
    }
    ~XformJoin() { (void)join(); }
  } xjoin{d, st};
  auto xs_begin = [&]() -> int {
    if (xst == st) return H2G_OK;
    HIPCHK(hipEventRecord(d->xev_in, st));
    HIPCHK(hipStreamWaitEvent(xst, d->xev_in, 0));
    return H2G_OK;
  };
  auto xs_end = [&]() -> int {
    if (xst == st) return H2G_OK;
    HIPCHK(hipEventRecord(d->xev_done, xst));
    xjoin.pending = true;
    return H2G_OK;
  };
  auto xform = [&](const std::vector<const Fr*>& lag, const std::vector<Fr*>& pol, const std::vector<Fr*>& cst,
                   const std::vector<int>* own) -> int {
    const int M = (int)lag.size();
    if (M == 0) return H2G_OK;
    if (own || pieces) {
      std::vector<int> o(M);
      for (int i = 0; i < M; i++) o[i] = own ? (*own)[i] : (tr_next + i) % Wsp;
      if (!own) tr_next += M;
      return colshard_distribute(d, pk, lag, pol, cst, o, st);
    }
    RCCHK(xs_begin());
    if (!coef_recv) RCCHK(lagrange_to_coeff_batch(d, D, lag.data(), pol.data(), M, xst));
    RCCHK(ext_cosets(d, pk, (const Fr* const*)pol.data(), cst.data(), M, xst));
    return xs_end();
  };
  // with row pieces the advice columns' transforms wait for the permutation stage: at the
  // advice commitments' all-gather every rank would otherwise wait for the ranks that
  // transform an advice column (their slab partials come late), and in the permutation
  // stage the ranks without a grand product's transform are idle -- run there, the advice
  // transforms overlap the products' (the owners are fixed here, in the same rotation)
  struct DeferredXform {
    std::vector<const Fr*> lag;
    std::vector<Fr*> pol, cst;
    std::vector<int> own;
  };
  std::vector<DeferredXform> deferred;
  // (the column transforms of the whole proof, an upper bound, against the ranks that are
  // not sub-coset leaders: C3 at 8 ranks has 3 advice + 3 grand products for 6 ranks; at 4
  // ranks two transforms would share a rank in the permutation stage, measured slower:
  // profiles/r05/emulation/defer_adv/)
  const int n_xf = ncirc * (pk.A + pk.nsets + 3 * pk.NL + pk.NS);
  const bool defer_adv = H2G_DEFER_ADV_XFORM && pieces && n_xf <= Wsp - E_sub;
  auto xform_later = [&](const std::vector<const Fr*>& lag, const std::vector<Fr*>& pol,
                         const std::vector<Fr*>& cst) {
    DeferredXform x{lag, pol, cst, std::vector<int>(lag.size())};
    for (size_t i = 0; i < lag.size(); i++) x.own[i] = (int)((tr_next + (int)i) % Wsp);
    tr_next += (int)lag.size();
    deferred.push_back(std::move(x));
  };
  auto run_deferred = [&]() -> int {
    for (DeferredXform& x : deferred) RCCHK(colshard_distribute(d, pk, x.lag, x.pol, x.cst, x.own, st));
    deferred.clear();
    return H2G_OK;
  };
  ProverRng& rng = *in.rng;
  Transcript tr(proof, pk.transcript);
  SpmdCheckScope spmd_check(&tr, &rng);
  auto write_point = [&](const G1Affine& p) -> int {
    if (!tr.write_point(p)) return fail(H2G_ERR_ARG, "cannot write points at infinity to the transcript");
    return H2G_OK;
  };
  // a stage's commitments: collected together (one SPMD all-gather), written in order
  auto collect_write = [&](const std::vector<MsmTicket*>& tks) -> int {
    std::vector<G1Affine> cms(tks.size());
    RCCHK(commit_collect_all(d, tks.data(), (int)tks.size(), cms.data()));
    for (const G1Affine& cm : cms) RCCHK(write_point(cm));
    return H2G_OK;
  };
  auto rng_ok = [&]() -> int { return rng.failed() ? fail(H2G_ERR_ARG, "create_proof: the caller's RNG failed") : H2G_OK; };

  // ---- vk.hash_into + every circuit's instances (prover.rs:187-271; KZG: QUERY_INSTANCE = false)
  tr.common_scalar(pk.transcript_repr);
  for (int ci = 0; ci < ncirc; ci++)
    for (int i = 0; i < pk.I; i++) {
      const uint32_t len = in.inst_lens[ci][i];
      if ((size_t)len > n - (size_t)(bf + 1)) return fail(H2G_ERR_ARG, "create_proof: InstanceTooLarge");
      const uint64_t* col = in.instance[ci] + 4 * n * i;
      for (uint32_t r = 0; r < len; r++) tr.common_scalar(fr_from_limbs(col + 4 * r));
      HIPCHK(hipMemcpyAsync(W[ci]->inst_val[i], col, n * sizeof(Fr), hipMemcpyHostToDevice, st));
      if (!coef_recv) RCCHK(lagrange_to_coeff(d, D, W[ci]->inst_val[i], W[ci]->inst_poly[i], st));
    }
  // ---- commit_phase per advice phase (prover.rs:309-494), circuit by circuit: the
  // phase's blinding rows, its blinds, its commitments; then the phase's challenges
  const size_t unusable = n - (size_t)(bf + 1);
  // host staging that device copies read asynchronously: lives until the proof returns
  // (every copy has completed by then: the final commitment is collected after it)
  std::vector<Fr> adv_blind((size_t)ncirc * pk.A * (bf + 1));
  const bool from_src = in.src || in.src1;
  if (from_src)  // a witness source writes straight into pinned staging, one per circuit,
    for (CircuitWs* w : W) {  // allocated once (a pinned allocation costs more than the copies it speeds up)
      if (w->wit_pin) continue;
      const size_t bytes = (size_t)std::max(pk.A, 1) * n * sizeof(Fr);
      if (hipHostMalloc((void**)&w->wit_pin, bytes, hipHostMallocDefault) == hipSuccess) {
        w->wit_pin_pinned = true;
      } else {  // pageable fallback: slower uploads, same bytes
        (void)hipGetLastError();
        w->wit_pin = static_cast<uint64_t*>(std::malloc(bytes));
        w->wit_pin_pinned = false;
        if (!w->wit_pin) return fail(H2G_ERR_NOMEM, "create_proof: witness staging allocation failed");
      }
    }
  const int NCH = (int)pk.ch_phase.size();
  std::vector<Fr> challenges(NCH);
  std::memset(challenges.data(), 0, challenges.size() * sizeof(Fr));
  StreamSyncGuard adv_guard{st};
  // the vanishing argument's seeds and chunk offsets (staging read by async copies: lives
  // until the proof returns), its commitment's ticket, and whether it was launched early
  // (queued behind phase 0's advice MSMs; placed after the advice commitments instead it
  // measured slower, profiles/r03/s3/ab_early_vanishing)
  std::vector<uint64_t> van_off;
  std::vector<uint32_t> van_seeds;
  StreamSyncGuard van_guard{st};  // destroyed before the staging above: the copies finish first
  {
    const uint64_t T = in.vthreads ? in.vthreads : 1;
    const uint64_t chunk = n / T, rem = n % T;
    for (uint64_t i = 0; i < rem && van_off.size() < T; i++) van_off.push_back(i * (chunk + 1));
    if (chunk)
      for (uint64_t o = rem * (chunk + 1); van_off.size() < T; o += chunk) van_off.push_back(o);
  }
  if ((int)van_off.size() > pk.max_chunks) {
    PALLOC(pk.pool, pk.d_seeds, van_off.size() * 8);
    PALLOC(pk.pool, pk.d_offsets, van_off.size());
    pk.max_chunks = (int)van_off.size();
  }
  MsmTicket van_tk;
  bool van_early = false;
  // it holds an MSM ring slot from phase 0 until y: only when every later stage's
  // outstanding commitments still fit beside it (advice phases, the permuted lookup
  // columns, the permutation / lookup / shuffle products)
  int peak_msms = 0;
  for (int ph = 0; ph <= pk.max_phase; ph++) {
    int a = 0;
    for (int c = 0; c < pk.A; c++) a += pk.adv_phase[c] == ph;
    peak_msms = std::max(peak_msms, a * ncirc);
  }
  peak_msms = std::max(peak_msms, 2 * ncirc * pk.NL);
  peak_msms = std::max(peak_msms, ncirc * (pk.nsets + pk.NL + pk.NS));
  const bool early_van = rng.seeded() && pk.van_pos >= 0 &&
                         pk.van_T == (uint32_t)van_off.size() && g_spmd.world <= 1 && g_shard.world <= 1 &&
                         peak_msms + 1 <= MSM_RING;
  auto launch_van_early = [&]() -> int {
    // the vanishing argument's random polynomial does not depend on the witness: with the
    // seeded RNG its seeds are the keystream bytes at the position the last proof drew
    // them from, so it is generated and its commitment MSM launched early -- queued behind
    // phase 0's advice MSMs, it runs under the advice transforms and the lookup and
    // permutation products instead of between the product commitments and y; the
    // vanishing stage checks that the real draws equal these bytes (else it redoes both)
    van_seeds.assign(van_off.size() * 8, 0);
    rng.peek((uint64_t)pk.van_pos, reinterpret_cast<uint8_t*>(van_seeds.data()), van_seeds.size() * 4);
    HIPCHK(pk_upload(pk, pk.d_seeds, van_seeds.data(), van_seeds.size() * 4, st));
    HIPCHK(pk_upload(pk, pk.d_offsets, van_off.data(), van_off.size() * 8, st));
    HIPCHK(chacha_random_poly(pk.random_poly, n, pk.d_seeds, pk.d_offsets, (int)van_off.size(), st, sl.lo, sl.hi1));
    RCCHK(commit_launch(d, prm, pk.random_poly, n, SRS_G, st, &van_tk));
    van_early = true;
    return H2G_OK;
  };
  std::vector<char> adv_shard((size_t)ncirc * pk.A, 0);  // advice columns distributed by their owners
  // advice handed over in host memory: the first column's upload has nothing to overlap
  // (its MSM needs the whole column), so the random polynomial's commitment goes first and
  // runs under that upload; device-resident advice keeps it behind the advice commitments
  // (H2G_VAN_FIRST=1: first in both cases -- A/B builds)
#ifndef H2G_VAN_FIRST
#define H2G_VAN_FIRST 0
#endif
#ifndef H2G_VAN_POS
#define H2G_VAN_POS 0
#endif
  const bool van_first = early_van && (!in.adv_dev || H2G_VAN_FIRST);
  for (int ph = 0; ph <= pk.max_phase; ph++) {
    if (ph == 0 && van_first) RCCHK(launch_van_early());
    std::vector<int> cols;
    for (int c = 0; c < pk.A; c++)
      if (pk.adv_phase[c] == ph) cols.push_back(c);
    if (from_src && ph > 0) HIPCHK(hipStreamSynchronize(st));  // the previous phase's uploads read the staging
    std::vector<MsmTicket> tk(cols.size() * ncirc);
    // a wide phase: column i (circuit-major) is rank i mod world's -- every rank uploads the
    // whole witness (the lookups and products read it), only the owner commits and
    // transforms the column
    const bool adv_wide = wide((int)(cols.size() * ncirc));
    const bool digest = g_spmd.world > 1 && !cols.empty();  // this phase's witness into the consistency digest
    if (digest) RCCHK(spmd_witness_prepare(pk, (int)(ncirc * cols.size()), st));
    for (int ci = 0; ci < ncirc; ci++) {
      CircuitWs& w = *W[ci];
      const uint64_t* from = in.advice ? in.advice[ci] : nullptr;
      bool from_dev = in.adv_dev;
      // copy_columns reads device advice in 16-byte chunks: refuse what it cannot
      if (from_dev && from && (reinterpret_cast<uintptr_t>(from) & 15) != 0)
        return fail(H2G_ERR_ARG, "create_proof: device advice must be 16-byte aligned");
      if (from_src) {
        // the staging outlives proofs: the unusable rows of unblinded columns start at zero
        // as the reference requires (prover.rs:417-421), whatever an earlier proof left there
        for (int c : cols)
          if (pk.unblinded[c]) std::memset(w.wit_pin + 4 * (n * c + unusable), 0, (n - unusable) * sizeof(Fr));
        const uint64_t* chp = reinterpret_cast<const uint64_t*>(challenges.data());
        const int frc = in.src ? in.src->fill(in.src->ctx, (uint32_t)ci, (uint32_t)ph, chp, w.wit_pin)
                               : in.src1->fill(in.src1->ctx, (uint32_t)ph, chp, w.wit_pin);
        if (frc)
          return fail(H2G_ERR_ARG, "create_proof: witness source failed at " +
                                       (ncirc > 1 ? "circuit " + std::to_string(ci) + " " : std::string()) + "phase " +
                                       std::to_string(ph));
        from = w.wit_pin;
        from_dev = false;
      }
      // column by column: upload, blinding rows, and (when the MSMs go one by one) the
      // commitment at once, so that a column's MSM overlaps the next column's upload
      // from host memory; the RNG draws keep the reference's order (every column's rows,
      // then every column's blind)
      const bool early = !adv_wide && commit_batch_chunk(prm, n, SRS_LAGRANGE) < 2;
      // device-resident columns come in through copy_columns (a streaming kernel, up to
      // COPY_COLS_MAX columns a launch; per-column DMA copies left the GPU idle for ~0.8 ms
      // of 32 columns at 2^18), host ones through the DMA upload; under SPMD either way
      // also takes each column's checksum before its blinding rows land (spmd_witness_fold)
      ColCopy cc{};
      int ncc = 0;
      auto flush = [&]() -> int {
        if (ncc) HIPCHK(copy_columns(cc, ncc, n, digest, st));
        ncc = 0;
        return H2G_OK;
      };
      auto blind = [&](int c) -> int {
        if (pk.unblinded[c]) return H2G_OK;
        Fr* rows = adv_blind.data() + ((size_t)ci * pk.A + c) * (bf + 1);
        for (int i = 0; i <= bf; i++) rows[i] = rng.random_fr();
        HIPCHK(pk_upload(pk, w.adv[c] + unusable, rows, (size_t)(bf + 1) * sizeof(Fr), st));
        return H2G_OK;
      };
      for (size_t k = 0; k < cols.size(); k++) {
        const int c = cols[k];
        const Fr* src = reinterpret_cast<const Fr*>(from + 4 * n * c);
        unsigned long long* sum = digest ? pk.wsum_d + (size_t)ci * cols.size() + k : nullptr;
        if (from_dev) {
          cc.src[ncc] = src;
          cc.dst[ncc] = w.adv[c];
          cc.sum[ncc++] = sum;
        } else {
          HIPCHK(hipMemcpyAsync(w.adv[c], src, n * sizeof(Fr), hipMemcpyHostToDevice, st));
          if (digest) {
            cc.src[ncc] = w.adv[c];
            cc.dst[ncc] = nullptr;
            cc.sum[ncc++] = sum;
          }
        }
        if (early || ncc == COPY_COLS_MAX || !from_dev) RCCHK(flush());
        if (early) {
          RCCHK(blind(c));
          RCCHK(commit_launch(d, prm, w.adv[c], n, SRS_LAGRANGE, st, &tk[(size_t)ci * cols.size() + k]));
        }
      }
      RCCHK(flush());
      if (!early) {  // every column's rows drawn in order, then one upload for the phase
        RCCHK(blind_stage(pk, (size_t)pk.A * (bf + 1)));
        std::vector<CopySeg> segs;
        for (int c : cols) {
          if (pk.unblinded[c]) continue;
          Fr* rows = adv_blind.data() + ((size_t)ci * pk.A + c) * (bf + 1);
          for (int i = 0; i <= bf; i++) rows[i] = rng.random_fr();
          segs.push_back(CopySeg{pk.blind_d + (size_t)c * (bf + 1), w.adv[c] + unusable, (uint64_t)(bf + 1)});
        }
        RCCHK(upload_rows_batch(pk, adv_blind.data() + (size_t)ci * pk.A * (bf + 1), (size_t)pk.A * (bf + 1), segs,
                                st));
      }
      for (int c : cols)
        if (!pk.unblinded[c]) (void)rng.random_fr();  // commitment blinds (unused by KZG)
      if (!cols.empty() && !early && !adv_wide) {
        std::vector<const Fr*> polys(cols.size());
        for (size_t i = 0; i < cols.size(); i++) polys[i] = w.adv[cols[i]];
        RCCHK(commit_launch_batch(d, prm, polys.data(), (int)cols.size(), n, SRS_LAGRANGE, st,
                                  tk.data() + (size_t)ci * cols.size()));
      }
    }
    if (digest) RCCHK(spmd_witness_fold(pk, (int)(ncirc * cols.size()), st));
    // H2G_VAN_POS 1: the random polynomial's commitment right behind the advice commitments,
    // ahead of the advice transforms on the prover's stream (0: behind them)
    if (ph == 0 && early_van && !van_first && H2G_VAN_POS == 1) RCCHK(launch_van_early());
    std::vector<int> adv_owner;
    std::vector<const Fr*> adv_lag;
    std::vector<Fr*> adv_poly, adv_cst;
    if (adv_wide) {
      for (int ci = 0; ci < ncirc; ci++)
        for (int c : cols) {
          adv_owner.push_back((int)(adv_owner.size() % (size_t)Wsp));
          adv_lag.push_back(W[ci]->adv[c]);
          adv_poly.push_back(W[ci]->adv_poly[c]);
          adv_cst.push_back(W[ci]->adv_coset[c]);
        }
      RCCHK(commit_launch_owned(d, prm, adv_lag.data(), adv_owner.data(), (int)adv_lag.size(), n, SRS_LAGRANGE, st,
                                tk.data()));
    }
    // the phase's advice to coefficient form and its extended-domain cosets do not depend
    // on any challenge: queued behind the uploads, they run while the commitment MSMs
    // (their own streams) are in flight (lagrange_to_coeff, prover.rs:673-689; the
    // cosets of evaluation.rs:344-361)
    if (pieces && !adv_wide && !cols.empty()) {  // one owner per column, every circuit's
      std::vector<const Fr*> l2;
      std::vector<Fr*> p2, c2;
      for (int ci = 0; ci < ncirc; ci++)
        for (int c : cols) {
          l2.push_back(W[ci]->adv[c]);
          p2.push_back(W[ci]->adv_poly[c]);
          c2.push_back(W[ci]->adv_coset[c]);
        }
      if (defer_adv) xform_later(l2, p2, c2);
      else RCCHK(xform(l2, p2, c2, nullptr));
    }
    for (int ci = 0; ci < ncirc && !cols.empty() && !adv_wide && !pieces; ci++) {
      CircuitWs& w = *W[ci];
      std::vector<const Fr*> src;
      std::vector<Fr*> dst, cst;
      for (int c : cols) {
        src.push_back(w.adv[c]);
        dst.push_back(w.adv_poly[c]);
        cst.push_back(w.adv_coset[c]);
      }
      if (coef_recv) continue;  // coefficients from the owners (coef_exchange), no cosets
      RCCHK(xs_begin());
      RCCHK(lagrange_to_coeff_batch(d, D, src.data(), dst.data(), (int)cols.size(), xst));
      RCCHK(ext_cosets(d, pk, (const Fr* const*)dst.data(), cst.data(), (int)cols.size(), xst));
      RCCHK(xs_end());
    }
    if (adv_wide) {
      RCCHK(xform(adv_lag, adv_poly, adv_cst, &adv_owner));
      for (int ci = 0; ci < ncirc; ci++)
        for (int c : cols) adv_shard[(size_t)ci * pk.A + c] = 1;
    }
    if (ph == 0 && early_van && !van_first && H2G_VAN_POS == 0) RCCHK(launch_van_early());
    if (ph == 0) clk.mark("upload+instances");
    {  // circuit by circuit, column by column
      std::vector<MsmTicket*> tl;
      for (auto& t : tk) tl.push_back(&t);
      RCCHK(collect_write(tl));
    }
    RCCHK(rng_ok());
    for (int i = 0; i < NCH; i++)
      if (pk.ch_phase[i] == ph) challenges[i] = tr.squeeze();
  }
  if (NCH)
    HIPCHK(pk_upload(pk, pk.consts + pk.num_consts, challenges.data(), NCH * sizeof(Fr), st));
  g_last_challenges = challenges;
  clk.mark("advice commit");

  const Fr theta = tr.squeeze();
  auto compress = [&](const CircuitWs& w, int2 seg, Fr* out) -> int {
    CompressArgs ca;
    ca.prog = pk.prog;
    ca.seg = seg;
    ca.n_slots = pk.n_slots;
    ca.consts = pk.consts;
    ca.load_col = w.d_load_col_lag;
    ca.load_rot = pk.d_load_rot;
    ca.n = n;
    ca.theta = theta;
    ca.out = out;
    HIPCHK(compress_lagrange(ca, st));
    return H2G_OK;
  };
  // ---- lookup_commit_permuted, per circuit, per lookup (lookup/prover.rs:64-173, 410-494)
  const int NLT = ncirc * pk.NL;  // (circuit, lookup) pairs, circuit-major: j = ci * NL + l
  bool lk_shard = false;  // the lookups went to their owners (A', S' and z distributed)
  std::vector<int> lk_owner_all(NLT, g_spmd.rank);
  {
    std::vector<MsmTicket> tk(2 * NLT);
    const size_t u = unusable;
    // per-lookup host staging (random rows, match counters): no host synchronisation
    // between lookups, so their device pipelines queue back to back; the counters are
    // checked once all lookups are queued
    std::vector<Fr> rows((size_t)NLT * 2 * (bf + 1));
    constexpr int LKC = ProvingKey::LKC;
    if ((size_t)NLT * LKC > pk.lk_cnt_len) {
      if (pk.lk_cnt) (void)hipHostFree(pk.lk_cnt);
      pk.lk_cnt = nullptr;
      pk.lk_cnt_len = 0;
      HIPCHK(hipHostMalloc((void**)&pk.lk_cnt, (size_t)NLT * LKC * sizeof(uint32_t), hipHostMallocDefault));
      pk.lk_cnt_len = (size_t)NLT * LKC;
    }
    constexpr int LKF = ProvingKey::LKF;
    if ((size_t)NLT > pk.lk_or_len) {
      if (pk.lk_or_d) (void)hipFree(pk.lk_or_d);
      if (pk.lk_or_h) (void)hipHostFree(pk.lk_or_h);
      pk.lk_or_d = pk.lk_or_h = nullptr;
      pk.lk_or_len = 0;
      HIPCHK(hipMalloc((void**)&pk.lk_or_d, (size_t)NLT * LKF * sizeof(unsigned long long)));
      HIPCHK(hipHostMalloc((void**)&pk.lk_or_h, (size_t)NLT * LKF * sizeof(unsigned long long), hipHostMallocDefault));
      pk.lk_or_len = (size_t)NLT;
    }
    if ((int)pk.lk_hb.size() < NLT) pk.lk_hb.resize(NLT, 64);
    if (NLT) HIPCHK(hipMemsetAsync(pk.lk_or_d, 0, (size_t)NLT * LKF * sizeof(unsigned long long), st));
    // permute_expression_pair (lookup/prover.rs:410-494): sort by Ord (canonical value),
    // match, fill leftovers; then the bf + 1 random rows (input first, then table).
    // Every lookup's two columns go through ONE radix sort (radix.hip): column g = 2 j + side
    // keys on a 48-bit window of its canonical values -- bits [hb - 48, hb) below the value
    // width hb the previous proof measured for that lookup (lk_hb) -- with g above the
    // window, so each column's rows come out contiguous and sorted.  The gather of the
    // canonical values checks the order (a window that tied different values); a lookup
    // whose check or width failed, or whose width is unknown (hb 0), is sorted in full
    // (four stable 64-bit limb sorts, least significant first).
    // a wide lookup stage: lookup j is rank j mod world's (its compression, sort, match and
    // fill, commitments and transforms); every rank still makes every RNG draw.  lq[j]:
    // the lookup's region in the batch buffers (-1: another rank's)
    const bool lk_wide = wide(NLT);
    std::vector<int>& lk_owner = lk_owner_all;
    std::vector<int> lq(NLT, -1);
    int nown = 0;
    for (int j = 0; j < NLT; j++) {
      if (lk_wide) lk_owner[j] = j % Wsp;
      if (lk_owner[j] == g_spmd.rank) lq[j] = nown++;
    }
    // Lookups with identical table expressions (the same table, e.g. keccak's nibble-xor
    // columns for every lookup) share one sorted table: lookup j gathers it from lookup
    // tsrc[j]'s group.  Batch groups: the inputs [0, nown), then one per distinct table
    // (H2G_LK_SHARED_TABLES; single-owner stages, and only while every lookup sorts by its
    // window -- a full sort writes its table group).  Otherwise two groups per lookup.
    std::vector<int> tsrc(NLT), gi0(NLT, -1), gi1(NLT, -1);
    bool share = H2G_LK_SHARED_TABLES && !lk_wide && pk.lk_trep.size() == (size_t)pk.NL &&
                 (int)pk.lk_hb.size() >= NLT;
    for (int j = 0; j < NLT && share; j++)
      if (lq[j] >= 0 && pk.lk_hb[j] == 0) share = false;
    int ntab = 0;
    for (int j = 0; j < NLT; j++) {
      tsrc[j] = j;
      if (lq[j] < 0) continue;
      if (share) {
        const int r = (j / pk.NL) * pk.NL + pk.lk_trep[j % pk.NL];
        if (lq[r] >= 0) tsrc[j] = r;
        gi0[j] = lq[j];
        if (tsrc[j] == j) gi1[j] = nown + ntab++;
        else gi1[j] = gi1[tsrc[j]];  // (r < j: assigned already)
      } else {
        gi0[j] = 2 * lq[j];
        gi1[j] = 2 * lq[j] + 1;
      }
    }
    const int G = share ? nown + ntab : 2 * nown;
    int gbits = 0;
    while ((1 << gbits) < G) gbits++;
    if (NLT && (size_t)G * u > pk.lkb_len) {  // grow-only batch buffers
      const size_t m = (size_t)G * u;
      PALLOC(pk.pool, pk.lkb_canon, m);
      for (int q = 0; q < 2; q++) {
        PALLOC(pk.pool, pk.lkb_key[q], m);
        PALLOC(pk.pool, pk.lkb_idx[q], m);
      }
      const size_t sb = std::max(std::max(radix_sort_scratch_bytes(m), radix_sort_scratch_bytes(n)),
                                 compact_scratch_bytes(n));
      HIPCHK(pk.pool.get(&pk.lkb_scr, sb));
      pk.lkb_len = m;
    }
    // the match and fill of lookup j from its sorted columns (pk.ck_a2 input, pk.ck_t2 table)
    // every lookup's counters and flags cleared at once (a redo clears its own again)
    if ((size_t)NLT > pk.lk_cf_n || u > pk.lk_cf_u) {
      PALLOC(pk.pool, pk.lk_counters, (size_t)NLT * LKC);
      PALLOC(pk.pool, pk.lk_flags, (size_t)NLT * u);
      pk.lk_cf_n = (size_t)NLT;
      pk.lk_cf_u = u;
    }
    if (NLT) {
      HIPCHK(hipMemsetAsync(pk.lk_counters, 0, (size_t)NLT * LKC * sizeof(uint32_t), st));
      HIPCHK(hipMemsetAsync(pk.lk_flags, 1, (size_t)NLT * u, st));
    }
    // scratch set q (0: the key's own) for the gathers and matches
    struct LkSet {
      CanonKey *a2, *t2, *left;
      uint8_t* rep;
      uint32_t* rows;
      void* scr;
    };
    auto lk_set = [&](int q) -> LkSet {
      if (q == 0) return LkSet{pk.ck_a2, pk.ck_t2, pk.ck_left, pk.rep_flag, pk.rep_rows, pk.lkb_scr};
      return LkSet{pk.lks_a2[q], pk.lks_t2[q], pk.lks_left[q], pk.lks_rep[q], pk.lks_rows[q], pk.lks_scr[q]};
    };
    auto match_fill = [&](int j, bool again, const LkSet& z, hipStream_t sj) -> int {
      const int ci = j / pk.NL, l = j % pk.NL;
      CircuitWs& w = *W[ci];
      uint32_t* cnt = pk.lk_counters + (size_t)LKC * j;
      uint8_t* flags = pk.lk_flags + (size_t)j * u;
      if (again) {
        HIPCHK(hipMemsetAsync(flags, 1, u, sj));
        HIPCHK(hipMemsetAsync(cnt, 0, LKC * sizeof(uint32_t), sj));
      }
      HIPCHK(lookup_mark(z.a2, z.t2, u, z.rep, flags, cnt + 2, sj));
      HIPCHK(compact_canon(z.t2, flags, u, z.left, cnt, z.scr, sj));
      HIPCHK(compact_index(z.rep, u, z.rows, cnt + 1, z.scr, sj));
      HIPCHK(lookup_assign(z.a2, z.rep, u, w.lk_ap[l], w.lk_sp[l], sj));
      HIPCHK(lookup_scatter(z.left, z.rows, cnt + 1, u, w.lk_sp[l], sj));
      if (again)
        HIPCHK(hipMemcpyAsync(pk.lk_cnt + (size_t)LKC * j, cnt, LKC * sizeof(uint32_t), hipMemcpyDeviceToHost, sj));
      return H2G_OK;  // the blinding rows of every lookup land together below (upload_rows_batch)
    };
    // the full sort of lookup j's columns into pk.ck_a2 / ck_t2 (radix sorts on the limbs,
    // in lookup j's own regions of the batch's key / index buffers)
    auto full_sort = [&](int j) -> int {
      const int ci = j / pk.NL, l = j % pk.NL;
      CircuitWs& w = *W[ci];
      const Fr* srcs[2] = {w.lk_a[l], w.lk_s[l]};
      CanonKey* sorted[2] = {pk.ck_a2, pk.ck_t2};
      for (int side = 0; side < 2; side++) {
        CanonKey* canon = pk.lkb_canon + (size_t)(side ? gi1[j] : gi0[j]) * u;
        HIPCHK(lookup_keys(srcs[side], u, 0, canon, nullptr, nullptr, pk.lk_or_d + (size_t)LKF * j, st));
        const size_t o = (size_t)gi0[j] * u;  // (the sort's scratch: the lookup's input group)
        uint64_t *k0 = pk.lkb_key[0] + o, *k1 = pk.lkb_key[1] + o;
        uint32_t *i0 = pk.lkb_idx[0] + o, *i1 = pk.lkb_idx[1] + o;
        HIPCHK(iota_u32(i0, u, st));
        for (int limb = 0; limb < 4; limb++) {  // least significant first; 8 passes end where they began
          HIPCHK(canon_limb_keys(canon, i0, u, limb, k0, st));
          bool alt = false;
          HIPCHK(radix_sort_pairs(k0, i0, k1, i1, u, 0, 64, pk.lkb_scr, st, &alt));
          if (alt) return fail(H2G_ERR_STATE, "lookup full sort: unexpected pass parity");
        }
        HIPCHK(lookup_gather(canon, i0, u, sorted[side], pk.lk_or_d + (size_t)LKF * j + 4, st));
      }
      return H2G_OK;
    };
    std::vector<int> used(NLT);
    {  // every lookup's compressed input and table, batched launches
      CompressBatch cb;
      cb.prog = pk.prog;
      cb.n_slots = pk.n_slots;
      cb.consts = pk.consts;
      cb.load_rot = pk.d_load_rot;
      cb.n = n;
      cb.theta = theta;
      auto add = [&](int2 seg, const CircuitWs& w, Fr* out) -> int {
        if (cb.count == COMPRESS_BATCH_MAX) {
          HIPCHK(compress_lagrange_batch(cb, st));
          cb.count = 0;
        }
        cb.seg[cb.count] = seg;
        cb.load_col[cb.count] = w.d_load_col_lag;
        cb.out[cb.count++] = out;
        return H2G_OK;
      };
      for (int ci = 0; ci < ncirc; ci++)
        for (int l = 0; l < pk.NL; l++)
          if (lq[ci * pk.NL + l] >= 0) {
            RCCHK(add(pk.seg_lk_in[l], *W[ci], W[ci]->lk_a[l]));
            RCCHK(add(pk.seg_lk_tab[l], *W[ci], W[ci]->lk_s[l]));
          }
      HIPCHK(compress_lagrange_batch(cb, st));
    }
    LookupKeysBatch kb;  // every column's keys, batched launches
    kb.n = u;
    kb.canon = pk.lkb_canon;
    kb.key = pk.lkb_key[0];
    kb.idx = pk.lkb_idx[0];
    kb.kbits = 48;
    kb.kmask = (1ull << 48) - 1;
    for (int ci = 0; ci < ncirc; ci++)
      for (int l = 0; l < pk.NL; l++) {
        const int j = ci * pk.NL + l;
        for (int which = 0; which < 2; which++) {
          Fr* r = rows.data() + ((size_t)2 * j + which) * (bf + 1);
          for (int i = 0; i <= bf; i++) r[i] = rng.random_fr();
        }
        (void)rng.random_fr();  // permuted input blind
        (void)rng.random_fr();  // permuted table blind
        if (lq[j] < 0) continue;
        used[j] = pk.lk_hb[j];
        const int shift = used[j] > 48 ? used[j] - 48 : 0;
        const Fr* srcs[2] = {W[ci]->lk_a[l], W[ci]->lk_s[l]};
        for (int side = 0; side < 2; side++) {  // every column keys (a full-sort lookup's are ignored)
          if (side == 1 && tsrc[j] != j) continue;  // a shared table: keyed once, by tsrc[j]
          if (kb.count == LOOKUP_KEYS_BATCH_MAX) {
            HIPCHK(lookup_keys_batch(kb, st));
            kb.count = 0;
          }
          kb.in[kb.count] = srcs[side];
          kb.s[kb.count] = shift;
          kb.g[kb.count] = side ? gi1[j] : gi0[j];
          kb.d_or[kb.count++] = pk.lk_or_d + (size_t)LKF * j;
        }
      }
    HIPCHK(lookup_keys_batch(kb, st));
    if (nown) {
      bool alt = false;
      HIPCHK(radix_sort_pairs(pk.lkb_key[0], pk.lkb_idx[0], pk.lkb_key[1], pk.lkb_idx[1], (size_t)G * u, 0,
                              48 + gbits, pk.lkb_scr, st, &alt));
      const uint32_t* sidx = pk.lkb_idx[alt ? 1 : 0];
      // the lookups' gathers and matches on LKS streams when none needs the full sort (its
      // radix passes use the key's scratch); lookup q-th of this rank on stream q mod LKS
      bool multi = nown > 1;
      for (int j = 0; j < NLT; j++) multi = multi && (lq[j] < 0 || used[j] != 0);
      const int S = multi ? std::min(nown, ProvingKey::LKS) : 1;
      if (S > 1) {
        if (pk.lks_n < u) {
          for (int q = 1; q < ProvingKey::LKS; q++) {
            PALLOC(pk.pool, pk.lks_a2[q], u);
            PALLOC(pk.pool, pk.lks_t2[q], u);
            PALLOC(pk.pool, pk.lks_left[q], u);
            PALLOC(pk.pool, pk.lks_rep[q], u);
            PALLOC(pk.pool, pk.lks_rows[q], u);
            HIPCHK(pk.pool.get(&pk.lks_scr[q], compact_scratch_bytes(u)));
          }
          pk.lks_n = u;
        }
        if (!pk.lk_st[0]) {
          for (int q = 0; q < ProvingKey::LKS; q++) HIPCHK(hipStreamCreateWithFlags(&pk.lk_st[q], hipStreamNonBlocking));
          for (int q = 0; q <= ProvingKey::LKS; q++) HIPCHK(hipEventCreateWithFlags(&pk.lk_ev[q], hipEventDisableTiming));
        }
        HIPCHK(hipEventRecord(pk.lk_ev[0], st));  // the sort is done
        for (int q = 0; q < S; q++) HIPCHK(hipStreamWaitEvent(pk.lk_st[q], pk.lk_ev[0], 0));
      }
      int qi = 0;
      for (int j = 0; j < NLT; j++) {
        if (lq[j] < 0) continue;
        const int q = S > 1 ? qi % S : 0;
        qi++;
        const LkSet z = lk_set(q);
        hipStream_t sj = S > 1 ? pk.lk_st[q] : st;
        if (used[j] == 0) {
          RCCHK(full_sort(j));
        } else {
          for (int side = 0; side < 2; side++) {
            const size_t g = (size_t)(side ? gi1[j] : gi0[j]);
            HIPCHK(lookup_gather(pk.lkb_canon + g * u, sidx + g * u, u, side ? z.t2 : z.a2,
                                 pk.lk_or_d + (size_t)LKF * j + 4, sj));
          }
        }
        RCCHK(match_fill(j, false, z, sj));
      }
      if (S > 1) {  // join
        for (int q = 0; q < S; q++) {
          HIPCHK(hipEventRecord(pk.lk_ev[q + 1], pk.lk_st[q]));
          HIPCHK(hipStreamWaitEvent(st, pk.lk_ev[q + 1], 0));
        }
      }
    }
    if (NLT) {
      HIPCHK(hipMemcpyAsync(pk.lk_cnt, pk.lk_counters, (size_t)NLT * LKC * sizeof(uint32_t), hipMemcpyDeviceToHost,
                            st));
      HIPCHK(hipMemcpyAsync(pk.lk_or_h, pk.lk_or_d, (size_t)NLT * LKF * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));  // counters and value masks landed; rows (host) read
    }
    // a sort whose assumption failed (values wider than its window, or a window that tied
    // different values out of order) is redone with the full sort; the width is
    // remembered for the next proof
    bool redo = false;
    std::vector<char> redone(NLT, 0);  // a lookup matched against a shared table redone with it
    for (int j = 0; j < NLT; j++) {
      if (lq[j] < 0 || used[j] == 0) continue;
      const unsigned long long* f = pk.lk_or_h + (size_t)LKF * j;
      int hb = 0;
      for (int q = 3; q >= 0 && !hb; q--)
        if (f[q]) hb = 64 * q + 64 - __builtin_clzll(f[q]);
      if (hb == 0) hb = 1;
      const bool tie = f[4] != 0;
      pk.lk_hb[j] = tie && hb == used[j] ? 0 : hb;  // ties at the right width: full sort from now on
      if (tie || hb > used[j] || redone[tsrc[j]]) {
        RCCHK(full_sort(j));
        RCCHK(match_fill(j, true, lk_set(0), st));
        redo = true;
        redone[j] = 1;
      }
    }
    if (redo) HIPCHK(hipStreamSynchronize(st));
    {  // the blinding rows of A'_l and S'_l of every lookup this rank sorted, one upload
      RCCHK(blind_stage(pk, rows.size()));
      std::vector<CopySeg> segs;
      for (int j = 0; j < NLT; j++) {
        if (lq[j] < 0) continue;
        CircuitWs& w = *W[j / pk.NL];
        const int l = j % pk.NL;
        for (int which = 0; which < 2; which++)
          segs.push_back(CopySeg{pk.blind_d + ((size_t)2 * j + which) * (bf + 1), (which ? w.lk_sp[l] : w.lk_ap[l]) + u,
                                 (uint64_t)(bf + 1)});
      }
      RCCHK(upload_rows_batch(pk, rows.data(), rows.size(), segs, st));
    }
    bool lk_ok = true;
    for (int j = 0; j < NLT; j++) {
      const uint32_t* cnt = pk.lk_cnt + (size_t)LKC * j;
      if (lq[j] >= 0 && (cnt[2] != 0 || cnt[0] != cnt[1])) lk_ok = false;
    }
    if (lk_wide) {  // every rank learns whether any owner's lookup failed (none may hang in a collective)
      std::vector<Fr> mine(1, lk_ok ? Fr::zero() : Fr::one()), all;
      RCCHK(spmd_allgather_fr(mine, &all));
      for (const Fr& f : all) lk_ok = lk_ok && f.is_zero();
    }
    if (!lk_ok) return fail(H2G_ERR_ARG, "create_proof: lookup input value not in the table (ConstraintSystemFailure)");
    std::vector<const Fr*> perm_cols;  // (A'_l, S'_l) in transcript order
    std::vector<Fr*> perm_polys, perm_cosets;
    for (int ci = 0; ci < ncirc; ci++)
      for (int l = 0; l < pk.NL; l++) {
        CircuitWs& w = *W[ci];
        perm_cols.push_back(w.lk_ap[l]);
        perm_cols.push_back(w.lk_sp[l]);
        perm_polys.push_back(w.lk_ap_poly[l]);
        perm_polys.push_back(w.lk_sp_poly[l]);
        perm_cosets.push_back(w.lk_apc[l]);
        perm_cosets.push_back(w.lk_spc[l]);
      }
    std::vector<int> own2(2 * NLT);
    for (int j = 0; j < NLT; j++) own2[2 * j] = own2[2 * j + 1] = lk_wide ? lk_owner[j] : g_spmd.rank;
    // A', S' against the prefix-summed Lagrange basis (params_prefix): the same commitments
    std::vector<const Fr*> com_cols = perm_cols;
    int com_set = SRS_LAGRANGE;
    if (H2G_LOOKUP_PREFIX) {
      RCCHK(params_prefix(prm, st));
      // scalars only for the columns this rank commits (all of them but in a wide stage,
      // where a column belongs to its owner)
      size_t owned = 0;
      for (int i = 0; i < 2 * NLT; i++) owned += own2[i] == g_spmd.rank;
      const size_t need = std::max<size_t>(owned, 1) * n;
      if (need > pk.lk_diff_len) {
        PALLOC(pk.pool, pk.lk_diff, need);
        pk.lk_diff_len = need;
      }
      PrefixDiff pd{};
      int m = 0;
      size_t slot = 0;
      for (int i = 0; i < 2 * NLT; i++) {
        if (own2[i] != g_spmd.rank) {  // another rank's column (wide stage): not read here
          com_cols[i] = perm_cols[i];
          continue;
        }
        Fr* e = pk.lk_diff + (slot++) * n;
        com_cols[i] = e;
        pd.a[m] = perm_cols[i];
        pd.e[m] = e;
        if (++m == PREFIX_DIFF_MAX) {
          HIPCHK(prefix_diff(pd, m, n, st));
          m = 0;
        }
      }
      if (m) HIPCHK(prefix_diff(pd, m, n, st));
      com_set = SRS_LAGRANGE_PREFIX;
    }
    if (lk_wide) {
      RCCHK(commit_launch_owned(d, prm, com_cols.data(), own2.data(), 2 * NLT, n, com_set, st, tk.data()));
      RCCHK(xform(perm_cols, perm_polys, perm_cosets, &own2));
    } else {
      RCCHK(commit_launch_batch(d, prm, com_cols.data(), 2 * NLT, n, com_set, st, tk.data()));
      // coefficient forms and cosets, batched transforms (they overlap the commitments)
      RCCHK(xform(perm_cols, perm_polys, perm_cosets, nullptr));
    }
    lk_shard = lk_wide;
    {
      std::vector<MsmTicket*> tl;
      for (int i = 0; i < 2 * NLT; i++) tl.push_back(&tk[i]);
      RCCHK(collect_write(tl));
    }
    RCCHK(rng_ok());
  }
  if (pk.NL) clk.mark("lookup permuted");
  const Fr beta = tr.squeeze(), gamma = tr.squeeze();
  dump("beta", &beta, 1, st, true);
  dump("gamma", &gamma, 1, st, true);

  // ---- permutation_commit per circuit (permutation/prover.rs:50-197); commitments are
  // written after the loop (nothing is squeezed in between, so the transcript is unchanged)
  const int NST = ncirc * pk.nsets;  // (circuit, set), circuit-major
  std::vector<MsmTicket> perm_tk(NST);
  // large MSMs start as soon as their set's z is ready; small ones wait and go as a batch
  const bool perm_batched = commit_batch_chunk(prm, n, SRS_LAGRANGE) > 1;
  // host staging of every set's / product's blinding rows: no host synchronisation per
  // set, the transforms of all sets go as batches after the loop
  std::vector<Fr> perm_blind((size_t)NST * bf), prod_blind((size_t)ncirc * (pk.NL + pk.NS) * bf);
  StreamSyncGuard blind_guard{st};
  std::vector<Fr*> all_z_lag, all_z, all_z_coset;
  for (CircuitWs* w : W)
    for (int s = 0; s < pk.nsets; s++) {
      all_z_lag.push_back(w->z_lag[s]);
      all_z.push_back(w->z[s]);
      all_z_coset.push_back(w->z_coset[s]);
    }
  auto col_vals = [&](const CircuitWs& w, int c) -> const Fr* {
    const auto& pc = pk.perm_cols[c];
    return pc.first == COL_ADVICE ? w.adv[pc.second]
                                  : (pc.first == COL_FIXED ? pk.fixed_lag[pc.second] : w.inst_val[pc.second]);
  };
  // with row pieces the grand products go by slabs: each rank forms its MSM slab's rows of
  // every set (denominators, inversion, numerators, a slab-local running product), one host
  // all-gather of the slabs' products chains the slabs and the sets (z_0 of set s + 1 is
  // set s's last product row), the commitments take the slabs, and each set's transform
  // owner gathers the whole column
  const bool perm_slab = pieces && NST > 0;
  if (perm_slab) {
    const int me = g_spmd.rank;
    const size_t plo = shard_lo(prm.n, n, Wsp, me), phi = shard_lo(prm.n, n, Wsp, me + 1), len = phi - plo;
    std::vector<Fr*> zl(NST), zs(NST);
    for (int i = 0; i < NST; i++) {
      zl[i] = all_z_lag[i] + plo;
      zs[i] = all_z[i] + plo;
    }
    for (int ci = 0; ci < ncirc; ci++)
      for (int s = 0; s < pk.nsets; s++) {
        const int c0 = s * pk.chunk_len, c1 = std::min(c0 + pk.chunk_len, pk.P);
        for (int c = c0; c < c1 && len; c += PERM_MAXC) {
          PermCols pc;
          pc.m = std::min(PERM_MAXC, c1 - c);
          for (int j = 0; j < pc.m; j++) {
            pc.v[j] = col_vals(*W[ci], c + j) + plo;
            pc.sigma[j] = pk.sigma_lag[c + j] + plo;
          }
          HIPCHK(perm_denominators(zl[(size_t)ci * pk.nsets + s], len, pc, beta, gamma, c == c0, st));
        }
      }
    if (len) HIPCHK(poly_batch_invert_multi(zl.data(), zs.data(), NST, len, st));
    for (int ci = 0; ci < ncirc; ci++) {
      Fr deltaomega = Fr::one();
      for (int s = 0; s < pk.nsets; s++) {
        const int c0 = s * pk.chunk_len, c1 = std::min(c0 + pk.chunk_len, pk.P);
        for (int c = c0; c < c1; c += PERM_MAXC) {
          PermCols pc;
          pc.m = std::min(PERM_MAXC, c1 - c);
          for (int j = 0; j < pc.m; j++) {
            pc.v[j] = col_vals(*W[ci], c + j) + plo;
            pc.beta_delta[j] = deltaomega * beta;
            deltaomega = deltaomega * fr_delta();
          }
          if (len) HIPCHK(perm_numerators(zl[(size_t)ci * pk.nsets + s], len, pc, gamma, pk.om, st, plo));
        }
      }
    }
    if (len)
      HIPCHK(poly_prefix_product_multi((const Fr* const*)zl.data(), zs.data(), NST, len, pk.scr, pk.scr_len, st));
    // the slab's product of the rows that feed z (factors below n - bf - 1)
    const size_t hc = std::min(phi, n - (size_t)bf - 1);
    std::vector<Fr> tp(NST, Fr::one());
    if (hc > plo)
      for (int i = 0; i < NST; i++)
        HIPCHK(hipMemcpyAsync(&tp[i], all_z[i] + hc - 1, sizeof(Fr), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::vector<Fr> allp;
    RCCHK(spmd_allgather_fr(tp, &allp));
    std::vector<Fr> lzp(NST);  // z at this slab's first row = z_0 * (the slabs below)
    for (int ci = 0; ci < ncirc; ci++) {
      Fr lz = Fr::one();
      for (int s = 0; s < pk.nsets; s++) {
        const int i = ci * pk.nsets + s;
        Fr below = Fr::one(), all = Fr::one();
        for (int r = 0; r < Wsp; r++) {
          if (r < me) below = below * allp[(size_t)r * NST + i];
          all = all * allp[(size_t)r * NST + i];
        }
        lzp[i] = lz * below;
        lz = lz * all;
      }
    }
    if (!pk.perm_lz || pk.perm_lz_len < (size_t)NST) {
      PALLOC(pk.pool, pk.perm_lz, NST);
      pk.perm_lz_len = (size_t)NST;
    }
    HIPCHK(pk_upload(pk, pk.perm_lz, lzp.data(), NST * sizeof(Fr), st));
    for (int i = 0; i < NST; i++) {
      Fr* blind_rows = perm_blind.data() + (size_t)i * bf;
      for (int q = 0; q < bf; q++) blind_rows[q] = rng.random_fr();
      (void)rng.random_fr();  // blind
      HIPCHK(pk_upload(pk, pk.small, blind_rows, bf * sizeof(Fr), st));
      HIPCHK(perm_z_assemble(all_z_lag[i], n, bf, all_z[i], pk.perm_lz + i, pk.small, st, plo, phi));
    }
    HIPCHK(hipStreamSynchronize(st));  // lzp (host) was read
    RCCHK(commit_launch_batch(d, prm, (const Fr* const*)all_z_lag.data(), NST, n, SRS_LAGRANGE, st, perm_tk.data()));
    // each set's owner gathers its column, then transforms and distributes it
    std::vector<int> own(NST);
    for (int i = 0; i < NST; i++) own[i] = (tr_next + i) % Wsp;
    tr_next += NST;
    RCCHK(gather_to_owners(pk, all_z_lag, own, prm.n, st));
    RCCHK(xform(std::vector<const Fr*>(all_z_lag.begin(), all_z_lag.end()), all_z, all_z_coset, &own));
    RCCHK(run_deferred());  // the advice columns' transforms beside the products
  }
  if (!perm_slab) {
    // every set's denominators (into z_lag), one batched inversion over all circuits'
    // sets (z as its scratch until the iNTT fills it), then per set numerators, scan and z
    for (int ci = 0; ci < ncirc; ci++)
      for (int s = 0; s < pk.nsets; s++) {
        const int c0 = s * pk.chunk_len, c1 = std::min(c0 + pk.chunk_len, pk.P);
        for (int c = c0; c < c1; c += PERM_MAXC) {
          PermCols pc;
          pc.m = std::min(PERM_MAXC, c1 - c);
          for (int j = 0; j < pc.m; j++) {
            pc.v[j] = col_vals(*W[ci], c + j);
            pc.sigma[j] = pk.sigma_lag[c + j];
          }
          HIPCHK(perm_denominators(W[ci]->z_lag[s], n, pc, beta, gamma, c == c0, st));
        }
      }
    if (NST) dump("den0", W[0]->z_lag[0], n, st);
    HIPCHK(poly_batch_invert_multi(all_z_lag.data(), all_z.data(), NST, n, st));
    if (NST) dump("inv0", W[0]->z_lag[0], n, st);
#ifndef H2G_PERM_MULTI  // 1: every set's numerators, then ONE batched scan of all sets (A/B)
#define H2G_PERM_MULTI 0
#endif
    if (H2G_PERM_MULTI && NST > 1) {
      // the sets' running products do not depend on each other (z_s = z_{s-1}'s last usable
      // value x its own scan): one batched scan of every set's products into z's coefficient
      // arrays (free until the iNTT), then each z assembled from the previous set's last value
      // on the device -- the same values, the same RNG draws in the same order
      for (int ci = 0; ci < ncirc; ci++) {
        Fr deltaomega = Fr::one();
        for (int s = 0; s < pk.nsets; s++) {
          const int c0 = s * pk.chunk_len, c1 = std::min(c0 + pk.chunk_len, pk.P);
          for (int c = c0; c < c1; c += PERM_MAXC) {
            PermCols pc;
            pc.m = std::min(PERM_MAXC, c1 - c);
            for (int j = 0; j < pc.m; j++) {
              pc.v[j] = col_vals(*W[ci], c + j);
              pc.beta_delta[j] = deltaomega * beta;
              deltaomega = deltaomega * fr_delta();
            }
            HIPCHK(perm_numerators(W[ci]->z_lag[s], n, pc, gamma, pk.om, st));
          }
        }
      }
      HIPCHK(poly_prefix_product_multi((const Fr* const*)all_z_lag.data(), all_z.data(), NST, n, pk.scr, pk.scr_len,
                                       st));
      for (int ci = 0; ci < ncirc; ci++) {
        CircuitWs& w = *W[ci];
        HIPCHK(hipMemcpyAsync(pk.last_z, pk.one, sizeof(Fr), hipMemcpyDeviceToDevice, st));  // z_0 starts at one
        for (int s = 0; s < pk.nsets; s++) {
          const size_t i = (size_t)ci * pk.nsets + s;
          Fr* blind_rows = perm_blind.data() + i * bf;
          for (int q = 0; q < bf; q++) blind_rows[q] = rng.random_fr();
          (void)rng.random_fr();  // blind
          HIPCHK(pk_upload(pk, pk.small, blind_rows, bf * sizeof(Fr), st));
          HIPCHK(perm_z_assemble(w.z_lag[s], n, bf, all_z[i], pk.last_z, pk.small, st));
          HIPCHK(hipMemcpyAsync(pk.last_z, w.z_lag[s] + (n - (size_t)(bf + 1)), sizeof(Fr), hipMemcpyDeviceToDevice,
                                st));
          if (!perm_batched) RCCHK(commit_launch(d, prm, w.z_lag[s], n, SRS_LAGRANGE, st, &perm_tk[i]));
        }
      }
    }
    for (int ci = 0; ci < ncirc && !(H2G_PERM_MULTI && NST > 1); ci++) {
      CircuitWs& w = *W[ci];
      HIPCHK(hipMemcpyAsync(pk.last_z, pk.one, sizeof(Fr), hipMemcpyDeviceToDevice, st));  // z_0 starts at one
      Fr deltaomega = Fr::one();
      for (int s = 0; s < pk.nsets; s++) {
        Fr* blind_rows = perm_blind.data() + ((size_t)ci * pk.nsets + s) * bf;
        const int c0 = s * pk.chunk_len, c1 = std::min(c0 + pk.chunk_len, pk.P);
        Fr* prod = w.z_lag[s];
        for (int c = c0; c < c1; c += PERM_MAXC) {
          PermCols pc;
          pc.m = std::min(PERM_MAXC, c1 - c);
          for (int j = 0; j < pc.m; j++) {
            pc.v[j] = col_vals(w, c + j);
            pc.beta_delta[j] = deltaomega * beta;
            deltaomega = deltaomega * fr_delta();
          }
          HIPCHK(perm_numerators(prod, n, pc, gamma, pk.om, st));
        }
        // z = last_z * running product, blinding rows from the rng
        if (ci == 0 && s == 0) dump("mod0", prod, n, st);
        HIPCHK(poly_prefix_product(prod, pk.pre, n, pk.scr, pk.scr_len, st));
        if (ci == 0 && s == 0) dump("pre0", pk.pre, n, st);
        for (int i = 0; i < bf; i++) blind_rows[i] = rng.random_fr();
        (void)rng.random_fr();  // blind
        HIPCHK(pk_upload(pk, pk.small, blind_rows, bf * sizeof(Fr), st));
        HIPCHK(perm_z_assemble(w.z_lag[s], n, bf, pk.pre, pk.last_z, pk.small, st));
        HIPCHK(hipMemcpyAsync(pk.last_z, w.z_lag[s] + (n - (size_t)(bf + 1)), sizeof(Fr), hipMemcpyDeviceToDevice,
                              st));
        if (ci == 0 && s == 0) {
          dump("z0", w.z_lag[s], n, st);
          dump("sigma0", pk.sigma_lag[0], n, st);
          dump("v0", col_vals(w, 0), n, st);
        }
        if (!perm_batched)
          RCCHK(commit_launch(d, prm, w.z_lag[s], n, SRS_LAGRANGE, st, &perm_tk[(size_t)ci * pk.nsets + s]));
      }
    }
    RCCHK(xform(std::vector<const Fr*>(all_z_lag.begin(), all_z_lag.end()), all_z, all_z_coset, nullptr));
  }
  if (perm_batched && !perm_slab)
    RCCHK(commit_launch_batch(d, prm, (const Fr* const*)all_z_lag.data(), NST, n, SRS_LAGRANGE, st, perm_tk.data()));
  clk.mark("permutation products");
  // ---- lookup products (lookup/prover.rs:182-325), every circuit's, then shuffle
  // products (shuffle/prover.rs:97-206): z = [1, running product ...], bf random rows, blind
  const int NSH = ncirc * pk.NS;
  std::vector<MsmTicket> lkz_tk(NLT), shz_tk(NSH);
  {
    std::vector<const Fr*> z_lags;
    std::vector<Fr*> z_polys, z_cosets;
    // a wide lookup stage keeps its owners here: lookup j's product is rank j mod world's
    // (the permuted columns are already there); the others only make the RNG draws
    const bool lz_wide = lk_shard;
    auto mine = [&](int j) { return lk_owner_all[j] == g_spmd.rank; };
    size_t zrow = 0;
    // every product's random rows and blind, drawn up front in the products' order (no
    // other draws come between them) and uploaded once
    const size_t nprod = (size_t)NLT + (size_t)NSH;
    for (size_t z = 0; z < nprod; z++) {
      Fr* rows = prod_blind.data() + z * (size_t)bf;
      for (int i = 0; i < bf; i++) rows[i] = rng.random_fr();
      (void)rng.random_fr();  // product blind
    }
    if (nprod) {
      RCCHK(blind_stage(pk, nprod * (size_t)bf));
      HIPCHK(pk_upload(pk, pk.blind_d, prod_blind.data(), nprod * (size_t)bf * sizeof(Fr), st));
    }
    // prod: the running product's factors, or (scanned) already its prefix products
    auto finish_z = [&](const Fr* prod, Fr* z_lag, Fr* z_poly, Fr* z_coset, bool scanned, bool here,
                        bool listed) -> int {
      const Fr* rows_d = pk.blind_d + (zrow++) * (size_t)bf;
      if (!here) return H2G_OK;
      const Fr* pre = prod;
      if (!scanned) {
        HIPCHK(poly_prefix_product(prod, pk.pre, n, pk.scr, pk.scr_len, st));
        pre = pk.pre;
      }
      HIPCHK(perm_z_assemble(z_lag, n, bf, pre, pk.one, rows_d, st));
      if (listed) {
        z_lags.push_back(z_lag);
        z_polys.push_back(z_poly);
        z_cosets.push_back(z_coset);
      }
      return H2G_OK;
    };
    // every lookup's denominators go through one batched inversion (the per-thread
    // inversion's latency is paid once); z_poly holds the product until its iNTT,
    // z_lag serves as the inversion's scratch until z is assembled into it
    std::vector<Fr*> dens, dens_scr;
    for (int ci = 0, j = 0; ci < ncirc; ci++)
      for (int l = 0; l < pk.NL; l++, j++) {
        if (!mine(j)) continue;
        CircuitWs* w = W[ci];
        HIPCHK(lookup_prod_den(w->lk_ap[l], w->lk_sp[l], beta, gamma, w->lk_z_poly[l], n, st));
        dens.push_back(w->lk_z_poly[l]);
        dens_scr.push_back(w->lk_z[l]);
      }
    if (!dens.empty()) HIPCHK(poly_batch_invert_multi(dens.data(), dens_scr.data(), (int)dens.size(), n, st));
    // numerators, then every lookup's running product in one batched scan (in place)
    for (int ci = 0, j = 0; ci < ncirc; ci++)
      for (int l = 0; l < pk.NL; l++, j++)
        if (mine(j)) HIPCHK(lookup_prod_num(W[ci]->lk_a[l], W[ci]->lk_s[l], beta, gamma, W[ci]->lk_z_poly[l], n, st));
    if (!dens.empty())
      HIPCHK(poly_prefix_product_multi((const Fr* const*)dens.data(), dens.data(), (int)dens.size(), n, pk.scr,
                                       pk.scr_len, st));
    std::vector<const Fr*> lkz_lag;
    std::vector<Fr*> lkz_poly, lkz_cst;
    for (int ci = 0, j = 0; ci < ncirc; ci++)
      for (int l = 0; l < pk.NL; l++, j++) {
        CircuitWs* w = W[ci];
        RCCHK(finish_z(w->lk_z_poly[l], w->lk_z[l], w->lk_z_poly[l], w->lk_zc[l], true, mine(j), !lz_wide));
        lkz_lag.push_back(w->lk_z[l]);
        lkz_poly.push_back(w->lk_z_poly[l]);
        lkz_cst.push_back(w->lk_zc[l]);
      }
    for (CircuitWs* w : W)
      for (int s = 0; s < pk.NS; s++) {
        RCCHK(compress(*w, pk.seg_sh_in[s], pk.tmp_a));
        RCCHK(compress(*w, pk.seg_sh_sh[s], pk.tmp_b));
        HIPCHK(shuffle_prod_den(pk.tmp_b, gamma, pk.mod, n, st));
        HIPCHK(poly_batch_invert(pk.mod, n, pk.scr, st));
        HIPCHK(shuffle_prod_num(pk.tmp_a, gamma, pk.mod, n, st));
        RCCHK(finish_z(pk.mod, w->sh_z[s], w->sh_z_poly[s], w->sh_zc[s], false, true, true));
      }
    RCCHK(xform(z_lags, z_polys, z_cosets, nullptr));
    // product commitments: every circuit's lookups, then every circuit's shuffles
    std::vector<const Fr*> zs;
    for (CircuitWs* w : W) zs.insert(zs.end(), w->lk_z.begin(), w->lk_z.end());
    for (CircuitWs* w : W) zs.insert(zs.end(), w->sh_z.begin(), w->sh_z.end());
    std::vector<MsmTicket> zt(zs.size());
    if (lz_wide) {
      RCCHK(commit_launch_owned(d, prm, zs.data(), lk_owner_all.data(), NLT, n, SRS_LAGRANGE, st, zt.data()));
      if (NSH) RCCHK(commit_launch_batch(d, prm, zs.data() + NLT, NSH, n, SRS_LAGRANGE, st, zt.data() + NLT));
      RCCHK(xform(lkz_lag, lkz_poly, lkz_cst, &lk_owner_all));
    } else if (!zs.empty()) {
      RCCHK(commit_launch_batch(d, prm, zs.data(), (int)zs.size(), n, SRS_LAGRANGE, st, zt.data()));
    }
    for (int j = 0; j < NLT; j++) lkz_tk[j] = zt[j];
    for (int j = 0; j < NSH; j++) shz_tk[j] = zt[NLT + j];
  }
  if (pk.NL + pk.NS) clk.mark("lookup/shuffle products");
  // ---- vanishing commit (vanishing/prover.rs:40-98)
  {
    const uint64_t at = rng.position();
    std::vector<uint32_t> drawn(van_off.size() * 8, 0);
    for (size_t i = 0; i < van_off.size(); i++) rng.fill(reinterpret_cast<uint8_t*>(&drawn[8 * i]), 32);
    if (van_early && (at != (uint64_t)pk.van_pos || drawn != van_seeds)) {
      // the early draws were not the real ones: drop that commitment, redo it below
      G1Affine unused;
      RCCHK(commit_collect(d, &van_tk, &unused));
      van_early = false;
    }
    if (rng.seeded()) {
      pk.van_pos = (int64_t)at;
      pk.van_T = (uint32_t)van_off.size();
    }
    if (!van_early) {
      van_seeds = drawn;
      HIPCHK(pk_upload(pk, pk.d_seeds, van_seeds.data(), van_seeds.size() * 4, st));
      HIPCHK(pk_upload(pk, pk.d_offsets, van_off.data(), van_off.size() * 8, st));
      // a slab-mode rank draws only its coefficients (and the halo) of the random polynomial
      HIPCHK(chacha_random_poly(pk.random_poly, n, pk.d_seeds, pk.d_offsets, (int)van_off.size(), st, sl.lo,
                                sl.hi1));
    }
    (void)rng.random_fr();  // random_blind
    RCCHK(rng_ok());
    if (!van_early) RCCHK(commit_launch(d, prm, pk.random_poly, n, SRS_G, st, &van_tk));
  }
  // the instance columns' cosets do not depend on y: they overlap the permutation /
  // vanishing MSMs (the advice went to coefficients and cosets under its own MSMs)
  for (CircuitWs* w : W)
    RCCHK(ext_cosets(d, pk, (const Fr* const*)w->inst_poly.data(), w->inst_coset.data(), pk.I, st));
  {
    std::vector<MsmTicket*> tl;
    for (auto* tks : {&perm_tk, &lkz_tk, &shz_tk})
      for (auto& t : *tks) tl.push_back(&t);
    tl.push_back(&van_tk);
    RCCHK(collect_write(tl));
  }
  RCCHK(run_deferred());  // (no permutation stage ran them)
  RCCHK(xp_flush(pk, st));  // the overlapped exchanges' rows, before h(X) reads them
  clk.mark("perm+vanishing commits, cosets");
  HIPCHK(xjoin.join());  // the columns' cosets and coefficients (the transform stream)
  const Fr y = tr.squeeze();
  // ---- evaluate_h (evaluation.rs:317-620): one launch per circuit, each continuing the
  // previous circuit's Horner chain in y; the last one divides by t(X)
  const bool subc = spmd_subcosets();
  for (int ci = 0; ci < ncirc && !subc; ci++) {
    const CircuitWs& w = *W[ci];
    EvalHArgs a;
    a.prog = pk.prog;
    a.gates = pk.seg_gates;
    a.n_slots = pk.n_slots;
    a.theta = theta;
    a.nlookups = pk.NL;
    a.nshuffles = pk.NS;
    a.lookups = w.d_lookups;
    a.shuffles = w.d_shuffles;
    a.consts = pk.consts;
    a.query_col = w.d_load_col;
    a.query_rot = pk.d_load_rot;
    a.nsets = pk.nsets;
    a.chunk_len = pk.chunk_len;
    a.P = pk.P;
    a.z = w.d_z;
    a.perm_v = w.d_perm_v;
    a.sigma = pk.d_sigma;
    a.l0 = pk.l0;
    a.l_last = pk.l_last;
    a.l_active = pk.l_active;
    a.beta = beta;
    a.gamma = gamma;
    a.y = y;
    a.delta_start = beta * zeta();
    a.delta = fr_delta();
    a.ext_omega = pk.eo;
    a.ext = ext;
    a.rot_scale = pk.rot_scale;
    a.last_rot = -(bf + 1);
    a.t_evals = D.d_t;
    a.t_mask = D.t_evals.size() - 1;
    a.acc_in = ci > 0 ? pk.h_ext : nullptr;
    a.divide = ci + 1 == ncirc;
    a.out = pk.h_ext;
    HIPCHK(evaluate_h(a, st));
  }
  if (subc) {  // rows of this rank's sub-cosets, then every sub-coset's h from its owner
    const int e = (int)(D.ek - D.k);
    for (CircuitWs* w : W) RCCHK(sub_ws_tables(pk, *w));
    for (size_t i = 0; i < pk.sub_ts.size(); i++) {
      const uint64_t t = pk.sub_ts[i];
      Fr* slot = pk.h_gather + t * n;
      for (int ci = 0; ci < ncirc; ci++) {
        const CircuitWs& w = *W[ci];
        EvalHArgs a;
        a.prog = pk.prog;
        a.gates = pk.seg_gates;
        a.n_slots = pk.n_slots;
        a.theta = theta;
        a.nlookups = pk.NL;
        a.nshuffles = pk.NS;
        a.lookups = w.sub[i].lookups;
        a.shuffles = w.sub[i].shuffles;
        a.consts = pk.consts;
        a.query_col = w.sub[i].load_col;
        a.query_rot = pk.d_load_rot;
        a.nsets = pk.nsets;
        a.chunk_len = pk.chunk_len;
        a.P = pk.P;
        a.z = w.sub[i].z;
        a.perm_v = w.sub[i].perm_v;
        a.sigma = pk.d_sigma_sub[i];
        a.l0 = pk.sub_l0 + i * n;
        a.l_last = pk.sub_ll + i * n;
        a.l_active = pk.sub_la + i * n;
        a.beta = beta;
        a.gamma = gamma;
        a.y = y;
        a.delta_start = beta * zeta() * pow_u64(D.ext_omega, t);  // X = zeta w_ext^t w^m
        a.delta = fr_delta();
        a.ext_omega = pk.om;
        a.ext = n;
        a.rot_scale = 1;
        a.last_rot = -(bf + 1);
        a.t_evals = D.d_t + t;  // t(X) is constant on a sub-coset
        a.t_mask = 0;
        a.acc_in = ci > 0 ? slot : nullptr;
        a.divide = ci + 1 == ncirc;
        a.out = slot;
        if (pieces) {  // this rank's rows of the sub-coset
          a.row0 = pk.sub_lo;
          a.rows = pk.sub_hi - pk.sub_lo;
        }
        HIPCHK(evaluate_h(a, st));
      }
    }
    if (h_slabs) {
      if (pieces) RCCHK(h_gather_pieces(pk, st));
      RCCHK(h_by_slabs(d, pk, sl, st));
    } else {
      HIPCHK(hipStreamSynchronize(st));
      for (uint64_t t = 0; t < (1ull << e); t++)
        if (spmd_timed(3, n * sizeof(Fr), [&] {
              return g_spmd.bcast(g_spmd.ctx, pk.h_gather + t * n, n * sizeof(Fr), (int)(t % (uint64_t)g_spmd.world));
            }) != 0)
          return fail(H2G_ERR_STATE, "spmd transport: broadcast of sub-coset " + std::to_string(t) + " failed");
      HIPCHK(subcoset_scatter(pk.h_gather, pk.h_ext, n, e, st));
    }
  }
  if (!h_slabs) dump("h_ext", pk.h_ext, ext, st);
  clk.mark("evaluate_h");
  // ---- vanishing construct (vanishing/prover.rs:102-155): h(X) pieces of size n (a rank
  // that received h by slabs holds its slab of each piece already)
  if (!h_slabs) RCCHK(extended_to_coeff(d, D, pk.h_ext, pk.h_coeff, st));
  const int npieces = pk.degree - 1;
  for (int p = 0; p < npieces; p++) (void)rng.random_fr();  // h blinds
  RCCHK(rng_ok());
  {
    std::vector<MsmTicket> tk(npieces);
    std::vector<const Fr*> pieces(npieces);
    for (int p = 0; p < npieces; p++) pieces[p] = pk.h_coeff + (size_t)p * n;
    RCCHK(commit_launch_batch(d, prm, pieces.data(), npieces, n, SRS_G, st, tk.data()));
    std::vector<MsmTicket*> tl;
    for (int p = 0; p < npieces; p++) tl.push_back(&tk[p]);
    RCCHK(collect_write(tl));
  }
  clk.mark("h commit");
  const Fr x = tr.squeeze();
  const Fr xn = pow_u64(x, n);
  // h(X) = sum_p X^(n p) h_p(X)  (vanishing/prover.rs:166-170)
  {
    LinTerms t;
    Fr c = Fr::one();
    bool first = true;
    for (int p = 0; p < npieces; p++) {
      if (t.k == LIN_MAXT) {
        RCCHK(lincomb_range(pk.h_poly, sl.lo, sl.hi1, t, !first, st));  // a slab rank: its slab + halo
        first = false;
        t.k = 0;
      }
      t.p[t.k] = pk.h_coeff + (size_t)p * n;
      t.len[t.k] = n;
      t.coef[t.k] = c;
      t.k++;
      c = c * xn;
    }
    RCCHK(lincomb_range(pk.h_poly, sl.lo, sl.hi1, t, !first, st));
  }

  // ---- the polynomial openings (prover.rs:840-889) and their evaluations
  // poly ids: per circuit ci (base ci * per_c): advice c, z s, lookup l (z, A', S'),
  // shuffle s; then fixed, sigma, h, random
  const int per_c = pk.A + pk.nsets + 3 * pk.NL + pk.NS;
  auto id_adv = [&](int ci) { return ci * per_c; };
  auto id_z = [&](int ci) { return ci * per_c + pk.A; };
  auto id_lk = [&](int ci) { return ci * per_c + pk.A + pk.nsets; };  // lookup l: z, A', S' at + 3 l
  auto id_sh = [&](int ci) { return ci * per_c + pk.A + pk.nsets + 3 * pk.NL; };
  std::vector<PolyRef> polys;
  for (const CircuitWs* w : W) {
    for (int c = 0; c < pk.A; c++) polys.push_back({w->adv_poly[c], n});
    for (int s = 0; s < pk.nsets; s++) polys.push_back({w->z[s], n});
    for (int l = 0; l < pk.NL; l++) {
      polys.push_back({w->lk_z_poly[l], n});
      polys.push_back({w->lk_ap_poly[l], n});
      polys.push_back({w->lk_sp_poly[l], n});
    }
    for (int s = 0; s < pk.NS; s++) polys.push_back({w->sh_z_poly[s], n});
  }
  const int id_fix = (int)polys.size();
  if (coef_send || coef_recv) {  // the per-circuit coefficient columns' slabs, owners -> the others
    std::vector<Fr*> cols;     // (the columns of wide stages reached every rank from their owners)
    for (int ci = 0; ci < ncirc; ci++)
      for (int i = 0; i < per_c; i++) {
        if (i < pk.A && adv_shard[(size_t)ci * pk.A + i]) continue;
        if (lk_shard && i >= pk.A + pk.nsets && i < pk.A + pk.nsets + 3 * pk.NL) continue;
        cols.push_back(const_cast<Fr*>(polys[(size_t)ci * per_c + i].p));
      }
    RCCHK(coef_exchange(pk, cols, st));
  }
  for (int c = 0; c < pk.F; c++) polys.push_back({pk.fixed_poly[c], n});
  const int id_sig = (int)polys.size();
  for (int c = 0; c < pk.P; c++) polys.push_back({pk.sigma_poly[c], n});
  const int id_h = (int)polys.size();
  polys.push_back({pk.h_poly, n});
  const int id_r = (int)polys.size();
  polys.push_back({pk.random_poly, n});
  const Fr x_next = rotate_omega(D, x, 1), x_last = rotate_omega(D, x, -(bf + 1));
  const Fr x_prev = rotate_omega(D, x, -1);
  struct Q2 {
    int poly;
    Fr pt;
  };
  std::vector<Q2> queries;
  for (int ci = 0; ci < ncirc; ci++) {  // per circuit: advice, permutation, lookups, shuffles
    for (auto& q : pk.adv_q) queries.push_back({id_adv(ci) + q.index, rotate_omega(D, x, q.rot)});
    for (int s = 0; s < pk.nsets; s++) {  // permutation/prover.rs:300-333
      queries.push_back({id_z(ci) + s, x});
      queries.push_back({id_z(ci) + s, x_next});
    }
    for (int s = pk.nsets - 2; s >= 0; s--) queries.push_back({id_z(ci) + s, x_last});
    for (int l = 0; l < pk.NL; l++) {  // lookup/prover.rs:364-405
      const int zi = id_lk(ci) + 3 * l;
      queries.push_back({zi, x});
      queries.push_back({zi + 1, x});
      queries.push_back({zi + 2, x});
      queries.push_back({zi + 1, x_prev});
      queries.push_back({zi, x_next});
    }
    for (int s = 0; s < pk.NS; s++) {  // shuffle/prover.rs:234-254
      queries.push_back({id_sh(ci) + s, x});
      queries.push_back({id_sh(ci) + s, x_next});
    }
  }
  for (auto& q : pk.fix_q) queries.push_back({id_fix + q.index, rotate_omega(D, x, q.rot)});
  for (int c = 0; c < pk.P; c++) queries.push_back({id_sig + c, x});
  queries.push_back({id_h, x});
  queries.push_back({id_r, x});
  // unique (poly, point) evaluations, one batched launch
  std::vector<Q2> ev_keys;
  std::vector<std::vector<int>> ev_of(polys.size());  // per polynomial its ev_keys entries (a few points)
  auto ev_index = [&](int poly, const Fr& pt) -> int {
    if ((size_t)poly >= ev_of.size()) ev_of.resize((size_t)poly + 1);
    for (int i : ev_of[poly])
      if (ev_keys[i].pt == pt) return i;
    ev_keys.push_back({poly, pt});
    ev_of[poly].push_back((int)ev_keys.size() - 1);
    return (int)ev_keys.size() - 1;
  };
  for (auto& q : queries) ev_index(q.poly, q.pt);
  std::vector<Fr> evals(ev_keys.size());
  {
    const int nreq = (int)ev_keys.size();
    if (nreq > pk.max_reqs) {
      PALLOC(pk.pool, pk.d_reqs, nreq);
      PALLOC(pk.pool, pk.evals, nreq);
      pk.max_reqs = nreq;
    }
    const size_t need = poly_eval_scratch_len(nreq, n);
    if (need > pk.eval_scr_len) {
      PALLOC(pk.pool, pk.eval_scr, need);
      pk.eval_scr_len = need;
    }
    std::vector<EvalReq> reqs(nreq);
    for (int i = 0; i < nreq; i++) {  // a slab rank evaluates its coefficients [lo, hi) only
      const PolyRef& pr = polys[ev_keys[i].poly];
      const uint64_t len = pr.len > sl.lo ? std::min<uint64_t>(pr.len, sl.hi) - sl.lo : 0;
      reqs[i] = EvalReq{pr.p + (len ? sl.lo : 0), len, ev_keys[i].pt};
    }
    HIPCHK(pk_upload(pk, pk.d_reqs, reqs.data(), nreq * sizeof(EvalReq), st));
    HIPCHK(poly_eval_batch(pk.d_reqs, nreq, sl.hi - sl.lo, pk.evals, pk.eval_scr, st));
    HIPCHK(hipMemcpyAsync(evals.data(), pk.evals, nreq * sizeof(Fr), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (slabs) {  // p(x) = sum_r x^lo_r (slab r's partial evaluation), summed in rank order
      std::vector<std::pair<Fr, Fr>> shift;  // (point, point^lo): a few distinct points
      for (int i = 0; i < nreq; i++) {
        const Fr& pt = ev_keys[i].pt;
        size_t j = 0;
        while (j < shift.size() && !(shift[j].first == pt)) j++;
        if (j == shift.size()) shift.emplace_back(pt, pow_u64(pt, sl.lo));
        evals[i] = evals[i] * shift[j].second;
      }
      std::vector<Fr> all;
      RCCHK(spmd_allgather_fr(evals, &all));
      for (int i = 0; i < nreq; i++) {
        Fr acc = Fr::zero();
        for (int r = 0; r < g_spmd.world; r++) acc = acc + all[(size_t)r * nreq + i];
        evals[i] = acc;
      }
    }
  }
  auto ev = [&](int poly, const Fr& pt) { return evals[ev_index(poly, pt)]; };
  for (int ci = 0; ci < ncirc; ci++)  // [TRANSCRIPT-17] every circuit's advice evaluations
    for (auto& q : pk.adv_q) tr.write_scalar(ev(id_adv(ci) + q.index, rotate_omega(D, x, q.rot)));
  for (auto& q : pk.fix_q) tr.write_scalar(ev(id_fix + q.index, rotate_omega(D, x, q.rot)));
  tr.write_scalar(ev(id_r, x));
  for (int c = 0; c < pk.P; c++) tr.write_scalar(ev(id_sig + c, x));
  for (int ci = 0; ci < ncirc; ci++)
    for (int s = 0; s < pk.nsets; s++) {
      tr.write_scalar(ev(id_z(ci) + s, x));
      tr.write_scalar(ev(id_z(ci) + s, x_next));
      if (s + 1 < pk.nsets) tr.write_scalar(ev(id_z(ci) + s, x_last));
    }
  for (int ci = 0; ci < ncirc; ci++)
    for (int l = 0; l < pk.NL; l++) {  // product, product_next, A', A'_inv, S' (lookup/prover.rs:330-361)
      const int zi = id_lk(ci) + 3 * l;
      tr.write_scalar(ev(zi, x));
      tr.write_scalar(ev(zi, x_next));
      tr.write_scalar(ev(zi + 1, x));
      tr.write_scalar(ev(zi + 1, x_prev));
      tr.write_scalar(ev(zi + 2, x));
    }
  for (int ci = 0; ci < ncirc; ci++)
    for (int s = 0; s < pk.NS; s++) {
      tr.write_scalar(ev(id_sh(ci) + s, x));
      tr.write_scalar(ev(id_sh(ci) + s, x_next));
    }
  clk.mark("evaluations");

  if (pk.multiopen == 1) {
    // ---- ProverGWC::create_proof_with_engine (gwc/prover.rs:40-90): the queries grouped
    // by point in first-appearance order (construct_intermediate_sets, gwc.rs:25-50); per
    // point W(X) = (sum_i v^i p_i(X) - sum_i v^i p_i(z)) / (X - z), committed against g.
    // The points' MSMs are independent, so all are launched before the first is collected.
    const Fr v = tr.squeeze();
    std::vector<char> done(queries.size(), 0);
    std::vector<MsmTicket> tk;
    std::vector<Fr> neg_evb;
    neg_evb.reserve(queries.size());
    for (size_t i = 0; i < queries.size(); i++) {
      if (done[i]) continue;
      const Fr z = queries[i].pt;
      const size_t g = tk.size();
      if (g >= pk.gwc_q.size()) {
        Fr* q;
        PALLOC(pk.pool, q, n);
        pk.gwc_q.push_back(q);
      }
      LinTerms t;
      bool first = true;
      Fr vp = Fr::one(), evb = Fr::zero();
      for (size_t j = i; j < queries.size(); j++) {
        if (done[j] || queries[j].pt != z) continue;
        done[j] = 1;
        if (t.k == LIN_MAXT - 1) {
          HIPCHK(lincomb(pk.nx, n, t, !first, st));
          first = false;
          t.k = 0;
        }
        t.p[t.k] = polys[queries[j].poly].p;
        t.len[t.k] = polys[queries[j].poly].len;
        t.coef[t.k] = vp;
        t.k++;
        evb = evb + vp * ev(queries[j].poly, z);
        vp = vp * v;
      }
      neg_evb.push_back(Fr::zero() - evb);  // poly_batch - eval_batch (poly.rs:268-276)
      HIPCHK(pk_upload(pk, pk.small + g, &neg_evb.back(), sizeof(Fr), st));
      t.p[t.k] = pk.small + g;
      t.len[t.k] = 1;
      t.coef[t.k] = Fr::one();
      t.k++;
      HIPCHK(lincomb(pk.nx, n, t, !first, st));
      HIPCHK(kate_division(pk.nx, n, z, pk.gwc_q[g], pk.scr, st));
      tk.emplace_back();
      RCCHK(commit_launch(d, prm, pk.gwc_q[g], n - 1, SRS_G, st, &tk.back()));  // commit (kzg/commitment.rs:354-366)
    }
    {
      std::vector<MsmTicket*> tl;
      for (auto& t : tk) tl.push_back(&t);
      RCCHK(collect_write(tl));
    }
    HIPCHK(hipStreamSynchronize(st));  // neg_evb (host) is read by the copies above
    clk.mark("gwc");
    return H2G_OK;
  }

  // ---- SHPLONK (shplonk/prover.rs:121-305; construct_intermediate_sets shplonk.rs:48-140)
  // host values the device copies read asynchronously (live until the proof returns)
  std::vector<std::vector<Fr>> corr_stage;
  Fr c0_stage;
  StreamSyncGuard corr_guard{st};
  const Fr sy = tr.squeeze();
  std::vector<Fr> super_pts;
  for (auto& q : queries) {
    bool f = false;
    for (auto& p : super_pts) f = f || p == q.pt;
    if (!f) super_pts.push_back(q.pt);
  }
  std::sort(super_pts.begin(), super_pts.end(), [](const Fr& a, const Fr& b) { return fr_cmp(a, b) < 0; });
  std::vector<int> cm_ids;
  std::vector<std::vector<Fr>> cm_pts;
  for (auto& q : queries) {
    int f = -1;
    for (size_t i = 0; i < cm_ids.size(); i++)
      if (cm_ids[i] == q.poly) f = (int)i;
    if (f < 0) {
      f = (int)cm_ids.size();
      cm_ids.push_back(q.poly);
      cm_pts.emplace_back();
    }
    auto& ps = cm_pts[f];
    if (std::find(ps.begin(), ps.end(), q.pt) == ps.end()) ps.push_back(q.pt);
  }
  for (auto& ps : cm_pts) std::sort(ps.begin(), ps.end(), [](const Fr& a, const Fr& b) { return fr_cmp(a, b) < 0; });
  std::vector<int> rs_of(cm_ids.size()), rs_rep;
  for (size_t c = 0; c < cm_ids.size(); c++) {
    int f = -1;
    for (size_t r = 0; r < rs_rep.size(); r++)
      if (cm_pts[rs_rep[r]] == cm_pts[c]) f = (int)r;
    if (f < 0) {
      f = (int)rs_rep.size();
      rs_rep.push_back((int)c);
    }
    rs_of[c] = f;
  }
  // r_c: the interpolation through c's evaluations, from its rotation set's Lagrange basis
  // (one set of inversions per set, not per commitment)
  std::vector<std::vector<std::vector<Fr>>> basis(rs_rep.size());
  for (size_t r = 0; r < rs_rep.size(); r++) basis[r] = lagrange_basis(cm_pts[rs_rep[r]]);
  std::vector<std::vector<Fr>> low(cm_ids.size());
  for (size_t c = 0; c < cm_ids.size(); c++) {
    const auto& B = basis[rs_of[c]];
    const size_t m = cm_pts[c].size();
    low[c].assign(m, Fr::zero());
    for (size_t j = 0; j < m; j++) {
      const Fr e = ev(cm_ids[c], cm_pts[c][j]);
      for (size_t i = 0; i < m; i++) low[c][i] = low[c][i] + B[j][i] * e;
    }
  }
  const Fr v = tr.squeeze();
  // h_x = sum_s v^s (sum_i y^i (p_i - r_i)) / Z_s (the reference divides by Z_s with one
  // kate division per point of S_s, shplonk/prover.rs:142-176).  Partial fractions instead:
  // 1 / Z_s = sum_{p in S_s} c_{s,p} / (X - p) with c_{s,p} = prod_{p' in S_s \ p} (p - p')^-1,
  // and (g_s - r_s) / (X - p) is exact for every p in S_s, so with
  // G_p = sum_{s : p in S_s} v^s c_{s,p} (g_s - r_s), h_x = sum_p G_p / (X - p): one kate
  // division per distinct point (accumulated into h_x) instead of one per (set, point).
  // Exact field arithmetic, so h_x is the same polynomial.
  {
    std::vector<Fr> vpow(rs_rep.size()), ypow(cm_ids.size());
    {
      Fr vp = Fr::one();
      for (size_t r = 0; r < rs_rep.size(); r++) {
        vpow[r] = vp;
        vp = vp * v;
        Fr yp = Fr::one();
        for (size_t c = 0; c < cm_ids.size(); c++)
          if (rs_of[c] == (int)r) {
            ypow[c] = yp;
            yp = yp * sy;
          }
      }
    }
    // slab mode: per point a (slab + halo) buffer; gbuf(i) indexes it globally
    const size_t np = super_pts.size(), cap = sl.hi1 - sl.lo + 1;
    if (slabs && np * cap > pk.slab_buf_len) {
      PALLOC(pk.pool, pk.slab_buf, np * cap);
      pk.slab_buf_len = np * cap;
    }
    auto gbuf = [&](size_t i) { return pk.slab_buf + i * cap - sl.lo; };
    if (slabs) HIPCHK(hipMemsetAsync(pk.hx + sl.lo, 0, (sl.hi1 - sl.lo) * sizeof(Fr), st));
    else HIPCHK(hipMemsetAsync(pk.hx, 0, n * sizeof(Fr), st));
    for (size_t pi = 0; pi < np; pi++) {
      const Fr& p = super_pts[pi];
      Fr* gp = slabs ? gbuf(pi) : pk.nx;
      // alpha_s = v^s c_{s,p} for the sets containing p
      std::vector<Fr> alpha(rs_rep.size(), Fr::zero());
      std::vector<char> has(rs_rep.size(), 0);
      size_t ncorr = 0;
      for (size_t r = 0; r < rs_rep.size(); r++) {
        const std::vector<Fr>& pts = cm_pts[rs_rep[r]];
        if (std::find(pts.begin(), pts.end(), p) == pts.end()) continue;
        Fr den = Fr::one();
        for (const Fr& q : pts)
          if (!(q == p)) den = den * (p - q);
        alpha[r] = vpow[r] * inv(den);
        has[r] = 1;
        ncorr = std::max(ncorr, pts.size());
      }
      corr_stage.emplace_back(ncorr, Fr::zero());  // read by an async copy
      std::vector<Fr>& corr = corr_stage.back();
      LinTerms t;
      bool first = true;
      for (size_t c = 0; c < cm_ids.size(); c++) {
        const int r = rs_of[c];
        if (!has[r]) continue;
        if (t.k == LIN_MAXT - 1) {
          RCCHK(lincomb_range(gp, sl.lo, sl.hi1, t, !first, st));
          first = false;
          t.k = 0;
        }
        const Fr coef = alpha[r] * ypow[c];
        t.p[t.k] = polys[cm_ids[c]].p;
        t.len[t.k] = polys[cm_ids[c]].len;
        t.coef[t.k] = coef;
        t.k++;
        for (size_t j = 0; j < low[c].size(); j++) corr[j] = corr[j] + coef * low[c][j];
      }
      HIPCHK(pk_upload(pk, pk.small, corr.data(), corr.size() * sizeof(Fr), st));
      t.p[t.k] = pk.small;
      t.len[t.k] = corr.size();
      t.coef[t.k] = fr_neg_one();
      t.k++;
      RCCHK(lincomb_range(gp, sl.lo, sl.hi1, t, !first, st));
      if (!slabs) HIPCHK(kate_division(pk.nx, n, p, pk.hx, pk.scr, st, true));
    }
    if (slabs) {
      // G_p / (X - p) on slabs: q[i] = sum_{j >= i} a[j + 1] p^(j - i).  The slab's own part
      // plus p^(hi' - i) C, with C = q[hi'] the quotient just above the slab = sum over the
      // higher slabs of their partial Horner values E_s (one all-gather for every point);
      // C enters as p C added to a[hi'], so the division runs unchanged on the slab.
      std::vector<Fr> carry;
      RCCHK(slab_carries(pk, sl, n, super_pts, [&](size_t i) { return gbuf(i); }, &carry, st));
      Fr halo = Fr::zero();
      for (size_t pi = 0; pi < np; pi++) {
        const size_t hq = std::min(sl.hi, n - 1);
        if (hq <= sl.lo) continue;
        HIPCHK(poly_binop(POLY_ADD_CONST, gbuf(pi) + hq, nullptr, super_pts[pi] * carry[pi], gbuf(pi) + hq, 1, st));
        HIPCHK(kate_division(gbuf(pi) + sl.lo, hq - sl.lo + 1, super_pts[pi], pk.hx + sl.lo, pk.scr, st, true));
        halo = halo + carry[pi];
      }
      if (sl.hi < n) {  // h_x's halo coefficient (read by the linearisation): q[hi] = sum of the carries
        corr_stage.emplace_back(1, halo);
        HIPCHK(pk_upload(pk, pk.hx + sl.hi, corr_stage.back().data(), sizeof(Fr), st));
      }
    }
  }
  {
    G1Affine cm;
    RCCHK(commit(d, prm, pk.hx, n, SRS_G, &cm, st));
    RCCHK(write_point(cm));
  }
  clk.mark("shplonk h");
  const Fr u = tr.squeeze();
  // linearisation: l_x = sum_s v^s Z_{T\S_s}(u) sum_i y^i (p_i - r_i(u)) - Z_T(u) h_x
  Fr z0 = Fr::one();
  {
    Fr vpow = Fr::one(), c0 = Fr::zero();
    LinTerms t;
    bool first = true;
    auto flush = [&]() -> int {
      RCCHK(lincomb_range(pk.lx, sl.lo, sl.hi1, t, !first, st));  // a slab rank: slab + halo
      first = false;
      t.k = 0;
      return H2G_OK;
    };
    for (size_t r = 0; r < rs_rep.size(); r++) {
      const std::vector<Fr>& pts = cm_pts[rs_rep[r]];
      Fr zi = Fr::one();
      for (auto& sp : super_pts)
        if (std::find(pts.begin(), pts.end(), sp) == pts.end()) zi = (u - sp) * zi;
      if (r == 0) z0 = zi;
      Fr ypow = Fr::one();
      for (size_t c = 0; c < cm_ids.size(); c++) {
        if (rs_of[c] != (int)r) continue;
        if (t.k == LIN_MAXT - 2) RCCHK(flush());
        const Fr coef = ypow * zi * vpow;
        t.p[t.k] = polys[cm_ids[c]].p;
        t.len[t.k] = polys[cm_ids[c]].len;
        t.coef[t.k] = coef;
        t.k++;
        c0 = c0 - coef * eval_host(low[c], u);
        ypow = ypow * sy;
      }
      vpow = vpow * v;
    }
    Fr zt = Fr::one();
    for (auto& sp : super_pts) zt = (u - sp) * zt;
    c0_stage = c0;
    HIPCHK(pk_upload(pk, pk.small, &c0_stage, sizeof(Fr), st));
    t.p[t.k] = pk.small;
    t.len[t.k] = 1;
    t.coef[t.k] = Fr::one();
    t.k++;
    t.p[t.k] = pk.hx;
    t.len[t.k] = n;
    t.coef[t.k] = Fr::zero() - zt;
    t.k++;
    RCCHK(flush());
  }
  if (slabs) {  // the same slab division by (X - u), one carry
    std::vector<Fr> carry;
    const std::vector<Fr> pts{u};
    RCCHK(slab_carries(pk, sl, n, pts, [&](size_t) { return pk.lx; }, &carry, st));
    const size_t hq = std::min(sl.hi, n - 1);
    if (hq > sl.lo) {
      HIPCHK(poly_binop(POLY_ADD_CONST, pk.lx + hq, nullptr, u * carry[0], pk.lx + hq, 1, st));
      HIPCHK(kate_division(pk.lx + sl.lo, hq - sl.lo + 1, u, pk.q1 + sl.lo, pk.scr, st));
      HIPCHK(poly_binop(POLY_SCALE, pk.q1 + sl.lo, nullptr, inv(z0), pk.q1 + sl.lo, hq - sl.lo, st));
    }
  } else {
    HIPCHK(kate_division(pk.lx, n, u, pk.q1, pk.scr, st));
    HIPCHK(poly_binop(POLY_SCALE, pk.q1, nullptr, inv(z0), pk.q1, n - 1, st));
  }
  {
    G1Affine cm;
    RCCHK(commit(d, prm, pk.q1, n - 1, SRS_G, &cm, st));
    RCCHK(write_point(cm));
  }
  clk.mark("shplonk final");
  return H2G_OK;
}

}  // namespace

#define NEED_DEV_P()                                                          \
  std::lock_guard<std::recursive_mutex> _lk(g_mu);                            \
  Device* d = cur();                                                          \
  if (!d) return fail(H2G_ERR_STATE, "h2g_init has not been called");         \
  HIPCHK(hipSetDevice(d->id));

extern "C" {

int h2g_params_create(uint32_t k, const uint64_t* g, const uint64_t* g_lagrange, uint64_t* handle) {
  NEED_DEV_P();
  if (!g || !g_lagrange || !handle || k > 27) return fail(H2G_ERR_ARG, "params_create: bad arguments");
  auto p = std::make_unique<Params>();
  p->device = d->id;
  p->k = k;
  p->n = (size_t)1 << k;
  PALLOC(p->pool, p->g, p->n);
  PALLOC(p->pool, p->gl, p->n);
  HIPCHK(hipMemcpy(p->g, g, p->n * sizeof(G1Affine), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(p->gl, g_lagrange, p->n * sizeof(G1Affine), hipMemcpyHostToDevice));
  RCCHK(params_finish(*p, d->stream));
  *handle = g_next_handle++;
  g_params[*handle] = std::move(p);
  return H2G_OK;
}

int h2g_params_setup(uint32_t k, const uint64_t s_limbs[4], uint64_t* handle) {
  NEED_DEV_P();
  if (!s_limbs || !handle || k > 27) return fail(H2G_ERR_ARG, "params_setup: bad arguments");
  hipStream_t st = d->stream;
  auto p = std::make_unique<Params>();
  p->device = d->id;
  p->k = k;
  p->n = (size_t)1 << k;
  const size_t n = p->n;
  PALLOC(p->pool, p->g, n);
  PALLOC(p->pool, p->gl, n);
  const Fr s = fr_from_limbs(s_limbs);
  HIPCHK(srs_setup(s, n, p->g, st));
  Fr omega = root_of_unity();
  for (uint32_t i = k; i < FR_S; i++) omega = sqr(omega);
  Pool tmp;
  PowTable om;
  RCCHK(build_pow_table(tmp, omega, (int)k, &om, st));
  Fr *sc, *scr;
  HIPCHK(tmp.get((void**)&sc, n * sizeof(Fr)));
  HIPCHK(tmp.get((void**)&scr, n * sizeof(Fr)));
  const Fr mult = (pow_u64(s, n) - Fr::one()) * inv(from_u64<FrParams>(n));
  HIPCHK(srs_lagrange_scalars(sc, n, s, mult, om, scr, st));
  HIPCHK(g1_generator_mul(sc, n, p->gl, st));
  HIPCHK(hipStreamSynchronize(st));
  RCCHK(params_finish(*p, st));
  // g2 = generator, s_g2 = [s] g2 (kzg/commitment.rs:122-123)
  p->g2 = g2_generator();
  const Fr s_can = to_canonical(s);
  p->s_g2 = g2_mul(p->g2, s_can.l);
  p->has_g2 = true;
  *handle = g_next_handle++;
  g_params[*handle] = std::move(p);
  return H2G_OK;
}

int h2g_params_export(uint64_t params, uint64_t* g, uint64_t* g_lagrange) {
  NEED_DEV_P();
  auto it = g_params.find(params);
  if (it == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (g) HIPCHK(hipMemcpy(g, it->second->g, it->second->n * sizeof(G1Affine), hipMemcpyDeviceToHost));
  if (g_lagrange) HIPCHK(hipMemcpy(g_lagrange, it->second->gl, it->second->n * sizeof(G1Affine), hipMemcpyDeviceToHost));
  return H2G_OK;
}

int h2g_params_free(uint64_t params) {
  NEED_DEV_P();
  if (!g_params.erase(params)) return fail(H2G_ERR_HANDLE, "unknown params");
  return H2G_OK;
}

int h2g_keygen(uint64_t params, const h2g_circuit* circuit, uint64_t* pk_out) {
  NEED_DEV_P();
  auto it = g_params.find(params);
  if (it == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (!circuit || !pk_out) return fail(H2G_ERR_ARG, "keygen: null argument");
  auto pk = std::make_unique<ProvingKey>();
  pk->params = params;
  int rc = keygen_impl(d, *it->second, circuit, *pk);
  // the lookup commitments' basis (params_prefix) now, not inside the first proof
  if (!rc && circuit->num_lookups > 0 && H2G_LOOKUP_PREFIX) rc = params_prefix(*it->second, d->stream);
  if (rc) {
    domain_release(&pk->dom);
    return rc;
  }
  *pk_out = g_next_handle++;
  g_pks[*pk_out] = std::move(pk);
  return H2G_OK;
}

// ------------------------------------------------------------------ serialisation
// SerdeFormat (halo2_backend/src/helpers.rs:8-21): 0 Processed, 1 RawBytes,
// 2 RawBytesUnchecked.  RawBytes writes points uncompressed and field elements as their
// Montgomery limbs -- the device layout, so arrays move with one copy -- and on read
// checks that every element is below its modulus and every point is on its curve (on
// the device for the n-sized arrays).  Processed (compressed points, canonical field
// elements) is refused: halo2curves' compressed-point flag bits cannot be pinned here.
}  // extern "C"

namespace {
enum { SERDE_PROCESSED = 0, SERDE_RAW = 1, SERDE_RAW_UNCHECKED = 2 };
constexpr uint8_t PK_VERSION = 0x04;  // plonk.rs:58

struct DevScratch {
  void* p = nullptr;
  ~DevScratch() {
    if (p) (void)hipFree(p);
  }
};
// GroupEncoding::to_bytes / from_bytes of one G1 point on the host (the VK's commitments);
// the device form for whole arrays is g1_compress / g1_decompress (serde.hip)
void g1_compress_host(const G1Affine& a, uint8_t c[32]) {
  Fq x = Fq::zero();
  if (!a.is_identity()) {
    x = to_canonical(a.x);
    x.l[7] |= (to_canonical(a.y).l[0] & 1u) << 31;
  }
  std::memcpy(c, x.l, 32);
}
bool g1_decompress_host(const uint8_t c[32], G1Affine* out) {
  static constexpr uint32_t SQRT_EXP[8] = {0xb61f3f52u, 0x4f082305u, 0x5a1c72a3u, 0x65e05aa4u,
                                           0xa0605617u, 0x6e14116du, 0xb84c680au, 0x0c19139cu};  // (p+1)/4
  Fq x;
  std::memcpy(x.l, c, 32);
  const uint32_t ysign = x.l[7] >> 31;
  x.l[7] &= 0x7fffffffu;
  unsigned br = 0;
  for (int i = 0; i < 8; i++) (void)__builtin_subc(x.l[i], FqParams::M[i], br, &br);
  if (!br) return false;  // x >= p
  out->x = out->y = Fq::zero();
  if (x.is_zero() && !ysign) return true;  // identity
  const Fq xm = from_canonical(x);
  const Fq y2 = sqr(xm) * xm + from_u64<FqParams>(3);
  Fq y = pow_limbs(y2, SQRT_EXP);
  if (sqr(y) != y2) return false;
  if ((to_canonical(y).l[0] & 1u) != ysign) y = neg(y);
  out->x = xm;
  out->y = y;
  return true;
}

struct ByteWriter {  // out == NULL: count only
  uint8_t* out;
  size_t cap;
  // the library stream the arrays were produced on: copies and conversions queue behind
  // its work (it is non-blocking, so the NULL stream would not order with it)
  hipStream_t st;
  size_t len = 0;
  bool fits(size_t k) const { return out && len + k <= cap; }
  void put(const void* p, size_t k) {
    if (fits(k)) std::memcpy(out + len, p, k);
    len += k;
  }
  void u8(uint8_t v) { put(&v, 1); }
  void u32le(uint32_t v) { put(&v, 4); }
  void u32be(uint32_t v) {
    const uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    put(b, 4);
  }
  bool proc = false;  // SerdeFormat::Processed: compressed points, canonical field elements
  int dev(const void* d, size_t k) {  // device bytes
    if (fits(k)) {
      HIPCHK(hipMemcpyAsync(out + len, d, k, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    len += k;
    return H2G_OK;
  }
  // `cnt` elements converted on the device into a scratch array of `k` bytes, then copied
  template <class Conv>
  int dev_conv(size_t k, Conv conv) {
    if (fits(k)) {
      DevScratch t;
      HIPCHK(hipMalloc(&t.p, k));
      HIPCHK(conv(t.p));
      HIPCHK(hipMemcpyAsync(out + len, t.p, k, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    len += k;
    return H2G_OK;
  }
  int g1s(const G1Affine* d, size_t cnt) {  // SerdeCurveAffine::write of cnt device points
    if (!proc) return dev(d, cnt * sizeof(G1Affine));
    return dev_conv(cnt * 32, [&](void* t) { return g1_compress(d, cnt, (uint8_t*)t, st); });
  }
  void g1(const G1Affine& a) {
    if (!proc) return put(&a, sizeof(G1Affine));
    uint8_t c[32];
    g1_compress_host(a, c);
    put(c, 32);
  }
  void g2(const G2Affine& a) {
    if (!proc) return put(&a, sizeof(G2Affine));
    uint8_t c[64];
    g2_compress(a, c);
    put(c, 64);
  }
  int poly(const Fr* d, size_t cnt) {  // Polynomial::write (poly.rs:187-197)
    u32be((uint32_t)cnt);
    if (!proc) return dev(d, cnt * sizeof(Fr));
    return dev_conv(cnt * sizeof(Fr), [&](void* t) { return fr_to_repr(d, cnt, (Fr*)t, st); });
  }
  int polys(const std::vector<Fr*>& v, size_t cnt) {  // write_polynomial_slice (helpers.rs:119-129)
    u32be((uint32_t)v.size());
    for (const Fr* p : v) RCCHK(poly(p, cnt));
    return H2G_OK;
  }
};

struct ByteReader {
  const uint8_t* p;
  size_t len, pos = 0;
  bool ok = true;
  const uint8_t* take(size_t k) {
    if (!ok || pos + k > len) {
      ok = false;
      return nullptr;
    }
    const uint8_t* r = p + pos;
    pos += k;
    return r;
  }
  uint8_t u8() {
    const uint8_t* b = take(1);
    return b ? b[0] : 0;
  }
  uint32_t u32le() {
    const uint8_t* b = take(4);
    return b ? (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24 : 0;
  }
  uint32_t u32be() {
    const uint8_t* b = take(4);
    return b ? (uint32_t)b[3] | (uint32_t)b[2] << 8 | (uint32_t)b[1] << 16 | (uint32_t)b[0] << 24 : 0;
  }
  // one polynomial of exactly `cnt` elements (read_polynomial_vec / Polynomial::read)
  const uint8_t* poly(size_t cnt) {
    if (u32be() != cnt) ok = false;
    return take(cnt * sizeof(Fr));
  }
  bool polys(std::vector<const uint8_t*>& v, size_t count, size_t cnt) {
    if (u32be() != count) return ok = false;
    v.resize(count);
    for (auto& q : v) q = poly(cnt);
    return ok;
  }
};

bool fq_below(const Fq& a) {
  unsigned br = 0;
  for (int i = 0; i < 8; i++) (void)__builtin_subc(a.l[i], FqParams::M[i], br, &br);
  return br != 0;
}
bool g2_valid(const G2Affine& a) {
  return fq_below(a.x.c0) && fq_below(a.x.c1) && fq_below(a.y.c0) && fq_below(a.y.c1) && g2_on_curve(a);
}
bool g1_valid_host(const G1Affine& a) {
  if (!fq_below(a.x) || !fq_below(a.y)) return false;
  return a.is_identity() || sqr(a.y) == sqr(a.x) * a.x + from_u64<FqParams>(3);
}

// device RawBytes checks of uploaded arrays: number of bad elements
int count_bad_fr(const std::vector<std::pair<const Fr*, size_t>>& arrays, hipStream_t st, uint32_t* bad_out) {
  uint32_t* bad;
  HIPCHK(hipMalloc(&bad, 4));
  HIPCHK(hipMemsetAsync(bad, 0, 4, st));
  for (const auto& a : arrays) HIPCHK(fr_count_unreduced(a.first, a.second, bad, st));
  HIPCHK(hipMemcpyAsync(bad_out, bad, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  (void)hipFree(bad);
  return H2G_OK;
}
}  // namespace

extern "C" {

/* ParamsKZG::write_custom (kzg/commitment.rs:166-181): k (u32 LE), g, g_lagrange, g2, s_g2 */
int h2g_params_write(uint64_t params, int format, uint8_t* out, size_t cap, size_t* len) {
  NEED_DEV_P();
  auto it = g_params.find(params);
  if (it == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (!len) return fail(H2G_ERR_ARG, "params_write: null length");
  if (format != SERDE_RAW && format != SERDE_RAW_UNCHECKED && format != SERDE_PROCESSED)
    return fail(H2G_ERR_ARG, "params_write: unknown SerdeFormat");
  const Params& p = *it->second;
  if (!p.has_g2) return fail(H2G_ERR_STATE, "params_write: the params have no G2 points (h2g_params_set_g2)");
  ByteWriter w{out, out ? cap : 0, d->stream};
  w.proc = format == SERDE_PROCESSED;
  w.u32le(p.k);
  RCCHK(w.g1s(p.g, p.n));
  RCCHK(w.g1s(p.gl, p.n));
  w.g2(p.g2);
  w.g2(p.s_g2);
  *len = w.len;
  if (out && w.len > cap) return fail(H2G_ERR_ARG, "params_write: buffer too small");
  return H2G_OK;
}

/* ParamsKZG::read_custom (kzg/commitment.rs:183-267) */
int h2g_params_read(const uint8_t* buf, size_t len, int format, uint64_t* handle) {
  NEED_DEV_P();
  if (!buf || !handle) return fail(H2G_ERR_ARG, "params_read: null argument");
  if (format != SERDE_RAW && format != SERDE_RAW_UNCHECKED && format != SERDE_PROCESSED)
    return fail(H2G_ERR_ARG, "params_read: unknown SerdeFormat");
  const bool proc = format == SERDE_PROCESSED;
  const size_t g1b = proc ? 32 : sizeof(G1Affine), g2b = proc ? 64 : sizeof(G2Affine);
  ByteReader r{buf, len};
  const uint32_t k = r.u32le();
  if (!r.ok || k > 27) return fail(H2G_ERR_ARG, "params_read: bad k");
  const size_t n = (size_t)1 << k;
  const uint8_t* g = r.take(n * g1b);
  const uint8_t* gl = r.take(n * g1b);
  const uint8_t* g2 = r.take(g2b);
  const uint8_t* sg2 = r.take(g2b);
  if (!r.ok) return fail(H2G_ERR_ARG, "params_read: truncated input");
  hipStream_t st = d->stream;
  auto p = std::make_unique<Params>();
  p->device = d->id;
  p->k = k;
  p->n = n;
  PALLOC(p->pool, p->g, n);
  PALLOC(p->pool, p->gl, n);
  if (proc) {  // load_points_from_file_parallelly (kzg/commitment.rs:195-213), on the device
    DevScratch t, bad;
    uint32_t nbad = 0;
    HIPCHK(hipMalloc(&t.p, 2 * n * 32));
    HIPCHK(hipMalloc(&bad.p, 4));
    HIPCHK(hipMemsetAsync(bad.p, 0, 4, st));
    HIPCHK(hipMemcpyAsync(t.p, g, n * 32, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync((uint8_t*)t.p + n * 32, gl, n * 32, hipMemcpyHostToDevice, st));
    HIPCHK(g1_decompress((const uint8_t*)t.p, n, p->g, (uint32_t*)bad.p, st));
    HIPCHK(g1_decompress((const uint8_t*)t.p + n * 32, n, p->gl, (uint32_t*)bad.p, st));
    HIPCHK(hipMemcpyAsync(&nbad, bad.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (nbad) return fail(H2G_ERR_ARG, "params_read: " + std::to_string(nbad) + " invalid point encodings");
    if (!g2_decompress(g2, &p->g2) || !g2_decompress(sg2, &p->s_g2))
      return fail(H2G_ERR_ARG, "params_read: invalid G2 point encoding");
  } else {
    HIPCHK(hipMemcpyAsync(p->g, g, n * sizeof(G1Affine), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(p->gl, gl, n * sizeof(G1Affine), hipMemcpyHostToDevice, st));
    std::memcpy(&p->g2, g2, sizeof(G2Affine));
    std::memcpy(&p->s_g2, sg2, sizeof(G2Affine));
  }
  p->has_g2 = true;
  if (format == SERDE_RAW) {
    uint32_t* bad;
    uint32_t nbad = 0;
    HIPCHK(hipMalloc(&bad, 4));
    HIPCHK(hipMemsetAsync(bad, 0, 4, st));
    HIPCHK(g1_count_invalid(p->g, n, bad, st));
    HIPCHK(g1_count_invalid(p->gl, n, bad, st));
    HIPCHK(hipMemcpyAsync(&nbad, bad, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    (void)hipFree(bad);
    if (nbad) return fail(H2G_ERR_ARG, "params_read: " + std::to_string(nbad) + " G1 points off the curve or unreduced");
    if (!g2_valid(p->g2) || !g2_valid(p->s_g2)) return fail(H2G_ERR_ARG, "params_read: invalid G2 point");
  }
  RCCHK(params_finish(*p, st));
  *handle = g_next_handle++;
  g_params[*handle] = std::move(p);
  return H2G_OK;
}

/* the G2 points of the params: 16 u64 each (x.c0, x.c1, y.c0, y.c1, Montgomery) */
int h2g_params_g2(uint64_t params, uint64_t g2[16], uint64_t s_g2[16]) {
  NEED_DEV_P();
  auto it = g_params.find(params);
  if (it == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (!it->second->has_g2) return fail(H2G_ERR_STATE, "params have no G2 points");
  if (g2) std::memcpy(g2, &it->second->g2, sizeof(G2Affine));
  if (s_g2) std::memcpy(s_g2, &it->second->s_g2, sizeof(G2Affine));
  return H2G_OK;
}
int h2g_params_set_g2(uint64_t params, const uint64_t g2[16], const uint64_t s_g2[16]) {
  NEED_DEV_P();
  auto it = g_params.find(params);
  if (it == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (!g2 || !s_g2) return fail(H2G_ERR_ARG, "params_set_g2: null argument");
  G2Affine a, b;
  std::memcpy(&a, g2, sizeof(G2Affine));
  std::memcpy(&b, s_g2, sizeof(G2Affine));
  if (!g2_valid(a) || !g2_valid(b)) return fail(H2G_ERR_ARG, "params_set_g2: invalid G2 point");
  it->second->g2 = a;
  it->second->s_g2 = b;
  it->second->has_g2 = true;
  return H2G_OK;
}

/* ProvingKey::write (plonk.rs:311-321) with VerifyingKey::write (plonk.rs:73-86) */
int h2g_pk_write(uint64_t pk_h, int format, uint8_t* out, size_t cap, size_t* len) {
  NEED_DEV_P();
  auto it = g_pks.find(pk_h);
  if (it == g_pks.end()) return fail(H2G_ERR_HANDLE, "unknown proving key");
  if (!len) return fail(H2G_ERR_ARG, "pk_write: null length");
  if (format != SERDE_RAW && format != SERDE_RAW_UNCHECKED && format != SERDE_PROCESSED)
    return fail(H2G_ERR_ARG, "pk_write: unknown SerdeFormat");
  ProvingKey& pk = *it->second;
  auto pit = g_params.find(pk.params);
  if (pit == g_params.end()) return fail(H2G_ERR_HANDLE, "pk_write: the key's params were freed");
  RCCHK(h2g_pk_vk_commitments(pk_h, nullptr, nullptr));  // commit_lagrange, once
  HIPCHK(hipStreamSynchronize(d->stream));
  ByteWriter w{out, out ? cap : 0, d->stream};
  w.proc = format == SERDE_PROCESSED;
  w.u8(PK_VERSION);
  w.u8((uint8_t)pk.k);
  w.u32le((uint32_t)pk.F);
  for (const auto& c : pk.vk_fixed) w.g1(c);
  for (const auto& c : pk.vk_perm) w.g1(c);  // permutation::VerifyingKey::write
  RCCHK(w.poly(pk.l0, pk.ext));
  RCCHK(w.poly(pk.l_last, pk.ext));
  RCCHK(w.poly(pk.l_active, pk.ext));
  RCCHK(w.polys(pk.fixed_lag, pk.n));
  RCCHK(w.polys(pk.fixed_poly, pk.n));
  RCCHK(w.polys(pk.fixed_coset, pk.ext));
  RCCHK(w.polys(pk.sigma_lag, pk.n));  // permutation::ProvingKey::write (permutation.rs:82-91)
  RCCHK(w.polys(pk.sigma_poly, pk.n));
  RCCHK(w.polys(pk.sigma_coset, pk.ext));
  *len = w.len;
  if (out && w.len > cap) return fail(H2G_ERR_ARG, "pk_write: buffer too small");
  return H2G_OK;
}

/* ProvingKey::read (plonk.rs:334-359): like the reference, the circuit (its constraint
 * system) comes from the caller; the key's arrays and commitments come from the bytes
 * (circuit->fixed_values and ->copies are not used and may be NULL). */
int h2g_pk_read(uint64_t params, const h2g_circuit* circuit, const uint8_t* buf, size_t len, int format,
                uint64_t* pk_out) {
  NEED_DEV_P();
  auto it = g_params.find(params);
  if (it == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (!circuit || !buf || !pk_out) return fail(H2G_ERR_ARG, "pk_read: null argument");
  if (format != SERDE_RAW && format != SERDE_RAW_UNCHECKED && format != SERDE_PROCESSED)
    return fail(H2G_ERR_ARG, "pk_read: unknown SerdeFormat");
  const bool proc = format == SERDE_PROCESSED;
  ByteReader r{buf, len};
  if (r.u8() != PK_VERSION) return fail(H2G_ERR_ARG, "pk_read: unexpected version byte");
  const uint32_t k = r.u8();
  if (!r.ok || k != circuit->k || k != it->second->k) return fail(H2G_ERR_ARG, "pk_read: k does not match");
  const uint32_t F = r.u32le();
  if (!r.ok || F != circuit->num_fixed) return fail(H2G_ERR_ARG, "pk_read: fixed column count does not match");
  const uint32_t P = circuit->num_perm_columns;
  std::vector<G1Affine> vf(F), vp(P);
  bool enc_ok = true;
  for (auto* v : {&vf, &vp})
    for (auto& c : *v) {
      if (proc) {
        if (const uint8_t* b = r.take(32)) enc_ok = g1_decompress_host(b, &c) && enc_ok;
      } else if (const uint8_t* b = r.take(sizeof(G1Affine))) {
        std::memcpy(&c, b, sizeof(G1Affine));
      }
    }
  if (!r.ok) return fail(H2G_ERR_ARG, "pk_read: truncated verifying key");
  if (!enc_ok) return fail(H2G_ERR_ARG, "pk_read: invalid point encoding in the verifying key");
  if (format == SERDE_RAW) {
    for (const auto& c : vf)
      if (!g1_valid_host(c)) return fail(H2G_ERR_ARG, "pk_read: invalid fixed commitment");
    for (const auto& c : vp)
      if (!g1_valid_host(c)) return fail(H2G_ERR_ARG, "pk_read: invalid permutation commitment");
  }
  // the extended domain size follows from the constraint system (keygen::create_domain):
  // taken from the first polynomial here and checked against the keygen's below
  const size_t n = (size_t)1 << k;
  PkImage img;
  const uint8_t *l0, *ll, *la;
  const uint32_t ext_len = r.u32be();
  if (!r.ok || ext_len < n || (ext_len & (ext_len - 1))) return fail(H2G_ERR_ARG, "pk_read: bad l0 length");
  l0 = r.take((size_t)ext_len * sizeof(Fr));
  ll = r.poly(ext_len);
  la = r.poly(ext_len);
  img.l0 = l0;
  img.l_last = ll;
  img.l_active = la;
  r.polys(img.fixed_lag, F, n);
  r.polys(img.fixed_poly, F, n);
  r.polys(img.fixed_coset, F, ext_len);
  r.polys(img.sigma_lag, P, n);
  r.polys(img.sigma_poly, P, n);
  r.polys(img.sigma_coset, P, ext_len);
  if (!r.ok) return fail(H2G_ERR_ARG, "pk_read: truncated or mis-sized proving key");
  if (r.pos != len) return fail(H2G_ERR_ARG, "pk_read: trailing bytes");
  DevScratch bad;
  if (proc) {
    img.canonical = true;
    HIPCHK(hipMalloc(&bad.p, 4));
    HIPCHK(hipMemsetAsync(bad.p, 0, 4, d->stream));
    img.bad = (uint32_t*)bad.p;
  }
  auto pk = std::make_unique<ProvingKey>();
  pk->params = params;
  int rc = keygen_impl(d, *it->second, circuit, *pk, &img);
  if (rc == H2G_OK && proc) {
    uint32_t nbad = 0;
    if (hipMemcpyAsync(&nbad, bad.p, 4, hipMemcpyDeviceToHost, d->stream) != hipSuccess ||
        hipStreamSynchronize(d->stream) != hipSuccess)
      rc = fail(H2G_ERR_DEVICE, "pk_read: counter copy");
    else if (nbad) rc = fail(H2G_ERR_ARG, "pk_read: " + std::to_string(nbad) + " field elements not below the modulus");
  }
  if (rc == H2G_OK && pk->ext != ext_len) rc = fail(H2G_ERR_ARG, "pk_read: extended domain size does not match the circuit");
  if (rc == H2G_OK && format == SERDE_RAW) {
    std::vector<std::pair<const Fr*, size_t>> arrays = {{pk->l0, pk->ext}, {pk->l_last, pk->ext}, {pk->l_active, pk->ext}};
    for (int i = 0; i < pk->F; i++) {
      arrays.push_back({pk->fixed_lag[i], n});
      arrays.push_back({pk->fixed_poly[i], n});
      arrays.push_back({pk->fixed_coset[i], pk->ext});
    }
    for (int i = 0; i < pk->P; i++) {
      arrays.push_back({pk->sigma_lag[i], n});
      arrays.push_back({pk->sigma_poly[i], n});
      arrays.push_back({pk->sigma_coset[i], pk->ext});
    }
    uint32_t nbad = 0;
    rc = count_bad_fr(arrays, d->stream, &nbad);
    if (rc == H2G_OK && nbad) rc = fail(H2G_ERR_ARG, "pk_read: " + std::to_string(nbad) + " field elements not below the modulus");
  }
  if (rc) {
    domain_release(&pk->dom);
    return rc;
  }
  pk->vk_fixed = vf;
  pk->vk_perm = vp;
  *pk_out = g_next_handle++;
  g_pks[*pk_out] = std::move(pk);
  return H2G_OK;
}

int h2g_pk_free(uint64_t pk) {
  NEED_DEV_P();
  auto it = g_pks.find(pk);
  if (it == g_pks.end()) return fail(H2G_ERR_HANDLE, "unknown proving key");
  (void)hipStreamSynchronize(d->stream);
  xp_drain(*it->second);
  for (auto& x : it->second->xp)
    if (x.done) (void)hipEventDestroy(x.done);
  domain_release(&it->second->dom);
  if (it->second->lk_cnt) (void)hipHostFree(it->second->lk_cnt);
  if (it->second->lk_or_h) (void)hipHostFree(it->second->lk_or_h);
  if (it->second->lk_or_d) (void)hipFree(it->second->lk_or_d);
  if (it->second->wsum_h) (void)hipHostFree(it->second->wsum_h);
  if (it->second->wsum_d) (void)hipFree(it->second->wsum_d);
  if (it->second->wsum_ev) (void)hipEventDestroy(it->second->wsum_ev);
  for (hipStream_t q : it->second->lk_st)
    if (q) (void)hipStreamDestroy(q);
  for (hipEvent_t e : it->second->lk_ev)
    if (e) (void)hipEventDestroy(e);
  if (it->second->up_h) (void)hipHostFree(it->second->up_h);
  g_pks.erase(it);
  return H2G_OK;
}

/* VerifyingKey::fixed_commitments() (plonk.rs:228-231) and the permutation VerifyingKey's
 * commitments (plonk/permutation.rs:18-47): commit_lagrange of the fixed and sigma columns
 * (keygen.rs, permutation/keygen.rs:269), computed once */
int h2g_pk_vk_commitments(uint64_t pk_h, uint64_t* fixed, uint64_t* perm) {
  NEED_DEV_P();
  auto it = g_pks.find(pk_h);
  if (it == g_pks.end()) return fail(H2G_ERR_HANDLE, "unknown proving key");
  ProvingKey& pk = *it->second;
  auto pit = g_params.find(pk.params);
  if (pit == g_params.end()) return fail(H2G_ERR_HANDLE, "pk_vk_commitments: the key's params were freed");
  if (pk.vk_fixed.size() != (size_t)pk.F || pk.vk_perm.size() != (size_t)pk.P) {
    std::vector<G1Affine> f(pk.F), q(pk.P);
    for (int i = 0; i < pk.F; i++) RCCHK(commit(d, *pit->second, pk.fixed_lag[i], pk.n, SRS_LAGRANGE, &f[i], d->stream));
    for (int i = 0; i < pk.P; i++) RCCHK(commit(d, *pit->second, pk.sigma_lag[i], pk.n, SRS_LAGRANGE, &q[i], d->stream));
    pk.vk_fixed = f;
    pk.vk_perm = q;
  }
  if (fixed && pk.F) std::memcpy(fixed, pk.vk_fixed.data(), pk.vk_fixed.size() * sizeof(G1Affine));
  if (perm && pk.P) std::memcpy(perm, pk.vk_perm.data(), pk.vk_perm.size() * sizeof(G1Affine));
  return H2G_OK;
}

int h2g_pk_set_multiopen(uint64_t pk, int scheme) {
  NEED_DEV_P();
  auto it = g_pks.find(pk);
  if (it == g_pks.end()) return fail(H2G_ERR_HANDLE, "unknown proving key");
  if (scheme != 0 && scheme != 1) return fail(H2G_ERR_ARG, "pk_set_multiopen: scheme must be 0 (SHPLONK) or 1 (GWC)");
  it->second->multiopen = scheme;
  return H2G_OK;
}

int h2g_pk_set_transcript(uint64_t pk, int kind) {
  NEED_DEV_P();
  auto it = g_pks.find(pk);
  if (it == g_pks.end()) return fail(H2G_ERR_HANDLE, "unknown proving key");
  if (kind != TRANSCRIPT_BLAKE2B && kind != TRANSCRIPT_KECCAK256)
    return fail(H2G_ERR_ARG, "pk_set_transcript: kind must be 0 (Blake2bWrite) or 1 (Keccak256Write)");
  it->second->transcript = kind;
  return H2G_OK;
}

int h2g_pk_info(uint64_t pk, int32_t info[8]) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  auto it = g_pks.find(pk);
  if (it == g_pks.end()) return fail(H2G_ERR_HANDLE, "unknown proving key");
  const ProvingKey& p = *it->second;
  const int32_t v[8] = {p.degree, p.bf, (int32_t)p.dom.ek, p.nsets, (int32_t)p.adv_q.size(),
                        (int32_t)p.fix_q.size(), (int32_t)p.ins_q.size(), p.n_slots};
  std::memcpy(info, v, sizeof(v));
  return H2G_OK;
}

}  // extern "C"

namespace {
// the checks and output handling every create_proof entry point shares
int create_proof_entry(Device* d, uint64_t params, uint64_t pk, ProveIn& in, uint8_t* proof, size_t proof_cap,
                       size_t* proof_len) {
  auto ip = g_params.find(params);
  if (ip == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  auto ik = g_pks.find(pk);
  if (ik == g_pks.end()) return fail(H2G_ERR_HANDLE, "unknown proving key");
  ProvingKey& K = *ik->second;
  if (K.params != params) return fail(H2G_ERR_ARG, "create_proof: pk was generated with other params");
  if (K.device != d->id) return fail(H2G_ERR_ARG, "create_proof: pk lives on another device");
  if (!proof_len || in.nc < 1 || in.nc > 1024) return fail(H2G_ERR_ARG, "create_proof: bad arguments");
  for (int c = 0; c < in.nc; c++) {
    if (K.A && !in.src && !in.src1 && (!in.advice || !in.advice[c])) return fail(H2G_ERR_ARG, "create_proof: null advice");
    if (K.I && (!in.instance || !in.inst_lens || !in.instance[c] || !in.inst_lens[c]))
      return fail(H2G_ERR_ARG, "create_proof: null instance");  // InvalidInstances
  }
  std::vector<uint8_t> out;
  out.reserve(32 * 256);
  int rc = prove_impl(d, *ip->second, K, in, &out);
  if (rc) {
    (void)hipStreamSynchronize(d->stream);
    return rc;
  }
  *proof_len = out.size();
  if (out.size() > proof_cap) return fail(H2G_ERR_ARG, "create_proof: proof buffer too small");
  if (proof) std::memcpy(proof, out.data(), out.size());
  return H2G_OK;
}
}  // namespace

extern "C" {

int h2g_create_proof(uint64_t params, uint64_t pk, const uint64_t* advice, int advice_on_device,
                     const uint64_t* instance, const uint32_t* instance_lens, const uint8_t rng_seed[32],
                     uint32_t vanishing_threads, uint8_t* proof, size_t proof_cap, size_t* proof_len) {
  NEED_DEV_P();
  if (!rng_seed) return fail(H2G_ERR_ARG, "create_proof: null rng seed");
  ProverRng rng(rng_seed);
  ProveIn in;
  in.advice = &advice;
  in.adv_dev = advice_on_device != 0;
  in.instance = &instance;
  in.inst_lens = &instance_lens;
  in.rng = &rng;
  in.vthreads = vanishing_threads;
  return create_proof_entry(d, params, pk, in, proof, proof_cap, proof_len);
}

int h2g_create_proof_phased(uint64_t params, uint64_t pk, const h2g_witness_source* witness,
                            const uint64_t* instance, const uint32_t* instance_lens, const uint8_t rng_seed[32],
                            uint32_t vanishing_threads, uint8_t* proof, size_t proof_cap, size_t* proof_len) {
  NEED_DEV_P();
  if (!rng_seed || !witness || !witness->fill) return fail(H2G_ERR_ARG, "create_proof: null argument");
  ProverRng rng(rng_seed);
  ProveIn in;
  in.src1 = witness;
  in.instance = &instance;
  in.inst_lens = &instance_lens;
  in.rng = &rng;
  in.vthreads = vanishing_threads;
  return create_proof_entry(d, params, pk, in, proof, proof_cap, proof_len);
}

int h2g_create_proof_multi(uint64_t params, uint64_t pk, const h2g_prove_inputs* p, uint8_t* proof,
                           size_t proof_cap, size_t* proof_len) {
  NEED_DEV_P();
  if (!p || p->num_circuits < 1) return fail(H2G_ERR_ARG, "create_proof: no circuits");
  if (p->witness && !p->witness->fill) return fail(H2G_ERR_ARG, "create_proof: null witness fill");
  if (!p->rng && !p->rng_seed) return fail(H2G_ERR_ARG, "create_proof: neither an rng nor a seed");
  // fill_bytes is required: the vanishing argument's ChaCha seeds are fill_bytes draws
  // (vanishing/prover.rs:69-73) whatever F::random uses
  if (p->rng && !p->rng->fill_bytes) return fail(H2G_ERR_ARG, "create_proof: the caller's rng needs fill_bytes");
  std::unique_ptr<ProverRng> rng = p->rng ? std::make_unique<ProverRng>(p->rng->fill_bytes, p->rng->random_fr, p->rng->ctx)
                                          : std::make_unique<ProverRng>(p->rng_seed);
  ProveIn in;
  in.nc = (int)std::min<uint32_t>(p->num_circuits, 1u << 20);
  in.advice = p->advice;
  in.adv_dev = p->advice_on_device != 0;
  in.src = p->witness;
  in.instance = p->instance;
  in.inst_lens = p->instance_lens;
  in.rng = rng.get();
  in.vthreads = p->vanishing_threads;
  return create_proof_entry(d, params, pk, in, proof, proof_cap, proof_len);
}

// a ChaCha20Rng::from_seed (rand_chacha 0.3) behind the h2g_rng callbacks: the RngCore
// a Rust host passes to create_proof, here native -- the caller-RNG path of
// h2g_create_proof_multi (no early vanishing commitment) with the seeded path's bytes
std::map<uint64_t, std::unique_ptr<ChaChaRng>> g_rngs;
int rng_fill_cb(void* ctx, uint8_t* out, size_t len) {
  static_cast<ChaChaRng*>(ctx)->fill(out, len);
  return 0;
}
int h2g_rng_chacha20(const uint8_t seed[32], h2g_rng* out, uint64_t* handle) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!seed || !out || !handle) return fail(H2G_ERR_ARG, "rng_chacha20: null argument");
  auto r = std::make_unique<ChaChaRng>(seed);
  out->ctx = r.get();
  out->fill_bytes = rng_fill_cb;
  out->random_fr = nullptr;
  *handle = g_next_handle++;
  g_rngs[*handle] = std::move(r);
  return H2G_OK;
}
int h2g_rng_free(uint64_t handle) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g_rngs.erase(handle)) return fail(H2G_ERR_HANDLE, "rng_free: unknown handle");
  return H2G_OK;
}

int h2g_last_challenges(uint64_t* out, int max, int* count) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!count) return fail(H2G_ERR_ARG, "last_challenges: null count");
  *count = (int)g_last_challenges.size();
  if (out)
    for (int i = 0; i < *count && i < max; i++) std::memcpy(out + 4 * i, &g_last_challenges[i], sizeof(Fr));
  return H2G_OK;
}

int h2g_set_shard_transport(const h2g_shard_transport* t) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (t && t->world > 1) {
    if (!t->launch || !t->collect || t->world > 4096) return fail(H2G_ERR_ARG, "set_shard_transport: bad transport");
    g_shard = *t;
    g_spmd = h2g_spmd_transport{nullptr, 1, 0, nullptr, nullptr, nullptr, nullptr};
  } else {
    g_shard = h2g_shard_transport{nullptr, 1, nullptr, nullptr};
  }
  g_shard_seq = 0;
  return H2G_OK;
}

int h2g_spmd_set_weights(const uint32_t* weights, int world) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  g_spmd_wprefix.clear();
  if (!weights || world <= 1) return H2G_OK;
  if (world > 4096) return fail(H2G_ERR_ARG, "spmd_set_weights: bad world");
  std::vector<uint64_t> pre(1, 0);
  for (int r = 0; r < world; r++) {
    if (weights[r] == 0) return fail(H2G_ERR_ARG, "spmd_set_weights: every rank needs a nonzero weight");
    pre.push_back(pre.back() + weights[r]);
  }
  g_spmd_wprefix = pre;
  return H2G_OK;
}

int h2g_spmd_stats(double* out, int max, int reset) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  for (int k = 0; k < 4; k++) {
    const double v[3] = {g_spmd_stats.ms[k], (double)g_spmd_stats.calls[k], (double)g_spmd_stats.bytes[k]};
    for (int j = 0; j < 3; j++)
      if (out && 3 * k + j < max) out[3 * k + j] = v[j];
  }
  if (reset) g_spmd_stats = SpmdStats{};
  return H2G_OK;
}

int h2g_spmd_set_column_owners(int on) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  g_spmd_colshard = on != 0;
  return H2G_OK;
}

int h2g_set_spmd_exchange_async(h2g_spmd_exchange_post post, h2g_spmd_exchange_wait wait) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (post && (!g_spmd.exchange || g_spmd.world < 2))
    return fail(H2G_ERR_STATE, "set_spmd_exchange_async: install an SPMD transport with an exchange first");
  g_xpost = post;
  g_xwait = post ? wait : nullptr;
  return H2G_OK;
}

int h2g_event_wait(void* done) {
  if (!done) return fail(H2G_ERR_ARG, "event_wait: null event");
  HIPCHK(hipEventSynchronize(static_cast<hipEvent_t>(done)));
  return H2G_OK;
}

int h2g_debug_link_delay(void* stream, void* done, double us) {
  if (!done) return fail(H2G_ERR_ARG, "debug_link_delay: null event");
  HIPCHK(link_delay(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(done), us));
  return H2G_OK;
}

int h2g_set_spmd_transport(const h2g_spmd_transport* t) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  g_xpost = nullptr;
  g_xwait = nullptr;
  if (t && t->world > 1) {
    if (!t->allgather || t->world > 4096 || t->rank < 0 || t->rank >= t->world)
      return fail(H2G_ERR_ARG, "set_spmd_transport: bad transport");
    g_spmd = *t;
    g_shard = h2g_shard_transport{nullptr, 1, nullptr, nullptr};
  } else {
    g_spmd = h2g_spmd_transport{nullptr, 1, 0, nullptr, nullptr, nullptr, nullptr};
  }
  g_spmd_seq = 0;
  return H2G_OK;
}

int h2g_params_set_slab(uint64_t params, uint64_t lo, uint64_t hi) {
  NEED_DEV_P();
  auto ip = g_params.find(params);
  if (ip == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  Params& prm = *ip->second;
  if (prm.device != d->id) return fail(H2G_ERR_ARG, "params_set_slab: params live on another device");
  if (lo > hi || hi > prm.n) return fail(H2G_ERR_ARG, "params_set_slab: bad range");
  msm_fixed_base_free(&prm.sg);
  msm_fixed_base_free(&prm.sgl);
  msm_fixed_base_free(&prm.sgp);
  prm.slab_lo = prm.slab_hi = 0;
  if (hi == lo || (lo == 0 && hi == prm.n)) return H2G_OK;  // none / the full tables
  HIPCHK(msm_fixed_base_build(prm.g + lo, hi - lo, 0, &prm.sg, d->stream));
  HIPCHK(msm_fixed_base_build(prm.gl + lo, hi - lo, 0, &prm.sgl, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  // the lookup basis's windows for the slab (sgp) are built on the first set-2 MSM inside
  // the slab (params_prefix), so a peer serving set-2 slabs never builds the full-size table
  prm.slab_lo = lo;
  prm.slab_hi = hi;
  return H2G_OK;
}

int h2g_params_table_bytes(uint64_t params, uint64_t out[4]) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  auto ip = g_params.find(params);
  if (ip == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (!out) return fail(H2G_ERR_ARG, "params_table_bytes: null output");
  const Params& p = *ip->second;
  auto bytes = [](const MsmFixedBase& t) -> uint64_t {
    return t.table ? (uint64_t)t.W * (uint64_t)t.n * sizeof(G1Affine) : 0;
  };
  out[0] = bytes(p.fg) + bytes(p.fgl);
  out[1] = bytes(p.sg) + bytes(p.sgl);
  out[2] = bytes(p.fgp);
  out[3] = bytes(p.sgp);
  return H2G_OK;
}

int h2g_params_msm_dev(uint64_t params, int32_t base_set, uint64_t offset, uint64_t n, const void* d_scalars,
                       uint64_t out_affine[8], int32_t* out_is_identity) {
  NEED_DEV_P();
  auto ip = g_params.find(params);
  if (ip == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  Params& prm = *ip->second;
  if (prm.device != d->id) return fail(H2G_ERR_ARG, "params_msm_dev: params live on another device");
  if (base_set < SRS_G || base_set > SRS_LAGRANGE_PREFIX || offset > prm.n || n > prm.n - offset || !out_affine ||
      (n && !d_scalars))
    return fail(H2G_ERR_ARG, "params_msm_dev: bad arguments");
  if (base_set == SRS_LAGRANGE_PREFIX) RCCHK(params_prefix(prm, d->stream, offset, n));
  int id = 0;
  size_t toff = 0;
  const MsmFixedBase& tb = prm.tables(base_set, offset, n, &toff);
  RCCHK(msm_fixed_host_impl(d, d_scalars, tb, toff, n, out_affine, &id, d->stream));
  if (out_is_identity) *out_is_identity = id;
  return H2G_OK;
}

int h2g_prover_stage_sync(int on) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  g_stage_sync = on != 0;
  return H2G_OK;
}

int h2g_prover_stages(double* ms, int max, int* count) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  const int c = (int)g_stages.size();
  for (int i = 0; i < c && i < max; i++) ms[i] = g_stages[i].second;
  if (count) *count = c;
  return H2G_OK;
}

const char* h2g_prover_stage_name(int i) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (i < 0 || i >= (int)g_stages.size()) return "";
  return g_stages[i].first;
}


/* ---- native multi-GPU exchange (csrc/comm.cpp) --------------------------------------- */
int h2g_comm_unique_id(uint8_t id[256]) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!id) return fail(H2G_ERR_ARG, "comm_unique_id: null id");
  return comm_unique_id(id);
}

int h2g_comm_init(const uint8_t id[256], int world, int rank) {
  NEED_DEV_P();
  if (!id) return fail(H2G_ERR_ARG, "comm_init: null id");
  return comm_init(id, world, rank);
}

int h2g_comm_set_timeout(double seconds) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return comm_set_timeout(seconds);
}

int h2g_comm_info(int32_t* rccl_count, int32_t* rccl_rank) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  int c = 0, r = -1;
  RCCHK(comm_rccl_info(&c, &r));
  if (rccl_count) *rccl_count = c;
  if (rccl_rank) *rccl_rank = r;
  return H2G_OK;
}

int h2g_comm_destroy(void) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (g_shard.launch == comm_launch) g_shard = h2g_shard_transport{nullptr, 1, nullptr, nullptr};
  if (g_spmd.allgather == comm_allgather_partial) g_spmd = h2g_spmd_transport{nullptr, 1, 0, nullptr, nullptr, nullptr, nullptr};
  if (g_xpost == comm_exchange_post) g_xpost = nullptr, g_xwait = nullptr;
  return comm_destroy();
}

int h2g_comm_set_exchange_overlap(int on) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  g_comm_overlap = on != 0;
  return H2G_OK;
}

int h2g_comm_set_serve_timeout(double seconds) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return comm_set_serve_timeout(seconds);
}

int h2g_comm_keepalive(void) {
  NEED_DEV_P();
  return comm_keepalive();
}

int h2g_comm_spmd_install(int split_subcosets) {
  NEED_DEV_P();
  if (comm_world() < 2) return fail(H2G_ERR_STATE, "comm_spmd_install: needs a communicator (h2g_comm_init)");
  g_spmd = h2g_spmd_transport{comm_spmd_ctx(), comm_world(), comm_rank(), comm_allgather_partial,
                              split_subcosets ? comm_bcast : nullptr, comm_allgather_host,
                              split_subcosets ? comm_exchange : nullptr};
  // the column-ownership exchanges overlap the later stages on the second communicator
  // only when asked (h2g_comm_set_exchange_overlap): two communicators in flight from two
  // streams has not run on multi-GPU hardware yet, so blocking is the default
  g_xpost = split_subcosets && g_comm_overlap ? comm_exchange_post : nullptr;
  g_xwait = g_xpost ? comm_exchange_wait : nullptr;
  g_shard = h2g_shard_transport{nullptr, 1, nullptr, nullptr};
  g_spmd_seq = 0;
  return H2G_OK;
}

int h2g_comm_spmd_uninstall(void) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (g_spmd.allgather == comm_allgather_partial) g_spmd = h2g_spmd_transport{nullptr, 1, 0, nullptr, nullptr, nullptr, nullptr};
  if (g_xpost == comm_exchange_post) g_xpost = nullptr, g_xwait = nullptr;
  g_spmd_seq = 0;
  return H2G_OK;
}

int h2g_comm_install(uint64_t params) {
  NEED_DEV_P();
  auto ip = g_params.find(params);
  if (ip == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  if (comm_world() < 2 || comm_rank() != 0) return fail(H2G_ERR_STATE, "comm_install: needs rank 0 of a communicator");
  g_shard = h2g_shard_transport{comm_transport_ctx(ip->second->n), comm_world(), comm_launch, comm_collect};
  g_shard_seq = 0;
  return H2G_OK;
}

int h2g_comm_stop(void) {
  NEED_DEV_P();
  if (g_shard.launch == comm_launch) g_shard = h2g_shard_transport{nullptr, 1, nullptr, nullptr};
  return comm_stop();
}

/* ranks 1..: answer rank 0's MSM slabs against `params` until it stops the session */
int h2g_comm_serve(uint64_t params, uint64_t* served) {
  NEED_DEV_P();
  auto ip = g_params.find(params);
  if (ip == g_params.end()) return fail(H2G_ERR_HANDLE, "unknown params");
  Params& prm = *ip->second;
  if (prm.device != d->id) return fail(H2G_ERR_ARG, "comm_serve: params live on another device");
  static_assert(COMM_OP_STOP == commwait::REQ_STOP && COMM_OP_MSM == commwait::REQ_MSM &&
                    COMM_OP_PING == commwait::REQ_PING,
                "serve loop request codes");
  int32_t set = 0;
  uint64_t lo = 0, cnt = 0;
  const void* slab = nullptr;
  hipStream_t ready = nullptr;
  auto next = [&](int* op) -> int {  // the idle deadline applies (h2g_comm_set_serve_timeout)
    int32_t o = 0;
    RCCHK(comm_next_request(&o, &set, &lo, &cnt, &slab, &ready));
    *op = o;
    return H2G_OK;
  };
  auto answer = [&](int op) -> int {
    if (op != COMM_OP_MSM || set < SRS_G || set > SRS_LAGRANGE_PREFIX || lo > prm.n || cnt > prm.n - lo)
      return fail(H2G_ERR_STATE, "comm_serve: malformed request");
    // the slab's windows of the prefix basis (built on the first set-2 request inside the
    // slab), never the full-size table on a peer that only serves slabs
    if (set == SRS_LAGRANGE_PREFIX) RCCHK(params_prefix(prm, d->stream, lo, cnt));
    uint64_t out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (cnt) {
      size_t toff = 0;
      MsmTicket t;
      RCCHK(msm_fixed_launch(d, slab, prm.tables(set, lo, cnt, &toff), toff, cnt, ready, &t));
      RCCHK(msm_collect(d, &t, out));
    }
    uint64_t nz = 0;
    for (uint64_t v : out) nz |= v;
    RCCHK(comm_send_partial(out, nz == 0));
    return H2G_OK;
  };
  unsigned long long count = 0;
  RCCHK(commwait::serve_requests(next, answer, &count));
  if (served) *served = count;
  return H2G_OK;
}

}  // extern "C"
