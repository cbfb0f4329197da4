/*
 * h2g.h -- C ABI of the MI355X-native halo2 prover hot path (libh2g.so).
 *
 * This is the drop-in boundary a halo2 (yetanotherco/yet-another-halo2-fork)
 * host binds over FFI.  Plain pointers and sizes only; no torch or HIP types.
 *
 * Data layout (identical to halo2curves 0.6 in memory, so Rust slices are passed
 * by pointer with no conversion):
 *   Fr  : 4 x uint64_t little-endian limbs, Montgomery form (R = 2^256), < r
 *   G1Affine : x[4], y[4] Fq limbs, Montgomery form; identity = (0, 0)
 * Host-pointer entry points copy in/out and return when the result is ready.
 * `_dev` entry points take device pointers (hipMalloc'd, or torch tensors'
 * data_ptr()) and a `stream` (hipStream_t; NULL = the library's stream for the
 * current device); they are asynchronous unless noted.
 *
 * Every function returns H2G_OK (0) or an error code; h2g_last_error() gives a
 * message.  Reference interfaces replaced are cited per entry point
 * (paths relative to the reference snapshot root).
 */
#ifndef H2G_H
#define H2G_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  H2G_OK = 0,
  H2G_ERR_ARG = 1,     /* invalid argument (the reference panics: assert_eq! in best_multiexp/commit) */
  H2G_ERR_DEVICE = 2,  /* HIP runtime error */
  H2G_ERR_NOMEM = 3,
  H2G_ERR_STATE = 4,   /* not initialised */
  H2G_ERR_HANDLE = 5   /* unknown descriptor / domain handle */
};

int h2g_abi_version(void);
const char* h2g_last_error(void);

/* ---- engine lifecycle ---------------------------------------------------
 * Replaces PlonkEngineConfig::new().set_curve::<G1Affine>().set_msm(engine).build()
 * (halo2_middleware/src/zal.rs:204-243): initialises the listed HIP devices
 * (NULL/0 = device 0). */
int h2g_init(const int* devices, int ndev);
int h2g_shutdown(void);
int h2g_device_count(int* out);
int h2g_set_device(int index); /* index into the h2g_init list */
/* free / total device memory of the current device, after a device-wide synchronize
 * (hipMemGetInfo): what a caller checks descriptor lifetimes against */
int h2g_device_mem_info(uint64_t* free_bytes, uint64_t* total_bytes);

/* ---- MsmAccel<G1Affine> (halo2_middleware/src/zal.rs:57-103) ----------------
 * msm(coeffs, base) -> C::Curve  (zal.rs:58; H2cEngine::msm = best_multiexp, zal.rs:136-138).
 * Result returned affine (out[8]) + identity flag; the shim converts with G1::from. */
int h2g_msm(const uint64_t* coeffs, const uint64_t* bases, size_t n, uint64_t out_affine[8],
            int* out_is_identity);
/* get_coeffs_descriptor / get_base_descriptor (zal.rs:83-84): upload once, keep on device */
int h2g_msm_coeffs_descriptor(const uint64_t* coeffs, size_t n, uint64_t* handle);
int h2g_msm_base_descriptor(const uint64_t* bases, size_t n, uint64_t* handle);
int h2g_msm_descriptor_free(uint64_t handle); /* Drop of a descriptor (zal.rs:47) */
/* Base descriptors keep fixed-base windows ([2^(o_w)] P_i at each window's bit offset o_w,
 * W x n x 64 B of HBM) so the MSM runs one shared bucket set; the _dev variants take device-resident bases /
 * scalars (window_bits 0 = choose). */
int h2g_msm_base_descriptor_dev(const void* d_bases, size_t n, int window_bits, uint64_t* handle);
int h2g_msm_with_cached_base_dev(const void* d_scalars, size_t n, uint64_t base, size_t base_offset,
                                 uint64_t out_affine[8], int* out_is_identity, void* stream);
/* msm_with_cached_scalars / _base / _inputs (zal.rs:86-102); base_offset selects the
 * prefix/sub-slice &bases[off..off+n] used by commit / commit_lagrange
 * (halo2_backend/src/poly/kzg/commitment.rs:316, 365) */
int h2g_msm_with_cached_scalars(uint64_t coeffs, const uint64_t* bases, size_t n, uint64_t out_affine[8],
                                int* out_is_identity);
int h2g_msm_with_cached_base(const uint64_t* coeffs, size_t n, uint64_t base, size_t base_offset,
                             uint64_t out_affine[8], int* out_is_identity);
int h2g_msm_with_cached_inputs(uint64_t coeffs, uint64_t base, size_t base_offset, uint64_t out_affine[8],
                               int* out_is_identity);
/* device-resident MSM: d_out receives 8 u64 (affine, identity = zeros) */
int h2g_msm_dev(const void* d_coeffs, const void* d_bases, size_t n, void* d_out_affine, void* stream);
/* same, with an explicit Pippenger window size c (0 = automatic) */
int h2g_msm_dev_cfg(const void* d_coeffs, const void* d_bases, size_t n, int window_bits, void* d_out_affine,
                    void* stream);
/* device-resident inputs, result returned to the host (synchronous) -- the path
 * MsmAccel::msm takes when the prover keeps polynomials in HBM */
int h2g_msm_dev_host(const void* d_coeffs, const void* d_bases, size_t n, int window_bits, uint64_t out_affine[8],
                     int* out_is_identity, void* stream);
int h2g_descriptor_device_ptr(uint64_t handle, void** d_ptr, size_t* n);

/* ---- SRS generation on device: g_i = [s^i] G, i < n
 * (ParamsKZG::setup, halo2_backend/src/poly/kzg/commitment.rs:64-90). s in Montgomery form. */
int h2g_srs_setup_dev(const uint64_t s[4], size_t n, void* d_out_affine, void* stream);

/* ---- NTT boundary (new seam; best_fft call sites halo2_backend/src/poly/domain.rs:238, 344
 * and halo2_backend/src/arithmetic.rs:38).  In place, natural order in and out:
 * a_k <- sum_i a_i omega^(ik), n = 2^log_n. */
int h2g_fft(uint64_t* a, uint32_t log_n, const uint64_t omega[4]);
int h2g_fft_dev(void* d_a, uint32_t log_n, const uint64_t omega[4], void* stream);

/* ---- EvaluationDomain (halo2_backend/src/poly/domain.rs) -------------------- */
/* EvaluationDomain::new(j, k) (domain.rs:38-144) */
int h2g_domain_create(uint32_t j, uint32_t k, uint64_t* handle);
int h2g_domain_free(uint64_t handle);
/* consts9 = omega, omega_inv, extended_omega, extended_omega_inv, g_coset, g_coset_inv,
 * ifft_divisor, extended_ifft_divisor, barycentric_weight (Fr, 4 limbs each) */
int h2g_domain_info(uint64_t handle, uint32_t* k, uint32_t* extended_k, uint64_t consts9[36]);
/* lagrange_to_coeff (domain.rs:216-226): in place, n = 2^k */
int h2g_lagrange_to_coeff(uint64_t dom, uint64_t* a);
int h2g_lagrange_to_coeff_dev(uint64_t dom, void* d_a, void* stream);
/* coeff_to_extended (domain.rs:230-244): in n, out 2^extended_k */
int h2g_coeff_to_extended(uint64_t dom, const uint64_t* a, uint64_t* out);
int h2g_coeff_to_extended_dev(uint64_t dom, const void* d_a, void* d_out, void* stream);
/* extended_to_coeff (domain.rs:271-293): in 2^extended_k, out n*(j-1) (truncated) */
int h2g_extended_to_coeff(uint64_t dom, const uint64_t* a, uint64_t* out);
int h2g_extended_to_coeff_dev(uint64_t dom, const void* d_a, void* d_out, void* stream);
/* divide_by_vanishing_poly (domain.rs:297-316): in place on 2^extended_k */
int h2g_divide_by_vanishing_poly(uint64_t dom, uint64_t* a);
int h2g_divide_by_vanishing_poly_dev(uint64_t dom, void* d_a, void* stream);

/* ---- Polynomial<F, B> arithmetic (halo2_backend/src/poly.rs:200-276) ---------
 * op: 0 add a+b, 1 sub a-b, 2 mul a*b, 3 scale a*c, 4 sub_const a-c, 5 add_const a+c,
 *     6 axpy a*c+b.  c is a host Fr (4 limbs), ignored by ops 0-2. */
int h2g_fr_op(int op, const uint64_t* a, const uint64_t* b, const uint64_t c[4], uint64_t* out, size_t n);
int h2g_fr_op_dev(int op, const void* d_a, const void* d_b, const uint64_t c[4], void* d_out, size_t n,
                  void* stream);
/* ff::BatchInvert (zeros stay zero); permutation/prover.rs:124, lookup/prover.rs:225 */
int h2g_fr_batch_invert(uint64_t* a, size_t n);
int h2g_fr_batch_invert_dev(void* d_a, size_t n, void* stream);
/* out_i = prod_{j<=i} a_j; grand products permutation/prover.rs:160-166 */
int h2g_fr_prefix_product(const uint64_t* a, uint64_t* out, size_t n);
int h2g_fr_prefix_product_dev(const void* d_a, void* d_out, size_t n, void* stream);
/* exclusive prefix sum of n u32 (n < 2^32; d_in == d_out allowed): the counts-to-offsets scan
 * of the lookup argument's sorts and compactions (lookup/prover.rs:410-494) */
int h2g_u32_exclusive_scan_dev(const void* d_in, void* d_out, size_t n, void* stream);

/* ---- device memory / stream helpers --------------------------------------- */
int h2g_dev_alloc(size_t bytes, void** d_ptr);
int h2g_dev_free(void* d_ptr);
int h2g_memcpy_htod(void* d_dst, const void* h_src, size_t bytes);
int h2g_memcpy_dtoh(void* h_dst, const void* d_src, size_t bytes);
int h2g_synchronize(void);
/* elapsed time (ms) of `fn`-free timing: record events on a stream */
int h2g_event_create(void** ev);
int h2g_event_destroy(void* ev);
int h2g_event_record(void* ev, void* stream);
int h2g_event_elapsed_ms(void* start, void* stop, float* ms);

/* ---- profiling: per-phase HIP-event times of MSM calls made while enabled.
 * Phases (in order): partition_coarse (digits -> coarse bins), partition_fine (bins -> bucket
 * order), bucket_bounds, accumulate, bucket_fixup, reduce.  collect() synchronises, returns the
 * per-phase sums (ms) over `calls` MSMs and resets.  With max_phases >= 8, ms[6] and ms[7] are
 * the busy time (union of the intervals) of the accumulate phases and of the whole MSMs:
 * MSMs on the two MSM streams overlap, so work / union is the aggregate rate. */
int h2g_profile_enable(int on);
int h2g_profile_msm_collect(float* ms, int max_phases, int* n_phases, int* calls);
/* the profiled MSMs' sorted entries (nonzero signed digits = mixed additions in the
 * accumulation) summed, before collect() resets them; *uncounted = MSMs past the
 * recorder's capacity (may be NULL) */
int h2g_profile_msm_entries(uint64_t* total, int* uncounted);
/* box calibration (bench line): Montgomery product throughput of this GPU now, in the two
 * limb forms the prover uses -- out[0] 8 x 32-bit FIPS, out[1] 9 x 29-bit (G products/s)
 * -- out[2] the shader clock during the run (GHz, s_memtime vs s_memrealtime), out[3] the
 * wall ms spent (~100); max >= 4.  Not part of the prover's interface. */
int h2g_profile_box_calibrate(double* out, int max);

/* ---- host-side point helpers (used to combine per-GPU MSM partials) -------- */
int h2g_g1_add_affine(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]);


/* ---- create_proof (BN254 / KZG / SHPLONK, Blake2b transcript) -------------
 * The backend entry points of halo2_backend/src/plonk/{keygen.rs, prover.rs}:
 *   ParamsKZG::{setup, read}   poly/kzg/commitment.rs:64-131,167-267  -> h2g_params_*
 *   keygen_vk + keygen_pk      plonk/keygen.rs:43-190                  -> h2g_keygen
 *   create_proof(params, pk, circuits=[1], instances, rng, transcript)
 *                              plonk/prover.rs:174-899 (ProverSingle)  -> h2g_create_proof
 * The circuit is the backend's CompiledCircuit (halo2_middleware/src/circuit.rs):
 * gates as flattened ExpressionMid nodes, permutation columns + copies, fixed values.
 * Node = 4 x int32 (op, a, b, c): op 0 CONST (a = constant index), 1 QUERY (a = column
 * type 0 advice / 1 fixed / 2 instance, b = column index, c = rotation), 2 NEG (a),
 * 3 SUM (a, b), 4 PROD (a, b), 5 CHALLENGE (a = challenge index; ExpressionMid::Challenge).
 * Copy = 6 x int32 (ltype, lindex, lrow, rtype, rindex, rrow).
 * Supported: advice phases and challenges (advice_column_phase / challenge_phase of
 * ConstraintSystemMid, circuit.rs), gates, permutation, lookups, shuffles.
 * rng: ChaCha20Rng::from_seed(rng_seed); vanishing_threads: the thread count that
 * splits the vanishing argument's random polynomial into ChaCha streams
 * (vanishing/prover.rs:57-81), part of the proof's determinism. */
typedef struct {
  uint32_t k, num_advice, num_fixed, num_instance;
  uint32_t num_gates;
  const int32_t* gate_roots;
  uint32_t num_nodes;
  const int32_t* nodes;
  uint32_t num_constants;
  const uint64_t* constants;      /* Fr */
  uint32_t num_perm_columns;
  const int32_t* perm_columns;    /* (type, index) pairs, permutation ArgumentMid.columns order */
  uint32_t num_copies;
  const int32_t* copies;
  const uint64_t* fixed_values;   /* num_fixed x n Fr (Lagrange) */
  const uint8_t* unblinded;       /* num_advice flags (unblinded_advice_columns) or NULL */
  const uint64_t* transcript_repr; /* vk.transcript_repr (Fr) */
  /* lookup arguments (lookup::Argument): per lookup m (input, table) expression pairs;
   * roots: per lookup m input roots then m table roots */
  uint32_t num_lookups;
  const uint32_t* lookup_sizes;
  const int32_t* lookup_roots;
  /* shuffle arguments (shuffle::Argument): per shuffle m input roots then m shuffle roots */
  uint32_t num_shuffles;
  const uint32_t* shuffle_sizes;
  const int32_t* shuffle_roots;
  /* phases (appended; NULL / 0 = one phase, no challenges): advice_phase[num_advice]
   * (advice_column_phase), challenge_phase[num_challenges] (challenge_phase) */
  const uint8_t* advice_phase;
  uint32_t num_challenges;
  const uint8_t* challenge_phase;
} h2g_circuit;

/* SRS resident on the current device: g[n] and g_lagrange[n] (G1Affine) from the host... */
int h2g_params_create(uint32_t k, const uint64_t* g, const uint64_t* g_lagrange, uint64_t* handle);
/* ...or generated on the device from the toxic secret s (ParamsKZG::setup; tests/bench) */
int h2g_params_setup(uint32_t k, const uint64_t s[4], uint64_t* handle);
int h2g_params_export(uint64_t params, uint64_t* g, uint64_t* g_lagrange); /* n x 8 u64 each, may be NULL */
int h2g_params_free(uint64_t params);
/* the G2 points of ParamsKZG (kzg/commitment.rs:26-27): g2 and s_g2, 16 u64 each
 * (x.c0, x.c1, y.c0, y.c1 in Montgomery form); setup computes them, create needs set_g2
 * before the params can be written */
int h2g_params_g2(uint64_t params, uint64_t g2[16], uint64_t s_g2[16]);
int h2g_params_set_g2(uint64_t params, const uint64_t g2[16], const uint64_t s_g2[16]);

/* ---- serialisation: SerdeFormat (halo2_backend/src/helpers.rs:8-21) -----------------
 * format 1 RawBytes (uncompressed points, Montgomery limbs; reads check that field
 * elements are below the modulus and points lie on the curve), 2 RawBytesUnchecked
 * (no checks), 0 Processed (helpers.rs:36-100: G1 points as 32-B GroupEncoding -- x
 * canonical LE, bit 7 of the last byte = y odd, identity all zero --, G2 points as 64 B
 * (x.c0 || x.c1, sign from y.c0), field elements canonical LE (to_repr); reads decompress
 * on the device and refuse x >= p, x without a curve point and field elements >= r).
 * Writers: out == NULL returns the byte length in *len.
 *   ParamsKZG::write_custom / read_custom  kzg/commitment.rs:166-267
 *   ProvingKey::write / read               plonk.rs:311-359 (+ VerifyingKey::write/read :73-129)
 * h2g_pk_read takes the constraint system from `circuit` (as the reference takes `cs`)
 * and every array of the key from the bytes; circuit->fixed_values / ->copies unused. */
int h2g_params_write(uint64_t params, int format, uint8_t* out, size_t cap, size_t* len);
int h2g_params_read(const uint8_t* buf, size_t len, int format, uint64_t* handle);

int h2g_keygen(uint64_t params, const h2g_circuit* circuit, uint64_t* pk);
int h2g_pk_free(uint64_t pk);
int h2g_pk_write(uint64_t pk, int format, uint8_t* out, size_t cap, size_t* len);
int h2g_pk_read(uint64_t params, const h2g_circuit* circuit, const uint8_t* buf, size_t len, int format,
                uint64_t* pk);
/* degree, blinding_factors, extended_k, #perm sets, #advice/#fixed/#instance queries */
int h2g_pk_info(uint64_t pk, int32_t info[8]);
/* the verifying key's commitments: VerifyingKey::fixed_commitments() (plonk.rs:228-231) and
 * the permutation VerifyingKey's commitments (plonk/permutation.rs:18-47), G1Affine (8 u64 each):
 * fixed[num_fixed], perm[num_perm_columns]; either may be NULL */
int h2g_pk_vk_commitments(uint64_t pk, uint64_t* fixed, uint64_t* perm);
/* the multi-open argument h2g_create_proof ends with -- the reference's Prover type
 * parameter of create_proof (halo2_proofs/src/plonk/prover.rs:19-36): 0 ProverSHPLONK
 * (default; poly/kzg/multiopen/shplonk/prover.rs:121-305), 1 ProverGWC
 * (poly/kzg/multiopen/gwc/prover.rs:40-90) */
int h2g_pk_set_multiopen(uint64_t pk, int scheme);
/* the transcript the proof is written with -- create_proof's TranscriptWrite type
 * parameter: 0 Blake2bWrite (default; halo2_backend/src/transcript.rs:291-419),
 * 1 Keccak256Write (EVM-verifiable; transcript.rs:299-463) */
int h2g_pk_set_transcript(uint64_t pk, int kind);

/* advice: num_advice x n Fr; instance: num_instance x n Fr (zero padded), of which
 * instance_lens[i] values enter the transcript.  Writes the proof bytes.
 * advice_on_device != 0: `advice` is a device pointer (inputs resident in HBM), 16-byte
 * aligned (H2G_ERR_ARG otherwise; the columns are read in 16-byte chunks). */
int h2g_create_proof(uint64_t params, uint64_t pk, const uint64_t* advice, int advice_on_device,
                     const uint64_t* instance, const uint32_t* instance_lens, const uint8_t rng_seed[32],
                     uint32_t vanishing_threads, uint8_t* proof, size_t proof_cap, size_t* proof_len);
/* Prover::commit_phase driven by the caller's witness generator (plonk/prover.rs:309-494):
 * before committing phase p (0..max advice phase) the prover calls
 *   fill(ctx, p, challenges, advice)
 * with the challenges squeezed so far (num_challenges x 4 u64 Montgomery limbs; those of
 * phases >= p are zero) and the host advice buffer (num_advice x n Fr), in which the
 * callback writes the columns of phase p (staging owned by the key, pinned when the host
 * allows: num_advice x n x 32 B for the key's lifetime; the prover reads only phase p's
 * columns from it, other columns may hold anything).  fill must write rows
 * [0, n - blinding_factors - 1) of every phase-p column; the prover zeroes the unusable rows
 * of unblinded columns before calling it (blinded ones receive randomness).  Nonzero from
 * fill fails the proof with H2G_ERR_ARG.  Callbacks (fill, and the shard transport's
 * launch / collect) run on the calling thread with the library lock held: they must not
 * wait on h2g calls made from other threads.  h2g_create_proof is the same prover with every phase read from
 * `advice` (a witness that was computed with the challenges already known). */
typedef struct {
  void* ctx;
  int (*fill)(void* ctx, uint32_t phase, const uint64_t* challenges, uint64_t* advice);
} h2g_witness_source;
int h2g_create_proof_phased(uint64_t params, uint64_t pk, const h2g_witness_source* witness,
                            const uint64_t* instance, const uint32_t* instance_lens, const uint8_t rng_seed[32],
                            uint32_t vanishing_threads, uint8_t* proof, size_t proof_cap, size_t* proof_len);
/* ---- create_proof with the reference's full argument list ------------------------
 * create_proof(params, pk, circuits: &[C], instances: &[&[&[F]]], rng: R: RngCore,
 * transcript) (halo2_proofs/src/plonk/prover.rs:19-36; Prover::new_with_engine /
 * commit_phase / create_proof, halo2_backend/src/plonk/prover.rs:174-899): several
 * circuits of one key in one proof, in the reference's interleaving -- instances per
 * circuit, each phase's advice commitments circuit by circuit, then per circuit its
 * lookups, permutation sets, lookup products and shuffles, one vanishing argument and one
 * h(X) over all circuits (evaluation.rs:365-620), evaluations and queries circuit by
 * circuit before the fixed and common ones.
 * rng: the caller's `R: RngCore`, drawn in the reference's order.  Two kinds
 * of draw exist: F::random(&mut rng) (blinding rows and blinds) and rng.fill_bytes(&mut
 * [u8; 32]) (the vanishing argument's ChaCha20 seeds, vanishing/prover.rs:69-73).
 *   random_fr : F::random(&mut rng) as 4 Montgomery limbs (the Rust shim calls
 *               Fr::random itself, so the proof does not depend on how halo2curves
 *               consumes the RNG); NULL = fill_bytes(64) read as from_uniform_bytes
 *   fill_bytes: RngCore::fill_bytes(out[0..len]); required, even with random_fr (the
 *               vanishing seeds are fill_bytes draws) -- NULL fails the call up front
 * Nonzero from either fails the proof with H2G_ERR_ARG. */
typedef struct {
  void* ctx;
  int (*fill_bytes)(void* ctx, uint8_t* out, size_t len);
  int (*random_fr)(void* ctx, uint64_t out[4]);
} h2g_rng;
/* Prover::commit_phase's witness per circuit: like h2g_witness_source.fill, for circuit c */
typedef struct {
  void* ctx;
  int (*fill)(void* ctx, uint32_t circuit, uint32_t phase, const uint64_t* challenges, uint64_t* advice);
} h2g_witness_source_multi;
typedef struct {
  uint32_t num_circuits;                /* >= 1 */
  const uint64_t* const* advice;        /* [num_circuits] num_advice x n Fr, or NULL with `witness` */
  int advice_on_device;                 /* advice[c] are device pointers */
  const h2g_witness_source_multi* witness;
  const uint64_t* const* instance;      /* [num_circuits] num_instance x n Fr (zero padded) */
  const uint32_t* const* instance_lens; /* [num_circuits] num_instance values each */
  const h2g_rng* rng;                   /* NULL: ChaCha20Rng::from_seed(rng_seed) */
  const uint8_t* rng_seed;
  uint32_t vanishing_threads;
} h2g_prove_inputs;
int h2g_create_proof_multi(uint64_t params, uint64_t pk, const h2g_prove_inputs* in, uint8_t* proof,
                           size_t proof_cap, size_t* proof_len);
/* a native ChaCha20Rng::from_seed(seed) (rand_chacha 0.3) as an h2g_rng: *out's callbacks
 * draw from it (the RngCore a Rust host passes to create_proof, without the host); the
 * proof equals the rng_seed path's bytes.  h2g_rng_free releases it. */
int h2g_rng_chacha20(const uint8_t seed[32], h2g_rng* out, uint64_t* handle);
int h2g_rng_free(uint64_t handle);
/* the challenges of the last proof (num_challenges x 4 u64), *count = num_challenges */
int h2g_last_challenges(uint64_t* out, int max, int* count);
/* wall milliseconds of the stages of the last h2g_create_proof (names: h2g_prover_stage_name).
 * Stages end when their work is queued, unless h2g_prover_stage_sync(1) is set: then each
 * stage boundary synchronises the prover stream and the times are GPU completion times
 * (diagnostics only -- it serialises the pipeline) */
int h2g_prover_stage_sync(int on);
int h2g_prover_stages(double* ms, int max, int* count);
const char* h2g_prover_stage_name(int i);

/* ---- one proof across several GPUs: MSM point slabs ------------
 * Every commitment MSM of create_proof (the MsmAccel::msm call sites of SURVEY 8a-1)
 * is split into `world` contiguous point slabs [P r / world, P (r + 1) / world) (P = 2^k
 * of the params, clipped to the MSM length n); rank 0 (the
 * prover) computes slab 0 and the transport hands slabs 1.. to the peer ranks, each of
 * which holds the same SRS (h2g_params_setup / _create) and answers with the affine
 * partial sum of its slab (h2g_params_msm_dev).  Rank 0 adds the partials (the group sum
 * is exact, so the proof bytes do not depend on `world`).  The transport is the host's
 * (one process per GPU over RCCL in yet-another-halo2-fork_amd/h2g_dist.py).
 *   launch : called once per MSM, in transcript order, after the scalars (n Fr,
 *            device pointer, valid until the matching collect) are complete;
 *            base_set 0 = params.g (commit), 1 = params.g_lagrange (commit_lagrange),
 *            2 = the prefix sums P_i = L_0 + ... + L_i of g_lagrange (a lookup's permuted
 *            columns, committed as sum_i (a_i - a_{i+1}) P_i: the same point, from
 *            scalars that vanish inside the columns' runs of equal values)
 *   collect: the world - 1 partials of MSM `seq` (8 u64 affine each, is_identity flags)
 * Both return 0 on success; nonzero fails the proof with H2G_ERR_STATE. */
typedef struct {
  void* ctx;
  int32_t world;
  int (*launch)(void* ctx, uint64_t seq, int32_t base_set, uint64_t n, const void* d_scalars);
  int (*collect)(void* ctx, uint64_t seq, uint64_t* partials, int32_t* is_identity);
} h2g_shard_transport;
/* install (world >= 2) or remove (NULL or world <= 1) the transport of h2g_create_proof */
int h2g_set_shard_transport(const h2g_shard_transport* t);
/* this rank's slab [lo, hi) of the params' points: builds fixed-base windows sized for
 * the slab (used by h2g_params_msm_dev and, on rank 0, by create_proof's own slab);
 * lo == hi removes them */
int h2g_params_set_slab(uint64_t params, uint64_t lo, uint64_t hi);
/* peer side: MSM of n device scalars against params' base set [offset, offset + n) */
int h2g_params_msm_dev(uint64_t params, int32_t base_set, uint64_t offset, uint64_t n, const void* d_scalars,
                       uint64_t out_affine[8], int32_t* out_is_identity);
/* device bytes the params hold in fixed-base windows: out[0] g and g_lagrange (full), out[1]
 * their slab windows, out[2] the prefix-summed Lagrange basis's full windows (built for a
 * key with lookups, or on a set-2 MSM outside the slab), out[3] its slab windows (built on
 * the first set-2 MSM inside the slab) -- a serving peer's footprint, observable */
int h2g_params_table_bytes(uint64_t params, uint64_t out[4]);
/* synchronous device-to-device copy (staging slabs for the transport) */
int h2g_memcpy_dtod(void* d_dst, const void* d_src, size_t bytes);

/* ---- the same sharding with the library's own RCCL transport (xGMI), no host callbacks:
 * a Rust (or any) host binds these five calls and shards create_proof's MSMs natively.
 * One process per GPU, each after h2g_init on its own device and with the same params:
 *   rank 0:  h2g_comm_unique_id(id) -> the host sends the 256 bytes to every rank
 *   all:     h2g_comm_init(id, world, rank)          (ncclCommInitRank x 2: slabs, partials)
 *   rank 0:  h2g_comm_install(params)  -> create_proof shards every commitment MSM
 *            ... h2g_create_proof* ...  -> h2g_comm_stop() ends the peers' sessions
 *   ranks 1..: h2g_comm_serve(params, &served)     (returns when rank 0 stops)
 *   all:     h2g_comm_destroy()
 * Slab r = points [P r / world, P (r + 1) / world) of the params' P, as for
 * h2g_shard_transport; rank 0 stages the peers' scalars with one device copy, sends them
 * over one communicator and receives the 64-B partials over the other, so later MSMs'
 * slabs stream while the peers compute.  The proof bytes do not depend on `world`. */
int h2g_comm_unique_id(uint8_t id[256]);
int h2g_comm_init(const uint8_t id[256], int world, int rank);
/* deadline (seconds; <= 0: none; default 300) of every wait on the library's RCCL
 * communicators: their non-blocking setup in h2g_comm_init, each call's enqueue and each
 * collective's completion.  Past it -- or on an RCCL error -- the communicators are aborted
 * (ncclCommAbort) and the call fails with H2G_ERR_DEVICE, so a run that would hang inside
 * RCCL returns and the caller can fall back to another transport (bench.py).  The peers'
 * wait for rank 0's next slab request (h2g_comm_serve) has its own deadline, below. */
int h2g_comm_set_timeout(double seconds);
/* shard mode: a serving peer's longest wait (seconds; <= 0: none, the default) for rank 0's
 * next request header in h2g_comm_serve.  Rank 0 that aborts its communicators (a timed-out
 * wait) or dies need not surface as an RCCL error on the peer; past this deadline the peer
 * aborts its own and h2g_comm_serve fails with H2G_ERR_DEVICE instead of waiting forever.
 * Rank 0 renews the peers' deadline with h2g_comm_keepalive while it idles between proofs
 * (a header the serve loop only counts as a sign of life). */
int h2g_comm_set_serve_timeout(double seconds);
int h2g_comm_keepalive(void);
int h2g_comm_install(uint64_t params);
int h2g_comm_serve(uint64_t params, uint64_t* served);
int h2g_comm_stop(void);
int h2g_comm_destroy(void);
/* the communicator as RCCL reports it (ncclCommCount / ncclCommUserRank); 0 / -1 without one */
int h2g_comm_info(int32_t* rccl_count, int32_t* rccl_rank);

/* ---- one proof across several GPUs, SPMD: every rank runs the same create_proof (same
 * key, witness, instances and RNG stream -- a seed, or draws the host replicates -- hence
 * the same transcript).  Rank r computes point slab r ([P r / world, P (r + 1) / world),
 * h2g_params_set_slab) of every commitment MSM from its own copy of the scalars, and the
 * 64-B partials are all-gathered and summed in rank order, so every rank writes the same
 * proof bytes as one GPU would and no scalars cross the links.
 *   allgather: in = this rank's H2G_SPMD_WORDS words: its partial (8 u64 affine limbs,
 *              then 1 if the identity) and 4 words of consistency digest (a Blake2b of
 *              the transcript state, of every RNG draw so far and of the advice columns'
 *              values at a fixed point, each rank evaluating its whole copy of every
 *              column once per advice phase); out = world x H2G_SPMD_WORDS u64 in rank
 *              order; 0 on success.  Every rank compares the digests and fails the proof
 *              (H2G_ERR_STATE) if any rank's differ: ranks fed different witnesses,
 *              instances or RNG draws would otherwise sum slabs of different polynomials
 *              into one invalid proof without an error (the commitments and evaluations
 *              are sums of the ranks' slabs, so they alone cannot reveal it). */
#define H2G_SPMD_WORDS 13
/*
 * The host transport (callbacks) or the library's RCCL all-gather (h2g_comm_spmd_install,
 * after h2g_comm_init on every rank).  Installing one sharding mode removes the other. */
typedef struct {
  void* ctx;
  int32_t world;
  int32_t rank;
  int (*allgather)(void* ctx, uint64_t seq, const uint64_t in[9], uint64_t* out);
  /* optional -- NULL replicates the extended-domain work on every rank.  Otherwise the
   * 2^e sub-cosets of the extended domain (e = extended_k - k; row t + 2^e m is point
   * zeta w_ext^t w^m) are divided over the ranks: rank r computes the sub-cosets
   * t = r, r + world, ... of every column and h(X) on those rows, and each sub-coset's
   * h evaluations (n Fr, device memory) are broadcast from their owner t mod world:
   * bcast(ctx, d_buf, bytes, root) in place, complete on return */
  int (*bcast)(void* ctx, void* d_buf, size_t bytes, int root);
  /* optional -- NULL replicates the multi-open tail.  Otherwise the evaluations and the
   * SHPLONK multi-open (poly/kzg/multiopen/shplonk/prover.rs:121-305) run on coefficient
   * slabs: rank r evaluates, combines and divides only coefficients [P r / world,
   * P (r + 1) / world) of each polynomial -- the points its MSM slabs cover -- and the
   * few scalars that join the slabs (partial evaluations, the kate divisions' carries
   * between slabs) are all-gathered: allgather_host(ctx, in, bytes, out) with `bytes`
   * host bytes from this rank, out = world x bytes in rank order, complete on return */
  int (*allgather_host)(void* ctx, const void* in, size_t bytes, void* out);
  /* optional, with bcast and allgather_host -- h(X) reaches the ranks as coefficient
   * slabs instead of broadcast evaluations: the owner of sub-coset t interpolates its h
   * evaluations (an n-point inverse NTT instead of everyone's 2^e n-point one) and every
   * rank receives slab r of each sub-coset's folded coefficients, from which it forms
   * its slab of the h pieces (vanishing/prover.rs:102-155).  exchange(ctx, d_send,
   * send_bytes, d_recv, recv_bytes): device buffers, all-to-all with per-peer byte counts
   * (world entries each; peer p's data contiguous, in peer order; the rank's own entry
   * is a local copy), complete on return */
  int (*exchange)(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv, const size_t* recv_bytes);
} h2g_spmd_transport;
/* install (world >= 2) or remove (NULL or world <= 1); either removes the overlapped
 * exchange below */
int h2g_set_spmd_transport(const h2g_spmd_transport* t);
/* optional, with exchange: the column-ownership exchanges (h2g_spmd_set_column_owners)
 * overlap the stages after them instead of draining the stream.  post(ctx, d_send,
 * send_bytes, d_recv, recv_bytes, stream, done) queues the same all-to-all as exchange()
 * behind the work queued on `stream` (a hipStream_t) so far and returns without waiting for
 * the transfer; `done` (a hipEvent_t the library owns) is recorded once the received bytes
 * are in place.  wait(ctx, done) returns once `done` has been recorded and the transfer has
 * finished, 0 on success (a transport with a deadline fails it there).  The prover posts a
 * stage's exchange right after its sub-cosets are packed and waits for all of them after
 * the vanishing commitments, before h(X) reads them; every rank posts in the same order.
 * ctx is the transport's.  NULL post: every exchange completes on return. */
typedef int (*h2g_spmd_exchange_post)(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv,
                                      const size_t* recv_bytes, void* stream, void* done);
typedef int (*h2g_spmd_exchange_wait)(void* ctx, void* done);
int h2g_set_spmd_exchange_async(h2g_spmd_exchange_post post, h2g_spmd_exchange_wait wait);
/* helpers for host transports of the overlapped exchange (with h2g_event_record):
 * hipEventSynchronize(done); and, for the one-GPU SPMD emulation (tools/spmd_emulate.py),
 * `done` recorded `us` microseconds of device time after the work queued on `stream` so
 * far (a one-thread wait kernel on a side stream stands for a modelled transfer) */
int h2g_event_wait(void* done);
int h2g_debug_link_delay(void* stream, void* done, double us);
/* SPMD slab partition (optional): rank r's slab -- of every commitment MSM and of the
 * multi-open tail's coefficients -- is [P S_r / S, P S_{r+1} / S) with S_r = weights[0] +
 * ... + weights[r - 1] and S their total, instead of [P r / world, P (r + 1) / world).
 * Every rank must pass the same weights, and its h2g_params_set_slab the same slab.  The
 * ranks that own extended-domain sub-cosets carry that extra work; smaller slabs balance
 * them against the others.  NULL (or world <= 1) restores the uniform partition. */
int h2g_spmd_set_weights(const uint32_t* weights, int world);
/* SPMD column ownership of wide stages (on by default; used with bcast, allgather_host and
 * exchange installed): an advice phase, the lookups' permuted columns or their products
 * with as many columns as ranks or more (a multiple of the ranks, or 4x them) go to the
 * ranks whole, column i to rank i mod world -- the owner commits it (its rank's partial is
 * the whole commitment, the others' the identity), forms its coefficients and its
 * sub-cosets, and one exchange per stage hands every sub-coset owner its sub-cosets and
 * every rank its coefficient slab; a lookup's sort, match and product run on its owner
 * only.  Stages with fewer columns keep the point slabs.  Applies from 4 ranks up: at 2
 * the exchange puts a quarter of the extended-domain data on the one link between the
 * ranks (more time than the transforms it saves).  0 turns it off. */
int h2g_spmd_set_column_owners(int on);
/* time inside the SPMD transport since the last reset, per collective kind k (0 the MSM
 * partials' all-gathers, 1 the host all-gathers, 2 the exchanges, 3 the broadcasts):
 * out[3k] milliseconds (host wall clock around the call), out[3k + 1] calls, out[3k + 2]
 * bytes sent + received; reset != 0 zeroes the counters after reading */
int h2g_spmd_stats(double* out, int max, int reset);
/* split_subcosets: 1 divides the extended domain's sub-cosets over the ranks (bcast over
 * the communicator), 0 replicates that work; the multi-open tail always runs on
 * coefficient slabs (allgather_host over the communicator) */
int h2g_comm_spmd_install(int split_subcosets);
/* SPMD over the library's communicators: 1 posts the column-ownership exchanges on the
 * second communicator's stream so they overlap the stages after them (the prover waits for
 * them before h(X)); 0 (the default) keeps them blocking on the first.  Read at
 * h2g_comm_spmd_install.  Both produce the same proof bytes. */
int h2g_comm_set_exchange_overlap(int on);
int h2g_comm_spmd_uninstall(void);

#ifdef __cplusplus
}
#endif

#endif /* H2G_H */
