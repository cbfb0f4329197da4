/*
 * prover.c -- CPU restatement of halo2's create_proof over BN254 / KZG / SHPLONK
 * with the Blake2b transcript.  TEST INFRASTRUCTURE ONLY (the parity checker for the
 * device pipeline and the CPU baseline).  This translation unit includes oracle.c
 * (field, G1, best_multiexp, best_fft, EvaluationDomain) and is the only file the
 * oracle Makefile compiles.
 *
 * Restated reference code (paths relative to the reference root):
 *   keygen_pk                          halo2_backend/src/plonk/keygen.rs:94-190
 *   query collection / degree / bf     halo2_backend/src/plonk/keygen.rs:191-394, plonk/circuit.rs:95-180,292-320
 *   permutation Assembly / build_pk    halo2_backend/src/plonk/permutation/keygen.rs:16-213
 *   Prover::new_with_engine            halo2_backend/src/plonk/prover.rs:174-305
 *   commit_phase                       halo2_backend/src/plonk/prover.rs:309-494
 *   create_proof                       halo2_backend/src/plonk/prover.rs:512-899
 *   permutation_commit / evaluate / open  halo2_backend/src/plonk/permutation/prover.rs:50-333
 *   vanishing commit / construct / evaluate / open  halo2_backend/src/plonk/vanishing/prover.rs:40-205
 *   evaluate_h (gates + permutation)   halo2_backend/src/plonk/evaluation.rs:317-483
 *   SHPLONK create_proof               halo2_backend/src/poly/kzg/multiopen/shplonk/prover.rs:121-305
 *   GWC create_proof                   halo2_backend/src/poly/kzg/multiopen/gwc/prover.rs:40-90, gwc.rs:25-50
 *   construct_intermediate_sets        halo2_backend/src/poly/kzg/multiopen/shplonk.rs:48-140
 *   Blake2bWrite transcript            halo2_backend/src/transcript.rs:120-130,353-419,500-539
 *   lookup argument                    halo2_backend/src/plonk/lookup/prover.rs:64-494
 *   shuffle argument                   halo2_backend/src/plonk/shuffle/prover.rs:36-255
 * Scope: several circuits per proof, advice phases and challenges, fixed and instance
 * columns, custom gates (expression graphs with rotations), the permutation, lookup and
 * shuffle arguments; the prover rng is ChaCha20Rng::from_seed or the caller's RngCore.
 * Unverifiable-here details (isolated): G1 compressed encoding (x LE, bit 7 of byte 31
 * = y odd); vk.transcript_repr is taken as an input (plonk.rs:189-200 hashes the Rust
 * Debug text of the pinned VK).
 */
#include "oracle.c"
#include "hash.h"

#include <stdio.h>

/* ====================================================================== spec */
enum { COL_ADVICE = 0, COL_FIXED = 1, COL_INSTANCE = 2 };
enum { OP_CONST = 0, OP_QUERY = 1, OP_NEG = 2, OP_SUM = 3, OP_PROD = 4, OP_CHALLENGE = 5 };

typedef struct {
    uint32_t k, num_advice, num_fixed, num_instance;
    uint32_t num_gates;
    const int32_t *gate_roots;
    uint32_t num_nodes;
    const int32_t *nodes; /* 4 ints per node: op, a, b, c */
    uint32_t num_constants;
    const uint64_t *constants;
    uint32_t num_perm_columns;
    const int32_t *perm_columns; /* (type, index) pairs */
    uint32_t num_copies;
    const int32_t *copies; /* (ltype, lindex, lrow, rtype, rindex, rrow) */
    const uint64_t *fixed_values;    /* num_fixed * n Fr */
    const uint64_t *advice_values;   /* num_advice * n Fr */
    const uint64_t *instance_values; /* num_instance * n Fr (zero padded) */
    const uint32_t *instance_lens;
    const uint64_t *transcript_repr; /* Fr */
    const uint8_t *rng_seed;         /* 32 bytes: ChaCha20Rng::from_seed */
    uint32_t vanishing_threads;
    const uint64_t *srs_g;          /* n G1Affine */
    const uint64_t *srs_g_lagrange; /* n G1Affine */
    const uint8_t *unblinded;       /* num_advice flags (unblinded_advice_columns) or NULL */
    uint32_t num_lookups;
    const uint32_t *lookup_sizes;   /* m_l (input, table) expression pairs per lookup */
    const int32_t *lookup_roots;    /* per lookup: m_l input roots, then m_l table roots */
    uint32_t num_shuffles;
    const uint32_t *shuffle_sizes;
    const int32_t *shuffle_roots;   /* per shuffle: m input roots, then m shuffle roots */
    uint32_t multiopen;             /* 0 ProverSHPLONK, 1 ProverGWC (poly/kzg/multiopen) */
    /* phases (ConstraintSystemMid advice_column_phase / challenge_phase; NULL / 0 = one
     * phase, no challenges) and the witness source of Prover::commit_phase
     * (prover.rs:309-494): fill(ctx, phase, challenges so far, advice num_advice x n) writes
     * the phase's columns; NULL fill = every phase read from advice_values */
    const uint8_t *advice_phase;
    uint32_t num_challenges;
    const uint8_t *challenge_phase;
    int (*fill)(void *ctx, uint32_t phase, const uint64_t *challenges, uint64_t *advice);
    void *fill_ctx;
    uint64_t *challenges_out;       /* num_challenges x 4 (may be NULL) */
    const uint64_t *challenge_values; /* set by or_prove: the squeezed challenges */
    /* several circuits of one key in one proof (create_proof's circuits: &[C] and
     * instances: &[&[&[F]]], halo2_proofs/src/plonk/prover.rs:19-36); num_circuits 0 = one
     * circuit from advice_values / instance_values / instance_lens / fill above */
    uint32_t num_circuits;
    const uint64_t *const *advice_c;       /* [num_circuits] num_advice x n Fr */
    const uint64_t *const *instance_c;     /* [num_circuits] num_instance x n Fr */
    const uint32_t *const *instance_lens_c;
    int (*fill_multi)(void *ctx, uint32_t circuit, uint32_t phase, const uint64_t *challenges, uint64_t *advice);
    /* the caller's `rng: R: RngCore` (NULL both = ChaCha20Rng::from_seed(rng_seed)):
     * random_fr = F::random(rng) (Montgomery limbs; NULL = 64 fill_bytes, from_uniform_bytes),
     * fill_bytes = RngCore::fill_bytes (the vanishing seeds) */
    int (*rng_fill_bytes)(void *ctx, uint8_t *out, size_t len);
    int (*rng_random_fr)(void *ctx, uint64_t *out);
    void *rng_ctx;
    /* 0 Blake2bWrite, 1 Keccak256Write (halo2_backend/src/transcript.rs:299-463) */
    uint32_t transcript;
} or_spec;

typedef struct { int type, index, rot; } query_t;

/* ====================================================================== small helpers */
static fe fe_from(const uint64_t *p) { fe r; memcpy(r.v, p, 32); return r; }

static void fr_random(chacha_rng *rng, fe *out) {   /* Fr::random: LE512 mod r */
    uint8_t b[64];
    chacha_rng_fill(rng, b, 64);
    uint64_t d[8];
    for (int i = 0; i < 8; i++) d[i] = load64le(b + 8 * i);
    static const fe R3 = {{0x5e94d8e1b4bf0040ULL, 0x2a489cbe1cfbb6b8ULL, 0x893cc664a19fcfedULL, 0x0cf8594b7fcc657cULL}};
    fe lo = fe_from(d), hi = fe_from(d + 4), t1, t2;
    fr_mul(&t1, &lo, &fr_R2);   /* d0 * R2 * R^-1 = mont(d0) */
    fr_mul(&t2, &hi, &R3);      /* d1 * R3 * R^-1 = mont(d1 * 2^256) */
    fr_add(out, &t1, &t2);
}

/* the prover's rng: ChaCha20Rng::from_seed, or the caller's RngCore (or_spec rng_*) */
typedef struct {
    chacha_rng cc;
    int (*fb)(void *, uint8_t *, size_t);
    int (*fr)(void *, uint64_t *);
    void *ctx;
    int failed;
} prng_t;
static void prng_fill(prng_t *r, uint8_t *out, size_t len) {
    if (!r->fb && !r->fr) { chacha_rng_fill(&r->cc, out, len); return; }
    if (r->failed || !r->fb || r->fb(r->ctx, out, len)) { r->failed = 1; memset(out, 0, len); }
}
static void prng_random(prng_t *r, fe *out) {   /* F::random(&mut rng) */
    if (r->fr) {
        uint64_t v[4] = {0, 0, 0, 0};
        if (r->failed || r->fr(r->ctx, v)) { r->failed = 1; memset(out, 0, sizeof(fe)); return; }
        int below = 0;   /* an Fr must be below r */
        for (int i = 3; i >= 0; i--) if (v[i] != fr_MOD[i]) { below = v[i] < fr_MOD[i]; break; }
        if (!below) { r->failed = 1; memset(out, 0, sizeof(fe)); return; }
        *out = fe_from(v);
        return;
    }
    uint8_t b[64];
    prng_fill(r, b, 64);
    uint64_t d[8];
    for (int i = 0; i < 8; i++) d[i] = load64le(b + 8 * i);
    static const fe R3 = {{0x5e94d8e1b4bf0040ULL, 0x2a489cbe1cfbb6b8ULL, 0x893cc664a19fcfedULL, 0x0cf8594b7fcc657cULL}};
    fe lo = fe_from(d), hi = fe_from(d + 4), t1, t2;
    fr_mul(&t1, &lo, &fr_R2); fr_mul(&t2, &hi, &R3); fr_add(out, &t1, &t2);
}

static fe fr_pow_u64(const fe *a, uint64_t e) {
    uint64_t ee[4] = {e, 0, 0, 0};
    fe r; fr_pow(&r, a, ee); return r;
}

/* ====================================================================== transcript */
/* Blake2bWrite (transcript.rs:120-130,353-419) or Keccak256Write (transcript.rs:299-463):
 * the same prefixes (challenge 0, point 1, scalar 2) absorbed into the growing state;
 * Keccak256 squeezes [0] into the state, then hashes two copies with the extra bytes 10
 * and 11 (not kept in the state) for the low and high 32 bytes of the 64 uniform bytes */
typedef struct {
    int kind;
    blake2b_state st;
    keccak_state ks;
    uint8_t *proof;
    size_t len, cap;
} transcript_t;

static void tr_init(transcript_t *t, int kind, uint8_t *buf, size_t cap) {
    t->kind = kind;
    if (kind == 1) {
        keccak_init(&t->ks);
        keccak_update(&t->ks, "Halo2-Transcript", 16);
    } else {
        blake2b_init(&t->st, 64, (const uint8_t *)"Halo2-Transcript");
    }
    t->proof = buf; t->len = 0; t->cap = cap;
}
static void tr_absorb(transcript_t *t, const uint8_t *b, size_t len) {
    if (t->kind == 1) keccak_update(&t->ks, b, len);
    else blake2b_update(&t->st, b, len);
}
static void fr_repr(const fe *a, uint8_t out[32]) {
    uint64_t c[4]; fr_to_canonical(c, a);
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(c[i / 8] >> (8 * (i % 8)));
}
static void fq_repr(const fe *a, uint8_t out[32]) {
    uint64_t c[4]; fq_to_canonical(c, a);
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(c[i / 8] >> (8 * (i % 8)));
}
static void tr_common_scalar(transcript_t *t, const fe *s) {
    uint8_t b[33]; b[0] = 2; fr_repr(s, b + 1);
    tr_absorb(t, b, 33);
}
static void tr_write_scalar(transcript_t *t, const fe *s) {
    tr_common_scalar(t, s);
    uint8_t r[32]; fr_repr(s, r);
    if (t->len + 32 <= t->cap) memcpy(t->proof + t->len, r, 32);
    t->len += 32;
}
static int tr_write_point(transcript_t *t, const g1a *p) {
    if (g1a_is_id(p)) return -1;  /* "cannot write points at infinity to the transcript" */
    uint8_t b[65]; b[0] = 1; fq_repr(&p->x, b + 1); fq_repr(&p->y, b + 33);
    tr_absorb(t, b, 65);
    uint8_t c[32]; memcpy(c, b + 1, 32);
    if (b[33] & 1) c[31] |= 0x80;  /* compressed: x, sign of y in the top bit */
    if (t->len + 32 <= t->cap) memcpy(t->proof + t->len, c, 32);
    t->len += 32;
    return 0;
}
static fe tr_squeeze(transcript_t *t) {
    uint8_t z = 0; tr_absorb(t, &z, 1);
    uint8_t h[64];
    if (t->kind == 1) {
        keccak_state lo = t->ks, hi = t->ks;
        const uint8_t plo = 10, phi = 11;
        keccak_update(&lo, &plo, 1);
        keccak_update(&hi, &phi, 1);
        keccak_final_copy(&lo, 0x01, h);
        keccak_final_copy(&hi, 0x01, h + 32);
    } else {
        blake2b_final_copy(&t->st, h);
    }
    uint64_t d[8];
    for (int i = 0; i < 8; i++) d[i] = load64le(h + 8 * i);
    static const fe R3 = {{0x5e94d8e1b4bf0040ULL, 0x2a489cbe1cfbb6b8ULL, 0x893cc664a19fcfedULL, 0x0cf8594b7fcc657cULL}};
    fe lo = fe_from(d), hi = fe_from(d + 4), t1, t2, r;
    fr_mul(&t1, &lo, &fr_R2); fr_mul(&t2, &hi, &R3); fr_add(&r, &t1, &t2);
    return r;   /* Challenge255: from_uniform_bytes, stored as repr, re-read: same value */
}

/* ====================================================================== expressions */
static int node_degree(const or_spec *s, int i) {
    const int32_t *nd = s->nodes + 4 * i;
    switch (nd[0]) {
        case OP_CONST: case OP_CHALLENGE: return 0;
        case OP_QUERY: return 1;
        case OP_NEG: return node_degree(s, nd[1]);
        case OP_SUM: { int a = node_degree(s, nd[1]), b = node_degree(s, nd[2]); return a > b ? a : b; }
        default: return node_degree(s, nd[1]) + node_degree(s, nd[2]);
    }
}

typedef struct { query_t *q; int n, cap; } qlist;
static int qlist_add(qlist *l, int type, int index, int rot) {
    for (int i = 0; i < l->n; i++)
        if (l->q[i].type == type && l->q[i].index == index && l->q[i].rot == rot) return i;
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 16; l->q = (query_t *)realloc(l->q, l->cap * sizeof(query_t)); }
    l->q[l->n].type = type; l->q[l->n].index = index; l->q[l->n].rot = rot;
    return l->n++;
}
/* QueriesMap::as_expression: depth first, lhs before rhs (keygen.rs:217-249) */
static void collect_queries(const or_spec *s, int i, qlist *adv, qlist *fix, qlist *ins) {
    const int32_t *nd = s->nodes + 4 * i;
    switch (nd[0]) {
        case OP_CONST: case OP_CHALLENGE: return;
        case OP_QUERY:
            if (nd[1] == COL_ADVICE) qlist_add(adv, nd[1], nd[2], nd[3]);
            else if (nd[1] == COL_FIXED) qlist_add(fix, nd[1], nd[2], nd[3]);
            else qlist_add(ins, nd[1], nd[2], nd[3]);
            return;
        case OP_NEG: collect_queries(s, nd[1], adv, fix, ins); return;
        default: collect_queries(s, nd[1], adv, fix, ins); collect_queries(s, nd[2], adv, fix, ins); return;
    }
}

/* evaluate expression i at extended row idx over coset arrays */
static fe eval_node(const or_spec *s, int i, fe *const *adv, fe *const *fix, fe *const *ins, uint64_t idx,
                    uint64_t rot_scale, uint64_t ext) {
    const int32_t *nd = s->nodes + 4 * i;
    fe r, a, b;
    switch (nd[0]) {
        case OP_CONST: return fe_from(s->constants + 4 * nd[1]);
        case OP_CHALLENGE: return fe_from(s->challenge_values + 4 * nd[1]);
        case OP_QUERY: {
            int64_t j = ((int64_t)idx + (int64_t)nd[3] * (int64_t)rot_scale) % (int64_t)ext;
            if (j < 0) j += (int64_t)ext;
            fe *const *cols = nd[1] == COL_ADVICE ? adv : (nd[1] == COL_FIXED ? fix : ins);
            return cols[nd[2]][j];
        }
        case OP_NEG: a = eval_node(s, nd[1], adv, fix, ins, idx, rot_scale, ext); fr_neg(&r, &a); return r;
        case OP_SUM:
            a = eval_node(s, nd[1], adv, fix, ins, idx, rot_scale, ext);
            b = eval_node(s, nd[2], adv, fix, ins, idx, rot_scale, ext);
            fr_add(&r, &a, &b); return r;
        default:
            a = eval_node(s, nd[1], adv, fix, ins, idx, rot_scale, ext);
            b = eval_node(s, nd[2], adv, fix, ins, idx, rot_scale, ext);
            fr_mul(&r, &a, &b); return r;
    }
}

/* ====================================================================== polynomial helpers */
static fe *fr_alloc(uint64_t n) { return (fe *)calloc(n ? n : 1, sizeof(fe)); }
static fe eval_poly(const fe *p, uint64_t n, const fe *x) {
    fe r; or_fr_eval((const uint64_t *)p, n, x->v, r.v); return r;
}
static fe rotate_omega(const domain_t *d, const fe *x, int rot) {
    fe w = rot >= 0 ? d->omega : d->omega_inv;
    fe p = fr_pow_u64(&w, (uint64_t)(rot >= 0 ? rot : -rot)), r;
    fr_mul(&r, x, &p); return r;
}
/* CPU-baseline mode: 0 = MSM/FFT use the prover's thread count ("all cores");
 * t > 0 = MSM/FFT on t threads while parallelize-style loops keep the prover's count -- 1
 * is the "faithful" mode of a halo2curves build without its multicore feature */
static int g_kernel_threads = 0;
void or_set_kernel_threads(int t) { g_kernel_threads = t > 0 ? t : 0; }
static int kt(int threads) { return g_kernel_threads ? g_kernel_threads : threads; }

static void lagrange_to_coeff_d(const domain_t *d, fe *a, int threads) {
    or_fft((uint64_t *)a, d->k, d->omega_inv.v, kt(threads));
    ifft_scale(a, d->n, &d->ifft_divisor);
}
static void coeff_to_extended_d(const domain_t *d, const fe *in, fe *out, int threads) {
    uint64_t ext = 1ULL << d->extended_k;
    memcpy(out, in, d->n * sizeof(fe));
    distribute_powers_zeta(d, out, d->n, 1);
    memset(out + d->n, 0, (ext - d->n) * sizeof(fe));
    or_fft((uint64_t *)out, d->extended_k, d->extended_omega.v, kt(threads));
}
static int commit_msm(const fe *scalars, uint64_t n, const uint64_t *bases, int threads, g1a *out) {
    or_msm_best((const uint64_t *)scalars, bases, n, kt(threads), (uint64_t *)out);
    return 0;
}
/* lagrange_interpolate (arithmetic.rs:177-230): coefficients of the unique poly of
 * degree < m through (points[i], evals[i]) */
static void lagrange_interpolate(const fe *pts, const fe *ev, int m, fe *coeffs) {
    for (int i = 0; i < m; i++) coeffs[i] = (fe){{0, 0, 0, 0}};
    fe *basis = fr_alloc(m), *tmp = fr_alloc(m + 1);
    for (int j = 0; j < m; j++) {
        /* numerator prod_{k != j} (X - x_k), denominator prod (x_j - x_k) */
        for (int i = 0; i <= m; i++) tmp[i] = (fe){{0, 0, 0, 0}};
        tmp[0] = fr_ONE;
        int deg = 0;
        fe den = fr_ONE;
        for (int kk = 0; kk < m; kk++) {
            if (kk == j) continue;
            fe nx; fr_neg(&nx, &pts[kk]);
            for (int i = deg + 1; i >= 0; i--) {   /* tmp *= (X - x_k) */
                fe a = i > 0 ? tmp[i - 1] : (fe){{0, 0, 0, 0}}, b, c;
                fr_mul(&b, &tmp[i], &nx);
                fr_add(&c, &a, &b);
                tmp[i] = c;
            }
            deg++;
            fe dd; fr_sub(&dd, &pts[j], &pts[kk]); fr_mul(&den, &den, &dd);
        }
        fe inv, sc; fr_inv(&inv, &den); fr_mul(&sc, &inv, &ev[j]);
        for (int i = 0; i < m; i++) { fe t; fr_mul(&t, &tmp[i], &sc); fr_add(&coeffs[i], &coeffs[i], &t); }
    }
    free(basis); free(tmp);
}
static int fe_cmp_canon(const fe *a, const fe *b) {  /* Ord on Fr: canonical numeric order */
    uint64_t ca[4], cb[4]; fr_to_canonical(ca, a); fr_to_canonical(cb, b);
    for (int i = 3; i >= 0; i--) { if (ca[i] < cb[i]) return -1; if (ca[i] > cb[i]) return 1; }
    return 0;
}

/* ====================================================================== permutation Assembly */
typedef struct { int col, row; } cell_t;
typedef struct { cell_t *mapping, *aux; uint64_t *sizes; int cols; uint64_t n; } assembly_t;
static int perm_col_pos(const or_spec *s, int type, int index) {
    for (uint32_t i = 0; i < s->num_perm_columns; i++)
        if (s->perm_columns[2 * i] == type && s->perm_columns[2 * i + 1] == index) return (int)i;
    return -1;
}
static void assembly_copy(assembly_t *A, int lc, int lr, int rc, int rr) {  /* permutation/keygen.rs:48-97 */
    cell_t lcyc = A->aux[(uint64_t)lc * A->n + lr], rcyc = A->aux[(uint64_t)rc * A->n + rr];
    if (lcyc.col == rcyc.col && lcyc.row == rcyc.row) return;
    if (A->sizes[(uint64_t)lcyc.col * A->n + lcyc.row] < A->sizes[(uint64_t)rcyc.col * A->n + rcyc.row]) {
        cell_t t = lcyc; lcyc = rcyc; rcyc = t;
    }
    A->sizes[(uint64_t)lcyc.col * A->n + lcyc.row] += A->sizes[(uint64_t)rcyc.col * A->n + rcyc.row];
    cell_t i = rcyc;
    for (;;) {
        A->aux[(uint64_t)i.col * A->n + i.row] = lcyc;
        i = A->mapping[(uint64_t)i.col * A->n + i.row];
        if (i.col == rcyc.col && i.row == rcyc.row) break;
    }
    cell_t tmp = A->mapping[(uint64_t)lc * A->n + lr];
    A->mapping[(uint64_t)lc * A->n + lr] = A->mapping[(uint64_t)rc * A->n + rr];
    A->mapping[(uint64_t)rc * A->n + rr] = tmp;
}

/* ====================================================================== lookup / shuffle helpers */
/* compress_expressions: fold_e (acc * theta + e(row)) over Lagrange columns (lookup/prover.rs:85-103;
 * evaluate() evaluation.rs:838-872 with rot_scale 1 over n rows) */
static void compress_lagrange(const or_spec *s, const int32_t *roots, int m, fe *const *adv, fe *const *fix,
                              fe *const *ins, uint64_t n, const fe *theta, fe *out, int threads) {
#pragma omp parallel for num_threads(threads) schedule(static)
    for (uint64_t i = 0; i < n; i++) {
        fe acc = {{0, 0, 0, 0}};
        for (int e = 0; e < m; e++) {
            fe v = eval_node(s, roots[e], adv, fix, ins, i, 1, n);
            fr_mul(&acc, &acc, theta); fr_add(&acc, &acc, &v);
        }
        out[i] = acc;
    }
}
/* the same fold on the extended coset (the lookup/shuffle GraphEvaluators, evaluation.rs:245-300) */
static fe compress_coset(const or_spec *s, const int32_t *roots, int m, fe *const *adv, fe *const *fix,
                         fe *const *ins, uint64_t idx, uint64_t rot_scale, uint64_t ext, const fe *theta) {
    fe acc = {{0, 0, 0, 0}};
    for (int e = 0; e < m; e++) {
        fe v = eval_node(s, roots[e], adv, fix, ins, idx, rot_scale, ext);
        fr_mul(&acc, &acc, theta); fr_add(&acc, &acc, &v);
    }
    return acc;
}

typedef struct { uint64_t c[4]; fe v; } keyed;
static int keyed_cmp(const void *a_, const void *b_) {
    const keyed *a = (const keyed *)a_, *b = (const keyed *)b_;
    for (int i = 3; i >= 0; i--) { if (a->c[i] < b->c[i]) return -1; if (a->c[i] > b->c[i]) return 1; }
    return 0;
}
/* permute_expression_pair (lookup/prover.rs:410-494): sorted input; table value = input at the
 * first row of each run, leftover table values (ascending, BTreeMap order) fill the repeated
 * rows from the last one backwards; then bf+1 random rows each (input first). */
static int permute_pair(const fe *A, const fe *S, uint64_t n, int bf, prng_t *rng, fe *Ap, fe *Sp) {
    const uint64_t u = n - (uint64_t)(bf + 1);
    keyed *ia = (keyed *)malloc((u + 1) * sizeof(keyed)), *ta = (keyed *)malloc((u + 1) * sizeof(keyed));
    for (uint64_t i = 0; i < u; i++) {
        ia[i].v = A[i]; fr_to_canonical(ia[i].c, &A[i]);
        ta[i].v = S[i]; fr_to_canonical(ta[i].c, &S[i]);
    }
    qsort(ia, u, sizeof(keyed), keyed_cmp);
    qsort(ta, u, sizeof(keyed), keyed_cmp);
    uint64_t *rep = (uint64_t *)malloc((u + 1) * sizeof(uint64_t)), nrep = 0;
    uint8_t *used = (uint8_t *)calloc(u + 1, 1);
    uint64_t tp = 0;
    int ok = 1;
    for (uint64_t r = 0; r < u; r++) {
        Ap[r] = ia[r].v;
        if (r == 0 || keyed_cmp(&ia[r], &ia[r - 1]) != 0) {
            Sp[r] = ia[r].v;
            while (tp < u && keyed_cmp(&ta[tp], &ia[r]) < 0) tp++;
            if (tp < u && keyed_cmp(&ta[tp], &ia[r]) == 0) used[tp++] = 1;
            else ok = 0;
        } else {
            rep[nrep++] = r;
        }
    }
    if (ok) {
        uint64_t li = 0;
        for (uint64_t t = 0; t < u; t++)
            if (!used[t]) Sp[rep[nrep - 1 - li++]] = ta[t].v;
    }
    free(ia); free(ta); free(rep); free(used);
    if (!ok) return -7;   /* Error::ConstraintSystemFailure: an input value is not in the table */
    for (uint64_t r = u; r < n; r++) prng_random(rng, &Ap[r]);
    for (uint64_t r = u; r < n; r++) prng_random(rng, &Sp[r]);
    return 0;
}

/* z = [1, prod_0, prod_0 prod_1, ...] over n - bf rows, then bf random rows */
static void grand_product(const fe *prod, uint64_t n, int bf, prng_t *rng, fe *z) {
    z[0] = fr_ONE;
    for (uint64_t i = 1; i < n - (uint64_t)bf; i++) fr_mul(&z[i], &z[i - 1], &prod[i - 1]);
    for (uint64_t i = n - (uint64_t)bf; i < n; i++) prng_random(rng, &z[i]);
}

/* ====================================================================== keygen */
typedef struct { fe point; int poly_id; } query_ref;

/* ProvingKey restated (plonk.rs ProvingKey + permutation::ProvingKey), plus the
 * ConstraintSystem facts the prover needs.  Circuit arrays stay owned by the caller. */
typedef struct {
    uint32_t k;
    uint64_t n, ext, rot_scale;
    int degree, bf, P;
    qlist adv_q, fix_q, ins_q;
    domain_t D;
    fe **fixed_polys, **fixed_cosets;
    fe *l0, *l_last, *l_active;
    fe **sigma_lag, **sigma_polys, **sigma_cosets;
} or_pk;

void or_pk_free(or_pk *pk);

or_pk *or_keygen(const or_spec *s, int threads) {   /* keygen_vk + keygen_pk (keygen.rs:43-190) */
    if (threads < 1) threads = 1;
    const uint32_t k = s->k;
    const uint64_t n = 1ULL << k;
    int degree = 3;  /* permutation_argument_required_degree (circuit.rs:292-320) */
    {   /* lookup_argument_required_degree / shuffle_argument_required_degree (circuit.rs:327-389) */
        const int32_t *r = s->lookup_roots;
        for (uint32_t l = 0; l < s->num_lookups; l++) {
            int m = (int)s->lookup_sizes[l], di = 1, dt = 1;
            for (int i = 0; i < m; i++) { int d = node_degree(s, r[i]); if (d > di) di = d; }
            for (int i = 0; i < m; i++) { int d = node_degree(s, r[m + i]); if (d > dt) dt = d; }
            int need = 2 + di + dt > 4 ? 2 + di + dt : 4;
            if (need > degree) degree = need;
            r += 2 * m;
        }
        r = s->shuffle_roots;
        for (uint32_t l = 0; l < s->num_shuffles; l++) {
            int m = (int)s->shuffle_sizes[l], di = 1, ds = 1;
            for (int i = 0; i < m; i++) { int d = node_degree(s, r[i]); if (d > di) di = d; }
            for (int i = 0; i < m; i++) { int d = node_degree(s, r[m + i]); if (d > ds) ds = d; }
            int need = 2 + (di > ds ? di : ds);
            if (need > degree) degree = need;
            r += 2 * m;
        }
    }
    for (uint32_t g = 0; g < s->num_gates; g++) { int dg = node_degree(s, s->gate_roots[g]); if (dg > degree) degree = dg; }
    qlist adv_q = {0}, fix_q = {0}, ins_q = {0};
    for (uint32_t g = 0; g < s->num_gates; g++) collect_queries(s, s->gate_roots[g], &adv_q, &fix_q, &ins_q);
    {   /* lookups then shuffles (keygen.rs:266-321), each input expressions then tables */
        const int32_t *r = s->lookup_roots;
        for (uint32_t l = 0; l < s->num_lookups; l++) {
            for (uint32_t i = 0; i < 2 * s->lookup_sizes[l]; i++) collect_queries(s, r[i], &adv_q, &fix_q, &ins_q);
            r += 2 * s->lookup_sizes[l];
        }
        r = s->shuffle_roots;
        for (uint32_t l = 0; l < s->num_shuffles; l++) {
            for (uint32_t i = 0; i < 2 * s->shuffle_sizes[l]; i++) collect_queries(s, r[i], &adv_q, &fix_q, &ins_q);
            r += 2 * s->shuffle_sizes[l];
        }
    }
    for (uint32_t i = 0; i < s->num_perm_columns; i++) {
        int t = s->perm_columns[2 * i], idx = s->perm_columns[2 * i + 1];
        qlist_add(t == COL_ADVICE ? &adv_q : (t == COL_FIXED ? &fix_q : &ins_q), t, idx, 0);
    }
    int max_q = 1;
    {
        int *cnt = (int *)calloc(s->num_advice + 1, sizeof(int));
        for (int i = 0; i < adv_q.n; i++) cnt[adv_q.q[i].index]++;
        if (s->num_advice) { max_q = 0; for (uint32_t i = 0; i < s->num_advice; i++) if (cnt[i] > max_q) max_q = cnt[i]; }
        free(cnt);
    }
    const int bf = (max_q > 3 ? max_q : 3) + 2;   /* circuit.rs:143-170 */
    if ((int64_t)n < bf + 3) return NULL;          /* minimum_rows */
    or_pk *pk = (or_pk *)calloc(1, sizeof(or_pk));
    pk->k = k; pk->n = n; pk->degree = degree; pk->bf = bf;
    pk->adv_q = adv_q; pk->fix_q = fix_q; pk->ins_q = ins_q;
    domain_new(&pk->D, (uint32_t)degree, k);
    const domain_t *D = &pk->D;
    const uint64_t ext = 1ULL << D->extended_k;
    pk->ext = ext;
    pk->rot_scale = 1ULL << (D->extended_k - k);

    pk->fixed_polys = (fe **)calloc(s->num_fixed + 1, sizeof(fe *));
    pk->fixed_cosets = (fe **)calloc(s->num_fixed + 1, sizeof(fe *));
    for (uint32_t i = 0; i < s->num_fixed; i++) {
        pk->fixed_polys[i] = fr_alloc(n);
        memcpy(pk->fixed_polys[i], s->fixed_values + 4 * n * i, n * 32);
        lagrange_to_coeff_d(D, pk->fixed_polys[i], threads);
        pk->fixed_cosets[i] = fr_alloc(ext);
        coeff_to_extended_d(D, pk->fixed_polys[i], pk->fixed_cosets[i], threads);
    }
    pk->l0 = fr_alloc(ext); pk->l_last = fr_alloc(ext); pk->l_active = fr_alloc(ext);
    {
        fe *t = fr_alloc(n);
        t[0] = fr_ONE; lagrange_to_coeff_d(D, t, threads); coeff_to_extended_d(D, t, pk->l0, threads);
        fe *lb = fr_alloc(ext);
        memset(t, 0, n * 32);
        for (int i = 0; i < bf; i++) t[n - 1 - i] = fr_ONE;
        lagrange_to_coeff_d(D, t, threads); coeff_to_extended_d(D, t, lb, threads);
        memset(t, 0, n * 32);
        t[n - bf - 1] = fr_ONE;
        lagrange_to_coeff_d(D, t, threads); coeff_to_extended_d(D, t, pk->l_last, threads);
        for (uint64_t i = 0; i < ext; i++) { fe a; fr_add(&a, &pk->l_last[i], &lb[i]); fr_sub(&pk->l_active[i], &fr_ONE, &a); }
        free(t); free(lb);
    }
    /* permutation keygen (permutation/keygen.rs:16-213) */
    const int P = (int)s->num_perm_columns;
    pk->P = P;
    assembly_t A; A.cols = P; A.n = n;
    A.mapping = (cell_t *)malloc((size_t)P * n * sizeof(cell_t) + 1);
    A.aux = (cell_t *)malloc((size_t)P * n * sizeof(cell_t) + 1);
    A.sizes = (uint64_t *)malloc((size_t)P * n * sizeof(uint64_t) + 1);
    for (int c = 0; c < P; c++)
        for (uint64_t r = 0; r < n; r++) {
            A.mapping[c * n + r] = (cell_t){c, (int)r}; A.aux[c * n + r] = (cell_t){c, (int)r}; A.sizes[c * n + r] = 1;
        }
    for (uint32_t i = 0; i < s->num_copies; i++) {
        const int32_t *cp = s->copies + 6 * i;
        int lc = perm_col_pos(s, cp[0], cp[1]), rc = perm_col_pos(s, cp[3], cp[4]);
        if (lc < 0 || rc < 0 || cp[2] < 0 || cp[5] < 0 || cp[2] >= (int)n || cp[5] >= (int)n) {
            free(A.mapping); free(A.aux); free(A.sizes); or_pk_free(pk); return NULL;
        }
        assembly_copy(&A, lc, cp[2], rc, cp[5]);
    }
    pk->sigma_lag = (fe **)calloc(P + 1, sizeof(fe *));
    pk->sigma_polys = (fe **)calloc(P + 1, sizeof(fe *));
    pk->sigma_cosets = (fe **)calloc(P + 1, sizeof(fe *));
    {
        fe *omega_pow = fr_alloc(n);
        omega_pow[0] = fr_ONE;
        for (uint64_t j = 1; j < n; j++) fr_mul(&omega_pow[j], &omega_pow[j - 1], &D->omega);
        fe *delta_pow = fr_alloc(P + 1);
        delta_pow[0] = fr_ONE;
        for (int i = 1; i <= P; i++) fr_mul(&delta_pow[i], &delta_pow[i - 1], &FR_DELTA);
        for (int i = 0; i < P; i++) {
            pk->sigma_lag[i] = fr_alloc(n);
            for (uint64_t j = 0; j < n; j++) {
                cell_t m = A.mapping[(uint64_t)i * n + j];
                fr_mul(&pk->sigma_lag[i][j], &delta_pow[m.col], &omega_pow[m.row]);
            }
            pk->sigma_polys[i] = fr_alloc(n);
            memcpy(pk->sigma_polys[i], pk->sigma_lag[i], n * 32);
            lagrange_to_coeff_d(D, pk->sigma_polys[i], threads);
            pk->sigma_cosets[i] = fr_alloc(ext);
            coeff_to_extended_d(D, pk->sigma_polys[i], pk->sigma_cosets[i], threads);
        }
        free(omega_pow); free(delta_pow);
    }
    free(A.mapping); free(A.aux); free(A.sizes);
    return pk;
}

void or_pk_free(or_pk *pk) {
    if (!pk) return;
    for (int i = 0; pk->fixed_polys && pk->fixed_polys[i]; i++) { free(pk->fixed_polys[i]); free(pk->fixed_cosets[i]); }
    free(pk->fixed_polys); free(pk->fixed_cosets);
    free(pk->l0); free(pk->l_last); free(pk->l_active);
    for (int i = 0; i < pk->P && pk->sigma_lag; i++) { free(pk->sigma_lag[i]); free(pk->sigma_polys[i]); free(pk->sigma_cosets[i]); }
    free(pk->sigma_lag); free(pk->sigma_polys); free(pk->sigma_cosets);
    free(pk->adv_q.q); free(pk->fix_q.q); free(pk->ins_q.q);
    domain_free(&pk->D);
    free(pk);
}

/* sizes the verifier side needs */
void or_pk_info(const or_pk *pk, int32_t *out8) {
    out8[0] = pk->degree; out8[1] = pk->bf; out8[2] = (int32_t)pk->D.extended_k; out8[3] = pk->P;
    out8[4] = pk->adv_q.n; out8[5] = pk->fix_q.n; out8[6] = pk->ins_q.n; out8[7] = (pk->P + pk->degree - 3) / (pk->degree - 2);
}
/* sigma values (Lagrange) of permutation column i: the vk commitments are commit_lagrange of these */
void or_pk_sigma(const or_pk *pk, int i, uint64_t *out) { memcpy(out, pk->sigma_lag[i], pk->n * 32); }

/* ====================================================================== create_proof */
/* one circuit's state through create_proof (prover.rs:187-899 keep one of each per circuit:
 * InstanceSingle, AdviceSingle, the permutation / lookup / shuffle arguments) */
typedef struct {
    const uint64_t *advice, *instance;
    const uint32_t *inst_lens;
    fe **inst_vals, **inst_polys, **adv;
    fe **lk_A, **lk_S, **lk_Ap, **lk_Sp, **lk_Ap_poly, **lk_Sp_poly, **lk_z_poly, **sh_z_poly;
    fe **z_poly;
} circ_t;

/* create_proof (prover.rs:174-899) over the spec's circuits.  The witnesses (advice,
 * instance) and the prover inputs (rng, vanishing thread count, SRS) come from `s`. */
int or_prove(const or_pk *pk, const or_spec *s_in, uint8_t *proof, uint64_t proof_cap, uint64_t *proof_len, int threads) {
    if (threads < 1) threads = 1;
    or_spec s_local = *s_in;   /* + the challenge values, once squeezed */
    const or_spec *s = &s_local;
    const uint32_t k = pk->k;
    const uint64_t n = pk->n, ext = pk->ext, rot_scale = pk->rot_scale;
    const int degree = pk->degree, bf = pk->bf, P = pk->P;
    const domain_t D = pk->D;
    const qlist adv_q = pk->adv_q, fix_q = pk->fix_q;
    fe *const *fixed_polys = pk->fixed_polys, *const *fixed_cosets = pk->fixed_cosets;
    fe *const *sigma_lag = pk->sigma_lag, *const *sigma_polys = pk->sigma_polys, *const *sigma_cosets = pk->sigma_cosets;
    const fe *l0 = pk->l0, *l_last = pk->l_last, *l_active = pk->l_active;
    const int NL = (int)s->num_lookups, NS = (int)s->num_shuffles;
    const int NC = s->num_circuits ? (int)s->num_circuits : 1;
    circ_t *C = (circ_t *)calloc(NC, sizeof(circ_t));
    for (int ci = 0; ci < NC; ci++) {
        C[ci].advice = s->num_circuits ? s->advice_c[ci] : s->advice_values;
        C[ci].instance = s->num_circuits ? (s->instance_c ? s->instance_c[ci] : NULL) : s->instance_values;
        C[ci].inst_lens = s->num_circuits ? (s->instance_lens_c ? s->instance_lens_c[ci] : NULL) : s->instance_lens;
    }

    prng_t rng = {0};
    chacha_rng_init(&rng.cc, s->rng_seed ? s->rng_seed : (const uint8_t *)"\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0\0");
    rng.fb = s->rng_fill_bytes; rng.fr = s->rng_random_fr; rng.ctx = s->rng_ctx;
    transcript_t T; tr_init(&T, (int)s->transcript, proof, proof_cap);
    { fe tr = fe_from(s->transcript_repr); tr_common_scalar(&T, &tr); }       /* vk.hash_into */
    /* every circuit's instances (prover.rs:187-271; KZG: QUERY_INSTANCE = false) */
    for (int ci = 0; ci < NC; ci++) {
        circ_t *c = &C[ci];
        c->inst_vals = (fe **)calloc(s->num_instance + 1, sizeof(fe *));
        c->inst_polys = (fe **)calloc(s->num_instance + 1, sizeof(fe *));
        for (uint32_t i = 0; i < s->num_instance; i++) {
            if (c->inst_lens[i] > n - (bf + 1)) return -4;   /* InstanceTooLarge */
            c->inst_vals[i] = fr_alloc(n);
            memcpy(c->inst_vals[i], c->instance + 4 * n * i, n * 32);
            for (uint32_t r = 0; r < c->inst_lens[i]; r++) tr_common_scalar(&T, &c->inst_vals[i][r]);
            c->inst_polys[i] = fr_alloc(n);
            memcpy(c->inst_polys[i], c->inst_vals[i], n * 32);
            lagrange_to_coeff_d(&D, c->inst_polys[i], threads);
        }
    }
    /* commit_phase per advice phase (prover.rs:309-494), circuit by circuit: the phase's
     * blinding rows, its blinds, its commitments; then the challenges of the phase */
    const uint64_t unusable = n - (uint64_t)(bf + 1);
    int max_phase = 0;
    for (uint32_t c = 0; c < s->num_advice; c++)
        if (s->advice_phase && s->advice_phase[c] > max_phase) max_phase = s->advice_phase[c];
    uint64_t *ch = (uint64_t *)calloc(4 * (s->num_challenges + 1), sizeof(uint64_t));
    const int has_fill = s->fill || s->fill_multi;
    uint64_t *src = has_fill ? (uint64_t *)calloc(4 * n * (s->num_advice + 1), sizeof(uint64_t)) : NULL;
    for (int ci = 0; ci < NC; ci++) C[ci].adv = (fe **)calloc(s->num_advice + 1, sizeof(fe *));
    for (int ph = 0; ph <= max_phase; ph++) {
#define IN_PHASE(c) ((s->advice_phase ? s->advice_phase[c] : 0) == ph)
        for (int ci = 0; ci < NC; ci++) {
            fe **adv = C[ci].adv;
            const uint64_t *from = C[ci].advice;
            if (has_fill) {
                memset(src, 0, 4 * n * (s->num_advice + 1) * sizeof(uint64_t));
                int rc = s->fill_multi ? s->fill_multi(s->fill_ctx, (uint32_t)ci, (uint32_t)ph, ch, src)
                                       : s->fill(s->fill_ctx, (uint32_t)ph, ch, src);
                if (rc) return -7;
                from = src;
            }
            for (uint32_t c = 0; c < s->num_advice; c++) {
                if (!IN_PHASE(c)) continue;
                adv[c] = fr_alloc(n);
                memcpy(adv[c], from + 4 * n * c, n * 32);
                if (s->unblinded && s->unblinded[c]) continue;
                for (uint64_t r = unusable; r < n; r++) prng_random(&rng, &adv[c][r]);
            }
            for (uint32_t c = 0; c < s->num_advice; c++) {
                if (!IN_PHASE(c) || (s->unblinded && s->unblinded[c])) continue;
                fe blind; prng_random(&rng, &blind);
            }
            for (uint32_t c = 0; c < s->num_advice; c++) {
                if (!IN_PHASE(c)) continue;
                g1a cm; commit_msm(adv[c], n, s->srs_g_lagrange, threads, &cm);
                if (tr_write_point(&T, &cm)) return -5;
            }
        }
        for (uint32_t i = 0; i < s->num_challenges; i++)
            if (s->challenge_phase[i] == ph) { fe v = tr_squeeze(&T); memcpy(ch + 4 * i, &v, 32); }
#undef IN_PHASE
    }
    free(src);
    s_local.challenge_values = ch;
    if (s->challenges_out) memcpy(s->challenges_out, ch, 32 * s->num_challenges);
    fe theta = tr_squeeze(&T);
    /* lookup_commit_permuted, per circuit, per lookup (lookup/prover.rs:64-173) */
    fe **fix_lag = (fe **)calloc(s->num_fixed + 1, sizeof(fe *));
    for (uint32_t i = 0; i < s->num_fixed; i++) fix_lag[i] = (fe *)(s->fixed_values + 4 * n * i);
    for (int ci = 0; ci < NC; ci++) {
        circ_t *c = &C[ci];
        c->lk_A = (fe **)calloc(NL + 1, sizeof(fe *)); c->lk_S = (fe **)calloc(NL + 1, sizeof(fe *));
        c->lk_Ap = (fe **)calloc(NL + 1, sizeof(fe *)); c->lk_Sp = (fe **)calloc(NL + 1, sizeof(fe *));
        c->lk_Ap_poly = (fe **)calloc(NL + 1, sizeof(fe *)); c->lk_Sp_poly = (fe **)calloc(NL + 1, sizeof(fe *));
        c->lk_z_poly = (fe **)calloc(NL + 1, sizeof(fe *)); c->sh_z_poly = (fe **)calloc(NS + 1, sizeof(fe *));
        const int32_t *r = s->lookup_roots;
        for (int l = 0; l < NL; l++) {
            const int m = (int)s->lookup_sizes[l];
            c->lk_A[l] = fr_alloc(n); c->lk_S[l] = fr_alloc(n); c->lk_Ap[l] = fr_alloc(n); c->lk_Sp[l] = fr_alloc(n);
            compress_lagrange(s, r, m, c->adv, fix_lag, c->inst_vals, n, &theta, c->lk_A[l], threads);
            compress_lagrange(s, r + m, m, c->adv, fix_lag, c->inst_vals, n, &theta, c->lk_S[l], threads);
            if (permute_pair(c->lk_A[l], c->lk_S[l], n, bf, &rng, c->lk_Ap[l], c->lk_Sp[l])) return -7;
            fe b1, b2; prng_random(&rng, &b1); prng_random(&rng, &b2);
            g1a c1, c2;
            commit_msm(c->lk_Ap[l], n, s->srs_g_lagrange, threads, &c1);
            commit_msm(c->lk_Sp[l], n, s->srs_g_lagrange, threads, &c2);
            c->lk_Ap_poly[l] = fr_alloc(n); memcpy(c->lk_Ap_poly[l], c->lk_Ap[l], n * 32); lagrange_to_coeff_d(&D, c->lk_Ap_poly[l], threads);
            c->lk_Sp_poly[l] = fr_alloc(n); memcpy(c->lk_Sp_poly[l], c->lk_Sp[l], n * 32); lagrange_to_coeff_d(&D, c->lk_Sp_poly[l], threads);
            if (tr_write_point(&T, &c1) || tr_write_point(&T, &c2)) return -5;
            r += 2 * m;
        }
    }
    fe beta = tr_squeeze(&T), gamma = tr_squeeze(&T);
    /* permutation_commit per circuit (permutation/prover.rs:50-197) */
    const int chunk_len = degree - 2;
    const int nsets = (P + chunk_len - 1) / chunk_len;
    for (int ci = 0; ci < NC; ci++) {
        circ_t *cc = &C[ci];
        fe **adv = cc->adv;
        cc->z_poly = (fe **)calloc(nsets + 1, sizeof(fe *));
        fe deltaomega = fr_ONE, last_z = fr_ONE;
        fe *mod = fr_alloc(n);
        for (int st = 0; st < nsets; st++) {
            int c0 = st * chunk_len, c1 = c0 + chunk_len < P ? c0 + chunk_len : P;
            for (uint64_t r = 0; r < n; r++) mod[r] = fr_ONE;
            for (int c = c0; c < c1; c++) {
                int t = s->perm_columns[2 * c], idx = s->perm_columns[2 * c + 1];
                fe *vals = t == COL_ADVICE ? adv[idx] : (t == COL_FIXED ? (fe *)(s->fixed_values + 4 * n * idx) : cc->inst_vals[idx]);
#pragma omp parallel for num_threads(threads) schedule(static)
                for (uint64_t r = 0; r < n; r++) {
                    fe a, b; fr_mul(&a, &beta, &sigma_lag[c][r]); fr_add(&a, &a, &gamma); fr_add(&b, &a, &vals[r]);
                    fr_mul(&mod[r], &mod[r], &b);
                }
            }
            or_fr_batch_invert((uint64_t *)mod, n);
            for (int c = c0; c < c1; c++) {
                int t = s->perm_columns[2 * c], idx = s->perm_columns[2 * c + 1];
                fe *vals = t == COL_ADVICE ? adv[idx] : (t == COL_FIXED ? (fe *)(s->fixed_values + 4 * n * idx) : cc->inst_vals[idx]);
                fe dw = deltaomega;
                for (uint64_t r = 0; r < n; r++) {
                    fe a, b; fr_mul(&a, &dw, &beta); fr_add(&a, &a, &gamma); fr_add(&b, &a, &vals[r]);
                    fr_mul(&mod[r], &mod[r], &b);
                    fr_mul(&dw, &dw, &D.omega);
                }
                fr_mul(&deltaomega, &deltaomega, &FR_DELTA);
            }
            fe *z = fr_alloc(n);
            z[0] = last_z;
            for (uint64_t r = 1; r < n; r++) fr_mul(&z[r], &z[r - 1], &mod[r - 1]);
            for (uint64_t r = n - bf; r < n; r++) prng_random(&rng, &z[r]);
            last_z = z[n - (bf + 1)];
            fe blind; prng_random(&rng, &blind);
            g1a cm; commit_msm(z, n, s->srs_g_lagrange, threads, &cm);
            lagrange_to_coeff_d(&D, z, threads);
            cc->z_poly[st] = z;
            if (tr_write_point(&T, &cm)) return -5;
        }
        free(mod);
    }
    /* lookup products, every circuit's (lookup/prover.rs:182-325), then shuffle products
     * (shuffle/prover.rs:97-206) */
    {
        fe *prod = fr_alloc(n);
        for (int ci = 0; ci < NC; ci++) {
            circ_t *c = &C[ci];
            for (int l = 0; l < NL; l++) {
#pragma omp parallel for num_threads(threads) schedule(static)
                for (uint64_t i = 0; i < n; i++) {
                    fe a, b; fr_add(&a, &beta, &c->lk_Ap[l][i]); fr_add(&b, &gamma, &c->lk_Sp[l][i]); fr_mul(&prod[i], &a, &b);
                }
                or_fr_batch_invert((uint64_t *)prod, n);
#pragma omp parallel for num_threads(threads) schedule(static)
                for (uint64_t i = 0; i < n; i++) {
                    fe a, b; fr_add(&a, &c->lk_A[l][i], &beta); fr_add(&b, &c->lk_S[l][i], &gamma);
                    fr_mul(&prod[i], &prod[i], &a); fr_mul(&prod[i], &prod[i], &b);
                }
                fe *z = fr_alloc(n);
                grand_product(prod, n, bf, &rng, z);
                fe blind; prng_random(&rng, &blind);
                g1a cm; commit_msm(z, n, s->srs_g_lagrange, threads, &cm);
                lagrange_to_coeff_d(&D, z, threads);
                c->lk_z_poly[l] = z;
                if (tr_write_point(&T, &cm)) return -5;
            }
        }
        fe *ci_ = fr_alloc(n), *cs_ = fr_alloc(n);
        for (int ci = 0; ci < NC; ci++) {
            circ_t *c = &C[ci];
            const int32_t *r = s->shuffle_roots;
            for (int l = 0; l < NS; l++) {
                const int m = (int)s->shuffle_sizes[l];
                compress_lagrange(s, r, m, c->adv, fix_lag, c->inst_vals, n, &theta, ci_, threads);
                compress_lagrange(s, r + m, m, c->adv, fix_lag, c->inst_vals, n, &theta, cs_, threads);
                for (uint64_t i = 0; i < n; i++) fr_add(&prod[i], &gamma, &cs_[i]);
                or_fr_batch_invert((uint64_t *)prod, n);
                for (uint64_t i = 0; i < n; i++) { fe a; fr_add(&a, &gamma, &ci_[i]); fr_mul(&prod[i], &prod[i], &a); }
                fe *z = fr_alloc(n);
                grand_product(prod, n, bf, &rng, z);
                fe blind; prng_random(&rng, &blind);
                g1a cm; commit_msm(z, n, s->srs_g_lagrange, threads, &cm);
                lagrange_to_coeff_d(&D, z, threads);
                c->sh_z_poly[l] = z;
                if (tr_write_point(&T, &cm)) return -5;
                r += 2 * m;
            }
        }
        free(prod); free(ci_); free(cs_);
    }
    /* vanishing::Argument::commit (vanishing/prover.rs:40-98) */
    fe *random_poly = fr_alloc(n);
    {
        uint64_t nt = s->vanishing_threads ? s->vanishing_threads : 1;
        uint64_t chunk = n / nt, rem = n % nt;
        uint64_t noff = 0, *off = (uint64_t *)calloc(nt + 1, sizeof(uint64_t));
        for (uint64_t i = 0; i < rem && noff < nt; i++) off[noff++] = i * (chunk + 1);
        if (chunk) for (uint64_t o = rem * (chunk + 1); noff < nt; o += chunk) off[noff++] = o;
        uint8_t (*seeds)[32] = (uint8_t (*)[32])calloc(noff + 1, 32);
        for (uint64_t i = 0; i < noff; i++) prng_fill(&rng, seeds[i], 32);
        for (uint64_t i = 0; i < noff; i++) {
            uint64_t lo = off[i], hi = i + 1 < noff ? off[i + 1] : n;
            chacha_rng cr; chacha_rng_init(&cr, seeds[i]);
            for (uint64_t r = lo; r < hi; r++) fr_random(&cr, &random_poly[r]);
        }
        free(off); free(seeds);
    }
    fe random_blind; prng_random(&rng, &random_blind); (void)random_blind;
    {
        g1a cm; commit_msm(random_poly, n, s->srs_g, threads, &cm);
        if (tr_write_point(&T, &cm)) return -5;
    }
    /* advice to coefficient form */
    for (int ci = 0; ci < NC; ci++)
        for (uint32_t c = 0; c < s->num_advice; c++) lagrange_to_coeff_d(&D, C[ci].adv[c], threads);
    fe y = tr_squeeze(&T);
    /* evaluate_h (evaluation.rs:317-620): circuit by circuit, each continuing the Horner
     * chain in y of the circuits before it (evaluation.rs:367-373) */
    fe *h = fr_alloc(ext);
    for (int ci = 0; ci < NC; ci++) {
        circ_t *cc = &C[ci];
        fe **adv_c = (fe **)calloc(s->num_advice + 1, sizeof(fe *)), **ins_c = (fe **)calloc(s->num_instance + 1, sizeof(fe *));
        for (uint32_t c = 0; c < s->num_advice; c++) { adv_c[c] = fr_alloc(ext); coeff_to_extended_d(&D, cc->adv[c], adv_c[c], threads); }
        for (uint32_t c = 0; c < s->num_instance; c++) { ins_c[c] = fr_alloc(ext); coeff_to_extended_d(&D, cc->inst_polys[c], ins_c[c], threads); }
        fe **z_coset = (fe **)calloc(nsets + 1, sizeof(fe *));
        for (int st = 0; st < nsets; st++) { z_coset[st] = fr_alloc(ext); coeff_to_extended_d(&D, cc->z_poly[st], z_coset[st], threads); }
        fe **lk_zc = (fe **)calloc(NL + 1, sizeof(fe *)), **lk_Apc = (fe **)calloc(NL + 1, sizeof(fe *));
        fe **lk_Spc = (fe **)calloc(NL + 1, sizeof(fe *)), **sh_zc = (fe **)calloc(NS + 1, sizeof(fe *));
        for (int l = 0; l < NL; l++) {
            lk_zc[l] = fr_alloc(ext); coeff_to_extended_d(&D, cc->lk_z_poly[l], lk_zc[l], threads);
            lk_Apc[l] = fr_alloc(ext); coeff_to_extended_d(&D, cc->lk_Ap_poly[l], lk_Apc[l], threads);
            lk_Spc[l] = fr_alloc(ext); coeff_to_extended_d(&D, cc->lk_Sp_poly[l], lk_Spc[l], threads);
        }
        for (int l = 0; l < NS; l++) { sh_zc[l] = fr_alloc(ext); coeff_to_extended_d(&D, cc->sh_z_poly[l], sh_zc[l], threads); }
        const fe delta_start_beta = beta;   /* delta_start = beta * ZETA */
        fe delta_start; fr_mul(&delta_start, &delta_start_beta, &FR_ZETA);
        const int last_rot = -(bf + 1);
#pragma omp parallel for num_threads(threads) schedule(static)
        for (uint64_t idx = 0; idx < ext; idx++) {
            fe v = h[idx];
            for (uint32_t g = 0; g < s->num_gates; g++) {
                fe gv = eval_node(s, s->gate_roots[g], adv_c, fixed_cosets, ins_c, idx, rot_scale, ext);
                fr_mul(&v, &v, &y); fr_add(&v, &v, &gv);
            }
            if (nsets > 0) {
                uint64_t r_next = (idx + rot_scale) % ext;
                int64_t rl = ((int64_t)idx + (int64_t)last_rot * (int64_t)rot_scale) % (int64_t)ext;
                uint64_t r_last = (uint64_t)(rl < 0 ? rl + (int64_t)ext : rl);
                fe t, u;
                /* l0 (1 - z_0) */
                fr_sub(&t, &fr_ONE, &z_coset[0][idx]); fr_mul(&t, &t, &l0[idx]);
                fr_mul(&v, &v, &y); fr_add(&v, &v, &t);
                /* l_last (z_last^2 - z_last) */
                fe *zl = z_coset[nsets - 1];
                fr_mul(&t, &zl[idx], &zl[idx]); fr_sub(&t, &t, &zl[idx]); fr_mul(&t, &t, &l_last[idx]);
                fr_mul(&v, &v, &y); fr_add(&v, &v, &t);
                for (int st = 1; st < nsets; st++) {
                    fr_sub(&t, &z_coset[st][idx], &z_coset[st - 1][r_last]); fr_mul(&t, &t, &l0[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t);
                }
                fe beta_term = fr_pow_u64(&D.extended_omega, idx), cur;
                fr_mul(&cur, &delta_start, &beta_term);
                for (int st = 0; st < nsets; st++) {
                    int c0 = st * chunk_len, c1 = c0 + chunk_len < P ? c0 + chunk_len : P;
                    fe left = z_coset[st][r_next], right = z_coset[st][idx];
                    for (int c = c0; c < c1; c++) {
                        int tt = s->perm_columns[2 * c], ix = s->perm_columns[2 * c + 1];
                        fe *col = tt == COL_ADVICE ? adv_c[ix] : (tt == COL_FIXED ? fixed_cosets[ix] : ins_c[ix]);
                        fr_mul(&t, &beta, &sigma_cosets[c][idx]); fr_add(&t, &t, &col[idx]); fr_add(&t, &t, &gamma);
                        fr_mul(&left, &left, &t);
                    }
                    for (int c = c0; c < c1; c++) {
                        int tt = s->perm_columns[2 * c], ix = s->perm_columns[2 * c + 1];
                        fe *col = tt == COL_ADVICE ? adv_c[ix] : (tt == COL_FIXED ? fixed_cosets[ix] : ins_c[ix]);
                        fr_add(&t, &col[idx], &cur); fr_add(&t, &t, &gamma);
                        fr_mul(&right, &right, &t);
                        fr_mul(&cur, &cur, &FR_DELTA);
                    }
                    fr_sub(&u, &left, &right); fr_mul(&u, &u, &l_active[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &u);
                }
            }
            {   /* lookups (evaluation.rs:486-558), shuffles (:561-620) */
                uint64_t r_next = (idx + rot_scale) % ext, r_prev = (idx + ext - rot_scale) % ext;
                const int32_t *r = s->lookup_roots;
                for (int l = 0; l < NL; l++) {
                    const int m = (int)s->lookup_sizes[l];
                    fe ci = compress_coset(s, r, m, adv_c, fixed_cosets, ins_c, idx, rot_scale, ext, &theta);
                    fe ct = compress_coset(s, r + m, m, adv_c, fixed_cosets, ins_c, idx, rot_scale, ext, &theta);
                    fe tv, t1, t2, t3;
                    fr_add(&t1, &ci, &beta); fr_add(&t2, &ct, &gamma); fr_mul(&tv, &t1, &t2);
                    const fe zc = lk_zc[l][idx], ap = lk_Apc[l][idx], sp = lk_Spc[l][idx];
                    fe ams; fr_sub(&ams, &ap, &sp);
                    fr_sub(&t1, &fr_ONE, &zc); fr_mul(&t1, &t1, &l0[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    fr_mul(&t1, &zc, &zc); fr_sub(&t1, &t1, &zc); fr_mul(&t1, &t1, &l_last[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    fr_add(&t2, &ap, &beta); fr_add(&t3, &sp, &gamma);
                    fr_mul(&t1, &lk_zc[l][r_next], &t2); fr_mul(&t1, &t1, &t3);
                    fr_mul(&t2, &zc, &tv); fr_sub(&t1, &t1, &t2); fr_mul(&t1, &t1, &l_active[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    fr_mul(&t1, &ams, &l0[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    fr_sub(&t2, &ap, &lk_Apc[l][r_prev]); fr_mul(&t1, &ams, &t2); fr_mul(&t1, &t1, &l_active[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    r += 2 * m;
                }
                r = s->shuffle_roots;
                for (int l = 0; l < NS; l++) {
                    const int m = (int)s->shuffle_sizes[l];
                    fe ci = compress_coset(s, r, m, adv_c, fixed_cosets, ins_c, idx, rot_scale, ext, &theta);
                    fe cs = compress_coset(s, r + m, m, adv_c, fixed_cosets, ins_c, idx, rot_scale, ext, &theta);
                    fr_add(&ci, &ci, &gamma); fr_add(&cs, &cs, &gamma);
                    const fe zc = sh_zc[l][idx];
                    fe t1, t2;
                    fr_sub(&t1, &fr_ONE, &zc); fr_mul(&t1, &t1, &l0[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    fr_mul(&t1, &zc, &zc); fr_sub(&t1, &t1, &zc); fr_mul(&t1, &t1, &l_last[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    fr_mul(&t1, &sh_zc[l][r_next], &cs); fr_mul(&t2, &zc, &ci); fr_sub(&t1, &t1, &t2);
                    fr_mul(&t1, &t1, &l_active[idx]);
                    fr_mul(&v, &v, &y); fr_add(&v, &v, &t1);
                    r += 2 * m;
                }
            }
            h[idx] = v;
        }
        for (int l = 0; l < NL; l++) { free(lk_zc[l]); free(lk_Apc[l]); free(lk_Spc[l]); }
        for (int l = 0; l < NS; l++) free(sh_zc[l]);
        for (int st = 0; st < nsets; st++) free(z_coset[st]);
        free(lk_zc); free(lk_Apc); free(lk_Spc); free(sh_zc); free(z_coset);
        for (uint32_t c = 0; c < s->num_advice; c++) free(adv_c[c]);
        for (uint32_t c = 0; c < s->num_instance; c++) free(ins_c[c]);
        free(adv_c); free(ins_c);
    }
    /* vanishing.construct (vanishing/prover.rs:102-155) */
    const int npieces = degree - 1;
    fe **pieces = (fe **)calloc(npieces + 1, sizeof(fe *));
    {
        for (uint64_t i = 0; i < ext; i++) fr_mul(&h[i], &h[i], &D.t_evaluations[i % D.t_len]);
        fe *hc = fr_alloc(n * npieces);
        or_extended_to_coeff((uint64_t *)h, (uint64_t *)hc, (uint32_t)degree, k, kt(threads));
        for (int p = 0; p < npieces; p++) { pieces[p] = fr_alloc(n); memcpy(pieces[p], hc + n * p, n * 32); }
        free(hc);
        for (int p = 0; p < npieces; p++) { fe b; prng_random(&rng, &b); }
        for (int p = 0; p < npieces; p++) {
            g1a cm; commit_msm(pieces[p], n, s->srs_g, threads, &cm);
            if (tr_write_point(&T, &cm)) return -5;
        }
    }
    free(h);
    if (rng.failed) return -8;   /* the caller's RNG failed */
    fe x = tr_squeeze(&T);
    fe xn = fr_pow_u64(&x, n);
    const fe x_next = rotate_omega(&D, &x, 1), x_last = rotate_omega(&D, &x, -(bf + 1));
    const fe x_prev = rotate_omega(&D, &x, -1);
    /* evaluations (prover.rs:735-836): every circuit's advice, fixed, vanishing, common
     * permutation, then every circuit's permutation, lookups, shuffles */
    for (int ci = 0; ci < NC; ci++)
        for (int i = 0; i < adv_q.n; i++) {
            fe pt = rotate_omega(&D, &x, adv_q.q[i].rot), e = eval_poly(C[ci].adv[adv_q.q[i].index], n, &pt);
            tr_write_scalar(&T, &e);
        }
    for (int i = 0; i < fix_q.n; i++) {
        fe pt = rotate_omega(&D, &x, fix_q.q[i].rot), e = eval_poly(fixed_polys[fix_q.q[i].index], n, &pt);
        tr_write_scalar(&T, &e);
    }
    fe *h_poly = fr_alloc(n);   /* h(X) = sum_p x^{n p} piece_p (vanishing/prover.rs:166-170) */
    for (int p = npieces - 1; p >= 0; p--)
        for (uint64_t i = 0; i < n; i++) { fe t; fr_mul(&t, &h_poly[i], &xn); fr_add(&h_poly[i], &t, &pieces[p][i]); }
    { fe e = eval_poly(random_poly, n, &x); tr_write_scalar(&T, &e); }
    for (int c = 0; c < P; c++) { fe e = eval_poly(sigma_polys[c], n, &x); tr_write_scalar(&T, &e); }
    for (int ci = 0; ci < NC; ci++)
        for (int st = 0; st < nsets; st++) {
            fe *zp = C[ci].z_poly[st];
            fe e0 = eval_poly(zp, n, &x), e1 = eval_poly(zp, n, &x_next);
            tr_write_scalar(&T, &e0); tr_write_scalar(&T, &e1);
            if (st + 1 < nsets) { fe e2 = eval_poly(zp, n, &x_last); tr_write_scalar(&T, &e2); }
        }
    for (int ci = 0; ci < NC; ci++)
        for (int l = 0; l < NL; l++) {   /* lookup/prover.rs:330-361 */
            circ_t *c = &C[ci];
            fe e[5] = {eval_poly(c->lk_z_poly[l], n, &x), eval_poly(c->lk_z_poly[l], n, &x_next), eval_poly(c->lk_Ap_poly[l], n, &x),
                       eval_poly(c->lk_Ap_poly[l], n, &x_prev), eval_poly(c->lk_Sp_poly[l], n, &x)};
            for (int i = 0; i < 5; i++) tr_write_scalar(&T, &e[i]);
        }
    for (int ci = 0; ci < NC; ci++)
        for (int l = 0; l < NS; l++) {   /* shuffle/prover.rs:210-231 */
            fe e0 = eval_poly(C[ci].sh_z_poly[l], n, &x), e1 = eval_poly(C[ci].sh_z_poly[l], n, &x_next);
            tr_write_scalar(&T, &e0); tr_write_scalar(&T, &e1);
        }
    /* queries (prover.rs:840-889) -- poly ids: per circuit ci (base ci * per_c) advice c,
       z st, lookup l (z, A', S'), shuffle l; then fixed, sigma, h, random */
    const int A_ = (int)s->num_advice, F_ = (int)s->num_fixed;
    const int per_c = A_ + nsets + 3 * NL + NS;
    const int id_fix = NC * per_c, id_sig = id_fix + F_, id_h = id_sig + P, id_r = id_h + 1, npolys = id_r + 1;
    fe **polys = (fe **)calloc(npolys, sizeof(fe *));
    for (int ci = 0; ci < NC; ci++) {
        const int b = ci * per_c;
        for (int c = 0; c < A_; c++) polys[b + c] = C[ci].adv[c];
        for (int st = 0; st < nsets; st++) polys[b + A_ + st] = C[ci].z_poly[st];
        for (int l = 0; l < NL; l++) {
            polys[b + A_ + nsets + 3 * l] = C[ci].lk_z_poly[l];
            polys[b + A_ + nsets + 3 * l + 1] = C[ci].lk_Ap_poly[l];
            polys[b + A_ + nsets + 3 * l + 2] = C[ci].lk_Sp_poly[l];
        }
        for (int l = 0; l < NS; l++) polys[b + A_ + nsets + 3 * NL + l] = C[ci].sh_z_poly[l];
    }
    for (int c = 0; c < F_; c++) polys[id_fix + c] = fixed_polys[c];
    for (int c = 0; c < P; c++) polys[id_sig + c] = sigma_polys[c];
    polys[id_h] = h_poly; polys[id_r] = random_poly;
    int nq = 0, qcap = NC * (adv_q.n + 3 * nsets + 5 * NL + 2 * NS) + fix_q.n + P + 2;
    query_ref *Q = (query_ref *)calloc(qcap, sizeof(query_ref));
    for (int ci = 0; ci < NC; ci++) {
        const int b = ci * per_c, id_z = b + A_, id_lk = b + A_ + nsets, id_sh = id_lk + 3 * NL;
        for (int i = 0; i < adv_q.n; i++) { Q[nq].point = rotate_omega(&D, &x, adv_q.q[i].rot); Q[nq++].poly_id = b + adv_q.q[i].index; }
        for (int st = 0; st < nsets; st++) {
            Q[nq].point = x; Q[nq++].poly_id = id_z + st;
            Q[nq].point = x_next; Q[nq++].poly_id = id_z + st;
        }
        for (int st = nsets - 2; st >= 0; st--) { Q[nq].point = x_last; Q[nq++].poly_id = id_z + st; }
        for (int l = 0; l < NL; l++) {   /* lookup/prover.rs:364-405 */
            const int zi = id_lk + 3 * l;
            Q[nq].point = x; Q[nq++].poly_id = zi;
            Q[nq].point = x; Q[nq++].poly_id = zi + 1;
            Q[nq].point = x; Q[nq++].poly_id = zi + 2;
            Q[nq].point = x_prev; Q[nq++].poly_id = zi + 1;
            Q[nq].point = x_next; Q[nq++].poly_id = zi;
        }
        for (int l = 0; l < NS; l++) {   /* shuffle/prover.rs:234-254 */
            Q[nq].point = x; Q[nq++].poly_id = id_sh + l;
            Q[nq].point = x_next; Q[nq++].poly_id = id_sh + l;
        }
    }
    for (int i = 0; i < fix_q.n; i++) { Q[nq].point = rotate_omega(&D, &x, fix_q.q[i].rot); Q[nq++].poly_id = id_fix + fix_q.q[i].index; }
    for (int c = 0; c < P; c++) { Q[nq].point = x; Q[nq++].poly_id = id_sig + c; }
    Q[nq].point = x; Q[nq++].poly_id = id_h;
    Q[nq].point = x; Q[nq++].poly_id = id_r;

    if (s->multiopen == 1) {
        /* ---- ProverGWC::create_proof_with_engine (gwc/prover.rs:40-90): queries grouped by
           point in first-appearance order (construct_intermediate_sets, gwc.rs:25-50); per
           point sum_i v^i (p_i - e_i), divided by (X - z), committed against g ---- */
        fe v = tr_squeeze(&T);
        int *done = (int *)calloc(nq, sizeof(int));
        fe *batch = fr_alloc(n), *q = fr_alloc(n);
        for (int i = 0; i < nq; i++) {
            if (done[i]) continue;
            const fe z = Q[i].point;
            fe evb, vp = fr_ONE;
            memset(&evb, 0, sizeof(evb));
            memset(batch, 0, n * 32);
            for (int j = i; j < nq; j++) {
                if (done[j] || !fe_eq(&Q[j].point, &z)) continue;
                done[j] = 1;
                const fe *pj = polys[Q[j].poly_id];
                fe e = eval_poly(pj, n, &z), t;
                for (uint64_t r = 0; r < n; r++) { fr_mul(&t, &pj[r], &vp); fr_add(&batch[r], &batch[r], &t); }
                fr_mul(&t, &e, &vp); fr_add(&evb, &evb, &t);
                fr_mul(&vp, &vp, &v);
            }
            fr_sub(&batch[0], &batch[0], &evb);   /* poly_batch - eval_batch (Sub<F>, poly.rs:268-276) */
            or_kate_division((uint64_t *)batch, n, z.v, (uint64_t *)q);
            g1a cm; commit_msm(q, n - 1, s->srs_g, threads, &cm);
            if (tr_write_point(&T, &cm)) return -5;
        }
        free(done); free(batch); free(q);
        *proof_len = T.len;
        free(h_poly); free(random_poly);
        return T.len <= proof_cap ? 0 : -6;
    }

    /* ---- SHPLONK (shplonk/prover.rs:121-305, shplonk.rs:48-140) ---- */
    fe sy = tr_squeeze(&T);
    /* super point set (sorted, unique) */
    fe *sps = fr_alloc(nq); int nsp = 0;
    for (int i = 0; i < nq; i++) {
        int found = 0; for (int j = 0; j < nsp; j++) if (fe_eq(&sps[j], &Q[i].point)) { found = 1; break; }
        if (!found) sps[nsp++] = Q[i].point;
    }
    for (int i = 1; i < nsp; i++) for (int j = i; j > 0 && fe_cmp_canon(&sps[j - 1], &sps[j]) > 0; j--) { fe t = sps[j]; sps[j] = sps[j - 1]; sps[j - 1] = t; }
    /* commitment -> sorted point set, in order of first appearance */
    int *cm_id = (int *)calloc(nq, sizeof(int)), ncm = 0;
    fe **cm_pts = (fe **)calloc(nq, sizeof(fe *)); int *cm_npts = (int *)calloc(nq, sizeof(int));
    for (int i = 0; i < nq; i++) {
        int f = -1; for (int j = 0; j < ncm; j++) if (cm_id[j] == Q[i].poly_id) { f = j; break; }
        if (f < 0) { f = ncm++; cm_id[f] = Q[i].poly_id; cm_pts[f] = fr_alloc(nq); cm_npts[f] = 0; }
        int dup = 0; for (int j = 0; j < cm_npts[f]; j++) if (fe_eq(&cm_pts[f][j], &Q[i].point)) dup = 1;
        if (!dup) {
            fe *pp = cm_pts[f]; int m = cm_npts[f]++; pp[m] = Q[i].point;
            for (int j = m; j > 0 && fe_cmp_canon(&pp[j - 1], &pp[j]) > 0; j--) { fe t = pp[j]; pp[j] = pp[j - 1]; pp[j - 1] = t; }
        }
    }
    /* rotation sets grouped by equal point sets, first appearance order */
    int nrs = 0; int *rs_of = (int *)calloc(ncm, sizeof(int)); int *rs_rep = (int *)calloc(ncm, sizeof(int));
    for (int c = 0; c < ncm; c++) {
        int f = -1;
        for (int r = 0; r < nrs; r++) {
            int rep = rs_rep[r];
            if (cm_npts[rep] != cm_npts[c]) continue;
            int same = 1; for (int j = 0; j < cm_npts[c]; j++) if (!fe_eq(&cm_pts[rep][j], &cm_pts[c][j])) { same = 0; break; }
            if (same) { f = r; break; }
        }
        if (f < 0) { f = nrs++; rs_rep[f] = c; }
        rs_of[c] = f;
    }
    /* low degree equivalents r_i (lagrange_interpolate over each set's points) */
    fe **low = (fe **)calloc(ncm, sizeof(fe *));
    for (int c = 0; c < ncm; c++) {
        int m = cm_npts[c];
        fe *ev = fr_alloc(m);
        for (int j = 0; j < m; j++) ev[j] = eval_poly(polys[cm_id[c]], n, &cm_pts[c][j]);
        low[c] = fr_alloc(m);
        lagrange_interpolate(cm_pts[c], ev, m, low[c]);
        free(ev);
    }
    fe v = tr_squeeze(&T);
    fe *hx = fr_alloc(n);
    {
        fe vpow = fr_ONE;
        fe *nx = fr_alloc(n), *tmp = fr_alloc(n), *q = fr_alloc(n);
        for (int r = 0; r < nrs; r++) {
            memset(nx, 0, n * 32);
            fe ypow = fr_ONE;
            for (int c = 0; c < ncm; c++) {
                if (rs_of[c] != r) continue;
                memcpy(tmp, polys[cm_id[c]], n * 32);
                for (int j = 0; j < cm_npts[c]; j++) fr_sub(&tmp[j], &tmp[j], &low[c][j]);
                for (uint64_t i = 0; i < n; i++) { fe t; fr_mul(&t, &tmp[i], &ypow); fr_add(&nx[i], &nx[i], &t); }
                fr_mul(&ypow, &ypow, &sy);
            }
            /* div_by_vanishing: successive kate_division by each point */
            int rep = rs_rep[r]; uint64_t len = n;
            memcpy(q, nx, n * 32);
            for (int j = 0; j < cm_npts[rep]; j++) {
                fe *qq = fr_alloc(len);
                or_kate_division((uint64_t *)q, len, cm_pts[rep][j].v, (uint64_t *)qq);
                len--; memset(q, 0, n * 32); memcpy(q, qq, len * 32); free(qq);
            }
            for (uint64_t i = 0; i < n; i++) { fe t; fr_mul(&t, &q[i], &vpow); fr_add(&hx[i], &hx[i], &t); }
            fr_mul(&vpow, &vpow, &v);
        }
        free(nx); free(tmp); free(q);
    }
    { g1a cm; commit_msm(hx, n, s->srs_g, threads, &cm); if (tr_write_point(&T, &cm)) return -5; }
    fe u = tr_squeeze(&T);
    fe *lx = fr_alloc(n);
    fe z0 = fr_ONE;
    {
        fe vpow = fr_ONE;
        fe *ls = fr_alloc(n);
        for (int r = 0; r < nrs; r++) {
            int rep = rs_rep[r];
            fe zi = fr_ONE;   /* prod over super points not in this set of (u - p) */
            for (int j = 0; j < nsp; j++) {
                int in = 0; for (int t = 0; t < cm_npts[rep]; t++) if (fe_eq(&cm_pts[rep][t], &sps[j])) in = 1;
                if (in) continue;
                fe d; fr_sub(&d, &u, &sps[j]); fr_mul(&zi, &d, &zi);
            }
            if (r == 0) z0 = zi;
            memset(ls, 0, n * 32);
            fe ypow = fr_ONE;
            for (int c = 0; c < ncm; c++) {
                if (rs_of[c] != r) continue;
                fe reval = eval_poly(low[c], cm_npts[c], &u);
                for (uint64_t i = 0; i < n; i++) {
                    fe t = polys[cm_id[c]][i];
                    if (i == 0) fr_sub(&t, &t, &reval);
                    fr_mul(&t, &t, &ypow); fr_add(&ls[i], &ls[i], &t);
                }
                fr_mul(&ypow, &ypow, &sy);
            }
            for (uint64_t i = 0; i < n; i++) { fe t; fr_mul(&t, &ls[i], &zi); fr_mul(&t, &t, &vpow); fr_add(&lx[i], &lx[i], &t); }
            fr_mul(&vpow, &vpow, &v);
        }
        free(ls);
        fe zt = fr_ONE;
        for (int j = 0; j < nsp; j++) { fe d; fr_sub(&d, &u, &sps[j]); fr_mul(&zt, &d, &zt); }
        for (uint64_t i = 0; i < n; i++) { fe t; fr_mul(&t, &hx[i], &zt); fr_sub(&lx[i], &lx[i], &t); }
    }
    {
        fe *q = fr_alloc(n);
        or_kate_division((uint64_t *)lx, n, u.v, (uint64_t *)q);
        fe zinv; fr_inv(&zinv, &z0);
        for (uint64_t i = 0; i + 1 < n; i++) fr_mul(&q[i], &q[i], &zinv);
        g1a cm; commit_msm(q, n - 1, s->srs_g, threads, &cm);
        if (tr_write_point(&T, &cm)) return -5;
        free(q);
    }
    *proof_len = T.len;
    /* (small per-proof buffers of this test-infrastructure routine are not all
       released; the large ones are) */
    free(lx); free(hx); free(h_poly); free(random_poly); free(ch);
    return T.len <= proof_cap ? 0 : -6;
}

int or_create_proof(const or_spec *s, uint8_t *proof, uint64_t proof_cap, uint64_t *proof_len, int threads) {
    or_pk *pk = or_keygen(s, threads);
    if (!pk) return -2;
    int rc = or_prove(pk, s, proof, proof_cap, proof_len, threads);
    or_pk_free(pk);
    return rc;
}

/* exported helpers for tests */
void or_blake2b(const uint8_t *in, uint64_t len, const uint8_t *personal, uint8_t *out64) {
    blake2b_state S; blake2b_init(&S, 64, personal);
    blake2b_update(&S, in, len);
    blake2b_final_copy(&S, out64);
}
/* pad 0x01: Keccak-256 (Keccak256Write); 0x06: SHA3-256 (pins the permutation) */
void or_keccak(const uint8_t *in, uint64_t len, uint8_t pad, uint8_t *out32) {
    keccak_state S; keccak_init(&S);
    keccak_update(&S, in, len);
    keccak_final_copy(&S, pad, out32);
}
void or_chacha20_block(const uint8_t *key, uint64_t counter, uint8_t *out64) { chacha20_block(key, counter, out64); }
void or_fr_random_stream(const uint8_t *seed, uint64_t count, uint64_t *out) {
    chacha_rng r; chacha_rng_init(&r, seed);
    for (uint64_t i = 0; i < count; i++) fr_random(&r, (fe *)(out + 4 * i));
}

/* g_lagrange_i = [L_i(s)] G, L_i(s) = omega^i (s^n - 1) / (n (s - omega^i))
 * (ParamsKZG::setup, halo2_backend/src/poly/kzg/commitment.rs:92-131) */
void or_srs_lagrange(const uint64_t *s_, uint32_t k, uint64_t *out) {
    static const uint64_t GEN[8] = {0xd35d438dc58f0d9dULL, 0x0a78eb28f5c70b3dULL, 0x666ea36f7879462cULL, 0x0e0a77c19a07df2fULL,
                                    0xa6ba871b8b1e1b3aULL, 0x14f1d651eb8e167bULL, 0xccdd46def0f28c58ULL, 0x1c14ef83340fbe5eULL};
    const uint64_t n = 1ULL << k;
    const fe s = fe_from(s_);
    fe root = FR_ROOT_OF_UNITY;
    for (uint32_t i = k; i < FR_S; i++) fr_sqr(&root, &root);
    fe ninv, mult; fr_from_u64(&ninv, n); fr_inv(&ninv, &ninv);
    mult = fr_pow_u64(&s, n); fr_sub(&mult, &mult, &fr_ONE); fr_mul(&mult, &mult, &ninv);
    g1j g; g1j_from_a(&g, (const g1a *)GEN);
#pragma omp parallel for schedule(dynamic, 16)
    for (uint64_t i = 0; i < n; i++) {
        fe rp = fr_pow_u64(&root, i), d, sc;
        fr_sub(&d, &s, &rp); fr_inv(&d, &d);
        fr_mul(&sc, &mult, &rp); fr_mul(&sc, &sc, &d);
        g1j r; g1j_mul(&r, &g, &sc);
        g1j_to_a((g1a *)(out + 8 * i), &r);
    }
}
