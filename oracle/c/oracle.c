/*
 * oracle.c -- CPU restatement of the halo2 prover hot path (BN254 / KZG).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the timed
 * CPU baseline ("kind": "port").  The product (yet-another-halo2-fork_amd/,
 * libh2g.so) never links, loads or calls it.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg use it, through ctypes.
 *
 * Every routine cites the reference code it restates (paths relative to the
 * reference snapshot root).  The third-party arithmetic (halo2curves 0.6:
 * best_multiexp / best_fft / bn256) is not vendored in the reference; its
 * published algorithms are restated here.
 *
 * Data layout everywhere: halo2curves in-memory layout -- Fr/Fq Montgomery
 * form, 4 x u64 little-endian limbs; G1Affine = {x[4], y[4]}, identity = (0,0).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "ff.h"

/* ======================================================================
 * G1 in Jacobian coordinates (X/Z^2, Y/Z^3); Z == 0 is the identity.
 * ==================================================================== */
typedef struct { fe x, y; } g1a;          /* affine, identity = (0,0) */
typedef struct { fe x, y, z; } g1j;       /* jacobian */

static inline int g1a_is_id(const g1a *p) { return fe_is_zero(&p->x) && fe_is_zero(&p->y); }
static inline int g1j_is_id(const g1j *p) { return fe_is_zero(&p->z); }
static inline void g1j_set_id(g1j *p) { memset(p, 0, sizeof(*p)); p->x = fq_ONE; p->y = fq_ONE; }
static inline void g1j_from_a(g1j *o, const g1a *p) {
    if (g1a_is_id(p)) { g1j_set_id(o); return; }
    o->x = p->x; o->y = p->y; o->z = fq_ONE;
}

static void g1j_dbl(g1j *o, const g1j *p) {   /* dbl-2009-l, a = 0 */
    if (g1j_is_id(p)) { *o = *p; return; }
    fe A, B, C, D, E, F, t, X3, Y3, Z3;
    fq_sqr(&A, &p->x);
    fq_sqr(&B, &p->y);
    fq_sqr(&C, &B);
    fq_add(&t, &p->x, &B); fq_sqr(&t, &t); fq_sub(&t, &t, &A); fq_sub(&t, &t, &C); fq_dbl(&D, &t);
    fq_dbl(&E, &A); fq_add(&E, &E, &A);
    fq_sqr(&F, &E);
    fq_dbl(&t, &D); fq_sub(&X3, &F, &t);
    fq_sub(&t, &D, &X3); fq_mul(&Y3, &E, &t);
    fq_dbl(&t, &C); fq_dbl(&t, &t); fq_dbl(&t, &t); fq_sub(&Y3, &Y3, &t);
    fq_mul(&Z3, &p->y, &p->z); fq_dbl(&Z3, &Z3);
    o->x = X3; o->y = Y3; o->z = Z3;
}

static void g1j_add(g1j *o, const g1j *p, const g1j *q) {   /* add-2007-bl */
    if (g1j_is_id(p)) { *o = *q; return; }
    if (g1j_is_id(q)) { *o = *p; return; }
    fe z1z1, z2z2, u1, u2, s1, s2, h, i, j, r, v, t;
    fq_sqr(&z1z1, &p->z); fq_sqr(&z2z2, &q->z);
    fq_mul(&u1, &p->x, &z2z2); fq_mul(&u2, &q->x, &z1z1);
    fq_mul(&s1, &p->y, &q->z); fq_mul(&s1, &s1, &z2z2);
    fq_mul(&s2, &q->y, &p->z); fq_mul(&s2, &s2, &z1z1);
    fq_sub(&h, &u2, &u1); fq_sub(&r, &s2, &s1);
    if (fe_is_zero(&h)) {
        if (fe_is_zero(&r)) { g1j_dbl(o, p); return; }
        g1j_set_id(o); return;
    }
    fq_dbl(&r, &r);
    fq_dbl(&i, &h); fq_sqr(&i, &i);
    fq_mul(&j, &h, &i);
    fq_mul(&v, &u1, &i);
    g1j res;
    fq_sqr(&res.x, &r); fq_sub(&res.x, &res.x, &j); fq_dbl(&t, &v); fq_sub(&res.x, &res.x, &t);
    fq_sub(&t, &v, &res.x); fq_mul(&res.y, &r, &t); fq_mul(&t, &s1, &j); fq_dbl(&t, &t); fq_sub(&res.y, &res.y, &t);
    fq_add(&t, &p->z, &q->z); fq_sqr(&t, &t); fq_sub(&t, &t, &z1z1); fq_sub(&t, &t, &z2z2); fq_mul(&res.z, &t, &h);
    *o = res;
}

static void g1j_madd(g1j *o, const g1j *p, const g1a *q) {  /* madd-2007-bl */
    if (g1a_is_id(q)) { *o = *p; return; }
    if (g1j_is_id(p)) { g1j_from_a(o, q); return; }
    fe z1z1, u2, s2, h, hh, i, j, r, v, t;
    fq_sqr(&z1z1, &p->z);
    fq_mul(&u2, &q->x, &z1z1);
    fq_mul(&s2, &q->y, &p->z); fq_mul(&s2, &s2, &z1z1);
    fq_sub(&h, &u2, &p->x); fq_sub(&r, &s2, &p->y);
    if (fe_is_zero(&h)) {
        if (fe_is_zero(&r)) { g1j_dbl(o, p); return; }
        g1j_set_id(o); return;
    }
    fq_dbl(&r, &r);
    fq_sqr(&hh, &h);
    fq_dbl(&i, &hh); fq_dbl(&i, &i);
    fq_mul(&j, &h, &i);
    fq_mul(&v, &p->x, &i);
    g1j res;
    fq_sqr(&res.x, &r); fq_sub(&res.x, &res.x, &j); fq_dbl(&t, &v); fq_sub(&res.x, &res.x, &t);
    fq_sub(&t, &v, &res.x); fq_mul(&res.y, &r, &t); fq_mul(&t, &p->y, &j); fq_dbl(&t, &t); fq_sub(&res.y, &res.y, &t);
    fq_add(&t, &p->z, &h); fq_sqr(&t, &t); fq_sub(&t, &t, &z1z1); fq_sub(&res.z, &t, &hh);
    *o = res;
}

static void g1j_to_a(g1a *o, const g1j *p) {
    if (g1j_is_id(p)) { memset(o, 0, sizeof(*o)); return; }
    fe zi, zi2, zi3;
    fq_inv(&zi, &p->z);
    fq_sqr(&zi2, &zi); fq_mul(&zi3, &zi2, &zi);
    fq_mul(&o->x, &p->x, &zi2); fq_mul(&o->y, &p->y, &zi3);
}

static void g1j_mul(g1j *o, const g1j *p, const fe *scalar_mont) {
    uint64_t k[4];
    fr_to_canonical(k, scalar_mont);
    g1j acc; g1j_set_id(&acc);
    for (int i = 3; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            g1j_dbl(&acc, &acc);
            if ((k[i] >> b) & 1) g1j_add(&acc, &acc, p);
        }
    *o = acc;
}

/* ======================================================================
 * Exported: point helpers
 * ==================================================================== */
int or_g1_is_on_curve(const uint64_t *aff) {
    const g1a *p = (const g1a *)aff;
    if (g1a_is_id(p)) return 1;
    fe y2, x3;
    fq_sqr(&y2, &p->y);
    fq_sqr(&x3, &p->x); fq_mul(&x3, &x3, &p->x); fq_add(&x3, &x3, &FQ_B3);
    return fe_eq(&y2, &x3);
}

/* out = [scalar] P (affine in / out) */
void or_g1_mul(const uint64_t *aff, const uint64_t *scalar, uint64_t *out) {
    g1j p, r;
    g1j_from_a(&p, (const g1a *)aff);
    g1j_mul(&r, &p, (const fe *)scalar);
    g1j_to_a((g1a *)out, &r);
}

void or_g1_add(const uint64_t *a, const uint64_t *b, uint64_t *out) {
    g1j p, q, r;
    g1j_from_a(&p, (const g1a *)a);
    g1j_from_a(&q, (const g1a *)b);
    g1j_add(&r, &p, &q);
    g1j_to_a((g1a *)out, &r);
}

/* g_i = [s^i] G for i < n (ParamsKZG::setup, halo2_backend/src/poly/kzg/commitment.rs:64-90).
 * Serial, O(n) scalar multiplications -- small n only. */
void or_srs_powers(const uint64_t *s, uint64_t n, uint64_t *out) {
    static const uint64_t GEN[8] = {0xd35d438dc58f0d9dULL, 0x0a78eb28f5c70b3dULL, 0x666ea36f7879462cULL, 0x0e0a77c19a07df2fULL,
                                    0xa6ba871b8b1e1b3aULL, 0x14f1d651eb8e167bULL, 0xccdd46def0f28c58ULL, 0x1c14ef83340fbe5eULL};
    g1j g; g1j_from_a(&g, (const g1a *)GEN);
    fe pw = fr_ONE;
#pragma omp parallel for schedule(dynamic, 16)
    for (uint64_t i = 0; i < n; i++) {
        fe e = fr_ONE, base = *(const fe *)s;
        /* s^i by square-and-multiply on i */
        for (int b = 63; b >= 0; b--) {
            fr_sqr(&e, &e);
            if ((i >> b) & 1) fr_mul(&e, &e, &base);
        }
        g1j r; g1j_mul(&r, &g, &e);
        g1j_to_a((g1a *)(out + 8 * i), &r);
    }
    (void)pw;
}

/* ======================================================================
 * MSM
 * ==================================================================== */

/* Naive sum_i [s_i] P_i -- the MsmAccel::msm contract (halo2_middleware/src/zal.rs:58) */
void or_msm_naive(const uint64_t *scalars, const uint64_t *bases, uint64_t n, uint64_t *out_aff) {
    g1j acc; g1j_set_id(&acc);
    for (uint64_t i = 0; i < n; i++) {
        g1j p, r;
        g1j_from_a(&p, (const g1a *)(bases + 8 * i));
        g1j_mul(&r, &p, (const fe *)(scalars + 4 * i));
        g1j_add(&acc, &acc, &r);
    }
    g1j_to_a((g1a *)out_aff, &acc);
}

/* halo2curves msm.rs get_booth_index: Booth window of size c over LE bytes. */
static int32_t booth_index(size_t window_index, size_t window_size, const uint8_t *el, size_t el_len) {
    size_t skip_bits = window_index * window_size;
    skip_bits = skip_bits ? skip_bits - 1 : 0;
    size_t skip_bytes = skip_bits / 8;
    uint8_t v[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < 4 && skip_bytes + i < el_len; i++) v[i] = el[skip_bytes + i];
    uint32_t tmp = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
    if (window_index == 0) tmp <<= 1;
    tmp >>= skip_bits - skip_bytes * 8;
    tmp &= (1u << (window_size + 1)) - 1;
    int sign = (tmp & (1u << window_size)) == 0;
    tmp = (tmp + 1) >> 1;
    if (sign) return (int32_t)tmp;
    return -(int32_t)((~(tmp - 1)) & ((1u << window_size) - 1));
}

/* halo2curves 0.6 msm.rs multiexp_serial: Booth-encoded Pippenger, c = ceil(ln n),
 * buckets as {None, Affine, Projective}, summation by parts. */
static void multiexp_serial(const uint64_t *scalars_mont, const uint64_t *bases, size_t n, g1j *acc) {
    uint64_t *repr = (uint64_t *)malloc(n * 32);
    for (size_t i = 0; i < n; i++) fr_to_canonical(repr + 4 * i, (const fe *)(scalars_mont + 4 * i));
    size_t c;
    if (n < 4) c = 1;
    else if (n < 32) c = 3;
    else c = (size_t)ceil(log((double)n));
    const size_t field_bytes = 32;
    uint8_t acc_or[32] = {0};
    for (size_t i = 0; i < n; i++)
        for (size_t b = 0; b < field_bytes; b++) acc_or[b] |= ((const uint8_t *)(repr + 4 * i))[b];
    size_t max_byte = field_bytes;
    while (max_byte > 0 && acc_or[max_byte - 1] == 0) max_byte--;
    if (max_byte == 0) { free(repr); return; }
    size_t windows = max_byte * 8 / c + 1;
    size_t nb = (size_t)1 << (c - 1);
    g1j *bj = (g1j *)malloc(nb * sizeof(g1j));
    uint8_t *state = (uint8_t *)malloc(nb);  /* 0 None, 1 Affine(in bj.x/y), 2 Projective */
    for (size_t w = windows; w-- > 0;) {
        for (size_t d = 0; d < c; d++) g1j_dbl(acc, acc);
        memset(state, 0, nb);
        for (size_t i = 0; i < n; i++) {
            int32_t idx = booth_index(w, c, (const uint8_t *)(repr + 4 * i), field_bytes);
            if (idx == 0) continue;
            g1a b = *(const g1a *)(bases + 8 * i);
            if (idx < 0 && !g1a_is_id(&b)) fq_neg(&b.y, &b.y);
            size_t k = (size_t)(idx < 0 ? -idx : idx) - 1;
            if (state[k] == 0) { g1j_from_a(&bj[k], &b); state[k] = 1; }
            else { g1j_madd(&bj[k], &bj[k], &b); state[k] = 2; }
        }
        g1j running; g1j_set_id(&running);
        for (size_t k = nb; k-- > 0;) {
            if (state[k]) g1j_add(&running, &running, &bj[k]);
            g1j_add(acc, acc, &running);
        }
    }
    free(state); free(bj); free(repr);
}

/* best_multiexp (halo2curves): split into `threads` chunks, multiexp_serial each, sum.
 * threads == 1 reproduces the single-threaded (no `multicore` feature) reference. */
void or_msm_best(const uint64_t *scalars, const uint64_t *bases, uint64_t n, int threads, uint64_t *out_aff) {
    g1j total; g1j_set_id(&total);
    if (threads < 1) threads = 1;
    if (n > (uint64_t)threads && threads > 1) {
        size_t chunk = n / threads;
        size_t nchunks = (n + chunk - 1) / chunk;
        g1j *res = (g1j *)malloc(nchunks * sizeof(g1j));
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
        for (size_t ci = 0; ci < nchunks; ci++) {
            size_t lo = ci * chunk, len = (lo + chunk <= n) ? chunk : n - lo;
            g1j_set_id(&res[ci]);
            multiexp_serial(scalars + 4 * lo, bases + 8 * lo, len, &res[ci]);
        }
        for (size_t ci = 0; ci < nchunks; ci++) g1j_add(&total, &total, &res[ci]);
        free(res);
    } else {
        multiexp_serial(scalars, bases, n, &total);
    }
    g1j_to_a((g1a *)out_aff, &total);
}

/* ======================================================================
 * FFT: halo2curves fft.rs best_fft -- bit-reverse, twiddles w^i (i < n/2),
 * recursive radix-2 DIT butterflies; natural order in and out.
 * ==================================================================== */
static uint64_t bitrev(uint64_t x, unsigned l) {
    uint64_t r = 0;
    for (unsigned i = 0; i < l; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

static void rec_butterfly(fe *a, size_t n, size_t tw_chunk, const fe *tw, int par_depth) {
    if (n == 2) {
        fe t = a[1];
        fr_sub(&a[1], &a[0], &t);
        fr_add(&a[0], &a[0], &t);
        return;
    }
    size_t h = n / 2;
    if (par_depth > 0) {
#pragma omp task
        rec_butterfly(a, h, tw_chunk * 2, tw, par_depth - 1);
#pragma omp task
        rec_butterfly(a + h, h, tw_chunk * 2, tw, par_depth - 1);
#pragma omp taskwait
    } else {
        rec_butterfly(a, h, tw_chunk * 2, tw, 0);
        rec_butterfly(a + h, h, tw_chunk * 2, tw, 0);
    }
    {
        fe t = a[h];
        fr_sub(&a[h], &a[0], &t);
        fr_add(&a[0], &a[0], &t);
    }
    for (size_t i = 1; i < h; i++) {
        fe t;
        fr_mul(&t, &a[h + i], &tw[i * tw_chunk]);
        fr_sub(&a[h + i], &a[i], &t);
        fr_add(&a[i], &a[i], &t);
    }
}

void or_fft(uint64_t *a_, uint32_t log_n, const uint64_t *omega, int threads) {
    fe *a = (fe *)a_;
    size_t n = (size_t)1 << log_n;
    if (n == 1) return;
    for (size_t k = 0; k < n; k++) {
        size_t rk = bitrev(k, log_n);
        if (k < rk) { fe t = a[k]; a[k] = a[rk]; a[rk] = t; }
    }
    fe *tw = (fe *)malloc((n / 2) * sizeof(fe));
    fe w = fr_ONE;
    for (size_t i = 0; i < n / 2; i++) { tw[i] = w; fr_mul(&w, &w, (const fe *)omega); }
    int depth = 0;
    if (threads > 1) { while ((1 << depth) < threads * 4 && depth < (int)log_n - 1) depth++; }
#ifdef _OPENMP
    if (threads > 1) {
#pragma omp parallel num_threads(threads)
#pragma omp single
        rec_butterfly(a, n, 1, tw, depth);
    } else
#endif
        rec_butterfly(a, n, 1, tw, 0);
    free(tw);
}

/* ======================================================================
 * EvaluationDomain (halo2_backend/src/poly/domain.rs)
 * ==================================================================== */
typedef struct {
    uint32_t k, extended_k;
    uint64_t n, quotient_poly_degree;
    fe omega, omega_inv, extended_omega, extended_omega_inv, g_coset, g_coset_inv;
    fe ifft_divisor, extended_ifft_divisor, barycentric_weight;
    fe *t_evaluations; uint64_t t_len;
} domain_t;

static void domain_new(domain_t *d, uint32_t j, uint32_t k) {   /* domain.rs:38-144 */
    d->quotient_poly_degree = j - 1;
    d->n = 1ULL << k;
    d->k = k;
    uint32_t ek = k;
    while ((1ULL << ek) < d->n * d->quotient_poly_degree) ek++;
    d->extended_k = ek;
    fe eo = FR_ROOT_OF_UNITY;
    for (uint32_t i = ek; i < FR_S; i++) fr_sqr(&eo, &eo);
    d->extended_omega = eo;
    fe o = eo;
    for (uint32_t i = k; i < ek; i++) fr_sqr(&o, &o);
    d->omega = o;
    d->g_coset = FR_ZETA;
    fr_sqr(&d->g_coset_inv, &FR_ZETA);
    d->t_len = 1ULL << (ek - k);
    d->t_evaluations = (fe *)malloc(d->t_len * sizeof(fe));
    uint64_t nexp[4] = {d->n, 0, 0, 0};
    fe orig, step, cur;
    fr_pow(&orig, &FR_ZETA, nexp);
    fr_pow(&step, &eo, nexp);
    cur = orig;
    for (uint64_t i = 0; i < d->t_len; i++) { d->t_evaluations[i] = cur; fr_mul(&cur, &cur, &step); }
    for (uint64_t i = 0; i < d->t_len; i++) { fr_sub(&d->t_evaluations[i], &d->t_evaluations[i], &fr_ONE); fr_inv(&d->t_evaluations[i], &d->t_evaluations[i]); }
    fr_from_u64(&d->ifft_divisor, 1ULL << k); fr_inv(&d->ifft_divisor, &d->ifft_divisor);
    fr_from_u64(&d->extended_ifft_divisor, 1ULL << ek); fr_inv(&d->extended_ifft_divisor, &d->extended_ifft_divisor);
    fr_from_u64(&d->barycentric_weight, d->n); fr_inv(&d->barycentric_weight, &d->barycentric_weight);
    fr_inv(&d->extended_omega_inv, &eo);
    fr_inv(&d->omega_inv, &o);
}
static void domain_free(domain_t *d) { free(d->t_evaluations); }

/* Expose the constants (9 Fr values) + t_evaluations so tests can pin them. */
uint32_t or_domain_constants(uint32_t j, uint32_t k, uint64_t *consts9, uint64_t *t_out) {
    domain_t d; domain_new(&d, j, k);
    fe c[9] = {d.omega, d.omega_inv, d.extended_omega, d.extended_omega_inv, d.g_coset, d.g_coset_inv,
               d.ifft_divisor, d.extended_ifft_divisor, d.barycentric_weight};
    memcpy(consts9, c, sizeof(c));
    if (t_out) memcpy(t_out, d.t_evaluations, d.t_len * sizeof(fe));
    uint32_t ek = d.extended_k;
    domain_free(&d);
    return ek;
}

static void distribute_powers_zeta(const domain_t *d, fe *a, uint64_t len, int into_coset) {  /* domain.rs:325-341 */
    fe pw[2];
    if (into_coset) { pw[0] = d->g_coset; pw[1] = d->g_coset_inv; }
    else { pw[0] = d->g_coset_inv; pw[1] = d->g_coset; }
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < len; i++) {
        uint64_t r = i % 3;
        if (r) fr_mul(&a[i], &a[i], &pw[r - 1]);
    }
}

static void ifft_scale(fe *a, uint64_t len, const fe *div) {   /* domain.rs:343-351 */
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < len; i++) fr_mul(&a[i], &a[i], div);
}

/* lagrange_to_coeff (domain.rs:216-226), in place, length n */
void or_lagrange_to_coeff(uint64_t *a, uint32_t j, uint32_t k, int threads) {
    domain_t d; domain_new(&d, j, k);
    or_fft(a, k, d.omega_inv.v, threads);
    ifft_scale((fe *)a, d.n, &d.ifft_divisor);
    domain_free(&d);
}

/* coeff_to_extended (domain.rs:230-244): in n, out 2^extended_k */
void or_coeff_to_extended(const uint64_t *in, uint64_t *out, uint32_t j, uint32_t k, int threads) {
    domain_t d; domain_new(&d, j, k);
    uint64_t ext = 1ULL << d.extended_k;
    memcpy(out, in, d.n * 32);
    distribute_powers_zeta(&d, (fe *)out, d.n, 1);
    memset(out + 4 * d.n, 0, (ext - d.n) * 32);
    or_fft(out, d.extended_k, d.extended_omega.v, threads);
    domain_free(&d);
}

/* extended_to_coeff (domain.rs:271-293): in 2^extended_k (clobbered), out n*(j-1) */
void or_extended_to_coeff(uint64_t *in, uint64_t *out, uint32_t j, uint32_t k, int threads) {
    domain_t d; domain_new(&d, j, k);
    uint64_t ext = 1ULL << d.extended_k;
    or_fft(in, d.extended_k, d.extended_omega_inv.v, threads);
    ifft_scale((fe *)in, ext, &d.extended_ifft_divisor);
    distribute_powers_zeta(&d, (fe *)in, ext, 0);
    memcpy(out, in, d.n * d.quotient_poly_degree * 32);
    domain_free(&d);
}

/* divide_by_vanishing_poly (domain.rs:297-316), in place on 2^extended_k */
void or_divide_by_vanishing_poly(uint64_t *a_, uint32_t j, uint32_t k) {
    domain_t d; domain_new(&d, j, k);
    fe *a = (fe *)a_;
    uint64_t ext = 1ULL << d.extended_k;
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < ext; i++) fr_mul(&a[i], &a[i], &d.t_evaluations[i % d.t_len]);
    domain_free(&d);
}

/* ======================================================================
 * Polynomial ops / scalar helpers (poly.rs:200-276, arithmetic.rs)
 * ==================================================================== */
void or_fr_add(const uint64_t *a, const uint64_t *b, uint64_t *o, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) fr_add((fe *)(o + 4 * i), (const fe *)(a + 4 * i), (const fe *)(b + 4 * i));
}
void or_fr_sub(const uint64_t *a, const uint64_t *b, uint64_t *o, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) fr_sub((fe *)(o + 4 * i), (const fe *)(a + 4 * i), (const fe *)(b + 4 * i));
}
void or_fr_mul(const uint64_t *a, const uint64_t *b, uint64_t *o, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) fr_mul((fe *)(o + 4 * i), (const fe *)(a + 4 * i), (const fe *)(b + 4 * i));
}
void or_fr_scale(const uint64_t *a, const uint64_t *x, uint64_t *o, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) fr_mul((fe *)(o + 4 * i), (const fe *)(a + 4 * i), (const fe *)x);
}
/* canonical <-> Montgomery conversions for test plumbing */
void or_fr_from_canonical(const uint64_t *c, uint64_t *o, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) fr_from_canonical((fe *)(o + 4 * i), c + 4 * i);
}
void or_fr_to_canonical(const uint64_t *a, uint64_t *c, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) fr_to_canonical(c + 4 * i, (const fe *)(a + 4 * i));
}
void or_fq_from_canonical(const uint64_t *c, uint64_t *o, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) fq_from_canonical((fe *)(o + 4 * i), c + 4 * i);
}

/* eval_polynomial (arithmetic.rs:57-82): Horner from the top coefficient */
void or_fr_eval(const uint64_t *poly, uint64_t n, const uint64_t *x, uint64_t *out) {
    fe acc = {{0, 0, 0, 0}};
    for (uint64_t i = n; i-- > 0;) {
        fr_mul(&acc, &acc, (const fe *)x);
        fr_add(&acc, &acc, (const fe *)(poly + 4 * i));
    }
    memcpy(out, acc.v, 32);
}

/* kate_division (arithmetic.rs:101-120): q = a / (X - b), len(q) = n - 1 */
void or_kate_division(const uint64_t *a, uint64_t n, const uint64_t *b, uint64_t *q) {
    fe nb; fr_neg(&nb, (const fe *)b);
    fe tmp = {{0, 0, 0, 0}};
    for (uint64_t idx = n - 1; idx >= 1; idx--) {
        fe lead;
        fr_sub(&lead, (const fe *)(a + 4 * idx), &tmp);
        memcpy(q + 4 * (idx - 1), lead.v, 32);
        fr_mul(&tmp, &lead, &nb);
    }
}

/* ff::BatchInvert semantics: every nonzero element inverted, zeros stay zero. */
void or_fr_batch_invert(uint64_t *a_, uint64_t n) {
    fe *a = (fe *)a_;
    fe *pref = (fe *)malloc(n * sizeof(fe));
    fe acc = fr_ONE;
    for (uint64_t i = 0; i < n; i++) {
        pref[i] = acc;
        if (!fe_is_zero(&a[i])) fr_mul(&acc, &acc, &a[i]);
    }
    fr_inv(&acc, &acc);
    for (uint64_t i = n; i-- > 0;) {
        if (fe_is_zero(&a[i])) continue;
        fe t;
        fr_mul(&t, &acc, &pref[i]);
        fr_mul(&acc, &acc, &a[i]);
        a[i] = t;
    }
    free(pref);
}

/* running product z_i = prod_{j<=i} a_j (permutation/prover.rs:160-166 shape) */
void or_fr_prefix_product(const uint64_t *a, uint64_t *o, uint64_t n) {
    fe acc = fr_ONE;
    for (uint64_t i = 0; i < n; i++) {
        fr_mul(&acc, &acc, (const fe *)(a + 4 * i));
        memcpy(o + 4 * i, acc.v, 32);
    }
}

int or_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
