/*
 * ff.h -- BN254 Fr / Fq Montgomery arithmetic, 4 x u64 little-endian limbs.
 *
 * TEST INFRASTRUCTURE (oracle): CPU restatement of halo2curves 0.6 bn256
 * field arithmetic (third-party crate, not vendored -- SURVEY 0.2, A.1).
 * Same in-memory layout as halo2curves: Montgomery form, R = 2^256, limbs
 * little-endian; values are always fully reduced (< modulus), so equality is
 * limb equality.  Only tests/, smoke() and bench.py's cpu_baseline may use it.
 */
#ifndef ORACLE_FF_H
#define ORACLE_FF_H
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe;

static inline int fe_is_zero(const fe *a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static inline int fe_eq(const fe *a, const fe *b) { return memcmp(a, b, sizeof(fe)) == 0; }

/* Generic helpers parameterised by modulus (inlined with constant arrays). */
static inline int fe_geq_m(const uint64_t *a, const uint64_t *m) {
    for (int i = 3; i >= 0; i--) {
        if (a[i] > m[i]) return 1;
        if (a[i] < m[i]) return 0;
    }
    return 1;
}
static inline void fe_sub_m(uint64_t *a, const uint64_t *m) {
    u128 br = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a[i] - m[i] - br;
        a[i] = (uint64_t)d;
        br = (d >> 64) & 1;
    }
}
static inline void fe_add_g(fe *o, const fe *a, const fe *b, const uint64_t *m) {
    u128 c = 0;
    uint64_t t[4];
    for (int i = 0; i < 4; i++) {
        c += (u128)a->v[i] + b->v[i];
        t[i] = (uint64_t)c;
        c >>= 64;
    }
    if (fe_geq_m(t, m)) fe_sub_m(t, m);
    memcpy(o->v, t, 32);
}
static inline void fe_sub_g(fe *o, const fe *a, const fe *b, const uint64_t *m) {
    u128 br = 0;
    uint64_t t[4];
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a->v[i] - b->v[i] - br;
        t[i] = (uint64_t)d;
        br = (d >> 64) & 1;
    }
    if (br) {
        u128 c = 0;
        for (int i = 0; i < 4; i++) {
            c += (u128)t[i] + m[i];
            t[i] = (uint64_t)c;
            c >>= 64;
        }
    }
    memcpy(o->v, t, 32);
}
/* CIOS Montgomery multiplication: o = a * b * 2^-256 mod m */
static inline void fe_mul_g(fe *o, const fe *a, const fe *b, const uint64_t *m, uint64_t inv) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)a->v[j] * b->v[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[4] = (uint64_t)c;
        t[5] = (uint64_t)(c >> 64);
        uint64_t q = t[0] * inv;
        c = ((u128)q * m[0] + t[0]) >> 64;
        for (int j = 1; j < 4; j++) {
            c += (u128)q * m[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[3] = (uint64_t)c;
        t[4] = t[5] + (uint64_t)(c >> 64);
    }
    if (t[4] || fe_geq_m(t, m)) fe_sub_m(t, m);
    memcpy(o->v, t, 32);
}

#define DEFINE_FIELD(F, M0, M1, M2, M3, INV, R10, R11, R12, R13, R20, R21, R22, R23)          \
    static const uint64_t F##_MOD[4] = {M0, M1, M2, M3};                                       \
    static const fe F##_ONE = {{R10, R11, R12, R13}};                                          \
    static const fe F##_R2 = {{R20, R21, R22, R23}};                                           \
    static inline void F##_add(fe *o, const fe *a, const fe *b) { fe_add_g(o, a, b, F##_MOD); } \
    static inline void F##_sub(fe *o, const fe *a, const fe *b) { fe_sub_g(o, a, b, F##_MOD); } \
    static inline void F##_mul(fe *o, const fe *a, const fe *b) { fe_mul_g(o, a, b, F##_MOD, INV); } \
    static inline void F##_sqr(fe *o, const fe *a) { fe_mul_g(o, a, a, F##_MOD, INV); }       \
    static inline void F##_dbl(fe *o, const fe *a) { fe_add_g(o, a, a, F##_MOD); }            \
    static inline void F##_neg(fe *o, const fe *a) {                                           \
        fe z = {{0, 0, 0, 0}};                                                                 \
        fe_sub_g(o, &z, a, F##_MOD);                                                           \
    }                                                                                          \
    static inline void F##_from_canonical(fe *o, const uint64_t c[4]) {                        \
        fe t; memcpy(t.v, c, 32); fe_mul_g(o, &t, &F##_R2, F##_MOD, INV);                      \
    }                                                                                          \
    static inline void F##_to_canonical(uint64_t c[4], const fe *a) {                          \
        fe one = {{1, 0, 0, 0}}; fe t; fe_mul_g(&t, a, &one, F##_MOD, INV); memcpy(c, t.v, 32); \
    }                                                                                          \
    static inline void F##_from_u64(fe *o, uint64_t x) {                                       \
        uint64_t c[4] = {x, 0, 0, 0}; F##_from_canonical(o, c);                                \
    }                                                                                          \
    /* exponent given as 4 little-endian u64 limbs, vartime square-and-multiply */              \
    static inline void F##_pow(fe *o, const fe *a, const uint64_t e[4]) {                      \
        fe acc = F##_ONE;                                                                      \
        for (int i = 3; i >= 0; i--)                                                           \
            for (int b = 63; b >= 0; b--) {                                                    \
                F##_sqr(&acc, &acc);                                                           \
                if ((e[i] >> b) & 1) F##_mul(&acc, &acc, a);                                   \
            }                                                                                  \
        *o = acc;                                                                              \
    }                                                                                          \
    static inline void F##_inv(fe *o, const fe *a) { /* Fermat: a^(m-2); inv(0) = 0 */        \
        uint64_t e[4] = {F##_MOD[0] - 2, F##_MOD[1], F##_MOD[2], F##_MOD[3]};                  \
        F##_pow(o, a, e);                                                                      \
    }

DEFINE_FIELD(fr, 0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL,
             0xc2e1f593efffffffULL,
             0xac96341c4ffffffbULL, 0x36fc76959f60cd29ULL, 0x666ea36f7879462eULL, 0x0e0a77c19a07df2fULL,
             0x1bb8e645ae216da7ULL, 0x53fe3ab1e35c59e3ULL, 0x8c49833d53bb8085ULL, 0x0216d0b17f4e44a5ULL)

DEFINE_FIELD(fq, 0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL,
             0x87d20782e4866389ULL,
             0xd35d438dc58f0d9dULL, 0x0a78eb28f5c70b3dULL, 0x666ea36f7879462cULL, 0x0e0a77c19a07df2fULL,
             0xf32cfc5b538afa89ULL, 0xb5e71911d44501fbULL, 0x47ab1eff0a417ff6ULL, 0x06d89f71cab8351fULL)

/* Fr constants (halo2curves bn256::Fr, Montgomery form) -- SURVEY A.1 */
static const fe FR_ROOT_OF_UNITY = {{0x9632c7c5b639feb8ULL, 0x985ce3400d0ff299ULL, 0xb2dd880001b0ecd8ULL, 0x1d69070d6d98ce29ULL}};
static const fe FR_DELTA = {{0x9a0c322befd78855ULL, 0x46e82d14249b563cULL, 0x5983a663e0b0b7a7ULL, 0x22ab452baaa111adULL}};
static const fe FR_ZETA = {{0x93e7cede4a0329b3ULL, 0x7d4fdca77a96c167ULL, 0x8be4ba08b19a750aULL, 0x1cbd5653a5661c25ULL}};
#define FR_S 28

/* G1: y^2 = x^3 + 3 over Fq; b in Montgomery form */
static const fe FQ_B3 = {{0x7a17caa950ad28d7ULL, 0x1f6ac17ae15521b9ULL, 0x334bea4e696bd284ULL, 0x2a1f6744ce179d8eULL}};

#endif
