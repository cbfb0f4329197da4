/*
 * hash.h -- BLAKE2b (RFC 7693, with personalisation) and ChaCha20 block function.
 * TEST INFRASTRUCTURE (oracle).  Restates the third-party crates the reference's
 * transcript and RNG use: blake2b_simd 1.x (halo2_backend/src/transcript.rs:120-130,
 * Blake2bWrite personal "Halo2-Transcript") and rand_chacha 0.3 ChaCha20Rng
 * (vanishing/prover.rs:57-81; the prover RNG in the build's tests).
 */
#ifndef ORACLE_HASH_H
#define ORACLE_HASH_H
#include <stdint.h>
#include <string.h>

/* ---------------------------------------------------------------- BLAKE2b */
typedef struct {
    uint64_t h[8];
    uint64_t t[2];
    uint8_t buf[128];
    size_t buflen;
    size_t outlen;
} blake2b_state;

static const uint64_t B2B_IV[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const uint8_t B2B_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
static inline uint64_t load64le(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

static void blake2b_compress(blake2b_state *S, const uint8_t *block, int last) {
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; i++) m[i] = load64le(block + 8 * i);
    for (int i = 0; i < 8; i++) { v[i] = S->h[i]; v[i + 8] = B2B_IV[i]; }
    v[12] ^= S->t[0];
    v[13] ^= S->t[1];
    if (last) v[14] = ~v[14];
#define B2G(a, b, c, d, x, y)            \
    do {                                 \
        v[a] = v[a] + v[b] + (x);        \
        v[d] = rotr64(v[d] ^ v[a], 32);  \
        v[c] = v[c] + v[d];              \
        v[b] = rotr64(v[b] ^ v[c], 24);  \
        v[a] = v[a] + v[b] + (y);        \
        v[d] = rotr64(v[d] ^ v[a], 16);  \
        v[c] = v[c] + v[d];              \
        v[b] = rotr64(v[b] ^ v[c], 63);  \
    } while (0)
    for (int r = 0; r < 12; r++) {
        const uint8_t *s = B2B_SIGMA[r];
        B2G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        B2G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        B2G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        B2G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        B2G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        B2G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        B2G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        B2G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef B2G
    for (int i = 0; i < 8; i++) S->h[i] ^= v[i] ^ v[i + 8];
}

/* outlen bytes, no key, 16-byte personalisation (may be NULL) */
static void blake2b_init(blake2b_state *S, size_t outlen, const uint8_t personal[16]) {
    memset(S, 0, sizeof(*S));
    for (int i = 0; i < 8; i++) S->h[i] = B2B_IV[i];
    S->h[0] ^= 0x01010000ULL ^ (uint64_t)outlen;  /* depth 1, fanout 1, keylen 0 */
    if (personal) {
        S->h[6] ^= load64le(personal);
        S->h[7] ^= load64le(personal + 8);
    }
    S->outlen = outlen;
}

static void blake2b_update(blake2b_state *S, const void *in_, size_t inlen) {
    const uint8_t *in = (const uint8_t *)in_;
    while (inlen > 0) {
        if (S->buflen == 128) {  /* buffer full and more input: compress it (not last) */
            S->t[0] += 128;
            if (S->t[0] < 128) S->t[1]++;
            blake2b_compress(S, S->buf, 0);
            S->buflen = 0;
        }
        size_t take = 128 - S->buflen;
        if (take > inlen) take = inlen;
        memcpy(S->buf + S->buflen, in, take);
        S->buflen += take;
        in += take;
        inlen -= take;
    }
}

/* finalize a COPY (the state stays usable, like blake2b_simd's State::clone().finalize()) */
static void blake2b_final_copy(const blake2b_state *S0, uint8_t *out) {
    blake2b_state S = *S0;
    S.t[0] += S.buflen;
    if (S.t[0] < S.buflen) S.t[1]++;
    memset(S.buf + S.buflen, 0, 128 - S.buflen);
    blake2b_compress(&S, S.buf, 1);
    for (size_t i = 0; i < S.outlen; i++) out[i] = (uint8_t)(S.h[i / 8] >> (8 * (i % 8)));
}

/* ---------------------------------------------------------------- ChaCha20 */
static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* one 64-byte block of ChaCha20 (rand_chacha: 64-bit block counter, 64-bit stream = 0) */
static void chacha20_block(const uint8_t key[32], uint64_t counter, uint8_t out[64]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; i++)
        s[4 + i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
                   ((uint32_t)key[4 * i + 3] << 24);
    s[12] = (uint32_t)counter;
    s[13] = (uint32_t)(counter >> 32);
    s[14] = 0;
    s[15] = 0;
    memcpy(x, s, sizeof(s));
#define QR(a, b, c, d)                 \
    do {                               \
        x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16); \
        x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12); \
        x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);  \
        x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);  \
    } while (0)
    for (int i = 0; i < 10; i++) {
        QR(0, 4, 8, 12); QR(1, 5, 9, 13); QR(2, 6, 10, 14); QR(3, 7, 11, 15);
        QR(0, 5, 10, 15); QR(1, 6, 11, 12); QR(2, 7, 8, 13); QR(3, 4, 9, 14);
    }
#undef QR
    for (int i = 0; i < 16; i++) {
        uint32_t v = x[i] + s[i];
        out[4 * i] = (uint8_t)v; out[4 * i + 1] = (uint8_t)(v >> 8);
        out[4 * i + 2] = (uint8_t)(v >> 16); out[4 * i + 3] = (uint8_t)(v >> 24);
    }
}

/* ChaCha20Rng as a byte stream (next_u64 / fill_bytes consume bytes in order; the
 * build only consumes whole 32-bit words, so rand_core's word buffering agrees) */
typedef struct {
    uint8_t key[32];
    uint64_t counter;
    uint8_t block[64];
    int pos;  /* bytes of `block` consumed; 64 = empty */
} chacha_rng;

static void chacha_rng_init(chacha_rng *r, const uint8_t seed[32]) {
    memcpy(r->key, seed, 32);
    r->counter = 0;
    r->pos = 64;
}
static void chacha_rng_fill(chacha_rng *r, uint8_t *out, size_t len) {
    while (len) {
        if (r->pos == 64) {
            chacha20_block(r->key, r->counter++, r->block);
            r->pos = 0;
        }
        size_t take = 64 - (size_t)r->pos;
        if (take > len) take = len;
        memcpy(out, r->block + r->pos, take);
        r->pos += (int)take;
        out += take;
        len -= take;
    }
}

/* Keccak-256 (the original Keccak padding 0x01 .. 0x80, as the `sha3` crate's Keccak256 used
 * by Keccak256Write, halo2_backend/src/transcript.rs:299-463): Keccak-f[1600], rate 136 bytes.
 * pad = 0x06 gives SHA3-256 (the permutation is pinned against hashlib.sha3_256). */
typedef struct {
    uint64_t a[25];
    uint8_t buf[136];
    size_t fill;
} keccak_state;

static void keccak_f1600(uint64_t a[25]) {
    static const uint64_t RC[24] = {
        0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
        0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
        0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
        0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
        0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
        0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
    static const int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int round = 0; round < 24; round++) {
        uint64_t c[5], d[5], b[25];
        for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; x++) d[x] = c[(x + 4) % 5] ^ ((c[(x + 1) % 5] << 1) | (c[(x + 1) % 5] >> 63));
        for (int i = 0; i < 25; i++) a[i] ^= d[i % 5];
        /* rho + pi: B[y, 2x + 3y] = rot(A[x, y], r[x, y]) (lane index x + 5 y) */
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) {
                const int r = ROT[x + 5 * y];
                const uint64_t v = a[x + 5 * y];
                b[y + 5 * ((2 * x + 3 * y) % 5)] = r ? (v << r) | (v >> (64 - r)) : v;
            }
        for (int y = 0; y < 5; y++)
            for (int x = 0; x < 5; x++) a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= RC[round];
    }
}
static void keccak_absorb_block(keccak_state *S, const uint8_t *blk) {
    for (int i = 0; i < 17; i++) S->a[i] ^= load64le(blk + 8 * i);
    keccak_f1600(S->a);
}
static void keccak_init(keccak_state *S) { memset(S, 0, sizeof(*S)); }
static void keccak_update(keccak_state *S, const void *in_, size_t len) {
    const uint8_t *in = (const uint8_t *)in_;
    while (len) {
        size_t take = 136 - S->fill;
        if (take > len) take = len;
        memcpy(S->buf + S->fill, in, take);
        S->fill += take; in += take; len -= take;
        if (S->fill == 136) { keccak_absorb_block(S, S->buf); S->fill = 0; }
    }
}
/* finalize a COPY (Keccak256::clone().finalize()) */
static void keccak_final_copy(const keccak_state *S0, uint8_t pad, uint8_t out[32]) {
    keccak_state S = *S0;
    memset(S.buf + S.fill, 0, 136 - S.fill);
    S.buf[S.fill] ^= pad;
    S.buf[135] ^= 0x80;
    keccak_absorb_block(&S, S.buf);
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(S.a[i / 8] >> (8 * (i % 8)));
}

#endif
