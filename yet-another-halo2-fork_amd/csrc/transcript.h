// transcript.h -- host-side Fiat-Shamir transcript and prover RNG.
//
//   Blake2bWrite<_, G1Affine, Challenge255>  halo2_backend/src/transcript.rs:120-130,353-419
//   Keccak256Write<_, G1Affine, Challenge255> halo2_backend/src/transcript.rs:299-351,370-463
//     personal "Halo2-Transcript"; absorb prefixes: challenge 0, point 1, scalar 2;
//     squeeze = absorb [0] then finalize a copy of the state -> 64 bytes ->
//     from_uniform_bytes (LE512 mod r).  Points: x, y canonical LE absorbed; the
//     proof stream carries the compressed encoding (x LE, bit 7 of byte 31 = y odd).
//   ChaCha20Rng (rand_chacha 0.3): 20-round ChaCha, 64-bit block counter, stream 0;
//     consumed as a byte stream by Fr::random (64 bytes -> LE512 mod r).
// These run on the host: they are sequential and touch a few KB per proof.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

#include "bn254.h"

namespace h2g {

class Blake2b {
 public:
  explicit Blake2b(const char personal[16]) {
    static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    std::memcpy(h_, iv, sizeof(h_));
    h_[0] ^= 0x01010000ULL ^ 64ULL;  // digest 64, key 0, fanout 1, depth 1
    h_[6] ^= le64(reinterpret_cast<const uint8_t*>(personal));
    h_[7] ^= le64(reinterpret_cast<const uint8_t*>(personal) + 8);
  }
  void update(const void* data, size_t len) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    while (len) {
      if (fill_ == 128) {
        count(128);
        compress(buf_, false);
        fill_ = 0;
      }
      size_t take = 128 - fill_ < len ? 128 - fill_ : len;
      std::memcpy(buf_ + fill_, p, take);
      fill_ += take;
      p += take;
      len -= take;
    }
  }
  // digest of everything absorbed so far; the state keeps absorbing afterwards
  void digest(uint8_t out[64]) const {
    Blake2b c = *this;
    c.count(c.fill_);
    std::memset(c.buf_ + c.fill_, 0, 128 - c.fill_);
    c.compress(c.buf_, true);
    for (int i = 0; i < 64; i++) out[i] = (uint8_t)(c.h_[i / 8] >> (8 * (i % 8)));
  }

 private:
  static uint64_t le64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
  }
  static uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
  void count(size_t n) {
    t_[0] += n;
    if (t_[0] < n) t_[1]++;
  }
  void compress(const uint8_t* block, bool last) {
    static const uint8_t sigma[10][16] = {
        {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
        {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
        {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
        {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
        {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
    static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; i++) m[i] = le64(block + 8 * i);
    for (int i = 0; i < 8; i++) {
      v[i] = h_[i];
      v[8 + i] = iv[i];
    }
    v[12] ^= t_[0];
    v[13] ^= t_[1];
    if (last) v[14] = ~v[14];
    auto G = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
      v[a] += v[b] + x;
      v[d] = rotr(v[d] ^ v[a], 32);
      v[c] += v[d];
      v[b] = rotr(v[b] ^ v[c], 24);
      v[a] += v[b] + y;
      v[d] = rotr(v[d] ^ v[a], 16);
      v[c] += v[d];
      v[b] = rotr(v[b] ^ v[c], 63);
    };
    for (int r = 0; r < 12; r++) {
      const uint8_t* s = sigma[r % 10];
      G(0, 4, 8, 12, m[s[0]], m[s[1]]);
      G(1, 5, 9, 13, m[s[2]], m[s[3]]);
      G(2, 6, 10, 14, m[s[4]], m[s[5]]);
      G(3, 7, 11, 15, m[s[6]], m[s[7]]);
      G(0, 5, 10, 15, m[s[8]], m[s[9]]);
      G(1, 6, 11, 12, m[s[10]], m[s[11]]);
      G(2, 7, 8, 13, m[s[12]], m[s[13]]);
      G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; i++) h_[i] ^= v[i] ^ v[8 + i];
  }
  uint64_t h_[8];
  uint64_t t_[2] = {0, 0};
  uint8_t buf_[128] = {};
  size_t fill_ = 0;
};

// ChaCha20 block: 64 bytes of keystream for (key, 64-bit counter), stream id 0.
// __host__ __device__: the vanishing argument's random polynomial is drawn on the GPU.
__host__ __device__ inline void chacha20_block(const uint32_t key[8], uint64_t counter, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4], key[5], key[6], key[7], (uint32_t)counter, (uint32_t)(counter >> 32), 0u, 0u};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = s[i];
#define H2G_QR(a, b, c, d)                               \
  x[a] += x[b]; x[d] ^= x[a]; x[d] = (x[d] << 16) | (x[d] >> 16); \
  x[c] += x[d]; x[b] ^= x[c]; x[b] = (x[b] << 12) | (x[b] >> 20); \
  x[a] += x[b]; x[d] ^= x[a]; x[d] = (x[d] << 8) | (x[d] >> 24);  \
  x[c] += x[d]; x[b] ^= x[c]; x[b] = (x[b] << 7) | (x[b] >> 25);
#pragma unroll
  for (int r = 0; r < 10; r++) {
    H2G_QR(0, 4, 8, 12) H2G_QR(1, 5, 9, 13) H2G_QR(2, 6, 10, 14) H2G_QR(3, 7, 11, 15)
    H2G_QR(0, 5, 10, 15) H2G_QR(1, 6, 11, 12) H2G_QR(2, 7, 8, 13) H2G_QR(3, 4, 9, 14)
  }
#undef H2G_QR
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

// x mod r for any 256-bit x (2^256 < 6r): conditional subtractions
__host__ __device__ inline Fr reduce_256(Fr x) {
  for (int it = 0; it < 5; it++) {
    uint32_t d[8];
    int64_t br = 0;
    for (int i = 0; i < 8; i++) {
      const int64_t u = (int64_t)x.l[i] - (int64_t)FrParams::M[i] + br;
      d[i] = (uint32_t)u;
      br = u >> 32;
    }
    if (br) break;  // x < r
    for (int i = 0; i < 8; i++) x.l[i] = d[i];
  }
  return x;
}

// from_uniform_bytes: 512-bit little-endian (16 x u32) mod r, Montgomery form out.
// mont(lo) = lo * R2 * R^-1, mont(hi * 2^256) = hi * R3 * R^-1.
__host__ __device__ inline Fr fr_from_u512(const uint32_t w[16]) {
  Fr lo, hi, r2, r3;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    lo.l[i] = w[i];
    hi.l[i] = w[8 + i];
  }
  // R^2 mod r and R^3 mod r (R = 2^256), plain integers
  const uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                          0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  const uint32_t R3[8] = {0xb4bf0040u, 0x5e94d8e1u, 0x1cfbb6b8u, 0x2a489cbeu,
                          0xa19fcfedu, 0x893cc664u, 0x7fcc657cu, 0x0cf8594bu};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r2.l[i] = R2[i];
    r3.l[i] = R3[i];
  }
  // the Montgomery products take operands < r: reduce each 256-bit half (< 6r) first
  return reduce_256(lo) * r2 + reduce_256(hi) * r3;
}

class ChaChaRng {
 public:
  explicit ChaChaRng(const uint8_t seed[32]) {
    for (int i = 0; i < 8; i++) std::memcpy(&key_[i], seed + 4 * i, 4);
  }
  void fill(uint8_t* out, size_t len) {
    while (len) {
      if (pos_ == 64) {
        uint32_t w[16];
        chacha20_block(key_, ctr_++, w);
        std::memcpy(block_, w, 64);
        pos_ = 0;
      }
      size_t take = 64 - pos_ < len ? 64 - pos_ : len;
      std::memcpy(out, block_ + pos_, take);
      pos_ += take;
      out += take;
      len -= take;
    }
  }
  Fr random_fr() {  // Fr::random: 64 bytes -> LE512 mod r
    uint32_t w[16];
    fill(reinterpret_cast<uint8_t*>(w), 64);
    return fr_from_u512(w);
  }
  // bytes of keystream consumed so far, and a jump to any such position
  uint64_t position() const { return ctr_ * 64 - (64 - (uint64_t)pos_); }
  void seek(uint64_t at) {
    ctr_ = at / 64;
    pos_ = 64;
    if (at % 64) {
      uint32_t w[16];
      chacha20_block(key_, ctr_++, w);
      std::memcpy(block_, w, 64);
      pos_ = (size_t)(at % 64);
    }
  }

 private:
  uint32_t key_[8];
  uint64_t ctr_ = 0;
  uint8_t block_[64];
  size_t pos_ = 64;
};

// The prover's `rng: R: RngCore` (halo2_proofs/src/plonk/prover.rs:27,34): either
// ChaCha20Rng::from_seed, or the caller's RNG (h2g_rng): F::random draws through its
// random_fr (or 64 bytes of fill_bytes), seed draws through fill_bytes, in the
// reference's order.  A failed callback latches: later draws return zeros
// and the prover fails the proof once it checks failed().
class ProverRng {
 public:
  using FillFn = int (*)(void*, uint8_t*, size_t);
  using FrFn = int (*)(void*, uint64_t*);
  explicit ProverRng(const uint8_t seed[32]) : cc_(seed) {}
  ProverRng(FillFn fill_bytes, FrFn random, void* ctx) : cc_(kZeroSeed), fb_(fill_bytes), fr_(random), ctx_(ctx) {}
  void fill(uint8_t* out, size_t len) {
    if (!fb_ && !fr_) {
      cc_.fill(out, len);
    } else if (failed_ || !fb_ || fb_(ctx_, out, len) != 0) {
      failed_ = true;
      std::memset(out, 0, len);
    }
    draws_.update(out, len);
  }
  Fr random_fr() {
    if (fr_) {  // the caller's F::random, Montgomery limbs
      uint64_t v[4] = {0, 0, 0, 0};
      if (failed_ || fr_(ctx_, v) != 0) {
        failed_ = true;
        return Fr::zero();
      }
      Fr r;
      std::memcpy(r.l, v, 32);
      draws_.update(v, 32);
      unsigned br = 0;  // an Fr must be below r
      for (int i = 0; i < 8; i++) (void)__builtin_subc(r.l[i], FrParams::M[i], br, &br);
      if (!br) {
        failed_ = true;
        return Fr::zero();
      }
      return r;
    }
    uint32_t w[16];  // from_uniform_bytes of 64 bytes: LE512 mod r
    fill(reinterpret_cast<uint8_t*>(w), 64);
    return fr_from_u512(w);
  }
  bool failed() const { return failed_; }
  // ChaCha20Rng::from_seed only (no caller callbacks): the keystream position, and the
  // bytes a later draw at position `at` will return, without consuming them
  bool seeded() const { return !fb_ && !fr_; }
  uint64_t position() const { return cc_.position(); }
  void peek(uint64_t at, uint8_t* out, size_t len) const {
    ChaChaRng c = cc_;
    c.seek(at);
    c.fill(out, len);
  }
  // digest of every draw so far (SPMD ranks must draw the same values)
  void draws_digest(uint8_t out[64]) const { draws_.digest(out); }

 private:
  static constexpr uint8_t kZeroSeed[32] = {};
  ChaChaRng cc_;
  Blake2b draws_{"h2g-rng-draws\0\0\0"};
  FillFn fb_ = nullptr;
  FrFn fr_ = nullptr;
  void* ctx_ = nullptr;
  bool failed_ = false;
};

// Keccak-256 (the `sha3` crate's Keccak256: Keccak-f[1600], rate 136, padding 0x01..0x80)
class Keccak256 {
 public:
  Keccak256() { std::memset(a_, 0, sizeof(a_)); }
  void update(const void* data, size_t len) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    while (len) {
      size_t take = 136 - fill_ < len ? 136 - fill_ : len;
      std::memcpy(buf_ + fill_, p, take);
      fill_ += take;
      p += take;
      len -= take;
      if (fill_ == 136) {
        absorb(buf_);
        fill_ = 0;
      }
    }
  }
  // digest of a copy (the state stays usable: Keccak256::clone().finalize())
  void digest(uint8_t out[32]) const {
    Keccak256 k = *this;
    std::memset(k.buf_ + k.fill_, 0, 136 - k.fill_);
    k.buf_[k.fill_] ^= 0x01;
    k.buf_[135] ^= 0x80;
    k.absorb(k.buf_);
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(k.a_[i / 8] >> (8 * (i % 8)));
  }

 private:
  static uint64_t rotl(uint64_t v, int r) { return r ? (v << r) | (v >> (64 - r)) : v; }
  void absorb(const uint8_t* blk) {
    for (int i = 0; i < 17; i++) {
      uint64_t w;
      std::memcpy(&w, blk + 8 * i, 8);
      a_[i] ^= w;
    }
    permute();
  }
  void permute() {
    static const uint64_t RC[24] = {
        0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
        0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
        0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
        0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
        0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
        0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
    // rotation of lane x + 5 y (FIPS 202 rho)
    static const int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int round = 0; round < 24; round++) {
      uint64_t c[5], b[25];
      for (int x = 0; x < 5; x++) c[x] = a_[x] ^ a_[x + 5] ^ a_[x + 10] ^ a_[x + 15] ^ a_[x + 20];
      for (int x = 0; x < 5; x++) {
        const uint64_t d = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
        for (int y = 0; y < 25; y += 5) a_[x + y] ^= d;
      }
      for (int x = 0; x < 5; x++)
        for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(a_[x + 5 * y], ROT[x + 5 * y]);
      for (int y = 0; y < 25; y += 5)
        for (int x = 0; x < 5; x++) a_[x + y] = b[x + y] ^ (~b[(x + 1) % 5 + y] & b[(x + 2) % 5 + y]);
      a_[0] ^= RC[round];
    }
  }
  uint64_t a_[25];
  uint8_t buf_[136] = {};
  size_t fill_ = 0;
};

// Blake2bWrite (transcript.rs:120-130,353-419) or Keccak256Write (transcript.rs:299-463):
// the same prefixes absorbed into the growing state; a Keccak256 squeeze absorbs [0], then
// hashes two copies with the extra bytes 10 and 11 (not kept) for the low and high 32 of
// the 64 uniform bytes
enum { TRANSCRIPT_BLAKE2B = 0, TRANSCRIPT_KECCAK256 = 1 };

class Transcript {
 public:
  explicit Transcript(std::vector<uint8_t>* proof, int kind = TRANSCRIPT_BLAKE2B)
      : h_("Halo2-Transcript"), kind_(kind), proof_(proof) {
    if (kind_ == TRANSCRIPT_KECCAK256) k_.update("Halo2-Transcript", 16);
  }
  void common_scalar(const Fr& s) {
    uint8_t b[33];
    b[0] = 2;
    repr(to_canonical(s), b + 1);
    absorb(b, 33);
  }
  void write_scalar(const Fr& s) {
    common_scalar(s);
    uint8_t r[32];
    repr(to_canonical(s), r);
    proof_->insert(proof_->end(), r, r + 32);
  }
  // false for the point at infinity ("cannot write points at infinity to the transcript")
  bool write_point(const G1Affine& p) {
    if (p.x.is_zero() && p.y.is_zero()) return false;
    uint8_t b[65];
    b[0] = 1;
    repr(to_canonical(p.x), b + 1);
    repr(to_canonical(p.y), b + 33);
    absorb(b, 65);
    uint8_t c[32];
    std::memcpy(c, b + 1, 32);
    if (b[33] & 1) c[31] |= 0x80;
    proof_->insert(proof_->end(), c, c + 32);
    return true;
  }
  // digest of everything absorbed so far (SPMD consistency check; the state is unchanged)
  void state_digest(uint8_t out[64]) const {
    std::memset(out, 0, 64);
    if (kind_ == TRANSCRIPT_KECCAK256) k_.digest(out);
    else h_.digest(out);
  }
  Fr squeeze() {
    const uint8_t z = 0;
    absorb(&z, 1);
    uint8_t d[64];
    if (kind_ == TRANSCRIPT_KECCAK256) {
      Keccak256 lo = k_, hi = k_;
      const uint8_t plo = 10, phi = 11;
      lo.update(&plo, 1);
      hi.update(&phi, 1);
      lo.digest(d);
      hi.digest(d + 32);
    } else {
      h_.digest(d);
    }
    uint32_t w[16];
    std::memcpy(w, d, 64);
    return fr_from_u512(w);
  }

 private:
  template <class F>
  static void repr(const F& c, uint8_t out[32]) {
    std::memcpy(out, c.l, 32);  // canonical limbs, little-endian
  }
  void absorb(const uint8_t* b, size_t len) {
    if (kind_ == TRANSCRIPT_KECCAK256) k_.update(b, len);
    else h_.update(b, len);
  }
  Blake2b h_;
  Keccak256 k_;
  int kind_;
  std::vector<uint8_t>* proof_;
};

}  // namespace h2g
