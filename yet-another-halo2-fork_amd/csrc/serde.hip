// serde.hip -- SerdeFormat::Processed on the device (halo2_backend/src/helpers.rs:36-100):
// G1 points compressed with GroupEncoding::to_bytes / from_bytes (halo2curves 0.6 bn256,
// the encoding the transcript's write_point uses: x canonical LE, bit 7 of byte 31 = y
// odd, identity = 32 zero bytes) and field elements as PrimeField::to_repr / from_repr
// (canonical LE; from_repr refuses values >= r).  One element per thread; a whole ParamsKZG
// (2 x 2^k points) decompresses in one launch per array instead of a parallelize() over
// host cores (kzg/commitment.rs:194-232).
#include "prover_kernels.h"

namespace h2g {
namespace {
constexpr int ST = 256;

// (p + 1) / 4: p = 3 mod 4, so a square a has the root a^((p+1)/4)
constexpr uint32_t FQ_SQRT_EXP[8] = {0xb61f3f52u, 0x4f082305u, 0x5a1c72a3u, 0x65e05aa4u,
                                     0xa0605617u, 0x6e14116du, 0xb84c680au, 0x0c19139cu};

template <class P>
__device__ __forceinline__ bool below(const Fe<P>& a) {
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)__builtin_subc(a.l[i], P::M[i], br, &br);
  return br != 0;
}
__device__ __forceinline__ void count_bad_lane(bool bad, uint32_t* out) {
  const uint64_t m = __ballot(bad);
  if (m && __lane_id() == (uint32_t)__builtin_ctzll(m)) atomicAdd(out, (uint32_t)__popcll(m));
}

// G1Affine::to_bytes: the compressed point as 8 LE words (word 7 carries the sign bit)
__global__ void __launch_bounds__(ST) g1_compress_kernel(const G1Affine* __restrict__ p, size_t n,
                                                         uint32_t* __restrict__ out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1Affine q = p[i];
  Fq x = Fq::zero();
  if (!q.is_identity()) {
    x = to_canonical(q.x);
    x.l[7] |= (to_canonical(q.y).l[0] & 1u) << 31;
  }
  uint4* o = reinterpret_cast<uint4*>(out + 8 * i);
  o[0] = make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]);
  o[1] = make_uint4(x.l[4], x.l[5], x.l[6], x.l[7]);
}

// G1Affine::from_bytes: sign bit off, x must be canonical; x = 0 with the sign clear is the
// identity; otherwise y = sqrt(x^3 + 3) (None if x^3 + 3 is a non-residue), negated when its
// parity differs from the sign bit.  A point that fails is written as the identity and counted.
__global__ void __launch_bounds__(ST) g1_decompress_kernel(const uint32_t* __restrict__ in, size_t n,
                                                           G1Affine* __restrict__ out, uint32_t* bad) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  bool b = false;
  if (i < n) {
    const uint4* s = reinterpret_cast<const uint4*>(in + 8 * i);
    const uint4 a = s[0], c = s[1];
    Fq x;
    x.l[0] = a.x, x.l[1] = a.y, x.l[2] = a.z, x.l[3] = a.w;
    x.l[4] = c.x, x.l[5] = c.y, x.l[6] = c.z, x.l[7] = c.w & 0x7fffffffu;
    const uint32_t ysign = c.w >> 31;
    G1Affine r;
    r.x = Fq::zero();
    r.y = Fq::zero();
    if (!below(x)) {
      b = true;
    } else if (!(x.is_zero() && !ysign)) {
      const Fq xm = from_canonical(x);
      const Fq y2 = sqr(xm) * xm + from_u64<FqParams>(3);
      Fq y = pow_limbs(y2, FQ_SQRT_EXP);
      if (sqr(y) != y2) {
        b = true;
      } else {
        if ((to_canonical(y).l[0] & 1u) != ysign) y = neg(y);
        r.x = xm;
        r.y = y;
      }
    }
    out[i] = r;
  }
  count_bad_lane(b, bad);
}

__global__ void __launch_bounds__(ST) fr_to_repr_kernel(const Fr* __restrict__ a, size_t n, Fr* __restrict__ out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = to_canonical(a[i]);
}

// from_repr in place: canonical -> Montgomery; values >= r are counted (and left as read)
__global__ void __launch_bounds__(ST) fr_from_repr_kernel(Fr* __restrict__ a, size_t n, uint32_t* bad) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  bool b = false;
  if (i < n) {
    const Fr v = a[i];
    b = !below(v);
    if (!b) a[i] = from_canonical(v);
  }
  count_bad_lane(b, bad);
}

unsigned blocks(size_t n) { return (unsigned)((n + ST - 1) / ST); }
}  // namespace

hipError_t g1_compress(const G1Affine* p, size_t n, uint8_t* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(g1_compress_kernel, dim3(blocks(n)), dim3(ST), 0, st, p, n, reinterpret_cast<uint32_t*>(out));
  return hipGetLastError();
}
hipError_t g1_decompress(const uint8_t* in, size_t n, G1Affine* out, uint32_t* bad, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(g1_decompress_kernel, dim3(blocks(n)), dim3(ST), 0, st, reinterpret_cast<const uint32_t*>(in),
                     n, out, bad);
  return hipGetLastError();
}
hipError_t fr_to_repr(const Fr* a, size_t n, Fr* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fr_to_repr_kernel, dim3(blocks(n)), dim3(ST), 0, st, a, n, out);
  return hipGetLastError();
}
hipError_t fr_from_repr(Fr* a, size_t n, uint32_t* bad, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fr_from_repr_kernel, dim3(blocks(n)), dim3(ST), 0, st, a, n, bad);
  return hipGetLastError();
}

}  // namespace h2g
