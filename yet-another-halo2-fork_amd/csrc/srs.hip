// srs.hip -- KZG SRS powers on device: g_i = [s^i] G  (ParamsKZG::setup,
// halo2_backend/src/poly/kzg/commitment.rs:64-90).  Setup-time only.
#include "srs.h"

namespace h2g {

__global__ void __launch_bounds__(256) srs_kernel(Fr s, size_t n, G1Affine* __restrict__ out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr e = to_canonical(pow_u64(s, (uint64_t)i));
  G1Affine g;
  g.x = Fq::one();             // generator (1, 2)
  g.y = from_u64<FqParams>(2);
  const G1xyzz p = xyzz_mul_canonical(G1xyzz::from_affine(g), e.l);
  out[i] = xyzz_to_affine_by(p);
}

hipError_t srs_setup(const Fr& s, size_t n, G1Affine* d_out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(srs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s, n, d_out);
  return hipGetLastError();
}

}  // namespace h2g
