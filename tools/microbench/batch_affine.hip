// Microbenchmark: bucket-accumulation add cost on gfx950, XYZZ mixed add (the MSM's
// accumulate kernel, 8M + 2S) vs batched affine addition (Montgomery's trick: 3M per add
// for the shared inversion + lambda, lambda^2, y3 = 6M, plus one inversion per K adds).
// Streams its operands from HBM the way a level of a pairwise bucket tree would.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 batch_affine.hip -o batch_affine
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../yet-another-halo2-fork_amd/csrc/bn254.h"
using namespace h2g;

template <int K>
__global__ void __launch_bounds__(256) madd_stream(const G1Affine* __restrict__ pts, Fq* __restrict__ out,
                                                    size_t NT) {
  const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  G1xyzz acc = G1xyzz::identity();
  for (int k = 0; k < K; k++) acc = xyzz_madd_lazy(acc, pts[k * NT + g]);
  out[g] = acc.X;
}

template <int K>
__global__ void __launch_bounds__(256) affine_pairs(const G1Affine* __restrict__ A, const G1Affine* __restrict__ B,
                                                     Fq* __restrict__ pref, G1Affine* __restrict__ out,
                                                     size_t NT) {
  const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  Fq acc = Fq::one();
  for (int k = 0; k < K; k++) {
    const size_t i = k * NT + g;
    pref[i] = acc;
    acc = mont_mul_lazy(acc, sub2(B[i].x, A[i].x));
  }
  Fq iv = inv(reduce_once(acc));
  for (int k = K - 1; k >= 0; k--) {
    const size_t i = k * NT + g;
    const G1Affine a = A[i], b = B[i];
    const Fq d = sub2(b.x, a.x);
    const Fq id = mont_mul_lazy(iv, pref[i]);
    iv = mont_mul_lazy(iv, d);
    const Fq lam = mont_mul_lazy(sub2(b.y, a.y), id);
    G1Affine r;
    r.x = sub2(sub2(mont_mul_lazy(lam, lam), a.x), b.x);
    r.y = sub2(mont_mul_lazy(lam, sub2(a.x, r.x)), a.y);
    out[i] = r;
  }
}

__global__ void __launch_bounds__(256) inv_only(Fq* __restrict__ x, int reps) {
  const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  Fq a = x[g];
  for (int r = 0; r < reps; r++) a = inv(a) + Fq::one();
  x[g] = a;
}

__global__ void __launch_bounds__(256) fermat_only(Fq* __restrict__ x, int reps) {
  const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  Fq a = x[g];
  for (int r = 0; r < reps; r++) a = inv_fermat(a) + Fq::one();
  x[g] = a;
}

// random-looking points: x, y < M (not on the curve; the formulas do not care)
__global__ void fill(G1Affine* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t s = (uint32_t)i * 2654435761u ^ seed;
    G1Affine q;
    for (int j = 0; j < 8; j++) {
      s = s * 1664525u + 1013904223u;
      q.x.l[j] = j == 7 ? (s & 0x0fffffffu) : s;
      s = s * 1664525u + 1013904223u;
      q.y.l[j] = j == 7 ? (s & 0x0fffffffu) : s;
    }
    p[i] = q;
  }
}

template <class F>
static float timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

template <int K>
static void run_k(size_t NT, G1Affine* A, G1Affine* B, Fq* pref, G1Affine* out, Fq* o2) {
  const unsigned blocks = (unsigned)(NT / 256);
  const double adds = (double)K * NT;
  const float m1 = timeit([&] { hipLaunchKernelGGL(madd_stream<K>, dim3(blocks), dim3(256), 0, 0, A, o2, NT); });
  const float m2 =
      timeit([&] { hipLaunchKernelGGL(affine_pairs<K>, dim3(blocks), dim3(256), 0, 0, A, B, pref, out, NT); });
  printf("NT %7zu K %4d  xyzz madd %7.2f G add/s (%.3f ms)   batch affine %7.2f G add/s (%.3f ms)  ratio %.2f\n",
         NT, K, adds / m1 / 1e6, m1, adds / m2 / 1e6, m2, m1 / m2);
}

int main() {
  const size_t NTMAX = 1u << 19, KMAX = 128;
  const size_t n = NTMAX * KMAX;
  G1Affine *A, *B, *out;
  Fq *pref, *o2;
  if (hipMalloc(&A, n * sizeof(G1Affine)) || hipMalloc(&B, n * sizeof(G1Affine)) ||
      hipMalloc(&out, n * sizeof(G1Affine)) || hipMalloc(&pref, n * sizeof(Fq)) ||
      hipMalloc(&o2, NTMAX * sizeof(Fq))) {
    printf("alloc failed\n");
    return 1;
  }
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, n, 1u);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, B, n, 2u);
  hipDeviceSynchronize();
  for (size_t NT : {(size_t)1 << 17, (size_t)1 << 18, (size_t)1 << 19}) {
    run_k<16>(NT, A, B, pref, out, o2);
    run_k<32>(NT, A, B, pref, out, o2);
    run_k<64>(NT, A, B, pref, out, o2);
    run_k<128>(NT, A, B, pref, out, o2);
  }
  for (size_t NT : {(size_t)1 << 16, (size_t)1 << 18}) {
    const int reps = 8;
    const float mi = timeit([&] { hipLaunchKernelGGL(inv_only, dim3(NT / 256), dim3(256), 0, 0, (Fq*)A, reps); });
    const float mf =
        timeit([&] { hipLaunchKernelGGL(fermat_only, dim3(NT / 256), dim3(256), 0, 0, (Fq*)B, reps); });
    printf("NT %7zu  binary-gcd inv %.3f G inv/s   fermat inv %.3f G inv/s\n", NT, NT * reps / mi / 1e6,
           NT * reps / mf / 1e6);
  }
  printf("status %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
