// Microbenchmark: FIPS Montgomery multiply with G products per inline-asm block
// (non-volatile asm), G in {1, 2, 4}.  hipcc pads every asm-block boundary with an
// s_nop; bigger blocks pad less but schedule coarser.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "../../yet-another-halo2-fork_amd/csrc/bn254.h"
using namespace h2g;

#define MAC1S "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
__device__ __forceinline__ void m1(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
  asm(MAC1S : "+v"(lo), "+v"(hi) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ void m2(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(lo), "+v"(hi) : "v"(a), "v"(b), "v"(c), "v"(d) : "vcc");
}
__device__ __forceinline__ void m4(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                   uint32_t e, uint32_t f, uint32_t g, uint32_t h) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %6, %7, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(lo), "+v"(hi) : "v"(a), "v"(b), "v"(c), "v"(d), "v"(e), "v"(f), "v"(g), "v"(h) : "vcc");
}

// products of column k as (x, y) pairs, then grouped
template <int G>
__device__ __forceinline__ void column(uint64_t& lo, uint32_t& hi, const uint32_t* xs, const uint32_t* ys, int np) {
  int i = 0;
  if (G >= 4)
    for (; i + 4 <= np; i += 4) m4(lo, hi, xs[i], ys[i], xs[i + 1], ys[i + 1], xs[i + 2], ys[i + 2], xs[i + 3], ys[i + 3]);
  if (G >= 2)
    for (; i + 2 <= np; i += 2) m2(lo, hi, xs[i], ys[i], xs[i + 1], ys[i + 1]);
  for (; i < np; i++) m1(lo, hi, xs[i], ys[i]);
}

template <int G>
__device__ __forceinline__ Fq mulG(const Fq& A, const Fq& B) {
  const uint32_t* a = A.l;
  const uint32_t* b = B.l;
  uint32_t m[8];
  Fq r, d;
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t xs[16], ys[16];
    int np = 0;
#pragma unroll
    for (int i = 0; i < k; i++) {
      xs[np] = a[i]; ys[np++] = b[k - i];
      xs[np] = m[i]; ys[np++] = FqParams::M[k - i];
    }
    xs[np] = a[k]; ys[np++] = b[0];
    column<G>(lo, hi, xs, ys, np);
    m[k] = (uint32_t)lo * FqParams::INV;
    m1(lo, hi, m[k], FqParams::M[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
    uint32_t xs[16], ys[16];
    int np = 0;
#pragma unroll
    for (int i = k - 7; i < 8; i++) {
      xs[np] = a[i]; ys[np++] = b[k - i];
      xs[np] = m[i]; ys[np++] = FqParams::M[k - i];
    }
    column<G>(lo, hi, xs, ys, np);
    r.l[k - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r.l[7] = (uint32_t)lo;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    int64_t u = (int64_t)r.l[i] - FqParams::M[i] + br;
    d.l[i] = (uint32_t)u;
    br = u >> 32;
  }
  return br ? r : d;
}

template <int V>
__global__ void __launch_bounds__(256) bench(Fq* x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = x[i], b = x[i + 1], c = x[i + 2];
  for (int it = 0; it < iters; it++) {
    if (V == 0) { a = a * b; c = c * b; }
    if (V == 1) { a = mulG<1>(a, b); c = mulG<1>(c, b); }
    if (V == 2) { a = mulG<2>(a, b); c = mulG<2>(c, b); }
    if (V == 4) { a = mulG<4>(a, b); c = mulG<4>(c, b); }
  }
  x[i] = a + c;
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 1000;
  const size_t n = (size_t)blocks * threads + 2;
  Fq *d, *h = (Fq*)malloc(n * sizeof(Fq)), *h2 = (Fq*)malloc(n * sizeof(Fq));
  hipMalloc(&d, n * sizeof(Fq));
  for (size_t i = 0; i < n; i++)
    for (int j = 0; j < 8; j++) h[i].l[j] = (uint32_t)(i * 2654435761u + j * 40503u) & (j == 7 ? 0x0fffffffu : 0xffffffffu);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int vs[4] = {0, 1, 2, 4};
  for (int vi = 0; vi < 4; vi++) {
    const int v = vs[vi];
    hipMemcpy(d, h, n * sizeof(Fq), hipMemcpyHostToDevice);
    auto launch = [&](int it) {
      if (v == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(threads), 0, 0, d, it);
      if (v == 1) hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(threads), 0, 0, d, it);
      if (v == 2) hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(threads), 0, 0, d, it);
      if (v == 4) hipLaunchKernelGGL(bench<4>, dim3(blocks), dim3(threads), 0, 0, d, it);
    };
    launch(3);
    hipMemcpy(h2, d, n * sizeof(Fq), hipMemcpyDeviceToHost);
    static Fq ref[1];
    if (vi == 0) memcpy(ref, h2, sizeof(Fq));
    hipMemcpy(d, h, n * sizeof(Fq), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      launch(iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("group %d: %.1f Gmodmul/s  (check %08x)\n", v, 2.0 * blocks * threads * iters / ms / 1e6, h2[0].l[0]);
    }
  }
  return 0;
}
