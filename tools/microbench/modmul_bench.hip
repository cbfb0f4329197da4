// Microbenchmark: BN254 Fq Montgomery multiplication throughput on gfx950.
// Variants: (0) C CIOS from csrc/bn254.h, (1) inline-asm FIPS product scanning
// with v_mad_u64_u32 carry-out, (2) raw v_mad_u64_u32 issue rate.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <stdint.h>
#include "../../yet-another-halo2-fork_amd/csrc/bn254.h"
using namespace h2g;

__device__ __forceinline__ void mac(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
  asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
               : "+v"(lo), "+v"(hi) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ Fq fips_mul(const Fq& A, const Fq& B) {
  const uint32_t* a = A.l; const uint32_t* b = B.l;
  uint32_t m[8], r[8];
  uint64_t lo = 0; uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) { mac(lo, hi, a[i], b[k - i]); mac(lo, hi, m[i], FqParams::M[k - i]); }
    mac(lo, hi, a[k], b[0]);
    m[k] = (uint32_t)lo * FqParams::INV;
    mac(lo, hi, m[k], FqParams::M[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32); hi = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int i = k - 7; i < 8; i++) { mac(lo, hi, a[i], b[k - i]); mac(lo, hi, m[i], FqParams::M[k - i]); }
    r[k - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32); hi = 0;
  }
  r[7] = (uint32_t)lo;
  Fq R, D;
  for (int i = 0; i < 8; i++) R.l[i] = r[i];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) { int64_t u = (int64_t)R.l[i] - FqParams::M[i] + br; D.l[i] = (uint32_t)u; br = u >> 32; }
  return br ? R : D;
}

template <int V>
__global__ void __launch_bounds__(256) bench(Fq* x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = x[i], b = x[i + 1];
  if (V == 2) {
    uint64_t acc = a.l[0];
    uint32_t p = a.l[1], q = b.l[2];
    for (int it = 0; it < iters * 128; it++) {
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc) : "v"(p), "v"(q) : "s0", "s1");
    }
    a.l[0] = (uint32_t)acc;
  } else {
    for (int it = 0; it < iters; it++) a = (V == 0) ? a * b : fips_mul(a, b);
  }
  x[i] = a;
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 2000;
  const size_t n = (size_t)blocks * threads + 1;
  Fq* d; hipMalloc(&d, n * sizeof(Fq));
  Fq* h = (Fq*)malloc(n * sizeof(Fq));
  for (size_t i = 0; i < n; i++) for (int j = 0; j < 8; j++) h[i].l[j] = (uint32_t)(i * 2654435761u + j * 40503u) & (j == 7 ? 0x0fffffffu : 0xffffffffu);
  hipMemcpy(d, h, n * sizeof(Fq), hipMemcpyHostToDevice);
  // correctness: variant 0 vs 1 on a short run
  Fq* d2; hipMalloc(&d2, n * sizeof(Fq)); hipMemcpy(d2, h, n * sizeof(Fq), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(threads), 0, 0, d, 3);
  hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(threads), 0, 0, d2, 3);
  Fq* h2 = (Fq*)malloc(n * sizeof(Fq));
  hipMemcpy(h, d, n * sizeof(Fq), hipMemcpyDeviceToHost);
  hipMemcpy(h2, d2, n * sizeof(Fq), hipMemcpyDeviceToHost);
  size_t bad = 0; for (size_t i = 0; i + 1 < n; i++) bad += memcmp(&h[i], &h2[i], 32) != 0;
  printf("fips vs cios mismatches: %zu\n", bad);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int v = 0; v < 3; v++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(threads), 0, 0, d, iters);
      if (v == 1) hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(threads), 0, 0, d, iters);
      if (v == 2) hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(threads), 0, 0, d, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double ops = (double)blocks * threads * iters;
      if (v < 2) printf("variant %d: %.3f ms  %.1f Gmodmul/s\n", v, ms, ops / ms / 1e6);
      else printf("raw v_mad_u64_u32: %.1f Gop/s (x128 per iter)\n", ops * 128 / ms / 1e6);
    }
  }
  return 0;
}
