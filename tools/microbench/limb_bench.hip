// Microbenchmark: gfx950 issue cost of the integer instructions a 256-bit Montgomery product
// is built from, and the product itself in two limb layouts:
//   fips : bn254.h mont_mul_lazy -- 8 x 32-bit limbs, 128 v_mad_u64_u32 + 128 v_addc_co_u32
//   u29  : f29.h mul29           -- 9 x 29-bit limbs, 162 v_mad_u64_u32, no carry ops
// Raw rates: 8 independent instances per loop iteration (no dependences between them), one
// wave per SIMD and four waves per SIMD.  The shader clock comes from s_memtime against
// s_memrealtime (100 MHz) inside the kernel, so cycles per wave-instruction are clock-free.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I yet-another-halo2-fork_amd/csrc \
//         tools/microbench/limb_bench.hip -o tools/microbench/limb_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "f29.h"
using namespace h2g;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__device__ unsigned long long g_t0[1 << 16], g_t1[1 << 16], g_r0[1 << 16], g_r1[1 << 16];

template <int V>
__global__ void __launch_bounds__(256) raw(uint32_t* out, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a0 = tid, a1 = tid + 1, a2 = tid + 2, a3 = tid + 3, a4 = tid + 4, a5 = tid + 5, a6 = tid + 6, a7 = tid + 7;
  uint32_t x = tid * 7 + 1, y = tid * 13 + 5;
  double f0 = tid, f1 = tid + 1, f2 = tid + 2, f3 = tid + 3, f4 = tid + 4, f5 = tid + 5, f6 = tid + 6, f7 = tid + 7;
  const double fx = 1.0000001, fy = 0.5;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
    if (V == 0) {  // v_mad_u64_u32 (carry-out to an SGPR pair, unused)
#define M(i) asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %2, %0" : "+v"(a##i) : "v"(x), "v"(y) : "s20", "s21");
      REP8(M)
#undef M
    } else if (V == 1) {  // v_add_u32
#define M(i) asm volatile("v_add_u32 %0, %1, %0" : "+v"(*(uint32_t*)&a##i) : "v"(x));
      REP8(M)
#undef M
    } else if (V == 2) {  // v_addc_co_u32 (the FIPS carry catch), independent SGPR carries
#define M(i) asm volatile("v_addc_co_u32 %0, s[22:23], %1, %0, s[22:23]" : "+v"(*(uint32_t*)&a##i) : "v"(x) : "s22", "s23");
      REP8(M)
#undef M
    } else if (V == 3) {  // v_lshrrev_b64
#define M(i) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(a##i));
      REP8(M)
#undef M
    } else if (V == 4) {  // v_mul_lo_u32
#define M(i) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(*(uint32_t*)&a##i) : "v"(y));
      REP8(M)
#undef M
    } else if (V == 5) {  // v_fma_f64
#define M(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(f##i) : "v"(fx), "v"(fy));
      REP8(M)
#undef M
    } else if (V == 6) {  // v_lshl_add_u64
#define M(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a##i) : "v"(a0));
      REP8(M)
#undef M
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x < (1 << 16)) {
    g_t0[blockIdx.x] = t0; g_t1[blockIdx.x] = t1; g_r0[blockIdx.x] = r0; g_r1[blockIdx.x] = r1;
  }
  out[tid] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) ^ (uint32_t)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
}

// product throughput: two independent chains per thread
template <int V>
__global__ void __launch_bounds__(256) prod(Fq* x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = x[2 * i], b = x[2 * i + 1];
  if (V == 0) {
    Fq c = a, d = b;
    for (int it = 0; it < iters; it++) {
      c = mont_mul_lazy(c, b);
      d = mont_mul_lazy(d, a);
    }
    x[2 * i] = reduce_once(c);
    x[2 * i + 1] = reduce_once(d);
  } else {
    F29 A = to29(a), B = to29(b), c = A, d = B;
    for (int it = 0; it < iters; it++) {
      c = mul29<FqParams>(c, B);
      d = mul29<FqParams>(d, A);
    }
    x[2 * i] = from29<FqParams>(c);
    x[2 * i + 1] = from29<FqParams>(d);
  }
}

static double clock_ghz(int blocks) {
  static unsigned long long t0[1 << 16], t1[1 << 16], r0[1 << 16], r1[1 << 16];
  int nb = blocks < (1 << 16) ? blocks : (1 << 16);
  hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_t0), nb * 8);
  hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_t1), nb * 8);
  hipMemcpyFromSymbol(r0, HIP_SYMBOL(g_r0), nb * 8);
  hipMemcpyFromSymbol(r1, HIP_SYMBOL(g_r1), nb * 8);
  double s = 0;
  int c = 0;
  for (int i = 0; i < nb; i++)
    if (r1[i] > r0[i]) { s += (double)(t1[i] - t0[i]) / (double)(r1[i] - r0[i]) * 0.1; c++; }
  return c ? s / c : 0;
}

int main(int argc, char** argv) {
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, 0);
  const int cus = pr.multiProcessorCount, simds = cus * 4;
  printf("device %s, %d CUs\n", pr.gcnArchName, cus);
  uint32_t* out;
  hipMalloc(&out, (size_t)cus * 16 * 256 * 4);
  const char* names[] = {"v_mad_u64_u32", "v_add_u32", "v_addc_co_u32", "v_lshrrev_b64", "v_mul_lo_u32", "v_fma_f64",
                         "v_lshl_add_u64"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wps = 1; wps <= 4; wps *= 4) {  // waves per SIMD
    const int blocks = cus * wps, iters = 20000;
    for (int v = 0; v < 7; v++) {
      float best = 1e30f;
      double ghz = 0;
      for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        switch (v) {
          case 0: hipLaunchKernelGGL(raw<0>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
          case 1: hipLaunchKernelGGL(raw<1>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
          case 2: hipLaunchKernelGGL(raw<2>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
          case 3: hipLaunchKernelGGL(raw<3>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
          case 4: hipLaunchKernelGGL(raw<4>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
          case 5: hipLaunchKernelGGL(raw<5>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
          case 6: hipLaunchKernelGGL(raw<6>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) { best = ms; ghz = clock_ghz(blocks); }
      }
      // wave-instructions issued per SIMD, cycles per wave-instruction at the measured clock
      const double per_simd = (double)blocks * 4 / simds * iters * 8;
      const double cyc = best * 1e-3 * ghz * 1e9 / per_simd;
      printf("%-16s waves/SIMD %d: %8.3f ms  clock %.3f GHz  %.2f cycles per wave64 instruction\n", names[v], wps,
             best, ghz, cyc);
    }
  }
  // products
  const int blocks = cus * 8, threads = 256, iters = 2000;
  const size_t n = (size_t)blocks * threads * 2;
  Fq* h = (Fq*)malloc(n * sizeof(Fq));
  for (size_t i = 0; i < n; i++)
    for (int j = 0; j < 8; j++)
      h[i].l[j] = (uint32_t)(i * 2654435761u + j * 40503u + 17) & (j == 7 ? 0x0fffffffu : 0xffffffffu);
  Fq *d0, *d1;
  hipMalloc(&d0, n * sizeof(Fq));
  hipMalloc(&d1, n * sizeof(Fq));
  hipMemcpy(d0, h, n * sizeof(Fq), hipMemcpyHostToDevice);
  hipMemcpy(d1, h, n * sizeof(Fq), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(prod<0>, dim3(blocks), dim3(threads), 0, 0, d0, 7);
  hipLaunchKernelGGL(prod<1>, dim3(blocks), dim3(threads), 0, 0, d1, 7);
  Fq *h0 = (Fq*)malloc(n * sizeof(Fq)), *h1 = (Fq*)malloc(n * sizeof(Fq));
  hipMemcpy(h0, d0, n * sizeof(Fq), hipMemcpyDeviceToHost);
  hipMemcpy(h1, d1, n * sizeof(Fq), hipMemcpyDeviceToHost);
  size_t bad = 0;
  for (size_t i = 0; i < n; i++) bad += memcmp(&h0[i], &h1[i], 32) != 0;
  printf("u29 vs fips mismatches after 7 chained products: %zu of %zu\n", bad, n);
  for (int v = 0; v < 2; v++) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(prod<0>, dim3(blocks), dim3(threads), 0, 0, d0, iters);
      else hipLaunchKernelGGL(prod<1>, dim3(blocks), dim3(threads), 0, 0, d1, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double ops = (double)blocks * threads * iters * 2;
    printf("%s product: %.3f ms  %.1f G modmul/s\n", v == 0 ? "fips" : "u29 ", best, ops / best / 1e6);
  }
  return 0;
}
