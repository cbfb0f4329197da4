// calib.hip -- box calibration for the bench line (h2g_profile_box_calibrate).
//
// GPUs of one model differ in sustained clock (power and thermal state), and the prover
// is bound by 256-bit modular products on the VALU, so a proof time from one box cannot be
// compared with another's without the product rate that box delivered.  This measures,
// right before a timed region: the Montgomery product throughput in both limb forms the
// prover uses (bn254.h's 8 x 32-bit FIPS product, f29.h's 9 x 29-bit product), two
// independent chains per thread on every SIMD, and the shader clock the kernel ran at
// (s_memtime against the 100 MHz s_memrealtime, median over workgroups).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "f29.h"

namespace h2g {

static constexpr int CAL_THREADS = 256;

template <int V>
__global__ void __launch_bounds__(CAL_THREADS) calib_kernel(Fq* x, int iters, unsigned long long* clk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
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
    const F29 A = to29(a), B = to29(b);
    F29 c = A, d = B;
    for (int it = 0; it < iters; it++) {
      c = mul29<FqParams>(c, B);
      d = mul29<FqParams>(d, A);
    }
    x[2 * i] = from29<FqParams>(c);
    x[2 * i + 1] = from29<FqParams>(d);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

__global__ void calib_fill(Fq* x, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fq v;
#pragma unroll
  for (int j = 0; j < 8; j++) v.l[j] = (uint32_t)(i * 2654435761u + j * 40503u + 17u) & (j == 7 ? 0x0fffffffu : ~0u);
  x[i] = v;
}

}  // namespace h2g

using namespace h2g;

// out[0] FIPS G modmul/s, out[1] F29 G modmul/s, out[2] shader GHz during the F29 run,
// out[3] wall ms of the whole calibration; returns 0 or a HIP error code
extern "C" int h2g_profile_box_calibrate(double* out, int max) {
  if (!out || max < 4) return 1;
  int dev = 0;
  hipDeviceProp_t pr;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&pr, dev) != hipSuccess) return 2;
  const int blocks = pr.multiProcessorCount * 8;  // 8 waves per CU
  const int iters = 1000;
  const size_t n = (size_t)blocks * CAL_THREADS * 2;
  Fq* x = nullptr;
  unsigned long long* clk = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr, w0 = nullptr;
  hipError_t e = hipMalloc(&x, n * sizeof(Fq));
  if (e == hipSuccess) e = hipMalloc(&clk, (size_t)blocks * 2 * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) e = hipEventCreate(&w0);
  double rate[2] = {0, 0}, ghz = 0;
  if (e == hipSuccess) {
    (void)hipEventRecord(w0, nullptr);
    hipLaunchKernelGGL(calib_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, x, n);
    for (int v = 0; v < 2 && e == hipSuccess; v++) {
      float best = 1e30f;
      for (int rep = 0; rep < 3 && e == hipSuccess; rep++) {  // the first run warms the clock up
        (void)hipEventRecord(e0, nullptr);
        if (v == 0) hipLaunchKernelGGL(calib_kernel<0>, dim3(blocks), dim3(CAL_THREADS), 0, nullptr, x, iters, clk);
        else hipLaunchKernelGGL(calib_kernel<1>, dim3(blocks), dim3(CAL_THREADS), 0, nullptr, x, iters, clk);
        (void)hipEventRecord(e1, nullptr);
        e = hipEventSynchronize(e1);
        float ms = 0;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        if (e == hipSuccess && ms < best) best = ms;
      }
      rate[v] = (double)blocks * CAL_THREADS * iters * 2 / (best * 1e-3) / 1e9;
    }
    if (e == hipSuccess) {
      std::vector<unsigned long long> h((size_t)blocks * 2);
      e = hipMemcpy(h.data(), clk, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      std::vector<double> g;
      for (int b = 0; b < blocks; b++)
        if (h[2 * b + 1] > 0) g.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);  // cycles / (10 ns)
      if (!g.empty()) {
        std::nth_element(g.begin(), g.begin() + g.size() / 2, g.end());
        ghz = g[g.size() / 2];
      }
    }
  }
  float wall = 0;
  if (e == hipSuccess) (void)hipEventElapsedTime(&wall, w0, e1);
  if (x) (void)hipFree(x);
  if (clk) (void)hipFree(clk);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (w0) (void)hipEventDestroy(w0);
  if (e != hipSuccess) return (int)e;
  out[0] = rate[0];
  out[1] = rate[1];
  out[2] = ghz;
  out[3] = wall;
  return 0;
}
