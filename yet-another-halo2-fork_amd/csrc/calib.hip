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

// the round-4 reference measurement (tools/microbench/modmul_bench.hip, variant 1): the FIPS
// product with one volatile inline-asm block per mac, one dependent chain per thread --
// 125 G/s on the round-4 boxes, the reference of the bench line's value_normalised
__device__ __forceinline__ void ref_mac(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
  asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
               : "+v"(lo), "+v"(hi)
               : "v"(a), "v"(b)
               : "vcc");
}
__device__ __forceinline__ Fq ref_fips_mul(const Fq& A, const Fq& B) {
  const uint32_t* a = A.l;
  const uint32_t* b = B.l;
  uint32_t m[8], r[8];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      ref_mac(lo, hi, a[i], b[k - i]);
      ref_mac(lo, hi, m[i], FqParams::M[k - i]);
    }
    ref_mac(lo, hi, a[k], b[0]);
    m[k] = (uint32_t)lo * FqParams::INV;
    ref_mac(lo, hi, m[k], FqParams::M[0]);
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int i = k - 7; i < 8; i++) {
      ref_mac(lo, hi, a[i], b[k - i]);
      ref_mac(lo, hi, m[i], FqParams::M[k - i]);
    }
    r[k - 8] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r[7] = (uint32_t)lo;
  Fq R, D;  // the reference's final subtraction (64-bit signed borrow), kept as it was measured
#pragma unroll
  for (int i = 0; i < 8; i++) R.l[i] = r[i];
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t u = (int64_t)R.l[i] - FqParams::M[i] + br;
    D.l[i] = (uint32_t)u;
    br = u >> 32;
  }
  return br ? R : D;
}
__global__ void __launch_bounds__(CAL_THREADS) calib_ref_kernel(Fq* x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = x[i], b = x[i + 1];
  for (int it = 0; it < iters; it++) a = ref_fips_mul(a, b);
  x[i] = a;
}

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

// the one-GPU SPMD emulation's stand-in for a transfer (h2g_debug_link_delay): one thread
// waits `ticks` of the 100 MHz real-time counter, napping between reads; the count is
// capped by the host, so every launch ends
__global__ void link_delay_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

// `done` recorded `us` microseconds of device time after the work queued on `after` so far:
// the wait kernel runs on a side stream of its own (the modelled transfer overlaps the
// prover's stream as an RCCL exchange on its communicator's stream would)
hipError_t link_delay(hipStream_t after, hipEvent_t done, double us) {
  static hipStream_t side = nullptr;
  static hipEvent_t ready = nullptr;
  hipError_t e = hipSuccess;
  if (!side) e = hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
  if (e == hipSuccess && !ready) e = hipEventCreateWithFlags(&ready, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(ready, after);
  if (e == hipSuccess) e = hipStreamWaitEvent(side, ready, 0);
  if (e != hipSuccess) return e;
  const double capped = us < 0 ? 0 : (us > 10e6 ? 10e6 : us);  // at most 10 s
  hipLaunchKernelGGL(link_delay_kernel, dim3(1), dim3(1), 0, side, (unsigned long long)(capped * 100.0));
  e = hipGetLastError();
  if (e == hipSuccess) e = hipEventRecord(done, side);
  return e;
}

}  // namespace h2g

using namespace h2g;

// out[0] G modmul/s of the round-4 reference kernel (FIPS, one chain per thread, 2048 x
// 256 threads x 2000 products as tools/microbench/modmul_bench.hip), out[1] F29 G modmul/s
// (two chains per thread), out[2] shader GHz during the F29 run, out[3] wall ms of the
// whole calibration, out[4] (max >= 5) the FIPS product with two chains per thread;
// returns 0 or a HIP error code
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
  double rate[2] = {0, 0}, ghz = 0, ref = 0;
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
    {  // the reference kernel: 2048 blocks of 256 threads, 2000 products each
      const int rb = 256 * 8, riters = 2000;
      float best = 1e30f;
      for (int rep = 0; rep < 2 && e == hipSuccess && (size_t)rb * CAL_THREADS + 1 <= n; rep++) {
        (void)hipEventRecord(e0, nullptr);
        hipLaunchKernelGGL(calib_ref_kernel, dim3(rb), dim3(CAL_THREADS), 0, nullptr, x, riters);
        (void)hipEventRecord(e1, nullptr);
        e = hipEventSynchronize(e1);
        float ms = 0;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        if (e == hipSuccess && ms < best) best = ms;
      }
      ref = (double)rb * CAL_THREADS * riters / (best * 1e-3) / 1e9;
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
  out[0] = ref;
  out[1] = rate[1];
  out[2] = ghz;
  out[3] = wall;
  if (max >= 5) out[4] = rate[0];
  return 0;
}
