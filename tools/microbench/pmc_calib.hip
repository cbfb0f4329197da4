// PMC calibration: what FETCH_SIZE / WRITE_SIZE (rocprofv3 --pmc, KiB) report on gfx950
// for access patterns of known byte counts, so that the bench line's roofline.traffic
// for msm_acc_kernel can be corrected per pattern instead of with one blanket factor.
//   calib_stream_read   : 16 B per lane, coalesced, over STREAM_BYTES (the guide's case)
//   calib_gather64      : one 64-B affine point per lane (4 x 16-B loads, ld_aff in
//                         msm.hip) at pseudo-random indices into a TABLE_POINTS table --
//                         msm_acc_kernel's base gathers
//   calib_entries_read  : 8 B per lane, coalesced (msm_acc_kernel's sorted entries)
//   calib_stream_write  : 16 B per lane, coalesced
// Each kernel runs once per process; the host prints the algorithmic bytes of each.
// Build: hipcc -O3 --offload-arch=gfx950 -o pmc_calib pmc_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib ; rocprofv3 --pmc WRITE_SIZE -- ./pmc_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                               \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                              \
    }                                                                        \
  } while (0)

static constexpr size_t STREAM_BYTES = 1ull << 30;   // 1 GiB
static constexpr size_t TABLE_POINTS = 1ull << 25;   // 2 GiB of 64-B points
static constexpr size_t GATHERS = 1ull << 25;        // 2 GiB gathered
static constexpr size_t ENTRIES = 1ull << 27;        // 1 GiB of 8-B entries

__global__ void __launch_bounds__(256) calib_stream_read(const uint4* __restrict__ a, size_t n, uint4* __restrict__ out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = acc;  // keeps the loads live
}

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return (uint32_t)x;
}

__global__ void __launch_bounds__(256) calib_gather64(const uint4* __restrict__ table, size_t npts, size_t ng,
                                                     uint4* __restrict__ out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < ng; i += (size_t)gridDim.x * blockDim.x) {
    const size_t p = mix(i) & (npts - 1);
    const uint4* q = table + 4 * p;
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    acc.x ^= a.x ^ b.y ^ c.z ^ d.w; acc.y ^= a.y ^ b.z; acc.z ^= c.x ^ d.y; acc.w ^= a.w ^ b.x ^ c.y ^ d.z;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = acc;
}

__global__ void __launch_bounds__(256) calib_entries_read(const uint64_t* __restrict__ a, size_t n,
                                                         uint64_t* __restrict__ out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i];
  if (acc == 0x9e3779b97f4a7c15ULL) out[0] = acc;
}

__global__ void __launch_bounds__(256) calib_stream_write(uint4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 32), 7u, 9u);
}

__global__ void fill_kernel(uint4* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i * 2654435761u, (uint32_t)i, 3u, 5u);
}

int main() {
  uint4 *buf, *out;
  const size_t table_bytes = TABLE_POINTS * 64;
  const size_t bytes = table_bytes > STREAM_BYTES ? table_bytes : STREAM_BYTES;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc(&out, 64));
  const unsigned grid = 256 * 8;  // 8 blocks per CU, grid-stride loops
  hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, 0, buf, bytes / 16);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float ms;
  // algorithmic bytes, one line per kernel (rocprofv3 reports per launch)
  CHK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(calib_stream_read, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, STREAM_BYTES / 16, out);
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  CHK(hipEventElapsedTime(&ms, e0, e1));
  printf("calib_stream_read  read_bytes %zu  write_bytes 0  ms %.3f  GB/s %.0f\n", STREAM_BYTES, ms,
         STREAM_BYTES / (ms * 1e6));
  CHK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(calib_gather64, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, TABLE_POINTS, GATHERS, out);
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  CHK(hipEventElapsedTime(&ms, e0, e1));
  printf("calib_gather64     read_bytes %zu  write_bytes 0  ms %.3f  GB/s %.0f  (table %zu B)\n", GATHERS * 64, ms,
         GATHERS * 64 / (ms * 1e6), table_bytes);
  CHK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(calib_entries_read, dim3(grid), dim3(256), 0, 0, (const uint64_t*)buf, ENTRIES, (uint64_t*)out);
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  CHK(hipEventElapsedTime(&ms, e0, e1));
  printf("calib_entries_read read_bytes %zu  write_bytes 0  ms %.3f  GB/s %.0f\n", ENTRIES * 8, ms,
         ENTRIES * 8 / (ms * 1e6));
  CHK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(calib_stream_write, dim3(grid), dim3(256), 0, 0, buf, STREAM_BYTES / 16);
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  CHK(hipEventElapsedTime(&ms, e0, e1));
  printf("calib_stream_write read_bytes 0  write_bytes %zu  ms %.3f  GB/s %.0f\n", STREAM_BYTES, ms,
         STREAM_BYTES / (ms * 1e6));
  CHK(hipFree(buf));
  CHK(hipFree(out));
  return 0;
}
