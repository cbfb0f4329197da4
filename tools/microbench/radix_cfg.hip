// Microbenchmark: rocprim onesweep radix sort of the fixed-base MSM bucket keys
// (20-bit keys, M = 13 * 2^22 entries) under different configurations, and a
// keys-only sort of 64-bit (bucket << 32 | value) words.  Prints ms per sort.
#include <hip/hip_runtime.h>
#include <string.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
__global__ void gen_keys(uint32_t* k, uint32_t* v, size_t M, uint32_t mask) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < M) { k[i] = hsh((uint32_t)i) & mask; v[i] = (uint32_t)i; }
}
__global__ void gen64(uint64_t* k, size_t M, uint32_t mask) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < M) k[i] = ((uint64_t)(hsh((uint32_t)i) & mask) << 32) | (uint32_t)i;
}

template <class Cfg>
int run(const char* name, uint32_t* k0, uint32_t* k1, uint32_t* v0, uint32_t* v1, size_t M, int bits) {
  size_t tb = 0;
  CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k0, k1, v0, v1, M, 0, bits));
  void* tmp;
  CK(hipMalloc(&tmp, tb));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float tot = 0;
  for (int r = 0; r < 6; r++) {
    CK(hipEventRecord(a));
    CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, k0, k1, v0, v1, M, 0, bits));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; hipEventElapsedTime(&ms, a, b);
    if (r) tot += ms / 5;
  }
  printf("%-40s bits=%d M=%zu: %.3f ms\n", name, bits, M, tot);
  hipFree(tmp);
  return 0;
}

using namespace rocprim;
int main() {
  const size_t M = 13ull << 22;
  const int bits = 20;
  uint32_t *k0, *k1, *v0, *v1;
  CK(hipMalloc(&k0, M * 4)); CK(hipMalloc(&k1, M * 4)); CK(hipMalloc(&v0, M * 4)); CK(hipMalloc(&v1, M * 4));
  gen_keys<<<(unsigned)((M + 255) / 256), 256>>>(k0, v0, M, (1u << bits) - 1);
  run<default_config>("pairs default", k0, k1, v0, v1, M, bits);
  run<radix_sort_config<default_config, default_config, radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<256, 16>, 7>>>("pairs onesweep 256x16 r7", k0, k1, v0, v1, M, bits);
  run<radix_sort_config<default_config, default_config, radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<256, 16>, 8>>>("pairs onesweep 256x16 r8", k0, k1, v0, v1, M, bits);
  run<radix_sort_config<default_config, default_config, radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<256, 24>, 7>>>("pairs onesweep 256x24 r7", k0, k1, v0, v1, M, bits);
  uint64_t *a, *b;
  CK(hipMalloc(&a, M * 8)); CK(hipMalloc(&b, M * 8));
  gen64<<<(unsigned)((M + 255) / 256), 256>>>(a, M, (1u << bits) - 1);
  size_t tb = 0;
  CK(rocprim::radix_sort_keys(nullptr, tb, a, b, M, 32, 32 + bits));
  void* tmp; CK(hipMalloc(&tmp, tb));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float tot = 0;
  for (int r = 0; r < 6; r++) {
    CK(hipEventRecord(e0));
    CK(rocprim::radix_sort_keys(tmp, tb, a, b, M, 32, 32 + bits));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1); if (r) tot += ms / 5;
  }
  printf("%-40s bits=%d M=%zu: %.3f ms\n", "keys-only u64 default", bits, M, tot);
  return 0;
}
