// Microbenchmark: grouping M = W * n (bucket, entry) pairs by bucket on gfx950.
// (a) global-atomic counting sort: histogram (no-return atomics) + scan + scatter
//     (returning atomics), with and without wave-level aggregation of equal keys;
// (b) hipcub radix sort of (key, value) pairs, as msm.hip uses today.
// Keys are uniform 19-bit or all-equal (skewed).  Prints ms per phase.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t key_of(uint32_t i, uint32_t mask, int skew) { return skew ? 7u : (hash32(i) & mask); }

__global__ void gen_keys(uint32_t* k, uint32_t* v, size_t M, uint32_t mask, int skew) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < M) { k[i] = key_of((uint32_t)i, mask, skew); v[i] = (uint32_t)i; }
}

template <int AGG>
__global__ void hist(size_t M, uint32_t mask, int skew, uint32_t* cnt) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t k = key_of((uint32_t)i, mask, skew);
  if (AGG) {
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(k);
    const uint64_t same = __ballot(k == k0);
    if (k == k0) {
      if (__lane_id() == (uint32_t)__builtin_ctzll(same)) atomicAdd(&cnt[k0], (uint32_t)__popcll(same));
      return;
    }
  }
  atomicAdd(&cnt[k], 1u);
}

template <int AGG>
__global__ void scatter(size_t M, uint32_t mask, int skew, uint32_t* cur, uint32_t* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t k = key_of((uint32_t)i, mask, skew);
  if (AGG) {
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(k);
    const uint64_t same = __ballot(k == k0);
    if (k == k0) {
      const uint32_t leader = __builtin_ctzll(same);
      uint32_t base = 0;
      if (__lane_id() == leader) base = atomicAdd(&cur[k0], (uint32_t)__popcll(same));
      base = __shfl(base, leader);
      const uint32_t rank = __popcll(same & ((1ull << __lane_id()) - 1));
      out[base + rank] = (uint32_t)i;
      return;
    }
  }
  out[atomicAdd(&cur[k], 1u)] = (uint32_t)i;
}

int main(int argc, char** argv) {
  const int bits = argc > 1 ? atoi(argv[1]) : 19;
  const size_t M = argc > 2 ? strtoull(argv[2], 0, 0) : 13ull << 22;
  const uint32_t NB = 1u << bits, mask = NB - 1;
  uint32_t *k0, *k1, *v0, *v1, *cnt, *cur, *out;
  CK(hipMalloc(&k0, M * 4)); CK(hipMalloc(&k1, M * 4)); CK(hipMalloc(&v0, M * 4)); CK(hipMalloc(&v1, M * 4));
  CK(hipMalloc(&cnt, NB * 4)); CK(hipMalloc(&cur, NB * 4)); CK(hipMalloc(&out, M * 4));
  size_t tmpb = 0, scanb = 0;
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmpb, k0, k1, v0, v1, (int)M, 0, bits + 1));
  CK(hipcub::DeviceScan::ExclusiveSum(nullptr, scanb, cnt, cur, (int)NB));
  void *tmp, *stmp;
  CK(hipMalloc(&tmp, tmpb)); CK(hipMalloc(&stmp, scanb));
  hipEvent_t e[8];
  for (auto& x : e) CK(hipEventCreate(&x));
  const unsigned G = (unsigned)((M + 255) / 256);
  for (int skew = 0; skew < 2; skew++) {
    for (int agg = 0; agg < 2; agg++) {
      float th = 0, ts = 0, tc = 0;
      for (int rep = 0; rep < 4; rep++) {
        CK(hipMemset(cnt, 0, NB * 4));
        CK(hipEventRecord(e[0]));
        if (agg) hist<1><<<G, 256>>>(M, mask, skew, cnt); else hist<0><<<G, 256>>>(M, mask, skew, cnt);
        CK(hipEventRecord(e[1]));
        CK(hipcub::DeviceScan::ExclusiveSum(stmp, scanb, cnt, cur, (int)NB));
        CK(hipEventRecord(e[2]));
        if (agg) scatter<1><<<G, 256>>>(M, mask, skew, cur, out); else scatter<0><<<G, 256>>>(M, mask, skew, cur, out);
        CK(hipEventRecord(e[3]));
        CK(hipEventSynchronize(e[3]));
        float a, b, c;
        hipEventElapsedTime(&a, e[0], e[1]); hipEventElapsedTime(&b, e[1], e[2]); hipEventElapsedTime(&c, e[2], e[3]);
        if (rep) { th += a / 3; tc += b / 3; ts += c / 3; }
      }
      printf("counting sort bits=%d M=%zu skew=%d agg=%d: hist %.3f ms scan %.3f ms scatter %.3f ms total %.3f\n",
             bits, M, skew, agg, th, tc, ts, th + tc + ts);
    }
    gen_keys<<<G, 256>>>(k0, v0, M, mask, skew);
    float t = 0;
    for (int rep = 0; rep < 4; rep++) {
      CK(hipEventRecord(e[0]));
      CK(hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, k0, k1, v0, v1, (int)M, 0, bits + 1));
      CK(hipEventRecord(e[1]));
      CK(hipEventSynchronize(e[1]));
      float a;
      hipEventElapsedTime(&a, e[0], e[1]);
      if (rep) t += a / 3;
    }
    printf("radix sort pairs bits=%d M=%zu skew=%d: %.3f ms\n", bits + 1, M, skew, t);
  }
  return 0;
}
