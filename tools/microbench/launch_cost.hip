// launch_cost.hip -- host cost of hipLaunchKernel / small hipMemcpyAsync D2H on gfx950,
// without a profiler: is the keccak-style proof's host thread bound by its ~600 launches
// (a kernel trace with --hip-trace showed ~58 us per launch while large kernels ran)?
// Cases: the GPU idle; a long kernel running on another stream; the same with many
// streams created (streams beyond GPU_MAX_HW_QUEUES share hardware queues); launches on a
// stream that shares its hardware queue with the busy one.
// build: hipcc --offload-arch=gfx950 -O2 -o launch_cost launch_cost.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void tiny_kernel(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] += 1;
}

// every wave spins for `ticks` of the 100 MHz wall clock, then exits (bounded)
__global__ void spin_kernel(uint64_t ticks, int* sink) {
  const uint64_t t0 = wall_clock64();
  uint64_t x = 0;
  while (wall_clock64() - t0 < ticks) x++;
  if (x == 0xffffffffffffull) sink[0] = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// mean host microseconds per call of `launches` tiny launches (grid g) on stream s
static double time_launches(hipStream_t s, int launches, unsigned g, int* d) {
  const double t0 = now_us();
  for (int i = 0; i < launches; i++) hipLaunchKernelGGL(tiny_kernel, dim3(g), dim3(256), 0, s, d);
  return (now_us() - t0) / launches;
}
static double time_copies(hipStream_t s, int copies, void* h, const void* d) {
  const double t0 = now_us();
  for (int i = 0; i < copies; i++) (void)hipMemcpyAsync(h, d, 128, hipMemcpyDeviceToHost, s);
  return (now_us() - t0) / copies;
}

int main() {
  int* d = nullptr;
  void* h = nullptr;
  CK(hipMalloc(&d, 16 << 20));  // the 8-MB memsets below stay inside
  CK(hipMemset(d, 0, 16 << 20));
  CK(hipHostMalloc(&h, 4096, hipHostMallocDefault));
  std::vector<hipStream_t> st(10);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint64_t spin = 100ull * 20000;  // 20 ms per wave
  // warm up
  for (int i = 0; i < 100; i++) hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, st[0], d);
  CK(hipDeviceSynchronize());

  std::printf("idle GPU, 1 stream:            launch %.1f us (grid 1), %.1f us (grid 4096); D2H copy %.1f us\n",
              time_launches(st[0], 200, 1, d), time_launches(st[0], 200, 4096, d), time_copies(st[0], 200, h, d));
  CK(hipDeviceSynchronize());
  for (int busy : {1, 2, 3, 4, 5, 6, 7, 8, 9}) {
    // a long kernel filling the chip (many workgroups) on stream `busy`, launches on stream 0
    hipLaunchKernelGGL(spin_kernel, dim3(4096), dim3(256), 0, st[busy], spin, d);
    const double l1 = time_launches(st[0], 100, 1, d);
    const double l2 = time_launches(st[0], 100, 4096, d);
    const double c1 = time_copies(st[0], 50, h, d);
    std::printf("busy stream %d (long kernel):  launch %.1f us (grid 1), %.1f us (grid 4096); D2H copy %.1f us\n",
                busy, l1, l2, c1);
    CK(hipDeviceSynchronize());
  }
  // hipMemsetAsync's host cost: idle, behind a long kernel on the same stream, and beside one
  for (size_t bytes : {(size_t)4, (size_t)8196, (size_t)8 << 20}) {
    double t0 = now_us();
    for (int i = 0; i < 20; i++) CK(hipMemsetAsync(d, 0, bytes, st[0]));
    const double idle = (now_us() - t0) / 20;
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(spin_kernel, dim3(4096), dim3(256), 0, st[0], spin, d + (1 << 18) / 4);
    t0 = now_us();
    CK(hipMemsetAsync(d, 0, bytes, st[0]));
    const double same = now_us() - t0;
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(spin_kernel, dim3(4096), dim3(256), 0, st[1], spin, d + (1 << 18) / 4);
    t0 = now_us();
    CK(hipMemsetAsync(d, 0, bytes, st[0]));
    const double other = now_us() - t0;
    CK(hipDeviceSynchronize());
    std::printf("hipMemsetAsync %zu B: idle %.1f us, behind a 20-ms kernel on its stream %.1f us, beside one %.1f us\n",
                bytes, idle, same, other);
  }
  // the same with a long kernel of few waves (one per CU)
  hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(64), 0, st[1], spin, d);
  std::printf("busy stream 1 (256 waves):      launch %.1f us (grid 4096); D2H copy %.1f us\n",
              time_launches(st[0], 100, 4096, d), time_copies(st[0], 50, h, d));
  CK(hipDeviceSynchronize());
  CK(hipHostFree(h));
  CK(hipFree(d));
  return 0;
}
