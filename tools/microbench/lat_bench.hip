// Microbenchmark: dependent-chain latency of one wave on gfx950 (no other waves).
// V=0: Fq product (mont_mul_lazy + reduce, the throughput form), V=1: mul_lat (16 column
// accumulators), V=2: XYZZ addition (lane form), V=3: XYZZ doubling.  Prints ns per
// operation and the shader clock (s_memtime ticks per s_memrealtime tick x 100 MHz).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I yet-another-halo2-fork_amd/csrc \
//         tools/microbench/lat_bench.hip -o /tmp/lat_bench && /tmp/lat_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../yet-another-halo2-fork_amd/csrc/bn254.h"
using namespace h2g;

template <int V>
__global__ void chain(G1xyzz* io, int iters, unsigned long long* t) {
  G1xyzz p = io[threadIdx.x], q = io[threadIdx.x + 64];
  Fq x = p.X, y = q.Y;
  const unsigned long long r0 = wall_clock64(), c0 = clock64();
  for (int i = 0; i < iters; i++) {
    if (V == 0) x = x * y;
    if (V == 1) x = mul_lat(x, y);
    if (V == 2) p = xyzz_add(p, q);
    if (V == 3) p = xyzz_dbl(p);
  }
  const unsigned long long r1 = wall_clock64(), c1 = clock64();
  if (V < 2) p.X = x;
  io[threadIdx.x] = p;
  if (threadIdx.x == 0) {
    t[0] = r1 - r0;
    t[1] = c1 - c0;
  }
}

int main() {
  G1xyzz* io;
  unsigned long long* t;
  hipMalloc(&io, 128 * sizeof(G1xyzz));
  hipMalloc(&t, 16);
  unsigned long long th[2];
  // arbitrary nonzero coordinates (the chain's values need not be curve points for timing)
  G1xyzz h[128];
  for (int i = 0; i < 128; i++)
    for (int j = 0; j < 8; j++) {
      h[i].X.l[j] = 0x1234567u * (i + 1) + j;
      h[i].Y.l[j] = 0x7654321u * (i + 3) + j;
      h[i].ZZ.l[j] = 1 + j + i;
      h[i].ZZZ.l[j] = 3 + j + i;
    }
  for (int i = 0; i < 128; i++) {
    h[i].X.l[7] &= 0x0fffffff;
    h[i].Y.l[7] &= 0x0fffffff;
  }
  hipMemcpy(io, h, sizeof(h), hipMemcpyHostToDevice);
  const char* names[4] = {"Fq mul (FIPS)", "Fq mul_lat", "xyzz_add", "xyzz_dbl"};
  const int iters = 256;
  for (int rep = 0; rep < 2; rep++)
    for (int v = 0; v < 4; v++) {
      if (v == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, io, iters, t);
      if (v == 1) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, io, iters, t);
      if (v == 2) hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, io, iters, t);
      if (v == 3) hipLaunchKernelGGL(chain<3>, dim3(1), dim3(64), 0, 0, io, iters, t);
      hipMemcpy(th, t, 16, hipMemcpyDeviceToHost);
      if (rep) printf("%-16s %8.1f ns/op  %7.0f shader cycles/op  clock %.2f GHz\n", names[v], th[0] * 10.0 / iters,
                      (double)th[1] / iters, (double)th[1] / (th[0] * 10.0));
    }
  return 0;
}
