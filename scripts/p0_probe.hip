// p0_probe.hip — cost of the client-injection draw (diagnostic): shader cycles per call of a
// Philox4x32-10 draw, of the geometric gap search (client_next_tick) and of both, as the general
// kernel's P0 runs them, at 1 and 4 waves per SIMD. C3's client (80,000 ppm, bursts of 2048 in
// 16384 ticks).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/p0_probe scripts/p0_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../raft-simulation_amd/csrc/device.hpp"

using namespace rs;

template <int MODE>   // 0 philox, 1 gap, 2 both
__global__ void __launch_bounds__(64) p0_kernel(DevSim S, const unsigned long long* pwg, uint32_t iters,
                                                uint32_t* out) {
  __shared__ uint32_t pw[32];
  if (threadIdx.x < 32) pw[threadIdx.x] = pwg[threadIdx.x];
  __syncthreads();
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  uint32_t t = 16384 + (g & 1023), acc = 0, w = g * 2654435761u;
  for (uint32_t j = 0; j < iters; ++j) {
    if (MODE != 1) {
      const uint4 d = philox(g, P_CLIENT << 8, j, 0, S.key0, S.key1);
      acc += d.y ^ d.z;
      w = d.w;
    } else {
      w = w * 1664525u + 1013904223u;
    }
    if (MODE != 0) {
      const uint32_t nt = client_next_tick(t, w, S, pw);
      acc += nt;
      t = nt == INF ? 16384 : (nt > 1u << 30 ? 16384 : nt);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  DevSim S;
  memset(&S, 0, sizeof(S));
  S.key0 = 1; S.key1 = 0;
  S.client_ppm = 80000; S.client_period = 16384; S.client_burst = 2048;
  S.div_period = make_div(16384); S.div_burst = make_div(2048);
  uint64_t pw[32];
  client_powers(80000, pw);
  S.client_top = -1;
  for (int i = 0; i < 32; ++i)
    if (pw[i]) S.client_top = i;
  unsigned long long* pwg;
  uint32_t* out;
  hipMalloc(&pwg, sizeof(pw));
  hipMalloc(&out, 4);
  hipMemcpy(pwg, pw, sizeof(pw), hipMemcpyHostToDevice);
  const uint32_t iters = 2000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("client_top %d\n", S.client_top);
  for (int wps : {1, 4}) {
    const uint32_t blocks = 1024 * wps;
    for (int mode = 0; mode < 3; ++mode) {
      auto launch = [&] {
        if (mode == 0) hipLaunchKernelGGL(p0_kernel<0>, dim3(blocks), dim3(64), 0, 0, S, pwg, iters, out);
        if (mode == 1) hipLaunchKernelGGL(p0_kernel<1>, dim3(blocks), dim3(64), 0, 0, S, pwg, iters, out);
        if (mode == 2) hipLaunchKernelGGL(p0_kernel<2>, dim3(blocks), dim3(64), 0, 0, S, pwg, iters, out);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      // cycles per call per wave at 2.4 GHz: each SIMD runs wps waves of iters calls
      const double cyc = ms * 1e-3 * 2.4e9 / iters;
      printf("%d wave(s)/SIMD  %-12s %.3f ms  %.0f SIMD cycles per call-round (%.0f per call per wave)\n",
             wps, mode == 0 ? "philox" : mode == 1 ? "gap" : "philox+gap", ms, cyc, cyc / wps);
    }
  }
  return 0;
}
