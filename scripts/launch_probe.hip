// launch_probe.hip — fixed costs of a dispatch on MI355X (diagnostic): the device time of
// back-to-back launches of a kernel that does nothing, with the steady kernel's grid and LDS, and
// of kernels that dirty one 64-B piece of a line per 640-B block over C2's 65,536 blocks (the
// steady kernel's write-back shape), with plain and with write-through (nontemporal) stores.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_probe scripts/launch_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) empty_kernel(uint32_t* p) {
  extern __shared__ uint32_t lds[];
  if (threadIdx.x == 1000) lds[0] = p[0];
}

// one lane per block: 4 x 16 B stores into the first line of its 640-B block
__global__ void __launch_bounds__(256) dirty_kernel(uint32_t* p, uint32_t v) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  uint4* b = reinterpret_cast<uint4*>(p + (size_t)c * 160 + 8);
  for (int i = 0; i < 4; ++i) b[i] = make_uint4(v, v + i, c, 0);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) dirty_nt_kernel(uint32_t* p, uint32_t v) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  u32x4* b = reinterpret_cast<u32x4*>(p + (size_t)c * 160 + 8);
  for (int i = 0; i < 4; ++i) {
    const u32x4 x = {v, v + i, c, 0u};
    __builtin_nontemporal_store(x, b + i);
  }
}

// empty, but each workgroup's first 5 threads add to 64 copies of a counter block at the end
__global__ void __launch_bounds__(256) atomics_kernel(unsigned long long* ctr) {
  __syncthreads();
  if (threadIdx.x < 5) atomicAdd(&ctr[(blockIdx.x % 64) * 32 + threadIdx.x], 1ull);
}

// the load shape of the steady kernel: 31 x 16 B per lane from its block, summed
__global__ void __launch_bounds__(256) load_kernel(const uint32_t* p, uint32_t* out) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  const uint4* b = reinterpret_cast<const uint4*>(p + (size_t)c * 160);
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 31; ++i) {
    const uint4 x = b[i];
    s += x.x ^ x.y ^ x.z ^ x.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

template <typename F>
static float time_launches(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.0f / reps;   // us per launch
}

int main() {
  const uint32_t C = 65536, blocks = C / 256;
  uint32_t* p = nullptr;
  hipMalloc(&p, (size_t)C * 640);
  hipMemset(p, 0, (size_t)C * 640);
  const int reps = 50;
  for (int lds : {0, 4096, 40960}) {
    const float us = time_launches([&] {
      hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), lds, 0, p);
    }, reps);
    printf("empty kernel, %u x 256 threads, %d B dynamic LDS: %.2f us per launch\n", blocks, lds, us);
  }
  {
    hipEvent_t e0, e1;
    hipEventCreateWithFlags(&e0, hipEventDisableSystemFence);
    hipEventCreateWithFlags(&e1, hipEventDisableSystemFence);
    printf("empty kernel with start/stop events in its packet: %.2f us per launch\n", time_launches([&] {
      hipExtLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 40960, 0, e0, e1, 0, p);
    }, reps));
  }
  unsigned long long* ctr = nullptr;
  hipMalloc(&ctr, 64 * 32 * 8);
  printf("empty kernel + 5 atomics per workgroup: %.2f us per launch\n", time_launches([&] {
    hipLaunchKernelGGL(atomics_kernel, dim3(blocks), dim3(256), 0, 0, ctr);
  }, reps));
  uint32_t v = 1;
  printf("dirty plain: %.2f us per launch\n", time_launches([&] {
    hipLaunchKernelGGL(dirty_kernel, dim3(blocks), dim3(256), 0, 0, p, v++);
  }, reps));
  printf("dirty nt:    %.2f us per launch\n", time_launches([&] {
    hipLaunchKernelGGL(dirty_nt_kernel, dim3(blocks), dim3(256), 0, 0, p, v++);
  }, reps));
  printf("load 31x16B: %.2f us per launch\n", time_launches([&] {
    hipLaunchKernelGGL(load_kernel, dim3(blocks), dim3(256), 0, 0, p, p);
  }, reps));
  printf("load + dirty: %.2f us per pair\n", time_launches([&] {
    hipLaunchKernelGGL(load_kernel, dim3(blocks), dim3(256), 0, 0, p, p);
    hipLaunchKernelGGL(dirty_kernel, dim3(blocks), dim3(256), 0, 0, p, v++);
  }, reps));
  hipFree(p);
  return 0;
}
