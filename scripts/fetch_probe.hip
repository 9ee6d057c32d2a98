// fetch_probe.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against known byte
// counts for the access shapes the tick kernel uses (MI355X_MICROARCH.md §HBM warns that the
// counters are exact only for what was measured). Every kernel walks a 1 GiB buffer once (4x the
// 256 MiB Infinity Cache; consecutive kernels alternate buffers so nothing is cache-resident):
//   rd_u32_contig    4 B per lane, lanes contiguous            node SoA words (launch start)
//   rd_msg32_contig  32 B per lane (2 x 16 B), lanes contiguous a queue slot row, heads aligned
//   rd_msg32_s128    32 B per lane at a 128 B stride            queue slots, heads diverged
//   wr_u32_contig / wr_msg32_contig / wr_msg32_s128             the same shapes stored
// Prints "probe KERNEL span_bytes requested_bytes" per kernel: span = bytes of the 128 B lines the
// kernel touches, requested = bytes the lanes load or store. scripts/summarize_profile.py divides
// the counters by these. Build and run: see scripts/profile.sh.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr size_t BYTES = 1ull << 30;

__global__ void rd_u32_contig(const uint32_t* a, uint32_t* sink) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const uint32_t v = a[i];
  if (v == 0xDEADBEEFu) sink[0] = v;
}
__global__ void rd_msg32_contig(const uint4* a, uint32_t* sink) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const uint4 v = a[2 * i], w = a[2 * i + 1];
  if ((v.x ^ v.w ^ w.y ^ w.z) == 0xDEADBEEFu) sink[0] = v.x;
}
__global__ void rd_msg32_s128(const uint4* a, uint32_t* sink) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const uint4 v = a[8 * i], w = a[8 * i + 1];
  if ((v.x ^ v.w ^ w.y ^ w.z) == 0xDEADBEEFu) sink[0] = v.x;
}
__global__ void wr_u32_contig(uint32_t* a) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  a[i] = (uint32_t)i;
}
__global__ void wr_msg32_contig(uint4* a) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  a[2 * i] = make_uint4((uint32_t)i, 1, 2, 3);
  a[2 * i + 1] = make_uint4(4, 5, 6, 7);
}
__global__ void wr_msg32_s128(uint4* a) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  a[8 * i] = make_uint4((uint32_t)i, 1, 2, 3);
  a[8 * i + 1] = make_uint4(4, 5, 6, 7);
}

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main() {
  void *a = nullptr, *b = nullptr;
  uint32_t* sink = nullptr;
  CHECK(hipMalloc(&a, BYTES));
  CHECK(hipMalloc(&b, BYTES));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(a, 1, BYTES));
  CHECK(hipMemset(b, 1, BYTES));
  CHECK(hipDeviceSynchronize());
  const dim3 blk(256);
  const unsigned g4 = BYTES / 4 / 256, g32 = BYTES / 32 / 256, g128 = BYTES / 128 / 256;
  hipLaunchKernelGGL(rd_u32_contig, dim3(g4), blk, 0, 0, (const uint32_t*)a, sink);
  hipLaunchKernelGGL(rd_msg32_contig, dim3(g32), blk, 0, 0, (const uint4*)b, sink);
  hipLaunchKernelGGL(rd_msg32_s128, dim3(g128), blk, 0, 0, (const uint4*)a, sink);
  hipLaunchKernelGGL(wr_u32_contig, dim3(g4), blk, 0, 0, (uint32_t*)b);
  hipLaunchKernelGGL(wr_msg32_contig, dim3(g32), blk, 0, 0, (uint4*)a);
  hipLaunchKernelGGL(wr_msg32_s128, dim3(g128), blk, 0, 0, (uint4*)b);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  printf("probe rd_u32_contig %zu %zu\n", BYTES, BYTES);
  printf("probe rd_msg32_contig %zu %zu\n", BYTES, BYTES);
  printf("probe rd_msg32_s128 %zu %zu\n", BYTES, BYTES / 4);
  printf("probe wr_u32_contig %zu %zu\n", BYTES, BYTES);
  printf("probe wr_msg32_contig %zu %zu\n", BYTES, BYTES);
  printf("probe wr_msg32_s128 %zu %zu\n", BYTES, BYTES / 4);
  return 0;
}
