// PMC calibration (diagnostic, not product): kernels that read or write a KNOWN number of bytes with
// the access widths the step kernels use (4-B/lane car words, 8-B and 16-B/lane records and
// observation stores), each launched 5x, so that rocprofv3's FETCH_SIZE / WRITE_SIZE per dispatch can
// be compared with the true byte count (tools/pmc_calib.py).  1 GiB buffers: far beyond the 256 MiB
// Infinity Cache, so every pass streams from HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <typename T>
__global__ void __launch_bounds__(256) k_read(const T* __restrict__ src, uint64_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const T v = src[i];
    acc ^= reinterpret_cast<const uint32_t*>(&v)[0];
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // data-dependent, never true for the fill pattern
}
template <typename T>
__global__ void __launch_bounds__(256) k_write(T* __restrict__ dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    T v;
    memset(&v, (int)(i & 0x7f), sizeof v);
    dst[i] = v;
  }
}

int main() {
  const uint64_t bytes = 1ull << 30;
  void* a = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(a, 0x11, bytes);
  const int grid = 256 * 8;
  for (int r = 0; r < 5; r++) {
    hipLaunchKernelGGL(k_read<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t*)a, bytes / 4, sink);
    hipLaunchKernelGGL(k_read<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2*)a, bytes / 8, sink);
    hipLaunchKernelGGL(k_read<uint4>, dim3(grid), dim3(256), 0, 0, (const uint4*)a, bytes / 16, sink);
    hipLaunchKernelGGL(k_read<uint8_t>, dim3(grid), dim3(256), 0, 0, (const uint8_t*)a, bytes, sink);
    hipLaunchKernelGGL(k_write<uint32_t>, dim3(grid), dim3(256), 0, 0, (uint32_t*)a, bytes / 4);
    hipLaunchKernelGGL(k_write<uint2>, dim3(grid), dim3(256), 0, 0, (uint2*)a, bytes / 8);
    hipLaunchKernelGGL(k_write<uint4>, dim3(grid), dim3(256), 0, 0, (uint4*)a, bytes / 16);
    hipLaunchKernelGGL(k_write<uint8_t>, dim3(grid), dim3(256), 0, 0, (uint8_t*)a, bytes);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("pmc_calib: %llu bytes per dispatch, 5 rounds of read u32/u64/u128/u8 and write u32/u64/u128/u8\n",
         (unsigned long long)bytes);
  hipFree(a);
  hipFree(sink);
  return 0;
}
