// Diagnostic: HBM bandwidth of write-only, read-only and copy streams on one GPU (best over shapes).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/wbw tools/micro/wbw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_fill(u32x4* __restrict__ dst, uint64_t n16, unsigned v) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  const u32x4 x = {v, v + 1, v + 2, v + 3};
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n16; b += stride)
#pragma unroll
    for (int j = 0; j < U; j++)
      if (b + j * 256 < n16) {
        if (NT) __builtin_nontemporal_store(x, dst + b + j * 256);
        else dst[b + j * 256] = x;
      }
}
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_read(const u32x4* __restrict__ src, uint64_t n16, unsigned* out) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  unsigned acc = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n16; b += stride) {
    u32x4 r[U];
#pragma unroll
    for (int j = 0; j < U; j++) {
      const uint64_t k = b + j * 256 < n16 ? b + j * 256 : b;
      r[j] = NT ? __builtin_nontemporal_load(src + k) : src[k];
    }
#pragma unroll
    for (int j = 0; j < U; j++) acc ^= r[j].x + r[j].y + r[j].z + r[j].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
// read 1 x 16 B, write W x 16 B per item (the step kernels' read:write mix)
template <int W>
__global__ void __launch_bounds__(256) k_mix(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < n16; b += stride) {
    const u32x4 r = src[b];
#pragma unroll
    for (int j = 0; j < W; j++) dst[(b / 256) * 256 * W + j * 256 + (b % 256)] = r + (unsigned)j;
  }
}
int main() {
  const uint64_t bytes = 2ull << 30, n16 = bytes / 16;
  u32x4 *a, *b;
  unsigned* o;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes * 8);
  hipMalloc(&o, 64);
  hipMemset(a, 1, bytes);
  hipMemset(b, 2, bytes * 8);
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](auto launch) {
    launch();
    hipEventRecord(e0);
    for (int r = 0; r < 10; r++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
  };
  const int wpcs[4] = {0, 4, 8, 16};
  double bw = 0, br = 0;
  for (int wi = 0; wi < 4; wi++) {
    const unsigned gfull = (unsigned)std::min<uint64_t>(n16 / 256, 1u << 30);
    const unsigned g = wpcs[wi] ? ncu * wpcs[wi] : gfull;
    float t[8];
    t[0] = timeit([&] { hipLaunchKernelGGL((k_fill<1, false>), dim3(g), dim3(256), 0, 0, a, n16, 7u); });
    t[1] = timeit([&] { hipLaunchKernelGGL((k_fill<4, false>), dim3(g), dim3(256), 0, 0, a, n16, 7u); });
    t[2] = timeit([&] { hipLaunchKernelGGL((k_fill<1, true>), dim3(g), dim3(256), 0, 0, a, n16, 7u); });
    t[3] = timeit([&] { hipLaunchKernelGGL((k_fill<4, true>), dim3(g), dim3(256), 0, 0, a, n16, 7u); });
    t[4] = timeit([&] { hipLaunchKernelGGL((k_read<1, false>), dim3(g), dim3(256), 0, 0, a, n16, o); });
    t[5] = timeit([&] { hipLaunchKernelGGL((k_read<4, false>), dim3(g), dim3(256), 0, 0, a, n16, o); });
    t[6] = timeit([&] { hipLaunchKernelGGL((k_read<1, true>), dim3(g), dim3(256), 0, 0, a, n16, o); });
    t[7] = timeit([&] { hipLaunchKernelGGL((k_read<4, true>), dim3(g), dim3(256), 0, 0, a, n16, o); });
    printf("wpc %2d  write GB/s:", wpcs[wi]);
    for (int k = 0; k < 4; k++) printf(" %7.0f", bytes / (t[k] * 1e-3) / 1e9), bw = std::max(bw, bytes / (t[k] * 1e-3) / 1e9);
    printf("   read GB/s:");
    for (int k = 4; k < 8; k++) printf(" %7.0f", bytes / (t[k] * 1e-3) / 1e9), br = std::max(br, bytes / (t[k] * 1e-3) / 1e9);
    printf("\n");
  }
  const unsigned gfull = (unsigned)(n16 / 256 / 8);
  float t6 = timeit([&] { hipLaunchKernelGGL((k_mix<6>), dim3(gfull), dim3(256), 0, 0, a, b, n16 / 8); });
  float t18 = timeit([&] { hipLaunchKernelGGL((k_mix<16>), dim3(gfull / 2), dim3(256), 0, 0, a, b, n16 / 16); });
  printf("best write %.0f GB/s, best read %.0f GB/s\n", bw, br);
  printf("mix 1:6  %.0f GB/s (read+write)\n", (bytes / 8) * 7.0 / (t6 * 1e-3) / 1e9);
  printf("mix 1:16 %.0f GB/s (read+write)\n", (bytes / 16) * 17.0 / (t18 * 1e-3) / 1e9);
  return 0;
}
