#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned long long* out, int iters) {
  uint32_t acc = threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) {
    acc = acc * 3u + 1u;
    acc ^= acc >> 5;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
  if (acc == 42) out[5] = acc;
}
int main() {
  unsigned long long* d; hipMalloc(&d, 64); unsigned long long h[2];
  for (int it : {10000, 100000, 1000000}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, it); hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a); hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, it); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("iters %d: memtime %llu  realtime %llu (x10ns => %.1f us)  event %.1f us  memtime/us %.1f  memtime/iter %.2f\n", it, h[0], h[1], h[1] / 100.0, ms * 1e3, h[0] / (h[1] / 100.0), (double)h[0] / it);
  }
}
