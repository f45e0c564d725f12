// Calibration microbenchmark (diagnostic, not product): cycles per primitive for one wave per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../pgtg_amd/csrc/pgtg_device.h"
using namespace pgtg;

__global__ void k(unsigned long long* out, int iters, int which) {
  Pcg g;
  g.shi = 0x1234 + threadIdx.x; g.slo = 0x9876ull * (threadIdx.x + 1); g.ihi = 7; g.ilo = 0x55555555555ull | 1; g.has = 0; g.buf = 0;
  uint64_t acc = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    switch (which) {
      case 0: acc += pcg_next64(g); break;
      case 1: acc += pcg_int(g, 23 - (i & 7)); break;
      case 2: acc += pcg_double(g) < 0.5 ? 1 : 0; break;
      case 3: { uint32_t x = (uint32_t)acc * 2654435761u + i; acc += x * x; break; }   // dependent mul chain
      case 4: { acc = (acc ^ (acc >> 7)) + i; break; }                                     // dependent alu chain
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = (t1 - t0);
  if (acc == 42) out[1000] = acc;
}

int main() {
  unsigned long long* d; hipMalloc(&d, 8 * 2048);
  unsigned long long h[8];
  const char* names[] = {"pcg_next64", "pcg_int", "pcg_double", "mul32 chain", "alu chain"};
  for (int w = 0; w < 5; w++) {
    int iters = 1000;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, iters, w);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, iters, w);
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("%-12s %.1f cycles/iter (1 wave)\n", names[w], (double)h[0] / iters);
  }
  // memtime vs realtime clock check
  return 0;
}
