// Placement probe: which SIMD each wave of a 128-thread (2-wave) workgroup lands on, with two such
// workgroups resident per CU (LDS-limited), i.e. whether co-resident workgroups use different SIMDs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void __launch_bounds__(128) k(unsigned* out) {
  extern __shared__ unsigned lds[];
  unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  lds[threadIdx.x] = hw;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < 200000) {}
  if ((threadIdx.x & 63) == 0) { out[(blockIdx.x * 2 + threadIdx.x / 64) * 2] = hw + lds[0] * 0; out[(blockIdx.x * 2 + threadIdx.x / 64) * 2 + 1] = xcc; }
}
int main() {
  const int B = 512;  // 2 per CU
  unsigned* d; hipMalloc(&d, B * 2 * 8);
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 70 * 1024);
  k<<<B, 128, 70 * 1024>>>(d); hipDeviceSynchronize();
  std::vector<unsigned> h(B * 4); hipMemcpy(h.data(), d, B * 16, hipMemcpyDeviceToHost);
  std::map<unsigned, unsigned> cu_simds;  // cu key -> SIMD mask over its blocks' waves
  std::map<unsigned, int> cu_waves;
  for (int b = 0; b < B; b++)
    for (int w = 0; w < 2; w++) {
      unsigned hw = h[(b * 2 + w) * 2], xcc = h[(b * 2 + w) * 2 + 1] & 0xf;
      unsigned key = (xcc << 16) | (hw & 0xff00u);
      cu_simds[key] |= 1u << ((hw >> 4) & 3);
      cu_waves[key]++;
    }
  std::map<int, int> hist;
  for (auto& kv : cu_simds) hist[__builtin_popcount(kv.second) * 10 + cu_waves[kv.first]]++;
  for (auto& kv : hist) printf("distinct SIMDs %d, waves on CU %d: %d CUs\n", kv.first / 10, kv.first % 10, kv.second);
}
