// Placement probe for the k_envq launch shape: 256-thread (4-wave) workgroups, four resident per CU
// (LDS-limited), one round.  For every CU: the SIMD of each wave index over its workgroups -- whether the
// map-generating wave (wave 2) of co-resident workgroups shares one SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void __launch_bounds__(256) k(unsigned* out) {
  extern __shared__ unsigned lds[];
  unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  lds[threadIdx.x] = hw;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < 400000) {}
  if ((threadIdx.x & 63) == 0) { out[(blockIdx.x * 4 + threadIdx.x / 64) * 2] = hw + lds[0] * 0; out[(blockIdx.x * 4 + threadIdx.x / 64) * 2 + 1] = xcc; }
}
int main() {
  const int B = 1024;
  unsigned* d; hipMalloc(&d, B * 4 * 8);
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 38 * 1024);
  k<<<B, 256, 38 * 1024>>>(d); hipDeviceSynchronize();
  std::vector<unsigned> h(B * 8); hipMemcpy(h.data(), d, B * 32, hipMemcpyDeviceToHost);
  std::map<unsigned, std::vector<int>> cu;  // cu key -> blocks
  for (int b = 0; b < B; b++) {
    unsigned hw = h[b * 8], xcc = h[b * 8 + 1] & 0xf;
    cu[(xcc << 16) | (hw & 0xff00u)].push_back(b);
  }
  std::map<int, int> nblk, distinct2;  // blocks per CU; distinct SIMDs of wave 2 over a CU's blocks
  std::map<int, int> rot;              // SIMD of wave 0 relative: wave w on SIMD (s0 + w) % 4 ?
  int rot_ok = 0, total = 0;
  for (auto& kv : cu) {
    nblk[(int)kv.second.size()]++;
    unsigned m = 0;
    for (int b : kv.second) {
      m |= 1u << ((h[(b * 4 + 2) * 2] >> 4) & 3);
      unsigned s0 = (h[b * 8] >> 4) & 3;
      bool ok = true;
      for (int w = 1; w < 4; w++) ok = ok && ((h[(b * 4 + w) * 2] >> 4) & 3) == ((s0 + w) & 3);
      rot_ok += ok;
      total++;
      rot[(int)s0]++;
    }
    distinct2[__builtin_popcount(m)]++;
  }
  for (auto& kv : nblk) printf("%d workgroups/CU: %d CUs\n", kv.first, kv.second);
  for (auto& kv : distinct2) printf("wave 2 of a CU's workgroups on %d distinct SIMDs: %d CUs\n", kv.first, kv.second);
  printf("workgroups whose wave w sits on SIMD (s0 + w) %% 4: %d / %d; wave 0 SIMD histogram:", rot_ok, total);
  for (auto& kv : rot) printf(" s%d=%d", kv.first, kv.second);
  printf("\n");
  for (int b = 0; b < 8; b++) {
    printf("b%d:", b);
    for (int w = 0; w < 4; w++) printf(" w%d->s%u", w, (h[(b * 4 + w) * 2] >> 4) & 3);
    printf("\n");
  }
}
