#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void __launch_bounds__(256) k(unsigned* out) {
  unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < 200000) {}
  if ((threadIdx.x & 63) == 0) { out[(blockIdx.x * 4 + threadIdx.x / 64) * 2] = hw; out[(blockIdx.x * 4 + threadIdx.x / 64) * 2 + 1] = xcc; }
}
int main() {
  const int B = 1024;
  unsigned* d; hipMalloc(&d, B * 4 * 8);
  k<<<B, 256>>>(d); hipDeviceSynchronize();
  std::vector<unsigned> h(B * 8); hipMemcpy(h.data(), d, B * 32, hipMemcpyDeviceToHost);
  std::map<unsigned, std::vector<int>> cu;  // cu key -> blocks
  int distinct_simd_blocks = 0;
  for (int b = 0; b < B; b++) {
    unsigned s = 0;
    for (int w = 0; w < 4; w++) s |= 1u << ((h[(b * 4 + w) * 2] >> 4) & 3);
    distinct_simd_blocks += s == 15;
    unsigned hw = h[b * 8], xcc = h[b * 8 + 1] & 0xf;
    unsigned key = (xcc << 16) | (hw & 0xff00u) | ((hw >> 13) & 0x7) << 12 | ((hw >> 12) & 1) << 15;
    cu[key].push_back(b);
  }
  printf("blocks with 4 distinct SIMDs: %d/%d, distinct CU keys %zu\n", distinct_simd_blocks, B, cu.size());
  for (int b = 0; b < 12; b++) {
    printf("b%d:", b);
    for (int w = 0; w < 4; w++) { unsigned hw = h[(b * 4 + w) * 2]; printf(" [w%u s%u cu%u sh%u se%u xcc%u]", hw & 15, (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7, h[(b*4+w)*2+1] & 0xf); }
    printf("\n");
  }
  int n = 0;
  for (auto& kv : cu) { if (n++ < 6) { printf("cu %x:", kv.first); for (int b : kv.second) printf(" %d(simd0 of w0=%u)", b, (h[b*8] >> 4) & 3); printf("\n"); } }
  std::map<size_t,int> hist; for (auto& kv : cu) hist[kv.second.size()]++;
  for (auto& kv : hist) printf("%zu blocks/cu: %d cus\n", kv.first, kv.second);
}
