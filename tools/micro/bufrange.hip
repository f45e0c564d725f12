// Range-check semantics of raw buffer loads that straddle num_records (gfx950): is a 16-byte or
// 4-byte access partly past the end dropped whole, or checked per dword / per byte?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void probe(const uint8_t* buf, uint32_t* out, int nrec) {
  const int ln = threadIdx.x;
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(buf), 0, nrec, 0x00020000);
  const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)ln * 16u, 0, 0);
  const uint32_t d = __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)ln * 4u, 0, 0);
  if (ln < 4) {
    out[ln * 4 + 0] = q[0];
    out[ln * 4 + 1] = q[1];
    out[ln * 4 + 2] = q[2];
    out[ln * 4 + 3] = q[3];
  }
  if (ln < 16) out[16 + ln] = d;
}
int main() {
  uint8_t h[64];
  for (int i = 0; i < 64; i++) h[i] = (uint8_t)(i + 1);
  uint8_t* d;
  uint32_t* o;
  hipMalloc(&d, 64);
  hipMalloc(&o, 32 * 4);
  hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  for (int nrec : {37, 38, 40, 42}) {
    hipMemset(o, 0xff, 32 * 4);
    probe<<<1, 64>>>(d, o, nrec);
    uint32_t r[32];
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    printf("nrec %d\n x4:", nrec);
    for (int i = 0; i < 16; i++) printf(" %08x", r[i]);
    printf("\n x1:");
    for (int i = 16; i < 32; i++) printf(" %08x", r[i]);
    printf("\n");
  }
  return 0;
}
