// Checks gfx950 raw-buffer bounds checking granularity: a multi-dword load
// that straddles num_records — are the in-range dwords returned and the rest
// zero (per-dword check), or is the whole access dropped?  Same for stores.
// Standalone tool.  Build: hipcc --offload-arch=gfx950 -O2 oob_test.hip -o oob_test
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__global__ void k(const unsigned* src, unsigned* out, unsigned* dst) {
  const int t = threadIdx.x;  // t = byte offset / 4
  rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 12, 0x00020000);  // 3 dwords valid
  auto a = __builtin_amdgcn_raw_buffer_load_b64(r, 4 * t, 0, 0);
  auto b = __builtin_amdgcn_raw_buffer_load_b128(r, 4 * t, 0, 0);
  out[t * 6 + 0] = a[0];
  out[t * 6 + 1] = a[1];
  for (int j = 0; j < 4; j++) out[t * 6 + 2 + j] = b[j];
  if (t == 0) {
    rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, 12, 0x00020000);
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    v4u d = {101, 102, 103, 104};
    __builtin_amdgcn_raw_buffer_store_b128(d, w, 4, 0, 0);  // dwords 1..4, only 1..2 in range
  }
}
int main() {
  unsigned h[16];
  for (int i = 0; i < 16; i++) h[i] = 0x1000 + i;
  unsigned *s, *o, *d;
  hipMalloc(&s, 64); hipMalloc(&o, 4 * 6 * 4); hipMalloc(&d, 64);
  hipMemcpy(s, h, 64, hipMemcpyHostToDevice);
  hipMemset(d, 0, 64);
  k<<<1, 4>>>(s, o, d);
  unsigned ho[24], hd[16];
  hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
  hipMemcpy(hd, d, sizeof(hd), hipMemcpyDeviceToHost);
  for (int t = 0; t < 4; t++)
    printf("off %2d: b64 %x %x | b128 %x %x %x %x\n", 4 * t, ho[t * 6], ho[t * 6 + 1], ho[t * 6 + 2], ho[t * 6 + 3],
           ho[t * 6 + 4], ho[t * 6 + 5]);
  printf("store b128 at 4 (nrec 12): %u %u %u %u %u %u\n", hd[0], hd[1], hd[2], hd[3], hd[4], hd[5]);
  return 0;
}
