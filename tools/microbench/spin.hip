// spin.hip -- a stand-in for a communication kernel in tools/overlap_probe.py:
// `blocks` workgroups of 256 lanes that each stay resident for `usec`
// microseconds (the 100 MHz s_memrealtime clock) and touch no memory, like
// RCCL's few-CU, link-bound kernels.  A tool, not the product.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC spin.hip -o libspin.so
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) k_spin(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

extern "C" int spin_launch(int blocks, double usec, void* stream) {
  if (blocks < 1 || usec < 0) return -1;
  hipLaunchKernelGGL(k_spin, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (uint64_t)(usec * 100.0));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
