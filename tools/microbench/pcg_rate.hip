// Microbenchmark: PCG64 (128-bit LCG + XSL-RR) draw rate and integer-multiply
// instruction throughput on gfx950. Standalone; not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 pcg_rate.hip -o pcg_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

typedef unsigned __int128 u128;

__device__ __forceinline__ uint64_t xslrr(u128 s) {
  uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
  unsigned r = hi >> 58;
  uint64_t x = hi ^ lo;
  return (x >> r) | (x << ((-r) & 63));
}

template <int S>
__global__ void __launch_bounds__(256) k_pcg(uint64_t* out, int iters, uint64_t seed) {
  const u128 A = ((u128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
  u128 s[S];
  u128 c[S];
  const unsigned tid = threadIdx.x + blockIdx.x * blockDim.x;
#pragma unroll
  for (int j = 0; j < S; j++) {
    s[j] = ((u128)(seed + j) << 64) | (tid * 0x9E3779B97F4A7C15ULL);
    c[j] = ((u128)j << 64) | (2 * j + 1);
  }
  uint64_t acc = 0;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < S; j++) {
      s[j] = s[j] * A + c[j];
      acc += xslrr(s[j]);
    }
  }
  out[tid] = acc;
}

// raw instruction throughput: 8 independent chains per lane
__global__ void __launch_bounds__(256) k_mad64(uint64_t* out, int iters) {
  uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3;
  uint64_t r0 = a, r1 = b, r2 = a ^ b, r3 = a + b, r4 = a * 3, r5 = b * 5, r6 = 7, r7 = 9;
  for (int i = 0; i < iters; i++) {
#define MAD(r) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(r) : "v"(a), "v"(b) : "vcc");
    MAD(r0) MAD(r1) MAD(r2) MAD(r3) MAD(r4) MAD(r5) MAD(r6) MAD(r7)
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}
__global__ void __launch_bounds__(256) k_mullo(uint64_t* out, int iters) {
  uint32_t a = threadIdx.x + 1;
  uint32_t r[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r[j]) : "v"(a));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
}
__global__ void __launch_bounds__(256) k_mulhi(uint64_t* out, int iters) {
  uint32_t a = threadIdx.x + 1;
  uint32_t r[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r[j]) : "v"(a));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
}
__global__ void __launch_bounds__(256) k_add(uint64_t* out, int iters) {
  uint32_t a = threadIdx.x + 1;
  uint32_t r[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[j]) : "v"(a));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
}
__global__ void __launch_bounds__(256) k_mul24(uint64_t* out, int iters) {
  uint32_t a = threadIdx.x + 1;
  uint32_t r[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r[j]) : "v"(a));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
}
__global__ void __launch_bounds__(256) k_fma64(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0000001;
  double r[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(r[j]) : "v"(b), "v"(a));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
}

__global__ void k_copy(const float4* __restrict__ in, float4* __restrict__ out, size_t n4) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n4; i += stride) out[i] = in[i];
}
__global__ void k_read(const float4* __restrict__ in, float* out, size_t n4) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (; i < n4; i += stride) { float4 v = in[i]; acc += v.x + v.y + v.z + v.w; }
  if (acc == 1234.5f) out[0] = acc;
}

int main() {
  const int blocks = 256 * 8, threads = 256;
  const size_t nthreads = (size_t)blocks * threads;
  uint64_t* d_out;
  CHECK(hipMalloc(&d_out, nthreads * sizeof(uint64_t)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float ms;
  auto timeit = [&](auto launch, const char* name, double ops_per_iter_per_thread, int iters) {
    launch(iters / 10);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    launch(iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double ops = ops_per_iter_per_thread * iters * (double)nthreads;
    // wave-instruction rate per SIMD-cycle at 2.4 GHz: ops/64 per (1024 SIMDs * 2.4e9 * t)
    double per_simd_cycle = ops / 64.0 / (1024.0 * 2.4e9 * ms * 1e-3);
    printf("%-12s %9.3f ms  %10.3f Gop/s  wave-instr/SIMD/cycle@2.4GHz=%.4f (cycles per wave-instr %.2f)\n", name, ms,
           ops / (ms * 1e-3) / 1e9, per_simd_cycle, 1.0 / per_simd_cycle);
  };
  timeit([&](int it) { k_mad64<<<blocks, threads>>>(d_out, it); }, "mad_u64_u32", 8, 20000);
  timeit([&](int it) { k_mullo<<<blocks, threads>>>(d_out, it); }, "mul_lo_u32", 8, 20000);
  timeit([&](int it) { k_mulhi<<<blocks, threads>>>(d_out, it); }, "mul_hi_u32", 8, 20000);
  timeit([&](int it) { k_mul24<<<blocks, threads>>>(d_out, it); }, "mul_u32_u24", 8, 20000);
  timeit([&](int it) { k_add<<<blocks, threads>>>(d_out, it); }, "add_u32", 8, 20000);
  timeit([&](int it) { k_fma64<<<blocks, threads>>>((double*)d_out, it); }, "fma_f64", 8, 20000);
  timeit([&](int it) { k_pcg<1><<<blocks, threads>>>(d_out, it, 42); }, "pcg S=1", 1, 20000);
  timeit([&](int it) { k_pcg<4><<<blocks, threads>>>(d_out, it, 42); }, "pcg S=4", 4, 5000);
  timeit([&](int it) { k_pcg<8><<<blocks, threads>>>(d_out, it, 42); }, "pcg S=8", 8, 2500);

  // HBM bandwidth
  size_t n = (size_t)1 << 28;  // 1 GiB of floats
  float4 *a, *b;
  CHECK(hipMalloc(&a, n * 4));
  CHECK(hipMalloc(&b, n * 4));
  hipMemset(a, 0, n * 4);
  for (int g : {1024, 2048, 4096, 8192}) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      k_copy<<<g, 256>>>(a, b, n / 4);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    printf("copy grid=%d: %.3f ms  %.1f GB/s (r+w)\n", g, ms, 2.0 * n * 4 / (ms * 1e-3) / 1e9);
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      k_read<<<g, 256>>>(a, (float*)b, n / 4);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    printf("read grid=%d: %.3f ms  %.1f GB/s\n", g, ms, 1.0 * n * 4 / (ms * 1e-3) / 1e9);
  }
  CHECK(hipGetLastError());
  return 0;
}
