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

// ---- candidate draw formulations (state + inc + signed xsl-rr + accumulate)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
struct St { uint64_t lo, hi; };
// B: explicit 32-bit limbs, inc folded into the mad chains, 64-bit-shift rotation
__device__ __forceinline__ void step_b(St& s, uint64_t c0z, uint64_t c1z, uint64_t chi, uint32_t m, uint64_t& acc) {
  const uint32_t a0 = 0x9FCCF645u, a1 = 0x4385DF64u, a2 = 0x1FC65DA4u, a3 = 0x2360ED05u;
  const uint32_t s0 = (uint32_t)s.lo, s1 = (uint32_t)(s.lo >> 32), s2 = (uint32_t)s.hi, s3 = (uint32_t)(s.hi >> 32);
  const uint64_t p00 = (uint64_t)s0 * a0 + c0z;
  const uint64_t q = (uint64_t)s1 * a0 + (p00 >> 32);
  const uint64_t r = (uint64_t)s0 * a1 + ((q & 0xFFFFFFFFull) + c1z);
  uint64_t h = (uint64_t)s0 * a2 + chi;
  h = (uint64_t)s2 * a0 + h;
  h = (uint64_t)s1 * a1 + h;
  h += (uint64_t)(s0 * a3 + s1 * a2 + s2 * a1 + s3 * a0) << 32;
  h += (q >> 32) + (r >> 32);
  s.lo = (r << 32) | (uint32_t)p00;
  s.hi = h;
  const uint32_t n0 = (uint32_t)s.lo, n1 = (uint32_t)(s.lo >> 32), n2 = (uint32_t)h, n3 = (uint32_t)(h >> 32);
  const uint64_t x = ((uint64_t)xor3(n3, n1, m) << 32) | xor3(n2, n0, m);
  const uint32_t rot = n3 >> 26;
  acc += (x >> rot) + ((x << (63 - rot)) << 1);
}
// A: the u128 formulation the kernel uses today
__device__ __forceinline__ void step_a(u128& s, u128 inc, uint64_t m, uint64_t& acc) {
  const u128 A = ((u128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
  s = s * A + inc;
  const uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
  acc += __builtin_rotateright64(hi ^ lo ^ m, (unsigned)(hi >> 58));
}
template <int S>
__global__ void __launch_bounds__(256) k_step_a(uint64_t* out, int iters, uint64_t seed) {
  u128 s[S];
  const unsigned tid = threadIdx.x + blockIdx.x * blockDim.x;
  for (int j = 0; j < S; j++) s[j] = ((u128)(seed + j) << 64) | (tid * 0x9E3779B97F4A7C15ULL);
  uint64_t acc = 0;
  const u128 inc = ((u128)seed << 64) | 12345;
  const uint64_t m = seed & 1 ? ~0ull : 0;
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int j = 0; j < S; j++) step_a(s[j], inc, m, acc);
  out[tid] = acc;
}
template <int S>
__global__ void __launch_bounds__(256) k_step_b(uint64_t* out, int iters, uint64_t seed) {
  St s[S];
  const unsigned tid = threadIdx.x + blockIdx.x * blockDim.x;
  for (int j = 0; j < S; j++) s[j] = St{tid * 0x9E3779B97F4A7C15ULL, seed + j};
  uint64_t acc = 0;
  const uint64_t c0z = 12345, c1z = 0, chi = seed;
  const uint32_t m = seed & 1 ? ~0u : 0;
  for (int i = 0; i < iters; i++)
#pragma unroll
    for (int j = 0; j < S; j++) step_b(s[j], c0z, c1z, chi, m, acc);
  out[tid] = acc;
}
__global__ void __launch_bounds__(256) k_shr64(uint64_t* out, int iters) {
  uint64_t r[8];
  for (int j = 0; j < 8; j++) r[j] = threadIdx.x * 77 + j;
  uint32_t sh = threadIdx.x & 63;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(r[j]) : "v"(sh));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
}
__global__ void __launch_bounds__(256) k_lshladd(uint64_t* out, int iters) {
  uint64_t r[8];
  for (int j = 0; j < 8; j++) r[j] = threadIdx.x * 77 + j;
  uint64_t b = threadIdx.x;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(r[j]) : "v"(b));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
}
__global__ void __launch_bounds__(256) k_bitop3(uint64_t* out, int iters) {
  uint32_t r[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  uint32_t a = threadIdx.x, b = blockIdx.x;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[j]) : "v"(a), "v"(b));
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = r[0] + r[1] + r[2] + r[3] + r[4] + r[5] + r[6] + r[7];
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
  timeit([&](int it) { k_shr64<<<blocks, threads>>>(d_out, it); }, "lshrrev_b64", 8, 20000);
  timeit([&](int it) { k_lshladd<<<blocks, threads>>>(d_out, it); }, "lshl_add_u64", 8, 20000);
  timeit([&](int it) { k_bitop3<<<blocks, threads>>>(d_out, it); }, "bitop3_b32", 8, 20000);
  timeit([&](int it) { k_step_a<4><<<blocks, threads>>>(d_out, it, 43); }, "draw A S=4", 4, 5000);
  timeit([&](int it) { k_step_b<4><<<blocks, threads>>>(d_out, it, 43); }, "draw B S=4", 4, 5000);
  timeit([&](int it) { k_step_a<1><<<blocks, threads>>>(d_out, it, 43); }, "draw A S=1", 1, 20000);
  timeit([&](int it) { k_step_b<1><<<blocks, threads>>>(d_out, it, 43); }, "draw B S=1", 1, 20000);
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
