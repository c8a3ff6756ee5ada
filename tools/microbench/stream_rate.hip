// HBM streaming shapes on MI355X, to choose the server kernels' form
// (sfl_amd/csrc/sa_api.hip: k_sum_u64, k_decode, k_sum_f64).  Every case
// moves 16-B per lane per access; what varies: accesses in flight per lane
// (U), grid (occupancy-sized grid-stride loop vs one tile per block), and
// non-temporal loads/stores.  Cases: copy (1 read : 1 write, decode's
// ratio) and sum8 (8 reads : 1 write, the wire sum's ratio).  Prints one
// line per case: ms (median of 15 after 10 warm-up launches) and TB/s.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 stream_rate.hip -o stream_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ u64x2 ld(const u64x2* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u64x2* p, u64x2 v) {
  if (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// grid-stride: U accesses per input per lane in flight
template <int K, int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_stride(const u64x2* const* in, u64x2* out, uint64_t n2) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n2; i += U * stride) {
    u64x2 s[U];
#pragma unroll
    for (int u = 0; u < U; u++) s[u] = ld<NTL>(in[0] + i + u * stride);
#pragma unroll
    for (int j = 1; j < K; j++) {
      u64x2 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = ld<NTL>(in[j] + i + u * stride);
#pragma unroll
      for (int u = 0; u < U; u++) s[u] += v[u];
    }
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(out + i + u * stride, s[u]);
  }
  for (; i < n2; i += stride) {
    u64x2 s = ld<NTL>(in[0] + i);
    for (int j = 1; j < K; j++) s += ld<NTL>(in[j] + i);
    st<NTS>(out + i, s);
  }
}

// one tile of 256*U 16-B accesses per block, blocks in order (no loop)
template <int K, int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_tile(const u64x2* const* in, u64x2* out, uint64_t n2) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  u64x2 s[U];
#pragma unroll
  for (int u = 0; u < U; u++) s[u] = base + u * 256 < n2 ? ld<NTL>(in[0] + base + u * 256) : u64x2{0, 0};
#pragma unroll
  for (int j = 1; j < K; j++) {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + u * 256 < n2) s[u] += ld<NTL>(in[j] + base + u * 256);
  }
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + u * 256 < n2) st<NTS>(out + base + u * 256, s[u]);
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;  // 8-B elements per vector
  const uint64_t n2 = n / 2;
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  u64x2* bufs[9];
  for (auto& b : bufs) {
    CHECK(hipMalloc(&b, n2 * 16));
    CHECK(hipMemset(b, 1, n2 * 16));
  }
  const u64x2** din;
  CHECK(hipMalloc(&din, 8 * sizeof(void*)));
  CHECK(hipMemcpy(din, bufs, 8 * sizeof(void*), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto run = [&](auto kern, int K, int U, const char* form, bool ntl, bool nts, int blocks_per_cu) {
    int nb = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, 0));
    const bool tile = form[0] == 't';
    const uint64_t grid = tile ? (n2 + 256ull * U - 1) / (256ull * U)
                               : (uint64_t)ncu * (blocks_per_cu ? std::min(blocks_per_cu, nb) : nb);
    float t[15];
    for (int r = 0; r < 25; r++) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, din, bufs[8], n2);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      if (r >= 10) CHECK(hipEventElapsedTime(&t[r - 10], e0, e1));
    }
    std::sort(t, t + 15);
    const double bytes = (double)(K + 1) * n2 * 16;
    printf("{\"K\": %d, \"U\": %d, \"form\": \"%s\", \"nt_load\": %d, \"nt_store\": %d, \"blocks_per_cu\": %d, "
           "\"grid\": %llu, \"ms\": %.4f, \"TBps\": %.3f}\n",
           K, U, form, ntl, nts, tile ? -1 : (int)(grid / ncu), (unsigned long long)grid, t[7],
           bytes / (t[7] * 1e-3) / 1e12);
    fflush(stdout);
  };
#define CASES(K)                                                         \
  run(k_stride<K, 1, false, false>, K, 1, "stride", 0, 0, 0);            \
  run(k_stride<K, 2, false, false>, K, 2, "stride", 0, 0, 0);            \
  run(k_stride<K, 4, false, false>, K, 4, "stride", 0, 0, 0);            \
  run(k_stride<K, 8, false, false>, K, 8, "stride", 0, 0, 0);            \
  run(k_stride<K, 4, false, false>, K, 4, "stride", 0, 0, 2);            \
  run(k_stride<K, 4, false, false>, K, 4, "stride", 0, 0, 4);            \
  run(k_stride<K, 4, true, false>, K, 4, "stride", 1, 0, 0);             \
  run(k_stride<K, 4, false, true>, K, 4, "stride", 0, 1, 0);             \
  run(k_stride<K, 4, true, true>, K, 4, "stride", 1, 1, 0);              \
  run(k_tile<K, 1, false, false>, K, 1, "tile", 0, 0, 0);                \
  run(k_tile<K, 4, false, false>, K, 4, "tile", 0, 0, 0);                \
  run(k_tile<K, 4, false, true>, K, 4, "tile", 0, 1, 0);                 \
  run(k_tile<K, 4, true, true>, K, 4, "tile", 1, 1, 0);
  CASES(1)
  CASES(2)
  CASES(8)
  return 0;
}
