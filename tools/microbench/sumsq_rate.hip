// Forms of the DP clipping norm's reduction (sfl_amd/csrc/sa_dp.hip:
// k_sumsq_partial + k_sumsq_final), to choose the product's: sum of x^2 in
// float64 over n float32, deterministic (fixed partial grouping).  Varies the
// partial kernel's grid G, 16-B loads in flight per lane U, non-temporal
// loads, and the final step: a 64-lane serial sum (round 4), a 256-lane
// parallel tree, or fused into the partial kernel through a last-block
// ticket (counter zeroed by hipMemsetAsync).  Prints per case the median of
// 25 timed sequences after 10 warm-ups: ms and TB/s of the 4n algorithmic bytes.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 sumsq_rate.hip -o sumsq_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f32x4 ld(const f32x4* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

__device__ __forceinline__ double sq4(f32x4 v) {
  return (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
}

__device__ __forceinline__ double block_sum(double acc) {
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __shared__ double w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = acc;
  __syncthreads();
  return (w[0] + w[1]) + (w[2] + w[3]);
}

// the partial sums; FUSED: the last block to finish also sums the partials
// (fixed order, so deterministic whichever block is last)
template <int U, bool NT, bool FUSED>
__global__ void __launch_bounds__(256) k_partial(const f32x4* __restrict__ x, uint64_t n4, double* partials,
                                                 unsigned* ticket, double* out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double acc = 0.0;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld<NT>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; u++) acc += sq4(v[u]);
  }
  for (; i < n4; i += stride) acc += sq4(ld<NT>(x + i));
  const double b = block_sum(acc);
  if (!FUSED) {
    if (threadIdx.x == 0) partials[blockIdx.x] = b;
    return;
  }
  __shared__ bool last;
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = b;
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  double s = 0.0;
  for (uint32_t j = threadIdx.x; j < gridDim.x; j += 256) s += __builtin_nontemporal_load(&partials[j]);
  s = block_sum(s);
  if (threadIdx.x == 0) {
    *out = s;
    *ticket = 0;
  }
}

__global__ void __launch_bounds__(64) k_final64(const double* partials, int k, double* out) {
  double acc = 0.0;
  for (int j = threadIdx.x; j < k; j += 64) acc += partials[j];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (threadIdx.x == 0) *out = acc;
}

__global__ void __launch_bounds__(256) k_final256(const double* partials, int k, double* out) {
  double acc = 0.0;
  for (int j = threadIdx.x; j < k; j += 256) acc += partials[j];
  acc = block_sum(acc);
  if (threadIdx.x == 0) *out = acc;
}

struct Case {
  const char* name;
  int grid;
  void (*run)(const f32x4*, uint64_t, double*, unsigned*, double*, int, hipStream_t);
};

template <int U, bool NT, int FIN>  // FIN: 0 serial 64, 1 tree 256, 2 fused (memset + last block)
void run_case(const f32x4* x, uint64_t n4, double* part, unsigned* ticket, double* out, int grid, hipStream_t s) {
  if (FIN == 2) {
    CHECK(hipMemsetAsync(ticket, 0, sizeof(unsigned), s));
    hipLaunchKernelGGL((k_partial<U, NT, true>), dim3(grid), dim3(256), 0, s, x, n4, part, ticket, out);
    return;
  }
  hipLaunchKernelGGL((k_partial<U, NT, false>), dim3(grid), dim3(256), 0, s, x, n4, part, ticket, out);
  if (FIN == 0)
    hipLaunchKernelGGL(k_final64, dim3(1), dim3(64), 0, s, part, grid, out);
  else
    hipLaunchKernelGGL(k_final256, dim3(1), dim3(256), 0, s, part, grid, out);
}

// fused without the memset: the ticket self-resets (valid after a zeroed start)
template <int U, bool NT>
void run_selfreset(const f32x4* x, uint64_t n4, double* part, unsigned* ticket, double* out, int grid, hipStream_t s) {
  hipLaunchKernelGGL((k_partial<U, NT, true>), dim3(grid), dim3(256), 0, s, x, n4, part, ticket, out);
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
  const uint64_t n4 = n / 4;
  f32x4* x;
  double *part, *out;
  unsigned* ticket;
  CHECK(hipMalloc(&x, n4 * 16));
  CHECK(hipMalloc(&part, 8192 * 8));
  CHECK(hipMalloc(&out, 8));
  CHECK(hipMalloc(&ticket, 4));
  CHECK(hipMemset(ticket, 0, 4));
  std::vector<float> h(n4 * 4);
  for (uint64_t i = 0; i < n4 * 4; i++) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  CHECK(hipMemcpy(x, h.data(), n4 * 16, hipMemcpyHostToDevice));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  std::vector<Case> cases;
  for (int g : {1024, 2048, 4096}) {
    cases.push_back({"U1 serial64 (round 4)", g, run_case<1, false, 0>});
    cases.push_back({"U4 serial64", g, run_case<4, false, 0>});
    cases.push_back({"U4 tree256", g, run_case<4, false, 1>});
    cases.push_back({"U4 NT tree256", g, run_case<4, true, 1>});
    cases.push_back({"U2 NT tree256", g, run_case<2, true, 1>});
    cases.push_back({"U4 NT fused+memset", g, run_case<4, true, 2>});
    cases.push_back({"U4 NT fused selfreset", g, run_selfreset<4, true>});
    cases.push_back({"U8 NT fused selfreset", g, run_selfreset<8, true>});
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  double ref = -1;
  for (int pass = 0; pass < 2; pass++) {
    for (auto& c : cases) {
      for (int w = 0; w < 10; w++) c.run(x, n4, part, ticket, out, c.grid, s);
      std::vector<float> ms;
      for (int r = 0; r < 25; r++) {
        CHECK(hipEventRecord(e0, s));
        c.run(x, n4, part, ticket, out, c.grid, s);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float t;
        CHECK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      double o;
      CHECK(hipMemcpy(&o, out, 8, hipMemcpyDeviceToHost));
      if (ref < 0) ref = o;
      const double med = ms[ms.size() / 2];
      printf("{\"pass\": %d, \"case\": \"%s\", \"grid\": %d, \"ms\": %.5f, \"TBps\": %.3f, \"hbm_frac\": %.3f, "
             "\"rel_diff\": %.3g}\n",
             pass, c.name, c.grid, med, 4.0 * n / (med * 1e-3) / 1e12, 4.0 * n / (med * 1e-3) / 8e12,
             (o - ref) / ref);
    }
  }
  return 0;
}
