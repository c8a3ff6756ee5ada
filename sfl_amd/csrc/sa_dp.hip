// sa_dp.hip — GaussianModelDP pre-step (sfl/security/privacy/mechanism/
// mechanism_fl.py:62-130): the clipping norm (deterministic two-level fp64
// reduction), the standalone clip+noise kernel, and sa_mask_dp, which runs
// the same clip+noise inside the single-client masking kernel.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/sfl_sa.h"
#include "pcg128.h"
#include "sa_internal.h"
#include "sa_tiles.h"
#include "sa_philox.h"

namespace sa {

int occupancy_blocks(const void* kernel);  // sa_api.hip

// per-block partial sums of x^2 in fp64 -> partials[blockIdx.x].  Two
// non-temporal 16-byte loads in flight per lane at a 1,024-block grid: the
// fastest of the forms tools/microbench/sumsq_rate.hip timed on MI355X
// (0.065 ms for 100M floats with the final step, 0.77 of HBM, where round
// 4's one load per lane took 0.077 ms; larger grids and a last-block fused
// final step -- whose device-wide fence costs ~45 us -- were slower).  The
// grid depends on n only, so the partials, and the float64 sum, are the
// same on every board and every run.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kSumsqUnroll = 2;

__device__ __forceinline__ double sq4(f32x4 v) {
  return (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
}

__device__ __forceinline__ double block_sum256(double acc) {
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __shared__ double w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = acc;
  __syncthreads();
  return (w[0] + w[1]) + (w[2] + w[3]);
}

__global__ void __launch_bounds__(256) k_sumsq_partial(const float* __restrict__ x, uint64_t n,
                                                       double* __restrict__ partials) {
  double acc = 0.0;
  const uint64_t n4 = n / 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (kSumsqUnroll - 1) * stride < n4; i += kSumsqUnroll * stride) {
    f32x4 v[kSumsqUnroll];
#pragma unroll
    for (int u = 0; u < kSumsqUnroll; u++) v[u] = __builtin_nontemporal_load(x4 + i + u * stride);
#pragma unroll
    for (int u = 0; u < kSumsqUnroll; u++) acc += sq4(v[u]);
  }
  for (; i < n4; i += stride) acc += sq4(__builtin_nontemporal_load(x4 + i));
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const double v = x[n4 * 4 + threadIdx.x];
    acc += v * v;
  }
  const double b = block_sum256(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = b;
}

// fixed-order sum of the partials (deterministic), then the layer's squared
// norm as the reference forms it (mechanism_fl.py:132-135 under numpy
// 1.23.5): np.linalg.norm of a float32 array is sqrt(float32 x.x) in
// float32; `** 2` of that float32 scalar with a python int is a float64
// square (numpy 1.x promotes scalar-scalar operations without value-based
// casting), exact; python's sum adds the layers in float64 from 0 ->
// *out (or *out + sq)
__global__ void __launch_bounds__(256) k_sumsq_final(const double* __restrict__ partials, int k, double* out,
                                                     int accumulate) {
  double acc = 0.0;
  for (int j = threadIdx.x; j < k; j += 256) acc += partials[j];
  acc = block_sum256(acc);
  if (threadIdx.x == 0) {
    const float norm = sqrt_f32_rn((float)acc);        // np.linalg.norm: float32 dot, float32 sqrt
    const double sq = __dmul_rn((double)norm, norm);  // ** 2: float64, exact
    *out = accumulate ? __dadd_rn(*out, sq) : sq;
  }
}

struct DpArgs {
  const float* x;
  float* out;
  uint64_t n;
  const double* sumsq;
  const double* sumsq_layer;
  double clip;                   // python float (the clip divides in float64)
  float sigma, updates, inv;     // inv: exact_recip_pow2(updates) or 0
  uint64_t key, block0;
};

// Grid-stride form (SA_DP_TILE = 0; the tile form below replaced it):
// x' = x * scale + N(0, sigma^2) / updates, 4 elements (one Philox block)
// per lane and block; kDpUnroll blocks per lane and trip, their 16-byte
// loads issued before the noise is formed.  With the libm Box-Muller, 2
// blocks in flight won (0.154 vs 0.164 ms at 100M); with the hardware
// transcendentals and bitop3 Philox, 1 block does (0.173-0.177 vs 0.186 for
// 2 and 0.197-0.200 for 4 on one box, tools/r05_dpu.sh,
// profiles/r05/dp_unroll_ab.txt).  Non-temporal accesses beat plain ones
// (0.165-0.170 vs 0.176-0.178 ms) and a grid of 2x or 4x the occupancy did
// not help (profiles/r05/dp_forms_ab.txt; SA_DP_PLAIN_MEM, SA_DP_GRID_MULT
// select those forms for such A/Bs).
#ifndef SA_DP_UNROLL
#define SA_DP_UNROLL 1
#endif
constexpr int kDpUnroll = SA_DP_UNROLL;

template <bool kPow2>
__device__ __forceinline__ f32x4 dp_apply4(f32x4 v, float scale, const Normal4& z, const DpArgs& a) {
  f32x4 o;
  o.x = dp_apply_t<kPow2>(v.x, scale, z.z[0], a.sigma, a.updates, a.inv);
  o.y = dp_apply_t<kPow2>(v.y, scale, z.z[1], a.sigma, a.updates, a.inv);
  o.z = dp_apply_t<kPow2>(v.z, scale, z.z[2], a.sigma, a.updates, a.inv);
  o.w = dp_apply_t<kPow2>(v.w, scale, z.z[3], a.sigma, a.updates, a.inv);
  return o;
}

template <bool kPow2>
__device__ __forceinline__ void dp_perturb_body(const DpArgs& a) {
  const float scale = dp_scale(a.sumsq, a.sumsq_layer, a.clip);
  const uint64_t nb = (a.n + 3) / 4;
  const uint64_t full = a.n / 4;  // blocks with 4 elements
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(a.x);
  f32x4* o4 = reinterpret_cast<f32x4*>(a.out);
  uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; b + (kDpUnroll - 1) * stride < full; b += kDpUnroll * stride) {
    f32x4 v[kDpUnroll];
#pragma unroll
    for (int u = 0; u < kDpUnroll; u++) {
#ifdef SA_DP_PLAIN_MEM
      v[u] = x4[b + u * stride];
#else
      v[u] = __builtin_nontemporal_load(x4 + b + u * stride);
#endif
    }
    // keep every load ahead of the noise (the scheduler otherwise sinks the
    // second load below the first block's Philox rounds)
#ifndef SA_DP_NO_SCHED_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int u = 0; u < kDpUnroll; u++) {
      const Normal4 z = gauss4(a.key, a.block0 + b + u * stride);
#ifdef SA_DP_PLAIN_MEM
      o4[b + u * stride] = dp_apply4<kPow2>(v[u], scale, z, a);
#else
      __builtin_nontemporal_store(dp_apply4<kPow2>(v[u], scale, z, a), o4 + b + u * stride);
#endif
    }
  }
  for (; b < nb; b += stride) {
    const Normal4 z = gauss4(a.key, a.block0 + b);
    if (b < full) {
      o4[b] = dp_apply4<kPow2>(x4[b], scale, z, a);
    } else {
      const uint64_t e = b * 4;
      for (int k = 0; e + k < a.n; k++)
        a.out[e + k] = dp_apply_t<kPow2>(a.x[e + k], scale, z.z[k], a.sigma, a.updates, a.inv);
    }
  }
}

// Tile form (SA_DP_TILE = T > 0, the product's with T = 1): no grid stride;
// a workgroup owns T * 256 consecutive Philox blocks, lane t blocks t,
// t + 256, ...  The grid is ceil(blocks / (256 T)), so every workgroup
// streams once and retires (the streaming shape that reached 0.77 of HBM for
// a copy, profiles/r05/stream_rate.jsonl "tile").  At 100M: 0.142-0.144 ms
// (0.70 of HBM) for T = 1, 0.148 for 2, 0.157 for 4, against 0.171-0.174 ms
// for the occupancy-sized grid-stride form (SA_DP_TILE = 0,
// profiles/r05/dp_tile_ab.txt).
#ifndef SA_DP_TILE
#define SA_DP_TILE 1
#endif
constexpr int kDpTile = SA_DP_TILE;

template <bool kPow2, int T>
__device__ __forceinline__ void dp_perturb_tile(const DpArgs& a) {
  const float scale = dp_scale(a.sumsq, a.sumsq_layer, a.clip);
  const uint64_t nb = (a.n + 3) / 4;
  const uint64_t full = a.n / 4;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(a.x);
  f32x4* o4 = reinterpret_cast<f32x4*>(a.out);
  const uint64_t b0 = (uint64_t)stream_tile() * (256 * T) + threadIdx.x;
  if (b0 + (uint64_t)(T - 1) * 256 < full) {
    f32x4 v[T];
#pragma unroll
    for (int u = 0; u < T; u++) v[u] = __builtin_nontemporal_load(x4 + b0 + u * 256);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < T; u++) {
      const Normal4 z = gauss4(a.key, a.block0 + b0 + u * 256);
      __builtin_nontemporal_store(dp_apply4<kPow2>(v[u], scale, z, a), o4 + b0 + u * 256);
    }
    return;
  }
  for (int u = 0; u < T; u++) {
    const uint64_t b = b0 + (uint64_t)u * 256;
    if (b >= nb) break;
    const Normal4 z = gauss4(a.key, a.block0 + b);
    if (b < full) {
      o4[b] = dp_apply4<kPow2>(x4[b], scale, z, a);
    } else {
      const uint64_t e = b * 4;
      for (int k = 0; e + k < a.n; k++)
        a.out[e + k] = dp_apply_t<kPow2>(a.x[e + k], scale, z.z[k], a.sigma, a.updates, a.inv);
    }
  }
}

__global__ void __launch_bounds__(256) k_dp_perturb(const DpArgs a) {
  if constexpr (kDpTile > 0) {
    if (a.inv != 0.0f)
      dp_perturb_tile<true, kDpTile>(a);
    else
      dp_perturb_tile<false, kDpTile>(a);
  } else {
    if (a.inv != 0.0f)  // uniform: num_updates a power of two, multiply by its exact reciprocal
      dp_perturb_body<true>(a);
    else
      dp_perturb_body<false>(a);
  }
}

}  // namespace sa

using namespace sa;

static bool dp_ok(const sa_dp* dp, const char* who) {
  if (!dp || !dp->sumsq || !(dp->num_updates > 0.0f) || (dp->counter0 & 3)) {
    sa_set_error("%s: bad sa_dp (sumsq set, num_updates > 0, counter0 %% 4 == 0 required)", who);
    return false;
  }
  return true;
}

extern "C" int sa_sumsq_f32(const float* x, uint64_t n, double* partials, double* sumsq, int accumulate,
                            void* stream) {
  if ((n > 0 && !x) || !partials || !sumsq || ((uintptr_t)x & 15)) {  // n == 0: x unread, *sumsq (+)= 0
    sa_set_error("sa_sumsq_f32: bad arguments (x must be 16-byte aligned)");
    return SA_ERR_ARG;
  }
  // the grid depends on n only (not on the device's occupancy): the same
  // partials, so the same float64 sum, on every board
  uint64_t want = (n / 4 + 255) / 256;
  if (want < 1) want = 1;
  const int grid = (int)(want < (uint64_t)SA_DP_PARTIALS ? want : (uint64_t)SA_DP_PARTIALS);
  hipLaunchKernelGGL(k_sumsq_partial, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, n, partials);
  SA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_sumsq_final, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, grid, sumsq,
                     accumulate);
  SA_HIP_CHECK(hipGetLastError());
  return SA_OK;
}

extern "C" int sa_dp_perturb_f32(const float* x, uint64_t n, const sa_dp* dp, float* out, void* stream) {
  if ((n > 0 && (!x || !out)) || ((uintptr_t)x & 15) || ((uintptr_t)out & 15)) {
    sa_set_error("sa_dp_perturb_f32: bad arguments (16-byte aligned x and out required)");
    return SA_ERR_ARG;
  }
  if (!dp_ok(dp, "sa_dp_perturb_f32")) return SA_ERR_ARG;
  if (n == 0) return SA_OK;
  DpArgs a{x,  out, n, dp->sumsq, dp->sumsq_layer, dp->l2_norm_clip, dp->noise_std, dp->num_updates,
           exact_recip_pow2(dp->num_updates), dp->key, dp->counter0 / 4};
#ifndef SA_DP_GRID_MULT
#define SA_DP_GRID_MULT 1
#endif
  int grid;
  if (kDpTile > 0) {
    const uint64_t want = ((n + 3) / 4 + 256 * kDpTile - 1) / (256 * kDpTile);
    if (want > 0x7fffffffull) {
      sa_set_error("sa_dp_perturb_f32: n too large for the tile grid");
      return SA_ERR_ARG;
    }
    grid = (int)want;
  } else {
    const int maxb = occupancy_blocks((const void*)&k_dp_perturb) * SA_DP_GRID_MULT;
    if (maxb <= 0) return SA_ERR_HIP;
    const uint64_t want = ((n + 3) / 4 + 255) / 256;
    grid = (int)(want < (uint64_t)maxb ? want : (uint64_t)maxb);
  }
  hipLaunchKernelGGL(k_dp_perturb, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  SA_HIP_CHECK(hipGetLastError());
  return SA_OK;
}

extern "C" int sa_mask_dp(const float* x, uint64_t n, double weight, int fxp_bits, const sa_mask_stream* streams,
                          int n_streams, const sa_dp* dp, uint64_t* out, uint64_t* sum_accum, uint64_t* digest,
                          uint32_t* flags, void* stream) {
  if (!x && n > 0) {
    sa_set_error("sa_mask_dp: x is required");
    return SA_ERR_ARG;
  }
  if (!dp_ok(dp, "sa_mask_dp")) return SA_ERR_ARG;
  return sa_mask_impl(x, SA_F32, SA_F32, n, weight, nullptr, fxp_bits, streams, n_streams, out, sum_accum, digest,
                      flags, stream, dp);
}
