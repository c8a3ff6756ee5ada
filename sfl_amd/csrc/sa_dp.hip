// sa_dp.hip — GaussianModelDP pre-step (sfl/security/privacy/mechanism/
// mechanism_fl.py:62-130): the clipping norm (deterministic two-level fp64
// reduction), the standalone clip+noise kernel, and sa_mask_dp, which runs
// the same clip+noise inside the single-client masking kernel.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/sfl_sa.h"
#include "pcg128.h"
#include "sa_internal.h"
#include "sa_philox.h"

namespace sa {

int occupancy_blocks(const void* kernel);  // sa_api.hip

// per-block partial sums of x^2 in fp64 -> partials[blockIdx.x]
__global__ void __launch_bounds__(256) k_sumsq_partial(const float* __restrict__ x, uint64_t n,
                                                       double* __restrict__ partials) {
  double acc = 0.0;
  const uint64_t n4 = n / 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const double v = x[n4 * 4 + threadIdx.x];
    acc += v * v;
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __shared__ double w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (w[0] + w[1]) + (w[2] + w[3]);
}

// fixed-order sum of the partials (deterministic), then the layer's squared
// norm as the reference forms it in float32 (mechanism_fl.py:132-135,
// numpy 1.23.5 on float32 arrays): np.linalg.norm -> sqrt(float32 x.x), ** 2
// in float32, and the layers' values summed in float32 (python sum from 0)
// -> *out (or += *out in float32), a float32 value held in a double
__global__ void __launch_bounds__(64) k_sumsq_final(const double* __restrict__ partials, int k, double* out,
                                                    int accumulate) {
  double acc = 0.0;
  for (int j = threadIdx.x; j < k; j += 64) acc += partials[j];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (threadIdx.x == 0) {
    const float norm = sqrt_f32_rn((float)acc);  // np.linalg.norm: float32 dot, float32 sqrt
    const float sq = __fmul_rn(norm, norm);      // ** 2
    *out = accumulate ? (double)__fadd_rn((float)*out, sq) : (double)sq;
  }
}

struct DpArgs {
  const float* x;
  float* out;
  uint64_t n;
  const double* sumsq;
  const double* sumsq_layer;
  float clip, sigma, updates, inv;  // inv: exact_recip_pow2(updates) or 0
  uint64_t key, block0;
};

// x' = x * scale + N(0, sigma^2) / updates, 4 elements (one Philox block) per lane
__global__ void __launch_bounds__(256) k_dp_perturb(const DpArgs a) {
  const float scale = dp_scale(a.sumsq, a.sumsq_layer, a.clip);
  const uint64_t nb = (a.n + 3) / 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += stride) {
    const Normal4 z = gauss4(a.key, a.block0 + b);
    const uint64_t e = b * 4;
    if (e + 4 <= a.n) {
      const float4 v = reinterpret_cast<const float4*>(a.x)[b];
      float4 o;
      o.x = dp_apply(v.x, scale, z.z[0], a.sigma, a.updates, a.inv);
      o.y = dp_apply(v.y, scale, z.z[1], a.sigma, a.updates, a.inv);
      o.z = dp_apply(v.z, scale, z.z[2], a.sigma, a.updates, a.inv);
      o.w = dp_apply(v.w, scale, z.z[3], a.sigma, a.updates, a.inv);
      reinterpret_cast<float4*>(a.out)[b] = o;
    } else {
      for (int k = 0; e + k < a.n; k++) a.out[e + k] = dp_apply(a.x[e + k], scale, z.z[k], a.sigma, a.updates, a.inv);
    }
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
  const int maxb = occupancy_blocks((const void*)&k_sumsq_partial);
  if (maxb <= 0) return SA_ERR_HIP;
  uint64_t want = (n / 4 + 255) / 256;
  if (want < 1) want = 1;
  int grid = (int)(want < (uint64_t)maxb ? want : (uint64_t)maxb);
  if (grid > SA_DP_PARTIALS) grid = SA_DP_PARTIALS;
  hipLaunchKernelGGL(k_sumsq_partial, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, n, partials);
  SA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_sumsq_final, dim3(1), dim3(64), 0, (hipStream_t)stream, partials, grid, sumsq,
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
  const int maxb = occupancy_blocks((const void*)&k_dp_perturb);
  if (maxb <= 0) return SA_ERR_HIP;
  const uint64_t want = ((n + 3) / 4 + 255) / 256;
  const int grid = (int)(want < (uint64_t)maxb ? want : (uint64_t)maxb);
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
