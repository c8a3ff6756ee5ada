// sa_philox.h — counter-based Gaussian noise for the DP pre-step.
//
// Philox4x32-10 (Salmon et al., SC'11; the Random123 reference constants)
// maps (counter, key) -> 4 uniform uint32; two Box-Muller pairs turn them
// into 4 standard normals.  Element e of a vector takes normal (e & 3) of
// counter block e >> 2, so any kernel that visits element e produces the same
// noise -- the fused masking kernel and the standalone perturb kernel agree
// bit for bit.
#pragma once
#include <stdint.h>

namespace sa {

struct Normal4 {
  float z[4];
};

#if defined(__HIPCC__)
#define SA_PHX_HD __host__ __device__
#else
#define SA_PHX_HD
#endif

SA_PHX_HD inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

#if defined(__HIPCC__)
// 4 standard normals of counter block `blk` under `key`.  Never inlined: the
// libm calls inside (logf, sincospif) are otherwise optimised together with
// the caller, and contraction / scheduling decisions that differ between the
// fused masking kernel and the standalone perturb kernel changed the last
// bit of some normals.  As a called function every kernel runs the same
// instruction sequence.
__device__ __noinline__ Normal4 gauss4(uint64_t key, uint64_t blk) {
  uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u};
  philox4x32_10(c, (uint32_t)key, (uint32_t)(key >> 32));
  Normal4 o;
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const float u1 = (float)((c[2 * j] >> 8) + 1u) * 0x1p-24f;  // (0, 1]
    const float u2 = (float)(c[2 * j + 1] >> 8) * 0x1p-24f;     // [0, 1)
    const float rad = sqrtf(-2.0f * logf(u1));
    float s, co;
    sincospif(2.0f * u2, &s, &co);
    o.z[2 * j] = rad * co;
    o.z[2 * j + 1] = rad * s;
  }
  return o;
}

// x' = x * scale + (z * sigma) / num_updates, float32 in the reference's
// operation order (mechanism_fl.py:112-127: clip, astype(float32) noise,
// noise / num_updates, np.add).
__device__ __forceinline__ float dp_apply(float x, float scale, float z, float sigma, float updates) {
  return __fadd_rn(__fmul_rn(x, scale), __fdiv_rn(__fmul_rn(z, sigma), updates));
}

// scale = min(1, clip / norm) in float32 (mechanism_fl.py:107); with a layer
// sum of squares, min(1, clip / sqrt(norm_layer * norm_all)) (:81-84).
__device__ __forceinline__ float dp_scale(const double* sumsq, const double* sumsq_layer, float clip) {
  const float norm_all = (float)sqrt(*sumsq);
  float denom = norm_all;
  if (sumsq_layer) denom = sqrtf(__fmul_rn((float)sqrt(*sumsq_layer), norm_all));
  const float r = __fdiv_rn(clip, denom);
  return r < 1.0f ? r : 1.0f;
}
#endif

}  // namespace sa
