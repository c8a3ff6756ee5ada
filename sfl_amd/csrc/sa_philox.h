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
#include <string.h>

namespace sa {

struct Normal4 {
  float z[4];
};

#if defined(__HIPCC__)
#define SA_PHX_HD __host__ __device__
#else
#define SA_PHX_HD
#endif

// the round's three-way XORs: one v_bitop3_b32 each on the device (0x96 =
// a ^ b ^ c), where the compiler emits two v_xor_b32
SA_PHX_HD inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

SA_PHX_HD inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c[1], k0);
    const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c[3], k1);
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

#if defined(__HIPCC__)
struct Normal2 {
  float z[2];
};

// Box-Muller of one pair of Philox words -> 2 standard normals, on the
// hardware transcendental units (8 issue cycles each, MI355X_MICROARCH.md):
// v_log_f32 (log2), v_sqrt_f32, and v_sin_f32 / v_cos_f32, which take their
// argument in revolutions -- sin(2*pi*u2) is v_sin_f32(u2) with no range
// reduction.  The libm forms (logf, sqrtf, sincospif) cost ~60 VALU per pair
// and made the noise VALU-bound (k_dp_perturb 0.55 of HBM); the noise is
// this build's own keyed stream (the reference draws unseeded
// np.random.normal), so its parity is distributional and the oracle's numpy
// restatement in the tests is matched within the tolerance
// tests/test_gpu_dp.py states.  u1 >= 2^-24 is a normal float, so v_log_f32
// needs no denormal path.
__device__ __forceinline__ Normal2 box_muller(uint32_t w0, uint32_t w1) {
  const float u1 = (float)((w0 >> 8) + 1u) * 0x1p-24f;  // (0, 1]
  const float u2 = (float)(w1 >> 8) * 0x1p-24f;         // [0, 1)
  const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // -2 ln 2 log2(u1)
  Normal2 o;
  o.z[0] = rad * __builtin_amdgcn_cosf(u2);
  o.z[1] = rad * __builtin_amdgcn_sinf(u2);
  return o;
}

__device__ __forceinline__ void philox_block(uint64_t key, uint64_t blk, uint32_t c[4]) {
  c[0] = (uint32_t)blk;
  c[1] = (uint32_t)(blk >> 32);
  c[2] = c[3] = 0u;
  philox4x32_10(c, (uint32_t)key, (uint32_t)(key >> 32));
}

// The two entry points below are inlined (round 5): with the libm forms of
// Box-Muller they had to stay out of line (the library code was contracted
// with the caller's arithmetic and the fused and standalone kernels then
// differed in the last bit of some normals); the hardware forms are single
// instructions and the build has -ffp-contract=off, so every normal is
// rounded the same way in both kernels -- tests/test_gpu_dp.py checks the
// two paths bit for bit.  Inlined, the key schedule stays on the SALU (the
// key is uniform) and the 10 unrolled rounds cost 2 v_mad_u64_u32 + 2
// three-way XORs each, where the call's rolled loop took ~9 VALU per round.

// Box-Muller pair j (normals 2j, 2j+1) of counter block `blk` under `key`:
// the fused masking kernel needs one pair per lane.
__device__ __forceinline__ Normal2 gauss2(uint64_t key, uint64_t blk, int j) {
  uint32_t c[4];
  philox_block(key, blk, c);
  return j ? box_muller(c[2], c[3]) : box_muller(c[0], c[1]);
}

// All 4 standard normals of counter block `blk` (one Philox block).
__device__ __forceinline__ Normal4 gauss4(uint64_t key, uint64_t blk) {
  uint32_t c[4];
  philox_block(key, blk, c);
  const Normal2 a = box_muller(c[0], c[1]), b = box_muller(c[2], c[3]);
  return Normal4{{a.z[0], a.z[1], b.z[0], b.z[1]}};
}

// 1/u when u is a positive normal power of two whose reciprocal is normal
// (then z·(1/u) rounded once IS z/u rounded once: the exact values are
// equal), else 0 -- the launchers pass it so dp_apply multiplies instead of
// dividing for the common num_updates = 2^k.
__host__ __device__ inline float exact_recip_pow2(float u) {
  uint32_t b;
  memcpy(&b, &u, sizeof(b));
  const uint32_t e = (b >> 23) & 0xFFu;
  if ((b & 0x807FFFFFu) || e == 0 || e >= 253) return 0.0f;
  const uint32_t r = (254u - e) << 23;
  float f;
  memcpy(&f, &r, sizeof(f));
  return f;
}

// x' = x * scale + (z * sigma) / num_updates, float32 in the reference's
// operation order (mechanism_fl.py:112-127: clip, astype(float32) noise,
// noise / num_updates, np.add); inv = exact_recip_pow2(updates) or 0.
template <bool kPow2>
__device__ __forceinline__ float dp_apply_t(float x, float scale, float z, float sigma, float updates, float inv) {
  const float zs = __fmul_rn(z, sigma);
  return __fadd_rn(__fmul_rn(x, scale), kPow2 ? __fmul_rn(zs, inv) : __fdiv_rn(zs, updates));
}

// callers hoist the (kernel-uniform) choice out of their loops: an inline
// select computed the IEEE division for every element even when inv != 0
__device__ __forceinline__ float dp_apply(float x, float scale, float z, float sigma, float updates, float inv) {
  return inv != 0.0f ? dp_apply_t<true>(x, scale, z, sigma, updates, inv)
                     : dp_apply_t<false>(x, scale, z, sigma, updates, inv);
}

// scale = min(1, clip / norm) (mechanism_fl.py:107); with a layer squared
// norm, min(1, clip / sqrt(norm_layer * norm_all)) (:81-84).
// float32 sqrt correctly rounded, as numpy's np.sqrt on float32: the float64
// square root rounded to float32 (innocuous double rounding for sqrt: 53 >=
// 2*24 + 2); gfx950's v_sqrt_f32 is 1 ulp, which the reference would see as
// a different clip scale.
__device__ __forceinline__ float sqrt_f32_rn(float x) { return (float)__dsqrt_rn((double)x); }

// numpy 1.23.5, scalars only from the squared norms on (sa_sumsq_f32: float64
// values): norm_all = np.sqrt(float64 sum); per layer np.sqrt(layer_norm *
// norm_all) with layer_norm = np.sqrt(its float64 square) (the float32 norm,
// exactly); clip / denom in float64; min(1, r); the float32 array times
// that float64 scalar (value-based casting: the scalar rounds to float32).
// Device double sqrt / div are the correctly rounded IEEE operations.
__device__ __forceinline__ float dp_scale(const double* sumsq, const double* sumsq_layer, double clip) {
  const double norm_all = __dsqrt_rn(*sumsq);
  double denom = norm_all;
  if (sumsq_layer) denom = __dsqrt_rn(__dmul_rn(__dsqrt_rn(*sumsq_layer), norm_all));
  const double r = __ddiv_rn(clip, denom);
  return r < 1.0 ? (float)r : 1.0f;
}
#endif

}  // namespace sa
