// sa_clients_impl.h — the masking kernel: quantize + pairwise PCG64 mask
// expansion + mod-2^64 accumulation for L co-located clients, gfx950.
//
// What one lane does.  A 256-lane workgroup owns a 1024-element tile; lane t
// owns elements [tile + 4t, tile + 4t + 4).  For every mask stream the lane
// keeps the 128-bit PCG64 state positioned at its own element (jumped there
// once in the prologue with the affine-power table), steps it 4 times per
// tile (one draw per element, numpy order) and then jumps it to its next
// tile with one affine map (A^J, inc*G_J) — so every draw costs exactly one
// 128-bit multiply-add and no lane ever waits on another.
//
// Data movement per tile (per lane): one 16-B load per client (4 fp32), two
// 16-B stores for the 4 u64 sums, optional 2x16-B stores per client for the
// wire image.  Consecutive lanes touch consecutive 16-B segments, so each
// wave-instruction moves 1 KiB contiguous (dwordx4 coalescing).  Loads are
// issued at the top of the tile and consumed at the bottom, so their HBM
// latency hides under the tile's PRG work (the kernel is VALU-bound: ~30
// VALU instructions, 10 of them 32x32->64 multiplies, per draw).
//
// Sign handling without branches.  A client adds m = raw + K (K = 2^63-1,
// numpy's Lemire offset) for a peer that sorts after it and subtracts it
// otherwise.  With t = raw ^ smask (smask = 0 or ~0):
//   +m = t + K          (smask = 0)
//   -m = t + (1 - K)    (smask = ~0, since ~raw = -raw - 1)
// and the pair partner gets -t plus the complementary constant.  All the
// constants are folded on the host into one per-client `bias`, and the XOR
// with smask commutes with the XSL-RR rotation, so a signed draw costs the
// same as an unsigned one.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/sfl_sa.h"
#include "pcg128.h"
#include "sa_internal.h"
#include "sa_philox.h"

namespace sa {

// Tuning-only ablations (results are WRONG when nonzero; never shipped):
// 1 = no zero-draw check, 2 = no quantize conversion, 8 = no global
// loads/stores, 16 = stream constants as immediates (no LDS reads).
#ifndef SA_ABLATE
#define SA_ABLATE 0
#endif

struct PowTable {
  Jump e[64];
};
constexpr PowTable make_pow_table() {
  PowTable t{};
  Jump cur{kPcgMult, 1};
  for (int b = 0; b < 64; b++) {
    t.e[b] = cur;
    cur = compose(cur, cur);
  }
  return t;
}
// jump by 2^b draws, b = 0..63 — identical in every translation unit
static __constant__ PowTable kPowTable = make_pow_table();

// ----------------------------------------------------------------------------
// element loads / quantize
// ----------------------------------------------------------------------------
template <typename T>
struct Vec4 {
  T v[4];
};

template <typename T>
__device__ __forceinline__ Vec4<T> load4(const T* __restrict__ p, uint64_t i, uint64_t n) {
  Vec4<T> r;
  if (i + 4 <= n) {
    if constexpr (sizeof(T) == 4) {
      const uint4 u = *reinterpret_cast<const uint4*>(p + i);
      r.v[0] = __builtin_bit_cast(T, u.x);
      r.v[1] = __builtin_bit_cast(T, u.y);
      r.v[2] = __builtin_bit_cast(T, u.z);
      r.v[3] = __builtin_bit_cast(T, u.w);
    } else {
      const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(p + i);
      const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(p + i + 2);
      r.v[0] = __builtin_bit_cast(T, a.x);
      r.v[1] = __builtin_bit_cast(T, a.y);
      r.v[2] = __builtin_bit_cast(T, b.x);
      r.v[3] = __builtin_bit_cast(T, b.y);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) r.v[k] = (i + k < n) ? p[i + k] : T(0);
  }
  return r;
}

__device__ __forceinline__ void store4_u64(uint64_t* __restrict__ p, uint64_t i, uint64_t n,
                                           const uint64_t (&v)[4]) {
  if (i + 4 <= n) {
    reinterpret_cast<ulonglong2*>(p + i)[0] = ulonglong2{v[0], v[1]};
    reinterpret_cast<ulonglong2*>(p + i)[1] = ulonglong2{v[2], v[3]};
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (i + k < n) p[i + k] = v[k];
  }
}

// Raw buffer descriptors (SGPR, built from kernel arguments only, so hipcc
// can prove them wave-uniform) + a 32-bit per-lane byte offset: one shared
// offset VGPR serves every client instead of a 64-bit address per client.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint64_t bytes) {
  const int nrec = bytes > 0xFFFFFFF0ull ? (int)0xFFFFFFF0u : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, nrec, 0x00020000);
}

template <typename T>
__device__ __forceinline__ Vec4<T> bload4(rsrc_t r, uint64_t i, uint64_t n) {
  Vec4<T> out;
  const int off = (int)(i * sizeof(T));
  if (i + 4 <= n) {
    if constexpr (sizeof(T) == 4) {
      const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
#pragma unroll
      for (int k = 0; k < 4; k++) out.v[k] = __builtin_bit_cast(T, (uint32_t)u[k]);
    } else {
      const auto u0 = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
      const auto u1 = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0);
      out.v[0] = __builtin_bit_cast(T, (uint64_t)u0[0] | ((uint64_t)u0[1] << 32));
      out.v[1] = __builtin_bit_cast(T, (uint64_t)u0[2] | ((uint64_t)u0[3] << 32));
      out.v[2] = __builtin_bit_cast(T, (uint64_t)u1[0] | ((uint64_t)u1[1] << 32));
      out.v[3] = __builtin_bit_cast(T, (uint64_t)u1[2] | ((uint64_t)u1[3] << 32));
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (i + k < n) {
        if constexpr (sizeof(T) == 4) {
          out.v[k] = __builtin_bit_cast(T, (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * k, 0, 0));
        } else {
          const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, off + 8 * k, 0, 0);
          out.v[k] = __builtin_bit_cast(T, (uint64_t)u[0] | ((uint64_t)u[1] << 32));
        }
      } else {
        out.v[k] = T(0);
      }
    }
  }
  return out;
}

__device__ __forceinline__ uint64_t bload_u64(rsrc_t r, uint64_t i) {
  const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(i * 8), 0, 0);
  return (uint64_t)u[0] | ((uint64_t)u[1] << 32);
}
struct Vec2u64 {
  uint64_t a, b;
};
// elements i, i+1 (either may lie past n: reads as 0)
__device__ __forceinline__ Vec2u64 bload2_u64(rsrc_t r, uint64_t i, uint64_t n) {
  Vec2u64 o{0, 0};
  if (i + 2 <= n) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 8), 0, 0);
    o.a = (uint64_t)u[0] | ((uint64_t)u[1] << 32);
    o.b = (uint64_t)u[2] | ((uint64_t)u[3] << 32);
  } else if (i < n) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(i * 8), 0, 0);
    o.a = (uint64_t)u[0] | ((uint64_t)u[1] << 32);
  }
  return o;
}
__device__ __forceinline__ void bstore2_u64(rsrc_t r, uint64_t i, uint64_t n, uint64_t v0, uint64_t v1) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  typedef unsigned int v2u __attribute__((ext_vector_type(2)));
  if (i + 2 <= n) {
    const v4u d = {(uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)(i * 8), 0, 0);
  } else if (i < n) {
    const v2u d = {(uint32_t)v0, (uint32_t)(v0 >> 32)};
    __builtin_amdgcn_raw_buffer_store_b64(d, r, (int)(i * 8), 0, 0);
  }
}
// Wave-level transpose through the wave's 256 LDS slots: lane l holds
// elements 4l..4l+3 of the wave's chunk in `in`, gets 2l, 2l+1, 128+2l,
// 129+2l in `out`.  LDS ops of one wave complete in order; the wave barriers
// keep the compiler from moving them across the exchange.
__device__ __forceinline__ void wave_transpose(uint64_t* tw, int lane, const uint64_t (&in)[4],
                                               uint64_t (&out)[4]) {
#pragma unroll
  for (int k = 0; k < 4; k++) tw[4 * lane + k] = in[k];
  __builtin_amdgcn_wave_barrier();
  out[0] = tw[2 * lane];
  out[1] = tw[2 * lane + 1];
  out[2] = tw[128 + 2 * lane];
  out[3] = tw[129 + 2 * lane];
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void bstore_u64(rsrc_t r, uint64_t i, uint64_t v) {
  typedef unsigned int v2u __attribute__((ext_vector_type(2)));
  v2u d;
  d[0] = (uint32_t)v;
  d[1] = (uint32_t)(v >> 32);
  __builtin_amdgcn_raw_buffer_store_b64(d, r, (int)(i * 8), 0, 0);
}

// float -> int64 truncation with x86 "integer indefinite" semantics
// (NaN / inf / |v| >= 2^63 -> INT64_MIN), i.e. numpy's astype(int64) on x86-64.
__device__ __forceinline__ uint64_t trunc_i64(float v) {
  if (!(__builtin_fabsf(v) < 0x1p63f)) return 0x8000000000000000ULL;
  return (uint64_t)(long long)v;
}
__device__ __forceinline__ uint64_t trunc_i64(double v) {
  if (!(__builtin_fabs(v) < 0x1p63)) return 0x8000000000000000ULL;
  return (uint64_t)(long long)v;
}

// q = trunc(x * w * 2^fxp) in the compute type CT (numpy promotion result).
template <typename XT, typename CT>
__device__ __forceinline__ uint64_t quantize(XT x, CT w, const KArgs& a) {
  if constexpr (std::is_integral<CT>::value) {  // int64 arithmetic, wraps mod 2^64
    return (uint64_t)(long long)x * (uint64_t)w * ((uint64_t)1 << a.fxp_bits);
  } else if constexpr (sizeof(CT) == 4) {
    // (x*w)*2^fxp == x*(w*2^fxp) exactly whenever w*2^fxp is finite: scaling
    // by a power of two commutes with rounding, and where the product is
    // subnormal it truncates to 0 either way.  Values of |p| < 2^31 (every
    // gradient in practice) convert with one v_cvt_i32_f32; a wave with any
    // larger / non-finite value takes the full int64 conversion.
    const float ws = __fmul_rn((float)w, a.scale_f);  // wave-uniform
    if (__builtin_isfinite(ws)) {
      const float p = __fmul_rn((float)x, ws);
      if (!__any(!(__builtin_fabsf(p) < 0x1p31f))) return (uint64_t)(int64_t)(int32_t)p;
      return trunc_i64(p);
    }
    const float p = __fmul_rn((float)x, (float)w);
    return trunc_i64(__fmul_rn(p, a.scale_f));
  } else {
    const double p = __dmul_rn((double)x, (double)w);
    return trunc_i64(__dmul_rn(p, a.scale_d));
  }
}

template <typename CT>
__device__ __forceinline__ CT scalar_weight(const ClientArg& c) {
  if constexpr (std::is_integral<CT>::value)
    return (CT)(long long)c.w;
  else
    return (CT)c.w;
}

// ----------------------------------------------------------------------------
// PCG64 draw helpers
// ----------------------------------------------------------------------------
__device__ __forceinline__ u128 ld128(uint64_t lo, uint64_t hi) { return mk128(hi, lo); }

// XSL-RR of the state with the stream's sign mask folded into the XOR.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = {lo, hi};
  return __builtin_bit_cast(uint64_t, v);
}
// XSL-RR output of state s with the sign mask m (0 / ~0) folded into the
// XOR (it commutes with the rotation).  32-bit form: two 3-input XORs
// (v_bitop3, gfx950) and a funnel-shift rotation (two v_alignbit + a swap
// when r >= 32), all full-rate, where the 64-bit shifts of the generic form
// issue at half rate.  Also folds the raw==0 test (raw == 0 <=> hi == lo <=>
// xl == xh == m, a 3-input "all equal" LUT) into a running per-lane minimum.
__device__ __forceinline__ uint64_t draw_signed(u128 s, uint32_t m, uint32_t& zmin) {
  const uint64_t hi = hi64(s), lo = lo64(s);
  const uint32_t s3 = (uint32_t)(hi >> 32);
  const uint32_t xl = xor3((uint32_t)lo, (uint32_t)hi, m);
  const uint32_t xh = xor3((uint32_t)(lo >> 32), s3, m);
  if (!(SA_ABLATE & 1)) {
    uint32_t z;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x7e" : "=v"(z) : "v"(xl), "v"(xh), "v"(m));
    zmin = zmin < z ? zmin : z;
  }
  const uint32_t r = s3 >> 26;                       // alignbit uses r & 31
  const uint32_t a = __builtin_amdgcn_alignbit(xh, xl, r);
  const uint32_t b = __builtin_amdgcn_alignbit(xl, xh, r);
  const bool big = (int32_t)s3 < 0;                  // r >= 32: halves swap
  return big ? pack64(b, a) : pack64(a, b);
}

// One PCG64 step + signed XSL-RR draw + accumulation, hand-scheduled for
// gfx950 (the whole inner loop of the kernel is this block, P times per element).
//
//   S' = S*A + C (mod 2^128) from 32-bit limbs: three 64-bit column chains
//   (limbs 0-1: s0a0 + C01; limbs 1-2: s0a1 + s1a0; limbs 2-3: s0a2 + s1a1 +
//   s2a0 + C23) on v_mad_u64_u32, the four limb-3 products on v_mul_lo_u32,
//   joined by carry adds whose carry-ins are the mads' own carry-outs -- 6
//   mads + 4 mul_lo + 8 adds, no register shuffling.  Then t = rotr(hi^lo^m,
//   hi>>58) in 32-bit halves (v_bitop3 + v_alignbit + swap), the raw==0 test
//   (hi == lo <=> xl == xh == m) folded into a running minimum, and
//   acc_u += t (and acc_v -= t for an internal pair) on 32-bit halves.
//
// Carries live in three SGPR pairs, reused as they die (k1: kE then the acc_u
// carry; k2: kO, c2, then the acc_v carry; k3: discarded carry-outs, c1, c3).
// Every VALU-written SGPR (carries, VCC) is read >= 2 instructions later
// (gfx950 VALU-SGPR-write -> VALU-read hazard).  v0-v9 are fixed scratch (low
// registers, so the kernel's VGPR budget is not raised).
#define SA_PCG_DRAW_ASM                                                                  \
  "v_mad_u64_u32 v[0:1], %[k1], %[s0], %[a0], %[c01]\n\t"   /* E0 = s0a0 + C01, kE */   \
  "v_mad_u64_u32 v[2:3], %[k3], %[s0], %[a1], 0\n\t"        /* O1 = s0a1 */             \
  "v_mad_u64_u32 v[4:5], %[k3], %[s0], %[a2], %[c23]\n\t"   /* E2 = s0a2 + C23 */       \
  "v_mul_lo_u32 v6, %[s0], %[a3]\n\t"                                                    \
  "v_mad_u64_u32 v[2:3], %[k2], %[s1], %[a0], v[2:3]\n\t"   /* O1 += s1a0, kO */        \
  "v_mad_u64_u32 v[4:5], %[k3], %[s1], %[a1], v[4:5]\n\t"                                \
  "v_mul_lo_u32 v7, %[s1], %[a2]\n\t"                                                    \
  "v_mad_u64_u32 v[4:5], %[k3], %[s2], %[a0], v[4:5]\n\t"                                \
  "v_mul_lo_u32 v8, %[s2], %[a1]\n\t"                                                    \
  "v_mul_lo_u32 v9, %[s3], %[a0]\n\t"                                                    \
  "v_add_co_u32_e64 %[s1], %[k3], v1, v2\n\t"              /* r1 = e1 + o1, c1 */       \
  "v_addc_co_u32_e64 %[s3], %[k2], v5, v6, %[k2]\n\t"      /* r3 = e3 + p03 + kO */     \
  "v_add_u32_e32 %[s3], %[s3], v9\n\t"                      /* r3 += p30 */              \
  "v_addc_co_u32_e64 %[s2], %[k2], v4, v3, %[k3]\n\t"      /* r2 = e2 + o2 + c1, c2 */  \
  "v_addc_co_u32_e64 %[s2], %[k3], %[s2], 0, %[k1]\n\t"    /* r2 += kE, c3 */           \
  "v_mov_b32_e32 %[s0], v0\n\t"                             /* r0 = e0 */                \
  "v_addc_co_u32_e64 %[s3], %[k2], %[s3], v7, %[k2]\n\t"   /* r3 += p12 + c2 */         \
  "v_addc_co_u32_e64 %[s3], %[k3], %[s3], v8, %[k3]\n\t"   /* r3 += p21 + c3 */         \
  "v_bitop3_b32 v0, %[s0], %[s2], %[m] bitop3:0x96\n\t"    /* xl */                     \
  "v_bitop3_b32 v1, %[s1], %[s3], %[m] bitop3:0x96\n\t"    /* xh */                     \
  "v_cmp_gt_i32_e32 vcc, 0, %[s3]\n\t"                      /* rot >= 32: swap */        \
  "v_lshrrev_b32_e32 v2, 26, %[s3]\n\t"                     /* rot (& 31 in alignbit) */ \
  "v_bitop3_b32 v3, v0, v1, %[m] bitop3:0x7e\n\t"          /* 0 iff raw == 0 */         \
  "v_alignbit_b32 v4, v1, v0, v2\n\t"                                                    \
  "v_alignbit_b32 v5, v0, v1, v2\n\t"                                                    \
  "v_min_u32_e32 %[zmin], %[zmin], v3\n\t"                                               \
  "v_cndmask_b32_e32 v6, v4, v5, vcc\n\t"                   /* t lo */                   \
  "v_add_co_u32_e64 %[ulo], %[k1], %[ulo], v6\n\t"

#define SA_PCG_DRAW_OUTS                                                                 \
  [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [zmin] "+v"(zmin),          \
      [ulo] "+v"(ulo), [uhi] "+v"(uhi), [k1] "=&s"(k1), [k2] "=&s"(k2), [k3] "=&s"(k3)
#define SA_PCG_DRAW_INS                                                                  \
  [a0] "s"(a0), [a1] "s"(a1), [a2] "s"(a2), [a3] "s"(a3), [c01] "v"(c01), [c23] "v"(c23),  \
      [m] "v"(m)
#define SA_PCG_DRAW_CLOBBERS \
  "vcc", "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9"

__device__ __forceinline__ void pcg_draw_pair(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3, uint32_t a0,
                                              uint32_t a1, uint32_t a2, uint32_t a3, uint64_t c01, uint64_t c23,
                                              uint32_t m, uint32_t& zmin, uint32_t& ulo, uint32_t& uhi,
                                              uint32_t& vlo, uint32_t& vhi) {
  uint64_t k1, k2, k3;
  asm volatile(SA_PCG_DRAW_ASM
               "v_sub_co_u32_e64 %[vlo], %[k2], %[vlo], v6\n\t"
               "v_cndmask_b32_e32 v7, v5, v4, vcc\n\t"  // t hi
               "v_addc_co_u32_e64 %[uhi], %[k1], %[uhi], v7, %[k1]\n\t"
               "v_subb_co_u32_e64 %[vhi], %[k2], %[vhi], v7, %[k2]"
               : SA_PCG_DRAW_OUTS, [vlo] "+v"(vlo), [vhi] "+v"(vhi)
               : SA_PCG_DRAW_INS
               : SA_PCG_DRAW_CLOBBERS);
}
__device__ __forceinline__ void pcg_draw_one(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3, uint32_t a0,
                                             uint32_t a1, uint32_t a2, uint32_t a3, uint64_t c01, uint64_t c23,
                                             uint32_t m, uint32_t& zmin, uint32_t& ulo, uint32_t& uhi) {
  uint64_t k1, k2, k3;
  asm volatile(SA_PCG_DRAW_ASM
               "v_cndmask_b32_e32 v7, v5, v4, vcc\n\t"  // t hi
               "s_nop 0\n\t"
               "v_addc_co_u32_e64 %[uhi], %[k1], %[uhi], v7, %[k1]"
               : SA_PCG_DRAW_OUTS
               : SA_PCG_DRAW_INS
               : SA_PCG_DRAW_CLOBBERS);
}

struct StreamLds {
  uint64_t inc_lo, inc_hi, cj_lo, cj_hi, smask, pad;
};

typedef __attribute__((address_space(3))) const StreamLds* lds_ptr;  // 32-bit LDS address

// Compile-time enumeration of the internal pairs (u < v) of L clients.
template <int L>
struct Pairs {
  static constexpr int count = L * (L - 1) / 2;
  static constexpr int u(int p) {
    int k = p;
    for (int a = 0; a < L; a++) {
      const int row = L - 1 - a;
      if (k < row) return a;
      k -= row;
    }
    return -1;
  }
  static constexpr int v(int p) {
    int k = p;
    for (int a = 0; a < L; a++) {
      const int row = L - 1 - a;
      if (k < row) return a + 1 + k;
      k -= row;
    }
    return -1;
  }
};

// ----------------------------------------------------------------------------
// the kernel
// ----------------------------------------------------------------------------

// waves per SIMD the register allocation must allow: shapes with 17+ streams
// (e.g. 4 local clients + 4 cross = 22) otherwise land a few VGPRs above the
// 3-wave limit of 168
constexpr int clients_waves(int streams) { return streams >= 17 ? 3 : (streams >= 13 && streams <= 15) ? 4 : 2; }

template <typename XT, typename CT, int L, int X>
__global__ void __launch_bounds__(kBlockThreads, clients_waves(Pairs<L>::count + L * X)) k_clients(const KArgs a) {
  constexpr int PI = Pairs<L>::count;
  constexpr int P = PI + L * X;
  constexpr bool kGeneral = (L == 1);  // continue mode + per-element weights
  static_assert(L >= 1 && L <= kMaxLocal, "L");
  static_assert(P <= kMaxStreams, "P");

  const uint64_t n = a.n;
  // lane t of block b owns elements [b*1024 + 4t, +4) of each tile; tiles
  // stride by the grid (16-B loads: 1 KiB contiguous per wave-instruction).
  const uint64_t first = (uint64_t)blockIdx.x * kTileElems + (uint64_t)threadIdx.x * kElemsPerLane;
  const uint64_t stride = (uint64_t)gridDim.x * kTileElems;

  // ---- per-stream constants go to LDS once (broadcast ds_read per use)
  __shared__ StreamLds sl[P > 0 ? P : 1];
  if constexpr (P > 0) {
    for (int j = threadIdx.x; j < P; j += blockDim.x) {
      const StreamArg& s = a.s[j];
      sl[j] = StreamLds{s.inc_lo, s.inc_hi, s.cj_lo, s.cj_hi, s.smask, 0};
    }
    __syncthreads();
  }

  // ---- prologue: jump every stream from draw 0 to this lane's first element
  uint32_t st[P > 0 ? P : 1][4];  // 128-bit states as 32-bit limbs
  if constexpr (P > 0) {
    Jump jl{1, 0};
    uint64_t pos = first;
    for (int b = 0; pos != 0; b++, pos >>= 1) {
      if (pos & 1) jl = compose(jl, kPowTable.e[b]);
    }
#pragma unroll
    for (int j = 0; j < P; j++) {
      const StreamArg& s = a.s[j];
      const u128 v = apply(jl, ld128(s.s_lo, s.s_hi), ld128(s.inc_lo, s.inc_hi));
      st[j][0] = (uint32_t)lo64(v);
      st[j][1] = (uint32_t)(lo64(v) >> 32);
      st[j][2] = (uint32_t)hi64(v);
      st[j][3] = (uint32_t)(hi64(v) >> 32);
    }
  }
  // The tile-to-tile jump is merged into the first draw of the next tile:
  // S_{i+4} -> S_{i+stride+1} is ONE affine step (A^(stride-3), inc*G_(stride-3)),
  // so moving to the next tile costs no multiply beyond the draw itself.
  const u128 AJ1 = ld128(a.aj_lo, a.aj_hi);

  uint32_t zmin = 0xFFFFFFFFu;  // 0 iff some raw PCG64 draw of this lane was 0

  // per-lane XOR digests live in LDS (one lane-private slot per client)
  __shared__ uint64_t dig_lds[L][kBlockThreads];
#pragma unroll
  for (int c = 0; c < L; c++) dig_lds[c][threadIdx.x] = 0;

  rsrc_t rx[L], rw[kGeneral ? L : 1], rm[L];
#pragma unroll
  for (int c = 0; c < L; c++) {
    rx[c] = make_rsrc(a.c[c].x, n * sizeof(XT));
    rm[c] = make_rsrc(a.c[c].masked_out, n * 8);
    if constexpr (kGeneral) rw[c] = make_rsrc(a.c[c].wvec, n * sizeof(CT));
  }
  const rsrc_t rs = make_rsrc(a.sum_out, n * 8);

  // wave-private LDS slots for the output transpose (see below)
  __shared__ uint64_t tr_lds[kBlockThreads * kElemsPerLane];
  const int lane = threadIdx.x & 63;
  uint64_t* const tw = tr_lds + (threadIdx.x & ~63) * kElemsPerLane;

  float dp_s = 1.0f;
  if constexpr (kGeneral && std::is_same<XT, float>::value && std::is_same<CT, float>::value) {
    if (a.dp_on) dp_s = dp_scale(a.dp_sumsq, a.dp_sumsq_layer, a.dp_clip);
  }

  lds_ptr slp = (lds_ptr)(sl);
  int tile = 0;
  // wave-uniform trip count: every lane of a wave runs the wave's last tile
  // (out-of-range elements are masked at load/store) so the transpose has
  // all 64 lanes.
  const uint64_t wave_off = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * 64 * kElemsPerLane);
  for (uint64_t base = (uint64_t)blockIdx.x * kTileElems; base + wave_off < n; base += stride, tile++) {
    const uint64_t i = base + (uint64_t)threadIdx.x * kElemsPerLane;
    const bool jstep = tile > 0;             // uniform: this tile's k=0 draws jump
    const u128 M0 = jstep ? AJ1 : kPcgMult;
    const int add0 = jstep ? 2 : 0;          // u64 offset of C_J1 vs inc in StreamLds

    // ---- issue this tile's loads early; consumed as each element finishes
    Vec4<XT> xv[L];
    Vec4<CT> wv[kGeneral ? L : 1];
    Vec4<uint64_t> pv[kGeneral ? L : 1];
#pragma unroll
    for (int c = 0; c < L; c++) {
      if (kGeneral && a.continue_mode) {
        pv[c] = bload4<uint64_t>(rm[c], i, n);
      } else {
        if (SA_ABLATE & 8) {
#pragma unroll
          for (int k = 0; k < 4; k++) xv[c].v[k] = (XT)(int)(i + k + c);
        } else {
          xv[c] = bload4<XT>(rx[c], i, n);
        }
        if (kGeneral && a.c[c].wvec) wv[c] = bload4<CT>(rw[kGeneral ? c : 0], i, n);
      }
    }
    if constexpr (kGeneral && std::is_same<XT, float>::value && std::is_same<CT, float>::value) {
      if (a.dp_on && !a.continue_mode) {  // fused DP pre-step (sa_mask_dp)
        const Normal4 z = gauss4(a.dp_key, a.dp_block0 + (i >> 2));
#pragma unroll
        for (int k = 0; k < 4; k++) xv[0].v[k] = dp_apply(xv[0].v[k], dp_s, z.z[k], a.dp_sigma, a.dp_updates);
      }
    }

    // ---- element-outer: one draw per stream per element.  Each stream's
    // step is fenced (empty volatile asm on its state, the LDS pointer and
    // the accumulators it touches), so only one stream's constants and
    // temporaries are live at a time: P*4 state VGPRs + L accumulators.
    uint64_t sum[4];
    uint64_t fin[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t al[L], ah[L];  // per-client accumulators as 32-bit halves
#pragma unroll
      for (int c = 0; c < L; c++) {
        al[c] = (uint32_t)a.c[c].bias;
        ah[c] = (uint32_t)(a.c[c].bias >> 32);
      }
      if constexpr (P > 0) {
        const u128 Mk = k == 0 ? M0 : kPcgMult;
        const uint32_t m0 = (uint32_t)lo64(Mk), m1 = (uint32_t)(lo64(Mk) >> 32);
        const uint32_t m2 = (uint32_t)hi64(Mk), m3 = (uint32_t)(hi64(Mk) >> 32);
#pragma unroll
        for (int q = 0; q < P; q++) {
          asm volatile("" : "+v"(slp));  // constants re-read from LDS per draw, never hoisted
          typedef __attribute__((address_space(3))) const uint64_t* lds_u64;
          const lds_u64 cp = (lds_u64)(slp + q) + (k == 0 ? add0 : 0);
          const uint64_t c01 = (SA_ABLATE & 16) ? 2 * q + 1 : cp[0];
          const uint64_t c23 = (SA_ABLATE & 16) ? q : cp[1];
          const uint32_t sm = (SA_ABLATE & 16) ? 0u : (uint32_t)slp[q].smask;
          const int cu = q < PI ? Pairs<L>::u(q) : (q - PI) / (X > 0 ? X : 1);
          if (q < PI) {
            const int cv = Pairs<L>::v(q);
            pcg_draw_pair(st[q][0], st[q][1], st[q][2], st[q][3], m0, m1, m2, m3, c01, c23, sm, zmin, al[cu],
                          ah[cu], al[cv], ah[cv]);
          } else {
            pcg_draw_one(st[q][0], st[q][1], st[q][2], st[q][3], m0, m1, m2, m3, c01, c23, sm, zmin, al[cu],
                         ah[cu]);
          }
        }
      }
      uint64_t acc[L];
#pragma unroll
      for (int c = 0; c < L; c++) acc[c] = pack64(al[c], ah[c]);
      // ---- finish element k: add the quantized value (or the prior pass)
      uint64_t s_k = 0;
#pragma unroll
      for (int c = 0; c < L; c++) {
        if (kGeneral && a.continue_mode) {
          acc[c] += pv[kGeneral ? c : 0].v[k];
        } else {
          const CT w = (kGeneral && a.c[c].wvec) ? wv[kGeneral ? c : 0].v[k] : scalar_weight<CT>(a.c[c]);
          const XT xk = xv[c].v[k];
          if (SA_ABLATE & 2)
            acc[c] += __builtin_bit_cast(uint32_t, (float)xk);
          else
            acc[c] += quantize<XT, CT>(xk, w, a);
        }
        s_k += acc[c];
        if (i + k < n)
          __hip_atomic_fetch_xor(&dig_lds[c][threadIdx.x], acc[c], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        if constexpr (kGeneral) {
          fin[k] = acc[c];
        } else {
          if (a.c[c].masked_out && i + k < n) bstore_u64(rm[c], i + k, acc[c]);
        }
      }
      sum[k] = s_k;
    }

    // ---- outputs.  A lane finishes 4 consecutive u64 (32 B); stored as is,
    // each 16-B store instruction would leave every 128-B line half written.
    // The wave's 256 results are transposed through LDS instead, so lane l
    // stores elements (2l, 2l+1) and (128+2l, 129+2l): each store instruction
    // writes 1 KiB contiguous.
    const uint64_t e0 = i - 4 * (uint64_t)lane + 2 * (uint64_t)lane;  // wave base + 2l
    const uint64_t e1 = e0 + 128;
    if constexpr (kGeneral) {
      if (a.c[0].masked_out) {
        uint64_t v[4];
        wave_transpose(tw, lane, fin, v);
        bstore2_u64(rm[0], e0, n, v[0], v[1]);
        bstore2_u64(rm[0], e1, n, v[2], v[3]);
      }
    }
    if (a.sum_mode != 0 && (!(SA_ABLATE & 8) || sum[0] == 0x123456789ull)) {
      uint64_t v[4];
      wave_transpose(tw, lane, sum, v);
      if (a.sum_mode == 2) {
        const Vec2u64 o0 = bload2_u64(rs, e0, n), o1 = bload2_u64(rs, e1, n);
        v[0] += o0.a;
        v[1] += o0.b;
        v[2] += o1.a;
        v[3] += o1.b;
      }
      bstore2_u64(rs, e0, n, v[0], v[1]);
      bstore2_u64(rs, e1, n, v[2], v[3]);
    }
  }

  // ---- wave-level XOR reduction of the digests, one atomic per wave
  if (a.do_digest) {
#pragma unroll
    for (int c = 0; c < L; c++) {
      uint64_t d = dig_lds[c][threadIdx.x];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) d ^= __shfl_xor(d, off, 64);
      if ((threadIdx.x & 63) == 0 && d) atomicXor((unsigned long long*)&a.digests[c], d);
    }
  }
  if (a.flags && !(SA_ABLATE & 1) && __any(zmin == 0) && (threadIdx.x & 63) == 0)
    atomicOr(a.flags, SA_FLAG_PRG_REJECT);
}

// ----------------------------------------------------------------------------
// launcher
// ----------------------------------------------------------------------------
int occupancy_blocks(const void* kernel);  // sa_api.hip

// Buffer offsets are 32-bit byte offsets, so one launch covers at most
// kChunkElems elements (4 GiB of u64); longer vectors are cut into chunks
// whose streams start kChunkElems draws further on.
constexpr uint64_t kChunkElems = (1ull << 29) - kTileElems;

template <typename XT, typename CT, int L, int X>
int launch_clients(const KArgs& in, void* stream) {
  constexpr int P = Pairs<L>::count + L * X;
  const void* kfn = reinterpret_cast<const void*>(&k_clients<XT, CT, L, X>);
  const int maxb = occupancy_blocks(kfn);
  if (maxb <= 0) return SA_ERR_HIP;
  for (uint64_t off = 0; off < in.n; off += kChunkElems) {
    KArgs a = in;
    a.n = in.n - off < kChunkElems ? in.n - off : kChunkElems;
    if (off) {
      for (int c = 0; c < L; c++) {
        if (a.c[c].x) a.c[c].x = static_cast<const XT*>(a.c[c].x) + off;
        if (a.c[c].wvec) a.c[c].wvec = static_cast<const CT*>(a.c[c].wvec) + off;
        if (a.c[c].masked_out) a.c[c].masked_out += off;
      }
      if (a.sum_out) a.sum_out += off;
      a.dp_block0 += off / kElemsPerLane;
      const Jump jo = jump_of(off);
      for (int j = 0; j < P; j++) {
        const u128 s = apply(jo, mk128(a.s[j].s_hi, a.s[j].s_lo), mk128(a.s[j].inc_hi, a.s[j].inc_lo));
        a.s[j].s_lo = lo64(s);
        a.s[j].s_hi = hi64(s);
      }
    }
    const uint64_t tiles = (a.n + kTileElems - 1) / kTileElems;
    const int grid = (int)(tiles < (uint64_t)maxb ? tiles : (uint64_t)maxb);
    // merged jump-step: S_{i+4} -> S_{i+stride+1}, i.e. stride - 3 draws
    const Jump jj = jump_of((uint64_t)grid * kTileElems - (kElemsPerLane - 1));
    a.aj_lo = lo64(jj.mult);
    a.aj_hi = hi64(jj.mult);
    for (int j = 0; j < P; j++) {
      const u128 cj = jj.gsum * mk128(a.s[j].inc_hi, a.s[j].inc_lo);
      a.s[j].cj_lo = lo64(cj);
      a.s[j].cj_hi = hi64(cj);
    }
    hipLaunchKernelGGL((k_clients<XT, CT, L, X>), dim3(grid), dim3(kBlockThreads), 0,
                       (hipStream_t)stream, a);
    SA_HIP_CHECK(hipGetLastError());
  }
  return SA_OK;
}

}  // namespace sa
