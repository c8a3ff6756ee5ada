// sa_clients_impl.h — the masking kernel: quantize + pairwise PCG64 mask
// expansion + mod-2^64 accumulation for L co-located clients, gfx950.
//
// What one lane does.  A 256-lane workgroup owns a 512-element tile; lane t
// owns elements [tile + 2t, tile + 2t + 2) (8-B fp32 loads, 16-B u64 stores:
// 512 B / 1 KiB contiguous per wave instruction).  For every mask stream the
// lane keeps one 128-bit PCG64 state and advances it with exactly one affine
// step per element: the first element of a tile is reached by the merged
// tile jump S -> A^J S + inc*G_J (J = grid stride - 1), the second by the
// plain step S -> A S + inc.  The prologue parks each state at the "virtual"
// position one jump before the lane's first element (the affine jump is
// invertible: A^J is odd), so every tile, the first included, runs the same
// straight-line code.
//
// Loop order inside a tile is stream-outer: streams are taken in groups of
// two (Sched: two streams whose accumulators are disjoint, drawn by one
// interleaved asm block from sa_draw2.h) and the lane draws both of its
// elements for a group back to back, so a group's constants (inc, inc*G_J,
// sign mask) serve two draws per stream.  They are scalar-loaded from the
// kernarg segment into SGPRs, group g+1's loads issued after group g's first
// draw (latency hidden under one draw; SMEM returns out of order, so the
// wait is lgkmcnt(0) right before g+1 starts).  No VGPRs or LDS traffic go
// to constants; the multiplier limbs (A, A^J) sit in 8 wave-uniform VGPRs.
// Measured on the draw alone (tools/microbench/draw_issue.hip): LDS-resident
// constants issue 10-15 % slower than SGPR ones.
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
#include <stddef.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "../../include/sfl_sa.h"
#include "pcg128.h"
#include "sa_draw2.h"
#include "sa_internal.h"
#include "sa_philox.h"

namespace sa {

// Tuning-only ablations (results are WRONG when nonzero; never shipped):
// 1 = no zero-draw check, 2 = no quantize conversion, 8 = no global
// loads/stores, 32 = no digests, 64 = no prologue jump, 128 = stream 0's
// constants for every stream (no per-stream scalar loads).
#ifndef SA_ABLATE
#define SA_ABLATE 0
#endif

// Tuning-only wave timeline (make VARIANT=_ts EXTRA=-DSA_TIMING; results stay
// correct): lane 0 of every wave records s_memrealtime (100 MHz) at entry,
// after the prologue, after its first tile and after its last tile, the end,
// its tile count and HW_ID / XCC_ID, read back by sa_debug_timeline
// (sa_clients_f32.hip, tools/wave_timeline.py).
// Issue-priority rotation (see the tile loop): windows of 2^SA_PRIO ticks of
// the 100 MHz clock (14: 164 us); 0 = off.
#ifndef SA_PRIO
#define SA_PRIO 14
#endif

#ifdef SA_TIMING
constexpr int kTsWaves = 16384, kTsWords = 8;
static __device__ uint64_t g_sa_ts[kTsWaves][kTsWords];
#define SA_TS(v) (v) = __builtin_amdgcn_s_memrealtime()
#else
#define SA_TS(v) (void)0
#endif

constexpr int kE = 2;                       // elements per lane per tile
constexpr int kTile = kBlockThreads * kE;   // elements per workgroup tile (512)

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

// kLaneJump[t] = jump by t*kE + 1 draws: from a block tile's base state to the
// state lane t draws its first element from.  With the uniform block part
// (bits of blockIdx * kTile, scalar-loaded from kPowTable) the prologue
// costs one coalesced table load per lane instead of a divergent chain of
// ~27 dependent table loads.
struct LaneTable {
  Jump e[kBlockThreads];
};
constexpr LaneTable make_lane_table() {
  LaneTable t{};
  for (int l = 0; l < kBlockThreads; l++) t.e[l] = jump_of((uint64_t)l * kE + 1);
  return t;
}
static __constant__ LaneTable kLaneJump = make_lane_table();
static_assert((kTile & (kTile - 1)) == 0, "kTile is a power of two");
constexpr int kTileLog2 = __builtin_ctz(kTile);
constexpr int kGridBits = 12;  // grids are < 2^12 blocks (launch_clients checks)

// ----------------------------------------------------------------------------
// element loads / quantize
// ----------------------------------------------------------------------------
// Raw buffer descriptors (SGPR, built from kernel arguments only, so hipcc
// can prove them wave-uniform) + a 32-bit per-lane byte offset: one shared
// offset VGPR serves every client instead of a 64-bit address per client.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint64_t bytes) {
  // launches are chunked so that every vector's bytes fit (kChunkElems)
  const int nrec = bytes > 0xFFFFFFF0ull ? (int)0xFFFFFFF0u : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, nrec, 0x00020000);
}

// Tails without branches: gfx950 bounds-checks raw buffer accesses per
// dword against the descriptor's num_records (tools/microbench/oob_test.hip:
// a straddling dwordx4 load returns the in-range dwords and zeros, a
// straddling store writes only the in-range dwords).  Descriptors carry the
// exact byte length of their vector (0 for an absent one), so every tile
// issues the same unconditional loads and stores — no per-lane tail paths,
// whose merged control flow made the compiler wait (vmcnt(0)) for the
// tile's loads before the mask expansion.
template <typename T>
struct Vec2 {
  T v[2];
};
// elements i, i+1 of a T vector (past the end: 0); i even, so the pair is one
// 8-B (fp32) or 16-B (8-B types) aligned load
template <typename T>
__device__ __forceinline__ Vec2<T> bload2(rsrc_t r, uint64_t i) {
  Vec2<T> out;
  const int off = (int)(i * sizeof(T));
  if constexpr (sizeof(T) == 4) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    out.v[0] = __builtin_bit_cast(T, (uint32_t)u[0]);
    out.v[1] = __builtin_bit_cast(T, (uint32_t)u[1]);
  } else {
    const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    out.v[0] = __builtin_bit_cast(T, (uint64_t)u[0] | ((uint64_t)u[1] << 32));
    out.v[1] = __builtin_bit_cast(T, (uint64_t)u[2] | ((uint64_t)u[3] << 32));
  }
  return out;
}
// u64 elements i, i+1 (the part past the end is dropped by the bounds check)
__device__ __forceinline__ void bstore2_u64(rsrc_t r, uint64_t i, uint64_t v0, uint64_t v1) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u d = {(uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)(i * 8), 0, 0);
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
struct QScale {
  float f;     // 2^fxp
  double d;    // 2^fxp
  int32_t fxp;
};
template <typename XT, typename CT>
__device__ __forceinline__ uint64_t quantize(XT x, CT w, const QScale& q) {
  if constexpr (std::is_integral<CT>::value) {  // int64 arithmetic, wraps mod 2^64
    return (uint64_t)(long long)x * (uint64_t)w * ((uint64_t)1 << q.fxp);
  } else if constexpr (sizeof(CT) == 4) {
    // (x*w)*2^fxp == x*(w*2^fxp) exactly whenever w*2^fxp is finite: scaling
    // by a power of two commutes with rounding, and where the product is
    // subnormal it truncates to 0 either way.  Values of |p| < 2^31 (every
    // gradient in practice) convert with one v_cvt_i32_f32; a wave with any
    // larger / non-finite value takes the full int64 conversion.
    const float ws = __fmul_rn((float)w, q.f);  // wave-uniform
    if (__builtin_isfinite(ws)) {
      const float p = __fmul_rn((float)x, ws);
      if (!__any(!(__builtin_fabsf(p) < 0x1p31f))) return (uint64_t)(int64_t)(int32_t)p;
      return trunc_i64(p);
    }
    const float p = __fmul_rn((float)x, (float)w);
    return trunc_i64(__fmul_rn(p, q.f));
  } else {
    const double p = __dmul_rn((double)x, (double)w);
    return trunc_i64(__dmul_rn(p, q.d));
  }
}

template <typename CT>
__device__ __forceinline__ CT scalar_weight(double w) {
  if constexpr (std::is_integral<CT>::value)
    return (CT)(long long)w;
  else
    return (CT)w;
}

// The tile's products p = x * (w * 2^fxp) for the fp32 fast path, and
// whether it applies: every product of the wave below 2^31 (one v_cmp each,
// ANDed into one wave vote per tile), so each converts with one
// v_cvt_i32_f32.  Otherwise the tile takes the exact x86-semantics int64
// path (NaN / inf / huge values) of quantize().
// (x*w)*2^fxp == x*(w*2^fxp) whenever w*2^fxp is finite (a power-of-two
// scale commutes with rounding; subnormal products truncate to 0 either way);
// a non-finite w*2^fxp yields a non-finite p, i.e. the exact path.
template <typename XT, typename CT, int L, bool kGeneral>
__device__ __forceinline__ bool fast_products(const Vec2<XT> (&xv)[L], const Vec2<CT> (&wv)[kGeneral ? L : 1],
                                              const __attribute__((address_space(4))) KArgs* ka,
                                              const QScale& qs, float (&p)[L][kE]) {
  if constexpr (std::is_same<CT, float>::value) {
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int c = 0; c < L; c++) {
      const bool has_wv = kGeneral && ka->c[c].wvec;
      if (has_wv) {
#pragma unroll
        for (int k = 0; k < kE; k++)
          p[c][k] = __fmul_rn((float)xv[c].v[k], __fmul_rn((float)wv[kGeneral ? c : 0].v[k], qs.f));
      } else {
        // scalar weight: the host rounded w * 2^fxp once (ClientArg::ws);
        // both elements in one packed multiply (v_pk_mul_f32, per-lane RN)
        const f2 w2 = {ka->c[c].ws[0], ka->c[c].ws[1]};
        const f2 x2 = {(float)xv[c].v[0], (float)xv[c].v[1]};
        const f2 p2 = x2 * w2;
        p[c][0] = p2[0];
        p[c][1] = p2[1];
      }
    }
    // The vote: the largest |p| of the lane through gfx950's NaN-propagating
    // v_maximum3_f32 (IEEE 754-2019 maximum: a NaN operand yields NaN, which
    // then fails the < 2^31 test like an infinity), one instruction per two
    // products instead of one compare each.
    const float* q = &p[0][0];
    constexpr int kN = L * kE;
    float mx;
    asm("v_maximum3_f32 %0, |%1|, |%2|, |%3|" : "=v"(mx) : "v"(q[0]), "v"(q[1 % kN]), "v"(q[2 % kN]));
#pragma unroll
    for (int i = 3; i < kN; i += 2)
      asm("v_maximum3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(q[i]), "v"(q[i + 1 < kN ? i + 1 : i]));
    const bool ok = mx < 0x1p31f;
    return !__any(!ok) || (SA_ABLATE & 2);
  } else {
    return false;
  }
}
template <typename XT, typename CT, int L, bool kGeneral>
__device__ __forceinline__ uint64_t exact_q(const Vec2<XT> (&xv)[L], const Vec2<CT> (&wv)[kGeneral ? L : 1],
                                            const __attribute__((address_space(4))) KArgs* ka, const QScale& qs,
                                            int c, int k) {
  const bool has_wv = kGeneral && ka->c[c].wvec;
  const CT w = has_wv ? wv[kGeneral ? c : 0].v[k] : scalar_weight<CT>(ka->c[c].w);
  return quantize<XT, CT>(xv[c].v[k], w, qs);
}

// ----------------------------------------------------------------------------
// PCG64 draw
// ----------------------------------------------------------------------------
__device__ __forceinline__ u128 ld128(uint64_t lo, uint64_t hi) { return mk128(hi, lo); }
// a wave-uniform value as an opaque VGPR (kept resident, never re-materialised)
__device__ __forceinline__ uint32_t vreg(uint32_t x) {
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
  return r;
}

// One PCG64 step + signed XSL-RR draw + accumulation, hand-scheduled for
// gfx950 (the whole inner loop of the kernel is this block, P times per element).
//
//   S' = S*A + C (mod 2^128) from 32-bit limbs: three 64-bit column chains
//   (limbs 0-1: s0a0 + c0; limbs 1-2: s0a1 + c1 + s1a0; limbs 2-3: s0a2 +
//   s1a1 + s2a0 + C23) on v_mad_u64_u32 -- the increment's two low words enter
//   as separate zero-extended addends so the first two mads cannot carry --
//   the four limb-3 products summed by one v_mul_lo_u32 and three
//   v_mad_u64_u32 (only the low word is kept), joined by carry adds whose
//   carry-ins are the mads' own carry-outs -- 9 mads + 1 mul_lo + 4 adds +
//   1 mov (the paired draws of sa_draw2.h, which do nearly all the work,
//   keep limbs 0-1 in one VGPR pair written in place and need no mov).
//   Then x = hi^lo^m (two v_bitop3) and t = rotr(x, hi>>58) as two 64-bit
//   shifts whose disjoint parts one v_lshl_add_u64 adds: y = x >> r,
//   z = x << (63 - r), t = (z << 1) + y (r = 0: z << 1 vanishes, t = x); the
//   raw==0 test (hi == lo <=> x == m:m) as one 64-bit compare whose lane
//   mask the SALU ORs into `zs` (a per-tile SGPR pair), and the accumulation
//   (below).  The same form as sa_draw2.h's paired draws (tools/gen_draw2.py).
//
// Carries live in three SGPR pairs, reused as they die (k1: a discarded
// carry-out; k2: kO, c2, then the acc_v borrow; k3: discarded carry-outs, c1).
// Every VALU-written SGPR (carries, VCC) is read >= 2 instructions later
// (gfx950 VALU-SGPR-write -> VALU-read hazard).  v0-v9 are fixed scratch (low
// registers, so the kernel's VGPR budget is not raised).  Single draws only
// serve schedules with an odd leftover stream.
#define SA_PCG_DRAW_ASM                                                                  \
  "v_mad_u64_u32 v[0:1], %[k1], %[s0], %[a0], %[c0]\n\t"    /* E0 = s0a0 + c0 < 2^64 */  \
  "v_mad_u64_u32 v[2:3], %[k3], %[s0], %[a1], %[c1]\n\t"    /* O1 = s0a1 + c1 < 2^64 */  \
  "v_mad_u64_u32 v[4:5], %[k3], %[s0], %[a2], %[c23]\n\t"   /* E2 = s0a2 + C23 */       \
  "v_mul_lo_u32 v6, %[s0], %[a3]\n\t"                       /* L3 = p03 */               \
  "v_mad_u64_u32 v[2:3], %[k2], %[s1], %[a0], v[2:3]\n\t"   /* O1 += s1a0, kO */        \
  "v_mad_u64_u32 v[4:5], %[k3], %[s1], %[a1], v[4:5]\n\t"                                \
  "v_mad_u64_u32 v[6:7], %[k3], %[s1], %[a2], v[6:7]\n\t"   /* L3 += p12 (low word) */  \
  "v_mad_u64_u32 v[4:5], %[k3], %[s2], %[a0], v[4:5]\n\t"                                \
  "v_mad_u64_u32 v[6:7], %[k3], %[s2], %[a1], v[6:7]\n\t"   /* L3 += p21 */             \
  "v_mad_u64_u32 v[6:7], %[k3], %[s3], %[a0], v[6:7]\n\t"   /* L3 += p30 */             \
  "v_add_co_u32_e64 %[s1], %[k3], v1, v2\n\t"              /* r1 = e1 + o1, c1 */       \
  "v_addc_co_u32_e64 %[s3], %[k2], v5, v6, %[k2]\n\t"      /* r3 = e3 + L3 + kO */      \
  "v_mov_b32_e32 %[s0], v0\n\t"                             /* r0 = e0 */                \
  "v_addc_co_u32_e64 %[s2], %[k2], v4, v3, %[k3]\n\t"      /* r2 = e2 + o2 + c1, c2 */  \
  "v_bitop3_b32 v0, %[s0], %[s2], %[m] bitop3:0x96\n\t"    /* xl */                     \
  "s_nop 0\n\t"                                                                          \
  "v_addc_co_u32_e64 %[s3], %[k3], %[s3], 0, %[k2]\n\t"    /* r3 += c2 */               \
  "v_bitop3_b32 v1, %[s1], %[s3], %[m] bitop3:0x96\n\t"    /* xh */                     \
  "v_lshrrev_b32_e32 v2, 26, %[s3]\n\t"                     /* r */                      \
  "v_xor_b32_e32 v3, 63, v2\n\t"                            /* 63 - r */                 \
  "v_cmp_eq_u64_e32 vcc, %[mm], v[0:1]\n\t"                 /* raw == 0 */               \
  "v_lshrrev_b64 v[4:5], v2, v[0:1]\n\t"                    /* y */                      \
  "v_lshlrev_b64 v[6:7], v3, v[0:1]\n\t"                    /* z */                      \
  "s_or_b64 %[zs], %[zs], vcc\n\t"                                                       \
  "v_lshl_add_u64 v[6:7], v[6:7], 1, v[4:5]\n\t"           /* t */

#define SA_PCG_DRAW_OUTS                                                                 \
  [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3), [zs] "+s"(zs),              \
      [u] "+v"(u), [k1] "=&s"(k1), [k2] "=&s"(k2), [k3] "=&s"(k3)
// Operand classes: the multiplier limbs are wave-uniform VGPRs (set once per
// launch), the stream constants SGPRs (scalar-loaded per stream and tile), so
// every VOP3 reads at most one SGPR (the gfx9 constant-bus limit).
#define SA_PCG_DRAW_INS                                                                  \
  [a0] "v"(a0), [a1] "v"(a1), [a2] "v"(a2), [a3] "v"(a3), [c0] "s"(inc.w0),                    \
      [c1] "s"(inc.w1), [c23] "s"(inc.hi), [m] "s"(m), [mm] "s"((uint64_t)m << 32 | m)
#define SA_PCG_DRAW_CLOBBERS \
  "vcc", "scc", "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9"

// acc_u += t with one v_lshl_add_u64 on the 64-bit accumulator (the issue cost
// of one v_add_co, tools/microbench/op_rate.hip); the internal pair's second
// client subtracts on 32-bit halves (pcg_draw_pair) or, when the kernel keeps
// that client negated, also adds (pcg_draw_pair_a).  zs: the per-tile lane
// mask of raw == 0 draws (an SGPR pair; 0 at the tile's start).
__device__ __forceinline__ void pcg_draw_pair(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3, uint32_t a0,
                                              uint32_t a1, uint32_t a2, uint32_t a3, const Inc& inc,
                                              uint32_t m, uint64_t& zs, uint64_t& u, uint64_t& v) {
  uint64_t k1, k2, k3;
  uint32_t vlo = (uint32_t)v, vhi = (uint32_t)(v >> 32);
  asm volatile(SA_PCG_DRAW_ASM
               "v_sub_co_u32_e64 %[vlo], %[k2], %[vlo], v6\n\t"
               "v_lshl_add_u64 %[u], v[6:7], 0, %[u]\n\t"
               "s_nop 0\n\t"
               "v_subb_co_u32_e64 %[vhi], %[k2], %[vhi], v7, %[k2]"
               : SA_PCG_DRAW_OUTS, [vlo] "+v"(vlo), [vhi] "+v"(vhi)
               : SA_PCG_DRAW_INS
               : SA_PCG_DRAW_CLOBBERS);
  v = ((uint64_t)vhi << 32) | vlo;
}
__device__ __forceinline__ void pcg_draw_pair_a(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3, uint32_t a0,
                                                uint32_t a1, uint32_t a2, uint32_t a3, const Inc& inc,
                                                uint32_t m, uint64_t& zs, uint64_t& u, uint64_t& v) {
  uint64_t k1, k2, k3;
  asm volatile(SA_PCG_DRAW_ASM
               "v_lshl_add_u64 %[u], v[6:7], 0, %[u]\n\t"
               "v_lshl_add_u64 %[v], v[6:7], 0, %[v]"
               : SA_PCG_DRAW_OUTS, [v] "+v"(v)
               : SA_PCG_DRAW_INS
               : SA_PCG_DRAW_CLOBBERS);
}
__device__ __forceinline__ void pcg_draw_one(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3, uint32_t a0,
                                             uint32_t a1, uint32_t a2, uint32_t a3, const Inc& inc,
                                             uint32_t m, uint64_t& zs, uint64_t& u) {
  uint64_t k1, k2, k3;
  asm volatile(SA_PCG_DRAW_ASM
               "v_lshl_add_u64 %[u], v[6:7], 0, %[u]"
               : SA_PCG_DRAW_OUTS
               : SA_PCG_DRAW_INS
               : SA_PCG_DRAW_CLOBBERS);
}

// Compile-time enumeration of the pairs (u < v) a launch's L local clients
// share.  K = kAllPairs: every internal pair of the L clients.  K =
// kBipartite: only the pairs between the lower and the upper half (a, b),
// a < L/2 <= b, a-major -- one block of the pair-shared schedule for more
// co-located clients than one launch holds (kernels.fused_many: the quads
// of clients pairwise, each pair stream still expanded exactly once).
template <int L, int K = kAllPairs>
struct Pairs {
  static constexpr int H = L / 2;
  static constexpr bool kBip = (K & kBipartite) != 0;
  static constexpr int count = kBip ? H * (L - H) : L * (L - 1) / 2;
  static constexpr int u(int p) {
    if (kBip) return p / (L - H);
    int k = p;
    for (int a = 0; a < L; a++) {
      const int row = L - 1 - a;
      if (k < row) return a;
      k -= row;
    }
    return -1;
  }
  static constexpr int v(int p) {
    if (kBip) return H + p % (L - H);
    int k = p;
    for (int a = 0; a < L; a++) {
      const int row = L - 1 - a;
      if (k < row) return a + 1 + k;
      k -= row;
    }
    return -1;
  }
};


// Clients whose accumulator holds the NEGATED running value (st = -acc): the
// upper half.  An internal pair (u, v) adds t to u and subtracts it from v;
// with u in the lower and v in the upper half both become adds (one
// v_lshl_add_u64 each instead of an add and a two-instruction subtract) --
// 16 of the 28 pairs of 8 clients.  A negated client's cross streams draw
// ~t = -t - 1 (sign mask inverted) and add; its accumulator starts at
// X - bias; the finish forms q - st.
template <int L>
constexpr bool negated(int c) {
  return L >= 2 && c >= L / 2;
}

// Draw schedule of a launch: the P streams grouped into interleaved pairs
// (sa_draw2.h) wherever two streams touch disjoint accumulators (or, for
// two cross streams of one client, one shared accumulator), singles
// otherwise.  Internal pairs of L clients are matched greedily
// (for L = 8: 14 disjoint pairs of pairs), cross streams by client.
//
// Groups are then ORDERED so that every client is first touched by a draw
// that ADDS to it (as the adding client u, or as a partner kept negated):
// such a first touch writes the accumulator from the client's bias constant
// (an SGPR pair) instead of reading it, so the tile presets no accumulator
// with v_movs (sa_draw2.h, first-touch variants F).  A client first touched
// as a subtracting partner or by a single draw (or never, P = 0) is preset
// instead (`preset`); for every instantiated shape that set is empty or
// holds only single-draw clients.
struct Group {
  int qa, qb;          // streams (qb < 0: single draw)
  int ua, va, ub, vb;  // accumulators: u adds t; v < 0: a cross stream (no partner)
  bool va_add, vb_add;  // the partner adds t (it is stored negated) instead of subtracting
  bool fa, fb;          // cross stream of a negated client: inverted sign mask
  int F;                // first-touch bits: 1 ua, 2 va, 4 ub, 8 vb (sa_draw2.h template argument)
};
template <int L, int X, int K = kAllPairs>
struct Sched {
  static constexpr int PI = Pairs<L, K>::count;
  static constexpr int P = PI + L * X;
  int n = 0;
  Group g[P > 0 ? P : 1] = {};
  uint32_t preset = 0;  // clients whose accumulators the tile presets to the bias
  struct Role {
    int u, v;  // add target, partner (-1: none)
    bool v_add, flip;
  };
  static constexpr Role role(int q) {
    if (q >= PI) {
      const int c = (q - PI) / (X > 0 ? X : 1);
      return Role{c, -1, false, negated<L>(c)};
    }
    const int u = Pairs<L, K>::u(q), v = Pairs<L, K>::v(q);
    if (!negated<L>(v)) return Role{u, v, false, false};  // both plain: u += t, v -= t
    if (!negated<L>(u)) return Role{u, v, true, false};   // v negated: both add
    return Role{v, u, false, false};                      // both negated: -u -= t, -v += t
  }
  constexpr Sched() {
    bool used[P > 0 ? P : 1] = {};
    Group tmp[P > 0 ? P : 1] = {};
    int m = 0;
    for (int q = 0; q < P; q++) {
      if (used[q]) continue;
      used[q] = true;
      const Role a = role(q);
      int mate = -1;
      for (int r = q + 1; r < P && mate < 0; r++) {
        if (used[r] || (q < PI) != (r < PI)) continue;
        const Role b = role(r);
        const bool disjoint = a.u != b.u && a.u != b.v && (a.v < 0 || (a.v != b.u && a.v != b.v));
        const bool same_one = q >= PI && a.u == b.u;  // two cross streams of one client
        if (disjoint || same_one) mate = r;
      }
      if (mate >= 0) used[mate] = true;
      const Role b = mate >= 0 ? role(mate) : Role{-1, -1, false, false};
      tmp[m++] = Group{q, mate, a.u, a.v, b.u, b.v, a.v_add, b.v_add, a.flip, b.flip, 0};
    }
    // order: repeatedly take the first remaining pair-group none of whose
    // subtracting partners is untouched yet; singles last among the candidates
    bool taken[P > 0 ? P : 1] = {};
    bool seen[kMaxLocal] = {};
    for (int k = 0; k < m; k++) {
      int pick = -1;
      for (int pass = 0; pass < 3 && pick < 0; pass++) {
        for (int i = 0; i < m && pick < 0; i++) {
          if (taken[i]) continue;
          const Group& G = tmp[i];
          const bool single = G.qb < 0;
          const bool sub_a = G.va >= 0 && !G.va_add && !seen[G.va];
          const bool sub_b = G.vb >= 0 && !G.vb_add && !seen[G.vb];
          if (pass == 0 && !single && !sub_a && !sub_b) pick = i;
          if (pass == 1 && !sub_a && !sub_b) pick = i;
          if (pass == 2) pick = i;
        }
      }
      taken[pick] = true;
      Group G = tmp[pick];
      int F = 0;
      const bool single = G.qb < 0;
      // first touch of each accumulator of this group (u before v, a before b)
      auto touch = [&](int c, bool adds, int bit) {
        if (c < 0 || seen[c]) return;
        seen[c] = true;
        if (adds && !single) F |= bit;
        else preset |= 1u << c;
      };
      touch(G.ua, true, 1);
      touch(G.va, G.va_add, 2);
      touch(G.ub, true, 4);
      if (G.ub != G.ua) touch(G.vb, G.vb_add, 8);
      G.F = F;
      g[n++] = G;
    }
    for (int c = 0; c < L; c++)
      if (!seen[c]) preset |= 1u << c;
  }
};

template <int L, int X, int K = kAllPairs>
struct SchedOf {
  static constexpr Sched<L, X, K> value{};
};

// f(std::integral_constant<int, 0>{}), ..., f(std::integral_constant<int, N-1>{}):
// a compile-time loop whose index is a constant expression in the body
template <typename Fn, int... I>
__device__ __forceinline__ void for_each_index(Fn&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

// ----------------------------------------------------------------------------
// the kernel
// ----------------------------------------------------------------------------

// Waves per SIMD the register allocation must allow (spill-free targets from
// the compiler's census, tools/kregs.py): 4 VGPRs per stream state, 4 per
// (client, element) (accumulator halves, input, product), 2 per client
// (digest), plus the draw scratch, multipliers and addressing; the
// single-client kernel also carries the continue / per-element-weight /
// DP-noise paths.  L = 8 (28 pair streams): 2 waves; 1 client + 7 cross
// streams: 5.
constexpr int clients_waves(int P, int L) {
  const int regs = 4 * P + 4 * L * kE + 2 * L + (L == 1 ? 64 : 56);
  const int w = 512 / regs;
  return w > 8 ? 8 : (w < 1 ? 1 : w);
}

typedef __attribute__((address_space(4))) const uint64_t* kptr_t;
static_assert(offsetof(StreamArg, inc_hi) == 24 && offsetof(StreamArg, cj_hi) == 40 &&
                  offsetof(StreamArg, smask) == 48 && offsetof(StreamArg, inc_w0) == 64 &&
                  offsetof(StreamArg, cj_w0) == 80,
              "StreamArg layout (scalar loads below)");

typedef __attribute__((address_space(4))) const KArgs kargs_t;

// The kernarg image through an opaque SGPR pointer: loads through it are
// scalar loads that cannot be hoisted above the fence, so per-client values
// (buffer bases, bias, weight) are re-read where they are used instead of
// pinning ~100 SGPRs (descriptors, biases, weights of 8 clients) across the
// whole tile loop.
__device__ __forceinline__ kargs_t* fenced_args() {
  kargs_t* p = (kargs_t*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

template <typename XT, typename CT, int L, int X, int K = kAllPairs>
__global__ void __launch_bounds__(kBlockThreads, clients_waves(Pairs<L, K>::count + L * X, L))
    k_clients(const KArgs a) {
  constexpr int PI = Pairs<L, K>::count;
  constexpr int P = PI + L * X;
  // the single-client kernel's general paths: continue mode + per-element
  // weights + DP (kLean1: the same single client without them)
  constexpr bool kGeneral = (L == 1) && !(K & kLean1);
  // only the masked sum leaves the launch (no digests, no wire images): the
  // finish and epilogue carry no digest / store code at all
  constexpr bool kSum = (K & (kSumOnly | kBipartite | kCrossOnly)) != 0;
  // cross streams only, masks only: one accumulator, nothing loaded
  constexpr bool kCross = (K & kCrossOnly) != 0;
  static_assert(!kCross || (L == 1 && !kGeneral), "kCrossOnly: one lean accumulator");
  static_assert(L >= 1 && L <= kMaxLocal, "L");
  static_assert(P <= kMaxStreams, "P");

  const uint64_t n = a.n;
  const uint64_t stride = (uint64_t)gridDim.x * kTile;
#ifdef SA_TIMING
  uint64_t ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, ts4 = 0;
  uint32_t tiles = 0;
#endif
  SA_TS(ts0);

  // ---- prologue: park every stream one tile jump before S_{first+1}, the
  // state element `first` is drawn from: V = A^-J (S_{first+1} - inc*G_J)
  // 128-bit states: limbs 0-1 as one 64-bit VGPR pair (the draw's first
  // mad writes it in place, sa_draw2.h), limbs 2 and 3 as 32-bit VGPRs
  struct State {
    uint64_t p01;
    uint32_t s2, s3;
  };
  State st[P > 0 ? P : 1];
  if constexpr (P > 0) {
    // J(first + 1) = J(blockIdx * kTile) o J(lane * kE + 1)
    // Block part: a fixed, fully unrolled bit loop (grids stay below 2^12
    // blocks: 8 waves/SIMD x 256 CUs / 4 waves per block = 512... 2048), so
    // the table loads are issued together instead of one dependent scalar
    // load per set bit.
    static_assert(kTileLog2 + kGridBits <= 64, "power table");
    Jump jb{1, 0};
    const uint32_t bid = (SA_ABLATE & 64) ? 0u : blockIdx.x;
#pragma unroll
    for (int b = 0; b < kGridBits; b++) {  // wave-uniform
      const Jump e = kPowTable.e[kTileLog2 + b];
      if ((bid >> b) & 1) jb = compose(jb, e);
    }
    const Jump jl = compose(kLaneJump.e[threadIdx.x], jb);
    const u128 aji = ld128(a.aji_lo, a.aji_hi);
#pragma unroll
    for (int j = 0; j < P; j++) {
      const StreamArg& s = a.s[j];
      const u128 sf = apply(jl, ld128(s.s_lo, s.s_hi), ld128(s.inc_lo, s.inc_hi));
      const u128 v = aji * (sf - ld128(s.cj_lo, s.cj_hi));
      st[j].p01 = lo64(v);
      st[j].s2 = (uint32_t)hi64(v);
      st[j].s3 = (uint32_t)(hi64(v) >> 32);
    }
  }
  // multiplier limbs: jump (first element of a tile) and plain step
  uint32_t mj[4], mp[4];
  if constexpr (P > 0) {
    const u128 AJ = ld128(a.aj_lo, a.aj_hi);
#pragma unroll
    for (int w = 0; w < 4; w++) {
      mj[w] = vreg((uint32_t)(AJ >> (32 * w)));
      mp[w] = vreg((uint32_t)(kPcgMult >> (32 * w)));
    }
  }

  // 0 iff some raw PCG64 draw of this lane (or, for the paired draws, of its
  // wave) was 0; the paired draws test per tile (sa_draw2.h, ZeroAcc)
  uint32_t zmin = 0xFFFFFFFFu;
  SA_TS(ts1);

  // per-lane XOR digests of the clients' masked values: VGPRs, or for the
  // register-bound shapes (5+ co-located clients) lane-private LDS slots
  // updated with one ds_xor_b64 per client and tile
  constexpr bool kDigLds = L >= 5;
  uint64_t dig[kDigLds ? 1 : L];
  __shared__ uint64_t dig_lds[kDigLds ? L : 1][kBlockThreads];
#pragma unroll
  for (int c = 0; c < L; c++) {
    if constexpr (kDigLds)
      dig_lds[c][threadIdx.x] = 0;
    else
      dig[c] = 0;
  }

  float dp_s = 1.0f;
  if constexpr (kGeneral && std::is_same<XT, float>::value && std::is_same<CT, float>::value) {
    if (a.dp_on) dp_s = dp_scale(a.dp_sumsq, a.dp_sumsq_layer, a.dp_clip);
  }

  // wave-uniform trip count: every lane of a wave runs the wave's last tile
  // (out-of-range elements are masked at load/store)
  const uint64_t wave_off = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * 64 * kE);
  // Two waves share a SIMD and its VALU issue is arbitrated by priority, then
  // age: at equal priority the older wave runs ~1.6x faster, ends ~40% early
  // and the younger then runs the rest alone, which issues fewer VALU per
  // cycle than two waves do (tools/wave_timeline.py: per-wave tile time
  // 5.2 vs 8.7 us, the last waves end at 1.7x the first).  Rotating priority
  // 1 between the wave slots in fixed clock windows makes the pair progress
  // equally and end together: 8 clients x 100M, 2.77 -> 2.49 ms.
#if SA_PRIO
  uint32_t slot;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 1)" : "=s"(slot));
#endif
  for (uint64_t base = (uint64_t)blockIdx.x * kTile; base + wave_off < n; base += stride) {
    const uint64_t i = base + (uint64_t)threadIdx.x * kE;
#if SA_PRIO
    if ((((uint32_t)__builtin_amdgcn_s_memrealtime() >> SA_PRIO) ^ slot) & 1)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
#endif

    // ---- issue this tile's loads first; consumed after the mask expansion.
    // Unconditional: an absent vector has a 0-byte descriptor (reads 0).
    Vec2<XT> xv[L];
    Vec2<CT> wv[kGeneral ? L : 1];
    Vec2<uint64_t> pv[kGeneral ? L : 1];
    uint64_t acc[kE][L];  // per-client accumulators (negated<L> clients: -acc)
    {
      kargs_t* ka = fenced_args();
      const bool cont = kGeneral && ka->continue_mode;
#pragma unroll
      for (int c = 0; c < L; c++) {
        if (SA_ABLATE & 8) {
#pragma unroll
          for (int k = 0; k < kE; k++) xv[c].v[k] = (XT)(int)(i + k + c);
        } else if constexpr ((K & (kBipartite | kCrossOnly)) != 0) {  // masks only: the values enter elsewhere
          xv[c].v[0] = xv[c].v[1] = (XT)0;
        } else {
          xv[c] = bload2<XT>(make_rsrc(ka->c[c].x, cont ? 0 : n * sizeof(XT)), i);
        }
        if constexpr (kGeneral) {
          const void* wp = ka->c[c].wvec;
          wv[c] = bload2<CT>(make_rsrc(wp, (wp && !cont) ? n * sizeof(CT) : 0), i);
          pv[c] = bload2<uint64_t>(make_rsrc(ka->c[c].masked_out, cont ? n * 8 : 0), i);
        }
        // accumulators start at the client's folded bias constant (negated
        // clients: X - bias, see negated<L>): written by the client's first
        // draw (first-touch variants), preset here only where the schedule
        // cannot (Sched::preset)
        if ((SchedOf<L, X, K>::value.preset >> c) & 1) {
          const uint64_t bias = negated<L>(c) ? (uint64_t)X - ka->c[c].bias : ka->c[c].bias;
#pragma unroll
          for (int k = 0; k < kE; k++) acc[k][c] = bias;
        }
      }
    }

    // ---- mask expansion, stream-outer, two streams per asm block where the
    // schedule pairs them; group g+1's constants are scalar-loaded during
    // group g's first draw
    // the raw == 0 tests, one lane mask per element slot k of the lane so
    // that a draw for an element past n (the wave's last tile draws for
    // every lane) is not counted: numpy draws exactly n
    ZeroAcc zh[kE];   // the paired draws' (sa_draw2.h)
    uint64_t zs[kE];  // the single draws' (SA_PCG_DRAW_ASM)
#pragma unroll
    for (int k = 0; k < kE; k++) {
      zh[k] = zero_acc_init();
      zs[k] = 0;
    }
    if constexpr (P > 0) {
      using SO = SchedOf<L, X, K>;  // the schedule (a static constexpr: usable in the lambdas)
      Inc ni[2], nj[2];  // next group's plain-step / tile-jump addends
      uint32_t nm[2];
      auto fetch = [&](int g) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const int q = h == 0 ? SO::value.g[g].qa : SO::value.g[g].qb;
          if (q < 0) continue;
          kptr_t c = (const kptr_t)(&fenced_args()->s[q]);
          ni[h] = Inc{c[8], c[9], c[3]};
          nj[h] = Inc{c[10], c[11], c[5]};
          nm[h] = (uint32_t)c[6] ^ ((h == 0 ? SO::value.g[g].fa : SO::value.g[g].fb) ? 0xFFFFFFFFu : 0u);
        }
      };
      // a first-touched accumulator starts from its client's bias (SGPRs)
      auto bias_of = [&](int c) -> uint64_t {
        if (c < 0) return 0;
        kargs_t* ka = fenced_args();
        return negated<L>(c) ? (uint64_t)X - ka->c[c].bias : ka->c[c].bias;
      };
      fetch(0);
      for_each_index([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        constexpr Group G = SO::value.g[g];
        Inc ci[2], cj[2];
        uint32_t m[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          ci[h] = ni[h];
          cj[h] = nj[h];
          m[h] = nm[h];
        }
        const uint64_t bua = (G.F & 1) ? bias_of(G.ua) : 0, bva = (G.F & 2) ? bias_of(G.va) : 0;
        const uint64_t bub = (G.F & 4) ? bias_of(G.ub) : 0, bvb = (G.F & 8) ? bias_of(G.vb) : 0;
#pragma unroll
        for (int k = 0; k < kE; k++) {
          const uint32_t* mk = k == 0 ? mj : mp;
          const Inc& ia = k == 0 ? cj[0] : ci[0];
          const Inc& ib = k == 0 ? cj[1] : ci[1];
          State& sa = st[G.qa];
          uint64_t* ak = acc[k];
          if constexpr (G.qb < 0) {  // singles never first-touch: their clients are preset
            uint32_t s0 = (uint32_t)sa.p01, s1 = (uint32_t)(sa.p01 >> 32);
            if constexpr (G.va >= 0 && G.va_add)
              pcg_draw_pair_a(s0, s1, sa.s2, sa.s3, mk[0], mk[1], mk[2], mk[3], ia, m[0], zs[k], ak[G.ua], ak[G.va]);
            else if constexpr (G.va >= 0)
              pcg_draw_pair(s0, s1, sa.s2, sa.s3, mk[0], mk[1], mk[2], mk[3], ia, m[0], zs[k], ak[G.ua], ak[G.va]);
            else
              pcg_draw_one(s0, s1, sa.s2, sa.s3, mk[0], mk[1], mk[2], mk[3], ia, m[0], zs[k], ak[G.ua]);
            sa.p01 = ((uint64_t)s1 << 32) | s0;
          } else {
            State& sb = st[G.qb];
#define SA_DRAW2_PAIR(fn)                                                                                 \
  fn<G.F>(sa.p01, sa.s2, sa.s3, sb.p01, sb.s2, sb.s3, mk[0], mk[1], mk[2], mk[3], ia, m[0], ib, m[1], zh[k],\
          ak[G.ua], ak[G.va], ak[G.ub], ak[G.vb], bua, bva, bub, bvb)
            if constexpr (G.va >= 0 && G.va_add && G.vb_add)
              SA_DRAW2_PAIR(pcg_draw2_pair_aa);
            else if constexpr (G.va >= 0 && G.va_add)
              SA_DRAW2_PAIR(pcg_draw2_pair_as);
            else if constexpr (G.va >= 0 && G.vb_add)
              SA_DRAW2_PAIR(pcg_draw2_pair_sa);
            else if constexpr (G.va >= 0)
              SA_DRAW2_PAIR(pcg_draw2_pair_ss);
#undef SA_DRAW2_PAIR
            else if constexpr (G.ua == G.ub)
              pcg_draw2_one_same<G.F>(sa.p01, sa.s2, sa.s3, sb.p01, sb.s2, sb.s3, mk[0], mk[1], mk[2], mk[3], ia,
                                      m[0], ib, m[1], zh[k], ak[G.ua], bua);
            else
              pcg_draw2_one<G.F>(sa.p01, sa.s2, sa.s3, sb.p01, sb.s2, sb.s3, mk[0], mk[1], mk[2], mk[3], ia, m[0],
                                 ib, m[1], zh[k], ak[G.ua], ak[G.ub], bua, bub);
          }
          if (k == 0 && g + 1 < SO::value.n && !(SA_ABLATE & 128)) fetch(g + 1);
        }
      }, std::make_integer_sequence<int, SO::value.n>{});
    }

    {
      uint64_t z0 = (uint64_t)zh[0] | zs[0], z1 = (uint64_t)zh[1] | zs[1];
      static_assert(kE == 2, "one mask per element slot");
      static_assert(std::is_same<ZeroAcc, uint64_t>::value, "sa_draw2.h's lane-mask form of the zero test");
      if (__builtin_expect((z0 | z1) != 0, 0)) {
        if (base + wave_off + 64 * kE > n) {
          // the wave's last tile: lanes whose elements are >= n drew too.
          // Lane l holds elements e + 2l, e + 2l + 1 (e = base + wave_off), so
          // with r = n - e slot 0 is valid for l < ceil(r/2), slot 1 for
          // l < floor(r/2): scalar masks, no per-lane compare
          const uint64_t r = n - (base + wave_off);  // 1 .. 127 here
          const uint32_t r0 = (uint32_t)((r + 1) >> 1), r1 = (uint32_t)(r >> 1);
          z0 &= r0 >= 64 ? ~0ull : (1ull << r0) - 1;
          z1 &= (1ull << r1) - 1;
        }
        if (z0 | z1) zmin = 0;
      }
    }

    // ---- finish: add the quantized value (or the prior pass), digest, sums
    kargs_t* ka = fenced_args();
    const bool cont = kGeneral && ka->continue_mode;
    if constexpr (kGeneral && std::is_same<XT, float>::value && std::is_same<CT, float>::value) {
      if (ka->dp_on && !cont) {  // fused DP pre-step (sa_mask_dp)
        // the lane's two elements are Box-Muller pair (i & 2) / 2 of their
        // Philox block: only that pair is formed
        const Normal2 z = gauss2(ka->dp_key, ka->dp_block0 + (i >> 2), (int)((i >> 1) & 1));
        if (ka->dp_inv != 0.0f) {  // uniform branch: a power-of-two num_updates multiplies
#pragma unroll
          for (int k = 0; k < kE; k++)
            xv[0].v[k] = dp_apply_t<true>(xv[0].v[k], dp_s, z.z[k], ka->dp_sigma, ka->dp_updates, ka->dp_inv);
        } else {
#pragma unroll
          for (int k = 0; k < kE; k++)
            xv[0].v[k] = dp_apply_t<false>(xv[0].v[k], dp_s, z.z[k], ka->dp_sigma, ka->dp_updates, ka->dp_inv);
        }
      }
    }
    const QScale qs{ka->scale_f, ka->scale_d, ka->fxp_bits};
    // elements past n only occur in the wave's last tile (uniform test)
    const bool wave_full = base + wave_off + 64 * kE <= n;
    const uint32_t mmask = kSum ? 0u : ka->masked_mask;
    // per-client XOR digests only when the caller asked for them (a
    // checksum for tests and the wire path, not part of the reference's
    // arithmetic): one wave-uniform branch per tile
    const bool dig_on = kSum ? false : (bool)ka->do_digest;
    uint64_t sum[kE] = {0, 0};
    auto finish = [&](int c, uint64_t q0, uint64_t q1) {
      const uint64_t a0 = negated<L>(c) ? q0 - acc[0][c] : acc[0][c] + q0;
      const uint64_t a1 = negated<L>(c) ? q1 - acc[1][c] : acc[1][c] + q1;
      sum[0] += a0;
      sum[1] += a1;
      if (dig_on && !(SA_ABLATE & 32)) {
        const uint64_t d = wave_full ? a0 ^ a1 : (i < n ? a0 : 0) ^ (i + 1 < n ? a1 : 0);
        if constexpr (kDigLds)
          __hip_atomic_fetch_xor(&dig_lds[c][threadIdx.x], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
          dig[kDigLds ? 0 : c] ^= d;
      }
      if ((mmask >> c) & 1) bstore2_u64(make_rsrc(ka->c[c].masked_out, n * 8), i, a0, a1);
    };
    static_assert(kE == 2, "finish() takes the lane's two elements");
    float p[L][kE];
    if constexpr (kCross) {
      // masks only (sa_fused_clients' later launches): the one accumulator
#pragma unroll
      for (int k = 0; k < kE; k++) sum[k] = acc[k][0];
    } else if constexpr ((K & kBipartite) != 0) {
      // masks only (sa_fused_bipartite): the sum of the 8 accumulators, the
      // upper quad's stored negated
#pragma unroll
      for (int k = 0; k < kE; k++) {
        uint64_t A = acc[k][0], B = acc[k][L / 2];
#pragma unroll
        for (int c = 1; c < L / 2; c++) A += acc[k][c];
#pragma unroll
        for (int c = L / 2 + 1; c < L; c++) B += acc[k][c];
        sum[k] = A - B;
      }
    } else if (cont) {  // a further pass: add the prior pass's masked vector
#pragma unroll
      for (int c = 0; c < L; c++) finish(c, pv[kGeneral ? c : 0].v[0], pv[kGeneral ? c : 0].v[1]);
    } else if (__builtin_expect(fast_products<XT, CT, L, kGeneral>(xv, wv, ka, qs, p), 1)) {
      if (!dig_on && mmask == 0) {
        // Only the sum leaves the tile: sum = sum_plain (acc + q) +
        // sum_negated (q - st) = A - B with A = sum_plain acc + sum_plain q
        // and B = sum_negated st - sum_negated q; each int32 q enters
        // sign-extended through one v_mad_i64_i32 (q * (+-1) + A), instead
        // of a sign extension plus a 64-bit add per client (and a subtract
        // pair for negated clients).
#pragma unroll
        for (int k = 0; k < kE; k++) {
          uint64_t A = 0, B = 0;
          bool a0 = false, b0 = false;
#pragma unroll
          for (int c = 0; c < L; c++) {
            uint64_t& t = negated<L>(c) ? B : A;
            bool& t0 = negated<L>(c) ? b0 : a0;
            t = t0 ? t + acc[k][c] : acc[k][c];
            t0 = true;
          }
#pragma unroll
          for (int c = 0; c < L; c++) {
            const int32_t q = (int32_t)p[c][k];
            uint64_t kc;
            if (negated<L>(c))
              asm("v_mad_i64_i32 %[d], %[k], %[q], -1, %[d]" : [d] "+v"(B), [k] "=s"(kc) : [q] "v"(q));
            else
              asm("v_mad_i64_i32 %[d], %[k], %[q], 1, %[d]" : [d] "+v"(A), [k] "=s"(kc) : [q] "v"(q));
          }
          sum[k] = A - B;
        }
      } else {
#pragma unroll
        for (int c = 0; c < L; c++)
          finish(c, (uint64_t)(int64_t)(int32_t)p[c][0], (uint64_t)(int64_t)(int32_t)p[c][1]);
      }
    } else {
#pragma unroll
      for (int c = 0; c < L; c++)
        finish(c, exact_q<XT, CT, L, kGeneral>(xv, wv, ka, qs, c, 0), exact_q<XT, CT, L, kGeneral>(xv, wv, ka, qs, c, 1));
    }
    const int sum_mode = ka->sum_mode;
    if (sum_mode != 0 && (!(SA_ABLATE & 8) || sum[0] == 0x123456789ull)) {
      const rsrc_t rs = make_rsrc(ka->sum_out, n * 8);
      if (sum_mode == 2) {
        const Vec2<uint64_t> o = bload2<uint64_t>(rs, i);
        sum[0] += o.v[0];
        sum[1] += o.v[1];
      }
      bstore2_u64(rs, i, sum[0], sum[1]);
    }
#ifdef SA_TIMING
    if (tiles++ == 0) SA_TS(ts2);
#endif
  }
  SA_TS(ts3);

  // ---- digests: wave XOR reduction (shuffles), then the block's 4 waves
  // through LDS, one 64-bit atomic per client per BLOCK.  Every wave ends at
  // about the same time, so per-wave atomics on the same L clients' words
  // serialised at the L2: ~2,000 per address cost ~0.13 ms per launch.
  if (!kSum && a.do_digest) {
    __shared__ uint64_t wdig[kBlockThreads / 64][L];
#pragma unroll
    for (int c = 0; c < L; c++) {
      uint64_t d = kDigLds ? dig_lds[c][threadIdx.x] : dig[kDigLds ? 0 : c];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) d ^= __shfl_xor(d, off, 64);
      if ((threadIdx.x & 63) == 0) wdig[threadIdx.x >> 6][c] = d;
    }
    __syncthreads();
    if (threadIdx.x < L) {
      uint64_t d = 0;
#pragma unroll
      for (int w = 0; w < kBlockThreads / 64; w++) d ^= wdig[w][threadIdx.x];
      if (d) atomicXor((unsigned long long*)&a.digests[threadIdx.x], d);
    }
  }
  if (a.flags && !(SA_ABLATE & 1) && __any(zmin == 0) && (threadIdx.x & 63) == 0)
    atomicOr(a.flags, SA_FLAG_PRG_REJECT);
#ifdef SA_TIMING
  SA_TS(ts4);
  const uint32_t wid = blockIdx.x * (kBlockThreads / 64) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && wid < kTsWaves) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint64_t* o = g_sa_ts[wid];
    o[0] = ts0; o[1] = ts1; o[2] = ts2; o[3] = ts3; o[4] = ts4;
    o[5] = tiles; o[6] = hw; o[7] = xcc;
  }
#endif
}

// ----------------------------------------------------------------------------
// launcher
// ----------------------------------------------------------------------------
int occupancy_blocks(const void* kernel);  // sa_api.hip
int masking_grid_cap(const void* kernel);  // sa_api.hip: occupancy less sa_set_masking_reserve's CUs

// Buffer offsets are 32-bit byte offsets, so one launch covers at most
// kChunkElems elements (4 GiB of u64); longer vectors are cut into chunks
// whose streams start kChunkElems draws further on.
constexpr uint64_t kChunkElems = (1ull << 29) - kTile;
static_assert(kChunkElems % kTile == 0, "chunk");

template <typename XT, typename CT, int L, int X, int K = kAllPairs>
int launch_clients(const KArgs& in, void* stream) {
  constexpr int P = Pairs<L, K>::count + L * X;
  const void* kfn = reinterpret_cast<const void*>(&k_clients<XT, CT, L, X, K>);
  const int maxb = masking_grid_cap(kfn);
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
      a.dp_block0 += off / kDpBlock;
      const Jump jo = jump_of(off);
      for (int j = 0; j < P; j++) {
        const u128 s = apply(jo, mk128(a.s[j].s_hi, a.s[j].s_lo), mk128(a.s[j].inc_hi, a.s[j].inc_lo));
        a.s[j].s_lo = lo64(s);
        a.s[j].s_hi = hi64(s);
      }
    }
    a.masked_mask = 0;
    for (int c = 0; c < L; c++)
      if (a.c[c].masked_out) a.masked_mask |= 1u << c;
    const uint64_t tiles = (a.n + kTile - 1) / kTile;
    const int grid = (int)(tiles < (uint64_t)maxb ? tiles : (uint64_t)maxb);
    if (grid >= (1 << kGridBits)) {
      sa_set_error("masking kernel: grid of %d blocks exceeds the prologue's %d-bit block jump", grid, kGridBits);
      return SA_ERR_UNSUPPORTED;
    }
    // merged tile jump: S_{i+kE} -> S_{i+stride+1}, i.e. stride - kE + 1 draws
    const Jump jj = jump_of((uint64_t)grid * kTile - (kE - 1));
    a.aj_lo = lo64(jj.mult);
    a.aj_hi = hi64(jj.mult);
    const u128 aji = inv128(jj.mult);
    a.aji_lo = lo64(aji);
    a.aji_hi = hi64(aji);
    for (int j = 0; j < P; j++) {
      const u128 cj = jj.gsum * mk128(a.s[j].inc_hi, a.s[j].inc_lo);
      a.s[j].cj_lo = lo64(cj);
      a.s[j].cj_hi = hi64(cj);
      a.s[j].inc_w0 = (uint32_t)a.s[j].inc_lo;
      a.s[j].inc_w1 = a.s[j].inc_lo >> 32;
      a.s[j].cj_w0 = (uint32_t)a.s[j].cj_lo;
      a.s[j].cj_w1 = a.s[j].cj_lo >> 32;
    }
    hipLaunchKernelGGL((k_clients<XT, CT, L, X, K>), dim3(grid), dim3(kBlockThreads), 0,
                       (hipStream_t)stream, a);
    SA_HIP_CHECK(hipGetLastError());
  }
  return SA_OK;
}

}  // namespace sa
