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

namespace sa {

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
__device__ __forceinline__ uint64_t draw_signed(u128 s, uint64_t smask) {
  const uint64_t hi = hi64(s), lo = lo64(s);
  const uint64_t x = hi ^ lo ^ smask;
  const unsigned r = (unsigned)(hi >> 58);
  return __builtin_rotateright64(x, r);
}

// Streams whose draws the scheduler may interleave inside one tile; a
// scheduling fence after each group bounds the live temporaries (unfenced,
// hipcc issues every stream's constant loads up front and spills past ~9).
#ifndef SA_SCHED_GROUP
#define SA_SCHED_GROUP 2
#endif
constexpr int kSchedGroup = SA_SCHED_GROUP;

struct StreamLds {
  uint64_t inc_lo, inc_hi, cj_lo, cj_hi, smask, pad;
};

typedef __attribute__((address_space(3))) const StreamLds* lds_ptr;  // 32-bit LDS address
__device__ __forceinline__ StreamLds read_stream(lds_ptr p, int j) {
  return StreamLds{p[j].inc_lo, p[j].inc_hi, p[j].cj_lo, p[j].cj_hi, p[j].smask, 0};
}

// raw == 0  <=>  hi == lo.  One v_cmp + one s_or into a wave-wide SGPR mask;
// written as volatile asm so hipcc cannot sink the compare to the loop latch
// (it did, keeping every intermediate state of the tile live).
__device__ __forceinline__ void note_zero_draw(uint64_t& badmask, u128 s) {
  const uint64_t hi = hi64(s), lo = lo64(s);
  asm volatile("v_cmp_eq_u64 vcc, %1, %2\n\ts_or_b64 %0, %0, vcc"
               : "+s"(badmask)
               : "v"(hi), "v"(lo)
               : "vcc");
}

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
template <typename XT, typename CT, int L, int X>
__global__ void __launch_bounds__(kBlockThreads, 2) k_clients(const KArgs a) {
  constexpr int PI = Pairs<L>::count;
  constexpr int P = PI + L * X;
  static_assert(L >= 1 && L <= kMaxLocal, "L");
  static_assert(P <= kMaxStreams, "P");

  const uint64_t n = a.n;
  const uint64_t first = (uint64_t)blockIdx.x * kTileElems + (uint64_t)threadIdx.x * kElemsPerLane;
  const uint64_t stride = (uint64_t)gridDim.x * kTileElems;

  // ---- per-stream constants go to LDS once; the tile loop re-reads them
  // right before each use (a compiler barrier stops LICM from hoisting 7
  // dwords x P streams into registers, which spills at P > 8).
  __shared__ StreamLds sl[P > 0 ? P : 1];
  if constexpr (P > 0) {
    for (int j = threadIdx.x; j < P; j += blockDim.x) {
      const StreamArg& s = a.s[j];
      sl[j] = StreamLds{s.inc_lo, s.inc_hi, s.cj_lo, s.cj_hi, s.smask, 0};
    }
    __syncthreads();
  }

  // ---- prologue: jump every stream from draw 0 to this lane's first element
  u128 st[P > 0 ? P : 1];
  if constexpr (P > 0) {
    Jump jl{1, 0};
    uint64_t pos = first;
    for (int b = 0; pos != 0; b++, pos >>= 1) {
      if (pos & 1) jl = compose(jl, kPowTable.e[b]);
    }
#pragma unroll
    for (int j = 0; j < P; j++) {
      const StreamArg& s = a.s[j];
      st[j] = apply(jl, ld128(s.s_lo, s.s_hi), ld128(s.inc_lo, s.inc_hi));
    }
  }
  const u128 AJ = ld128(a.aj_lo, a.aj_hi);

  uint64_t dig[L];
#pragma unroll
  for (int c = 0; c < L; c++) dig[c] = 0;
  uint64_t badmask = 0;  // lanes that saw a raw PCG64 draw of 0 (SGPR pair)

  lds_ptr slp = (lds_ptr)(sl);
  for (uint64_t i = first; i < n; i += stride) {
    // Opaque per tile: the stream constants are re-read from LDS (broadcast
    // ds_read) inside the tile instead of being hoisted into 7*P registers.
    asm volatile("" : "+v"(slp));

    // ---- issue this tile's loads early; consumed after the PRG work
    Vec4<XT> xv[L];
    Vec4<CT> wv[L];
    uint64_t acc[L][4];
#pragma unroll
    for (int c = 0; c < L; c++) {
      if (a.continue_mode) {
        const Vec4<uint64_t> p = load4<uint64_t>(a.c[c].masked_out, i, n);
#pragma unroll
        for (int k = 0; k < 4; k++) acc[c][k] = p.v[k] + a.c[c].bias;
      } else {
        xv[c] = load4<XT>(reinterpret_cast<const XT*>(a.c[c].x), i, n);
        if (a.c[c].wvec) wv[c] = load4<CT>(reinterpret_cast<const CT*>(a.c[c].wvec), i, n);
#pragma unroll
        for (int k = 0; k < 4; k++) acc[c][k] = a.c[c].bias;
      }
    }

    // ---- mask expansion, stream-outer: each stream's 4 draws back to back,
    // then its jump to the next tile.  Streams are processed in groups of
    // kSchedGroup; empty volatile asm statements on the group's states (in)
    // and on its states + accumulators (out) pin the order, so only one
    // group's constants and temporaries are live at a time (left alone,
    // hipcc re-interleaves every stream per element and spills past ~9).
    if constexpr (P > 0) {
#pragma unroll
      for (int g0 = 0; g0 < P; g0 += kSchedGroup) {
        constexpr int G = kSchedGroup;
        uint64_t slo[G], shi[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
          slo[g] = g0 + g < P ? lo64(st[g0 + g]) : 0;
          shi[g] = g0 + g < P ? hi64(st[g0 + g]) : 0;
        }
        if constexpr (G == 1)
          asm volatile("" : "+v"(slo[0]), "+v"(shi[0]), "+v"(slp));
        else
          asm volatile("" : "+v"(slo[0]), "+v"(shi[0]), "+v"(slo[1]), "+v"(shi[1]), "+v"(slp));
#pragma unroll
        for (int g = 0; g < G; g++) {
          const int q = g0 + g;
          if (q >= P) break;
          const StreamLds c = read_stream(slp, q);
          const u128 inc = ld128(c.inc_lo, c.inc_hi);
          u128 sv = mk128(shi[g], slo[g]);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            sv = sv * kPcgMult + inc;
            note_zero_draw(badmask, sv);
            const uint64_t t = draw_signed(sv, c.smask);
            if (q < PI) {  // internal pair: one draw, two clients
              acc[Pairs<L>::u(q)][k] += t;
              acc[Pairs<L>::v(q)][k] -= t;
            } else {  // cross-GPU peer: one client
              acc[(q - PI) / (X > 0 ? X : 1)][k] += t;
            }
          }
          sv = sv * AJ + ld128(c.cj_lo, c.cj_hi);
          slo[g] = lo64(sv);
          shi[g] = hi64(sv);
        }
        // fence out: this group's states and every accumulator it touched
#pragma unroll
        for (int g = 0; g < G; g++) {
          const int q = g0 + g;
          if (q >= P) break;
          const int cu = q < PI ? Pairs<L>::u(q) : (q - PI) / (X > 0 ? X : 1);
          const int cv = q < PI ? Pairs<L>::v(q) : cu;
          asm volatile("" : "+v"(slo[g]), "+v"(shi[g]), "+v"(acc[cu][0]), "+v"(acc[cu][1]),
                       "+v"(acc[cu][2]), "+v"(acc[cu][3]), "+v"(acc[cv][0]), "+v"(acc[cv][1]),
                       "+v"(acc[cv][2]), "+v"(acc[cv][3]));
          st[q] = mk128(shi[g], slo[g]);
        }
      }
    }

    // ---- finish: add the quantized values, digest, sum, store
    uint64_t sum[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < L; c++) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!a.continue_mode) {
          const CT w = a.c[c].wvec ? wv[c].v[k] : scalar_weight<CT>(a.c[c]);
          acc[c][k] += quantize<XT, CT>(xv[c].v[k], w, a);
        }
        sum[k] += acc[c][k];
        if (i + k < n) dig[c] ^= acc[c][k];
      }
      if (a.c[c].masked_out) store4_u64(a.c[c].masked_out, i, n, acc[c]);
    }
    if (a.sum_mode == 2) {
      const Vec4<uint64_t> o = load4<uint64_t>(a.sum_out, i, n);
#pragma unroll
      for (int k = 0; k < 4; k++) sum[k] += o.v[k];
    }
    if (a.sum_mode != 0) store4_u64(a.sum_out, i, n, sum);
  }

  // ---- wave-level XOR reduction of the digests, one atomic per wave
  if (a.do_digest) {
#pragma unroll
    for (int c = 0; c < L; c++) {
      uint64_t d = dig[c];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) d ^= __shfl_xor(d, off, 64);
      if ((threadIdx.x & 63) == 0 && d) atomicXor((unsigned long long*)&a.digests[c], d);
    }
  }
  if (a.flags && badmask != 0 && (threadIdx.x & 63) == 0) atomicOr(a.flags, SA_FLAG_PRG_REJECT);
}

// ----------------------------------------------------------------------------
// launcher
// ----------------------------------------------------------------------------
int occupancy_blocks(const void* kernel);  // sa_api.hip

template <typename XT, typename CT, int L, int X>
int launch_clients(const KArgs& in, void* stream) {
  constexpr int P = Pairs<L>::count + L * X;
  const void* kfn = reinterpret_cast<const void*>(&k_clients<XT, CT, L, X>);
  const int maxb = occupancy_blocks(kfn);
  if (maxb <= 0) return SA_ERR_HIP;
  const uint64_t tiles = (in.n + kTileElems - 1) / kTileElems;
  const int grid = (int)(tiles < (uint64_t)maxb ? tiles : (uint64_t)maxb);
  KArgs a = in;
  // per-tile jump J = grid*1024 - 4 draws (the lane already consumed 4)
  const Jump jj = jump_of((uint64_t)grid * kTileElems - kElemsPerLane);
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
  return SA_OK;
}

}  // namespace sa
