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
// Elements per lane per chunk.  A lane walks its run in steps of 4 (one 16-B
// load per client per step; lanes kRun*4 bytes apart, so each load
// instruction touches 64 lines that later steps finish consuming), and jumps
// its streams once per run: the jump costs one multiply-add like a draw, so
// kRun=4 (fully coalesced) pays 1 extra step per 4 draws, kRun=16 1 per 16.
#ifndef SA_RUN
#define SA_RUN 8
#endif
constexpr int kRun = SA_RUN;
// Streams whose draws may interleave between two fences (ILP inside a wave;
// more streams = more live temporaries).
#ifndef SA_GROUP
#define SA_GROUP 1
#endif
constexpr int kGroup = SA_GROUP;
static_assert(kRun % 4 == 0, "run is a multiple of the 4-element step");

template <typename XT, typename CT, int L, int X>
__global__ void __launch_bounds__(kBlockThreads, 2) k_clients(const KArgs a) {
  constexpr int PI = Pairs<L>::count;
  constexpr int P = PI + L * X;
  constexpr bool kGeneral = (L == 1);  // continue mode + per-element weights
  static_assert(L >= 1 && L <= kMaxLocal, "L");
  static_assert(P <= kMaxStreams, "P");

  const uint64_t n = a.n;
  // lane owns a run of kRun consecutive elements per chunk (draw order), the
  // block a chunk of 256*kRun; the grid strides over chunks.
  constexpr uint64_t kChunk = (uint64_t)kBlockThreads * kRun;
  const uint64_t first = (uint64_t)blockIdx.x * kChunk + (uint64_t)threadIdx.x * kRun;
  const uint64_t stride = (uint64_t)gridDim.x * kChunk;

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

  uint64_t badmask = 0;  // lanes that saw a raw PCG64 draw of 0 (SGPR pair)

  // per-lane XOR digests live in LDS (one lane-private slot per client):
  // ds_xor_b64 per finished element instead of 2 VGPRs per client
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

  lds_ptr slp = (lds_ptr)(sl);
  for (uint64_t run0 = first; run0 < n; run0 += stride) {
#pragma unroll 1
   for (int step = 0; step < kRun / 4; step++) {
    const uint64_t i = run0 + 4 * (uint64_t)step;
    // ---- issue this step's loads early; consumed as each element finishes
    // (continue mode and per-element weights exist only for the single-client
    // kernel; the fused kernel drops them at compile time to save registers)
    Vec4<XT> xv[L];
    Vec4<CT> wv[kGeneral ? L : 1];
    Vec4<uint64_t> pv[kGeneral ? L : 1];
#pragma unroll
    for (int c = 0; c < L; c++) {
      if (kGeneral && a.continue_mode) {
        pv[c] = bload4<uint64_t>(rm[c], i, n);
      } else {
        xv[c] = bload4<XT>(rx[c], i, n);
        if (kGeneral && a.c[c].wvec) wv[c] = bload4<CT>(rw[kGeneral ? c : 0], i, n);
      }
    }

    // ---- element-outer: one draw per stream per element.  Each stream's
    // step is fenced (empty volatile asm on its state, the LDS pointer and
    // the accumulators it touches), so only one stream's constants and
    // temporaries are live at a time: P*4 state VGPRs + L accumulators.
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint64_t acc[L];
#pragma unroll
      for (int c = 0; c < L; c++) acc[c] = a.c[c].bias;
      if constexpr (P > 0) {
#pragma unroll
        for (int g0 = 0; g0 < P; g0 += kGroup) {
          // fence in: the group's states and the LDS pointer (ordered after
          // the previous group's fence out), then the group's draws are free
          // to interleave (ILP), then fence out states + accumulators.
          uint64_t slo[kGroup], shi[kGroup], t[kGroup];
#pragma unroll
          for (int g = 0; g < kGroup; g++) {
            if (g0 + g < P) {
              slo[g] = lo64(st[g0 + g]);
              shi[g] = hi64(st[g0 + g]);
              asm volatile("" : "+v"(slo[g]), "+v"(shi[g]), "+v"(slp));
            }
          }
#pragma unroll
          for (int g = 0; g < kGroup; g++) {
            const int q = g0 + g;
            if (q < P) {
              const uint64_t inc_lo = slp[q].inc_lo, inc_hi = slp[q].inc_hi, smask = slp[q].smask;
              const u128 sv = mk128(shi[g], slo[g]) * kPcgMult + mk128(inc_hi, inc_lo);
              note_zero_draw(badmask, sv);
              t[g] = draw_signed(sv, smask);
              slo[g] = lo64(sv);
              shi[g] = hi64(sv);
              const int cu = q < PI ? Pairs<L>::u(q) : (q - PI) / (X > 0 ? X : 1);
              const int cv = q < PI ? Pairs<L>::v(q) : cu;
              acc[cu] += t[g];
              if (q < PI) acc[cv] -= t[g];
            }
          }
#pragma unroll
          for (int g = 0; g < kGroup; g++) {
            const int q = g0 + g;
            if (q < P) {
              const int cu = q < PI ? Pairs<L>::u(q) : (q - PI) / (X > 0 ? X : 1);
              const int cv = q < PI ? Pairs<L>::v(q) : cu;
              asm volatile("" : "+v"(slo[g]), "+v"(shi[g]), "+v"(acc[cu]), "+v"(acc[cv]));
              st[q] = mk128(shi[g], slo[g]);
            }
          }
        }
      }
      // ---- finish element k: add the quantized value (or the prior pass)
      uint64_t s_k = 0;
#pragma unroll
      for (int c = 0; c < L; c++) {
        if (kGeneral && a.continue_mode) {
          acc[c] += pv[kGeneral ? c : 0].v[k];
        } else {
          const CT w = (kGeneral && a.c[c].wvec) ? wv[kGeneral ? c : 0].v[k] : scalar_weight<CT>(a.c[c]);
          acc[c] += quantize<XT, CT>(xv[c].v[k], w, a);
        }
        s_k += acc[c];
        if (i + k < n) {
          __hip_atomic_fetch_xor(&dig_lds[c][threadIdx.x], acc[c], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
          if (a.c[c].masked_out) bstore_u64(rm[c], i + k, acc[c]);
        }
      }
      // the element's masked sum (8-B store; a lane's run fills whole lines)
      if (a.sum_mode != 0 && i + k < n) {
        if (a.sum_mode == 2) s_k += bload_u64(rs, i + k);
        bstore_u64(rs, i + k, s_k);
      }
    }
   }

    // ---- jump every stream to this lane's next run (same fencing)
    if constexpr (P > 0) {
#pragma unroll
      for (int q = 0; q < P; q++) {
        uint64_t slo = lo64(st[q]), shi = hi64(st[q]);
        asm volatile("" : "+v"(slo), "+v"(shi), "+v"(slp));
        const u128 sv = mk128(shi, slo) * AJ + mk128(slp[q].cj_hi, slp[q].cj_lo);
        slo = lo64(sv);
        shi = hi64(sv);
        asm volatile("" : "+v"(slo), "+v"(shi));
        st[q] = mk128(shi, slo);
      }
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
  const uint64_t tiles = (in.n + (uint64_t)kBlockThreads * kRun - 1) / ((uint64_t)kBlockThreads * kRun);
  const int grid = (int)(tiles < (uint64_t)maxb ? tiles : (uint64_t)maxb);
  KArgs a = in;
  // per-run jump J = grid*256*kRun - kRun draws (the lane consumed its run)
  const Jump jj = jump_of((uint64_t)grid * kBlockThreads * kRun - kRun);
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
