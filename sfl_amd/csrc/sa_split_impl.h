// sa_split_impl.h — the fused masking kernel for 5..8 co-located fp32 clients
// with the pair streams split over two waves.
//
// With all P = L(L-1)/2 pair states in one wave (k_clients), L = 8 needs
// ~230 VGPRs: 2 waves per SIMD, too few to hide the v_mad_u64_u32 chains of
// the PCG64 step.  Here the four waves of a workgroup form two groups of two;
// both waves of a group work on the SAME 256 elements (lane l: 4l..4l+3) and
// each expands half of the pair streams (wave half 0: streams [0, P/2), half
// 1: [P/2, P)).  After every element the halves swap the partial masks of
// each other's clients through LDS (half 0 finalizes clients [0, L/2), half
// 1 clients [L/2, L)): quantize, digest, optional masked vector, partial sum.
// Half 1 hands its partial sums to half 0, which writes the masked sum.
// Each wave holds half the states, so the kernel runs 4 waves per SIMD.
//
// Results are identical to k_clients: the same draws, the same per-client
// masked values and the same sums (uint64 addition commutes).
#pragma once
#include "sa_clients_impl.h"

namespace sa {

constexpr int kSplitSub = 64 * kElemsPerLane;  // elements per wave group (256)
constexpr int kSplitTile = 2 * kSplitSub;      // elements per block tile (512)

template <int L, int HALF>
__device__ __forceinline__ void split_run(const KArgs& a, const int g, const int lane, lds_ptr slp,
                                          uint64_t (*xch)[2][2][L / 2 + 1][64], uint64_t (*sx)[4][64],
                                          uint64_t (*dig)[kBlockThreads], uint64_t* tw) {
  using XT = float;
  using CT = float;
  constexpr int P = Pairs<L>::count;
  constexpr int H = L / 2;                    // half 0 finalizes [0, H), half 1 [H, L)
  constexpr int Q0 = P / 2;
  constexpr int qlo = HALF ? Q0 : 0, qhi = HALF ? P : Q0;
  constexpr int NQ = qhi - qlo;
  constexpr int clo = HALF ? H : 0, chi = HALF ? L : H;
  constexpr int NC = chi - clo;               // own clients
  constexpr int olo = HALF ? 0 : H, ohi = HALF ? H : L;
  constexpr int NO = ohi - olo;               // the other half's clients
  static_assert(NC <= L / 2 + 1 && NO <= L / 2 + 1, "exchange slots");

  const uint64_t n = a.n;
  const uint64_t first = (uint64_t)blockIdx.x * kSplitTile + (uint64_t)g * kSplitSub + (uint64_t)lane * kElemsPerLane;
  const uint64_t stride = (uint64_t)gridDim.x * kSplitTile;

  // ---- prologue: this half's streams jumped to the lane's first element
  uint32_t st[NQ][4];
  {
    Jump jl{1, 0};
    uint64_t pos = first;
    for (int b = 0; pos != 0; b++, pos >>= 1) {
      if (pos & 1) jl = compose(jl, kPowTable.e[b]);
    }
#pragma unroll
    for (int j = 0; j < NQ; j++) {
      const StreamArg& s = a.s[qlo + j];
      const u128 v = apply(jl, ld128(s.s_lo, s.s_hi), ld128(s.inc_lo, s.inc_hi));
      st[j][0] = (uint32_t)lo64(v);
      st[j][1] = (uint32_t)(lo64(v) >> 32);
      st[j][2] = (uint32_t)hi64(v);
      st[j][3] = (uint32_t)(hi64(v) >> 32);
    }
  }
  const u128 AJ1 = ld128(a.aj_lo, a.aj_hi);
  uint32_t zmin = 0xFFFFFFFFu;

  rsrc_t rx[NC], rm[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) {
    rx[c] = make_rsrc(a.c[clo + c].x, n * sizeof(XT));
    rm[c] = make_rsrc(a.c[clo + c].masked_out, n * 8);
  }
  const rsrc_t rs = make_rsrc(a.sum_out, n * 8);

  int tile = 0;
  // block-uniform trip count: both halves pass the same barriers
  for (uint64_t base = (uint64_t)blockIdx.x * kSplitTile; base < n; base += stride, tile++) {
    const uint64_t i = base + (uint64_t)g * kSplitSub + (uint64_t)lane * kElemsPerLane;
    const bool jstep = tile > 0;
    const u128 M0 = jstep ? AJ1 : kPcgMult;
    const int add0 = jstep ? 2 : 0;

    Vec4<XT> xv[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) xv[c] = bload4<XT>(rx[c], i, n);

    uint64_t sum[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t al[L], ah[L];
#pragma unroll
      for (int c = 0; c < L; c++) {
        const bool own = c >= clo && c < chi;
        al[c] = own ? (uint32_t)a.c[c].bias : 0u;
        ah[c] = own ? (uint32_t)(a.c[c].bias >> 32) : 0u;
      }
      const u128 Mk = k == 0 ? M0 : kPcgMult;
      const uint32_t m0 = (uint32_t)lo64(Mk), m1 = (uint32_t)(lo64(Mk) >> 32);
      const uint32_t m2 = (uint32_t)hi64(Mk), m3 = (uint32_t)(hi64(Mk) >> 32);
#pragma unroll
      for (int j = 0; j < NQ; j++) {
        const int q = qlo + j;
        asm volatile("" : "+v"(slp));
        typedef __attribute__((address_space(3))) const uint64_t* lds_u64;
        const lds_u64 cp = (lds_u64)(slp + q) + (k == 0 ? add0 : 0);
        const uint64_t c01 = cp[0], c23 = cp[1];
        const uint32_t sm = (uint32_t)slp[q].smask;
        const int cu = Pairs<L>::u(q), cv = Pairs<L>::v(q);
        pcg_draw_pair(st[j][0], st[j][1], st[j][2], st[j][3], m0, m1, m2, m3, c01, c23, sm, zmin, al[cu], ah[cu],
                      al[cv], ah[cv]);
      }
      // ---- swap partial masks with the other half of the group
      uint64_t* const mine = &xch[k & 1][g][HALF][0][0];
      const uint64_t* const theirs = &xch[k & 1][g][1 - HALF][0][0];
#pragma unroll
      for (int c = 0; c < NO; c++) mine[c * 64 + lane] = pack64(al[olo + c], ah[olo + c]);
      __syncthreads();
      uint64_t s_k = 0;
#pragma unroll
      for (int c = 0; c < NC; c++) {
        uint64_t acc = pack64(al[clo + c], ah[clo + c]) + theirs[c * 64 + lane];
        acc += quantize<XT, CT>(xv[c].v[k], scalar_weight<CT>(a.c[clo + c]), a);
        s_k += acc;
        if (i + k < n) {
          __hip_atomic_fetch_xor(&dig[c][threadIdx.x], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (a.c[clo + c].masked_out) bstore_u64(rm[c], i + k, acc);
        }
      }
      if (HALF) sx[g][k][lane] = s_k;
      sum[k] = s_k;
    }
    __syncthreads();  // half 1's partial sums are in sx
    if (!HALF && a.sum_mode != 0) {
#pragma unroll
      for (int k = 0; k < 4; k++) sum[k] += sx[g][k][lane];
      const uint64_t e0 = i - 4 * (uint64_t)lane + 2 * (uint64_t)lane;
      const uint64_t e1 = e0 + 128;
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

  if (a.do_digest) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
      uint64_t d = dig[c][threadIdx.x];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) d ^= __shfl_xor(d, off, 64);
      if (lane == 0 && d) atomicXor((unsigned long long*)&a.digests[clo + c], d);
    }
  }
  if (a.flags && __any(zmin == 0) && lane == 0) atomicOr(a.flags, SA_FLAG_PRG_REJECT);
}

// waves per SIMD the register allocation targets: L = 8 fits 148 VGPRs
// (3 waves); capping it at 128 for 4 waves spills to scratch
template <int L>
constexpr int split_waves() { return L == 8 ? 3 : 4; }

template <int L>
__global__ void __launch_bounds__(kBlockThreads, split_waves<L>()) k_clients_split(const KArgs a) {
  constexpr int P = Pairs<L>::count;
  static_assert(L >= 4 && L <= kMaxLocal, "split kernel is for 4..8 clients");
  __shared__ StreamLds sl[P];
  for (int j = threadIdx.x; j < P; j += blockDim.x) {
    const StreamArg& s = a.s[j];
    sl[j] = StreamLds{s.inc_lo, s.inc_hi, s.cj_lo, s.cj_hi, s.smask, 0};
  }
  // [k parity][group][writer half][client slot][lane]
  __shared__ uint64_t xch[2][2][2][L / 2 + 1][64];
  __shared__ uint64_t sx[2][4][64];                          // half 1's partial sums per group
  __shared__ uint64_t dig[L / 2 + 1][kBlockThreads];         // per-lane digests of own clients
  __shared__ uint64_t tr[2 * 64 * kElemsPerLane];            // transposes of the two half-0 waves
#pragma unroll
  for (int c = 0; c < L / 2 + 1; c++) dig[c][threadIdx.x] = 0;
  __syncthreads();

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave >> 1, lane = threadIdx.x & 63;
  uint64_t* const tw = tr + g * 64 * kElemsPerLane;
  lds_ptr slp = (lds_ptr)(sl);
  if (wave & 1)
    split_run<L, 1>(a, g, lane, slp, xch, sx, dig, tw);
  else
    split_run<L, 0>(a, g, lane, slp, xch, sx, dig, tw);
}

template <int L>
int launch_split(const KArgs& in, void* stream) {
  constexpr int P = Pairs<L>::count;
  const void* kfn = reinterpret_cast<const void*>(&k_clients_split<L>);
  const int maxb = occupancy_blocks(kfn);
  if (maxb <= 0) return SA_ERR_HIP;
  for (uint64_t off = 0; off < in.n; off += kChunkElems) {
    KArgs a = in;
    a.n = in.n - off < kChunkElems ? in.n - off : kChunkElems;
    if (off) {
      for (int c = 0; c < L; c++) {
        if (a.c[c].x) a.c[c].x = static_cast<const float*>(a.c[c].x) + off;
        if (a.c[c].masked_out) a.c[c].masked_out += off;
      }
      if (a.sum_out) a.sum_out += off;
      const Jump jo = jump_of(off);
      for (int j = 0; j < P; j++) {
        const u128 s = apply(jo, mk128(a.s[j].s_hi, a.s[j].s_lo), mk128(a.s[j].inc_hi, a.s[j].inc_lo));
        a.s[j].s_lo = lo64(s);
        a.s[j].s_hi = hi64(s);
      }
    }
    const uint64_t tiles = (a.n + kSplitTile - 1) / kSplitTile;
    const int grid = (int)(tiles < (uint64_t)maxb ? tiles : (uint64_t)maxb);
    const Jump jj = jump_of((uint64_t)grid * kSplitTile - (kElemsPerLane - 1));
    a.aj_lo = lo64(jj.mult);
    a.aj_hi = hi64(jj.mult);
    for (int j = 0; j < P; j++) {
      const u128 cj = jj.gsum * mk128(a.s[j].inc_hi, a.s[j].inc_lo);
      a.s[j].cj_lo = lo64(cj);
      a.s[j].cj_hi = hi64(cj);
    }
    hipLaunchKernelGGL((k_clients_split<L>), dim3(grid), dim3(kBlockThreads), 0, (hipStream_t)stream, a);
    SA_HIP_CHECK(hipGetLastError());
  }
  return SA_OK;
}

}  // namespace sa
