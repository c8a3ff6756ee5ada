// sa_reject.hip — numpy's rejection re-draw, reproduced after the fact.
//
// The masks are Generator.integers(int64.min, int64.max) draws (Lemire's
// bounded method over rng = 2^64 - 2): a raw PCG64 output of 0 is REJECTED
// and the next raw output taken instead, so from that element on the stream
// is one raw draw further along (p = 2^-64 per draw).  The masking kernels
// only detect it (SA_FLAG_PRG_REJECT); the host then
//   1. finds the rejected raw draws of every stream of the launch
//      (sa_pcg64_find_zero: the first raw index == 0 in a window),
//   2. shifts the affected clients' masked vectors from that element on
//      (sa_stream_shift: out[e] += sign * (raw[e+s] - raw[e+s-1])),
//   3. recomputes the XOR digests (sa_xor_u64)
// and advances the pair's stream position by the extra draws.  A pair stream
// enters its two clients with opposite signs, so the masked SUM never
// changes; only the per-client masked vectors (wire images) and digests do.
// None of this is on the hot path: it runs only after the flag is raised.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/sfl_sa.h"
#include "pcg128.h"
#include "sa_internal.h"

namespace sa {

constexpr int kRejBlocks = 1024;  // blocks per stream: each lane walks a contiguous run
constexpr int kFindMax = 64;      // streams per sa_pcg64_find_zero launch

struct FindArgs {
  uint64_t s_lo[kFindMax], s_hi[kFindMax], i_lo[kFindMax], i_hi[kFindMax];
  uint64_t n;
  uint64_t* first;
};

__device__ __forceinline__ u128 step(u128 s, u128 inc) { return s * kPcgMult + inc; }

// lane range [lo, hi) of a length-n index space split over `lanes` lanes
__device__ __forceinline__ void lane_range(uint64_t n, uint64_t lane, uint64_t lanes, uint64_t& lo, uint64_t& hi) {
  const uint64_t per = (n + lanes - 1) / lanes;
  lo = lane * per;
  hi = lo + per < n ? lo + per : n;
}

__global__ void __launch_bounds__(256) k_find_zero(const FindArgs a) {
  const int j = blockIdx.y;
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  uint64_t lo, hi;
  lane_range(a.n, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, lanes, lo, hi);
  if (lo >= hi) return;
  const u128 inc = mk128(a.i_hi[j], a.i_lo[j]);
  u128 s = apply(jump_of(lo), mk128(a.s_hi[j], a.s_lo[j]), inc);  // state before raw draw lo
  for (uint64_t i = lo; i < hi; i++) {
    s = step(s, inc);
    if (hi64(s) == lo64(s)) {  // XSL-RR output 0 <=> hi == lo
      atomicMin((unsigned long long*)&a.first[j], (unsigned long long)i);
      return;
    }
  }
}

// out[e] += sign * (raw[e + shift] - raw[e + shift - 1]) for e in [k, n)
__global__ void __launch_bounds__(256) k_stream_shift(uint64_t* __restrict__ out, uint64_t n, uint64_t k,
                                                      uint64_t shift, uint64_t s_lo, uint64_t s_hi, uint64_t i_lo,
                                                      uint64_t i_hi, int sign) {
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  uint64_t lo, hi;
  lane_range(n - k, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, lanes, lo, hi);
  if (lo >= hi) return;
  lo += k;
  hi += k;
  const u128 inc = mk128(i_hi, i_lo);
  u128 s = apply(jump_of(lo + shift - 1), mk128(s_hi, s_lo), inc);  // before raw[lo + shift - 1]
  s = step(s, inc);
  uint64_t prev = xslrr(s);
  for (uint64_t e = lo; e < hi; e++) {
    s = step(s, inc);
    const uint64_t cur = xslrr(s);
    const uint64_t d = cur - prev;
    out[e] += sign > 0 ? d : (uint64_t)0 - d;
    prev = cur;
  }
}

// XOR of n words: 16-byte loads, four independent ones in flight per lane,
// and ONE atomic per block (the waves' partials combined in LDS): one
// atomicXor per wave on the single digest word serialised 8,192 atomics and
// held a 100 MB vector to ~1 TB/s (rocprof of tools/party_bench.py,
// profiles/r06/dropin_rocprof_*).  v is 8-byte aligned: at most one word
// before the first 16-byte boundary, and at most one after the last pair.
__global__ void __launch_bounds__(256) k_xor_u64(const uint64_t* __restrict__ v, uint64_t n,
                                                 unsigned long long* digest) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t head = ((uintptr_t)v & 15) ? 1 : 0;
  const uint64_t m = n > head ? (n - head) / 2 : 0;  // 16-byte pairs
  const ulong2* __restrict__ p = reinterpret_cast<const ulong2*>(v + head);
  uint64_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
  uint64_t i = tid;
  for (; i + 3 * stride < m; i += 4 * stride) {
    const ulong2 a = p[i], b = p[i + stride], c = p[i + 2 * stride], e = p[i + 3 * stride];
    d0 ^= a.x ^ a.y;
    d1 ^= b.x ^ b.y;
    d2 ^= c.x ^ c.y;
    d3 ^= e.x ^ e.y;
  }
  for (; i < m; i += stride) {
    const ulong2 a = p[i];
    d0 ^= a.x ^ a.y;
  }
  if (tid == 0) {
    if (head) d1 ^= v[0];
    if (n > head && ((n - head) & 1)) d2 ^= v[n - 1];
  }
  uint64_t d = d0 ^ d1 ^ d2 ^ d3;
  for (int off = 32; off > 0; off >>= 1) d ^= __shfl_xor(d, off, 64);
  __shared__ uint64_t part[256 / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t b = part[0] ^ part[1] ^ part[2] ^ part[3];
    if (b) atomicXor(digest, (unsigned long long)b);
  }
}

}  // namespace sa

using namespace sa;

extern "C" int sa_pcg64_find_zero(const sa_pcg64* gens, int n_gens, uint64_t n, uint64_t* first_out,
                                  void* stream) {
  if (!gens || n_gens < 0 || (n_gens > 0 && !first_out)) {
    sa_set_error("sa_pcg64_find_zero: bad arguments (n_gens=%d)", n_gens);
    return SA_ERR_ARG;
  }
  if (n == 0 || n_gens == 0) return SA_OK;
  for (int j0 = 0; j0 < n_gens; j0 += kFindMax) {
    const int cnt = n_gens - j0 < kFindMax ? n_gens - j0 : kFindMax;
    FindArgs a;
    memset(&a, 0, sizeof(a));
    for (int j = 0; j < cnt; j++) {
      a.s_lo[j] = gens[j0 + j].state.lo;
      a.s_hi[j] = gens[j0 + j].state.hi;
      a.i_lo[j] = gens[j0 + j].inc.lo;
      a.i_hi[j] = gens[j0 + j].inc.hi;
    }
    a.n = n;
    a.first = first_out + j0;
    const uint64_t blocks = (n + 255) / 256 < (uint64_t)kRejBlocks ? (n + 255) / 256 : (uint64_t)kRejBlocks;
    hipLaunchKernelGGL(k_find_zero, dim3((unsigned)blocks, cnt), dim3(256), 0, (hipStream_t)stream, a);
    SA_HIP_CHECK(hipGetLastError());
  }
  return SA_OK;
}

extern "C" int sa_stream_shift(uint64_t* out, uint64_t n, const sa_pcg64* gen, int sign, uint64_t k,
                               uint64_t shift, void* stream) {
  if (!out || !gen || (sign != 1 && sign != -1) || shift < 1) {
    sa_set_error("sa_stream_shift: bad arguments (sign=%d shift=%llu)", sign, (unsigned long long)shift);
    return SA_ERR_ARG;
  }
  if (k >= n) return SA_OK;
  const uint64_t m = n - k;
  const uint64_t blocks = (m + 255) / 256 < (uint64_t)kRejBlocks ? (m + 255) / 256 : (uint64_t)kRejBlocks;
  hipLaunchKernelGGL(k_stream_shift, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, out, n, k, shift,
                     gen->state.lo, gen->state.hi, gen->inc.lo, gen->inc.hi, sign);
  SA_HIP_CHECK(hipGetLastError());
  return SA_OK;
}

extern "C" int sa_xor_u64(const uint64_t* v, uint64_t n, uint64_t* digest, void* stream) {
  if (!v || !digest) {
    sa_set_error("sa_xor_u64: bad arguments");
    return SA_ERR_ARG;
  }
  if (n == 0) return SA_OK;
  // 4 blocks per CU: enough 16-byte loads in flight for HBM, few atomics
  const uint64_t blocks = (n + 511) / 512 < 1024 ? (n + 511) / 512 : 1024;
  hipLaunchKernelGGL(k_xor_u64, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, v, n,
                     (unsigned long long*)digest);
  SA_HIP_CHECK(hipGetLastError());
  return SA_OK;
}
