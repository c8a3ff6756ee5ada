// pcg128.h — 128-bit LCG algebra for numpy's PCG64 (XSL-RR 128/64), usable on
// host and device and in constant expressions.
//
// numpy's PCG64 (numpy/random/src/pcg64/pcg64.h, the generator the reference
// names in docs/developer/algorithm/secure_aggregation.ipynb cell 15) steps
//     s <- s * A + inc   (mod 2^128),  A = 0x2360ED051FC65DA4_4385DF649FCCF645
// and emits rotr64(hi(s) ^ lo(s), hi(s) >> 58) of the NEW state.  Because the
// step is affine, k steps are s <- A^k s + inc * G_k with G_k = sum_{j<k} A^j,
// so any element of a mask stream is reachable in O(log k) (jump-ahead) and a
// GPU lane can start its stream at its own element with no inter-lane state.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SA_HD __host__ __device__
#else
#define SA_HD
#endif

namespace sa {

typedef unsigned __int128 u128;

constexpr u128 mk128(uint64_t hi, uint64_t lo) { return ((u128)hi << 64) | lo; }
constexpr uint64_t lo64(u128 x) { return (uint64_t)x; }
constexpr uint64_t hi64(u128 x) { return (uint64_t)(x >> 64); }

constexpr u128 kPcgMult = mk128(0x2360ED051FC65DA4ULL, 0x4385DF649FCCF645ULL);
// Generator.integers(int64.min, int64.max) == raw + kMaskOffset (mod 2^64)
// (numpy Lemire bounded draw with rng = 2^64-2; raw == 0 is rejected).
constexpr uint64_t kMaskOffset = 0x7FFFFFFFFFFFFFFFULL;

// An affine jump: s -> mult * s + plus_unit * inc.  `plus_unit` (= G_k) is
// independent of the stream's increment, so one table serves every stream.
struct Jump {
  u128 mult;  // A^k
  u128 gsum;  // G_k = sum_{j<k} A^j
};

// compose: first apply `a`, then `b`   (b ∘ a)
SA_HD constexpr Jump compose(Jump a, Jump b) {
  return Jump{b.mult * a.mult, b.mult * a.gsum + b.gsum};
}

SA_HD constexpr Jump jump_of(uint64_t k_lo, uint64_t k_hi = 0) {
  Jump acc{1, 0};
  Jump cur{kPcgMult, 1};
  u128 k = mk128(k_hi, k_lo);
  while (k) {
    if (k & 1) acc = compose(acc, cur);
    cur = compose(cur, cur);
    k >>= 1;
  }
  return acc;
}

SA_HD constexpr u128 apply(Jump j, u128 s, u128 inc) { return j.mult * s + j.gsum * inc; }

SA_HD constexpr uint64_t rotr64(uint64_t x, unsigned r) {
  return (x >> (r & 63)) | (x << ((64 - r) & 63));
}
SA_HD constexpr uint64_t xslrr(u128 s) { return rotr64(hi64(s) ^ lo64(s), (unsigned)(hi64(s) >> 58)); }

// inverse of an odd value mod 2^128 (Newton: x <- x(2 - a x) doubles the
// correct low bits; a*a == 1 mod 8 for odd a, so 6 steps reach 192 > 128)
SA_HD constexpr u128 inv128(u128 a) {
  u128 x = a;
  for (int i = 0; i < 6; i++) x *= (u128)2 - a * x;
  return x;
}

constexpr int kBlockThreads = 256;  // masking-kernel workgroup
constexpr int kDpBlock = 4;         // elements per Philox counter block (DP noise)

}  // namespace sa
