// Issue cost on gfx950 of every instruction form the PCG64 pair draw uses
// (sa_draw2.h), as the draw writes it: VOP3 forms with SGPR carry-outs,
// SGPR carry-ins, SGPR lane masks.  8 independent chains per lane, 16
// instructions per asm block, 8 waves per SIMD (2048 blocks of 256 on 256
// CUs), so the figure is the SIMD's issue throughput for that form, not a
// latency.  DESIGN.md §4's feasibility bound multiplies these by the draw's
// instruction counts.  Prints one JSON line per form: cycles per wave
// instruction per SIMD at the clock the run held (measured with
// s_memrealtime / s_memtime over the launch: no assumed clock).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 draw_ops.hip -o draw_ops
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <utility>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

enum {
  kMadS,      // v_mad_u64_u32 v[..], s[..], v, v, s[..]  (SGPR carry-out, SGPR 64-bit addend)
  kMadV,      // v_mad_u64_u32 v[..], s[..], v, v, v[..]  (VGPR addend)
  kMulLo,     // v_mul_lo_u32
  kAddCo,     // v_add_co_u32_e64 v, s[..], v, v
  kAddc,      // v_addc_co_u32_e64 v, s[..], v, v, s[..]
  kBitop3,    // v_bitop3_b32 v, v, v, s
  kCmp,       // v_cmp_gt_i32_e64 s[..], 0, v
  kLshr,      // v_lshrrev_b32_e32
  kAlignbit,  // v_alignbit_b32
  kCndmask,   // v_cndmask_b32_e64 v, v, v, s[..]
  kMin3,      // v_min3_u32
  kLshlAdd,   // v_lshl_add_u64 v[..], v[..], 0, v[..]
  kSubCo,     // v_sub_co_u32_e64 v, s[..], v, v
  kSubb,      // v_subb_co_u32_e64 v, s[..], v, v, s[..]
  kAdd32,     // v_add_u32_e32 (the full-rate reference)
  kCmp32,     // v_cmp_gt_i32_e32 vcc, 0, v
  kCndmask32, // v_cndmask_b32_e32 v, v, v, vcc
  kOr32,      // v_or_b32_e32 (the 64-bit-shift rotation's halves)
  kSubK,      // v_sub_u32_e32 v, 64, v (its 64 - r)
  kLshr64,    // v_lshrrev_b64 v[..], v, v[..]
  kLshl64,    // v_lshlrev_b64 v[..], v, v[..]
  kXorK,      // v_xor_b32_e32 v, 63, v (the shift-rotation form's 63 - r)
  kLshlAdd1,  // v_lshl_add_u64 v[..], v[..], 1, v[..] (its join of the two shifted parts)
  kCmpEq64,   // v_cmp_eq_u64_e32 vcc, s[..], v[..] (its raw == 0 test)
  kCmpEq64Or, // the same compare + s_or_b64 of the lane mask into an SGPR accumulator
  kNumOps
};
static const char* kNames[kNumOps] = {
    "v_mad_u64_u32 (sgpr addend)", "v_mad_u64_u32 (vgpr addend)", "v_mul_lo_u32", "v_add_co_u32_e64",
    "v_addc_co_u32_e64", "v_bitop3_b32", "v_cmp_gt_i32_e64", "v_lshrrev_b32", "v_alignbit_b32",
    "v_cndmask_b32_e64", "v_min3_u32", "v_lshl_add_u64", "v_sub_co_u32_e64", "v_subb_co_u32_e64",
    "v_add_u32_e32", "v_cmp_gt_i32_e32", "v_cndmask_b32_e32", "v_or_b32_e32", "v_sub_u32_e32 (64 - v)",
    "v_lshrrev_b64", "v_lshlrev_b64", "v_xor_b32_e32 (63 ^ v)", "v_lshl_add_u64 (shift 1)",
    "v_cmp_eq_u64_e32", "v_cmp_eq_u64_e32 + s_or_b64"};

template <int OP>
__global__ void __launch_bounds__(256) k_op(uint64_t* out, unsigned long long* clk, int iters, uint64_t seed) {
  uint64_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
           a6 = a0 * 17, a7 = a0 * 19;
  const uint64_t b = seed ^ 0x9E3779B97F4A7C15ull;
  const uint32_t bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
  uint64_t t0 = 0, c0 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0));
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
  }
  for (int it = 0; it < iters; it++) {
#define LO(i) (((uint32_t*)&a##i)[0])
#define HI(i) (((uint32_t*)&a##i)[1])
    if constexpr (OP == kMadS) {
#define X(i) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %3" : "+v"(a##i) : "v"(bl), "v"(bh), "s"(b) : "s40", "s41");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kMadV) {
#define X(i) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a##i) : "v"(bl), "v"(bh) : "s40", "s41");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kMulLo) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(LO(i)) : "v"(bl));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kAddCo) {
#define X(i) asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %1" : "+v"(LO(i)) : "v"(bl) : "s40", "s41");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kAddc) {
#define X(i) asm volatile("v_addc_co_u32_e64 %0, s[40:41], %0, %1, s[42:43]" : "+v"(LO(i)) : "v"(bl) : "s40", "s41");
      asm volatile("s_mov_b64 s[42:43], 0" ::: "s42", "s43");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kBitop3) {
#define X(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(LO(i)) : "v"(HI(i)), "s"(bl));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kCmp) {
#define X(i) asm volatile("v_cmp_gt_i32_e64 s[%c1:%c2], 0, %0" : : "v"(LO(i)), "i"(40 + 2 * (i)), "i"(41 + 2 * (i)) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kLshr) {
#define X(i) asm volatile("v_lshrrev_b32_e32 %0, 26, %0" : "+v"(LO(i)));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kAlignbit) {
#define X(i) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(LO(i)) : "v"(HI(i)), "v"(bl));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kCndmask) {
#define X(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(LO(i)) : "v"(HI(i)) : "s40", "s41");
      asm volatile("s_mov_b64 s[40:41], 0x5555" ::: "s40", "s41");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kMin3) {
#define X(i) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(LO(i)) : "v"(HI(i)), "v"(bl));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kLshlAdd) {
#define X(i) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(a##i) : "v"(b));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kSubCo) {
#define X(i) asm volatile("v_sub_co_u32_e64 %0, s[40:41], %0, %1" : "+v"(LO(i)) : "v"(bl) : "s40", "s41");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kSubb) {
#define X(i) asm volatile("v_subb_co_u32_e64 %0, s[40:41], %0, %1, s[42:43]" : "+v"(LO(i)) : "v"(bl) : "s40", "s41");
      asm volatile("s_mov_b64 s[42:43], 0" ::: "s42", "s43");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kCmp32) {
#define X(i) asm volatile("v_cmp_gt_i32_e32 vcc, 0, %0" : : "v"(LO(i)) : "vcc");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kCndmask32) {
#define X(i) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(LO(i)) : "v"(HI(i)) : "vcc");
      asm volatile("s_mov_b64 vcc, 0x5555" ::: "vcc");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kOr32) {
#define X(i) asm volatile("v_or_b32_e32 %0, %0, %1" : "+v"(LO(i)) : "v"(HI(i)));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kSubK) {
#define X(i) asm volatile("v_sub_u32_e32 %0, 64, %0" : "+v"(LO(i)));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kLshr64) {
#define X(i) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(a##i) : "v"(bl));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kLshl64) {
#define X(i) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(a##i) : "v"(bl));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kXorK) {
#define X(i) asm volatile("v_xor_b32_e32 %0, 63, %0" : "+v"(LO(i)));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kLshlAdd1) {
#define X(i) asm volatile("v_lshl_add_u64 %0, %1, 1, %0" : "+v"(a##i) : "v"(b));
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kCmpEq64) {
#define X(i) asm volatile("v_cmp_eq_u64_e32 vcc, %1, %0" : : "v"(a##i), "s"(b) : "vcc");
      R8(X) R8(X)
#undef X
    } else if constexpr (OP == kCmpEq64Or) {
      // per compare one SALU OR, as in the draw (counted as one wave instruction)
#define X(i) asm volatile("v_cmp_eq_u64_e32 vcc, %1, %0\n\ts_or_b64 s[40:41], s[40:41], vcc" : : "v"(a##i), "s"(b) : "vcc", "scc", "s40", "s41");
      asm volatile("s_mov_b64 s[40:41], 0" ::: "s40", "s41");
      R8(X) R8(X)
#undef X
    } else {
#define X(i) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(LO(i)) : "v"(bl));
      R8(X) R8(X)
#undef X
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    uint64_t t1, c1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0" : "=s"(c1));
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    clk[0] = c1 - c0;  // shader clock cycles over block 0's life
    clk[1] = t1 - t0;  // 100 MHz ticks over the same span
  }
}

template <int OP>
int run(uint64_t* out, unsigned long long* dclk, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; w++) k_op<OP><<<blocks, 256>>>(out, dclk, iters, 1);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  k_op<OP><<<blocks, 256>>>(out, dclk, iters, 1);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CHECK(hipMemcpy(h, dclk, sizeof(h), hipMemcpyDeviceToHost));
  const double mhz = h[1] ? (double)h[0] / ((double)h[1] / 100.0) : 0.0;  // s_memtime / (ticks at 100 MHz)
  const double winstr = blocks * 4.0 * iters * 16;                        // wave instructions
  const double per_simd = winstr / (256.0 * 4);
  const double cyc = ms * 1e-3 * mhz * 1e6;
  printf("{\"op\": \"%s\", \"ms\": %.4f, \"clock_mhz\": %.0f, \"cycles_per_wave_instr\": %.3f}\n", kNames[OP], ms,
         mhz, cyc / per_simd);
  fflush(stdout);
  return 0;
}

template <int... OPS>
int run_all(uint64_t* out, unsigned long long* dclk, int blocks, int iters, std::integer_sequence<int, OPS...>) {
  int rc = 0;
  ((rc = rc ? rc : run<OPS>(out, dclk, blocks, iters)), ...);
  return rc;
}

int main() {
  const int blocks = 2048, iters = 20000;  // 8 waves per SIMD
  uint64_t* out;
  unsigned long long* dclk;
  CHECK(hipMalloc(&out, blocks * 256 * sizeof(uint64_t)));
  CHECK(hipMalloc(&dclk, 2 * sizeof(unsigned long long)));
  if (run_all(out, dclk, blocks, iters, std::make_integer_sequence<int, kNumOps>{})) return 1;
  CHECK(hipFree(out));
  return 0;
}
