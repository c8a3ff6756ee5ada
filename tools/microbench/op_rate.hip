// Microbenchmark: issue cost (cycles per wave instruction per SIMD) of the
// 64-bit add forms the draw can use on gfx950 -- the v_add_co/v_addc pair the
// current asm emits, V_LSHL_ADD_U64 (one VOP3 64-bit add), V_ADD_U32 and
// V_MAD_U64_U32 for reference.  8 independent chains per lane, 8 waves per
// SIMD, 16 instructions per asm block.  Standalone tool; not the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 op_rate.hip -o op_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

// op 0: v_add_co_u32 + v_addc_co_u32 (2 instructions per 64-bit add)
// op 1: v_lshl_add_u64 (1 instruction per 64-bit add)
// op 2: v_add_u32 (1 instruction, 32-bit)
// op 3: v_mad_u64_u32 (1 instruction)
// op 4: raw==0 check of two draws as two v_cmp_eq_u64 into SGPR pairs + two
//       s_or_b64 into a wave-uniform accumulator (2 VALU + 2 SALU per 2 checks)
// op 5: the same check as the draw does it: two v_bitop3 + one v_min3
//       (3 VALU per 2 checks)
template <int OP>
__global__ void __launch_bounds__(256) k_op(uint64_t* out, int iters, uint64_t seed) {
  uint64_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
           a6 = a0 * 17, a7 = a0 * 19;
  const uint64_t b = seed ^ 0x9E3779B97F4A7C15ull;
  uint64_t zacc = 0;
  uint32_t zmin = 0xFFFFFFFFu;
  for (int it = 0; it < iters; it++) {
    if constexpr (OP == 0) {
#define ADDC(i)                                                                        \
  asm volatile("v_add_co_u32_e32 %0, vcc, %0, %2\n\tv_addc_co_u32_e32 %1, vcc, %1, %3, vcc" \
               : "+v"(((uint32_t*)&a##i)[0]), "+v"(((uint32_t*)&a##i)[1])               \
               : "v"((uint32_t)b), "v"((uint32_t)(b >> 32))                              \
               : "vcc");
      R8(ADDC) R8(ADDC)
    } else if constexpr (OP == 1) {
#define LSHLADD(i) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(a##i) : "v"(b));
      R8(LSHLADD) R8(LSHLADD)
    } else if constexpr (OP == 2) {
#define ADD32(i) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(((uint32_t*)&a##i)[0]) : "v"((uint32_t)b));
      R8(ADD32) R8(ADD32)
    } else if constexpr (OP == 4) {
#define ZCMP(i)                                                                              \
  asm volatile("v_cmp_eq_u64_e64 s[0:1], %1, %2\n\tv_cmp_eq_u64_e64 s[2:3], %1, %3\n\t"       \
               "s_or_b64 %0, %0, s[0:1]\n\ts_or_b64 %0, %0, s[2:3]"                            \
               : "+s"(zacc) : "s"(b), "v"(a##i), "v"(a0) : "s0", "s1", "s2", "s3", "scc");
      R8(ZCMP)
    } else if constexpr (OP == 5) {
#define ZMIN(i)                                                                              \
  asm volatile("v_bitop3_b32 v40, %1, %2, %5 bitop3:0x7e\n\tv_bitop3_b32 v41, %3, %4, %5 bitop3:0x7e\n\t" \
               "v_min3_u32 %0, %0, v40, v41"                                                 \
               : "+v"(zmin) : "v"((uint32_t)a##i), "v"((uint32_t)(a##i >> 32)), "v"((uint32_t)a0), \
                 "v"((uint32_t)(a0 >> 32)), "s"((uint32_t)b) : "v40", "v41");
      R8(ZMIN)
    } else {
#define MAD(i)                                                                        \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a##i) : "v"((uint32_t)b), \
               "v"((uint32_t)(b >> 32)) : "s0", "s1");
      R8(MAD) R8(MAD)
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ zacc ^ zmin;
}

template <int OP>
int run(const char* name, int instr_per_block, uint64_t* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  k_op<OP><<<blocks, 256>>>(out, iters, 1);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  k_op<OP><<<blocks, 256>>>(out, iters, 1);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  int clk_khz;
  CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const double waves = blocks * 4.0;
  const double winstr = waves * iters * instr_per_block;  // wave instructions
  const double simds = 256.0 * 4;
  const double cyc = (ms * 1e-3) * clk_khz * 1e3;          // cycles at the reported peak clock
  fflush(stdout);
  printf("%-28s %8.3f ms  %6.2f cycles per wave instruction per SIMD (clock %d MHz)\n", name, ms,
         cyc / (winstr / simds), clk_khz / 1000);
  return 0;
}

int main() {
  const int blocks = 2048, iters = 20000;  // 8 waves per SIMD
  uint64_t* out;
  CHECK(hipMalloc(&out, blocks * 256 * sizeof(uint64_t)));
  if (run<0>("add_co+addc (2 instr/add)", 32, out, blocks, iters)) return 1;
  if (run<1>("v_lshl_add_u64", 16, out, blocks, iters)) return 1;
  if (run<2>("v_add_u32", 16, out, blocks, iters)) return 1;
  if (run<3>("v_mad_u64_u32", 16, out, blocks, iters)) return 1;
  // per pair of checks: 2 VALU (op 4) vs 3 VALU (op 5); 8 pairs per block
  if (run<4>("zero check: 2 v_cmp_u64 + 2 s_or (per VALU)", 16, out, blocks, iters)) return 1;
  if (run<5>("zero check: 2 bitop3 + min3 (per VALU)", 24, out, blocks, iters)) return 1;
  if (run<0>("add_co+addc (again)", 32, out, blocks, iters)) return 1;
  if (run<1>("v_lshl_add_u64 (again)", 16, out, blocks, iters)) return 1;
  CHECK(hipFree(out));
  return 0;
}
