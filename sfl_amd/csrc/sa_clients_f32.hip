// sa_clients_f32.hip — fp32 instantiations of the masking kernel: the
// single-client path (1 client, 0..16 streams per pass) and the fused
// co-located-client shapes used by the benches (C clients over W GPUs:
// L = C/W local clients, X = C - L cross streams each).
#include "sa_clients_impl.h"
#include "sa_registry.h"

namespace sa {

LaunchFn find_other_kernel(int xt, int ct, int L, int X);

#define F32(L, X) SA_ENTRY(float, float, SA_F32, SA_F32, L, X)
#define L1(X) SA_ENTRY_K(float, float, SA_F32, SA_F32, 1, X, kLean1)
#define SO(L, X) SA_ENTRY_K(float, float, SA_F32, SA_F32, L, X, kSumOnly)
#define XO(X) SA_ENTRY_K(float, float, SA_F32, SA_F32, 1, X, kLean1 | kSumOnly | kCrossOnly)
LaunchFn find_clients_kernel(int xt, int ct, int L, int X, int K) {
  static const KernelEntry kEntriesF32[] = {
    F32(1, 0),  F32(1, 1),  F32(1, 2),  F32(1, 3),  F32(1, 4),  F32(1, 5),  F32(1, 6),
    F32(1, 7),  F32(1, 8),  F32(1, 9),  F32(1, 10), F32(1, 11), F32(1, 12), F32(1, 13),
    F32(1, 14), F32(1, 15), F32(1, 16),
    // fused: C clients on one GPU
    F32(2, 0), F32(3, 0), F32(4, 0), F32(5, 0), F32(6, 0), F32(7, 0), F32(8, 0),
    // fused: C = 8 over W = 2 / 4 GPUs, C = 4 over 2 GPUs
    F32(4, 4), F32(2, 6), F32(2, 2),
    // the pair-shared schedule of more than 8 co-located clients: two quads'
    // 16 cross pairs per launch (sa_fused_bipartite)
    SA_ENTRY_K(float, float, SA_F32, SA_F32, 8, 0, kBipartite),
    // sum-only fused launches (no digests / wire images): the co-located and
    // per-rank shapes above
    SO(2, 0), SO(3, 0), SO(4, 0), SO(5, 0), SO(6, 0), SO(7, 0), SO(8, 0), SO(4, 4), SO(2, 6), SO(2, 2),
    SA_ENTRY_K(float, float, SA_F32, SA_F32, 1, 1, kLean1 | kSumOnly),
    SA_ENTRY_K(float, float, SA_F32, SA_F32, 1, 3, kLean1 | kSumOnly),
    SA_ENTRY_K(float, float, SA_F32, SA_F32, 1, 7, kLean1 | kSumOnly),
    // masks only, one accumulator of one-sided streams added into the sum:
    // the later launches of sa_fused_clients' multi-launch schedule
    // (kCrossCounts)
    XO(1), XO(2), XO(4), XO(8), XO(16), XO(24), XO(32),
    // one client without the general paths (continue, weight vectors, DP)
    L1(0), L1(1), L1(2), L1(3), L1(4), L1(5), L1(6), L1(7), L1(8), L1(9), L1(10), L1(11), L1(12),
    L1(13), L1(14), L1(15), L1(16),
  };
  for (const KernelEntry& e : kEntriesF32)
    if (e.xt == xt && e.ct == ct && e.L == L && e.X == X && e.K == K) return e.fn;
  return K == kAllPairs ? find_other_kernel(xt, ct, L, X) : nullptr;
}
#undef F32
#undef L1
#undef SO
#undef XO

}  // namespace sa

#ifdef SA_TIMING
// Tuning-only: the wave timeline of the last fp32 masking launch (this TU's
// kernels), kTsWaves x kTsWords u64, zeroed by reset.
extern "C" int sa_debug_timeline(uint64_t* host_out, int reset) {
  using sa::g_sa_ts;
  const size_t bytes = sizeof(g_sa_ts);
  if (reset) {
    static uint64_t zeros[sa::kTsWaves][sa::kTsWords];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_sa_ts), zeros, bytes) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_sa_ts), bytes) == hipSuccess ? 0 : -1;
}
#endif
