// sa_internal.h — shared declarations for the libsfl_sa translation units.
#pragma once
#include <stdint.h>

void sa_set_error(const char* fmt, ...);

struct sa_mask_stream;
struct sa_dp;
// sa_mask with an optional fused GaussianModelDP pre-step (sa_api.hip)
int sa_mask_impl(const void* x, int x_type, int compute_type, uint64_t n, double weight, const void* weight_vec,
                 int fxp_bits, const struct sa_mask_stream* streams, int n_streams, uint64_t* out,
                 uint64_t* sum_accum, uint64_t* digest, uint32_t* flags, void* stream, const struct sa_dp* dp);

#define SA_HIP_CHECK(expr)                                                              \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      sa_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return SA_ERR_HIP;                                                                \
    }                                                                                   \
  } while (0)

// SA_HIP_CHECK for calls made after a blocking entry has enqueued work that
// reads the caller's scratch: on failure it drains the stream first
// (hipStreamSynchronize, its own result ignored), so the caller may reuse or
// free the scratch as soon as the entry returns.
#define SA_HIP_CHECK_DRAIN(s_, expr)                                                     \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      sa_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      (void)hipStreamSynchronize(s_);                                                   \
      return SA_ERR_HIP;                                                                \
    }                                                                                   \
  } while (0)

namespace sa {

constexpr int kMaxLocal = 8;     // co-located clients per fused launch
constexpr int kMaxStreams = 32;  // mask streams per launch (kernel-arg resident)
constexpr int kMaskPass = 16;    // streams per pass of the single-client kernel
constexpr int kBipartiteClients = 8;  // sa_fused_bipartite: two quads, their 16 cross pairs

// Pair set / variant of a masking-kernel instantiation (k_clients' K): every
// internal pair of its L clients; the pairs between the lower and the upper
// half (sa_fused_bipartite); or one client without the general paths.
constexpr int kAllPairs = 0;
constexpr int kBipartite = 1;
// kLean1: one client (L = 1) without the general single-client paths
// (continue mode, per-element weights, the DP pre-step): the fused per-rank
// shape <1, X> and first-pass sa_mask of float32 data with a scalar weight;
// 76 instead of 81 VGPRs for 7 streams and ~8 % less time per launch
// (profiles/r02/ab_lean1_kb.jsonl).  Pairs: as kAllPairs (none for L = 1).
constexpr int kLean1 = 2;
// kSumOnly: only the masked sum leaves the launch (no per-client digests, no
// wire images): the same arithmetic without the digest / store code; the
// fused launches of the benches and of the many-client schedule.  8-client
// launch -1.25 % in A/B (profiles/r02/ab_sum_only_kernel_kb.jsonl).  Flags
// combine (kLean1 | kSumOnly); kBipartite launches are masks-only sums.
constexpr int kSumOnly = 4;
// kCrossOnly: one accumulator (L = 1) of one-sided streams, masks only (no
// input loads, no quantize), added into the sum: the later launches of a
// per-rank shape with more streams than one launch holds (sa_fused_clients'
// multi-launch schedule, e.g. 4 local clients + 28 cross streams each at 32
// clients over 8 GPUs).  Used as kLean1 | kSumOnly | kCrossOnly.
constexpr int kCrossOnly = 8;
// the stream counts instantiated for kCrossOnly (sa_clients_f32.hip), largest
// first: a schedule takes the largest that fits its remaining streams, so any
// count is covered (the per-rank shapes of the benches by the first three)
constexpr int kCrossCounts[] = {32, 24, 16, 8, 4, 2, 1};


// Kernel-argument image (lives in the kernarg segment; read with scalar loads).
struct StreamArg {
  uint64_t s_lo, s_hi;      // generator state before draw 0 of this call
  uint64_t inc_lo, inc_hi;  // PCG64 increment
  uint64_t cj_lo, cj_hi;    // inc * G_J: constant part of the per-tile jump
  uint64_t smask;           // 0 (stream added) or ~0 (stream subtracted)
  uint64_t pad;
  // the draw's addends (filled by the launcher): inc_lo's and cj_lo's two
  // 32-bit words, zero-extended
  uint64_t inc_w0, inc_w1, cj_w0, cj_w1;
};

struct ClientArg {
  const void* x;         // input vector (XT); may be null in continue mode
  const void* wvec;      // optional per-element weights (CT)
  uint64_t* masked_out;  // optional masked vector out (required in continue mode)
  double w;              // scalar weight
  uint64_t bias;         // sum of the folded +/- mask offsets (see sa_kernels.hip)
  float ws[2];           // (float)w * 2^fxp twice, rounded once on the host: the fp32 fast
                         // path's packed scale (one SGPR pair for v_pk_mul_f32)
};

struct KArgs {
  ClientArg c[kMaxLocal];
  StreamArg s[kMaxStreams];
  uint64_t n;
  uint64_t aj_lo, aj_hi;    // A^J, J = grid stride - 1 (merged tile jump)
  uint64_t aji_lo, aji_hi;  // (A^J)^-1 mod 2^128 (prologue: park states one jump back)
  uint64_t* sum_out;
  uint64_t* digests;
  uint32_t* flags;
  double scale_d;  // 2^fxp
  float scale_f;
  int32_t fxp_bits;
  int32_t sum_mode;       // 0 none, 1 store, 2 accumulate
  int32_t continue_mode;  // acc starts from masked_out instead of quantize(x)
  int32_t do_digest;
  // bit c set iff c[c].masked_out is non-null (filled by the launcher): the
  // tile's finish tests one SGPR instead of loading every client's pointer
  uint32_t masked_mask;
  // GaussianModelDP pre-step fused into quantize (single-client fp32 only)
  int32_t dp_on;
  float dp_sigma, dp_updates, dp_inv;  // dp_inv: exact_recip_pow2(dp_updates) or 0
  double dp_clip;                      // python float: the reference divides by it in float64
  const double* dp_sumsq;
  const double* dp_sumsq_layer;
  uint64_t dp_key, dp_block0;  // Philox key; counter block of element 0
};

static_assert(sizeof(KArgs) <= 4096, "kernel arguments must fit the 4 KiB kernarg segment");

typedef int (*LaunchFn)(const KArgs& a, void* stream);

// Returns the launcher for (xt, ct, L, X) or nullptr when not instantiated.
// K: pair set of the launch (0: every internal pair of the L clients; 1:
// bipartite, the pairs between the lower and upper half -- sa_fused_bipartite)
LaunchFn find_clients_kernel(int xt, int ct, int L, int X, int K = kAllPairs);

}  // namespace sa
