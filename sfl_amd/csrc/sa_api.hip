// sa_api.hip — extern "C" entry points of libsfl_sa.so (see include/sfl_sa.h)
// plus the two HBM-streaming server kernels (masked-vector sum, decode).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <unordered_map>

#include "../../include/sfl_sa.h"
#include "pcg128.h"
#include "sa_internal.h"
#include "sa_tiles.h"
#include "sa_philox.h"

namespace sa {

// CUs' worth of the masking kernel's blocks left free for kernels on other
// streams (sa_set_masking_reserve); 0: the masking grid fills the GPU
static std::atomic<int> g_masking_reserve{0};

int occupancy_blocks(const void* kernel);

int masking_grid_cap(const void* kernel) {
  const int maxb = occupancy_blocks(kernel);
  const int reserve = g_masking_reserve.load(std::memory_order_relaxed);
  if (maxb <= 0 || reserve <= 0) return maxb;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
    sa_set_error("occupancy query failed");
    return -1;
  }
  const int keep = maxb - (maxb / cus) * reserve;
  return keep > maxb / 2 ? keep : maxb / 2;
}

int occupancy_blocks(const void* kernel) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> g(mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    sa_set_error("hipGetDevice failed");
    return -1;
  }
  const void* key = (const void*)((uintptr_t)kernel ^ ((uintptr_t)dev << 56));
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlockThreads, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    sa_set_error("occupancy query failed");
    return -1;
  }
  if (per_cu < 1) per_cu = 1;
  const int blocks = per_cu * cus;
  cache[key] = blocks;
  return blocks;
}

// ---------------------------------------------------------------------------
// The server kernels stream HBM: 16-B accesses (two 8-B elements per lane and
// access), one tile of 256 x kUnroll accesses per block over a grid that
// covers the vector (no grid-stride loop), non-temporal loads and stores (the
// vectors are read once and written once).  tools/microbench/stream_rate.hip
// measured these choices on MI355X (profiles/r03/stream_rate.jsonl): copy
// 6.38 TB/s, two inputs 6.42, eight inputs 6.20, against 4.9-5.6 TB/s for an
// occupancy-sized grid-stride loop with default-policy accesses.  An odd last
// element is done by one lane of block 0.
// ---------------------------------------------------------------------------
constexpr int kUnroll = 4;
constexpr int kTileAccesses = 256 * kUnroll;  // 16-B accesses per block and input

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
  return __builtin_nontemporal_load(p);
}
template <typename T>
__device__ __forceinline__ void st_nt(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

// server sum: out = sum_k in[k]  (mod 2^64)
constexpr int kSumMaxIn = 32;
struct SumArgs {
  const uint64_t* in[kSumMaxIn];
  uint64_t* out;
  uint64_t n;
  int k;
};

__global__ void __launch_bounds__(256) k_sum_u64(const SumArgs a) {
  const uint64_t n2 = a.n / 2;
  const uint64_t base = (uint64_t)stream_tile() * kTileAccesses + threadIdx.x;
  u64x2 s[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; u++)
    s[u] = base + u * 256 < n2 ? ld_nt(reinterpret_cast<const u64x2*>(a.in[0]) + base + u * 256) : u64x2{0, 0};
  for (int j = 1; j < a.k; j++) {
    const u64x2* in = reinterpret_cast<const u64x2*>(a.in[j]);
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
      if (base + u * 256 < n2) s[u] += ld_nt(in + base + u * 256);
  }
#pragma unroll
  for (int u = 0; u < kUnroll; u++)
    if (base + u * 256 < n2) st_nt(reinterpret_cast<u64x2*>(a.out) + base + u * 256, s[u]);
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t t = 0;
    for (int j = 0; j < a.k; j++) t += a.in[j][a.n - 1];
    a.out[a.n - 1] = t;
  }
}

// decode: out = (double)(int64)s / 2^fxp / div
__device__ __forceinline__ double decode1(uint64_t s, double inv_scale, double div) {
  const double v = (double)(long long)s * inv_scale;  // exact power-of-two scaling
  return v / div;                                     // IEEE division
}

// s, out (and divv) 16-B aligned
template <bool kVec>
__global__ void __launch_bounds__(256) k_decode(const uint64_t* __restrict__ s, uint64_t n, double inv_scale,
                                                double div, const double* __restrict__ divv,
                                                double* __restrict__ out) {
  const uint64_t n2 = n / 2;
  const uint64_t base = (uint64_t)stream_tile() * kTileAccesses + threadIdx.x;
  const u64x2* s2 = reinterpret_cast<const u64x2*>(s);
  const f64x2* d2 = reinterpret_cast<const f64x2*>(divv);
  f64x2* o2 = reinterpret_cast<f64x2*>(out);
  u64x2 v[kUnroll];
  f64x2 d[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; u++) {
    const bool in = base + u * 256 < n2;
    v[u] = in ? ld_nt(s2 + base + u * 256) : u64x2{0, 0};
    if (kVec) d[u] = in ? ld_nt(d2 + base + u * 256) : f64x2{1.0, 1.0};
  }
#pragma unroll
  for (int u = 0; u < kUnroll; u++)
    if (base + u * 256 < n2)
      st_nt(o2 + base + u * 256, f64x2{decode1(v[u].x, inv_scale, kVec ? d[u].x : div),
                                       decode1(v[u].y, inv_scale, kVec ? d[u].y : div)});
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
    out[n - 1] = decode1(s[n - 1], inv_scale, kVec ? divv[n - 1] : div);
}

// any alignment (8-B elements one per lane): sub-vectors the caller sliced at odd offsets
__global__ void __launch_bounds__(256) k_decode_unaligned(const uint64_t* __restrict__ s, uint64_t n,
                                                          double inv_scale, double div,
                                                          const double* __restrict__ divv,
                                                          double* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = decode1(s[i], inv_scale, divv ? divv[i] : div);
}

// per-element weight sums (the average's divisor vector): out = [out +] sum_k in[k]
struct SumF64Args {
  const double* in[kSumMaxIn];
  double* out;
  uint64_t n;
  int k;
  int accumulate;
};
__global__ void __launch_bounds__(256) k_sum_f64(const SumF64Args a) {
  const uint64_t n2 = a.n / 2;
  const uint64_t base = (uint64_t)stream_tile() * kTileAccesses + threadIdx.x;
  const int j0 = a.accumulate ? 0 : 1;
  const f64x2* first = reinterpret_cast<const f64x2*>(a.accumulate ? a.out : a.in[0]);
  f64x2 s[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; u++) s[u] = base + u * 256 < n2 ? ld_nt(first + base + u * 256) : f64x2{0, 0};
  for (int j = j0; j < a.k; j++) {
    const f64x2* in = reinterpret_cast<const f64x2*>(a.in[j]);
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
      if (base + u * 256 < n2) s[u] += ld_nt(in + base + u * 256);
  }
#pragma unroll
  for (int u = 0; u < kUnroll; u++)
    if (base + u * 256 < n2) st_nt(reinterpret_cast<f64x2*>(a.out) + base + u * 256, s[u]);
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    double t = a.accumulate ? a.out[a.n - 1] : a.in[0][a.n - 1];
    for (int j = j0; j < a.k; j++) t += a.in[j][a.n - 1];
    a.out[a.n - 1] = t;
  }
}

// any alignment: one element per lane
__global__ void __launch_bounds__(256) k_sum_f64_unaligned(const SumF64Args a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    double s = a.accumulate ? a.out[i] : a.in[0][i];
    for (int j = a.accumulate ? 0 : 1; j < a.k; j++) s += a.in[j][i];
    a.out[i] = s;
  }
}

// one block per tile of kTileAccesses 16-B accesses (at least one block for
// the odd-element lane)
static int tile_grid(uint64_t n) {
  const uint64_t b = (n / 2 + kTileAccesses - 1) / kTileAccesses;
  if (b >= (1ull << 31)) {
    sa_set_error("vector of %llu elements exceeds one server-kernel launch", (unsigned long long)n);
    return -1;
  }
  return b < 1 ? 1 : (int)b;
}

static int stream_grid(uint64_t work_items, const void* kfn) {
  const int maxb = occupancy_blocks(kfn);
  if (maxb <= 0) return -1;
  const uint64_t b = (work_items + 255) / 256;
  const uint64_t cap = (uint64_t)maxb;
  return (int)(b < 1 ? 1 : (b < cap ? b : cap));
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static uint64_t fold_plus() { return kMaskOffset; }        // +m = t + K
static uint64_t fold_minus() { return 1 - kMaskOffset; }   // -m = t + (1-K), t = ~raw

}  // namespace sa

using namespace sa;

static int check_type(int t, const char* what) {
  if (t != SA_F32 && t != SA_F64 && t != SA_I64) {
    sa_set_error("%s: unknown element type %d", what, t);
    return SA_ERR_ARG;
  }
  return SA_OK;
}

static void fill_stream(StreamArg& s, const sa_pcg64& g, int sign) {
  s.s_lo = g.state.lo;
  s.s_hi = g.state.hi;
  s.inc_lo = g.inc.lo;
  s.inc_hi = g.inc.hi;
  s.cj_lo = s.cj_hi = 0;
  s.smask = sign < 0 ? ~0ULL : 0ULL;
  s.pad = 0;
}

extern "C" int sa_mask(const void* x, int x_type, int compute_type, uint64_t n, double weight,
                       const void* weight_vec, int fxp_bits, const sa_mask_stream* streams,
                       int n_streams, uint64_t* out, uint64_t* sum_accum, uint64_t* digest,
                       uint32_t* flags, void* stream) {
  return sa_mask_impl(x, x_type, compute_type, n, weight, weight_vec, fxp_bits, streams, n_streams, out,
                      sum_accum, digest, flags, stream, nullptr);
}

int sa_mask_impl(const void* x, int x_type, int compute_type, uint64_t n, double weight, const void* weight_vec,
                 int fxp_bits, const sa_mask_stream* streams, int n_streams, uint64_t* out, uint64_t* sum_accum,
                 uint64_t* digest, uint32_t* flags, void* stream, const sa_dp* dp) {
  if (check_type(x_type, "sa_mask x_type") || check_type(compute_type, "sa_mask compute_type"))
    return SA_ERR_ARG;
  if (n == 0 && n_streams >= 0 && fxp_bits >= 0 && fxp_bits <= 62) return SA_OK;  // nothing to touch
  if (!out || n_streams < 0 || (n_streams > 0 && !streams) || fxp_bits < 0 || fxp_bits > 62) {
    sa_set_error("sa_mask: bad arguments (out=%p n_streams=%d fxp_bits=%d)", (void*)out,
                 n_streams, fxp_bits);
    return SA_ERR_ARG;
  }
  if (!aligned16(x) || !aligned16(out) || !aligned16(weight_vec) || !aligned16(sum_accum)) {
    sa_set_error("sa_mask: device buffers must be 16-byte aligned");
    return SA_ERR_ARG;
  }
  if (n == 0) return SA_OK;
  // fp32 has kernels for up to 16 streams per pass, the other types 8
  const int per_pass = (x_type == SA_F32 && compute_type == SA_F32) ? kMaskPass : kMaskPass / 2;
  const int passes = n_streams == 0 ? 1 : (n_streams + per_pass - 1) / per_pass;
  for (int p = 0; p < passes; p++) {
    const int j0 = p * per_pass;
    const int cnt = n_streams - j0 < per_pass ? n_streams - j0 : per_pass;
    const bool last = p == passes - 1;
    KArgs a;
    memset(&a, 0, sizeof(a));
    a.n = n;
    a.fxp_bits = fxp_bits;
    a.scale_d = (double)((uint64_t)1 << fxp_bits);
    a.scale_f = (float)a.scale_d;
    a.continue_mode = (p > 0 || x == nullptr) ? 1 : 0;
    a.c[0].x = x;
    a.c[0].wvec = weight_vec;
    a.c[0].masked_out = out;
    a.c[0].w = weight;
    a.c[0].ws[0] = a.c[0].ws[1] = (float)weight * a.scale_f;  // IEEE single multiply, as __fmul_rn on the device
    uint64_t bias = 0;
    for (int j = 0; j < cnt; j++) {
      const sa_mask_stream& ms = streams[j0 + j];
      if (ms.sign != 1 && ms.sign != -1) {
        sa_set_error("sa_mask: stream %d has sign %d (want +1/-1)", j0 + j, ms.sign);
        return SA_ERR_ARG;
      }
      fill_stream(a.s[j], ms.gen, ms.sign);
      bias += ms.sign > 0 ? fold_plus() : fold_minus();
    }
    a.c[0].bias = bias;
    a.sum_out = last ? sum_accum : nullptr;
    a.sum_mode = (last && sum_accum) ? 2 : 0;
    a.digests = last ? digest : nullptr;
    a.do_digest = (last && digest) ? 1 : 0;
    a.flags = flags;
    if (dp) {
      a.dp_on = 1;
      a.dp_clip = dp->l2_norm_clip;
      a.dp_sigma = dp->noise_std;
      a.dp_updates = dp->num_updates;
      a.dp_inv = exact_recip_pow2(dp->num_updates);
      a.dp_sumsq = dp->sumsq;
      a.dp_sumsq_layer = dp->sumsq_layer;
      a.dp_key = dp->key;
      a.dp_block0 = dp->counter0 / 4;
    }
    const int ct = compute_type;
    // the lean single-client kernel unless a general path is needed
    // (continue mode, per-element weights, DP): float32 kernels only
    LaunchFn fn = (!a.continue_mode && !weight_vec && !dp) ? find_clients_kernel(x_type, ct, 1, cnt, kLean1)
                                                           : nullptr;
    if (!fn) fn = find_clients_kernel(x_type, ct, 1, cnt);
    if (!fn) {
      sa_set_error("sa_mask: no kernel for x_type=%d compute_type=%d streams=%d", x_type, ct, cnt);
      return SA_ERR_UNSUPPORTED;
    }
    const int rc = fn(a, stream);
    if (rc) return rc;
  }
  return SA_OK;
}

// One masks-only launch: sum_out += sum over the cnt streams of +-(raw + K)
// mod 2^64 (the kCrossOnly kernel: no input vector, nothing quantized).
static int launch_cross_group(const sa_mask_stream* ms, int cnt, uint64_t n, uint64_t* sum_out, uint32_t* flags,
                              void* stream) {
  KArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n;
  a.scale_d = 1.0;
  a.scale_f = 1.0f;
  uint64_t bias = 0;
  for (int j = 0; j < cnt; j++) {
    fill_stream(a.s[j], ms[j].gen, ms[j].sign);
    bias += ms[j].sign > 0 ? fold_plus() : fold_minus();
  }
  a.c[0].x = nullptr;  // never read: the kCrossOnly kernel loads no input
  a.c[0].bias = bias;
  a.sum_out = sum_out;
  a.sum_mode = 2;
  a.flags = flags;
  const LaunchFn fn = find_clients_kernel(SA_F32, SA_F32, 1, cnt, kLean1 | kSumOnly | kCrossOnly);
  if (!fn) {
    sa_set_error("masks-only launch: no kernel for %d streams", cnt);
    return SA_ERR_UNSUPPORTED;
  }
  return fn(a, stream);
}

// the masks-only launch sizes for `count` one-sided streams: the largest
// instantiated count (kCrossCounts) that fits the remaining streams
static int cross_launch_size(int remaining) {
  for (int c : kCrossCounts)
    if (c <= remaining) return c;
  return 1;
}

// every masks-only kernel the schedule of `count` streams needs exists
// (checked before anything is launched: see sa_fused_clients)
static bool cross_plan_instantiated(int count) {
  for (int j = 0; j < count; j += cross_launch_size(count - j))
    if (!find_clients_kernel(SA_F32, SA_F32, 1, cross_launch_size(count - j), kLean1 | kSumOnly | kCrossOnly))
      return false;
  return true;
}

// sum_out += the masks of `count` one-sided streams, in launches of the
// largest instantiated count (kCrossCounts) that fits the remaining streams.
static int launch_cross(const sa_mask_stream* ms, int count, uint64_t n, uint64_t* sum_out, uint32_t* flags,
                        void* stream) {
  for (int j = 0; j < count;) {
    const int cnt = cross_launch_size(count - j);
    const int rc = launch_cross_group(ms + j, cnt, n, sum_out, flags, stream);
    if (rc) return rc;
    j += cnt;
  }
  return SA_OK;
}

extern "C" int sa_fused_clients(const sa_local_client* clients, int n_clients, int x_type,
                                uint64_t n, int fxp_bits, const sa_pcg64* pair_gens,
                                const int8_t* pair_sign, const sa_mask_stream* cross,
                                int n_cross, uint64_t* sum_out, int accumulate,
                                uint64_t* digests, uint32_t* flags, void* stream) {
  if (check_type(x_type, "sa_fused_clients x_type")) return SA_ERR_ARG;
  const int L = n_clients;
  const int PI = L * (L - 1) / 2;
  if (n == 0 && L >= 1 && n_cross >= 0 && fxp_bits >= 0 && fxp_bits <= 62) return SA_OK;  // empty vectors
  if (!clients || L < 1 || n_cross < 0 || !sum_out || fxp_bits < 0 ||
      fxp_bits > 62 || (PI > 0 && (!pair_gens || !pair_sign)) || (n_cross > 0 && !cross)) {
    sa_set_error("sa_fused_clients: bad arguments (n_clients=%d n_cross=%d)", L, n_cross);
    return SA_ERR_ARG;
  }
  if (L > kMaxLocal) {  // valid, but one launch holds at most kMaxLocal clients' accumulators
    sa_set_error("sa_fused_clients: %d co-located clients exceed the %d per launch", L, kMaxLocal);
    return SA_ERR_UNSUPPORTED;
  }
  if (PI + L * n_cross > kMaxStreams) {
    // More streams than one launch holds (config 5 at 8 GPUs: 4 local clients,
    // 6 internal pairs + 4 x 28 cross streams).  With only the sum wanted, a
    // multi-launch schedule that still draws every internal pair ONCE: a
    // fused sum-only launch with the pairs and the first X1 cross streams of
    // every client, then masks-only launches of the remaining cross streams
    // adding into the sum (their per-client split does not matter there).
    bool any_out = digests != nullptr;
    for (int c = 0; c < L; c++) any_out = any_out || clients[c].masked_out != nullptr;
    int X1 = -1;
    if (!any_out && x_type == SA_F32)
      for (int x = n_cross - 1; x >= 0 && X1 < 0; x--)
        if (PI + L * x <= kMaxStreams && find_clients_kernel(x_type, x_type, L, x, (L == 1 ? kLean1 : 0) | kSumOnly))
          X1 = x;
    if (X1 < 0) {  // digests / wire images wanted, or no first launch: the caller masks client by client
      sa_set_error("sa_fused_clients: %d streams exceed the %d per launch", PI + L * n_cross, kMaxStreams);
      return SA_ERR_UNSUPPORTED;
    }
    for (int j = 0; j < L * n_cross; j++)
      if (cross[j].sign != 1 && cross[j].sign != -1) {
        sa_set_error("sa_fused_clients: cross stream %d sign %d", j, cross[j].sign);
        return SA_ERR_ARG;
      }
    sa_mask_stream first[kMaxStreams], rest[kMaxLocal * (kMaxStreams + 1)];
    if (L * (n_cross - X1) > (int)(sizeof(rest) / sizeof(rest[0]))) {
      sa_set_error("sa_fused_clients: %d cross streams per client exceed the multi-launch schedule", n_cross);
      return SA_ERR_UNSUPPORTED;
    }
    int nr = 0;
    for (int c = 0; c < L; c++)
      for (int j = 0; j < n_cross; j++) {
        if (j < X1)
          first[c * X1 + j] = cross[c * n_cross + j];
        else
          rest[nr++] = cross[c * n_cross + j];
      }
    // all-or-nothing: SA_ERR_UNSUPPORTED tells the caller nothing ran (it
    // then masks client by client into the same sum_out), so every kernel
    // of the schedule is looked up BEFORE the first launch, and a failure
    // after it is reported as SA_ERR_HIP (sum_out partly written)
    if (!cross_plan_instantiated(nr)) {
      sa_set_error("sa_fused_clients: no masks-only kernel for part of %d cross streams", nr);
      return SA_ERR_UNSUPPORTED;
    }
    const int rc = sa_fused_clients(clients, L, x_type, n, fxp_bits, pair_gens, pair_sign, first, X1, sum_out,
                                    accumulate, nullptr, flags, stream);
    if (rc) return rc;
    const int rc2 = n == 0 ? SA_OK : launch_cross(rest, nr, n, sum_out, flags, stream);
    if (rc2 == SA_ERR_UNSUPPORTED) {
      sa_set_error("sa_fused_clients: masks-only launch failed after the first launch (sum_out partly written)");
      return SA_ERR_HIP;
    }
    return rc2;
  }
  if (!aligned16(sum_out)) {
    sa_set_error("sa_fused_clients: sum_out must be 16-byte aligned");
    return SA_ERR_ARG;
  }
  if (n == 0) return SA_OK;
  KArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n;
  a.fxp_bits = fxp_bits;
  a.scale_d = (double)((uint64_t)1 << fxp_bits);
  a.scale_f = (float)a.scale_d;
  uint64_t bias[kMaxLocal] = {0};
  for (int c = 0; c < L; c++) {
    if (!clients[c].x || !aligned16(clients[c].x) || ((uintptr_t)clients[c].masked_out & 7)) {
      sa_set_error("sa_fused_clients: client %d x null or buffers not 16-byte aligned", c);
      return SA_ERR_ARG;
    }
    a.c[c].x = clients[c].x;
    a.c[c].wvec = nullptr;
    a.c[c].masked_out = clients[c].masked_out;
    a.c[c].w = clients[c].weight;
    a.c[c].ws[0] = a.c[c].ws[1] = (float)clients[c].weight * a.scale_f;
  }
  int p = 0;
  for (int u = 0; u < L; u++)
    for (int v = u + 1; v < L; v++, p++) {
      const int sg = pair_sign[p];
      if (sg != 1 && sg != -1) {
        sa_set_error("sa_fused_clients: pair %d sign %d", p, sg);
        return SA_ERR_ARG;
      }
      fill_stream(a.s[p], pair_gens[p], sg);
      if (sg > 0) {  // u adds m (t = raw), v subtracts: -t - K
        bias[u] += kMaskOffset;
        bias[v] += 0 - kMaskOffset;
      } else {  // t = ~raw: u gets t + (1-K) = -m; v gets -t + (K-1) = +m
        bias[u] += 1 - kMaskOffset;
        bias[v] += kMaskOffset - 1;
      }
    }
  for (int c = 0; c < L; c++)
    for (int j = 0; j < n_cross; j++) {
      const sa_mask_stream& ms = cross[c * n_cross + j];
      if (ms.sign != 1 && ms.sign != -1) {
        sa_set_error("sa_fused_clients: cross stream (%d,%d) sign %d", c, j, ms.sign);
        return SA_ERR_ARG;
      }
      fill_stream(a.s[PI + c * n_cross + j], ms.gen, ms.sign);
      bias[c] += ms.sign > 0 ? fold_plus() : fold_minus();
    }
  for (int c = 0; c < L; c++) a.c[c].bias = bias[c];
  a.sum_out = sum_out;
  a.sum_mode = accumulate ? 2 : 1;
  a.digests = digests;
  a.do_digest = digests ? 1 : 0;
  a.flags = flags;
  // one client: the lean kernel (a fused launch never uses the general
  // paths); only the sum wanted: the sum-only instantiation where there is one
  bool any_out = digests != nullptr;
  for (int c = 0; c < L; c++) any_out = any_out || clients[c].masked_out != nullptr;
  const int lean = L == 1 ? kLean1 : 0;
  LaunchFn fn = any_out ? nullptr : find_clients_kernel(x_type, x_type, L, n_cross, lean | kSumOnly);
  if (!fn && lean) fn = find_clients_kernel(x_type, x_type, 1, n_cross, kLean1);
  if (!fn) fn = find_clients_kernel(x_type, x_type, L, n_cross);
  if (!fn) {
    sa_set_error("sa_fused_clients: no kernel for x_type=%d clients=%d cross=%d", x_type, L,
                 n_cross);
    return SA_ERR_UNSUPPORTED;
  }
  return fn(a, stream);
}

extern "C" int sa_fused_bipartite(const sa_local_client* clients, int x_type, uint64_t n, int fxp_bits,
                                  const sa_pcg64* pair_gens, const int8_t* pair_sign, uint64_t* sum_out,
                                  int accumulate, uint32_t* flags, void* stream) {
  constexpr int L = kBipartiteClients, H = L / 2, PB = H * (L - H);
  if (check_type(x_type, "sa_fused_bipartite x_type")) return SA_ERR_ARG;
  if (n == 0 && fxp_bits >= 0 && fxp_bits <= 62) return SA_OK;  // empty vectors
  if (!clients || !pair_gens || !pair_sign || !sum_out || fxp_bits < 0 || fxp_bits > 62) {
    sa_set_error("sa_fused_bipartite: bad arguments");
    return SA_ERR_ARG;
  }
  if (!aligned16(sum_out)) {
    sa_set_error("sa_fused_bipartite: sum_out must be 16-byte aligned");
    return SA_ERR_ARG;
  }
  KArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n;
  a.fxp_bits = fxp_bits;
  a.scale_d = (double)((uint64_t)1 << fxp_bits);
  a.scale_f = (float)a.scale_d;
  uint64_t bias[L] = {0};
  for (int c = 0; c < L; c++) {
    if (clients[c].x || clients[c].masked_out) {
      sa_set_error("sa_fused_bipartite: client %d: masks only (x and masked_out must be NULL)", c);
      return SA_ERR_ARG;
    }
    a.c[c].w = clients[c].weight;
    a.c[c].ws[0] = a.c[c].ws[1] = (float)clients[c].weight * a.scale_f;
  }
  for (int p = 0; p < PB; p++) {  // pair p = (p / (L - H), H + p % (L - H)), the kernel's Pairs<L, kBipartite>
    const int u = p / (L - H), v = H + p % (L - H);
    const int sg = pair_sign[p];
    if (sg != 1 && sg != -1) {
      sa_set_error("sa_fused_bipartite: pair %d sign %d", p, sg);
      return SA_ERR_ARG;
    }
    fill_stream(a.s[p], pair_gens[p], sg);
    if (sg > 0) {  // as sa_fused_clients: u adds m, v subtracts it
      bias[u] += kMaskOffset;
      bias[v] += 0 - kMaskOffset;
    } else {
      bias[u] += 1 - kMaskOffset;
      bias[v] += kMaskOffset - 1;
    }
  }
  for (int c = 0; c < L; c++) a.c[c].bias = bias[c];
  a.sum_out = sum_out;
  a.sum_mode = accumulate ? 2 : 1;
  a.flags = flags;
  LaunchFn fn = find_clients_kernel(x_type, x_type, L, 0, kBipartite);
  if (!fn) {
    sa_set_error("sa_fused_bipartite: no kernel for x_type=%d", x_type);
    return SA_ERR_UNSUPPORTED;
  }
  return fn(a, stream);
}

extern "C" int sa_set_masking_reserve(int cus) {
  if (cus < 0 || cus > 128) {
    sa_set_error("sa_set_masking_reserve: %d CUs (0..128)", cus);
    return SA_ERR_ARG;
  }
  g_masking_reserve.store(cus, std::memory_order_relaxed);
  return SA_OK;
}

extern "C" int sa_sum_u64(const uint64_t* const* in, int k, uint64_t n, uint64_t* out,
                          void* stream) {
  if (k >= 1 && n == 0) return SA_OK;  // empty vectors (their pointers may be null)
  if (!in || k < 1 || !out) {
    sa_set_error("sa_sum_u64: bad arguments (k=%d)", k);
    return SA_ERR_ARG;
  }
  for (int j = 0; j < k; j++)
    if (!in[j] || !aligned16(in[j])) {
      sa_set_error("sa_sum_u64: input %d null or not 16-byte aligned", j);
      return SA_ERR_ARG;
    }
  if (!aligned16(out)) {
    sa_set_error("sa_sum_u64: out not 16-byte aligned");
    return SA_ERR_ARG;
  }
  if (n == 0) return SA_OK;
  const int grid = tile_grid(n);
  if (grid < 0) return SA_ERR_ARG;
  // chain launches of up to 32 inputs; later launches fold the running sum in as input 0
  for (int j0 = 0; j0 < k;) {
    SumArgs a;
    memset(&a, 0, sizeof(a));
    int m = 0;
    if (j0 > 0) a.in[m++] = out;
    while (m < kSumMaxIn && j0 < k) a.in[m++] = in[j0++];
    a.k = m;
    a.out = out;
    a.n = n;
    hipLaunchKernelGGL(k_sum_u64, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    SA_HIP_CHECK(hipGetLastError());
  }
  return SA_OK;
}

extern "C" int sa_decode(const uint64_t* s, uint64_t n, int fxp_bits, double divisor,
                         const double* divisor_vec, double* out, void* stream) {
  if (fxp_bits < 0 || fxp_bits > 62 || (n > 0 && (!s || !out))) {
    sa_set_error("sa_decode: bad arguments");
    return SA_ERR_ARG;
  }
  if (n == 0) return SA_OK;
  const double inv_scale = 1.0 / (double)((uint64_t)1 << fxp_bits);
  const bool vec = aligned16(s) && aligned16(out) && aligned16(divisor_vec);
  const void* kfn = !vec ? (const void*)&k_decode_unaligned
                         : divisor_vec ? (const void*)&k_decode<true> : (const void*)&k_decode<false>;
  const int grid = vec ? tile_grid(n) : stream_grid(n, kfn);
  if (grid < 0) return vec ? SA_ERR_ARG : SA_ERR_HIP;
  if (!vec)
    hipLaunchKernelGGL(k_decode_unaligned, dim3(grid), dim3(256), 0, (hipStream_t)stream, s, n, inv_scale,
                       divisor, divisor_vec, out);
  else if (divisor_vec)
    hipLaunchKernelGGL(k_decode<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, s, n, inv_scale, divisor,
                       divisor_vec, out);
  else
    hipLaunchKernelGGL(k_decode<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, s, n, inv_scale,
                       divisor, divisor_vec, out);
  SA_HIP_CHECK(hipGetLastError());
  return SA_OK;
}

extern "C" int sa_sum_f64(const double* const* w, int k, uint64_t n, double* out, void* stream) {
  if (k >= 1 && n == 0) return SA_OK;
  if (!w || k < 1 || !out) {
    sa_set_error("sa_sum_f64: bad arguments");
    return SA_ERR_ARG;
  }
  bool vec = aligned16(out);
  for (int j = 0; j < k; j++) {
    if (!w[j]) {
      sa_set_error("sa_sum_f64: input %d null", j);
      return SA_ERR_ARG;
    }
    vec = vec && aligned16(w[j]);
  }
  const int grid = vec ? tile_grid(n) : stream_grid(n, (const void*)&k_sum_f64_unaligned);
  if (grid < 0) return vec ? SA_ERR_ARG : SA_ERR_HIP;
  for (int j0 = 0; j0 < k;) {
    SumF64Args a;
    memset(&a, 0, sizeof(a));
    a.accumulate = j0 > 0;
    int m = 0;
    while (m < kSumMaxIn && j0 < k) a.in[m++] = w[j0++];
    a.k = m;
    a.out = out;
    a.n = n;
    if (vec)
      hipLaunchKernelGGL(k_sum_f64, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(k_sum_f64_unaligned, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    SA_HIP_CHECK(hipGetLastError());
  }
  return SA_OK;
}

// The blocking small-call entries below lay their buffers out so that the
// words the kernels accumulate into (PRG flag, digests, and for
// sa_clients_host the masked sum) ride the one host-to-device copy as zeros
// -- no separate fill -- and the words read back sit right before the
// result, so one device-to-host copy brings everything (a small call is
// bound by its number of device operations).  An error after
// the first copy was enqueued drains the stream before returning, so the
// caller may reuse or free the scratch at once.
static int drain(hipStream_t s, int rc) {
  (void)hipStreamSynchronize(s);
  return rc;
}

static inline uint64_t even_words(uint64_t w) { return (w + 1) & ~1ull; }

extern "C" int sa_fused_clients_host_f32(const float* const* host_x, const double* weights, int n_clients,
                                         uint64_t n, int fxp_bits, const sa_pcg64* pair_gens,
                                         const int8_t* pair_sign, double divisor, void* pinned, void* dev,
                                         double* out, uint64_t* digests, uint32_t* flags, void* stream) {
  if (!host_x || !weights || n_clients < 2 || n_clients > 8 || n == 0 || !pair_gens || !pair_sign || !pinned ||
      !dev || !out || !digests || !flags || ((uintptr_t)pinned & 15) || ((uintptr_t)dev & 15)) {
    sa_set_error("sa_fused_clients_host_f32: bad arguments (2..8 clients, n > 0, 16-byte aligned buffers)");
    return SA_ERR_ARG;
  }
  for (int c = 0; c < n_clients; c++)
    if (!host_x[c]) {
      sa_set_error("sa_fused_clients_host_f32: host_x[%d] is NULL", c);
      return SA_ERR_ARG;
    }
  const uint64_t C = (uint64_t)n_clients, n_pad = (n + 3) & ~3ull, M = even_words(1 + C);
  // host and device: [inputs C x n_pad f32 | meta M words: flag, digests | result n_pad f64] (+ device: sum)
  float* pin_in = (float*)pinned;
  uint64_t* pin_meta = (uint64_t*)(pin_in + C * n_pad);
  double* pin_res = (double*)(pin_meta + M);
  float* d_in = (float*)dev;
  uint64_t* d_meta = (uint64_t*)(d_in + C * n_pad);
  double* d_res = (double*)(d_meta + M);
  uint64_t* d_sum = (uint64_t*)(d_res + n_pad);
  const hipStream_t s = (hipStream_t)stream;
  for (uint64_t c = 0; c < C; c++) memcpy(pin_in + c * n_pad, host_x[c], n * 4);
  memset(pin_meta, 0, M * 8);
  SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(d_in, pin_in, C * n_pad * 4 + M * 8, hipMemcpyHostToDevice, s));
  sa_local_client cl[8];
  for (uint64_t c = 0; c < C; c++) {
    cl[c].x = d_in + c * n_pad;
    cl[c].weight = weights[c];
    cl[c].masked_out = nullptr;
  }
  int rc = sa_fused_clients(cl, n_clients, SA_F32, n, fxp_bits, pair_gens, pair_sign, nullptr, 0, d_sum, 0,
                            d_meta + 1, (uint32_t*)d_meta, stream);
  if (rc) return drain(s, rc);
  rc = sa_decode(d_sum, n, fxp_bits, divisor, nullptr, d_res, stream);
  if (rc) return drain(s, rc);
  SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(pin_meta, d_meta, (M + n_pad) * 8, hipMemcpyDeviceToHost, s));
  SA_HIP_CHECK_DRAIN(s, hipStreamSynchronize(s));
  memcpy(out, pin_res, n * 8);
  *flags = (uint32_t)pin_meta[0];  // the flag word's low half (little-endian)
  memcpy(digests, pin_meta + 1, C * 8);
  return SA_OK;
}

extern "C" int sa_clients_host(const void* const* host_x, int x_type, int compute_type, const double* weights,
                               int n_clients, uint64_t n, int fxp_bits, const sa_mask_stream* streams,
                               double divisor, void* pinned, void* dev, double* out, uint64_t* digests,
                               uint32_t* flags, void* stream) {
  if (check_type(x_type, "sa_clients_host x_type") || check_type(compute_type, "sa_clients_host compute_type"))
    return SA_ERR_ARG;
  if (!host_x || !weights || n_clients < 2 || n_clients > 9 || n == 0 || !streams || !pinned || !dev || !out ||
      !digests || !flags || ((uintptr_t)pinned & 15) || ((uintptr_t)dev & 15)) {
    sa_set_error("sa_clients_host: bad arguments (2..9 clients, n > 0, 16-byte aligned buffers)");
    return SA_ERR_ARG;
  }
  for (int c = 0; c < n_clients; c++)
    if (!host_x[c]) {
      sa_set_error("sa_clients_host: host_x[%d] is NULL", c);
      return SA_ERR_ARG;
    }
  const uint64_t C = (uint64_t)n_clients, n_pad = (n + 3) & ~3ull, xs = x_type == SA_F32 ? 4 : 8;
  const uint64_t M = even_words(1 + C);
  // host and device: [inputs | sum n_pad u64 | meta M words: flag, digests | result n_pad f64] (+ device:
  // the masked vectors); a sum of up to 16 KiB rides the copy as zeros, a larger one is filled on the device
  const bool zero_by_copy = n_pad * 8 <= (16u << 10);
  char* pin_in = (char*)pinned;
  uint64_t* pin_sum = (uint64_t*)(pin_in + C * n_pad * xs);
  uint64_t* pin_meta = pin_sum + n_pad;
  double* pin_res = (double*)(pin_meta + M);
  char* d_in = (char*)dev;
  uint64_t* d_sum = (uint64_t*)(d_in + C * n_pad * xs);
  uint64_t* d_meta = d_sum + n_pad;
  double* d_res = (double*)(d_meta + M);
  uint64_t* d_masked = (uint64_t*)(d_res + n_pad);
  const hipStream_t s = (hipStream_t)stream;
  for (uint64_t c = 0; c < C; c++) memcpy(pin_in + c * n_pad * xs, host_x[c], n * xs);
  if (zero_by_copy) {
    memset(pin_sum, 0, (n_pad + M) * 8);
    SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(d_in, pin_in, C * n_pad * xs + (n_pad + M) * 8, hipMemcpyHostToDevice, s));
  } else {
    SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(d_in, pin_in, C * n_pad * xs, hipMemcpyHostToDevice, s));
    SA_HIP_CHECK_DRAIN(s, hipMemsetAsync(d_sum, 0, (n_pad + M) * 8, s));
  }
  for (uint64_t c = 0; c < C; c++) {
    const int rc = sa_mask(d_in + c * n_pad * xs, x_type, compute_type, n, weights[c], nullptr, fxp_bits,
                           streams + c * (C - 1), n_clients - 1, d_masked + c * n_pad, d_sum, d_meta + 1 + c,
                           (uint32_t*)d_meta, stream);
    if (rc) return drain(s, rc);
  }
  const int rc = sa_decode(d_sum, n, fxp_bits, divisor, nullptr, d_res, stream);
  if (rc) return drain(s, rc);
  SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(pin_meta, d_meta, (M + n_pad) * 8, hipMemcpyDeviceToHost, s));
  SA_HIP_CHECK_DRAIN(s, hipStreamSynchronize(s));
  memcpy(out, pin_res, n * 8);
  *flags = (uint32_t)pin_meta[0];
  memcpy(digests, pin_meta + 1, C * 8);
  return SA_OK;
}

extern "C" int sa_mask_host(const void* host_x, int x_type, int compute_type, uint64_t n, double weight,
                            int fxp_bits, const sa_mask_stream* streams, int n_streams, void* pinned, void* dev,
                            uint64_t* out, uint32_t* flags, void* stream) {
  if (check_type(x_type, "sa_mask_host x_type") || check_type(compute_type, "sa_mask_host compute_type"))
    return SA_ERR_ARG;
  if (!host_x || n == 0 || n_streams < 0 || (n_streams > 0 && !streams) || !pinned || !dev || !out || !flags ||
      ((uintptr_t)pinned & 15) || ((uintptr_t)dev & 15)) {
    sa_set_error("sa_mask_host: bad arguments (n > 0, 16-byte aligned buffers)");
    return SA_ERR_ARG;
  }
  const uint64_t n_pad = (n + 3) & ~3ull, xs = x_type == SA_F32 ? 4 : 8;
  // host and device: [input n_pad | flag word + pad (2 words) | masked vector n_pad u64]
  char* pin_in = (char*)pinned;
  uint64_t* pin_flag = (uint64_t*)(pin_in + n_pad * xs);
  char* d_in = (char*)dev;
  uint64_t* d_flag = (uint64_t*)(d_in + n_pad * xs);
  uint64_t* d_out = d_flag + 2;
  const hipStream_t s = (hipStream_t)stream;
  memcpy(pin_in, host_x, n * xs);
  pin_flag[0] = pin_flag[1] = 0;
  SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(d_in, pin_in, n_pad * xs + 16, hipMemcpyHostToDevice, s));
  const int rc = sa_mask(d_in, x_type, compute_type, n, weight, nullptr, fxp_bits, streams, n_streams, d_out,
                         nullptr, nullptr, (uint32_t*)d_flag, stream);
  if (rc) return drain(s, rc);
  SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(pin_flag, d_flag, 16 + n * 8, hipMemcpyDeviceToHost, s));
  SA_HIP_CHECK_DRAIN(s, hipStreamSynchronize(s));
  memcpy(out, pin_flag + 2, n * 8);
  *flags = (uint32_t)pin_flag[0];
  return SA_OK;
}

extern "C" int sa_sum_decode_host(const uint64_t* const* host_masked, int n_clients, uint64_t n, int fxp_bits,
                                  double divisor, void* pinned, void* dev, double* out, uint64_t* digests,
                                  void* stream) {
  if (!host_masked || n_clients < 1 || n_clients > kSumMaxIn || n == 0 || !pinned || !dev || !out || !digests ||
      ((uintptr_t)pinned & 15) || ((uintptr_t)dev & 15)) {
    sa_set_error("sa_sum_decode_host: bad arguments (1..%d vectors, n > 0, 16-byte aligned buffers)", kSumMaxIn);
    return SA_ERR_ARG;
  }
  for (int c = 0; c < n_clients; c++)
    if (!host_masked[c]) {
      sa_set_error("sa_sum_decode_host: host_masked[%d] is NULL", c);
      return SA_ERR_ARG;
    }
  const uint64_t C = (uint64_t)n_clients, n_pad = (n + 3) & ~3ull, M = even_words(C);
  // host and device: [masked vectors C x n_pad | digests M words | result n_pad f64] (+ device: sum)
  uint64_t* pin_in = (uint64_t*)pinned;
  uint64_t* pin_dig = pin_in + C * n_pad;
  double* pin_res = (double*)(pin_dig + M);
  uint64_t* d_in = (uint64_t*)dev;
  uint64_t* d_dig = d_in + C * n_pad;
  double* d_res = (double*)(d_dig + M);
  uint64_t* d_sum = (uint64_t*)(d_res + n_pad);
  const hipStream_t s = (hipStream_t)stream;
  for (uint64_t c = 0; c < C; c++) memcpy(pin_in + c * n_pad, host_masked[c], n * 8);
  memset(pin_dig, 0, M * 8);
  SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(d_in, pin_in, (C * n_pad + M) * 8, hipMemcpyHostToDevice, s));
  const uint64_t* ins[kSumMaxIn];
  for (uint64_t c = 0; c < C; c++) {
    ins[c] = d_in + c * n_pad;
    const int rc = sa_xor_u64(ins[c], n, d_dig + c, stream);
    if (rc) return drain(s, rc);
  }
  int rc = sa_sum_u64(ins, n_clients, n, d_sum, stream);
  if (rc) return drain(s, rc);
  rc = sa_decode(d_sum, n, fxp_bits, divisor, nullptr, d_res, stream);
  if (rc) return drain(s, rc);
  SA_HIP_CHECK_DRAIN(s, hipMemcpyAsync(pin_dig, d_dig, (M + n) * 8, hipMemcpyDeviceToHost, s));
  SA_HIP_CHECK_DRAIN(s, hipStreamSynchronize(s));
  memcpy(out, pin_res, n * 8);
  memcpy(digests, pin_dig, C * 8);
  return SA_OK;
}
