/*
 * sfl_sa.h — C-ABI of the MI355X secure-aggregation hot path (libsfl_sa.so).
 *
 * Drop-in boundary for the element-wise core of
 * secretflow.security.aggregation.SecureAggregator (un-vendored dependency
 * secretflow-lite==1.13.0b0, /root/reference/pyproject.toml:51).  Each entry
 * point below cites the reference interface it replaces.  Python reaches it
 * through ctypes (sfl_amd/_lib.py); INTEGRATION.md shows the binding a
 * maintainer would add on the reference side.
 *
 * Conventions
 *  - every function returns int: SA_OK (0) or a negative SA_ERR_* code; no
 *    exception crosses the ABI.  sa_last_error() returns a message.
 *  - device buffers are caller-owned; launches are asynchronous and ordered
 *    on the caller's hipStream_t (passed as void*; NULL = legacy stream).
 *  - the launch functions never allocate, copy or synchronise, so they can be
 *    captured into a hipGraph.  Re-entrant per stream.  The four *_host
 *    entries are the exception: blocking calls on host arrays for small
 *    payloads (they copy and synchronise, but allocate nothing either).
 *  - n == 0 is a no-op that returns SA_OK; the vector pointers of an empty
 *    call may be NULL (an empty framework tensor has no storage).
 *  - mask-stream generator states are numpy PCG64 states (state, inc) as
 *    128-bit little-endian pairs; the caller advances them between rounds
 *    with sa_pcg64_advance(), exactly like the reference's persistent
 *    np.random.Generator objects advance by one draw per masked element.
 */
#ifndef SFL_SA_H
#define SFL_SA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SA_ABI_VERSION 3

/* status codes */
#define SA_OK 0
#define SA_ERR_ARG (-1)         /* bad argument (null pointer, size, unsupported combo) */
#define SA_ERR_HIP (-2)         /* HIP runtime error */
#define SA_ERR_UNSUPPORTED (-3) /* valid request this build has no kernel for */
#define SA_ERR_RCCL (-4)        /* RCCL error */

/* element types */
#define SA_F32 0
#define SA_F64 1
#define SA_I64 2

/* bits set in *flags by the kernels */
#define SA_FLAG_PRG_REJECT 1u /* a PCG64 raw draw was 0: numpy's Lemire bounded
                                 draw would have rejected it and re-drawn (p=2^-64
                                 per draw).  The mask stream then differs from
                                 numpy's from that element on; the host
                                 re-positions it (sa_pcg64_find_zero,
                                 sa_stream_shift, sa_xor_u64 below). */

typedef struct sa_u128 {
  uint64_t lo, hi;
} sa_u128;

/* numpy PCG64 bit_generator.state['state'] = {state, inc} */
typedef struct sa_pcg64 {
  sa_u128 state;
  sa_u128 inc;
} sa_pcg64;

/* One pairwise mask stream as seen by ONE client (the owner of the stream
 * for this call).  sign = +1 when the peer's name sorts after the client's
 * (q += m), -1 otherwise (q -= m): the `party > self._party` rule of the
 * masking equation, docs/developer/algorithm/secure_aggregation.ipynb
 * cell 15. */
typedef struct sa_mask_stream {
  sa_pcg64 gen; /* generator state before draw 0 of this call */
  int32_t sign; /* +1 / -1 */
  int32_t peer; /* informational (peer client index) */
} sa_mask_stream;

/* A client co-located on this GPU for the fused kernel. */
typedef struct sa_local_client {
  const void* x;        /* n elements of x_type, device pointer */
  double weight;        /* scalar weight w_c (1.0 = none); applied in the compute type */
  uint64_t* masked_out; /* optional: this client's masked vector (wire image), n u64 */
} sa_local_client;

/* ------------------------------------------------------------------ */
/* library / setup (host only, no GPU needed)                          */
/* ------------------------------------------------------------------ */

int sa_abi_version(void);
const char* sa_last_error(void);

/* numpy.random.PCG64(seed) seeding: SeedSequence(entropy) -> generate_state(4,
 * uint64) -> pcg_setseq_128_srandom.  `words` is the entropy as 32-bit
 * little-endian words (numpy's _coerce_to_uint32_array of a non-negative int).
 * Replaces: `np.random.default_rng(seed)` inside the un-vendored _Masker
 * (secure_aggregation.ipynb cell 15 names numpy.random.PCG64). */
int sa_pcg64_from_seed(const uint32_t* words, int n_words, sa_pcg64* out);

/* == numpy PCG64.advance(delta): jump the generator by delta draws. */
int sa_pcg64_advance(sa_pcg64* g, sa_u128 delta);

/* out[i] = in[i] advanced by delta[i] draws, for count generators in one
 * call (the per-round positioning of a party's pair streams: one call per
 * round instead of one per stream; out may alias in). */
int sa_pcg64_advance_many(const sa_pcg64* in, const uint64_t* delta, int count, sa_pcg64* out);

/* Host-side reference draws, for validating the seeding/jump math only
 * (tests).  Not used by any hot-path entry point. */
int sa_pcg64_raw_host(sa_pcg64* g, uint64_t* out, uint64_t n);

/* ------------------------------------------------------------------ */
/* hot path (device, asynchronous on `stream`)                          */
/* ------------------------------------------------------------------ */

/* _Masker.mask for ONE client (un-vendored; equation at
 * secure_aggregation.ipynb cell 15, quantizer pinned by the KAT of cells
 * 17-18): masked[i] = trunc(x[i]*w*2^fxp) + sum_j sign_j * m_j[i]  (mod 2^64),
 * m_j = PCG64(gen_j).integers(int64.min, int64.max, n).astype(uint64).
 *
 *   x, x_type       input vector (SA_F32/SA_F64/SA_I64).  x == NULL means
 *                   "continue": start from the current contents of `out`
 *                   (multi-pass masking when n_streams exceeds one pass).
 *   compute_type    arithmetic type of x*w*2^fxp (numpy promotion result:
 *                   SA_F32 for float32 data with a python-scalar weight,
 *                   SA_F64 for float64 data or array weights, SA_I64 for
 *                   integer data and weights).
 *   weight          scalar weight (1.0 = none)
 *   weight_vec      optional per-element weights (n elements, compute_type)
 *   out             masked vector, n u64 (required)
 *   sum_accum       optional: sum_accum[i] += masked[i]
 *   digest          optional: *digest ^= XOR of all masked[i]
 *   flags           optional: |= SA_FLAG_*
 */
int sa_mask(const void* x, int x_type, int compute_type, uint64_t n, double weight,
            const void* weight_vec, int fxp_bits, const sa_mask_stream* streams, int n_streams,
            uint64_t* out, uint64_t* sum_accum, uint64_t* digest, uint32_t* flags, void* stream);

/* Fused single-GPU simulation of C = n_clients co-located clients (config 2
 * and the 1-GPU headline): quantize every client, expand every internal pair
 * stream ONCE and apply it +/- to both of its clients, apply each client's
 * n_cross cross-GPU streams, and write the masked sum.  Each client's masked
 * vector is formed in registers: it is XOR-folded into digests[c] and, when
 * clients[c].masked_out != NULL, stored (wire image).
 *
 *   pair_gens       n_clients*(n_clients-1)/2 generators, pair (u<v) at
 *                   index u*(2C-u-1)/2 + (v-u-1)
 *   pair_sign       +1 when client u adds the pair mask (name_v > name_u)
 *   cross           n_clients * n_cross streams, client-major
 *   sum_out         n u64; accumulate != 0 means sum_out[i] += local sum
 *   digests         n_clients u64 (XOR-accumulated; zero them first)
 * More than 32 streams with only the sum wanted (no digests, no masked_out;
 * float32; e.g. 32 clients, 4 per GPU: 6 pairs + 4 x 28 cross streams): a
 * multi-launch schedule on the same stream -- one fused launch with the
 * internal pairs (each still expanded once) and the first cross streams,
 * then masks-only launches of the remaining cross streams into sum_out.
 * Other shapes without a fused kernel (more than 8 clients, more than 32
 * streams with digests or wire images, or an uninstantiated (C, n_cross))
 * return SA_ERR_UNSUPPORTED: the caller then masks client by client with
 * sa_mask(..., sum_accum), same result, or -- more than 8 clients, only
 * the sum wanted -- runs the pair-shared schedule with sa_fused_bipartite.
 * Replaces: the client-side `mask` calls plus server `_sum`'s
 * np.sum(..., axis=0) for co-located parties. */
int sa_fused_clients(const sa_local_client* clients, int n_clients, int x_type, uint64_t n,
                     int fxp_bits, const sa_pcg64* pair_gens, const int8_t* pair_sign,
                     const sa_mask_stream* cross, int n_cross, uint64_t* sum_out, int accumulate,
                     uint64_t* digests, uint32_t* flags, void* stream);

/* Host-resident float32 clients, co-located on one GPU, in ONE blocking call:
 * the small-call path of `SecureAggregator.sum` / `.average` on host arrays
 * (FL rounds of small models, HomoBinning's
 * counts), where per-call latency, not bandwidth, decides.  Copies the
 * n_clients host vectors into `pinned`, ONE host-to-device copy (inputs and
 * zeroed flag + digest words), sa_fused_clients (masked_out NULL, no cross streams),
 * sa_decode by `divisor`, ONE device-to-host copy of result + flag word +
 * digests, synchronises `stream`, then fills the outputs (the zeroed flag
 * and digest words ride the host-to-device copy: no fill operation).  With
 * n_pad = n rounded up to a multiple of 4 and M = 1 + n_clients rounded up
 * to even, the caller owns (nothing is allocated):
 *   pinned  >= n_clients*n_pad*4 + (M + n_pad)*8 bytes of page-locked host
 *           memory, 16-byte aligned;
 *   dev     >= n_clients*n_pad*4 + (M + 2*n_pad)*8 bytes of device memory,
 *           16-byte aligned.
 * Outputs (host): out[n] the decoded float64, digests[n_clients] the masked
 * vectors' XOR digests, *flags the PRG flag word (SA_FLAG_PRG_REJECT: the
 * caller replays the round as after sa_fused_clients).  2..8 clients.
 * Unlike the launch functions this one blocks: it returns once the result
 * is on the host.  Replaces, for co-located parties, the per-party `mask`
 * calls plus the server's `_sum` and decode. */
int sa_fused_clients_host_f32(const float* const* host_x, const double* weights, int n_clients, uint64_t n,
                              int fxp_bits, const sa_pcg64* pair_gens, const int8_t* pair_sign, double divisor,
                              void* pinned, void* dev, double* out, uint64_t* digests, uint32_t* flags,
                              void* stream);

/* The same blocking small call for any element type (float64 / int64 data,
 * or float32 data with a float64 compute type): n_clients host vectors of
 * x_type, every party masked by sa_mask with its OWN streams (no pair
 * sharing: the non-float32 kernels hold one client) into a zeroed masked
 * sum, then sa_decode.  `streams`: n_clients * (n_clients - 1) entries,
 * client-major (client c's peers in its masker's order); `weights` are the
 * scalar weights as sa_mask takes them.  With n_pad = n rounded up to a
 * multiple of 4, xs the element size of x_type and M = 1 + n_clients
 * rounded up to even:
 *   pinned >= n_clients*n_pad*xs + (2*n_pad + M)*8 bytes, page-locked;
 *   dev    >= n_clients*n_pad*(xs + 8) + (2*n_pad + M)*8 bytes;
 * both 16-byte aligned.  2..9 clients.  Outputs as for
 * sa_fused_clients_host_f32.  Replaces, for co-located parties with small
 * integer / float64 vectors (HomoBinning's counts),
 * the per-party `mask` calls plus the server's `_sum` and decode. */
int sa_clients_host(const void* const* host_x, int x_type, int compute_type, const double* weights,
                    int n_clients, uint64_t n, int fxp_bits, const sa_mask_stream* streams, double divisor,
                    void* pinned, void* dev, double* out, uint64_t* digests, uint32_t* flags, void* stream);

/* The per-party drop-in's two device steps for small host payloads, each as
 * ONE blocking call (sfl_amd/security/aggregation/party.py; the reference's
 * `_Masker.mask` inside the participant and the server's `_sum` + decode,
 * secure_aggregation.ipynb:227-239, sparse_plain_aggregator.py:86-94).
 *
 * sa_mask_host: one party's masked vector.  Copies host_x (n elements of
 * x_type) into `pinned`, one host-to-device copy, zeroes the flag word,
 * sa_mask with `streams`, one device-to-host copy of the masked vector and
 * the flag word, synchronises, fills out[n] (host) and *flags.  n_pad = n
 * rounded up to a multiple of 4, xs = element size:
 *   pinned >= n_pad*xs + (2 + n_pad)*8 bytes, page-locked;  dev >= the same. */
int sa_mask_host(const void* host_x, int x_type, int compute_type, uint64_t n, double weight, int fxp_bits,
                 const sa_mask_stream* streams, int n_streams, void* pinned, void* dev, uint64_t* out,
                 uint32_t* flags, void* stream);

/* sa_sum_decode_host: the server's step.  Copies the n_clients host masked
 * vectors into `pinned`, one host-to-device copy, each vector's XOR digest,
 * their sum mod 2^64, decode by `divisor`, one device-to-host copy of the
 * result and the digests, synchronises, fills out[n] and digests[n_clients]
 * (host; the caller compares them with the digests the parties sent).
 * With M = n_clients rounded up to even:
 *   pinned >= (n_clients*n_pad + M + n_pad)*8 bytes, page-locked;
 *   dev    >= (n_clients*n_pad + M + 2*n_pad)*8 bytes;
 * 1..32 vectors, both buffers 16-byte aligned. */
int sa_sum_decode_host(const uint64_t* const* host_masked, int n_clients, uint64_t n, int fxp_bits, double divisor,
                       void* pinned, void* dev, double* out, uint64_t* digests, void* stream);

/* One block of the pair-shared schedule for MORE co-located clients than one
 * sa_fused_clients launch holds (more than 8): the 8 slots are two quads of
 * clients, (0-3) and (4-7), and the launch expands only the 16 streams of the
 * pairs BETWEEN the quads, each once, applied to both clients (pair_gens /
 * pair_sign a-major: pair p = (p / 4, 4 + p % 4); sign for the lower slot as
 * in sa_fused_clients).  Masks only: the slots' x and masked_out must be
 * NULL (the clients' quantized values, and each quad's internal pairs, come
 * from a sa_fused_clients launch over the clients of two quads); the 16
 * masks, added to both clients of each pair, go straight into the sum
 * (sum_out = or += their sum), so every pair stream of C clients is expanded
 * exactly once:
 * C(C-1)/2 draws per element instead of C(C-1) (sfl_amd/kernels.py
 * fused_many).  Replaces the per-party `_Masker.mask` + server sum of
 * SURVEY 8a a2-a5 for simulations with many parties per GPU.  float32 only. */
int sa_fused_bipartite(const sa_local_client* clients, int x_type, uint64_t n, int fxp_bits,
                       const sa_pcg64* pair_gens, const int8_t* pair_sign, uint64_t* sum_out,
                       int accumulate, uint32_t* flags, void* stream);

/* Host setting for this process's masking launches (sa_mask, sa_fused_*):
 * leave `cus` CUs' worth of the kernel's occupancy free for kernels that run
 * concurrently on other streams -- the RCCL exchange of the previous chunk
 * in the pipelined multi-GPU path, whose kernels otherwise wait for the
 * masking grid (occupancy-sized, it fills every CU) to drain.  0 (default):
 * the whole GPU.  At most half of the occupancy is ever reserved.  Results
 * are unchanged (the grid only decides which tiles a block takes). */
int sa_set_masking_reserve(int cus);

/* Server `_sum`: out[i] = sum_k in[k][i] mod 2^64 (np.sum over uint64,
 * pattern of sfl/security/aggregation/sparse_plain_aggregator.py:88-94).
 * `in` is a HOST array of k device pointers; out may alias in[0]. */
int sa_sum_u64(const uint64_t* const* in, int k, uint64_t n, uint64_t* out, void* stream);

/* Server decode: out[i] = (double)(int64)s[i] / 2^fxp / div, with
 * div = divisor_vec[i] when divisor_vec != NULL (per-element weights,
 * CHANGELOG.md:994) else `divisor` (1.0 for sum, C or sum(w) for average).
 * Division is IEEE (correctly rounded), matching numpy float64.  16-byte
 * aligned s / out / divisor_vec take 16-B accesses (two elements per lane),
 * other alignments one 8-B element per lane. */
int sa_decode(const uint64_t* s, uint64_t n, int fxp_bits, double divisor,
              const double* divisor_vec, double* out, void* stream);

/* Element-wise sum of per-client weight arrays for per-element-weight
 * averages: out[i] = sum_k w[k][i] (float64), `w` a HOST array of k device
 * pointers.  16-B accesses when every buffer is 16-byte aligned. */
int sa_sum_f64(const double* const* w, int k, uint64_t n, double* out, void* stream);

/* ------------------------------------------------------------------ */
/* numpy's rejection re-draw, reproduced after a SA_FLAG_PRG_REJECT     */
/* (never on the hot path).  Generator.integers(int64.min, int64.max)   */
/* rejects a raw PCG64 output of 0 and takes the next one, so from that */
/* element on the stream runs one raw draw further along.  A pair       */
/* stream enters its two clients with opposite signs: the masked SUM is */
/* unchanged, only per-client masked vectors and digests move.          */
/* ------------------------------------------------------------------ */

/* first_out[j] = min(first_out[j], smallest i in [0, n) whose raw draw i of
 * gens[j] (the output after i + 1 steps) is 0).  `gens` is a HOST array;
 * first_out is device memory the caller fills with UINT64_MAX first. */
int sa_pcg64_find_zero(const sa_pcg64* gens, int n_gens, uint64_t n, uint64_t* first_out, void* stream);

/* out[e] += sign * (raw[e + shift] - raw[e + shift - 1])  (mod 2^64) for e in
 * [k, n), raw relative to `gen` (raw[0] = the first step's output): moves a
 * masked vector that used raw[e + shift - 1] for element e onto
 * raw[e + shift] (the mask offset K cancels in the difference). */
int sa_stream_shift(uint64_t* out, uint64_t n, const sa_pcg64* gen, int sign, uint64_t k, uint64_t shift,
                    void* stream);

/* *digest ^= XOR of v[0..n) (the per-client digest of sa_fused_clients). */
int sa_xor_u64(const uint64_t* v, uint64_t n, uint64_t* digest, void* stream);

/* ------------------------------------------------------------------ */
/* GaussianModelDP pre-step (sfl/security/privacy/mechanism/            */
/* mechanism_fl.py:62-130), applied by a client before masking:         */
/*   x' = x * min(1, clip / ||x||) + N(0, sigma^2) / num_updates        */
/* in float32, sigma = noise_multiplier * clip * clip as the reference  */
/* computes it.  ||x|| is the global norm over all layers (or, with     */
/* sumsq_layer, min(1, clip / sqrt(||layer|| * ||all||)) per layer,     */
/* is_clip_each_layer).  The noise is Philox4x32-10 + Box-Muller keyed   */
/* by (key, element index), not numpy's unseeded global MT19937 stream:  */
/* parity for the noise is distributional; the clip follows the         */
/* reference's float32 norm arithmetic (sa_sumsq_f32), up to its BLAS    */
/* dot's float32 accumulation order.                                     */
/* ------------------------------------------------------------------ */

#define SA_DP_PARTIALS 1024 /* doubles of scratch for sa_sumsq_f32 */

typedef struct sa_dp {
  const double* sumsq;       /* device: the clipping group's squared norm (sa_sumsq_f32) */
  const double* sumsq_layer; /* device, optional: this layer's squared norm */
  double l2_norm_clip;       /* the reference's python float (the clip divides in float64) */
  float noise_std;   /* sigma */
  float num_updates; /* divisor of the noise (> 0) */
  uint64_t key;      /* Philox key */
  uint64_t counter0; /* noise index of element 0 (multiple of 4) */
} sa_dp;

/* *sumsq (+)= this layer's squared L2 norm as the reference forms it under
 * its numpy 1.23.5 (mechanism_fl.py:132-135 on float32 arrays):
 * np.linalg.norm is a float32 dot and a float32 sqrt (here the dot is the
 * deterministic fixed-order float64 sum of x[i]^2 rounded once to float32;
 * the reference's BLAS sdot adds in float32 in its own order);
 * `** 2` of that float32 scalar with a python int is float64 in numpy 1.x
 * (scalar-scalar operations promote without value-based casting), so the
 * square is exact; python's sum adds the layers in float64 from 0.
 * `partials` is caller scratch of SA_DP_PARTIALS doubles.  ABI version 3. */
int sa_sumsq_f32(const float* x, uint64_t n, double* partials, double* sumsq, int accumulate, void* stream);

/* out = clip-and-noise(x) (out may alias x). */
int sa_dp_perturb_f32(const float* x, uint64_t n, const sa_dp* dp, float* out, void* stream);

/* sa_mask of the DP-perturbed float32 x without materialising it: the
 * clip+noise runs inside the masking kernel on the loaded tile.  Equal bit
 * for bit to sa_dp_perturb_f32 followed by sa_mask. */
int sa_mask_dp(const float* x, uint64_t n, double weight, int fxp_bits, const sa_mask_stream* streams,
               int n_streams, const sa_dp* dp, uint64_t* out, uint64_t* sum_accum, uint64_t* digest,
               uint32_t* flags, void* stream);

/* ------------------------------------------------------------------ */
/* multi-GPU exchange: the masked-sum reduce over RCCL (xGMI)           */
/* Replaces the RayFed `.to(server)` transfer + server np.sum           */
/* (sfl/distributed/op_strategy.py:131-141; sparse_plain_aggregator.py:86) */
/* ------------------------------------------------------------------ */

#define SA_UNIQUE_ID_BYTES 128

int sa_comm_unique_id(void* id_out, int cap);
int sa_comm_init(void** comm, const void* id, int nranks, int rank, int device);
/* ncclReduce(ncclUint64, ncclSum): recv (on root) = sum over ranks of send.
 * Bit-exact for any RCCL algorithm: uint64 add is associative mod 2^64.
 * recv may be NULL on non-root ranks: the reduce then runs in place on send
 * (the call pattern torch.distributed.reduce uses), never on a null buffer. */
int sa_comm_reduce_u64(void* comm, const uint64_t* send, uint64_t* recv, uint64_t n, int root,
                       void* stream);
int sa_comm_allreduce_u64(void* comm, const uint64_t* send, uint64_t* recv, uint64_t n,
                          void* stream);
/* The sharded server (SURVEY.md §8(e) "ReduceScatter, then decode the shards
 * in parallel, then Gather float64"): ncclReduceScatter(ncclUint64, ncclSum),
 * rank r's recv (count elements) = sum over ranks of send[r*count, (r+1)*count);
 * in place when recv == send + r*count.  Same exchange as sa_comm_reduce_u64
 * (the server's np.sum, sparse_plain_aggregator.py:88-94), the server split
 * over the ranks. */
int sa_comm_reduce_scatter_u64(void* comm, const uint64_t* send, uint64_t* recv, uint64_t count,
                               void* stream);
/* The sharded server's exchange as direct transfers (each shard crosses one
 * point-to-point xGMI link): for every rank p != r, rank r's recv[p*count,
 * (p+1)*count) = rank p's send[r*count, (r+1)*count) (grouped ncclSend /
 * ncclRecv); recv's slot r is not written.  The caller sums the shards with
 * sa_sum_u64 (its own shard from send): the same result and wire bytes as
 * sa_comm_reduce_scatter_u64, without RCCL's reduce schedule. */
int sa_comm_alltoall_u64(void* comm, const uint64_t* send, uint64_t* recv, uint64_t count,
                         void* stream);
/* The decoded float64 shards to the server: on root, recv[r*count, (r+1)*count)
 * = rank r's send (grouped ncclSend/ncclRecv); recv may be NULL off root. */
int sa_comm_gather_f64(void* comm, const double* send, double* recv, uint64_t count, int root,
                       void* stream);
/* What RCCL made of the communicator (ncclCommCount, ncclCommUserRank,
 * ncclCommCuDevice): the bench line's `rccl` record, so a scaling run shows
 * by itself that RCCL saw N ranks on N devices.  Any pointer may be NULL. */
int sa_comm_info(void* comm, int* nranks, int* rank, int* device);
int sa_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* SFL_SA_H */
