/*
 * abi_roundtrip.c — a plain C client of libsfl_sa.so (no Python, no torch):
 * what a cgo / JNI / N-API binding of include/sfl_sa.h would do.  Three
 * parties, one secure-aggregation round on the GPU:
 *   sa_pcg64_from_seed -> sa_pcg64_advance -> sa_mask (x3) -> sa_sum_u64
 *   -> sa_decode,
 * with device memory and the stream managed through the HIP C API; then the
 * same round through the blocking host-array entries: sa_mask_host per
 * party -> sa_sum_decode_host, and sa_fused_clients_host_f32 (all parties,
 * pair-shared).  Writes the masked vectors, the masked sum, the decoded
 * float64 result and the host entries' outputs to a binary file;
 * tests/test_gpu_c_abi.py compares them with the numpy oracle.
 *
 * Inputs are integer-generated so the test recomputes them exactly:
 *   x_c[i] = (float)((int32_t)((i * 2654435761u + 97u * c) % 20001u) - 10000) / 1e6f
 * pair seeds: (0x5ECA66 << 32) | (min(u,v) << 16) | max(u,v); round offset 5.
 *
 * Build: tests/c_abi/Makefile (gcc, links libsfl_sa.so and libamdhip64).
 * usage: abi_roundtrip OUT.bin [n]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/sfl_sa.h"

#define P 3

static int fail(const char* what, int rc) {
  fprintf(stderr, "%s failed (%d): %s\n", what, rc, sa_last_error());
  return 1;
}
#define SA(call)                                  \
  do {                                            \
    int rc_ = (call);                             \
    if (rc_ != SA_OK) return fail(#call, rc_);    \
  } while (0)
#define HIPC(call)                                                            \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));       \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s OUT.bin [n]\n", argv[0]);
    return 2;
  }
  const uint64_t n = argc > 2 ? strtoull(argv[2], NULL, 10) : 10007;
  const uint64_t offset = 5;
  if (sa_abi_version() != SA_ABI_VERSION) {
    fprintf(stderr, "ABI version mismatch\n");
    return 1;
  }
  float* hx = (float*)malloc(n * sizeof(float) * P);
  uint64_t* hm = (uint64_t*)malloc(n * 8 * P);
  uint64_t* hs = (uint64_t*)malloc(n * 8);
  double* hd = (double*)malloc(n * 8);
  if (!hx || !hm || !hs || !hd) return 1;
  for (int c = 0; c < P; c++)
    for (uint64_t i = 0; i < n; i++)
      hx[c * n + i] = (float)((int32_t)(((uint32_t)i * 2654435761u + 97u * (uint32_t)c) % 20001u) - 10000) / 1e6f;

  hipStream_t st;
  HIPC(hipStreamCreate(&st));
  float* dx[P];
  uint64_t* dm[P];
  uint64_t *ds, *dsum_in[P];
  double* dd;
  for (int c = 0; c < P; c++) {
    HIPC(hipMalloc((void**)&dx[c], n * sizeof(float)));
    HIPC(hipMalloc((void**)&dm[c], n * 8));
    HIPC(hipMemcpyAsync(dx[c], hx + c * n, n * sizeof(float), hipMemcpyHostToDevice, st));
  }
  HIPC(hipMalloc((void**)&ds, n * 8));
  HIPC(hipMalloc((void**)&dd, n * 8));

  /* each party masks with its P-1 pair streams (advanced to this round) */
  for (int c = 0; c < P; c++) {
    sa_mask_stream ms[P - 1];
    int k = 0;
    for (int v = 0; v < P; v++) {
      if (v == c) continue;
      const uint64_t seed = (0x5ECA66ull << 32) | ((uint64_t)(c < v ? c : v) << 16) | (uint64_t)(c < v ? v : c);
      const uint32_t words[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
      SA(sa_pcg64_from_seed(words, 2, &ms[k].gen));
      const sa_u128 d = {offset, 0};
      SA(sa_pcg64_advance(&ms[k].gen, d));
      ms[k].sign = v > c ? 1 : -1; /* party names "p0" < "p1" < "p2" */
      ms[k].peer = v;
      k++;
    }
    SA(sa_mask(dx[c], SA_F32, SA_F32, n, 1.0, NULL, 18, ms, P - 1, dm[c], NULL, NULL, NULL, (void*)st));
    dsum_in[c] = dm[c];
  }
  SA(sa_sum_u64((const uint64_t* const*)dsum_in, P, n, ds, (void*)st));
  SA(sa_decode(ds, n, 18, 1.0, NULL, dd, (void*)st));
  for (int c = 0; c < P; c++) HIPC(hipMemcpyAsync(hm + c * n, dm[c], n * 8, hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(hs, ds, n * 8, hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(hd, dd, n * 8, hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));

  /* the same round through the blocking host-array entries */
  const uint64_t n_pad = (n + 3) & ~3ull, M = (P + 2) / 2 * 2;
  const uint64_t pin_bytes = P * n_pad * 8 + (M + 2 * n_pad) * 8 + 64, dev_bytes = pin_bytes + 2 * n_pad * 8;
  void *pin, *scratch;
  HIPC(hipHostMalloc(&pin, pin_bytes, 0));
  HIPC(hipMalloc(&scratch, dev_bytes));
  uint64_t* hmh = (uint64_t*)malloc(n * 8 * P);
  double* hdh = (double*)malloc(n * 8);
  double* hdf = (double*)malloc(n * 8);
  uint64_t dig_h[P], dig_f[P], fl[2] = {0, 0};
  sa_pcg64 pg[P * (P - 1) / 2];
  int8_t ps[P * (P - 1) / 2];
  if (!hmh || !hdh || !hdf) return 1;
  for (int c = 0, q = 0; c < P; c++) {
    sa_mask_stream ms[P - 1];
    int k = 0;
    for (int v = 0; v < P; v++) {
      if (v == c) continue;
      const uint64_t seed = (0x5ECA66ull << 32) | ((uint64_t)(c < v ? c : v) << 16) | (uint64_t)(c < v ? v : c);
      const uint32_t words[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
      SA(sa_pcg64_from_seed(words, 2, &ms[k].gen));
      const sa_u128 d = {offset, 0};
      SA(sa_pcg64_advance(&ms[k].gen, d));
      ms[k].sign = v > c ? 1 : -1;
      ms[k].peer = v;
      if (v > c) { /* the pair (c, v) for the fused call, in u-major order */
        pg[q] = ms[k].gen;
        ps[q++] = 1;
      }
      k++;
    }
    uint32_t f32 = 0;
    SA(sa_mask_host(hx + c * n, SA_F32, SA_F32, n, 1.0, 18, ms, P - 1, pin, scratch, hmh + c * n, &f32,
                    (void*)st));
    fl[0] |= f32;
  }
  const uint64_t* hin[P];
  for (int c = 0; c < P; c++) hin[c] = hmh + c * n;
  SA(sa_sum_decode_host(hin, P, n, 18, 1.0, pin, scratch, hdh, dig_h, (void*)st));
  const float* hxs[P];
  double w[P];
  for (int c = 0; c < P; c++) {
    hxs[c] = hx + c * n;
    w[c] = 1.0;
  }
  uint32_t f32 = 0;
  SA(sa_fused_clients_host_f32(hxs, w, P, n, 18, pg, ps, 1.0, pin, scratch, hdf, dig_f, &f32, (void*)st));
  fl[1] = f32;

  FILE* f = fopen(argv[1], "wb");
  if (!f) return 1;
  fwrite(&n, 8, 1, f);
  fwrite(hm, 8, n * P, f);
  fwrite(hs, 8, n, f);
  fwrite(hd, 8, n, f);
  fwrite(hmh, 8, n * P, f);
  fwrite(hdh, 8, n, f);
  fwrite(dig_h, 8, P, f);
  fwrite(hdf, 8, n, f);
  fwrite(dig_f, 8, P, f);
  fwrite(fl, 8, 2, f);
  fclose(f);
  hipHostFree(pin);
  hipFree(scratch);
  free(hmh);
  free(hdh);
  free(hdf);
  for (int c = 0; c < P; c++) {
    hipFree(dx[c]);
    hipFree(dm[c]);
  }
  hipFree(ds);
  hipFree(dd);
  hipStreamDestroy(st);
  free(hx);
  free(hm);
  free(hs);
  free(hd);
  printf("abi_roundtrip: %d parties x %llu elems written to %s\n", P, (unsigned long long)n, argv[1]);
  return 0;
}
