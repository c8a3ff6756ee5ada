// sa_host.cpp — host-side setup for the secure-aggregation C-ABI: error
// reporting, numpy-compatible PCG64 seeding (SeedSequence) and jump-ahead.
//
// This is the a1 row of SURVEY.md §8 (pairwise generator construction, once
// per FL job), not the hot path.  It restates numpy's published algorithms:
//   numpy/random/bit_generator.pyx  SeedSequence (hashmix / mix / generate_state)
//   numpy/random/_pcg64.pyx + src/pcg64/pcg64.h  pcg64_set_seed / advance
// numpy is the reference's arithmetic dependency (uv.lock:1189-1190 pins
// numpy 1.23.5; the seeding algorithm is unchanged through 2.2.6, which the
// CPU tests check against directly).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/sfl_sa.h"
#include "pcg128.h"
#include "sa_internal.h"

namespace {
thread_local char g_err[512] = "";
}

void sa_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// A tuning build (ablations that make results WRONG, or the wave-timeline
// instrumentation; sa_clients_impl.h) reports a different ABI version, so
// the product loader (sfl_amd/_lib.py) refuses it: such a library can never
// be measured or shipped as the product.
#if (defined(SA_ABLATE) && SA_ABLATE != 0) || defined(SA_TIMING)
extern "C" int sa_abi_version(void) { return SA_ABI_VERSION + 1000; }
#else
extern "C" int sa_abi_version(void) { return SA_ABI_VERSION; }
#endif
extern "C" const char* sa_last_error(void) { return g_err; }

namespace {
// SeedSequence constants (numpy/random/bit_generator.pyx)
constexpr uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u;
constexpr uint32_t INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
constexpr uint32_t MIX_MULT_L = 0xca01f9ddu, MIX_MULT_R = 0x4973f715u;
constexpr int XSHIFT = 16;
constexpr int POOL = 4;

inline uint32_t hashmix(uint32_t value, uint32_t& hc) {
  value ^= hc;
  hc *= MULT_A;
  value *= hc;
  value ^= value >> XSHIFT;
  return value;
}
inline uint32_t mix(uint32_t x, uint32_t y) {
  uint32_t r = MIX_MULT_L * x - MIX_MULT_R * y;
  r ^= r >> XSHIFT;
  return r;
}

sa::u128 to128(sa_u128 v) { return sa::mk128(v.hi, v.lo); }
sa_u128 from128(sa::u128 v) { return sa_u128{sa::lo64(v), sa::hi64(v)}; }
}  // namespace

extern "C" int sa_pcg64_from_seed(const uint32_t* words, int n_words, sa_pcg64* out) {
  if (!out || n_words < 0 || (n_words > 0 && !words)) {
    sa_set_error("sa_pcg64_from_seed: bad arguments");
    return SA_ERR_ARG;
  }
  // _coerce_to_uint32_array(0) == [0]
  std::vector<uint32_t> ent(words, words + n_words);
  if (ent.empty()) ent.push_back(0);
  // mix_entropy(pool, entropy)
  uint32_t pool[POOL];
  uint32_t hc = INIT_A;
  for (int i = 0; i < POOL; i++) pool[i] = hashmix(i < (int)ent.size() ? ent[i] : 0u, hc);
  for (int s = 0; s < POOL; s++)
    for (int d = 0; d < POOL; d++)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], hc));
  for (size_t s = POOL; s < ent.size(); s++)
    for (int d = 0; d < POOL; d++) pool[d] = mix(pool[d], hashmix(ent[s], hc));
  // generate_state(4, uint64) -> 8 uint32 words viewed as 4 little-endian u64
  uint32_t st[8];
  uint32_t hb = INIT_B;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i % POOL];
    v ^= hb;
    hb *= MULT_B;
    v *= hb;
    v ^= v >> XSHIFT;
    st[i] = v;
  }
  uint64_t val[4];
  for (int i = 0; i < 4; i++) val[i] = (uint64_t)st[2 * i] | ((uint64_t)st[2 * i + 1] << 32);
  // pcg64_set_seed(seed = val[0..1], inc = val[2..3]); PCG_128BIT_CONSTANT(high, low)
  sa::u128 initstate = sa::mk128(val[0], val[1]);
  sa::u128 initseq = sa::mk128(val[2], val[3]);
  // pcg_setseq_128_srandom_r
  sa::u128 inc = (initseq << 1) | 1;
  sa::u128 s = 0;
  s = s * sa::kPcgMult + inc;
  s += initstate;
  s = s * sa::kPcgMult + inc;
  out->state = from128(s);
  out->inc = from128(inc);
  return SA_OK;
}

extern "C" int sa_pcg64_advance(sa_pcg64* g, sa_u128 delta) {
  if (!g) {
    sa_set_error("sa_pcg64_advance: null generator");
    return SA_ERR_ARG;
  }
  sa::Jump j = sa::jump_of(delta.lo, delta.hi);
  g->state = from128(sa::apply(j, to128(g->state), to128(g->inc)));
  return SA_OK;
}

extern "C" int sa_pcg64_advance_many(const sa_pcg64* in, const uint64_t* delta, int count, sa_pcg64* out) {
  if (count < 0 || (count > 0 && (!in || !delta || !out))) {
    sa_set_error("sa_pcg64_advance_many: bad arguments");
    return SA_ERR_ARG;
  }
  for (int i = 0; i < count; i++) {
    const sa::Jump j = sa::jump_of(delta[i], 0);
    out[i].inc = in[i].inc;
    out[i].state = from128(sa::apply(j, to128(in[i].state), to128(in[i].inc)));
  }
  return SA_OK;
}

extern "C" int sa_pcg64_raw_host(sa_pcg64* g, uint64_t* out, uint64_t n) {
  if (!g || (n && !out)) {
    sa_set_error("sa_pcg64_raw_host: bad arguments");
    return SA_ERR_ARG;
  }
  sa::u128 s = to128(g->state), inc = to128(g->inc);
  for (uint64_t i = 0; i < n; i++) {
    s = s * sa::kPcgMult + inc;
    out[i] = sa::xslrr(s);
  }
  g->state = from128(s);
  return SA_OK;
}
