// Host build of the product's integer model (pluss_model.h) for CPU tests:
// lets the closed/generic reuse rules be checked against the stepping oracle
// without a GPU.  Test-only; the product library evaluates the model on the
// device exclusively.
#include <stdint.h>
#include "../../pluss_sampler_optimization_amd/csrc/pluss_model.h"

using namespace pluss;

static Model mk(int64_t N, int64_t T, int64_t CS, int64_t DS, int64_t CLS, int thr_variant) {
  return make_model(N, T, CS, DS, CLS, thr_variant != 0);
}

extern "C" int mh_ri(int64_t N, int64_t T, int64_t CS, int64_t DS, int64_t CLS, int thr_variant, int use_fast,
                     const uint64_t* smp, int64_t n, int64_t* ri, int32_t* kind, uint64_t* sink) {
  Model m = mk(N, T, CS, DS, CLS, thr_variant);
  if (use_fast && !m.fast) return -1;
  for (int64_t i = 0; i < n; i++) {
    Sample s = unpack(smp[i]);
    int64_t r = use_fast ? ri_fast(m, s.ref, s.c0, s.c1, s.c2) : ri_generic(m, s.ref, s.c0, s.c1, s.c2);
    if (use_fast) {  // the hot kernel's (case, key table) path must agree with ri_fast
      const uint64_t k = m.p2 ? m.keytab[s.ref * 3 + case_fast<true>(m, s.ref, s.c0, s.c1, s.c2)]
                              : m.keytab[s.ref * 3 + case_fast<false>(m, s.ref, s.c0, s.c1, s.c2)];
      if (k != make_key(s.ref, share_kind(m, s.ref, r), r)) return -2;
    }
    ri[i] = r;
    kind[i] = (int32_t)share_kind(m, s.ref, r);
    uint64_t P; uint32_t t;
    position(m, s.ref, s.c0, s.c1, s.c2, &P, &t);
    sink[i] = r < 0 ? ~0ull : (P + (uint64_t)r) * m.T + t;
  }
  return 0;
}

extern "C" uint32_t mh_fdiv(uint32_t n, uint32_t d) { FastDiv f = make_fastdiv(d); return fdiv(n, f); }

extern "C" int mh_expand(int64_t N, int range_full, uint64_t seed, int ref, uint64_t first, uint64_t n, uint64_t* out) {
  bool dim3 = !(ref == 0 || ref == 1);
  uint64_t span = range_full ? (uint64_t)N : (uint64_t)N - 1;
  Perm p = make_perm(seed, (uint32_t)ref, span, dim3);
  if (first + n > p.D) return -2;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t y = perm_apply(p, first + i), c2 = 0;
    if (dim3) { c2 = y % span; y /= span; }
    uint64_t c1 = y % span, c0 = y / span;
    out[i] = pack((uint32_t)ref, (uint32_t)c0, (uint32_t)c1, (uint32_t)c2);
  }
  return 0;
}

// key-order stratified lists (pluss_model.h KeyGen) and the 64-bit divider
extern "C" int mh_expand_sorted(int64_t N, int64_t T, int64_t CS, int range_full, uint64_t seed, int ref, uint64_t S,
                                uint64_t first, uint64_t n, uint64_t* out) {
  KeyGen k = make_keygen(N, T, CS, range_full != 0, seed, (uint32_t)ref, S);
  for (uint64_t i = 0; i < n; i++) out[i] = keygen_sample(k, first + i);
  return 0;
}
extern "C" uint64_t mh_div64(uint64_t n, uint64_t d) { Div64 f = make_div64(d); return div64(n, f); }
// the same list through the incremental run path (keyrun_*): runs of `run` samples
extern "C" int mh_expand_sorted_runs(int64_t N, int64_t T, int64_t CS, int range_full, uint64_t seed, int ref,
                                     uint64_t S, uint64_t first, uint64_t n, uint64_t run, uint64_t* out) {
  KeyGen k = make_keygen(N, T, CS, range_full != 0, seed, (uint32_t)ref, S);
  for (uint64_t a = 0; a < n; a += run) {
    KeyRun s;
    keyrun_start(k, s, first + a);
    for (uint64_t x = 0; x < run && a + x < n; ++x) {
      if (x) keyrun_next(k, s);
      out[a + x] = keygen_pack(k, keyrun_digits(k, s));
    }
  }
  return (int)k.fast;
}
// the 32-bit fast run path (keyrunf_*) where it applies, else the general run
extern "C" int mh_expand_sorted_fast(int64_t N, int64_t T, int64_t CS, int range_full, uint64_t seed, int ref,
                                     uint64_t S, uint64_t first, uint64_t n, uint64_t run, uint64_t* out) {
  KeyGen k = make_keygen(N, T, CS, range_full != 0, seed, (uint32_t)ref, S);
  int used = 0;
  for (uint64_t a = 0; a < n; a += run) {
    const uint64_t len = run < n - a ? run : n - a;
    if (keyrun_fast_ok(k, first + a, len)) {
      used = 1;
      KeyRunF s;
      keyrunf_start(k, s, first + a);
      for (uint64_t x = 0; x < len; ++x) {
        if (x) keyrunf_next(k, s);
        out[a + x] = keygen_pack(k, keyrunf_digits(k, s));
      }
    } else {
      for (uint64_t x = 0; x < len; ++x) out[a + x] = keygen_sample(k, first + a + x);
    }
  }
  return used;
}
