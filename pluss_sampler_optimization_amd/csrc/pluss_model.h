// pluss_model.h — integer model of the PLUSS GEMM sampler, evaluated per
// sampled access on the device (and on the host by the C-ABI for validation).
//
// The reference replays the simulated static OpenMP schedule access by access
// and finds a sample's reuse with a per-thread last-access table
// (r10 sampler_<REF>, c_lib/test/sampler/gemm-t4-pluss-pro-model-rs-ri-opt-r10.cpp:275-654;
// full trace seq.cpp:37-333).  Here the same forward search is done by
// JUMPING: for the sampled cache line we enumerate the <= CLS/DS array
// elements that map to it and compute, per element, the first touch by the
// same simulated thread after the sample, from the loop-nest structure.  The
// minimum over those candidates is the thread-local reuse interval.
//
// Loop nest (gemm.ppcg_omp.c:72-98; generated order seq.cpp:102-288):
//   for c0 in [0,N) (static, chunk CS, T threads):
//     for c1 in [0,N):  C0 C[c0][c1]; C1 C[c0][c1];
//       for c2 in [0,N): A0 A[c0][c2]; B0 B[c2][c1]; C2 C[c0][c1]; C3 C[c0][c1]
// Thread t owns rows c0 with (c0/CS)%T == t; its local row index is
// q = (c0/(CS*T))*CS + c0%CS (ChunkDispatcher, pluss_utils.h:410-439).
// Thread-local access position: P = q*R + c1*S + off, S = 4N+2, R = N*S,
// off(C0)=0, off(C1)=1, off(A0)=2+4c2, off(B0)=3+4c2, off(C2)=4+4c2, off(C3)=5+4c2.
// Line of element (i,j): (i*N+j)*DS/CLS (GetAddress_*, seq.cpp:12-35).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define PM_HD __host__ __device__ __forceinline__
#else
#define PM_HD inline
#endif

namespace pluss {

enum : uint32_t { C0 = 0, C1 = 1, A0 = 2, B0 = 3, C2 = 4, C3 = 5 };
enum : uint32_t { ARR_C = 0, ARR_A = 1, ARR_B = 2 };
PM_HD uint32_t ref_array(uint32_t ref) { return ref == A0 ? ARR_A : (ref == B0 ? ARR_B : ARR_C); }

// Division by a run-time invariant (round-up multiplier).  Valid for n < 2^31.
struct FastDiv {
  uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.s = l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  return f;
}
PM_HD uint32_t umulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(a, b);
#else
  return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}
PM_HD uint32_t fdiv(uint32_t n, const FastDiv& f) { return (umulhi32(n, f.m) + n) >> f.s; }
PM_HD uint32_t fmod_(uint32_t n, const FastDiv& f) { return n - fdiv(n, f) * f.d; }

// Everything a kernel needs, precomputed on the host.  Passed by value.
struct Model {
  uint32_t N, T, CS, W;  // W = CLS/DS elements per line
  uint32_t S;            // 4N+2 accesses per c1 iteration
  uint32_t fast;         // N % W == 0: the closed rules (ri_fast / case_fast) apply
  uint32_t p2;           // W and CS are powers of two (mask/shift instead of FastDiv)
  uint32_t wmask, csmask, csshift, wsh;  // wsh = log2(W) when W is a power of two
  uint64_t R;            // N*S accesses per row
  uint64_t thr;          // share threshold (B0 only)
  uint64_t A;            // accesses per simulated thread when N % (CS*T) == 0
  FastDiv dCS, dT, dW, dN;
  uint64_t keytab[18];   // fast path: histogram key of (ref, case), case 0/1/2 (see case_fast)
  uint32_t np2;          // N is a power of two: an index is out of range iff it has a bit in badlo/badhi
  uint32_t badlo, badhi; // bits of a packed sample's low/high word that hold index bits >= log2(N)
  uint32_t tcs;          // (T-1)*CS: distance from the last row of a chunk to the thread's next chunk
};

// Histogram key: ref(4) | kind(4) | (ri + 2)(56).  ri = -1 encodes cold.
constexpr uint64_t KEY_EMPTY = ~0ull;
PM_HD uint64_t make_key(uint32_t ref, uint32_t kind, int64_t ri) {
  return ((uint64_t)ref << 60) | ((uint64_t)kind << 56) | (uint64_t)(ri + 2);
}
PM_HD uint32_t key_ref(uint64_t k) { return (uint32_t)(k >> 60); }
PM_HD uint32_t key_kind(uint64_t k) { return (uint32_t)((k >> 56) & 0xF); }
PM_HD int64_t key_ri(uint64_t k) { return (int64_t)(k & ((1ull << 56) - 1)) - 2; }

// Packed sample: ref(4) | c0(20) | c1(20) | c2(20)   
struct Sample {
  uint32_t ref, c0, c1, c2;
};
PM_HD Sample unpack(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  Sample s;
  s.c2 = lo & 0xFFFFFu;
  s.c1 = (lo >> 20) | ((hi & 0xFFu) << 12);
  s.c0 = (hi >> 8) & 0xFFFFFu;
  s.ref = hi >> 28;
  return s;
}
PM_HD uint64_t pack(uint32_t ref, uint32_t c0, uint32_t c1, uint32_t c2) {
  return ((uint64_t)ref << 60) | ((uint64_t)c0 << 40) | ((uint64_t)c1 << 20) | (uint64_t)c2;
}

PM_HD uint32_t ref_off(uint32_t ref, uint32_t c2) { return ref < 2 ? ref : ref + 4u * c2; }

// Does thread owning row c0 own another row after it?
PM_HD bool next_row_exists(const Model& m, uint32_t c0, uint32_t p) {
  uint32_t nxt = (p + 1 != m.CS) ? c0 + 1 : c0 + 1 + (m.T - 1) * m.CS;
  return nxt < m.N;
}

constexpr int64_t RI_COLD = -1;

// Closed rules for N % W == 0 (every BASELINE configuration).  32-bit.
// These are the generic rules below specialised: a line never spans two rows.
PM_HD int64_t ri_fast(const Model& m, uint32_t ref, uint32_t c0, uint32_t c1, uint32_t c2) {
  const uint32_t Wm1 = m.W - 1;
  switch (ref) {
    case C0: return 1;                                   // -> C1 same element
    case C1: return 3;                                   // -> C2(c2=0)
    case C2: return 1;                                   // -> C3 same c2
    case C3:
      if (c2 + 1 < m.N) return 3;                        // -> C2(c2+1)
      return fmod_(c1, m.dW) != Wm1 ? 1 : RI_COLD;       // -> C0(c1+1) same line
    case A0:
      if (fmod_(c2, m.dW) != Wm1) return 4;              // -> A0(c2+1) same line
      return (c1 + 1 < m.N) ? (int64_t)(m.S - 4u * Wm1) : RI_COLD;  // -> first c2 of the line, next c1
    default: {                                           // B0
      if (fmod_(c1, m.dW) != Wm1) return m.S;            // -> B0(c1+1) same c2
      uint32_t p = fmod_(c0, m.dCS);
      return next_row_exists(m, c0, p) ? (int64_t)(m.R - (uint64_t)Wm1 * m.S) : RI_COLD;  // next owned row
    }
  }
}

// Generic rules (any N, W, T, CS).  64-bit positions.
PM_HD int64_t ri_generic(const Model& m, uint32_t ref, uint32_t c0, uint32_t c1, uint32_t c2) {
  const uint64_t INF = ~0ull;
  const uint32_t k = fdiv(c0, m.dCS), p = c0 - k * m.CS;
  const uint32_t t = fmod_(k, m.dT), q = fdiv(k, m.dT) * m.CS + p;
  const uint32_t off = ref_off(ref, c2);
  const uint64_t rowbase = (uint64_t)q * m.R;
  const uint64_t P = rowbase + (uint64_t)c1 * m.S + off;
  const uint32_t arr = ref_array(ref);
  uint32_t i, j;
  if (arr == ARR_A) { i = c0; j = c2; } else if (arr == ARR_B) { i = c2; j = c1; } else { i = c0; j = c1; }
  const uint64_t e = (uint64_t)i * m.N + j;
  const uint64_t elo = (e / m.W) * m.W;
  uint64_t ehi = elo + m.W - 1;
  const uint64_t emax = (uint64_t)m.N * m.N - 1;
  if (ehi > emax) ehi = emax;
  const bool more_rows = next_row_exists(m, c0, p);
  uint64_t best = INF;
  for (uint64_t e2 = elo; e2 <= ehi; ++e2) {
    const uint32_t i2 = (uint32_t)(e2 / m.N), j2 = (uint32_t)(e2 - (uint64_t)i2 * m.N);
    uint64_t cand = INF;
    if (arr == ARR_B) {                      // B[c2'][c1'] is touched in every owned row
      const uint64_t o = 3ull + 4ull * i2;
      const uint64_t same = rowbase + (uint64_t)j2 * m.S + o;
      if (same > P) cand = same;
      else if (more_rows) cand = rowbase + m.R + (uint64_t)j2 * m.S + o;
    } else {
      const uint32_t k2 = fdiv(i2, m.dCS);
      if (fmod_(k2, m.dT) != t) continue;    // row i2 belongs to another simulated thread
      const uint32_t q2 = fdiv(k2, m.dT) * m.CS + (i2 - k2 * m.CS);
      const uint64_t base2 = (uint64_t)q2 * m.R;
      if (arr == ARR_A) {                    // A[c0'][c2'] touched once per c1 of row c0'
        const uint64_t o = 2ull + 4ull * j2;
        if (q2 > q) cand = base2 + o;
        else if (q2 == q) {
          if (o > off) cand = P - off + o;
          else if (c1 + 1 < m.N) cand = P - off + m.S + o;
        }
      } else {                               // C[c0'][c1'] touched in column c1' of row c0'
        if (q2 > q || (q2 == q && j2 > c1)) cand = base2 + (uint64_t)j2 * m.S;
        else if (q2 == q && j2 == c1) {      // same element: next C offset in this column
          uint32_t no = 0xFFFFFFFFu;
          if (off == 0) no = 1;
          else if (off < 4) no = 4;
          else if (((off - 4) & 3) == 0) no = off + 1;       // C2 -> C3
          else if ((off - 4) / 4 + 1 < m.N) no = off + 3;    // C3 -> C2(c2+1)
          if (no != 0xFFFFFFFFu) cand = P - off + no;
        }
      }
    }
    if (cand < best) best = cand;
  }
  return best == INF ? RI_COLD : (int64_t)(best - P);
}

PM_HD uint32_t share_kind(const Model& m, uint32_t ref, int64_t ri) {
  // distance_to(reuse,0) > distance_to(reuse,THR)  <=>  2*ri > THR  (r10:2482, seq.cpp:203)
  return (ref == B0 && ri > 0 && 2ull * (uint64_t)ri > m.thr) ? 1u : 0u;
}

// The fast rules have three outcomes per reference: case 0 (the next touch
// inside the same c1/c2 sweep), case 1 (the next sweep or row) and case 2
// (cold).  case_fast() computes only the case; the key of every (ref, case)
// is precomputed on the host (Model::keytab, from ri_fast) so the hot kernel
// turns a sample into its histogram key with selects and one table read.
template <bool P2>
PM_HD uint32_t case_fast(const Model& m, uint32_t ref, uint32_t c0, uint32_t c1, uint32_t c2) {
  const uint32_t Wm1 = m.W - 1;
  const uint32_t r1 = P2 ? (c1 & m.wmask) : fmod_(c1, m.dW);
  const uint32_t r2 = P2 ? (c2 & m.wmask) : fmod_(c2, m.dW);
  const uint32_t p = P2 ? (c0 & m.csmask) : fmod_(c0, m.dCS);
  const bool c1last = r1 == Wm1, c2last = r2 == Wm1;
  const uint32_t nxt = (p + 1 != m.CS) ? c0 + 1 : c0 + 1 + (m.T - 1) * m.CS;
  // (first, second) condition per reference: case = first ? 0 : (second ? 1 : 2)
  bool a = true, b = true;
  a = (ref == C3) ? (c2 + 1 < m.N) : a;
  b = (ref == C3) ? !c1last : b;
  a = (ref == A0) ? !c2last : a;
  b = (ref == A0) ? (c1 + 1 < m.N) : b;
  a = (ref == B0) ? !c1last : a;
  b = (ref == B0) ? (nxt < m.N) : b;
  return a ? 0u : (b ? 1u : 2u);
}

template <bool FAST>
PM_HD int64_t ri_of(const Model& m, uint32_t ref, uint32_t c0, uint32_t c1, uint32_t c2) {
  return FAST ? ri_fast(m, ref, c0, c1, c2) : ri_generic(m, ref, c0, c1, c2);
}

// Host-side construction of the Model (validated inputs; see validate_cfg).
inline Model make_model(uint64_t N, uint64_t T, uint64_t CS, uint64_t DS, uint64_t CLS, bool thr_v1) {
  Model m;
  m.N = (uint32_t)N;
  m.T = (uint32_t)T;
  m.CS = (uint32_t)CS;
  m.W = (uint32_t)(CLS / DS);
  m.S = (uint32_t)(4 * N + 2);
  m.R = N * (4 * N + 2);
  m.fast = (N % m.W == 0) ? 1u : 0u;
  const bool wp2 = (m.W & (m.W - 1)) == 0, cp2 = (m.CS & (m.CS - 1)) == 0;
  m.p2 = (wp2 && cp2) ? 1u : 0u;
  m.wmask = m.W - 1;
  m.csmask = m.CS - 1;
  m.csshift = 0;
  while ((1u << m.csshift) < m.CS) ++m.csshift;
  m.wsh = 0;
  while ((1u << m.wsh) < m.W) ++m.wsh;
  m.thr = thr_v1 ? (N + 1) * N + 1 : (4 * N + 2) * N;
  m.A = (N % (CS * T) == 0) ? (N / T) * m.R : 0;
  m.dCS = make_fastdiv(m.CS);
  m.dT = make_fastdiv(m.T);
  m.dW = make_fastdiv(m.W);
  m.dN = make_fastdiv(m.N);
  // packed-sample range check for N = 2^L: c2 = bits [0,20), c1 = [20,40), c0 = [40,60)
  m.np2 = (N & (N - 1)) == 0 ? 1u : 0u;
  m.badlo = m.badhi = 0;
  if (m.np2) {
    uint32_t L = 0;
    while ((1ull << L) < N) ++L;
    auto bits = [](uint32_t a, uint32_t b) -> uint64_t { return a < b ? (1ull << b) - (1ull << a) : 0ull; };
    const uint64_t bad = bits(L, 20) | bits(20 + L, 40) | bits(40 + L, 60);
    m.badlo = (uint32_t)bad;
    m.badhi = (uint32_t)(bad >> 32);
  }
  m.tcs = (uint32_t)((T - 1) * CS);
  // (ref, case) -> key, from the same closed rules as ri_fast
  const int64_t Wm1 = m.W - 1;
  const int64_t ri[6][3] = {
      {1, 1, 1}, {3, 3, 3}, {4, (int64_t)m.S - 4 * Wm1, RI_COLD},
      {(int64_t)m.S, (int64_t)(m.R - (uint64_t)Wm1 * m.S), RI_COLD}, {1, 1, 1}, {3, 1, RI_COLD}};
  for (uint32_t r = 0; r < 6; ++r)
    for (uint32_t c = 0; c < 3; ++c) m.keytab[r * 3 + c] = make_key(r, share_kind(m, r, ri[r][c]), ri[r][c]);
  return m;
}

// Thread-local position P and simulated thread id of a sampled access.
PM_HD void position(const Model& m, uint32_t ref, uint32_t c0, uint32_t c1, uint32_t c2, uint64_t* P,
                    uint32_t* tid) {
  const uint32_t k = fdiv(c0, m.dCS), p = c0 - k * m.CS;
  const uint32_t t = fmod_(k, m.dT), q = fdiv(k, m.dT) * m.CS + p;
  *P = (uint64_t)q * m.R + (uint64_t)c1 * m.S + ref_off(ref, c2);
  *tid = t;
}

// ---- key-order stratified sample lists ----------------------
// A reference's list generated directly in the order r10 pops its samples
// (IterationComp, pluss_utils.h:175-267 = key a*T+tid when N % (CS*T) == 0),
// so faithful mode needs no sort and the list can be counted while it is
// generated.  The valid iteration points (indices in [0, span)) are
// enumerated in key order -- (q, c1, c2, tid), tid fastest -- in two blocks:
//   A: q in [0, QA), tid in [0, T)          QA = Q-1 if span < N, else Q
//   B: q = Q-1,      tid in [0, T-1)        only if span < N (c0 = N-1 is out)
// with Q = N/T local rows per thread.  S samples are split SA = floor(S*DA/D),
// SB = S - SA; inside a block of DX points and SX samples, sample j owns the
// stratum [j*g + min(j, rr), +g + (j < rr)) (g = DX / SX, rr = DX % SX) and
// sits at a keyed pseudo-random offset in it: distinct, strictly increasing
// keys, random access by sample index (any rank can generate any slice).

PM_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 64-bit division by a run-time invariant d >= 1 (round-up multiplier, any
// 64-bit numerator; Granlund-Montgomery).
struct Div64 {
  uint64_t d, m;
  uint32_t s, one;  // one: d == 1
};
inline Div64 make_div64(uint64_t d) {
  Div64 f;
  f.d = d;
  f.one = d == 1 ? 1u : 0u;
  uint32_t l = 0;
  while (l < 64 && (1ull << l) < d) ++l;  // 2^(l-1) < d <= 2^l
  if (d <= 1) l = 1;
  f.s = l;
  const unsigned __int128 two_l = (unsigned __int128)1 << l;
  f.m = (uint64_t)((((unsigned __int128)1 << 64) * (two_l - d)) / d + 1);
  return f;
}
PM_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
PM_HD uint64_t div64(uint64_t n, const Div64& f) {
  const uint64_t q = mulhi64(n, f.m);
  const uint64_t t = ((n - q) >> 1) + q;
  return f.one ? n : t >> (f.s - 1);
}

PM_HD uint32_t lowbias32(uint32_t x) {  // 32-bit integer hash (xorshift-multiply)
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// ---- sample-list bijection (cycle-walking 4-round Feistel) ----
// Sample i of reference r is decode(F(i)), F a Feistel permutation of
// [0, 2^2h) walked until it lands in [0, D), D = span^d.  D <= 2^60, so each
// half is at most 30 bits and a round is 32-bit integer work: R' = L ^
// (lowbias32(R ^ k_r) & mask), with 32-bit round keys from splitmix64 of
// (seed, ref, round).  The index -> (c0, c1, c2) decode divides by span
// with a precomputed multiplier.
struct Perm {
  uint32_t key[4];
  uint64_t D, mask, span;  // domain size, half mask, radix
  uint32_t h, dim3;
  Div64 dspan;
};
inline Perm make_perm(uint64_t seed, uint32_t ref, uint64_t span, bool dim3) {
  Perm p;
  p.dim3 = dim3;
  p.span = span;
  p.D = dim3 ? span * span * span : span * span;
  uint32_t h = 1;
  while ((1ull << (2 * h)) < p.D) ++h;
  p.h = h;
  p.mask = (1ull << h) - 1;
  for (int r = 0; r < 4; ++r)
    p.key[r] = (uint32_t)mix64(seed ^ ((uint64_t)(ref + 1) * 0x9E3779B97F4A7C15ull) ^
                               ((uint64_t)(r + 1) * 0xD1B54A32D192ED03ull));
  p.dspan = make_div64(span ? span : 1);
  return p;
}
PM_HD uint64_t perm_apply(const Perm& p, uint64_t y) {
  const uint32_t mask = (uint32_t)p.mask;
  do {
    uint32_t L = (uint32_t)(y >> p.h), R = (uint32_t)y & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t t = R;
      R = L ^ (lowbias32(R ^ p.key[r]) & mask);
      L = t;
    }
    y = ((uint64_t)L << p.h) | R;
  } while (y >= p.D);
  return y;
}
// packed sample of permuted index y (mixed radix span: c0, c1[, c2])
PM_HD uint64_t perm_sample(const Perm& p, uint32_t ref, uint64_t y) {
  uint64_t c2 = 0;
  if (p.dim3) {
    const uint64_t q = div64(y, p.dspan);
    c2 = y - q * p.span;
    y = q;
  }
  const uint64_t c0 = div64(y, p.dspan), c1 = y - c0 * p.span;
  return pack(ref, (uint32_t)c0, (uint32_t)c1, (uint32_t)c2);
}

struct KeyGen {
  uint32_t ref, dim3, N, T, CS, span, Q, k0, k1, wide;
  uint32_t fast, tsh;  // run fast path (keyrun_*): T = 2^tsh and block-A strata below T*span
  uint32_t gd[4];      // block-A stratum size g as digits: t, c2, c1, q (2-D: t, c1, q)
  uint32_t g0, rr0;    // block A's g and rr as 32-bit values (fast path)
  uint32_t cssh, csp2; // CS = 2^cssh (packing by shifts)
  uint64_t S, SA;    // samples of this reference; of them in block A
  uint64_t g[2];     // stratum size in block A / B
  uint64_t rr[2];    // strata of size g+1 (the first rr of the block)
  Div64 dt[2], dspan;  // radix of tid in block A (T) / B (T-1); radix of c1 and c2
};

// Host: the generator of S samples of reference `ref` (validated: the caller
// checks N % (CS*T) == 0, 1 <= S <= span^d, S < 2^32).
inline KeyGen make_keygen(uint64_t N, uint64_t T, uint64_t CS, bool range_full, uint64_t seed, uint32_t ref,
                          uint64_t S) {
  KeyGen k;
  k.ref = ref;
  k.dim3 = (ref == C0 || ref == C1) ? 0u : 1u;
  k.N = (uint32_t)N;
  k.T = (uint32_t)T;
  k.CS = (uint32_t)CS;
  k.span = (uint32_t)(range_full ? N : N - 1);
  k.Q = (uint32_t)(N / T);
  const uint64_t M = k.dim3 ? (uint64_t)k.span * k.span : (uint64_t)k.span;  // points per (q, tid)
  const uint64_t QA = range_full ? k.Q : k.Q - 1;
  const uint64_t DA = QA * M * T, DB = range_full ? 0 : M * (T - 1), D = DA + DB;
  k.S = S;
  k.SA = D ? (uint64_t)(((unsigned __int128)S * DA) / D) : 0;
  const uint64_t SX[2] = {k.SA, S - k.SA}, DX[2] = {DA, DB};
  uint64_t gmax = 0;
  for (int b = 0; b < 2; ++b) {
    k.g[b] = SX[b] ? DX[b] / SX[b] : 0;
    k.rr[b] = SX[b] ? DX[b] - k.g[b] * SX[b] : 0;
    const uint64_t len = k.g[b] + (k.rr[b] ? 1 : 0);
    gmax = len > gmax ? len : gmax;
  }
  k.wide = gmax > (1ull << 32) ? 1u : 0u;
  k.dt[0] = make_div64(T);
  k.dt[1] = make_div64(T > 1 ? T - 1 : 1);
  k.dspan = make_div64(k.span ? k.span : 1);
  k.tsh = 0;
  while ((1ull << k.tsh) < T) ++k.tsh;
  const bool tp2 = (1ull << k.tsh) == T;
  const uint64_t lenA = k.g[0] + (k.rr[0] ? 1 : 0);
  k.fast = (tp2 && k.span > 0 && lenA <= (uint64_t)T * k.span && !k.wide && k.SA < (1ull << 32)) ? 1u : 0u;
  k.g0 = (uint32_t)k.g[0];
  k.rr0 = (uint32_t)k.rr[0];
  k.cssh = 0;
  while ((1ull << k.cssh) < CS) ++k.cssh;
  k.csp2 = (1ull << k.cssh) == CS ? 1u : 0u;
  {  // digits of g (block A radices)
    uint64_t r = k.g[0];
    k.gd[0] = (uint32_t)(r % T);
    r /= T;
    const uint32_t nd = k.dim3 ? 2u : 1u;
    for (uint32_t x = 0; x < nd; ++x) {
      k.gd[1 + x] = (uint32_t)(k.span ? r % k.span : 0);
      r = k.span ? r / k.span : 0;
    }
    k.gd[1 + nd] = (uint32_t)r;
    if (!k.dim3) k.gd[3] = 0;
  }
  const uint64_t h = mix64(seed ^ ((uint64_t)(ref + 1) * 0x9E3779B97F4A7C15ull) ^ 0xA5A5A5A55A5A5A5Aull);
  k.k0 = (uint32_t)h;
  k.k1 = (uint32_t)(h >> 32);
  return k;
}

// ---- the same list as iteration digits, and incrementally along a run ----
// digits of a point of the key-ordered space: local row q, c1, c2 (0 for 2-D
// references) and simulated thread t
struct KeyDigits {
  uint32_t q, c1, c2, t;
};

// digits of position p of block b (full decode)
PM_HD KeyDigits keygen_digits(const KeyGen& k, uint32_t b, uint64_t p) {
  const Div64& dt = k.dt[b];
  uint64_t r = div64(p, dt);
  KeyDigits d;
  d.t = (uint32_t)(p - r * dt.d);
  d.c2 = 0;
  if (k.dim3) {
    const uint64_t r2 = div64(r, k.dspan);
    d.c2 = (uint32_t)(r - r2 * k.span);
    r = r2;
  }
  const uint64_t r3 = div64(r, k.dspan);
  d.c1 = (uint32_t)(r - r3 * k.span);
  d.q = b ? k.Q - 1 : (uint32_t)r3;
  return d;
}

PM_HD uint64_t keygen_offset(const KeyGen& k, uint64_t i, uint64_t len) {
  const uint32_t uh = lowbias32((uint32_t)i ^ k.k0);
  if (k.wide) return mulhi64(((uint64_t)uh << 32) | lowbias32((uint32_t)i ^ k.k1), len);
  return ((uint64_t)uh * len) >> 32;
}

PM_HD uint64_t keygen_pack(const KeyGen& k, const KeyDigits& d) {
  const uint32_t c0 = (k.csp2 && k.fast) ? (((((d.q >> k.cssh) << k.tsh) | d.t) << k.cssh) | (d.q & (k.CS - 1)))
                                         : ((d.q / k.CS) * k.T + d.t) * k.CS + d.q % k.CS;
  return pack(k.ref, c0, d.c1, d.c2);
}

// The fast path of a run as straight-line 32-bit code (KeyGen::fast, the
// whole run in block A): sample i, its stratum j (= i in block A), the digits
// of its stratum base.  keyrun_fast_ok() tells whether a run of `len` samples
// from i0 may take it.
struct KeyRunF {
  uint32_t i;
  KeyDigits ld;
};
PM_HD bool keyrun_fast_ok(const KeyGen& k, uint64_t i0, uint64_t len) { return k.fast && i0 + len <= k.SA; }
PM_HD void keyrunf_start(const KeyGen& k, KeyRunF& s, uint64_t i) {
  s.i = (uint32_t)i;
  const uint64_t lo = i * k.g[0] + (i < k.rr[0] ? i : k.rr[0]);
  s.ld = keygen_digits(k, 0, lo);
}
PM_HD KeyDigits keyrunf_digits(const KeyGen& k, const KeyRunF& s) {
  const uint32_t len = k.g0 + (s.i < k.rr0 ? 1u : 0u);
  const uint32_t off = umulhi32(lowbias32(s.i ^ k.k0), len);
  KeyDigits d = s.ld;
  const uint32_t t = d.t + (off & (k.T - 1));
  uint32_t c = t >= k.T ? 1u : 0u;
  d.t = t - (c ? k.T : 0u);
  const uint32_t orest = off >> k.tsh;
  if (k.dim3) {
    const uint32_t c2 = d.c2 + orest + c;
    c = c2 >= k.span ? 1u : 0u;
    d.c2 = c2 - (c ? k.span : 0u);
    const uint32_t c1 = d.c1 + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
  } else {
    const uint32_t c1 = d.c1 + orest + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
  }
  d.q += c;
  return d;
}
PM_HD void keyrunf_next(const KeyGen& k, KeyRunF& s) {
  KeyDigits& d = s.ld;
  const uint32_t t = d.t + k.gd[0] + (s.i < k.rr0 ? 1u : 0u);
  uint32_t c = t >= k.T ? 1u : 0u;
  d.t = t - (c ? k.T : 0u);
  if (k.dim3) {
    const uint32_t c2 = d.c2 + k.gd[1] + c;
    c = c2 >= k.span ? 1u : 0u;
    d.c2 = c2 - (c ? k.span : 0u);
    const uint32_t c1 = d.c1 + k.gd[2] + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
    d.q += k.gd[3] + c;
  } else {
    const uint32_t c1 = d.c1 + k.gd[1] + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
    d.q += k.gd[2] + c;
  }
  ++s.i;
}

// A run of consecutive samples i, i+1, ... of one list: the stratum base
// lo_j is carried as digits and advanced by the stratum size's digits with
// carries, and the sample's offset (< T*span in block A when the strata are
// "small", every BASELINE list) is added to them the same way, so a sample
// costs adds and compares instead of three 64-bit divisions.  Anything else
// (block B, wide strata) falls back to the full decode.  KeyGen::gd holds the
// block-A digits of g; fast = T is a power of two and g + 1 <= T*span.
struct KeyRun {
  uint64_t i, j, lo;  // sample, its index in its block, its stratum base
  uint32_t b;         // block
  KeyDigits ld;       // digits of lo (block A fast path)
};

PM_HD void keyrun_start(const KeyGen& k, KeyRun& s, uint64_t i) {
  s.i = i;
  s.b = i < k.SA ? 0u : 1u;
  s.j = s.b ? i - k.SA : i;
  const uint64_t g = k.g[s.b], rr = k.rr[s.b];
  s.lo = s.j * g + (s.j < rr ? s.j : rr);
  s.ld = keygen_digits(k, s.b, s.lo);
}

PM_HD KeyDigits keyrun_digits(const KeyGen& k, const KeyRun& s) {
  const uint64_t len = k.g[s.b] + (s.j < k.rr[s.b] ? 1u : 0u);
  const uint64_t off = keygen_offset(k, s.i, len);
  if (s.b || !k.fast) return keygen_digits(k, s.b, s.lo + off);
  KeyDigits d = s.ld;
  const uint32_t ot = (uint32_t)off & (k.T - 1), orest = (uint32_t)(off >> k.tsh);  // orest < span
  uint32_t t = d.t + ot, c = t >= k.T ? 1u : 0u;
  d.t = t - (c ? k.T : 0u);
  if (k.dim3) {
    uint32_t c2 = d.c2 + orest + c;
    c = c2 >= k.span ? 1u : 0u;
    d.c2 = c2 - (c ? k.span : 0u);
    uint32_t c1 = d.c1 + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
  } else {
    uint32_t c1 = d.c1 + orest + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
  }
  d.q += c;
  return d;
}

PM_HD void keyrun_next(const KeyGen& k, KeyRun& s) {
  const uint64_t step = k.g[s.b] + (s.j < k.rr[s.b] ? 1u : 0u);
  ++s.i;
  if (s.i == k.SA) {  // into block B
    keyrun_start(k, s, s.i);
    return;
  }
  ++s.j;
  s.lo += step;
  if (s.b || !k.fast) return;  // the digits are only kept on the fast path
  KeyDigits& d = s.ld;
  const uint32_t inc = (uint32_t)(step - k.g[0]);  // 0 or 1
  uint32_t t = d.t + k.gd[0] + inc, c = t >= k.T ? 1u : 0u;
  d.t = t - (c ? k.T : 0u);
  if (k.dim3) {
    uint32_t c2 = d.c2 + k.gd[1] + c;
    c = c2 >= k.span ? 1u : 0u;
    d.c2 = c2 - (c ? k.span : 0u);
    uint32_t c1 = d.c1 + k.gd[2] + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
    d.q += k.gd[3] + c;
  } else {
    uint32_t c1 = d.c1 + k.gd[1] + c;
    c = c1 >= k.span ? 1u : 0u;
    d.c1 = c1 - (c ? k.span : 0u);
    d.q += k.gd[2] + c;
  }
}

// Faithful sort key a*T + tid of a point given as digits, and
// its (ref, case) outcome (case_fast's rules; B0's "the thread owns a later
// row" is q < Q-1 when N % (CS*T) == 0).
PM_HD uint64_t key_of_digits(const Model& m, uint32_t ref, const KeyDigits& d) {
  const uint64_t a = ((uint64_t)d.q * m.N + d.c1) * m.S + ref_off(ref, d.c2);
  return a * m.T + d.t;
}
template <bool P2 = false>
PM_HD uint32_t case_of_digits(const Model& m, uint32_t ref, const KeyDigits& d, uint32_t Q) {
  const uint32_t Wm1 = m.W - 1;  // P2: W a power of two (a mask; no division evaluated)
  const bool c1last = (P2 ? (d.c1 & m.wmask) : fmod_(d.c1, m.dW)) == Wm1;
  const bool c2last = (P2 ? (d.c2 & m.wmask) : fmod_(d.c2, m.dW)) == Wm1;
  bool a = true, b = true;
  a = (ref == C3) ? (d.c2 + 1 < m.N) : a;
  b = (ref == C3) ? !c1last : b;
  a = (ref == A0) ? !c2last : a;
  b = (ref == A0) ? (d.c1 + 1 < m.N) : b;
  a = (ref == B0) ? !c1last : a;
  b = (ref == B0) ? (d.q + 1 < Q) : b;
  return a ? 0u : (b ? 1u : 2u);
}

// Sample i (0 <= i < S) of the list as digits, and packed ref|c0|c1|c2.
PM_HD KeyDigits keygen_digits_at(const KeyGen& k, uint64_t i) {
  const uint32_t b = i < k.SA ? 0u : 1u;
  const uint64_t j = b ? i - k.SA : i;
  const uint64_t g = k.g[b], rr = k.rr[b];
  const uint64_t lo = j * g + (j < rr ? j : rr);
  const uint64_t len = g + (j < rr ? 1u : 0u);
  return keygen_digits(k, b, lo + keygen_offset(k, i, len));
}
PM_HD uint64_t keygen_sample(const KeyGen& k, uint64_t i) { return keygen_pack(k, keygen_digits_at(k, i)); }

}  // namespace pluss
