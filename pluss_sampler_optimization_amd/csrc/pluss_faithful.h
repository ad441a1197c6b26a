// pluss_faithful.h — FAITHFUL mode's one-GPU scan pipeline (k_fa_*): the
// device code shared by the per-source translation units (pluss_fa_*.hip, one
// element source each, compiled in parallel) and the host side in
// pluss_faithful.hip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <type_traits>

#include "pluss_device.h"

namespace pluss {

// Faithful-mode key storage: FM_PAIRS = 64-bit (key, sink) pairs (any
// shape); FM_PK64 / FM_PK32 = packed (rank << 2 | case) words of 64 / 32 bits.
enum : int { FM_PAIRS = 0, FM_PK64 = 1, FM_PK32 = 2 };
template <int FM>
using fkey_t = typename std::conditional<FM == FM_PK32, uint32_t, unsigned long long>::type;

// Decoding of packed words for one reference.
struct PkView {
  int64_t ri[3];             // RI of case 0/1/2 (-1: cold)
  uint64_t T, N, R, S;
  uint32_t ref, p2, tsh, nsh;  // p2: N and T powers of two (shifts)
  uint32_t Q;                  // local rows per simulated thread, N / T
};
inline PkView make_pkview(const Model& m, uint32_t ref) {
  PkView v;
  for (int c = 0; c < 3; ++c) v.ri[c] = key_ri(m.keytab[ref * 3 + c]);
  v.T = m.T;
  v.N = m.N;
  v.R = m.R;
  v.S = m.S;
  v.ref = ref;
  v.tsh = v.nsh = 0;
  while ((1ull << v.tsh) < v.T) ++v.tsh;
  while ((1ull << v.nsh) < v.N) ++v.nsh;
  v.p2 = ((1ull << v.tsh) == v.T && (1ull << v.nsh) == v.N) ? 1u : 0u;
  v.Q = (uint32_t)(v.N / v.T);
  return v;
}
// the key a*T + tid of a packed word (KEY_EMPTY for the malformed marker ~0)
template <typename KT>
__host__ __device__ __forceinline__ unsigned long long pk_key(KT pk, const PkView& v) {
  if (pk == (KT) ~(KT)0) return KEY_EMPTY;
  uint64_t r = (uint64_t)(pk >> 2), t, c2, c1, q;
  if (v.p2) {
    t = r & (v.T - 1);
    r >>= v.tsh;
    c2 = r & (v.N - 1);
    r >>= v.nsh;
    c1 = r & (v.N - 1);
    q = r >> v.nsh;
  } else {
    t = r % v.T;
    r /= v.T;
    c2 = r % v.N;
    r /= v.N;
    c1 = r % v.N;
    q = r / v.N;
  }
  const uint64_t off = v.ref < 2 ? v.ref : v.ref + 4 * c2;
  return (q * v.R + c1 * v.S + off) * v.T + t;
}
template <typename KT>
__device__ __forceinline__ unsigned long long pk_sink(KT pk, const PkView& v) {
  const uint32_t c = (uint32_t)(pk & 3u);
  if (pk == (KT) ~(KT)0 || c == 3) return KEY_EMPTY;
  const int64_t ri = c == 0 ? v.ri[0] : (c == 1 ? v.ri[1] : v.ri[2]);
  return ri < 0 ? KEY_EMPTY : pk_key(pk, v) + (unsigned long long)ri * v.T;
}
// key / sink of sorted element i
template <int FM>
__device__ __forceinline__ unsigned long long key_at(const void* keys, uint64_t i, const PkView& v) {
  if (FM == FM_PAIRS) return static_cast<const unsigned long long*>(keys)[i];
  return pk_key(static_cast<const fkey_t<FM>*>(keys)[i], v);
}
template <int FM>
__device__ __forceinline__ unsigned long long sink_at(const void* keys, const unsigned long long* sinks, uint64_t i,
                                                      const PkView& v) {
  if (FM == FM_PAIRS) return sinks[i];
  return pk_sink(static_cast<const fkey_t<FM>*>(keys)[i], v);
}
template <typename KT>
struct PkSinkOp {  // rocprim transform: packed word -> sink
  PkView v;
  __device__ unsigned long long operator()(KT pk) const { return pk_sink(pk, v); }
};

template <bool MAX>
__device__ __forceinline__ unsigned long long sc_op(unsigned long long a, unsigned long long b) {
  return MAX ? (a > b ? a : b) : a + b;
}
template <bool MAX>
__device__ __forceinline__ unsigned long long sc_wave_red(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = sc_op<MAX>(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ unsigned long long sc_wave_red_min(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long x = __shfl_xor(v, o, 64);
    v = x < v ? x : v;
  }
  return v;
}
template <bool MAX>
__device__ __forceinline__ unsigned long long sc_wave_scan(unsigned long long v, uint32_t lane) {  // inclusive
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v = sc_op<MAX>(v, y);
  }
  return v;
}
// ---- the one-GPU scan over key-ordered elements: the six references of a
// list in one pipeline that reads its elements ONCE, whatever the element
// source (sorted packed words after the radix sort, a caller's key-ordered
// samples, or samples generated in key order):
//   k_fa_local   every tile of TILE elements independently, as if no replay
//                entered it: the key-order check (a caller's list), the largest
//                sink, the start count, the Q1 bound hmax, the records of all
//                its elements, the traversed sum, and its first KL local starts
//                (key, running max of sinks before it);
//   k_fa_prefix  one workgroup per reference: exclusive prefix max of the tile
//                maxima = the running max c entering each tile;
//   k_fa_fix     per tile: with c entering, element i starts iff key_i >
//                max(c, lp_{i-1}) (lp: the tile's own running max).  A local
//                start stays a start iff key_i > c, a local non-start stays one,
//                and keys increase, so c absorbs exactly the first m local
//                starts; the first surviving start's replay-before term becomes
//                max(c, lp) and every later running max is the local one.  So
//                the start count, hmax and traversed follow from the stored
//                list; a tile whose whole list is absorbed while it has more
//                starts is queued;
//   k_fa_rescan  the queued tiles (rare) scanned again with their carry;
//   k_fa_finish  one workgroup per reference: the exclusive sum of the start
//                counts locates the tile holding the Q1 cut (the condition
//                j - starts_before_j >= n - j is monotone in j), the tiles
//                before it are summed, that tile is scanned again below the
//                cut; Q3, the -1 key, traversed, the bins.
// HBM traffic: the elements once, plus per tile a few words and its list.
constexpr int TB = 256, TI = 16;            // threads per tile, elements per thread
constexpr uint32_t TILE = TB * TI;          // elements per tile
constexpr int FPART = 5;                    // per tile: cold (tid 0), traversed, case 0/1/2 counts
constexpr int FPW = FPART + 2;              // ... + the start count and the Q1 bound hmax
constexpr int KL = 64;                      // local starts kept per tile (one wave lane each)
__host__ __device__ inline uint64_t fa_tiles(uint64_t n) { return (n + TILE - 1) / TILE; }

enum : int { SRC_W32 = 0, SRC_W64 = 1, SRC_SAMPLES = 2, SRC_GEN = 3 };
enum : int { FA_LOCAL = 0, FA_FULL = 1, FA_CUT = 2 };

struct FaRefs {
  uint64_t n[6];
  uint64_t toff[7];    // first (global) tile of each reference; toff[6] = all tiles
  const void* src[6];  // SRC_W*: sorted packed words; SRC_SAMPLES: the key-ordered samples
  PkView pv[6];
  KeyGen kg[6];        // SRC_GEN
  uint32_t fast;       // the local pass's fast path applies to the shape (fa_run)
};

// key, sink, case (3: malformed, flagged) and tid == 0 of one element.  P2:
// N, T, CS and CLS/DS powers of two (every BASELINE shape) -- decoded with
// shifts; the general decode is a separate instantiation, so no division is
// ever evaluated on the P2 path.
struct Elem {
  unsigned long long key, sink;
  uint32_t c, t0;
  unsigned long long w;  // the packed sort word rank << 2 | case (~0: malformed)
};

template <bool P2>
__device__ __forceinline__ Elem elem_of_digits(const Model& m, const PkView& v, uint32_t ref, const KeyDigits& d) {
  // P2: q*N + c1 < N*N/T < 2^32 (fa_run), so one 32x32->64 multiply
  const uint64_t qc = P2 ? (uint64_t)((d.q << v.nsh) | d.c1) : (uint64_t)d.q * m.N + d.c1;
  const uint64_t a = (P2 ? (uint64_t)(uint32_t)qc * (uint32_t)m.S : qc * m.S) + ref_off(ref, d.c2);
  const uint64_t key = P2 ? ((a << v.tsh) | d.t) : a * m.T + d.t;
  const uint32_t c = case_of_digits<P2>(m, ref, d, v.Q);
  const int64_t ri = c == 0 ? v.ri[0] : (c == 1 ? v.ri[1] : v.ri[2]);
  const unsigned long long dt = P2 ? ((unsigned long long)ri << v.tsh) : (unsigned long long)ri * m.T;
  // rank = ((q*N + c1)*N + c2)*T + t
  const uint64_t rank = P2 ? ((((qc << v.nsh) | d.c2) << v.tsh) | d.t) : (qc * m.N + d.c2) * m.T + d.t;
  return Elem{key, ri < 0 ? KEY_EMPTY : key + dt, c, d.t == 0 ? 1u : 0u, (rank << 2) | c};
}

// a packed sort word (rank << 2 | case), rank = ((q*N + c1)*N + c2)*T + tid
template <bool P2, typename KT>
__device__ __forceinline__ Elem elem_of_word(const Model& m, const PkView& v, uint32_t ref, KT w) {
  if (w == (KT) ~(KT)0) return Elem{KEY_EMPTY, KEY_EMPTY, 3u, 0u, ~0ull};
  const uint32_t c = (uint32_t)(w & 3u);
  const uint64_t r = (uint64_t)(w >> 2);
  if (P2) {  // q*N + c1 < 2^32 (fa_run): the key needs only (q*N + c1, c2, t)
    const uint32_t t = (uint32_t)r & (uint32_t)(v.T - 1);
    const uint32_t c2 = (uint32_t)(r >> v.tsh) & (uint32_t)(v.N - 1);
    const uint32_t qc = (uint32_t)(r >> (v.tsh + v.nsh));
    const uint64_t a = (uint64_t)qc * (uint32_t)m.S + ref_off(ref, c2);
    const unsigned long long key = (a << v.tsh) | t;
    const int64_t ri = c == 0 ? v.ri[0] : (c == 1 ? v.ri[1] : v.ri[2]);
    return Elem{key, (c == 3 || ri < 0) ? KEY_EMPTY : key + ((unsigned long long)ri << v.tsh), c, t == 0 ? 1u : 0u,
                (unsigned long long)w};
  }
  KeyDigits d;
  uint64_t x = r;
  d.t = (uint32_t)(x % v.T);
  x /= v.T;
  d.c2 = (uint32_t)(x % v.N);
  x /= v.N;
  d.c1 = (uint32_t)(x % v.N);
  d.q = (uint32_t)(x / v.N);
  const uint64_t a = ((uint64_t)d.q * m.N + d.c1) * m.S + ref_off(ref, d.c2);
  const uint64_t key = a * m.T + d.t;
  const int64_t ri = c == 0 ? v.ri[0] : (c == 1 ? v.ri[1] : v.ri[2]);
  return Elem{key, (c == 3 || ri < 0) ? KEY_EMPTY : key + (unsigned long long)ri * m.T, c, d.t == 0 ? 1u : 0u,
              (unsigned long long)w};
}

template <int SRC>
using fa_raw_t = typename std::conditional<SRC == SRC_W32, uint32_t, unsigned long long>::type;

// the tile's reference (wave-uniform) and its place in it
struct FaTile {
  uint32_t r;
  uint64_t lt, base;  // tile index within the reference, its first element
  uint32_t mt;        // elements in the tile
};
__device__ __forceinline__ FaTile fa_tile(const FaRefs& a, uint64_t gt) {
  uint32_t r = 0;
#pragma unroll
  for (int x = 1; x < 6; ++x) r += gt >= a.toff[x] ? 1u : 0u;
  r = __builtin_amdgcn_readfirstlane(r);
  FaTile t;
  t.r = r;
  t.lt = gt - a.toff[r];
  t.base = t.lt * TILE;
  const uint64_t left = a.n[r] - t.base;
  t.mt = (uint32_t)(left < TILE ? left : TILE);
  return t;
}

// A caller's sample, decoded for reference REF (the body is instantiated per
// reference, so the decode and the case rules fold to its own few
// instructions); `bad`: another reference or an index out of range.
template <uint32_t REF, bool P2>
__device__ __forceinline__ Elem elem_of_sample_ref(const Model& m, const PkView& v, uint64_t x, bool& bad) {
  const Sample s = unpack(x);
  const uint32_t mx = s.c0 > s.c1 ? s.c0 : s.c1;
  const bool ok = s.ref == REF && (mx > s.c2 ? mx : s.c2) < m.N;
  bad |= !ok;
  KeyDigits d;
  d.c1 = s.c1;
  d.c2 = (REF == C0 || REF == C1) ? 0u : s.c2;
  if (P2) {
    const uint32_t k = s.c0 >> m.csshift;
    d.t = k & (m.T - 1);
    d.q = ((k >> v.tsh) << m.csshift) | (s.c0 & m.csmask);
  } else {
    const uint32_t k = fdiv(s.c0, m.dCS), kt = fdiv(k, m.dT);
    d.t = k - kt * m.T;
    d.q = kt * m.CS + (s.c0 - k * m.CS);
  }
  Elem e = elem_of_digits<P2>(m, v, REF, d);
  if (!ok) e = Elem{KEY_EMPTY, KEY_EMPTY, 3u, 0u, ~0ull};
  return e;
}

template <int SRC, bool P2, uint32_t REF>
__device__ __forceinline__ Elem fa_decode_ref(const Model& m, const PkView& v, fa_raw_t<SRC> w, bool& bad) {
  if constexpr (SRC == SRC_SAMPLES) return elem_of_sample_ref<REF, P2>(m, v, (uint64_t)w, bad);
  else return elem_of_word<P2>(m, v, REF, w);
}

// the reference's first tile also materialises its -1 (cold) key in the main
// table and keeps the slot, so the finish pass only adds the count
__device__ __forceinline__ void fa_cold_slot(const FaTile& T, GTable g, unsigned long long* slots) {
  if (T.lt == 0 && threadIdx.x == 0) slots[T.r] = g_slot(g, make_key(T.r, 0, -1));
}

// One workgroup per reference: pmin[t] = max of tmax over the reference's
// tiles before t (0 for its first).  Also empties the rescan queue.
constexpr int PB = 1024;
template <int SRC>  // (instantiated in each source's translation unit)
__global__ __launch_bounds__(PB) void k_fa_prefix(FaRefs a, const unsigned long long* __restrict__ tmax,
                                                  unsigned long long* __restrict__ pmin, unsigned int* queue,
                                                  unsigned int* slowq) {
  __shared__ unsigned long long s_w[PB / 64];
  const uint32_t r = blockIdx.x;
  if (r == 0 && threadIdx.x == 0) {  // the rescan queue starts empty; the slow-tile queue is left empty (it was read)
    queue[0] = 0;
    slowq[0] = 0;
  }
  const uint64_t t0 = a.toff[r], nt = a.toff[r + 1] - t0;
  if (nt == 0) return;
  const uint64_t per = (nt + PB - 1) / PB;
  const uint64_t lo = t0 + threadIdx.x * per, hi = lo + per < t0 + nt ? lo + per : t0 + nt;
  unsigned long long mx = 0;
  for (uint64_t t = lo; t < hi; ++t) mx = tmax[t] > mx ? tmax[t] : mx;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const unsigned long long inc = sc_wave_scan<true>(mx, lane);
  if (lane == 63) s_w[wid] = inc;
  __syncthreads();
  unsigned long long pre = 0;
  for (uint32_t w = 0; w < wid; ++w) pre = s_w[w] > pre ? s_w[w] : pre;
  const unsigned long long up = __shfl_up(inc, 1, 64);
  unsigned long long run = lane ? (up > pre ? up : pre) : pre;  // exclusive prefix of this thread's segment
  for (uint64_t t = lo; t < hi; ++t) {
    pmin[t] = run;
    run = tmax[t] > run ? tmax[t] : run;
  }
}

// ---- the tile scan (NT threads; thread x owns the run [x*EPT, (x+1)*EPT) of
// the tile, staged through LDS for memory sources).  sh.out[0, FPART): cold
// (tid 0), traversed, case 0/1/2 counts (FA_CUT: below the cut);
// sh.out[FPART]: the start count (FA_CUT: the cut); sh.out[FPART + 1]: hmax =
// 2j - (starts of the tile before j) at its last start j > 0.  traversed: a
// replay starting at p subtracts key_p and the replay ending just before it
// adds the running max there; FA_CUT adds the running max at the cut; the
// end of the list (no cut) is added by the finish.  (Results go through LDS:
// a store through a generic pointer here would keep the kernels' FaRefs
// argument copied to scratch.)
template <int SRC, int NT, int EPT>
struct FaLds {
  unsigned long long w[NT / 64], c[NT / 64], red[NT / 64][FPW], out[FPW + 1];
  unsigned long long rt[4];     // ri*T per case (KEY_EMPTY: cold; case 3: malformed)
  unsigned long long klast[NT / 64];
  unsigned long long kb[2];     // the tile's first and last keys (FA_LOCAL)
  fa_raw_t<SRC> raw[SRC == SRC_GEN ? 1 : TILE + TILE / EPT];
};
// LDS slot of tile element e for runs of EPT elements per thread (one pad per run)
template <int EPT>
__device__ __forceinline__ uint32_t fa_slot_n(uint32_t e) { return e + e / EPT; }

// the one reference a scanned tile belongs to (copied out of FaRefs inside a
// per-reference branch, so the kernel argument itself is never indexed)
struct FaOne {
  FaTile T;
  uint64_t n;
  const void* src;
  PkView pv;
};

// This thread's run of the tile: keys (KEY_EMPTY past the end), cases (2 bits
// at 2k) and tid == 0 flags (bit 2k).  Memory sources: coalesced loads
// (thread x, round k: element k*NT + x) staged in LDS, read back as runs;
// generated lists: each thread generates its run (keyrunf_* when the whole
// tile lies in block A with small strata -- tile-uniform -- else one direct
// decode per sample).
template <int SRC, bool P2, uint32_t REF, int NT, int EPT, bool FULLT>
__device__ __forceinline__ void fa_load_run(const Model& m, const FaOne& o, const KeyGen& kg, FaLds<SRC, NT, EPT>& sh,
                                            unsigned long long (&key)[EPT], uint32_t& cases, uint32_t& t0s,
                                            bool& bad) {
  const FaTile& T = o.T;
  const uint32_t e0 = threadIdx.x * EPT;
  cases = 0;
  t0s = 0;
  if constexpr (SRC != SRC_GEN) {
    const fa_raw_t<SRC>* src = static_cast<const fa_raw_t<SRC>*>(o.src) + T.base;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const uint32_t e = (uint32_t)k * NT + threadIdx.x;
      if (FULLT || e < T.mt) sh.raw[fa_slot_n<EPT>(e)] = src[e];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      key[k] = KEY_EMPTY;
      if (FULLT || e0 + k < T.mt) {
        const Elem x = fa_decode_ref<SRC, P2, REF>(m, o.pv, sh.raw[fa_slot_n<EPT>(e0 + k)], bad);
        key[k] = x.key;
        cases |= x.c << (2 * k);
        t0s |= x.t0 << (2 * k);
      }
    }
  } else {
    if (keyrun_fast_ok(kg, T.base, TILE)) {  // a whole tile: every run is in range
      KeyRunF run;
      keyrunf_start(kg, run, T.base + e0);
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const Elem x = elem_of_digits<P2>(m, o.pv, REF, keyrunf_digits(kg, run));
        keyrunf_next(kg, run);
        key[k] = x.key;
        cases |= x.c << (2 * k);
        t0s |= x.t0 << (2 * k);
      }
    } else {
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        key[k] = KEY_EMPTY;
        if (FULLT || e0 + k < T.mt) {
          const Elem x = elem_of_digits<P2>(m, o.pv, REF, keygen_digits_at(kg, T.base + e0 + k));
          key[k] = x.key;
          cases |= x.c << (2 * k);
          t0s |= x.t0 << (2 * k);
        }
      }
    }
  }
}

// The scan of a loaded run.  carry_in: the running max entering the tile
// (FA_LOCAL: none -- 0 -- and the tile's first element starts); c_in (FA_CUT):
// the starts before the tile.  FA_LOCAL also writes the tile's first KL local
// starts to klist (key, running max before it).
template <int MODE, int SRC, int NT, int EPT, bool FULLT>
__device__ __forceinline__ void fa_scan(const Model& m, const FaOne& o, const unsigned long long (&key)[EPT],
                                        uint32_t cases, uint32_t t0s, unsigned long long carry_in, uint64_t c_in,
                                        FaLds<SRC, NT, EPT>& sh, unsigned long long* klist) {
  static_assert(NT * EPT == (int)TILE && EPT <= 16, "a tile is NT threads x EPT elements");
  constexpr int NW = NT / 64;
  const FaTile& T = o.T;
  const uint64_t n = o.n;
  const unsigned long long endkey = m.A * m.T;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t e0 = threadIdx.x * EPT;                                        // this lane's run in the tile
  const uint32_t nv = FULLT ? EPT : (e0 < T.mt ? (T.mt - e0 < EPT ? T.mt - e0 : EPT) : 0u);  // its valid elements
  const uint64_t i0 = T.base + e0;                                              // index of its first element
  auto sink_of = [&](unsigned long long kk, uint32_t c) -> unsigned long long {
    const unsigned long long d = sh.rt[c];  // an LDS table: no divergent selects
    const unsigned long long x = kk + d;    // d == KEY_EMPTY wraps below d: the max keeps KEY_EMPTY
    return x > d ? x : d;
  };
  if (SRC == SRC_GEN) __syncthreads();  // sh.rt (memory sources: synchronised by the staging)
  unsigned long long lmax = 0;
#pragma unroll
  for (int k = 0; k < EPT; ++k)
    if (FULLT || (uint32_t)k < nv) {
      const unsigned long long sk = sink_of(key[k], (cases >> (2 * k)) & 3u);
      lmax = sk > lmax ? sk : lmax;
    }
  // running max of sinks entering this lane: the tile's incoming max, the
  // earlier waves' maxima, the earlier lanes' maxima
  const unsigned long long linc = sc_wave_scan<true>(lmax, lane);
  if (lane == 63) sh.w[wid] = linc;
  __syncthreads();
  unsigned long long carry = carry_in, tm = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    if (x < (int)wid) carry = sh.w[x] > carry ? sh.w[x] : carry;
    tm = sh.w[x] > tm ? sh.w[x] : tm;
  }
  {
    const unsigned long long up = __shfl_up(linc, 1, 64);
    if (lane) carry = up > carry ? up : carry;
  }
  uint32_t flags = 0;
  unsigned long long tpos = 0, tneg = 0;
  auto scan = [&](uint64_t lim, bool rec) {
    unsigned long long run = carry;
    flags = 0;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      if (FULLT || (uint32_t)k < nv) {
        const uint64_t p = i0 + k;
        bool f = key[k] > run;
        if (k == 0) f = f || (MODE == FA_LOCAL ? e0 == 0 : i0 == 0);
        flags |= (f ? 1u : 0u) << k;
        if (rec) {
          if (p < lim) {
            if (f) {  // f implies run is a sink (not KEY_EMPTY), or 0 before the tile's first element
              tneg += key[k];
              tpos += run;
            }
          } else if (MODE == FA_CUT && p == lim) {
            tpos += run == KEY_EMPTY ? endkey : run;
          }
        }
        const unsigned long long sk = sink_of(key[k], (cases >> (2 * k)) & 3u);
        run = sk > run ? sk : run;
      }
    }
  };
  scan(n, MODE != FA_CUT);
  // start counts: lanes, then waves (the tile's total)
  const uint32_t lcnt = (uint32_t)__popc(flags);
  const uint32_t cinc = (uint32_t)sc_wave_scan<false>(lcnt, lane);
  if (lane == 63) sh.c[wid] = cinc;
  __syncthreads();
  uint64_t cpre = 0, cagg = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    if (x < (int)wid) cpre += sh.c[x];
    cagg += sh.c[x];
  }
  const uint64_t lb = cpre + (cinc - lcnt);  // starts of the tile before this lane's first element
  if (MODE == FA_LOCAL && lb < (uint64_t)KL && flags) {  // the tile's first KL local starts
    uint64_t rank = lb;
    unsigned long long run = carry;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      if (FULLT || (uint32_t)k < nv) {
        if (((flags >> k) & 1u) && rank < (uint64_t)KL) {
          klist[2 * rank] = key[k];
          klist[2 * rank + 1] = run;
        }
        rank += (flags >> k) & 1u;
        const unsigned long long sk = sink_of(key[k], (cases >> (2 * k)) & 3u);
        run = sk > run ? sk : run;
      }
    }
  }
  uint64_t cut = n;
  unsigned long long hl = 0;
  if (MODE == FA_CUT) {  // the first start j > 0 with j - before_j >= n - j; then the records below it
    unsigned long long best = KEY_EMPTY;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const uint64_t j = i0 + k;
      const uint64_t before_j = c_in + lb + (uint64_t)__popc(flags & ((1u << k) - 1u));
      if (best == KEY_EMPTY && ((flags >> k) & 1u) && j > 0 && j - before_j >= n - j) best = j;
    }
    best = sc_wave_red_min(best);
    if (lane == 0) sh.red[wid][0] = best;
    __syncthreads();
#pragma unroll
    for (int x = 0; x < NW; ++x) cut = sh.red[x][0] < cut ? sh.red[x][0] : cut;
    __syncthreads();  // sh.red is reused below
    scan(cut, true);
  } else if (flags) {
    const int k = 31 - __clz(flags);
    const uint64_t j = i0 + k;
    if (j > 0) hl = 2 * j - (lb + (uint64_t)__popc(flags & ((1u << k) - 1u)));
  }
  // recorded elements (below the cut) per case: recorded, or cold (tid 0 only)
  const uint64_t nrec = cut <= i0 ? 0 : (cut - i0 < nv ? cut - i0 : nv);
  const uint32_t rec2 = nrec >= 16 ? 0x55555555u : (uint32_t)((1ull << (2 * nrec)) - 1) & 0x55555555u;
  const uint32_t lo = cases & rec2, hi = (cases >> 1) & rec2;
  const uint32_t mc[3] = {rec2 & ~lo & ~hi, lo & ~hi, hi & ~lo};
  unsigned long long packed = 0;  // cold | case 0 << 16 | case 1 << 32 | case 2 << 48 (each <= TILE per tile)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (sh.rt[c] == KEY_EMPTY) packed += (unsigned long long)__popc(mc[c] & t0s);
    else packed += (unsigned long long)__popc(mc[c]) << (16 * (c + 1));
  }
  const unsigned long long v[3] = {sc_wave_red<false>(packed), sc_wave_red<false>(tpos - tneg),
                                   MODE == FA_CUT ? 0ull : sc_wave_red<true>(hl)};
  if (lane == 0)
#pragma unroll
    for (int f = 0; f < 3; ++f) sh.red[wid][f] = v[f];
  __syncthreads();
  if (threadIdx.x < FPW + 1) {
    unsigned long long x = 0;
    const uint32_t f = threadIdx.x;
    if (f == FPART) {
      x = MODE == FA_CUT ? cut : cagg;
    } else if (f == FPART + 1) {
#pragma unroll
      for (int w = 0; w < NW; ++w) x = sh.red[w][2] > x ? sh.red[w][2] : x;
    } else if (f == FPW) {
      x = tm;  // the tile's largest sink
    } else if (f == 1) {
#pragma unroll
      for (int w = 0; w < NW; ++w) x += sh.red[w][1];
    } else {  // 0 cold, 2..4 case counts
      const uint32_t sh16 = f == 0 ? 0u : 16u * (f - 1);
#pragma unroll
      for (int w = 0; w < NW; ++w) x += (sh.red[w][0] >> sh16) & 0xFFFFull;
    }
    sh.out[f] = x;
  }
  __syncthreads();
}

// ri*T per case of the tile's reference into sh.rt (KEY_EMPTY: cold; case 3: malformed)
template <int SRC, int NT, int EPT>
__device__ __forceinline__ void fa_rt(const Model& m, const PkView& pv, FaLds<SRC, NT, EPT>& sh) {
  if (threadIdx.x < 4) {
    const uint32_t c = threadIdx.x;
    const int64_t ri = c == 0 ? pv.ri[0] : (c == 1 ? pv.ri[1] : pv.ri[2]);  // selects: no dynamic index
    sh.rt[c] = (c == 3 || ri < 0) ? KEY_EMPTY : (unsigned long long)ri * m.T;
  }
}

// The key-order check of a caller's list (strictly increasing keys): inside a
// run, against the previous lane, across waves (LDS) and against the element
// before the tile.
template <int SRC, bool P2, uint32_t REF, int NT, int EPT, bool FULLT>
__device__ __forceinline__ bool fa_unordered(const Model& m, const FaOne& o, const unsigned long long (&key)[EPT],
                                             FaLds<SRC, NT, EPT>& sh, bool& bad) {
  const FaTile& T = o.T;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t e0 = threadIdx.x * EPT;
  const uint32_t nv = FULLT ? EPT : (e0 < T.mt ? (T.mt - e0 < EPT ? T.mt - e0 : EPT) : 0u);
  bool u = false;
  unsigned long long last = 0;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    if (FULLT || (uint32_t)k < nv) {
      if (k > 0) u |= !(key[k] > key[k - 1]);
      last = key[k];
    }
  }
  const unsigned long long up = __shfl_up(last, 1, 64);
  if (lane > 0 && nv) u |= !(key[0] > up);
  if (lane == 63) sh.klast[wid] = last;
  __syncthreads();
  if (lane == 0 && wid > 0 && nv) u |= !(key[0] > sh.klast[wid - 1]);
  if (threadIdx.x == 0 && T.base > 0 && nv) {
    const fa_raw_t<SRC> w = static_cast<const fa_raw_t<SRC>*>(o.src)[T.base - 1];
    u |= !(key[0] > fa_decode_ref<SRC, P2, REF>(m, o.pv, w, bad).key);
  }
  return u;
}

// 32-bit inclusive max scan over a wave
__device__ __forceinline__ uint32_t wave_scan_max32(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v = v > y ? v : y;
  }
  return v;
}

// FA_LOCAL for a tile whose keys and (non-cold) sinks lie within 2^32 - 1 of
// its first key (every dense tile): the same scan on 32-bit offsets from that
// key, cold sinks saturated to 0xFFFFFFFF.  The traversed sum is exact in 32
// bits per thread: between consecutive starts s' < s, key_s - run_s <
// key_s - key_s' (run_s >= sink_s' > key_s'), so a tile's sum of key - run over
// its starts after the first is below its key span.
template <int SRC, int NT, int EPT, bool FULLT>
__device__ __forceinline__ void fa_scan_local32(const FaOne& o, const unsigned long long (&key)[EPT], uint32_t cases,
                                                uint32_t t0s, unsigned long long base, FaLds<SRC, NT, EPT>& sh,
                                                unsigned long long* klist) {
  constexpr int NW = NT / 64;
  const FaTile& T = o.T;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t e0 = threadIdx.x * EPT;
  const uint32_t nv = FULLT ? EPT : (e0 < T.mt ? (T.mt - e0 < EPT ? T.mt - e0 : EPT) : 0u);
  const uint64_t i0 = T.base + e0;
  uint32_t rt32[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) rt32[c] = sh.rt[c] == KEY_EMPTY ? 0xFFFFFFFFu : (uint32_t)sh.rt[c];
  uint32_t rk[EPT], sk[EPT], lmax = 0;
  const uint32_t b32 = (uint32_t)base;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    rk[k] = (uint32_t)key[k] - b32;
    const uint32_t c = (cases >> (2 * k)) & 3u;
    const uint32_t d = c == 0 ? rt32[0] : (c == 1 ? rt32[1] : (c == 2 ? rt32[2] : rt32[3]));
    const uint32_t x = rk[k] + d;  // d = 0xFFFFFFFF (cold) wraps below d: the max keeps it
    sk[k] = x > d ? x : d;
    if (FULLT || (uint32_t)k < nv) lmax = sk[k] > lmax ? sk[k] : lmax;
  }
  const uint32_t linc = wave_scan_max32(lmax, lane);
  if (lane == 63) sh.w[wid] = linc;
  __syncthreads();
  uint32_t carry = 0, tm = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    const uint32_t w = (uint32_t)sh.w[x];
    if (x < (int)wid) carry = w > carry ? w : carry;
    tm = w > tm ? w : tm;
  }
  {
    const uint32_t up = __shfl_up(linc, 1, 64);
    if (lane) carry = up > carry ? up : carry;
  }
  uint32_t flags = 0, dsum = 0;  // dsum: key - run over the starts (the tile's first excluded)
  {
    uint32_t run = carry;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      if (FULLT || (uint32_t)k < nv) {
        const bool first = k == 0 && e0 == 0;
        const bool f = rk[k] > run || first;
        flags |= (f ? 1u : 0u) << k;
        dsum += (f && !first) ? rk[k] - run : 0u;
        run = sk[k] > run ? sk[k] : run;
      }
    }
  }
  const uint32_t lcnt = (uint32_t)__popc(flags);
  const uint32_t cinc = (uint32_t)sc_wave_scan<false>(lcnt, lane);
  if (lane == 63) sh.c[wid] = cinc;
  __syncthreads();
  uint64_t cpre = 0, cagg = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    if (x < (int)wid) cpre += sh.c[x];
    cagg += sh.c[x];
  }
  const uint64_t lb = cpre + (cinc - lcnt);
  if (lb < (uint64_t)KL && flags) {  // the tile's first KL local starts (absolute key, running max before it)
    uint64_t rank = lb;
    uint32_t run = carry;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      if (FULLT || (uint32_t)k < nv) {
        if (((flags >> k) & 1u) && rank < (uint64_t)KL) {
          klist[2 * rank] = base + rk[k];
          klist[2 * rank + 1] = (k == 0 && e0 == 0) ? 0ull : base + run;
        }
        rank += (flags >> k) & 1u;
        run = sk[k] > run ? sk[k] : run;
      }
    }
  }
  unsigned long long hl = 0;
  if (flags) {
    const int k = 31 - __clz(flags);
    const uint64_t j = i0 + k;
    if (j > 0) hl = 2 * j - (lb + (uint64_t)__popc(flags & ((1u << k) - 1u)));
  }
  const uint32_t rec2 = nv >= 16 ? 0x55555555u : (uint32_t)((1ull << (2 * nv)) - 1) & 0x55555555u;
  const uint32_t lo = cases & rec2, hi = (cases >> 1) & rec2;
  const uint32_t mc[3] = {rec2 & ~lo & ~hi, lo & ~hi, hi & ~lo};
  unsigned long long packed = 0;  // cold | case 0 << 16 | case 1 << 32 | case 2 << 48
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (rt32[c] == 0xFFFFFFFFu) packed += (unsigned long long)__popc(mc[c] & t0s);
    else packed += (unsigned long long)__popc(mc[c]) << (16 * (c + 1));
  }
  const unsigned long long v[3] = {sc_wave_red<false>(packed), sc_wave_red<false>((unsigned long long)dsum),
                                   sc_wave_red<true>(hl)};
  if (lane == 0)
#pragma unroll
    for (int f = 0; f < 3; ++f) sh.red[wid][f] = v[f];
  __syncthreads();
  if (threadIdx.x < FPW + 1) {
    unsigned long long x = 0;
    const uint32_t f = threadIdx.x;
    if (f == FPART) {
      x = cagg;
    } else if (f == FPART + 1) {
#pragma unroll
      for (int w = 0; w < NW; ++w) x = sh.red[w][2] > x ? sh.red[w][2] : x;
    } else if (f == FPW) {
      x = tm == 0xFFFFFFFFu ? KEY_EMPTY : base + tm;  // the tile's largest sink
    } else if (f == 1) {  // traversed: -base (the first start's key; nothing before it) - sum(key - run)
#pragma unroll
      for (int w = 0; w < NW; ++w) x += sh.red[w][1];
      x = 0ull - base - x;
    } else {
      const uint32_t sh16 = f == 0 ? 0u : 16u * (f - 1);
#pragma unroll
      for (int w = 0; w < NW; ++w) x += (sh.red[w][0] >> sh16) & 0xFFFFull;
    }
    sh.out[f] = x;
  }
  __syncthreads();
}

// ---- the local pass's fast path: a full tile of a shape with N, T, CS and
// CLS/DS powers of two and q*N + c1, S below 2^24 (every BASELINE shape),
// whose keys and non-cold sinks lie within 2^32 - 1 of its first key (every
// dense tile).  Each element is decoded straight from its bits to the low 32
// bits of its key (one 24-bit multiply-add), its case flags and tid == 0;
// everything after that is 32-bit: offsets from the tile's first key, cold
// sinks saturated to 0xFFFFFFFF, counts accumulated per thread, wave scans
// by DPP.
template <int SRC>
__device__ __forceinline__ fa_raw_t<SRC> src_at(const FaOne& o, uint32_t e) {
  return static_cast<const fa_raw_t<SRC>*>(o.src)[o.T.base + e];
}

struct FaDec {
  uint32_t lk;             // low 32 bits of the key a*T + tid
  bool a, b, t0;           // case 0 = a, case 1 = !a && b, case 2 = neither; tid == 0
  unsigned long long key;  // the whole key (CHECK: the order check)
};

template <uint32_t REF, bool KEY64>
__device__ __forceinline__ FaDec fa_dec_digits(const Model& m, const PkView& v, uint32_t q, uint32_t c1, uint32_t c2,
                                               uint32_t t) {
  FaDec d;
  const uint32_t qc = (q << v.nsh) | c1;
  const uint32_t off = ref_off(REF, c2);
  if (KEY64) {
    d.key = ((((uint64_t)qc * m.S) + off) << v.tsh) | t;
    d.lk = (uint32_t)d.key;
  } else {
    d.key = 0;
    d.lk = ((__umul24(qc, m.S) + off) << v.tsh) | t;
  }
  const uint32_t Wm1 = m.W - 1;
  d.a = true;
  d.b = true;
  if (REF == C3) {
    d.a = c2 + 1 < m.N;
    d.b = (c1 & Wm1) != Wm1;
  } else if (REF == A0) {
    d.a = (c2 & Wm1) != Wm1;
    d.b = c1 + 1 < m.N;
  } else if (REF == B0) {
    d.a = (c1 & Wm1) != Wm1;
    d.b = q + 1 < v.Q;
  }
  d.t0 = t == 0;
  return d;
}

// a caller's packed sample ref(4)|c0(20)|c1(20)|c2(20); `odd` collects the
// bits of another reference or of an index >= N (N a power of two)
template <uint32_t REF, bool KEY64>
__device__ __forceinline__ FaDec fa_dec_sample(const Model& m, const PkView& v, uint64_t x, uint32_t& odd) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  odd |= ((hi ^ (REF << 28)) & (0xF0000000u | m.badhi)) | (lo & m.badlo);
  const uint32_t c2 = (REF == C0 || REF == C1) ? 0u : (lo & 0xFFFFFu);
  const uint32_t c1 = __builtin_amdgcn_alignbit(hi, lo, 20) & 0xFFFFFu;
  const uint32_t cs = m.csshift, ts = v.tsh;
  const uint32_t t = __builtin_amdgcn_ubfe(hi, 8 + cs, ts);
  const uint32_t q = (__builtin_amdgcn_ubfe(hi, 8 + cs + ts, 20 - cs - ts) << cs) | __builtin_amdgcn_ubfe(hi, 8, cs);
  return fa_dec_digits<REF, KEY64>(m, v, q, c1, c2, t);
}

// a packed sort word rank << 2 | case, rank = ((q*N + c1)*N + c2)*T + tid
template <uint32_t REF, typename KT>
__device__ __forceinline__ FaDec fa_dec_word(const Model& m, const PkView& v, KT w) {
  const uint32_t c = (uint32_t)w & 3u;
  const uint32_t t = ((uint32_t)w >> 2) & (uint32_t)(v.T - 1);
  const uint32_t c2 = (uint32_t)(w >> (2 + v.tsh)) & (uint32_t)(v.N - 1);
  const uint32_t qc = (uint32_t)(w >> (2 + v.tsh + v.nsh));
  FaDec d;
  d.key = 0;
  d.lk = ((__umul24(qc, m.S) + ref_off(REF, c2)) << v.tsh) | t;
  d.a = c == 0;
  d.b = c == 1;
  d.t0 = t == 0;
  return d;
}

// inclusive 32-bit wave scan (identity 0), Hillis-Steele by DPP: row_shr
// 1/2/4/8 inside rows of 16 lanes, then row_bcast 15 and 31 across rows
template <bool MAX>
__device__ __forceinline__ uint32_t dpp_op(uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : a + b; }
template <bool MAX>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
  v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}
// the previous lane's value (lane 0: 0)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(v), 63);
}

template <int SRC, bool CHECK, uint32_t REF>
__device__ __forceinline__ void fa_local_fast(const Model& m, const FaOne& o, const KeyGen& kg,
                                              FaLds<SRC, TB, TI>& sh, unsigned long long base, const uint32_t (&r)[3],
                                              unsigned long long* __restrict__ klist, GTable g) {
  constexpr int NW = TB / 64;
  const FaTile& T = o.T;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t e0 = threadIdx.x * TI;
  const uint64_t i0 = T.base + e0;
  const uint32_t b32 = (uint32_t)base;
  uint32_t rk[TI], sk[TI], lmax = 0, n0 = 0, n1 = 0, nc = 0, odd = 0;
  bool unordered = false;
  unsigned long long kfirst = 0, kprev = 0;
  KeyRunF run;
  if constexpr (SRC == SRC_GEN) keyrunf_start(kg, run, T.base + e0);
#pragma unroll
  for (int k = 0; k < TI; ++k) {
    FaDec d;
    if constexpr (SRC == SRC_SAMPLES) {
      d = fa_dec_sample<REF, CHECK>(m, o.pv, sh.raw[fa_slot_n<TI>(e0 + k)], odd);
    } else if constexpr (SRC == SRC_GEN) {
      const KeyDigits dg = keyrunf_digits(kg, run);
      keyrunf_next(kg, run);
      d = fa_dec_digits<REF, false>(m, o.pv, dg.q, dg.c1, dg.c2, dg.t);
    } else {
      d = fa_dec_word<REF>(m, o.pv, sh.raw[fa_slot_n<TI>(e0 + k)]);
    }
    if (CHECK) {
      if (k == 0) kfirst = d.key;
      else unordered |= !(d.key > kprev);
      kprev = d.key;
    }
    rk[k] = d.lk - b32;
    const uint32_t dd = d.a ? r[0] : (d.b ? r[1] : r[2]);
    const uint32_t x = rk[k] + dd;  // dd = 0xFFFFFFFF (cold) wraps below dd: the max keeps it
    sk[k] = x > dd ? x : dd;
    lmax = sk[k] > lmax ? sk[k] : lmax;
    n0 += d.a ? 1u : 0u;
    n1 += (!d.a && d.b) ? 1u : 0u;
    nc += (!d.a && !d.b && d.t0) ? 1u : 0u;
  }
  if (CHECK) {  // across lanes, waves and the tile's start (the element before it)
    const unsigned long long up = __shfl_up(kprev, 1, 64);
    if (lane > 0) unordered |= !(kfirst > up);
    if (lane == 63) sh.klast[wid] = kprev;
  }
  // running max of sinks entering this lane
  const uint32_t linc = wave_scan_dpp<true>(lmax);
  if (lane == 63) sh.w[wid] = linc;
  __syncthreads();
  if (CHECK) {
    if (lane == 0 && wid > 0) unordered |= !(kfirst > sh.klast[wid - 1]);
    if (threadIdx.x == 0 && T.base > 0) {
      bool b2 = false;
      const fa_raw_t<SRC> w = static_cast<const fa_raw_t<SRC>*>(o.src)[T.base - 1];
      unordered |= !(kfirst > fa_decode_ref<SRC, true, REF>(m, o.pv, w, b2).key);
    }
    if (__ballot(odd != 0 || unordered) && lane == 0) atomicOr(&g.flags[1], 1u);
  }
  uint32_t carry = wave_shr1(linc), tm = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    const uint32_t w = (uint32_t)sh.w[x];
    if (x < (int)wid) carry = w > carry ? w : carry;
    tm = w > tm ? w : tm;
  }
  uint32_t flags = 0, dsum = 0;  // dsum: key - run over the starts (the tile's first excluded)
  {
    uint32_t rn = carry;
#pragma unroll
    for (int k = 0; k < TI; ++k) {
      const bool f = rk[k] > rn || (k == 0 && e0 == 0);
      flags |= (f ? 1u : 0u) << k;
      dsum += __builtin_elementwise_sub_sat(rk[k], rn);  // key - run of a start, 0 otherwise (and for the tile's first)
      rn = sk[k] > rn ? sk[k] : rn;
    }
  }
  const uint32_t lcnt = (uint32_t)__popc(flags);
  const uint32_t cinc = wave_scan_dpp<false>(lcnt);
  // the wave's last start: its global index (the tile's last start has every other start of the tile before it)
  const unsigned long long hasf = __ballot(flags != 0);
  unsigned long long jl = 0;
  if (hasf) {
    const int ll = 63 - __builtin_clzll(hasf);
    const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)flags, ll);
    jl = T.base + (uint64_t)(wid * 64 + ll) * TI + (31 - __clz(fl)) + 1;  // + 1: 0 = none
  }
  // per-thread records -> wave sums (DPP), then LDS
  const uint32_t s0 = wave_sum_dpp(n0), s1 = wave_sum_dpp(n1), sc = wave_sum_dpp(nc), sd = wave_sum_dpp(dsum);
  if (lane == 63) {
    sh.c[wid] = cinc;
    sh.red[wid][0] = s0;
    sh.red[wid][1] = s1;
    sh.red[wid][2] = sc;
    sh.red[wid][3] = sd;
    sh.red[wid][4] = jl;
  }
  __syncthreads();
  uint64_t cpre = 0, cagg = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    if (x < (int)wid) cpre += sh.c[x];
    cagg += sh.c[x];
  }
  const uint64_t lb = cpre + (cinc - lcnt);
  if (lb < (uint64_t)KL && flags) {  // the tile's first KL local starts (absolute key, running max before it)
    uint64_t rank = lb;
    uint32_t rn = carry;
#pragma unroll
    for (int k = 0; k < TI; ++k) {
      if (((flags >> k) & 1u) && rank < (uint64_t)KL) {
        klist[2 * rank] = base + rk[k];
        klist[2 * rank + 1] = (k == 0 && e0 == 0) ? 0ull : base + rn;
      }
      rank += (flags >> k) & 1u;
      rn = sk[k] > rn ? sk[k] : rn;
    }
  }
  if (threadIdx.x < FPW + 1) {
    const uint32_t f = threadIdx.x;
    unsigned long long x = 0;
    if (f == FPART) {
      x = cagg;
    } else if (f == FPART + 1) {  // hmax = 2j - (starts before j) at the last start j > 0
      unsigned long long j = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) j = sh.red[w][4] > j ? sh.red[w][4] : j;
      x = j > 1 ? 2 * (j - 1) - (cagg - 1) : 0ull;
    } else if (f == FPW) {
      x = tm == 0xFFFFFFFFu ? KEY_EMPTY : base + tm;
    } else if (f == 1) {  // traversed: -base (the first start, nothing before it) - sum(key - run)
#pragma unroll
      for (int w = 0; w < NW; ++w) x += sh.red[w][3];
      x = 0ull - base - x;
    } else {  // 0: cold (tid 0) of case 2 when it is cold; 2..4: case 0/1/2 counts (case 2 when not cold)
      unsigned long long a0 = 0, a1 = 0, ac = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        a0 += sh.red[w][0];
        a1 += sh.red[w][1];
        ac += sh.red[w][2];
      }
      const bool cold2 = r[2] == 0xFFFFFFFFu;
      x = f == 0 ? (cold2 ? ac : 0ull) : f == 2 ? a0 : f == 3 ? a1 : (cold2 ? 0ull : TILE - a0 - a1);
    }
    sh.out[f] = x;
  }
  __syncthreads();
}

// ---- pass 1: every tile as if nothing entered it.  The fast path (a full
// tile of a shape with FaRefs::fast whose keys lie within 2^32 - 1 minus the
// longest reuse of its first key; tile-uniform) in k_fa_local_fast; the tiles
// it leaves (partial or wide ones) and shapes without it in k_fa_local.
template <int SRC, bool CHECK, uint32_t REF>
__device__ __forceinline__ bool fa_local_try_fast(const Model& m, const FaOne& o, const KeyGen& kg,
                                                  FaLds<SRC, TB, TI>& sh, unsigned long long* __restrict__ klist,
                                                  GTable g) {
  fa_rt(m, o.pv, sh);
  if constexpr (SRC != SRC_GEN) {
    const fa_raw_t<SRC>* src = static_cast<const fa_raw_t<SRC>*>(o.src) + o.T.base;
#pragma unroll
    for (int k = 0; k < TI; ++k) sh.raw[fa_slot_n<TI>((uint32_t)k * TB + threadIdx.x)] = src[k * TB + threadIdx.x];
  }
  if (threadIdx.x < 2) {  // the first and the last key, in 64 bits
    const uint32_t e = threadIdx.x ? TILE - 1 : 0;
    bool b2 = false;
    if constexpr (SRC == SRC_GEN)
      sh.kb[threadIdx.x] = elem_of_digits<true>(m, o.pv, REF, keygen_digits_at(kg, o.T.base + e)).key;
    else
      sh.kb[threadIdx.x] = fa_decode_ref<SRC, true, REF>(m, o.pv, src_at<SRC>(o, e), b2).key;
  }
  __syncthreads();
  const unsigned long long base = sh.kb[0], kl = sh.kb[1];
  uint32_t r[3];
  unsigned long long rmax = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const unsigned long long x = sh.rt[c];
    r[c] = x == KEY_EMPTY ? 0xFFFFFFFFu : (uint32_t)x;
    rmax = x != KEY_EMPTY && x > rmax ? x : rmax;
  }
  if (kl >= base && kl - base < 0xFFFFFFFFull - rmax && r[0] != 0xFFFFFFFFu && r[1] != 0xFFFFFFFFu &&
      (SRC != SRC_GEN || keyrun_fast_ok(kg, o.T.base, TILE))) {
    fa_local_fast<SRC, CHECK, REF>(m, o, kg, sh, base, r, klist + blockIdx.x * (uint64_t)(2 * KL), g);
    return true;
  }
  return false;
}

template <int SRC, bool P2, bool CHECK, uint32_t REF, bool FULLT>
__device__ __forceinline__ void fa_local_tile(const Model& m, const FaOne& o, const KeyGen& kg, uint64_t gt,
                                              FaLds<SRC, TB, TI>& sh, unsigned long long* __restrict__ tmax,
                                              unsigned long long* __restrict__ part,
                                              unsigned long long* __restrict__ klist, GTable g) {
  unsigned long long* kl_out = klist + gt * (uint64_t)(2 * KL);
  fa_rt(m, o.pv, sh);
  unsigned long long key[TI];
  uint32_t cases, t0s;
  bool bad = false;
  fa_load_run<SRC, P2, REF, TB, TI, FULLT>(m, o, kg, sh, key, cases, t0s, bad);
  bool unordered = false;
  if constexpr (CHECK) unordered = fa_unordered<SRC, P2, REF, TB, TI, FULLT>(m, o, key, sh, bad);
  if (SRC == SRC_SAMPLES && __ballot(bad || unordered) && __lane_id() == 0) atomicOr(&g.flags[1], 1u);
  // the tile's first and last keys: the 32-bit path when every key and
  // non-cold sink lies within 2^32 - 1 of the first (tile-uniform)
  {
    const uint32_t e0 = threadIdx.x * TI, last = o.T.mt - 1;
    if (threadIdx.x == 0) sh.kb[0] = key[0];
    if (last >= e0 && last < e0 + TI) {
#pragma unroll
      for (int k = 0; k < TI; ++k)
        if (e0 + k == last) sh.kb[1] = key[k];
    }
  }
  __syncthreads();
  const unsigned long long base = sh.kb[0], kl = sh.kb[1];
  unsigned long long rmax = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) rmax = sh.rt[c] != KEY_EMPTY && sh.rt[c] > rmax ? sh.rt[c] : rmax;
  if (kl >= base && kl - base < 0xFFFFFFFFull - rmax)  // (a flagged list's result is never read)
    fa_scan_local32<SRC, TB, TI, FULLT>(o, key, cases, t0s, base, sh, kl_out);
  else
    fa_scan<FA_LOCAL, SRC, TB, TI, FULLT>(m, o, key, cases, t0s, 0, 0, sh, kl_out);
  if (threadIdx.x < FPW) part[gt * FPW + threadIdx.x] = sh.out[threadIdx.x];
  if (threadIdx.x == FPW) tmax[gt] = sh.out[FPW];
}

// Per-reference dispatch (tile-uniform switch; the reference's view, source
// and generator copied out of the kernel argument inside its branch).
#define PLUSS_FA_REFS(BODY)            \
  switch (T.r) {                       \
    case C0: { BODY(C0); } break;      \
    case C1: { BODY(C1); } break;      \
    case A0: { BODY(A0); } break;      \
    case B0: { BODY(B0); } break;      \
    case C2: { BODY(C2); } break;      \
    default: { BODY(C3); } break;      \
  }
template <int SRC, uint32_t R>
__device__ __forceinline__ FaOne fa_one_ref(const FaRefs& a, const FaTile& T) {
  FaOne o;
  o.T = T;
  o.n = a.n[R];
  o.src = a.src[R];
  o.pv = a.pv[R];
  return o;
}

// Tiles: every tile (list == nullptr), or the tiles queued in list (list[0]
// = count, then tile indices; a grid of resident workgroups over it).
template <int SRC, bool P2, bool CHECK, bool LIST>
__global__ __launch_bounds__(TB) void k_fa_local(Model m, FaRefs a, unsigned long long* __restrict__ tmax,
                                                 unsigned long long* __restrict__ part,
                                                 unsigned long long* __restrict__ klist, unsigned long long* slots,
                                                 const unsigned int* list, GTable g) {
  __shared__ FaLds<SRC, TB, TI> sh;
  const uint32_t nl = LIST ? list[0] : 1u;
  for (uint32_t q = LIST ? blockIdx.x : 0u; q < nl; q += gridDim.x) {
    const uint64_t gt = LIST ? list[1 + q] : blockIdx.x;
    const FaTile T = fa_tile(a, gt);
    if (!LIST) fa_cold_slot(T, g, slots);
#define PLUSS_FA_LOCAL(R)                                                                                 \
  const FaOne o = fa_one_ref<SRC, R>(a, T);                                                               \
  KeyGen kg;                                                                                              \
  if constexpr (SRC == SRC_GEN) kg = a.kg[R];                                                             \
  if (T.mt == TILE) fa_local_tile<SRC, P2, CHECK, R, true>(m, o, kg, gt, sh, tmax, part, klist, g);       \
  else fa_local_tile<SRC, P2, CHECK, R, false>(m, o, kg, gt, sh, tmax, part, klist, g);
    PLUSS_FA_REFS(PLUSS_FA_LOCAL)
#undef PLUSS_FA_LOCAL
    __syncthreads();  // sh is reused by the next queued tile
  }
}

// The fast path over every tile (shapes with FaRefs::fast); the tiles it
// cannot take are queued in slowq for k_fa_local.
template <int SRC, bool CHECK>
__global__ __launch_bounds__(TB) void k_fa_local_fast(Model m, FaRefs a, unsigned long long* __restrict__ tmax,
                                                      unsigned long long* __restrict__ part,
                                                      unsigned long long* __restrict__ klist,
                                                      unsigned long long* slots, unsigned int* slowq, GTable g) {
  __shared__ FaLds<SRC, TB, TI> sh;
  const FaTile T = fa_tile(a, blockIdx.x);
  fa_cold_slot(T, g, slots);
  bool done = false;
  if (T.mt == TILE) {
#define PLUSS_FA_FAST(R)                                            \
  const FaOne o = fa_one_ref<SRC, R>(a, T);                         \
  KeyGen kg;                                                        \
  if constexpr (SRC == SRC_GEN) kg = a.kg[R];                       \
  done = fa_local_try_fast<SRC, CHECK, R>(m, o, kg, sh, klist, g);
    PLUSS_FA_REFS(PLUSS_FA_FAST)
#undef PLUSS_FA_FAST
  }
  if (done) {
    if (threadIdx.x < FPW) part[blockIdx.x * (uint64_t)FPW + threadIdx.x] = sh.out[threadIdx.x];
    if (threadIdx.x == FPW) tmax[blockIdx.x] = sh.out[FPW];
  } else if (threadIdx.x == 0) {
    slowq[1 + atomicAdd(&slowq[0], 1u)] = (unsigned int)blockIdx.x;
  }
}

// ---- pass 3: the carry entering each tile applied to its local results (one
// wave per tile).  A tile whose KL stored starts are all absorbed while it has
// more is queued for k_fa_rescan (queue[0] = count, then tile indices).
constexpr int FIXB = 256;
template <int SRC>  // (instantiated in each source's translation unit)
__global__ __launch_bounds__(FIXB) void k_fa_fix(FaRefs a, const unsigned long long* __restrict__ pmin,
                                                 unsigned long long* __restrict__ part,
                                                 const unsigned long long* __restrict__ klist, unsigned int* queue) {
  const uint32_t lane = __lane_id();
  const uint64_t t = (uint64_t)blockIdx.x * (FIXB / 64) + (threadIdx.x >> 6);
  if (t >= a.toff[6]) return;                 // wave-uniform
  const FaTile T = fa_tile(a, t);
  if (T.lt == 0) return;                      // the reference's first tile: nothing enters it
  const unsigned long long c = pmin[t];
  unsigned long long* pt = part + t * FPW;
  const uint64_t cnt = pt[FPART];
  const uint32_t nl = cnt < (uint64_t)KL ? (uint32_t)cnt : (uint32_t)KL;
  const unsigned long long* kl = klist + t * (uint64_t)(2 * KL);
  unsigned long long k = KEY_EMPTY, lp = 0;
  if (lane < nl) {
    k = kl[2 * lane];
    lp = kl[2 * lane + 1];
  }
  const bool absorbed = lane < nl && k <= c;
  const uint32_t mm = (uint32_t)__popcll(__ballot(absorbed));  // keys increase: the absorbed starts are a prefix
  if (mm == nl && cnt > nl) {
    if (lane == 0) queue[1 + atomicAdd(&queue[0], 1u)] = (unsigned int)t;
    return;
  }
  const unsigned long long dsum = sc_wave_red<false>(absorbed ? lp - k : 0ull);
  const unsigned long long lpm = __shfl(lp, (int)(mm < 64 ? mm : 0), 64);  // the first surviving start's
  if (lane == 0) {
    const bool any = mm < cnt;
    pt[1] = pt[1] - dsum + (any ? (c > lpm ? c : lpm) - lpm : 0ull);
    pt[FPART] = cnt - mm;
    pt[FPART + 1] = any ? pt[FPART + 1] + mm : 0ull;
  }
}

// ---- pass 4: the queued tiles scanned again with the running max entering
// them (a grid of resident workgroups over the queue; empty queue: nothing)
template <int SRC, bool P2>
__global__ __launch_bounds__(TB) void k_fa_rescan(Model m, FaRefs a, const unsigned long long* __restrict__ pmin,
                                                  unsigned long long* __restrict__ part, const unsigned int* queue) {
  __shared__ FaLds<SRC, TB, TI> sh;
  const uint32_t nq = queue[0];
  for (uint32_t q = blockIdx.x; q < nq; q += gridDim.x) {
    const uint64_t gt = queue[1 + q];
    const FaTile T = fa_tile(a, gt);
    const unsigned long long c = pmin[gt];
#define PLUSS_FA_RESCAN(R)                                                                                  \
  const FaOne o = fa_one_ref<SRC, R>(a, T);                                                                 \
  KeyGen kg;                                                                                                \
  if constexpr (SRC == SRC_GEN) kg = a.kg[R];                                                               \
  unsigned long long key[TI];                                                                               \
  uint32_t cases, t0s;                                                                                      \
  bool bad = false;                                                                                         \
  fa_rt(m, o.pv, sh);                                                                                       \
  if (T.mt == TILE) {                                                                                       \
    fa_load_run<SRC, P2, R, TB, TI, true>(m, o, kg, sh, key, cases, t0s, bad);                              \
    fa_scan<FA_FULL, SRC, TB, TI, true>(m, o, key, cases, t0s, c, 0, sh, nullptr);                          \
  } else {                                                                                                  \
    fa_load_run<SRC, P2, R, TB, TI, false>(m, o, kg, sh, key, cases, t0s, bad);                             \
    fa_scan<FA_FULL, SRC, TB, TI, false>(m, o, key, cases, t0s, c, 0, sh, nullptr);                         \
  }
    PLUSS_FA_REFS(PLUSS_FA_RESCAN)
#undef PLUSS_FA_RESCAN
    if (threadIdx.x < FPW) part[gt * FPW + threadIdx.x] = sh.out[threadIdx.x];
    __syncthreads();  // sh is reused by the next queued tile
  }
}

// ---- pass 5, one workgroup of FT threads per reference with samples: the
// exclusive sum of its tiles' start counts locates the tile holding the Q1
// cut (the first with hmax >= n + starts before it); the tiles before it are
// summed whole, that tile is scanned again with its incoming start count
// (FA_CUT; FT threads x TILE/FT elements); then Q3 (nothing dropped: the owner
// of the final largest sink stays in LAT, +1 cold if it is tid 0), the -1
// key (materialised even with 0, r10:196,671), traversed (+ the end of the
// last replay when nothing was cut) and the bins.
constexpr int FT = 1024;
template <int SRC, bool P2>
__global__ __launch_bounds__(FT) void k_fa_finish(Model m, FaRefs a, const unsigned long long* __restrict__ tmax,
                                                  const unsigned long long* __restrict__ pmin,
                                                  const unsigned long long* __restrict__ part,
                                                  const unsigned long long* __restrict__ slots, GTable g) {
  constexpr int NW = FT / 64;
  __shared__ FaLds<SRC, FT, TILE / FT> sh;
  __shared__ unsigned long long s_ct, s_red[NW][FPART];
  const uint32_t r = blockIdx.x;
  const uint64_t n = a.n[r];
  if (n == 0) return;
  const uint64_t t0 = a.toff[r], nt = a.toff[r + 1] - t0;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  // read early (latency): the cold key's slot, the last tile's sinks (Q3)
  const unsigned long long slot = slots[r];
  const unsigned long long gl = tmax[t0 + nt - 1] > pmin[t0 + nt - 1] ? tmax[t0 + nt - 1] : pmin[t0 + nt - 1];
  // 1. the cut tile; the partials of the tiles before it are summed on the way
  uint64_t ct = nt, cin = 0, c = 0;
  unsigned long long v[FPART] = {0, 0, 0, 0, 0};
  if (nt > FT) {  // many tiles (2^24+ samples per reference): each thread a contiguous run of them
    const uint64_t per = (nt + FT - 1) / FT;
    const uint64_t lo = threadIdx.x * per < nt ? threadIdx.x * per : nt, hi = lo + per < nt ? lo + per : nt;
    const unsigned long long* pt = part + t0 * FPW;
    constexpr int FB = 8;  // loads of a batch in flight together
    unsigned long long cs = 0;
    for (uint64_t t = lo; t < hi; t += FB) {
      unsigned long long x[FB];
#pragma unroll
      for (int k = 0; k < FB; ++k) x[k] = t + k < hi ? pt[(t + k) * FPW + FPART] : 0ull;
#pragma unroll
      for (int k = 0; k < FB; ++k) cs += x[k];
    }
    const unsigned long long inc = sc_wave_scan<false>(cs, lane);
    if (lane == 63) sh.c[wid] = inc;
    __syncthreads();
    unsigned long long run = inc - cs;
#pragma unroll
    for (int x = 0; x < NW; ++x)
      if (x < (int)wid) run += sh.c[x];
    unsigned long long hit = KEY_EMPTY, hcin = 0;
    for (uint64_t t = lo; t < hi; t += FB) {
      unsigned long long x[FB], h[FB];
#pragma unroll
      for (int k = 0; k < FB; ++k) {
        x[k] = t + k < hi ? pt[(t + k) * FPW + FPART] : 0ull;
        h[k] = t + k < hi ? pt[(t + k) * FPW + FPART + 1] : 0ull;
      }
#pragma unroll
      for (int k = 0; k < FB; ++k) {
        if (hit == KEY_EMPTY && t + k < hi && h[k] >= n + run) {
          hit = t + k;
          hcin = run;
        }
        run += x[k];
      }
    }
    const unsigned long long cand = sc_wave_red_min(hit);
    if (lane == 0) sh.w[wid] = cand;
    __syncthreads();
    unsigned long long best = KEY_EMPTY;
#pragma unroll
    for (int x = 0; x < NW; ++x) best = sh.w[x] < best ? sh.w[x] : best;
    if (best != KEY_EMPTY && hit == best) s_ct = hcin;
    __syncthreads();
    if (best != KEY_EMPTY) {  // block-uniform
      ct = best;
      cin = s_ct;
    }
    const uint64_t hi2 = hi < ct ? hi : ct;
    for (uint64_t t = lo; t < hi2; t += FB / 2) {
      unsigned long long x[FB / 2][FPART];
#pragma unroll
      for (int k = 0; k < FB / 2; ++k)
#pragma unroll
        for (int f = 0; f < FPART; ++f) x[k][f] = t + k < hi2 ? pt[(t + k) * FPW + f] : 0ull;
#pragma unroll
      for (int k = 0; k < FB / 2; ++k)
#pragma unroll
        for (int f = 0; f < FPART; ++f) v[f] += x[k][f];
    }
  } else
  for (uint64_t b0 = 0; b0 < nt; b0 += FT) {  // one chunk: one tile per thread
    const uint64_t t = b0 + threadIdx.x;
    unsigned long long pw[FPW];
#pragma unroll
    for (int f = 0; f < FPW; ++f) pw[f] = t < nt ? part[(t0 + t) * FPW + f] : 0ull;
    const unsigned long long cnt = pw[FPART], h = pw[FPART + 1];
    const unsigned long long inc = sc_wave_scan<false>(cnt, lane);
    if (lane == 63) sh.c[wid] = inc;
    __syncthreads();
    unsigned long long pre = c, tot = 0;
#pragma unroll
    for (int x = 0; x < NW; ++x) {
      if (x < (int)wid) pre += sh.c[x];
      tot += sh.c[x];
    }
    const unsigned long long excl = pre + inc - cnt;
    const bool hit = t < nt && h >= n + excl;
    const unsigned long long cand = sc_wave_red_min(hit ? t : KEY_EMPTY);
    if (lane == 0) sh.w[wid] = cand;
    __syncthreads();
    unsigned long long best = KEY_EMPTY;
#pragma unroll
    for (int x = 0; x < NW; ++x) best = sh.w[x] < best ? sh.w[x] : best;
    if (best == KEY_EMPTY || t < best)
#pragma unroll
      for (int f = 0; f < FPART; ++f) v[f] += pw[f];
    if (best != KEY_EMPTY) {  // block-uniform
      if (t == best) s_ct = excl;
      __syncthreads();
      ct = best;
      cin = s_ct;
      break;
    }
    c += tot;
    __syncthreads();  // sh.c / sh.w are rewritten by the next chunk
  }
#pragma unroll
  for (int f = 0; f < FPART; ++f) {
    v[f] = sc_wave_red<false>(v[f]);
    if (lane == 0) s_red[wid][f] = v[f];
  }
  // 2. the cut tile, below the cut
  uint64_t cut = n;
  if (ct < nt) {
    __syncthreads();
    const FaTile T = fa_tile(a, t0 + ct);
    const unsigned long long carry = pmin[t0 + ct];
    constexpr int FE = TILE / FT;
#define PLUSS_FA_CUT(R)                                                                                     \
  const FaOne o = fa_one_ref<SRC, R>(a, T);                                                                 \
  KeyGen kg;                                                                                                \
  if constexpr (SRC == SRC_GEN) kg = a.kg[R];                                                               \
  unsigned long long key[FE];                                                                               \
  uint32_t cases, t0s;                                                                                      \
  bool bad = false;                                                                                         \
  fa_rt(m, o.pv, sh);                                                                                       \
  if (T.mt == TILE) {                                                                                       \
    fa_load_run<SRC, P2, R, FT, FE, true>(m, o, kg, sh, key, cases, t0s, bad);                              \
    fa_scan<FA_CUT, SRC, FT, FE, true>(m, o, key, cases, t0s, carry, cin, sh, nullptr);                     \
  } else {                                                                                                  \
    fa_load_run<SRC, P2, R, FT, FE, false>(m, o, kg, sh, key, cases, t0s, bad);                             \
    fa_scan<FA_CUT, SRC, FT, FE, false>(m, o, key, cases, t0s, carry, cin, sh, nullptr);                    \
  }
    PLUSS_FA_REFS(PLUSS_FA_CUT)
#undef PLUSS_FA_CUT
  }
  __syncthreads();
  if (threadIdx.x < FPART) {  // one sum per thread, then plain no-return atomics
    const uint32_t f = threadIdx.x;
    unsigned long long x = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) x += s_red[w][f];
    if (ct < nt) {
      x += sh.out[f];
      cut = sh.out[FPART];
    }
    if (f == 0) {  // cold; Q3: +1 when nothing was cut and the final largest sink's owner is tid 0
      const unsigned long long tid = P2 ? (gl & (m.T - 1)) : gl % m.T;
      if (cut == n && gl != KEY_EMPTY && tid == 0) x += 1;
      if (slot != ~0ull && x) atomicAdd(&g.counts[slot], x);
    } else if (f == 1) {  // the last replay ends at the end of the list (no cut): its running max
      if (cut == n) x += gl == KEY_EMPTY ? m.A * m.T : gl;
      atomicAdd(&g.trav[r], x);
    } else if (x) {
      atomicAdd(&g.bins[r * 3 + (f - 2)], x);
    }
  }
}
#undef PLUSS_FA_REFS

// ---- launching the pipeline for one element source (each source's kernels
// are instantiated in their own translation unit, pluss_fa_<src>.hip)
struct FaLaunch {
  Model m;
  FaRefs a;
  GTable g;
  FaithfulBufs* b;
  bool p2;      // shift decoding (fa_run)
  uint64_t t;   // tiles of all references
  hipStream_t s;
};

template <int SRC, bool CHK, bool P2>
inline void fa_launch_t(const FaLaunch& L) {
  FaithfulBufs& b = *L.b;
  const unsigned t = (unsigned)L.t;
  const unsigned nfix = (unsigned)((L.t + FIXB / 64 - 1) / (FIXB / 64));
  const unsigned nres = t < 512 ? t : 512u;
  if (P2 && L.a.fast) {  // fast tiles, then the queued rest
    hipLaunchKernelGGL((k_fa_local_fast<SRC, CHK>), dim3(t), dim3(TB), 0, L.s, L.m, L.a, b.tmax, b.dpart, b.klist,
                       b.fslot, b.slowq, L.g);
    hipLaunchKernelGGL((k_fa_local<SRC, P2, CHK, true>), dim3(nres), dim3(TB), 0, L.s, L.m, L.a, b.tmax, b.dpart,
                       b.klist, b.fslot, (const unsigned int*)b.slowq, L.g);
  } else {
    hipLaunchKernelGGL((k_fa_local<SRC, P2, CHK, false>), dim3(t), dim3(TB), 0, L.s, L.m, L.a, b.tmax, b.dpart, b.klist,
                       b.fslot, (const unsigned int*)nullptr, L.g);
  }
  hipLaunchKernelGGL(k_fa_prefix<SRC>, dim3(6), dim3(PB), 0, L.s, L.a, b.tmax, b.pmin, b.queue, b.slowq);
  hipLaunchKernelGGL(k_fa_fix<SRC>, dim3(nfix), dim3(FIXB), 0, L.s, L.a, b.pmin, b.dpart, b.klist, b.queue);
  hipLaunchKernelGGL((k_fa_rescan<SRC, P2>), dim3(nres), dim3(TB), 0, L.s, L.m, L.a, b.pmin, b.dpart, b.queue);
  hipLaunchKernelGGL((k_fa_finish<SRC, P2>), dim3(6), dim3(FT), 0, L.s, L.m, L.a, b.tmax, b.pmin, b.dpart, b.fslot,
                     L.g);
}

// the four sources (pluss_fa_w32.hip, pluss_fa_w64.hip, pluss_fa_smp.hip, pluss_fa_gen.hip)
void fa_launch_w32(const FaLaunch& L);
void fa_launch_w64(const FaLaunch& L);
void fa_launch_smp(const FaLaunch& L);
void fa_launch_gen(const FaLaunch& L);

}  // namespace pluss
