// pluss_faithful.h — FAITHFUL mode's one-GPU scan pipeline (k_fa_*): the
// device code shared by the per-source translation units (pluss_fa_*.hip, one
// element source each, compiled in parallel) and the host side in
// pluss_faithful.hip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <type_traits>

#include "pluss_device.h"
#include "pluss_uniform.h"

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
//   k_fa_chunk   per chunk of CH tiles: the running max c entering each tile
//                (the chunk's maxima published and looked back at, then a scan
//                inside the chunk), the fix-up of each tile's results for its
//                c (below), and the chunk's summary;
//   k_fa_finish  one workgroup per reference: the exclusive sum of the start
//                counts over chunks, then tiles, locates the tile holding the
//                Q1 cut (the condition j - starts_before_j >= n - j is monotone
//                in j), everything before it is summed, that tile is scanned
//                again below the cut; Q3, the -1 key, traversed, the bins.
// HBM traffic: the elements once, plus per tile a few words and its list.
constexpr int TB = 256, TI = 16;            // threads per tile, elements per thread
constexpr uint32_t TILE = TB * TI;          // elements per tile
constexpr int FPART = 5;                    // per tile: cold (tid 0), traversed, case 0/1/2 counts
constexpr int FPW = FPART + 2;              // ... + the start count and the Q1 bound hmax
constexpr int KL = 64;                      // local starts kept per tile (one wave lane each)
__host__ __device__ inline uint64_t fa_tiles(uint64_t n) { return (n + TILE - 1) / TILE; }

enum : int { SRC_W32 = 0, SRC_W64 = 1, SRC_SAMPLES = 2, SRC_GEN = 3, SRC_UNI = 4, SRC_W32P = 5 };
// SRC_W32P: the radix sort's output as 4-byte payloads (words past 32 bits
// without their top-level digit); a payload's word is its parent bucket's
// digit put back, looked up from the sort's parents (FaRefs::ppar, w32p_*)
static_assert(TILE == UG_TILE, "the uniform generator stages the pipeline's tiles");
// sources whose elements are packed samples (SRC_UNI: generated into LDS from the plan)
template <int SRC>
constexpr bool fa_smp() { return SRC == SRC_SAMPLES || SRC == SRC_UNI; }
enum : int { FA_LOCAL = 0, FA_FULL = 1, FA_CUT = 2 };

// A key-range shard's exchange (include/pluss_gpu.h, PLUSS_SHARD_ROW): every
// phase writes words of this shard's summary row; the next phase reads the
// rows of all shards (gathered by the caller) and k_fa_xchg derives this
// shard's inputs into xin.
enum : int {
  ROW_N = 0,       // [6] samples of each reference in the shard (phase 1)
  ROW_MAX = 6,     // [6] the shard's largest sink per reference (phase 1; 0: none)
  ROW_STARTS = 12, // [6] replay starts in the shard (phase 2)
  ROW_CUT = 18,    // [6] the shard's first Q1 cut candidate, global index (phase 3; the list length: none)
  ROW_ERR = 31,    // nonzero: the shard failed a phase (set by the caller)
  ROW_W = 32
};
enum : int {
  XIN_CIN = 0,     // [6] the largest sink of the earlier shards with samples (0: none)
  XIN_SOFF = 6,    // [6] the replay starts of the earlier shards
  XIN_CUT = 12,    // [6] the global cut (the smallest candidate over the shards)
  XIN_LAST = 18,   // [6] no later shard has samples of the reference
  XIN_FAIL = 24,   // some shard's row carries an error word
  XIN_W = 32
};

struct FaRefs {
  uint64_t n[6];
  uint64_t toff[7];    // first (global) tile of each reference; toff[6] = all tiles
  uint64_t coff[7];    // first chunk (CH tiles) of each reference; coff[6] = all chunks
  // key-range shards (multi-GPU; one GPU: joff 0, ntot = n, xin null): the global
  // index of this shard's element 0 in the reference's list, the list's length;
  // xin (device memory, k_fa_xchg from the gathered summary rows): the running
  // max of sinks entering the shard, the starts before it, the global cut, the
  // last-shard flags, a failed-shard flag (XIN_* below)
  uint64_t joff[6], ntot[6];
  const unsigned long long* xin;
  const void* src[6];  // SRC_W*: sorted packed words; SRC_SAMPLES: the key-ordered samples
  PkView pv[6];
  KeyGen kg[6];        // SRC_GEN
  const UniSet* us;    // SRC_UNI: the plan of the uniform key-order lists (device memory)
  // SRC_W32P: the sort's parents (device memory; reference r's are ppar[ppb[r], ppb[r] + ppn[r]), their
  // starts in the concatenated lists, peoff[r] = reference r's first; a parent b's words are b << phi[r] | payload)
  const SrtParent* ppar;
  uint32_t ppb[6], ppn[6], phi[6];
  uint64_t peoff[6];
  uint32_t fast;       // the local pass's fast path applies to the shape (fa_run)
  uint32_t unidec;     // SRC_UNI: keys below 2^61 and leaf key spans below 2^32 (uni_stage DEC)
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
// an element as it is in memory (SRC_W32P: the 4-byte payload of a 64-bit word)
template <int SRC>
using fa_mem_t = typename std::conditional<SRC == SRC_W32 || SRC == SRC_W32P, uint32_t, unsigned long long>::type;

// the tile's reference (wave-uniform) and its place in it
struct FaTile {
  uint32_t r;
  uint64_t gt;        // tile index over all references
  uint64_t lt, base;  // tile index within the reference (shard), its first element (in memory)
  uint64_t gbase;     // the global index of its first element (base + the shard's joff)
  uint32_t mt;        // elements in the tile
};
__device__ __forceinline__ FaTile fa_tile(const FaRefs& a, uint64_t gt) {
  uint32_t r = 0;
#pragma unroll
  for (int x = 1; x < 6; ++x) r += gt >= a.toff[x] ? 1u : 0u;
  r = __builtin_amdgcn_readfirstlane(r);
  FaTile t;
  t.r = r;
  t.gt = gt;
  t.lt = gt - a.toff[r];
  t.base = t.lt * TILE;
  t.gbase = a.joff[r] + t.base;
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
  if constexpr (fa_smp<SRC>()) return elem_of_sample_ref<REF, P2>(m, v, (uint64_t)w, bad);
  else return elem_of_word<P2>(m, v, REF, w);
}

// the reference's first tile also materialises its -1 (cold) key in the main
// table and keeps the slot, so the finish pass only adds the count
__device__ __forceinline__ void fa_cold_slot(const FaTile& T, GTable g, unsigned long long* slots) {
  if (T.lt == 0 && threadIdx.x == 0) slots[T.r] = g_slot(g, make_key(T.r, 0, -1));
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
  uint32_t cand[SRC == SRC_UNI ? UG_CAND : 1];  // the uniform generator's scratch (uni_stage)
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
  const UniSet* us;
  const SrtParent* ppar;  // SRC_W32P: this reference's parents
  uint32_t pn, phi;
  uint64_t peoff;
};

// SRC_W32P: the parent holding element i of the reference (the last parent
// whose start is at most i; empty parents share their successor's start)
__device__ __forceinline__ uint32_t w32p_find(const FaOne& o, uint64_t i) {
  uint32_t lo = 0, hi = o.pn;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint64_t)o.ppar[mid].start - o.peoff <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}
// a tile's prefixes: its elements [base, base + mt) lie in at most two parents
// (ok; elements below B in the first), else each element looks its parent up
struct W32P {
  unsigned long long pa, pb;
  uint64_t B;
  bool ok;
};
// (every wave by itself: its lanes read the parents' starts at once and count
// those at or below the tile's first and last elements; starts never decrease)
__device__ __forceinline__ W32P w32p_tile(const FaOne& o, uint64_t base, uint32_t mt) {
  W32P w;
  const uint64_t lastx = base + (mt ? mt - 1 : 0);
  uint32_t n0 = 0, n1 = 0;
  for (uint32_t j0 = 0; j0 < o.pn; j0 += 64) {
    const uint32_t j = j0 + __lane_id();
    const uint64_t st = j < o.pn ? (uint64_t)o.ppar[j].start - o.peoff : ~0ull;
    n0 += (uint32_t)__popcll(__ballot(st <= base));
    n1 += (uint32_t)__popcll(__ballot(st <= lastx));
  }
  const uint32_t b0 = n0 ? n0 - 1 : 0, b1 = n1 ? n1 - 1 : 0;
  w.pa = (unsigned long long)b0 << o.phi;
  w.pb = (unsigned long long)b1 << o.phi;
  w.B = b1 > b0 ? (uint64_t)o.ppar[b1].start - o.peoff : ~0ull;
  w.ok = b1 <= b0 + 1;  // (an empty parent between them: each element looks up its own)
  return w;
}
__device__ __forceinline__ unsigned long long w32p_word(const FaOne& o, const W32P& w, uint64_t i, uint32_t v) {
  if (w.ok) return (i < w.B ? w.pa : w.pb) | v;
  return ((unsigned long long)w32p_find(o, i) << o.phi) | v;
}

// This thread's run of the tile: keys (KEY_EMPTY past the end), cases (2 bits
// at 2k) and tid == 0 flags (bit 2k).  Memory sources: coalesced loads
// (thread x, round k: element k*NT + x) staged in LDS, read back as runs;
// generated lists: each thread generates its run (keyrunf_* when the whole
// tile lies in block A with small strata -- tile-uniform -- else one direct
// decode per sample).
// (RANGE8: SRC_W32P tiles over three to nine parents take the parents' starts
// in registers -- the queued pass; the chunk and finish passes' rare rescans
// look each element's parent up, which keeps their registers below the
// point where the compiler reserved a scratch slot in them)
template <int SRC, bool P2, uint32_t REF, int NT, int EPT, bool FULLT, bool RANGE8 = true>
__device__ __forceinline__ void fa_load_run(const Model& m, const FaOne& o, const KeyGen& kg, FaLds<SRC, NT, EPT>& sh,
                                            unsigned long long (&key)[EPT], uint32_t& cases, uint32_t& t0s,
                                            bool& bad) {
  const FaTile& T = o.T;
  const uint32_t e0 = threadIdx.x * EPT;
  cases = 0;
  t0s = 0;
  if constexpr (SRC != SRC_GEN) {
    if constexpr (SRC == SRC_UNI) {
      // (generated into sh.raw by fa_uni_pre, once, before the per-reference dispatch)
    } else {
      const fa_mem_t<SRC>* src = static_cast<const fa_mem_t<SRC>*>(o.src) + T.base;
      fa_mem_t<SRC> v[EPT];  // every load issued before the first wait (partial tiles: clamped, no branch)
      const uint32_t last = T.mt - 1;
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const uint32_t e = (uint32_t)k * NT + threadIdx.x;
        v[k] = src[FULLT ? e : (e < last ? e : last)];
      }
      if constexpr (SRC == SRC_W32P) {  // the payloads' parent digits put back
        const W32P pw = w32p_tile(o, T.base, T.mt);
        const uint32_t b0 = (uint32_t)(pw.pa >> o.phi), b1 = (uint32_t)(pw.pb >> o.phi);
        if (!RANGE8 || pw.ok || b1 - b0 > 8u) {
#pragma unroll
          for (int k = 0; k < EPT; ++k) {
            const uint32_t e = (uint32_t)k * NT + threadIdx.x;
            sh.raw[fa_slot_n<EPT>(e)] = w32p_word(o, pw, T.base + (e < last ? e : last), v[k]);
          }
        } else {
          // a tile over three to nine parents (a sparse reference's, like C0's):
          // the starts of parents b0+1..b1 read once, each element's parent is b0
          // plus the starts at or below it (no search through memory per element)
          uint64_t st[8];
#pragma unroll
          for (uint32_t x = 0; x < 8; ++x) st[x] = b0 + 1 + x <= b1 ? (uint64_t)o.ppar[b0 + 1 + x].start - o.peoff : ~0ull;
#pragma unroll
          for (int k = 0; k < EPT; ++k) {
            const uint32_t e = (uint32_t)k * NT + threadIdx.x;
            const uint64_t i = T.base + (e < last ? e : last);
            uint32_t q = b0;
#pragma unroll
            for (uint32_t x = 0; x < 8; ++x) q += st[x] <= i ? 1u : 0u;
            sh.raw[fa_slot_n<EPT>(e)] = ((unsigned long long)q << o.phi) | v[k];
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) sh.raw[fa_slot_n<EPT>((uint32_t)k * NT + threadIdx.x)] = v[k];
      }
      __syncthreads();
    }
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
    if (keyrun_fast_ok(kg, T.gbase, TILE)) {  // a whole tile: every run is in range
      KeyRunF run;
      keyrunf_start(kg, run, T.gbase + e0);
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
          const Elem x = elem_of_digits<P2>(m, o.pv, REF, keygen_digits_at(kg, T.gbase + e0 + k));
          key[k] = x.key;
          cases |= x.c << (2 * k);
          t0s |= x.t0 << (2 * k);
        }
      }
    }
  }
}

// SRC_UNI: the tile generated into sh.raw (packed samples, runs of EPT per
// thread), before the kernels' per-reference dispatch (one copy of the
// generator per kernel, not one per reference)
template <int SRC, int NT, int EPT>
__device__ __forceinline__ void fa_uni_pre(const FaRefs& a, const FaTile& T, FaLds<SRC, NT, EPT>& sh) {
  if constexpr (SRC == SRC_UNI)
    uni_stage<NT, false>(a.us, T.r, T.lt, T.mt, sh.raw, sh.cand, a.us->flags,
                         [](uint32_t e) { return fa_slot_n<EPT>(e); });
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
  const uint64_t i0 = T.gbase + e0;                                             // global index of its first element
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
  const uint64_t i0 = T.gbase + e0;
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
  unsigned long long ord;  // (q*N + c1) << 32 | c2 << tsh | tid: increasing with the key (CHECK)
};

template <uint32_t REF>
__device__ __forceinline__ FaDec fa_dec_digits(const Model& m, const PkView& v, uint32_t q, uint32_t c1, uint32_t c2,
                                               uint32_t t) {
  FaDec d;
  const uint32_t qc = (q << v.nsh) | c1;
  d.lk = ((__umul24(qc, m.S) + ref_off(REF, c2)) << v.tsh) | t;
  d.ord = ((unsigned long long)qc << 32) | ((c2 << v.tsh) | t);
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
template <uint32_t REF>
__device__ __forceinline__ FaDec fa_dec_sample(const Model& m, const PkView& v, uint64_t x, uint32_t& odd) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  odd |= ((hi ^ (REF << 28)) & (0xF0000000u | m.badhi)) | (lo & m.badlo);
  const uint32_t c2 = (REF == C0 || REF == C1) ? 0u : (lo & 0xFFFFFu);
  const uint32_t c1 = __builtin_amdgcn_alignbit(hi, lo, 20) & 0xFFFFFu;
  const uint32_t cs = m.csshift, ts = v.tsh;
  const uint32_t t = __builtin_amdgcn_ubfe(hi, 8 + cs, ts);
  const uint32_t q = (__builtin_amdgcn_ubfe(hi, 8 + cs + ts, 20 - cs - ts) << cs) | __builtin_amdgcn_ubfe(hi, 8, cs);
  return fa_dec_digits<REF>(m, v, q, c1, c2, t);
}

// a packed sort word rank << 2 | case, rank = ((q*N + c1)*N + c2)*T + tid
template <uint32_t REF, typename KT>
__device__ __forceinline__ FaDec fa_dec_word(const Model& m, const PkView& v, KT w) {
  const uint32_t c = (uint32_t)w & 3u;
  const uint32_t t = ((uint32_t)w >> 2) & (uint32_t)(v.T - 1);
  const uint32_t c2 = (uint32_t)(w >> (2 + v.tsh)) & (uint32_t)(v.N - 1);
  const uint32_t qc = (uint32_t)(w >> (2 + v.tsh + v.nsh));
  FaDec d;
  d.ord = 0;
  d.lk = ((__umul24(qc, m.S) + ref_off(REF, c2)) << v.tsh) | t;
  d.a = c == 0;
  d.b = c == 1;
  d.t0 = t == 0;
  return d;
}

// a 4-byte payload of a longer word (SRC_W32P) whose parent's digit lies in the
// word's q*N + c1 field: pq = the digit shifted into that field (tile-uniform,
// one of two), so the decode stays in 32 bits like fa_dec_word's
template <uint32_t REF>
__device__ __forceinline__ FaDec fa_dec_w32p(const Model& m, const PkView& v, uint32_t w, uint32_t pq) {
  const uint32_t c = w & 3u;
  const uint32_t t = (w >> 2) & (uint32_t)(v.T - 1);
  const uint32_t c2 = (w >> (2 + v.tsh)) & (uint32_t)(v.N - 1);
  const uint32_t qc = pq | (w >> (2 + v.tsh + v.nsh));
  FaDec d;
  d.ord = 0;
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

// ri*T per case in 32 bits (0xFFFFFFFF: cold), as three fields: never an
// indexed array, which the compiler may place in scratch
struct FaRi {
  uint32_t r0, r1, r2;
};

// The scan of one tile by the fast path (mt elements: FULLT, or a partial
// tile's elements at e < mt).  `el(k)` decodes this thread's element k.
template <int SRC, bool CHECK, uint32_t REF, bool FULLT, class EL>
__device__ __forceinline__ void fa_local_fast(const Model& m, const FaOne& o, FaLds<SRC, TB, TI>& sh,
                                              unsigned long long base, const FaRi r, EL&& el,
                                              unsigned long long* __restrict__ klist, GTable g) {
  constexpr int NW = TB / 64;
  const FaTile& T = o.T;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t e0 = threadIdx.x * TI;
  const uint32_t nv = FULLT ? TI : (e0 < T.mt ? (T.mt - e0 < TI ? T.mt - e0 : TI) : 0u);
  static_assert(!CHECK, "generated lists are in key order by construction (the order check is fa_lane_tile's)");
  const uint32_t b32 = (uint32_t)base;
  uint32_t rk[TI], sk[TI], lmax = 0;
  uint32_t w0 = 0, w1 = 0, wc = 0;  // wave counts (ballots): case 0, case 1, case 2 of tid 0
#pragma unroll
  for (int k = 0; k < TI; ++k) {
    const bool v = FULLT || (uint32_t)k < nv;
    uint32_t oddk = 0;
    const FaDec d = el(k, oddk);
    rk[k] = v ? d.lk - b32 : 0u;
    const uint32_t dd = d.a ? r.r0 : (d.b ? r.r1 : r.r2);  // selects (an array here went to scratch)
    const uint32_t x = rk[k] + dd;  // dd = 0xFFFFFFFF (cold) wraps below dd: the max keeps it
    sk[k] = v ? (x > dd ? x : dd) : 0u;
    lmax = sk[k] > lmax ? sk[k] : lmax;
    w0 += (uint32_t)__popcll(__ballot(v && d.a));
    w1 += (uint32_t)__popcll(__ballot(v && !d.a && d.b));
    wc += (uint32_t)__popcll(__ballot(v && !d.a && !d.b && d.t0));
  }
  // running max of sinks entering this lane
  const uint32_t linc = wave_scan_dpp<true>(lmax);
  if (lane == 63) sh.w[wid] = linc;
  __syncthreads();
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
    jl = T.gbase + (uint64_t)(wid * 64 + ll) * TI + (31 - __clz(fl)) + 1;  // + 1: 0 = none
  }
  const uint32_t sd = wave_sum_dpp(dsum);
  if (lane == 63) {
    sh.c[wid] = cinc;
    sh.red[wid][0] = w0;
    sh.red[wid][1] = w1;
    sh.red[wid][2] = wc;
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
      const bool cold2 = r.r2 == 0xFFFFFFFFu;
      x = f == 0 ? (cold2 ? ac : 0ull) : f == 2 ? a0 : f == 3 ? a1 : (cold2 ? 0ull : T.mt - a0 - a1);
    }
    sh.out[f] = x;
  }
  __syncthreads();
}

template <int SRC>
__device__ __forceinline__ const void* fa_src_of(const FaRefs& a, uint32_t r) {
  // selects, not a switch (which can become an indexed load of the kernel
  // argument, and an indexed argument is copied to scratch)
  const void* p = a.src[0];
#pragma unroll
  for (uint32_t x = 1; x < 6; ++x) p = r == x ? a.src[x] : p;
  return p;
}

template <int SRC, uint32_t R>
__device__ __forceinline__ FaOne fa_one_ref(const FaRefs& a, const FaTile& T);

// One tile of the stratified generated lists by the thread-major fast path:
// the first and last keys in 64 bits, then the scan if the tile qualifies.
// Returns whether the fast path took the tile (tile-uniform).  (Lists in
// memory and the uniform lists take the lane-major path, fa_lane_tile.)
template <int SRC, bool CHECK, uint32_t REF>
__device__ __forceinline__ bool fa_fast_tile(const Model& m, const FaRefs& a, const FaTile& T,
                                             FaLds<SRC, TB, TI>& sh, unsigned long long* __restrict__ klist,
                                             GTable g) {
  static_assert(SRC == SRC_GEN, "the thread-major fast path serves the stratified generated lists");
  const FaOne o = fa_one_ref<SRC, REF>(a, T);
  const KeyGen kg = a.kg[REF];
  fa_rt(m, o.pv, sh);
  const bool full = T.mt == TILE;
  if (threadIdx.x < 2) {  // the first and the last key, in 64 bits
    const uint32_t e = threadIdx.x ? T.mt - 1 : 0;
    sh.kb[threadIdx.x] = elem_of_digits<true>(m, o.pv, REF, keygen_digits_at(kg, T.gbase + e)).key;
  }
  __syncthreads();
  const unsigned long long base = sh.kb[0], kl = sh.kb[1];
  unsigned long long rmax = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const unsigned long long x = sh.rt[c];
    rmax = x != KEY_EMPTY && x > rmax ? x : rmax;
  }
  auto r32 = [](unsigned long long x) { return x == KEY_EMPTY ? 0xFFFFFFFFu : (uint32_t)x; };
  const FaRi r{r32(sh.rt[0]), r32(sh.rt[1]), r32(sh.rt[2])};
  if (!(kl >= base && kl - base < 0xFFFFFFFFull - rmax && r.r0 != 0xFFFFFFFFu && r.r1 != 0xFFFFFFFFu &&
        keyrun_fast_ok(kg, T.gbase, T.mt)))
    return false;
  unsigned long long* kl_out = klist + T.gt * (uint64_t)(2 * KL);
  const uint32_t e0 = threadIdx.x * TI;
  KeyRunF run;
  keyrunf_start(kg, run, T.gbase + (e0 < T.mt ? e0 : 0u));
  auto el = [&](int, uint32_t&) -> FaDec {
    const KeyDigits dg = keyrunf_digits(kg, run);
    keyrunf_next(kg, run);
    return fa_dec_digits<REF>(m, o.pv, dg.q, dg.c1, dg.c2, dg.t);
  };
  if (full) fa_local_fast<SRC, CHECK, REF, true>(m, o, sh, base, r, el, kl_out, g);
  else fa_local_fast<SRC, CHECK, REF, false>(m, o, sh, base, r, el, kl_out, g);
  return true;
}

// ---- the fast path of memory sources, lane-major (k_fa_local_lm): wave w
// scans elements [1024w, 1024w + 1024) of the tile in 16 steps, lane L of
// step k holding element 1024w + 64k + L, loaded straight into registers
// (coalesced, all 16 loads issued before the first is used) -- no LDS staging
// of the tile, so occupancy is set by registers alone.  Per step: the decode,
// the sink, and a DPP max-scan of the sinks over the lanes (the running max
// before each lane within the step); the waves' largest sinks are exchanged
// once, and a second sweep over the kept offsets finds the starts.  The
// tile's first and last keys are decoded by every wave (two uniform loads):
// no barrier before the scan.  Results as fa_local_fast's.
template <int NT>  // threads of the workgroup (NT / 64 waves, TILE / NT steps each)
struct FaLm {
  unsigned long long out[FPW + 1];
  unsigned long long ordl[NT / 64];       // each wave's last element's order word (CHECK)
  unsigned long long red[NT / 64][6];     // per wave: starts, case 0, case 1, case 2 of tid 0, sum(key - run), last start + 1
  uint32_t wmax[NT / 64];                 // each wave's largest sink (offset)
  uint32_t kl[NT / 64][KL][2];            // each wave's first KL starts: key offset, running max before it
};

// (SRC_UNI: the tile generated into LDS first, `tile`, element e at tile[e])
// a uniform tile's staged element (uni_stage DEC): the key's low 32 bits and the case flags, no decode
__device__ __forceinline__ FaDec fa_dec_staged(unsigned long long w) {
  FaDec d;
  d.lk = (uint32_t)w;
  const uint32_t h = (uint32_t)(w >> 32);
  d.a = (h & 1u) != 0;
  d.b = (h & 2u) != 0;
  d.t0 = (h & 4u) != 0;
  d.ord = 0;
  return d;
}

template <int SRC, bool CHECK, uint32_t REF, bool FULLT, int NT>
__device__ __forceinline__ bool fa_lane_tile(const Model& m, const FaRefs& a, const FaTile& T, FaLm<NT>& sh,
                                             unsigned long long* __restrict__ klist, GTable g,
                                             const fa_raw_t<SRC>* tile = nullptr) {
  constexpr int NW = NT / 64, ST = TILE / NT;  // waves, steps per wave
  const FaOne o = fa_one_ref<SRC, REF>(a, T);
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const fa_raw_t<SRC>* src = SRC == SRC_UNI ? tile : static_cast<const fa_raw_t<SRC>*>(o.src) + T.base;
  const fa_mem_t<SRC>* msrc = static_cast<const fa_mem_t<SRC>*>(o.src) + T.base;  // (SRC_W32P: the payloads)
  const uint32_t last = T.mt - 1, e0 = wid * (64 * ST) + lane;
  fa_mem_t<SRC> v[ST];  // (SRC_W32P: the payloads; each word is made where it is decoded)
  W32P pw{};
  uint32_t be = 0xFFFFFFFFu;  // SRC_W32P: tile elements below be are in the first parent
  uint32_t qa = 0, qb = 0;    // ... and their parents' digits in the q*N + c1 field
  if constexpr (SRC == SRC_W32P) {
    pw = w32p_tile(o, T.base, T.mt);
    if (!pw.ok) return false;  // (more than two parents in the tile: the queued pass)
    be = pw.B - T.base > (uint64_t)TILE ? 0xFFFFFFFFu : (uint32_t)(pw.B - T.base);
    const uint32_t qs = 2 + o.pv.tsh + o.pv.nsh;  // (the host's condition: o.phi >= qs)
    qa = (uint32_t)(pw.pa >> qs);
    qb = (uint32_t)(pw.pb >> qs);
  }
#pragma unroll
  for (int k = 0; k < ST; ++k) {
    const uint32_t e = e0 + 64u * k;
    if constexpr (SRC == SRC_UNI) (void)e;  // (staged in LDS: each step reads its element where it decodes it)
    else if constexpr (SRC == SRC_W32P) v[k] = __builtin_nontemporal_load(msrc + (e < last ? e : last));
    else v[k] = __builtin_nontemporal_load(src + (e < last ? e : last));
  }
  // ri*T per case (0xFFFFFFFF: cold) and the tile's first and last keys, in every wave
  auto rt = [&](int c) -> unsigned long long {
    const int64_t ri = c == 0 ? o.pv.ri[0] : (c == 1 ? o.pv.ri[1] : o.pv.ri[2]);
    return ri < 0 ? KEY_EMPTY : (unsigned long long)ri * m.T;
  };
  const unsigned long long t0 = rt(0), t1 = rt(1), t2 = rt(2);
  unsigned long long rmax = 0;
  rmax = t0 != KEY_EMPTY && t0 > rmax ? t0 : rmax;
  rmax = t1 != KEY_EMPTY && t1 > rmax ? t1 : rmax;
  rmax = t2 != KEY_EMPTY && t2 > rmax ? t2 : rmax;
  bool b2 = false;
  // (SRC_UNI: a staged element holds its whole key, the high bits from bit 35)
  auto key_of = [&](fa_raw_t<SRC> w) -> unsigned long long {
    if constexpr (SRC == SRC_UNI) return ((unsigned long long)(w >> 35) << 32) | (uint32_t)w;
    else return fa_decode_ref<SRC, true, REF>(m, o.pv, w, b2).key;
  };
  unsigned long long base, kl;
  if constexpr (SRC == SRC_W32P) {
    base = key_of(pw.pa | msrc[0]);
    kl = key_of(pw.pb | msrc[last]);
  } else {
    base = key_of(src[0]);
    kl = key_of(src[last]);
  }
  auto r32 = [](unsigned long long x) { return x == KEY_EMPTY ? 0xFFFFFFFFu : (uint32_t)x; };
  const FaRi r{r32(t0), r32(t1), r32(t2)};
  if (!(kl >= base && kl - base < 0xFFFFFFFFull - rmax && r.r0 != 0xFFFFFFFFu && r.r1 != 0xFFFFFFFFu))
    return false;  // (the same decision in every wave)
  const uint32_t b32 = (uint32_t)base;
  // sweep 1: offsets, sinks, the running max of sinks before each lane within the wave
  uint32_t rk[ST], ex[ST], wm = 0, odd = 0;
  uint32_t w01 = 0, wc = 0, unord = 0;  // w01: case 0 | case 1 << 16; wc: case 2 of tid 0
  unsigned long long oprev = 0, ofirst = 0;
#pragma unroll
  for (int k = 0; k < ST; ++k) {
    const bool val = FULLT || e0 + 64u * k <= last;
    uint32_t oddk = 0;
    FaDec d;
    if constexpr (SRC == SRC_UNI) {
      const uint32_t e = e0 + 64u * k;
      d = fa_dec_staged(src[e < last ? e : last]);
    }
    else if constexpr (fa_smp<SRC>()) d = fa_dec_sample<REF>(m, o.pv, (uint64_t)v[k], oddk);
    else if constexpr (SRC == SRC_W32P) d = fa_dec_w32p<REF>(m, o.pv, v[k], e0 + 64u * k < be ? qa : qb);
    else d = fa_dec_word<REF>(m, o.pv, v[k]);
    odd |= val ? oddk : 0u;
    if (CHECK) {  // against the previous lane (the step before: its lane 63); integer
                  // arithmetic, not compare masks (which the unrolled steps kept in SGPRs)
      const uint32_t plo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)d.ord, 0x138, 0xf, 0xf, false);
      const uint32_t phi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(d.ord >> 32), 0x138, 0xf, 0xf, false);
      unsigned long long up = ((unsigned long long)phi << 32) | plo;
      if (lane == 0) up = k > 0 ? oprev : d.ord - 1;  // (the wave's first element: checked after the barrier)
      if (k == 0) ofirst = d.ord;
      const uint32_t bad = (uint32_t)((d.ord - up - 1) >> 63);  // ord <= up (orders stay below 2^56)
      unord |= val ? bad : 0u;
      oprev = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(d.ord >> 32), 63) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)d.ord, 63);
    }
    rk[k] = val ? d.lk - b32 : 0u;
    const uint32_t dd = d.a ? r.r0 : (d.b ? r.r1 : r.r2);
    const uint32_t x = rk[k] + dd;  // cold: dd = 0xFFFFFFFF, the max keeps it
    const uint32_t s = val ? (x > dd ? x : dd) : 0u;
    const uint32_t inc = wave_scan_dpp<true>(s), xk = wave_shr1(inc);
    ex[k] = xk > wm ? xk : wm;  // (the steps before: wm)
    const uint32_t sm = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    wm = sm > wm ? sm : wm;
    // per-lane counts (not ballots: every step's compare masks held in SGPRs spilled them)
    w01 += val ? (d.a ? 1u : (d.b ? 0x10000u : 0u)) : 0u;
    wc += (val && !d.a && !d.b && d.t0) ? 1u : 0u;
    // the checks are reduced step by step: left to their use after the
    // barrier, the compiler kept every step's raw element and order word live
    __asm__ volatile("" : "+v"(odd), "+v"(unord), "+v"(w01), "+v"(wc));
    __builtin_amdgcn_sched_barrier(0);  // one step at a time: hoisted decodes held every step's case masks in SGPRs
  }
  if (lane == 0) {
    sh.wmax[wid] = wm;
    sh.ordl[wid] = oprev;
  }
  __syncthreads();
  uint32_t pm = 0, tm = 0;  // the running max entering this wave; the tile's largest sink
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    const uint32_t w = sh.wmax[x];
    if (x < (int)wid) pm = w > pm ? w : pm;
    tm = w > tm ? w : tm;
  }
  if (CHECK) {  // the wave's first element against the element before it (the previous wave's last, or the tile's)
    bool unordered = unord != 0;
    if (lane == 0 && e0 <= last) {
      if (wid > 0) {
        unordered |= !(ofirst > sh.ordl[wid - 1]);
      } else if (T.base > 0) {
        uint32_t o2 = 0;
        unordered |= !(ofirst > fa_dec_sample<REF>(m, o.pv, (uint64_t)src[-1], o2).ord);
      }
    }
    if (__ballot(odd != 0 || unordered) && lane == 0) atomicOr(&g.flags[1], 1u);
  }
  // sweep 2: the starts (the tile's first element is one), their sum(key - run), the wave's first KL
  uint32_t dsum = 0, cnt = 0, kc = 0;
  unsigned long long jl = 0;
#pragma unroll
  for (int k = 0; k < ST; ++k) {
    const uint32_t rn = ex[k] > pm ? ex[k] : pm;  // (pm: the earlier waves)
    const bool st = rk[k] > rn || (k == 0 && e0 == 0);
    dsum += __builtin_elementwise_sub_sat(rk[k], rn);
    const unsigned long long bal = __ballot(st);
    if (bal) {
      const uint32_t nb = (uint32_t)__popcll(bal);
      jl = T.gbase + (uint64_t)(wid * (64 * ST) + 64 * k + (63 - __builtin_clzll(bal))) + 1;
      if (kc < (uint32_t)KL) {
        const uint32_t rank = kc + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (st && rank < (uint32_t)KL) {
          sh.kl[wid][rank][0] = rk[k];
          sh.kl[wid][rank][1] = rn;
        }
        kc += nb;
      }
      cnt += nb;
    }
  }
  const uint32_t sd = wave_sum_dpp(dsum), s01 = wave_sum_dpp(w01), sc = wave_sum_dpp(wc);
  if (lane == 0) {
    sh.red[wid][0] = cnt;
    sh.red[wid][1] = s01 & 0xFFFFu;
    sh.red[wid][2] = s01 >> 16;
    sh.red[wid][3] = sc;
    sh.red[wid][4] = sd;
    sh.red[wid][5] = jl;
  }
  __syncthreads();
  uint64_t cagg = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) cagg += sh.red[x][0];
  if (threadIdx.x < (uint32_t)KL) {  // the tile's first KL starts: the waves' lists in order
    const uint32_t i = threadIdx.x;
    uint64_t s0 = 0;
#pragma unroll
    for (int x = 0; x < NW; ++x) {
      const uint64_t c = sh.red[x][0];
      if (i >= s0 && i < s0 + c) {
        klist[2 * i] = base + sh.kl[x][i - s0][0];
        klist[2 * i + 1] = i == 0 ? 0ull : base + sh.kl[x][i - s0][1];
      }
      s0 += c;
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
      for (int w = 0; w < NW; ++w) j = sh.red[w][5] > j ? sh.red[w][5] : j;
      x = j > 1 ? 2 * (j - 1) - (cagg - 1) : 0ull;
    } else if (f == FPW) {
      x = tm == 0xFFFFFFFFu ? KEY_EMPTY : base + tm;
    } else if (f == 1) {
#pragma unroll
      for (int w = 0; w < NW; ++w) x += sh.red[w][4];
      x = 0ull - base - x;
    } else {
      unsigned long long a0 = 0, a1 = 0, ac = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        a0 += sh.red[w][1];
        a1 += sh.red[w][2];
        ac += sh.red[w][3];
      }
      const bool cold2 = r.r2 == 0xFFFFFFFFu;
      x = f == 0 ? (cold2 ? ac : 0ull) : f == 2 ? a0 : f == 3 ? a1 : (cold2 ? 0ull : T.mt - a0 - a1);
    }
    sh.out[f] = x;
  }
  __syncthreads();
  return true;
}

// ---- pass 1: every tile as if nothing entered it.  The fast path (a full
// tile of a shape with FaRefs::fast whose keys lie within 2^32 - 1 minus the
// longest reuse of its first key; tile-uniform) in k_fa_local_fast; the tiles
// it leaves (partial or wide ones) and shapes without it in k_fa_local.
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
  o.n = a.ntot[R];  // the reference's whole list (all shards)
  o.src = a.src[R];
  o.pv = a.pv[R];
  o.us = a.us;
  o.ppar = a.ppar ? a.ppar + a.ppb[R] : nullptr;
  o.pn = a.ppn[R];
  o.phi = a.phi[R];
  o.peoff = a.peoff[R];
  return o;
}

// Tiles: every tile (list == nullptr), or the tiles queued in list (list[0]
// = count, then tile indices; a grid of resident workgroups over it).
template <int SRC, bool P2, bool CHECK, bool LIST>
__global__ __launch_bounds__(TB) void k_fa_local(Model m, FaRefs a, unsigned long long* __restrict__ tmax,
                                                 unsigned long long* __restrict__ part,
                                                 unsigned long long* __restrict__ klist, unsigned long long* slots,
                                                 unsigned int* list, GTable g) {
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
    fa_uni_pre<SRC>(a, T, sh);
    PLUSS_FA_REFS(PLUSS_FA_LOCAL)
#undef PLUSS_FA_LOCAL
    __syncthreads();  // sh is reused by the next queued tile
  }
}

// The fast path over every tile (shapes with FaRefs::fast), one tile per
// workgroup; the tiles it cannot take are queued in slowq for k_fa_local.
// (A resident grid that loads the next tile into registers while scanning the
// current one ran at 2 waves per SIMD and was 1.4x slower at config 3: the
// scan's dependent chains need the 4 waves per SIMD of this form to issue.)
template <int SRC>
constexpr bool fa_mem() { return SRC == SRC_W32 || SRC == SRC_W64 || SRC == SRC_W32P || SRC == SRC_SAMPLES; }

template <int SRC, bool CHECK>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(4))) void k_fa_local_fast(Model m, FaRefs a, unsigned long long* __restrict__ tmax,
                                                      unsigned long long* __restrict__ part,
                                                      unsigned long long* __restrict__ klist,
                                                      unsigned long long* slots, unsigned int* slowq, GTable g) {
  static_assert(SRC == SRC_GEN, "lists in memory and uniform lists: k_fa_local_lm");
  __shared__ FaLds<SRC, TB, TI> sh;
  const FaTile T = fa_tile(a, blockIdx.x);
  fa_cold_slot(T, g, slots);
  bool done = false;
#define PLUSS_FA_FAST(R) done = fa_fast_tile<SRC, CHECK, R>(m, a, T, sh, klist, g);
  PLUSS_FA_REFS(PLUSS_FA_FAST)
#undef PLUSS_FA_FAST
  if (done) {
    if (threadIdx.x < FPW) part[blockIdx.x * (uint64_t)FPW + threadIdx.x] = sh.out[threadIdx.x];
    if (threadIdx.x == FPW) tmax[blockIdx.x] = sh.out[FPW];
  } else if (threadIdx.x == 0) {
    slowq[1 + atomicAdd(&slowq[0], 1u)] = (unsigned int)blockIdx.x;
  }
}

// The lane-major fast path over every tile of a memory source (fa_lane_tile);
// the tiles it cannot take are queued in slowq for k_fa_local.
// SRC_UNI: the tile is first generated into LDS (uni_stage, in key order), then
// scanned lane-major.  (512 threads per tile, so that each of a tile's ~258
// leaves had its own thread, ran 1.5x slower at config 3: 2 workgroups per CU.)
template <int SRC>
constexpr int fa_lm_nt() { return TB; }
template <int SRC>
struct FaLmLds {
  FaLm<fa_lm_nt<SRC>()> s;
  fa_raw_t<SRC> raw[SRC == SRC_UNI ? TILE : 1];  // (SRC_UNI: staged elements, uni_stage DEC)
  uint32_t cand[SRC == SRC_UNI ? UG_CAND : 1];
};
template <int SRC>
constexpr bool fa_lm() { return fa_mem<SRC>() || SRC == SRC_UNI; }

// waves per SIMD asked of the compiler: lists in memory fit 8 (<= 64 VGPRs and
// <= 80 SGPRs: at 83 SGPRs the SGPR file held 7); the uniform staging fits 4
// (127 VGPRs, no scratch: no product kernel may request scratch, DESIGN.md
// section 8, r5p) with its register network at 30 candidates (UG_NET), its
// per-leaf values computed where they are used and the tile's constants read
// again after it; at 3 waves (145 VGPRs) the config-3 pass took 2.58 ms, at 4
// 2.42 ms (r6r)
template <int SRC>
constexpr int fa_lm_waves() { return SRC == SRC_UNI || SRC == SRC_W32P ? 4 : 8; }
// (the references' partial last tiles of lists in memory go to the queued
// pass: every list at the BASELINE shapes already queues C0's and C1's tiles,
// whose keys span more than 32 bits, so a launch of their own for the partial
// tiles only added a kernel to the pass, r5 ab1)
template <int SRC, bool CHECK>
__global__ __launch_bounds__(fa_lm_nt<SRC>()) __attribute__((amdgpu_waves_per_eu(fa_lm_waves<SRC>()))) void k_fa_local_lm(Model m, FaRefs a, unsigned long long* __restrict__ tmax,
                                                    unsigned long long* __restrict__ part,
                                                    unsigned long long* __restrict__ klist, unsigned long long* slots,
                                                    unsigned int* slowq, GTable g, uint32_t g0) {
  static_assert(fa_lm<SRC>(), "the stratified generated source: k_fa_local_fast");
  constexpr int NT = fa_lm_nt<SRC>();
  __shared__ FaLmLds<SRC> L;
  FaLm<NT>& sh = L.s;
  const FaTile T = fa_tile(a, g0 + blockIdx.x);  // (g0: tiles before it run elsewhere, FaLaunch::side)
  fa_cold_slot(T, g, slots);
  unsigned long long* kl_out = klist + T.gt * (uint64_t)(2 * KL);
  bool done = false;
  // lists in memory: full tiles only, the few partial ones (a reference's last
  // tile) go to the slow pass, which keeps the kernel's registers at the full
  // tile's (8 waves per SIMD; with the partial-tile path in the same kernel: 85
  // VGPRs, 5 waves).  The uniform source takes its partial tiles here too (its
  // occupancy is set by the staging's registers and LDS either way; in the
  // slow pass they cost ~60 us per pass)
  if constexpr (SRC == SRC_UNI) {
    {
      // (T, N and their shifts are the same in every reference's view)
      const UniDec dz{(uint32_t)m.N, (uint32_t)m.W - 1u, a.pv[0].Q, (uint32_t)m.S, a.pv[0].nsh, a.pv[0].tsh};
      // (the leaf table of the two-phase emission lives in the scan's own LDS,
      // unused until the staging is done)
      uni_stage<NT, true>(a.us, T.r, T.lt, T.mt, L.raw, L.cand, a.us->flags, [](uint32_t e) { return e; }, dz,
                          reinterpret_cast<unsigned long long*>(&L.s), (uint32_t)(sizeof(L.s) / 8));
    }
    // the tile's constants read again for the scan (an opaque tile number: held
    // through the staging, they pushed it past 128 VGPRs into scratch)
    uint32_t bid = g0 + blockIdx.x;
    asm volatile("" : "+s"(bid));
    const FaTile T2 = fa_tile(a, bid);
    unsigned long long* kl2 = klist + T2.gt * (uint64_t)(2 * KL);
#define PLUSS_FA_LM(R)                                                                               \
  if (T2.mt == TILE) done = fa_lane_tile<SRC, CHECK, R, true, NT>(m, a, T2, sh, kl2, g, L.raw);     \
  else done = fa_lane_tile<SRC, CHECK, R, false, NT>(m, a, T2, sh, kl2, g, L.raw);
    PLUSS_FA_REFS(PLUSS_FA_LM)
#undef PLUSS_FA_LM
  } else if (T.mt == TILE) {
#define PLUSS_FA_LM(R) done = fa_lane_tile<SRC, CHECK, R, true, NT>(m, a, T, sh, kl_out, g, L.raw);
    PLUSS_FA_REFS(PLUSS_FA_LM)
#undef PLUSS_FA_LM
  }
  const uint64_t gt = g0 + blockIdx.x;  // (== T.gt)
  if (done) {
    if (threadIdx.x < FPW) part[gt * FPW + threadIdx.x] = sh.out[threadIdx.x];
    if (threadIdx.x == FPW) tmax[gt] = sh.out[FPW];
  } else if (threadIdx.x == 0) {
    slowq[1 + atomicAdd(&slowq[0], 1u)] = (unsigned int)gt;
  }
}

// ---- pass 2, one workgroup per chunk of CH tiles (thread i: tile i of the
// chunk): the chunk's largest sink is published at once (cval, cflag = this
// pass's epoch), the running max entering the chunk is the max over the
// reference's earlier chunks (a look-back over published values that never
// waits on anything but those publications), and the exclusive max scan over
// the chunk's tiles gives each tile's carry c (pmin).  Then the fix-up: with c
// entering, element i starts iff key_i > max(c, lp_{i-1}) (lp: the tile's own
// running max).  A local start stays a start iff key_i > c, a local non-start
// stays one, and keys increase, so c absorbs exactly the tile's first m local
// starts; the first surviving start's replay-before term becomes max(c, lp)
// and every later running max is the local one.  So the start count, hmax
// and traversed follow from the stored list; a tile whose whole stored list is
// absorbed while it has more starts is scanned again here by the workgroup
// (rare).  Last, the chunk's record for the finish: its start count, the
// largest hmax - (the chunk's starts before that tile), the records and
// traversed summed.
constexpr int CH = 256;  // tiles per chunk (== TB: the workgroup rescans a tile with the same threads)
constexpr int CW = 7;    // words of a chunk record: start count, h', cold, traversed, case 0/1/2 counts
static_assert(CH == TB, "a chunk workgroup is a tile workgroup");
__host__ __device__ inline uint64_t fa_chunks(uint64_t tiles) { return (tiles + CH - 1) / CH; }

__device__ __forceinline__ uint32_t fa_chunk_ref(const FaRefs& a, uint64_t c) {
  uint32_t r = 0;
#pragma unroll
  for (int x = 1; x < 6; ++x) r += c >= a.coff[x] ? 1u : 0u;
  return __builtin_amdgcn_readfirstlane(r);
}

// block-wide (CH threads) inclusive scan of one value per thread; returns (inclusive, aggregate)
template <bool MAX>
__device__ __forceinline__ void fa_block_scan(unsigned long long v, unsigned long long* sw, unsigned long long& inc,
                                              unsigned long long& agg) {
  constexpr int NW = CH / 64;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const unsigned long long w = sc_wave_scan<MAX>(v, lane);
  __syncthreads();  // sw is reused
  if (lane == 63) sw[wid] = w;
  __syncthreads();
  unsigned long long pre = 0, all = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    if (x < (int)wid) pre = sc_op<MAX>(pre, sw[x]);
    all = sc_op<MAX>(all, sw[x]);
  }
  inc = sc_op<MAX>(pre, w);
  agg = all;
}

template <int SRC, bool P2>
__global__ __launch_bounds__(CH) void k_fa_chunk(Model m, FaRefs a, const unsigned long long* __restrict__ tmax,
                                                 unsigned long long* __restrict__ pmin,
                                                 unsigned long long* __restrict__ part,
                                                 const unsigned long long* __restrict__ klist,
                                                 unsigned long long* __restrict__ cval, unsigned int* cflag,
                                                 unsigned long long* __restrict__ crec, uint32_t epoch,
                                                 unsigned int* slowq, GTable g) {
  __shared__ FaLds<SRC, TB, TI> sh;
  __shared__ unsigned long long sw[CH / 64], s_p;
  __shared__ unsigned int s_next;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint64_t c = blockIdx.x;
  if (c == 0 && threadIdx.x == 0) slowq[0] = 0;  // the local pass's queue was read: empty for the next pass
  const uint32_t r = fa_chunk_ref(a, c);
  const uint64_t c0 = a.coff[r], lc = c - c0;
  const uint64_t t0 = a.toff[r], nt = a.toff[r + 1] - t0;
  const uint64_t tl = lc * CH + threadIdx.x;  // tile within the reference
  const bool valid = tl < nt;
  const uint64_t t = t0 + tl;
  const unsigned long long tm = valid ? tmax[t] : 0ull;
  // 1. the chunk's largest sink, published; 2. the max over the earlier chunks
  unsigned long long inc, cmax;
  fa_block_scan<true>(tm, sw, inc, cmax);
  if (threadIdx.x == 0) {
    __hip_atomic_store(&cval[c], cmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cflag[c], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (wid == 0) {
    unsigned long long p = a.xin ? a.xin[XIN_CIN + r] : 0ull;  // what entered this shard (earlier shards' sinks)
    for (int64_t hi = (int64_t)lc - 1; hi >= 0; hi -= 64) {
      const int64_t j = hi - (int64_t)lane;
      uint32_t spins = 0;
      while (__ballot(j >= 0 && __hip_atomic_load(&cflag[c0 + j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch)) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 24)) {  // a predecessor never published: flag it and stop waiting
          if (lane == 0) atomicOr(&g.flags[0], FLAG_LOOKBACK);
          break;
        }
      }
      const unsigned long long v =
          j >= 0 ? __hip_atomic_load(&cval[c0 + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      p = sc_op<true>(p, sc_wave_red<true>(v));
    }
    if (lane == 0) s_p = p;
  }
  __syncthreads();
  // 3. the carry entering each tile: the chunk's incoming max and the tiles before it in the chunk
  const unsigned long long up = __shfl_up(inc, 1, 64);
  unsigned long long cy = s_p;
  {
    unsigned long long w = 0;  // sw: the waves' maxima
    for (int x = 0; x < (int)wid; ++x) w = sw[x] > w ? sw[x] : w;
    const unsigned long long ex = lane ? (up > w ? up : w) : w;
    cy = ex > cy ? ex : cy;
  }
  if (valid) pmin[t] = cy;
  // 4. the fix-up
  unsigned long long* pt = part + t * FPW;
  unsigned long long pv[FPW];
#pragma unroll
  for (int f = 0; f < FPW; ++f) pv[f] = valid ? pt[f] : 0ull;
  bool resc = false;
  if (valid && (tl > 0 || a.joff[r] > 0)) {  // (nothing enters the list's first tile)
    const uint64_t cnt = pv[FPART];
    const uint32_t nl = cnt < (uint64_t)KL ? (uint32_t)cnt : (uint32_t)KL;
    const unsigned long long* kl = klist + t * (uint64_t)(2 * KL);
    uint32_t mm = 0;
    unsigned long long dsum = 0, lpm = 0;
    for (; mm < nl; ++mm) {
      const unsigned long long k = kl[2 * mm], lp = kl[2 * mm + 1];
      if (k > cy) {
        lpm = lp;
        break;
      }
      dsum += lp - k;
    }
    if (mm == nl && cnt > nl) {
      resc = true;
    } else {
      const bool any = mm < cnt;
      pv[1] = pv[1] - dsum + (any ? (cy > lpm ? cy : lpm) - lpm : 0ull);
      pv[FPART] = cnt - mm;
      pv[FPART + 1] = any ? pv[FPART + 1] + mm : 0ull;
    }
  }
  // tiles whose stored starts ran out: scanned again by the whole workgroup, one by one
  while (__syncthreads_or(resc)) {
    if (threadIdx.x == 0) s_next = CH;
    __syncthreads();
    if (resc) atomicMin(&s_next, threadIdx.x);
    __syncthreads();
    const uint32_t who = s_next;
    const FaTile T = fa_tile(a, t0 + lc * CH + who);
#define PLUSS_FA_RESCAN(R)                                                                                  \
  const FaOne o = fa_one_ref<SRC, R>(a, T);                                                                 \
  KeyGen kg;                                                                                                \
  if constexpr (SRC == SRC_GEN) kg = a.kg[R];                                                               \
  unsigned long long key[TI];                                                                               \
  uint32_t cases, t0s;                                                                                      \
  bool bad = false;                                                                                         \
  const unsigned long long cin = pmin[T.gt];                                                                \
  fa_rt(m, o.pv, sh);                                                                                       \
  if (T.mt == TILE) {                                                                                       \
    fa_load_run<SRC, P2, R, TB, TI, true, false>(m, o, kg, sh, key, cases, t0s, bad);                              \
    fa_scan<FA_FULL, SRC, TB, TI, true>(m, o, key, cases, t0s, cin, 0, sh, nullptr);                        \
  } else {                                                                                                  \
    fa_load_run<SRC, P2, R, TB, TI, false, false>(m, o, kg, sh, key, cases, t0s, bad);                             \
    fa_scan<FA_FULL, SRC, TB, TI, false>(m, o, key, cases, t0s, cin, 0, sh, nullptr);                       \
  }
    __threadfence_block();  // pmin of the tile (written above) is read by every thread
    __syncthreads();
    fa_uni_pre<SRC>(a, T, sh);
    PLUSS_FA_REFS(PLUSS_FA_RESCAN)
#undef PLUSS_FA_RESCAN
    if (threadIdx.x == who) {
      pv[1] = sh.out[1];
      pv[FPART] = sh.out[FPART];
      pv[FPART + 1] = sh.out[FPART + 1];
      resc = false;
    }
    __syncthreads();  // sh is reused
  }
  if (valid) {
    pt[1] = pv[1];
    pt[FPART] = pv[FPART];
    pt[FPART + 1] = pv[FPART + 1];
  }
  // 5. the chunk's record
  unsigned long long cinc, ctot;
  fa_block_scan<false>(pv[FPART], sw, cinc, ctot);
  const unsigned long long hp = pv[FPART + 1] ? pv[FPART + 1] - (cinc - pv[FPART]) : 0ull;
  const unsigned long long red[6] = {sc_wave_red<true>(hp), sc_wave_red<false>(pv[0]), sc_wave_red<false>(pv[1]),
                                     sc_wave_red<false>(pv[2]), sc_wave_red<false>(pv[3]), sc_wave_red<false>(pv[4])};
  __shared__ unsigned long long s_red[CH / 64][6];
  if (lane == 0)
#pragma unroll
    for (int f = 0; f < 6; ++f) s_red[wid][f] = red[f];
  __syncthreads();
  if (threadIdx.x < CW) {
    const uint32_t f = threadIdx.x;
    unsigned long long x = 0;
    if (f == 0) {
      x = ctot;
    } else {
#pragma unroll
      for (int w = 0; w < CH / 64; ++w) x = f == 1 ? (s_red[w][0] > x ? s_red[w][0] : x) : x + s_red[w][f - 1];
    }
    crec[c * CW + f] = x;
  }
}

// ---- pass 3, one workgroup per reference with samples: the exclusive sum of
// the chunks' start counts locates the chunk holding the Q1 cut (the first
// whose h' >= n + starts before it: the condition j - starts_before_j >= n -
// j is monotone in j), then the tile inside it the same way; the chunks and
// tiles before it are summed, that tile is scanned again with its incoming
// start count (FA_CUT); then Q3 (nothing dropped: the owner of the final
// largest sink stays in LAT, +1 cold if it is tid 0), the -1 key
// (materialised even with 0, r10:196,671), traversed (+ the end of the last
// replay when nothing was cut) and the bins.
//
// STORE (a key-range shard, pass 3 of 4): the shard's first cut candidate
// (global index; the list's length if none), the sums below it (or of the
// whole shard) and the shard's final running max go to shrec[r]; the global
// cut decides later what is recorded (k_fa_shard_apply).
constexpr int SRW = FPART + 2;  // shard record: sums (cold, traversed, case 0/1/2), the cut candidate, the final max
template <int SRC, bool P2, bool STORE>
__global__ __launch_bounds__(CH) void k_fa_finish(Model m, FaRefs a, const unsigned long long* __restrict__ tmax,
                                                  const unsigned long long* __restrict__ pmin,
                                                  const unsigned long long* __restrict__ part,
                                                  const unsigned long long* __restrict__ crec,
                                                  const unsigned long long* __restrict__ slots,
                                                  unsigned long long* __restrict__ shrec,
                                                  unsigned long long* __restrict__ row, GTable g) {
  constexpr int NW = CH / 64;
  __shared__ FaLds<SRC, TB, TI> sh;
  __shared__ unsigned long long sw[NW], s_best, s_cin, s_red[NW][FPART];
  const uint32_t r = blockIdx.x;
  if (a.n[r] == 0) return;
  const uint64_t n = a.ntot[r];  // the Q1 condition is on the whole list
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint64_t t0 = a.toff[r], nt = a.toff[r + 1] - t0;
  const uint64_t c0 = a.coff[r], nc = a.coff[r + 1] - c0;
  const unsigned long long slot = slots[r];
  const unsigned long long gl = tmax[t0 + nt - 1] > pmin[t0 + nt - 1] ? tmax[t0 + nt - 1] : pmin[t0 + nt - 1];
  unsigned long long v[FPART] = {0, 0, 0, 0, 0};  // this thread's sums: cold, traversed, case 0/1/2
  // 1. the cut chunk (blocks of CH chunks); run: starts before (earlier shards' included)
  uint64_t run = a.xin ? a.xin[XIN_SOFF + r] : 0ull, cc = nc, ccin = 0;
  for (uint64_t b0 = 0; b0 < nc && cc == nc; b0 += CH) {
    const uint64_t i = b0 + threadIdx.x;
    const bool ok = i < nc;
    unsigned long long rec[CW];
#pragma unroll
    for (int f = 0; f < CW; ++f) rec[f] = ok ? crec[(c0 + i) * CW + f] : 0ull;
    unsigned long long inc, tot;
    fa_block_scan<false>(rec[0], sw, inc, tot);
    const unsigned long long ex = run + inc - rec[0];
    const bool hit = ok && rec[1] >= n + ex;
    const unsigned long long cand = sc_wave_red_min(hit ? i : KEY_EMPTY);
    __syncthreads();
    if (threadIdx.x == 0) s_best = KEY_EMPTY;
    __syncthreads();
    if (lane == 0 && cand != KEY_EMPTY) atomicMin(&s_best, cand);
    __syncthreads();
    const unsigned long long best = s_best;
    if (hit && i == best) s_cin = ex;
    if (ok && (best == KEY_EMPTY || i < best)) {
      v[0] += rec[2];
      v[1] += rec[3];
      v[2] += rec[4];
      v[3] += rec[5];
      v[4] += rec[6];
    }
    __syncthreads();
    if (best != KEY_EMPTY) {  // block-uniform
      cc = best;
      ccin = s_cin;
    }
    run += tot;
  }
  // 2. the cut tile inside the cut chunk
  uint64_t ct = nt, cin = 0;
  if (cc < nc) {
    const uint64_t tl = cc * CH + threadIdx.x;
    const bool ok = tl < nt;
    unsigned long long pw[FPW];
#pragma unroll
    for (int f = 0; f < FPW; ++f) pw[f] = ok ? part[(t0 + tl) * FPW + f] : 0ull;
    unsigned long long inc, tot;
    fa_block_scan<false>(pw[FPART], sw, inc, tot);
    const unsigned long long ex = ccin + inc - pw[FPART];
    const bool hit = ok && pw[FPART + 1] >= n + ex;
    const unsigned long long cand = sc_wave_red_min(hit ? tl : KEY_EMPTY);
    __syncthreads();
    if (threadIdx.x == 0) s_best = KEY_EMPTY;
    __syncthreads();
    if (lane == 0 && cand != KEY_EMPTY) atomicMin(&s_best, cand);
    __syncthreads();
    const unsigned long long best = s_best;  // the chunk holds a tile that qualifies
    if (hit && tl == best) s_cin = ex;
    if (ok && tl < best)
#pragma unroll
      for (int f = 0; f < FPART; ++f) v[f] += pw[f];
    __syncthreads();
    ct = best;
    cin = s_cin;
  }
#pragma unroll
  for (int f = 0; f < FPART; ++f) {
    v[f] = sc_wave_red<false>(v[f]);
    if (lane == 0) s_red[wid][f] = v[f];
  }
  // 3. the cut tile, below the cut
  uint64_t cut = n;
  if (ct < nt) {
    __syncthreads();
    const FaTile T = fa_tile(a, t0 + ct);
    const unsigned long long carry = pmin[t0 + ct];
#define PLUSS_FA_CUT(R)                                                                                     \
  const FaOne o = fa_one_ref<SRC, R>(a, T);                                                                 \
  KeyGen kg;                                                                                                \
  if constexpr (SRC == SRC_GEN) kg = a.kg[R];                                                               \
  unsigned long long key[TI];                                                                               \
  uint32_t cases, t0s;                                                                                      \
  bool bad = false;                                                                                         \
  fa_rt(m, o.pv, sh);                                                                                       \
  if (T.mt == TILE) {                                                                                       \
    fa_load_run<SRC, P2, R, TB, TI, true, false>(m, o, kg, sh, key, cases, t0s, bad);                              \
    fa_scan<FA_CUT, SRC, TB, TI, true>(m, o, key, cases, t0s, carry, cin, sh, nullptr);                     \
  } else {                                                                                                  \
    fa_load_run<SRC, P2, R, TB, TI, false, false>(m, o, kg, sh, key, cases, t0s, bad);                             \
    fa_scan<FA_CUT, SRC, TB, TI, false>(m, o, key, cases, t0s, carry, cin, sh, nullptr);                    \
  }
    fa_uni_pre<SRC>(a, T, sh);
    PLUSS_FA_REFS(PLUSS_FA_CUT)
#undef PLUSS_FA_CUT
  }
  __syncthreads();
  if (STORE) {
    if (threadIdx.x < FPART) {
      const uint32_t f = threadIdx.x;
      unsigned long long x = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) x += s_red[w][f];
      if (ct < nt) x += sh.out[f];
      shrec[r * SRW + f] = x;
    } else if (threadIdx.x == FPART) {
      const unsigned long long cand = ct < nt ? sh.out[FPART] : n;
      shrec[r * SRW + FPART] = cand;
      row[ROW_CUT + r] = cand;  // phase 3's summary word
    } else if (threadIdx.x == FPART + 1) {
      shrec[r * SRW + FPART + 1] = gl;
    }
    return;
  }
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
// pass 4 of a key-range shard: with the global cut of each reference (the
// smallest candidate over the shards, xin), record this shard's part: nothing
// if the cut lies before it; its sums below the cut if it holds the cut; all
// of it otherwise, and, on the list's last shard with nothing cut, Q3 and the
// end of the last replay (as k_fa_finish does on one GPU).  Nothing is
// recorded when a shard failed (the pass reports the failure at the fetch).
template <int X = 0>  // (a template: instantiated only where launched)
__global__ void k_fa_shard_apply(Model m, FaRefs a, const unsigned long long* __restrict__ shrec,
                                 const unsigned long long* __restrict__ xin,
                                 const unsigned long long* __restrict__ slots, GTable g) {
  const uint32_t r = threadIdx.x;
  if (r >= 6 || a.n[r] == 0 || xin[XIN_FAIL]) return;
  const unsigned long long* sr = shrec + r * SRW;
  const uint64_t G = xin[XIN_CUT + r], start = a.joff[r], n = a.ntot[r];
  if (G > n) {  // the gathered rows disagree with this shard's list length
    atomicOr(&g.flags[0], FLAG_SHARD);
    return;
  }
  if (G < start) return;  // dropped by Q1 in an earlier shard
  unsigned long long cold = sr[0], trav = sr[1];
  if (G == n && xin[XIN_LAST + r]) {
    const unsigned long long gl = sr[FPART + 1];
    if (gl != KEY_EMPTY && gl % m.T == 0) cold += 1;
    trav += gl == KEY_EMPTY ? m.A * m.T : gl;
  }
  if (slots[r] != ~0ull && cold) atomicAdd(&g.counts[slots[r]], cold);
  atomicAdd(&g.trav[r], trav);
  for (int c = 0; c < 3; ++c)
    if (sr[2 + c]) atomicAdd(&g.bins[r * 3 + c], sr[2 + c]);
}

// phase 1's summary row: every word's default (no starts, no cut candidate:
// the list's length), then per reference its sample count and the largest of
// its tiles' sinks (0: none).  what == 1 (phase 2): the sum of its chunks'
// start counts.  what == 2 (phase 3, before the finish): the cut candidates'
// default.  One workgroup of SS_NT per reference, each thread's loads issued
// in batches of 8 (a single wave walking 16K tiles took ~25 us per launch).
constexpr int SS_NT = 1024;
template <int X = 0>  // (a template: instantiated only where launched)
__global__ __launch_bounds__(SS_NT) void k_fa_shard_sums(FaRefs a, const unsigned long long* __restrict__ tmax,
                                                        const unsigned long long* __restrict__ crec,
                                                        unsigned long long* row, int what) {
  const uint32_t r = blockIdx.x, lane = __lane_id(), wid = threadIdx.x >> 6;
  __shared__ unsigned long long sw[SS_NT / 64];
  if (what == 2) {
    if (threadIdx.x == 0) row[ROW_CUT + r] = a.ntot[r];
    return;
  }
  unsigned long long acc = 0;
  const uint64_t lo = what == 0 ? a.toff[r] : a.coff[r], hi = what == 0 ? a.toff[r + 1] : a.coff[r + 1];
  const uint64_t stride = what == 0 ? 1 : CW;
  const unsigned long long* src = what == 0 ? tmax : crec;
  for (uint64_t i0 = lo + threadIdx.x; i0 < hi; i0 += 8 * SS_NT) {
    unsigned long long v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t i = i0 + (uint64_t)k * SS_NT;
      v[k] = i < hi ? src[i * stride] : 0ull;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc = what == 0 ? (v[k] > acc ? v[k] : acc) : acc + v[k];
  }
  acc = what == 0 ? sc_wave_red<true>(acc) : sc_wave_red<false>(acc);
  if (lane == 0) sw[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long x = 0;
#pragma unroll
    for (int w = 0; w < SS_NT / 64; ++w) x = what == 0 ? (sw[w] > x ? sw[w] : x) : x + sw[w];
    if (what == 0) {
      row[ROW_N + r] = a.n[r];
      row[ROW_MAX + r] = x;
      row[ROW_STARTS + r] = 0;
      row[ROW_CUT + r] = a.ntot[r];
      if (r == 0)
        for (int w = 24; w < ROW_W; ++w) row[w] = 0;
    } else {
      row[ROW_STARTS + r] = x;
    }
  }
}

// This shard's inputs from the gathered rows of all `ns` shards (rows[s *
// ROW_W ...], shard `me`), for the phase about to run: 2 carry (the largest
// sink of the earlier shards with samples), 3 cut (the starts of the earlier
// shards), 4 hist (the global cut and whether a later shard has samples).
// Any row's error word marks the pass failed (FLAG_SHARD at the next fetch).
template <int X = 0>  // (a template: instantiated only where launched)
__global__ void k_fa_xchg(const unsigned long long* __restrict__ rows, uint32_t ns, uint32_t me, int phase,
                          unsigned long long* __restrict__ xin, GTable g) {
  const uint32_t r = threadIdx.x;
  if (r == 6) {
    unsigned long long f = 0;
    for (uint32_t s = 0; s < ns; ++s) f |= rows[(uint64_t)s * ROW_W + ROW_ERR];
    xin[XIN_FAIL] = f ? 1ull : 0ull;
    if (f) atomicOr(&g.flags[0], FLAG_SHARD);
  }
  if (r >= 6) return;
  if (phase == 2) {
    unsigned long long c = 0;
    for (uint32_t s = 0; s < me; ++s) {
      const unsigned long long* w = rows + (uint64_t)s * ROW_W;
      if (w[ROW_N + r] && w[ROW_MAX + r] > c) c = w[ROW_MAX + r];
    }
    xin[XIN_CIN + r] = c;
  } else if (phase == 3) {
    unsigned long long b = 0;
    for (uint32_t s = 0; s < me; ++s) b += rows[(uint64_t)s * ROW_W + ROW_STARTS + r];
    xin[XIN_SOFF + r] = b;
  } else {
    unsigned long long c = KEY_EMPTY, later = 0;
    for (uint32_t s = 0; s < ns; ++s) {
      const unsigned long long* w = rows + (uint64_t)s * ROW_W;
      c = w[ROW_CUT + r] < c ? w[ROW_CUT + r] : c;
      if (s > me) later |= w[ROW_N + r];
    }
    xin[XIN_CUT + r] = c;
    xin[XIN_LAST + r] = later ? 0ull : 1ull;
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
  bool p2;        // shift decoding (fa_run)
  uint64_t t;     // tiles of all references
  uint32_t epoch; // this pass's chunk-publication epoch
  int phase;      // FA_PH_*
  hipStream_t s;
  unsigned long long* row;  // a key-range shard's summary row (FA_PH_CUT writes its cut candidates)
  uint32_t side = 0;        // (SRC_UNI) tiles [0, side) -- the sparse 2-D references' -- on b->side
};

// phases of the pipeline: 1 local pass, 2 chunks (carry, fix-up), 3 finish
// (one GPU: the bins; a shard: its record), 4 a shard's record applied
enum : int { FA_PH_ALL = 0, FA_PH_LOCAL = 1, FA_PH_CHUNK = 2, FA_PH_CUT = 3, FA_PH_APPLY = 4 };

template <int SRC, bool CHK, bool P2>
inline void fa_launch_t(const FaLaunch& L) {
  FaithfulBufs& b = *L.b;
  const unsigned t = (unsigned)L.t;
  const unsigned nres = t < 512 ? t : 512u;
  const int ph = L.phase;
  if (ph == FA_PH_ALL || ph == FA_PH_LOCAL) {
    bool fast = false;
    if constexpr (P2) {  // fast tiles, then the queued rest (an empty queue: the workgroups return at once)
      if (L.a.fast && (SRC != SRC_UNI || L.a.unidec)) {
        // the queue starts empty whatever an earlier, abandoned pass left in it
        // (a pass whose chunk phase ran left it empty: no fill launch then)
        if (!b.slowq_clean) (void)hipMemsetAsync(b.slowq, 0, sizeof(unsigned int), L.s);
        b.slowq_clean = false;
        const uint32_t t0 = SRC == SRC_UNI && L.side < t ? L.side : 0u;
        if (t0) {  // the sparse references' tiles: the generic pass on the side stream, beside the lane-major one
          (void)hipEventRecord(b.sev[0], L.s);
          (void)hipStreamWaitEvent(b.side, b.sev[0], 0);
          hipLaunchKernelGGL((k_fa_local<SRC, P2, CHK, false>), dim3(t0), dim3(TB), 0, b.side, L.m, L.a, b.tmax,
                             b.dpart, b.klist, b.fslot, (unsigned int*)nullptr, L.g);
        }
        if constexpr (fa_lm<SRC>())
          hipLaunchKernelGGL((k_fa_local_lm<SRC, CHK>), dim3(t - t0), dim3(fa_lm_nt<SRC>()), 0, L.s, L.m, L.a, b.tmax, b.dpart, b.klist,
                             b.fslot, b.slowq, L.g, t0);
        else
          hipLaunchKernelGGL((k_fa_local_fast<SRC, CHK>), dim3(t), dim3(TB), 0, L.s, L.m, L.a, b.tmax, b.dpart,
                             b.klist, b.fslot, b.slowq, L.g);
        PLUSS_STAGE(L.s, "pipeline: local fast pass");
        hipLaunchKernelGGL((k_fa_local<SRC, P2, CHK, true>), dim3(nres), dim3(TB), 0, L.s, L.m, L.a, b.tmax, b.dpart,
                           b.klist, b.fslot, b.slowq, L.g);
        if (t0) {  // (joined before the chunk pass reads every tile's record)
          (void)hipEventRecord(b.sev[1], b.side);
          (void)hipStreamWaitEvent(L.s, b.sev[1], 0);
        }
        PLUSS_STAGE(L.s, "pipeline: queued pass");
        fast = true;
      }
    }
    if (!fast) {
      hipLaunchKernelGGL((k_fa_local<SRC, P2, CHK, false>), dim3(t), dim3(TB), 0, L.s, L.m, L.a, b.tmax, b.dpart,
                         b.klist, b.fslot, (unsigned int*)nullptr, L.g);
    }
  }
  if (ph == FA_PH_ALL || ph == FA_PH_CHUNK) {
    b.slowq_clean = true;  // (k_fa_chunk empties the queue)
    // a replayed graph runs with the epoch it was captured with: the chunk
    // flags start from zero in it, so no look-back reads an earlier replay's values
    if (b.capture) (void)hipMemsetAsync(b.cflag, 0, L.a.coff[6] * sizeof(unsigned int), L.s);
  }
  if (ph == FA_PH_ALL || ph == FA_PH_CHUNK)
    hipLaunchKernelGGL((k_fa_chunk<SRC, P2>), dim3((unsigned)L.a.coff[6]), dim3(CH), 0, L.s, L.m, L.a, b.tmax,
                       b.pmin, b.dpart, b.klist, b.cval, b.cflag, b.crec, L.epoch, b.slowq, L.g);
  if (ph == FA_PH_ALL || ph == FA_PH_CHUNK) PLUSS_STAGE(L.s, "pipeline: chunks");
  if (ph == FA_PH_ALL)
    hipLaunchKernelGGL((k_fa_finish<SRC, P2, false>), dim3(6), dim3(CH), 0, L.s, L.m, L.a, b.tmax, b.pmin, b.dpart,
                       b.crec, b.fslot, b.shrec, (unsigned long long*)nullptr, L.g);
  if (ph == FA_PH_CUT)
    hipLaunchKernelGGL((k_fa_finish<SRC, P2, true>), dim3(6), dim3(CH), 0, L.s, L.m, L.a, b.tmax, b.pmin, b.dpart,
                       b.crec, b.fslot, b.shrec, L.row, L.g);
}

// a key-range shard's pass between its phases (pluss_dev_faithful_shards_*)
struct FaShards {
  FaLaunch L;
  int src = SRC_GEN;
  int phase = 0;  // last completed phase (SH_*)
  uint64_t tot[6] = {0, 0, 0, 0, 0, 0};  // SH_SELECTED, SH_UCOUNT: every reference's whole-list length
  int32_t shard = 0, nshards = 1;         // SH_UCOUNT: this shard's leaves
  bool has_slice = false;                 // the local phase ran: L.a holds this shard's slices
};
enum : int { SH_NONE = 0, SH_LOCAL = 1, SH_CARRY = 2, SH_CUT = 3, SH_SELECTED = 10, SH_UCOUNT = 11, SH_UWINDOW = 12 };

// the four sources (pluss_fa_w32.hip, pluss_fa_w64.hip, pluss_fa_smp.hip, pluss_fa_gen.hip)
void fa_launch_w32(const FaLaunch& L);
void fa_launch_w64(const FaLaunch& L);
void fa_launch_w32p(const FaLaunch& L);
void fa_launch_smp(const FaLaunch& L);
void fa_launch_gen(const FaLaunch& L);
void fa_launch_uni(const FaLaunch& L);

}  // namespace pluss
