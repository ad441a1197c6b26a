// pluss_faithful.hip — FAITHFUL mode: one r10 sampler_<REF> on the device.
//
// r10 pops samples in IterationComp order (pluss_utils.h:175-267) and replays
// all simulated threads in lockstep from each popped sample (r10:187-654).
// Because every simulated thread does the same number of accesses per chunk
// when N % (CS*T) == 0, the lockstep interleaving visits accesses in order of
// the 64-bit key  a*T + tid  (a = thread-local access position), which is also
// the IterationComp order of the samples.  A replay started at sample i stays
// open while an already-met sample's reuse has not been seen, i.e. while later
// sample keys are <= the running maximum of sink keys (a+RI)*T + tid.  So the
// whole sequential queue algorithm becomes:
//
//   sort samples by key; pmax = inclusive prefix-max of sink keys;
//   (start flags are recomputed wherever they are needed, never stored)
//   start_j  <=>  j == 0 || key_j > pmax_{j-1}               (new START_SAMPLE)
//   Q1 (r10:356): first start j > 0 with (j - starts_before_j) >= S - j  -> drop [j, S)
//   Q2 (r10:669-674): cold samples count only when tid == 0
//   Q3 (r10:345): if nothing was dropped and no sample is cold, the sample owning
//                 the largest sink is left in LAT: +1 cold if its tid == 0
//   traversed (r10:694) = sum over replays of (end key - start key), end key =
//                 the replay's last sink, or A*T for a replay that runs to the end.
//
// Packed keys (N % W == 0 shapes): a sample's sink is key + RI*T with RI one of
// its reference's three outcomes, so the sort carries only a packed word
// (rank << 2 | case), where rank = ((q*N + c1)*N + c2)*T + tid is the
// sample's position among its reference's N^3 possible keys in key order
// (q = thread-local row).  That is a keys-only radix sort over
// bitlen(N^3) + 2 bits -- 32-bit words up to N = 1024 -- instead of 64-bit
// (key, sink) pairs, and every later pass recomputes key and sink from the
// word (PkView).
//
// Validated against the reference's own dumps (tests/golden/r10_*, 42/42).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

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

// Packed word (rank << 2 | case) of sample x of reference `ref`; ~0 (and the
// bad-input flag) for a sample of another reference or out of range.
template <typename KT>
__device__ __forceinline__ KT pk_word_of(const Model& m, uint32_t ref, uint64_t x, GTable g) {
  const Sample s = unpack(x);
  if (s.ref != ref || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N) {
    atomicOr(&g.flags[1], 1u);
    return (KT) ~(KT)0;
  }
  const uint32_t c2 = (ref == C0 || ref == C1) ? 0u : s.c2;
  const uint32_t k = fdiv(s.c0, m.dCS), p = s.c0 - k * m.CS;
  const uint32_t kt = fdiv(k, m.dT), t = k - kt * m.T;
  const uint64_t q = (uint64_t)kt * m.CS + p;
  const uint64_t rank = ((q * m.N + s.c1) * m.N + c2) * m.T + t;
  return (KT)((rank << 2) | case_fast<false>(m, ref, s.c0, s.c1, c2));
}

// Key and sink of every sample.  cnt == nullptr: sample i -> slot i (one
// GPU).  Otherwise only samples with key in [lo, hi) are kept, compacted
// through a wave-aggregated counter (their order is irrelevant: they are
// sorted next).
template <bool FAST, int FM = FM_PAIRS>
__global__ __launch_bounds__(BLOCK) void k_faith_keys(Model m, uint32_t ref, const uint64_t* __restrict__ smp,
                                                      uint64_t n, uint64_t lo, uint64_t hi, void* __restrict__ keys_out,
                                                      unsigned long long* __restrict__ sinks, unsigned long long* cnt,
                                                      GTable g) {
  typedef fkey_t<FM> KT;
  KT* keys = static_cast<KT*>(keys_out);
  const uint64_t step = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t base = (uint64_t)blockIdx.x * BLOCK; base < n; base += step) {
    const uint64_t i = base + threadIdx.x;
    unsigned long long key = KEY_EMPTY, sink = KEY_EMPTY;
    KT word = (KT) ~(KT)0;
    bool keep = false;
    if (i < n) {
      const Sample s = unpack(smp[i]);
      if (s.ref != ref || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N) {
        atomicOr(&g.flags[1], 1u);
        keep = cnt == nullptr;  // one GPU: the slot still has to be filled
      } else {
        const uint32_t c2 = (ref == C0 || ref == C1) ? 0u : s.c2;
        uint64_t P;
        uint32_t t;
        position(m, ref, s.c0, s.c1, c2, &P, &t);
        key = P * m.T + t;
        keep = cnt == nullptr || (key >= lo && key < hi);
        if (FM != FM_PAIRS) {
          word = pk_word_of<KT>(m, ref, smp[i], g);
        } else {
          const int64_t ri = ri_of<FAST>(m, ref, s.c0, s.c1, c2);
          sink = ri < 0 ? KEY_EMPTY : (P + (uint64_t)ri) * m.T + t;
          word = (KT)key;
        }
      }
    }
    if (cnt == nullptr) {
      if (i < n) {
        keys[i] = word;
        if (FM == FM_PAIRS) sinks[i] = sink;
      }
      continue;
    }
    const unsigned long long mask = __ballot(keep);
    if (!mask) continue;
    unsigned long long at = 0;
    if (__lane_id() == (uint32_t)(__ffsll((long long)mask) - 1)) at = atomicAdd(cnt, (unsigned long long)__popcll(mask));
    at = __shfl(at, __ffsll((long long)mask) - 1, 64);
    if (keep) {
      const uint64_t o = at + __popcll(mask & ((1ull << __lane_id()) - 1));
      keys[o] = word;
      if (FM == FM_PAIRS) sinks[o] = sink;
    }
  }
}

// scal: [0] cut, [1] cold (tid 0), [2] traversed (mod 2^64), [3] shard size
__global__ void k_faith_init(unsigned long long* scal, uint64_t cut) {
  scal[0] = cut;
  scal[1] = 0;
  scal[2] = 0;
}

// Global prefix max at local i of a shard = max(pmax_in, local pmax_i);
// pmax_in = largest sink of every earlier shard (0 if none).
__device__ __forceinline__ unsigned long long gmax(const unsigned long long* pmax, uint64_t i,
                                                   unsigned long long pmax_in) {
  const unsigned long long v = pmax[i];
  return v > pmax_in ? v : pmax_in;
}

// What the start flag of sorted element i needs: START_i <=> it is the
// global first sample, or its key exceeds every earlier sink (the prefix max
// just before it).  Flags are never stored: the starts scan, the Q1 cut and
// the record pass each evaluate them where they need them.
struct FlagArgs {
  const void* keys;
  const unsigned long long* pmax;
  uint64_t j_off;
  unsigned long long pmax_in;
  PkView pv;
};
template <int FM>
__device__ __forceinline__ bool flag_at(const FlagArgs& a, uint64_t i) {
  const unsigned long long before = i == 0 ? a.pmax_in : gmax(a.pmax, i - 1, a.pmax_in);
  return a.j_off + i == 0 || key_at<FM>(a.keys, i, a.pv) > before;
}
template <int FM>
struct FlagOp {  // rocprim transform: element index -> start flag
  FlagArgs a;
  __device__ unsigned int operator()(uint64_t i) const { return flag_at<FM>(a, i) ? 1u : 0u; }
};

// Q1: the first START j > 0 (global index) whose met-sample count
// j - starts_before_j reaches the number of samples left, n_total - j.
template <int FM>
__global__ __launch_bounds__(BLOCK) void k_faith_cut(FlagArgs fa, const unsigned int* __restrict__ nstart, uint64_t n,
                                                     uint64_t s_off, uint64_t n_total, unsigned long long* scal) {
  const uint64_t j_off = fa.j_off;
  unsigned long long best = KEY_EMPTY;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    const uint64_t j = j_off + i;
    if (j > 0 && flag_at<FM>(fa, i)) {
      const uint64_t met = j - (s_off + (uint64_t)nstart[i] - 1);  // samples met before this START
      if (met >= n_total - j && j < best) best = j;
    }
  }
  // one atomic per wave instead of one per qualifying sample
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long x = __shfl_xor(best, o, 64);
    best = x < best ? x : best;
  }
  if (__lane_id() == 0 && best != KEY_EMPTY) atomicMin(&scal[0], best);
}

// ---- one-GPU scan: prefix max of sinks, start flags, start counts and the Q1
// cut in one pass over the sorted words (the shard path runs them as the
// separate rocPRIM scans and k_faith_cut above, because its start offset and
// cut need an exchange between the passes).  Tiles of SC_TILE elements take
// their index from a counter in arrival order and chain through decoupled
// look-back: each tile publishes its aggregate as soon as it has it and its
// inclusive prefix once the look-back resolves; a status word is
// flag (2 bits: 0 none, 1 aggregate, 2 inclusive) << 62 | value.
constexpr int SC_ITEMS = 8;
constexpr uint32_t SC_TILE = BLOCK * SC_ITEMS;
constexpr unsigned long long ST_AGG = 1ull << 62, ST_INC = 2ull << 62, ST_VAL = (1ull << 62) - 1;

__host__ __device__ inline uint64_t sc_tiles(uint64_t n) { return (n + SC_TILE - 1) / SC_TILE; }
// sinks < 2^62 (keys < A*T); KEY_EMPTY (no reuse) travels as ST_VAL
__device__ __forceinline__ unsigned long long st_cap(unsigned long long v) { return v > ST_VAL ? ST_VAL : v; }
__device__ __forceinline__ unsigned long long st_uncap(unsigned long long v) { return v == ST_VAL ? KEY_EMPTY : v; }
__device__ __forceinline__ unsigned long long st_ld(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_st(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
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
template <bool MAX>
__device__ __forceinline__ unsigned long long sc_wave_scan(unsigned long long v, uint32_t lane) {  // inclusive
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v = sc_op<MAX>(v, y);
  }
  return v;
}
// Exclusive prefix of tile t > 0 from the status words of tiles t-1, t-2, ...
// (one whole wave, 64 predecessors per round).  Every predecessor took its
// index earlier and publishes its aggregate without waiting on later tiles,
// so the spin ends.
template <bool MAX>
__device__ unsigned long long sc_lookback(const unsigned long long* st, uint32_t t, uint32_t lane) {
  unsigned long long acc = 0;
  int64_t hi = (int64_t)t - 1;
  while (true) {
    const int64_t j = hi - (int64_t)lane;
    unsigned long long w = j >= 0 ? st_ld(&st[j]) : ST_INC;  // before tile 0: the identity, inclusive
    while (__ballot((w >> 62) == 0) != 0) {
      __builtin_amdgcn_s_sleep(1);  // back off: the spinning waves share L2 with the publishers
      if ((w >> 62) == 0) w = st_ld(&st[j]);
    }
    const unsigned long long inc = __ballot((w >> 62) == 2);
    const uint32_t stop = inc ? (uint32_t)(__ffsll((long long)inc) - 1) : 64u;
    acc = sc_op<MAX>(acc, sc_wave_red<MAX>(lane <= stop ? (w & ST_VAL) : 0ull));
    if (inc) return acc;
    hi -= 64;
  }
}
// block-wide exclusive scan of one value per thread; returns (exclusive, aggregate)
template <bool MAX>
__device__ __forceinline__ void sc_block_scan(unsigned long long v, unsigned long long* sw, uint32_t lane, uint32_t wid,
                                              unsigned long long& excl, unsigned long long& agg) {
  const unsigned long long inc = sc_wave_scan<MAX>(v, lane);
  if (lane == 63) sw[wid] = inc;
  __syncthreads();
  unsigned long long pre = 0, all = 0;
#pragma unroll
  for (uint32_t w = 0; w < BLOCK / 64; ++w) {
    const unsigned long long x = sw[w];
    if (w < wid) pre = sc_op<MAX>(pre, x);
    all = sc_op<MAX>(all, x);
  }
  const unsigned long long up = __shfl_up(inc, 1, 64);
  excl = sc_op<MAX>(pre, lane ? up : 0ull);
  agg = all;
}
// publish the tile's aggregate, resolve its exclusive prefix, publish the inclusive one (wave 0)
template <bool MAX>
__device__ __forceinline__ unsigned long long sc_chain(unsigned long long* st, uint32_t t, unsigned long long agg,
                                                       uint32_t lane, unsigned long long* s_in) {
  if (threadIdx.x < 64) {
    unsigned long long in = 0;
    if (t == 0) {
      if (lane == 0) st_st(&st[0], ST_INC | st_cap(agg));
    } else {
      if (lane == 0) st_st(&st[t], ST_AGG | st_cap(agg));
      in = sc_lookback<MAX>(st, t, lane);
      if (lane == 0) st_st(&st[t], ST_INC | st_cap(sc_op<MAX>(in, agg)));
    }
    if (lane == 0) *s_in = in;
  }
  __syncthreads();
  return *s_in;
}

// scal: [0] cut (= n beforehand), [4] tile counter; st: 2 * sc_tiles(n) zeroed words.
// Wave w of a tile owns 64 * SC_ITEMS consecutive elements, visited as
// SC_ITEMS rounds of 64 (lane l: element l of the round), so every load and
// store is coalesced; the scans run across the lanes of each round with a
// carry between rounds.
template <int FM>
__global__ __launch_bounds__(BLOCK) void k_faith_scan(FlagArgs fa, const unsigned long long* __restrict__ sinks,
                                                      unsigned long long* __restrict__ pmax, uint64_t n,
                                                      unsigned long long* st, unsigned long long* scal) {
  __shared__ unsigned long long s_tile, s_w[BLOCK / 64], s_inm, s_inc;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_tile = atomicAdd(&scal[4], 1ull);
  __syncthreads();
  const uint32_t t = (uint32_t)s_tile;
  const uint64_t ntiles = sc_tiles(n);
  unsigned long long* stm = st;
  unsigned long long* stc = st + ntiles;
  const uint64_t wbase = (uint64_t)t * SC_TILE + (uint64_t)wid * (64 * SC_ITEMS);
  unsigned long long key[SC_ITEMS], snk[SC_ITEMS];
  unsigned long long tm = 0;
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    key[k] = KEY_EMPTY;
    snk[k] = 0;  // the identity of max
    if (i < n) {
      if (FM == FM_PAIRS) {
        key[k] = static_cast<const unsigned long long*>(fa.keys)[i];
        snk[k] = sinks[i];
      } else {
        const fkey_t<FM> w = static_cast<const fkey_t<FM>*>(fa.keys)[i];
        key[k] = pk_key(w, fa.pv);
        snk[k] = pk_sink(w, fa.pv);
      }
    }
    tm = snk[k] > tm ? snk[k] : tm;
  }
  // prefix max of sinks: wave aggregates -> tile aggregate -> look-back
  const unsigned long long wagg = sc_wave_red<true>(st_cap(tm));
  if (lane == 0) s_w[wid] = wagg;
  __syncthreads();
  unsigned long long pre = 0, agg = 0;
#pragma unroll
  for (uint32_t w = 0; w < BLOCK / 64; ++w) {
    const unsigned long long x = s_w[w];
    if (w < wid) pre = x > pre ? x : pre;
    agg = x > agg ? x : agg;
  }
  const unsigned long long m_in = sc_chain<true>(stm, t, agg, lane, &s_inm);
  unsigned long long carry = st_uncap(m_in > pre ? m_in : pre);  // prefix max before the wave's first element
  // per round: the prefix max (stored), the start flags (ballots), their count
  unsigned long long fmask[SC_ITEMS];
  uint32_t wcnt = 0;
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    const bool valid = i < n;
    unsigned long long inc = sc_wave_scan<true>(valid ? snk[k] : 0ull, lane);
    inc = inc > carry ? inc : carry;
    const unsigned long long up = __shfl_up(inc, 1, 64);
    const unsigned long long before = lane ? up : carry;
    fmask[k] = __ballot(valid && (i == 0 || key[k] > before));
    wcnt += (uint32_t)__popcll(fmask[k]);
    if (valid) pmax[i] = inc;
    carry = __shfl(inc, 63, 64);
  }
  // start counts: wave totals -> tile total -> look-back
  __syncthreads();  // s_w is reused
  if (lane == 0) s_w[wid] = wcnt;
  __syncthreads();
  unsigned long long cpre = 0, cagg = 0;
#pragma unroll
  for (uint32_t w = 0; w < BLOCK / 64; ++w) {
    const unsigned long long x = s_w[w];
    if (w < wid) cpre += x;
    cagg += x;
  }
  const unsigned long long c_in = sc_chain<false>(stc, t, cagg, lane, &s_inc);
  // Q1: the first start j > 0 whose met-sample count j - starts_before_j reaches n - j
  uint64_t cb = c_in + cpre;  // starts before the round's first element
  unsigned long long best = KEY_EMPTY;
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {
    const unsigned long long F = fmask[k];
    if (best == KEY_EMPTY && F) {
      const uint64_t j = wbase + (uint64_t)k * 64 + lane;
      const uint64_t before_j = cb + (uint64_t)__popcll(F & below);
      const unsigned long long q = __ballot(((F >> lane) & 1ull) && j > 0 && j - before_j >= n - j);
      if (q) best = wbase + (uint64_t)k * 64 + (uint64_t)(__ffsll((long long)q) - 1);
    }
    cb += (uint64_t)__popcll(F);
  }
  if (lane == 0 && best != KEY_EMPTY) atomicMin(&scal[0], best);
}

// scal [0] = cut default, [1] cold, [2] traversed, [4] tile counter; st zeroed
__global__ void k_faith_scan_init(unsigned long long* scal, uint64_t cut, unsigned long long* st, uint64_t nw) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    scal[0] = cut;
    scal[1] = 0;
    scal[2] = 0;
    scal[4] = 0;
  }
  for (uint64_t j = i; j < nw; j += (uint64_t)gridDim.x * blockDim.x) st[j] = 0;
}

// ---- one-GPU packed-word pass: scan, Q1 cut and record fused.  Chunks of
// FCHUNK elements (1024 threads x FI) chain their prefix max and start count
// through decoupled look-back (256 predecessors per round, so the chain
// over a 2^22-element reference resolves in a couple of rounds), find their
// own first qualifying start (the chunk's Q1 candidate) and record their
// elements below it into per-chunk partial sums.  The condition of Q1,
// j - starts_before_j >= n - j, is monotone in j, so the global cut is the
// smallest candidate; k_faith_fused_finish adds the partials of the chunks
// that start below it (the cut's own chunk recorded exactly the elements
// before it; chunks before it have no candidate and recorded everything).
// The prefix max is never stored.
constexpr int FB = 1024, FI = 8;
constexpr uint32_t FCHUNK = FB * FI;
constexpr int FPART = 5;  // per chunk: cold (tid 0), traversed, case 0/1/2 counts
__host__ __device__ inline uint64_t fu_tiles(uint64_t n) { return (n + FCHUNK - 1) / FCHUNK; }

// exclusive prefix of tile t > 0, 4 predecessors per lane (256 per round)
template <bool MAX>
__device__ unsigned long long sc_lookback4(const unsigned long long* st, uint32_t t, uint32_t lane) {
  unsigned long long acc = 0;
  int64_t hi = (int64_t)t - 1;
  while (true) {
    unsigned long long w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t j = hi - (int64_t)(q * 64 + lane);
      w[q] = j >= 0 ? st_ld(&st[j]) : ST_INC;
    }
    while (__ballot((w[0] >> 62) == 0 || (w[1] >> 62) == 0 || (w[2] >> 62) == 0 || (w[3] >> 62) == 0) != 0) {
      __builtin_amdgcn_s_sleep(1);  // back off: the spinning waves share L2 with the publishers
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t j = hi - (int64_t)(q * 64 + lane);
        if ((w[q] >> 62) == 0) w[q] = st_ld(&st[j]);
      }
    }
    bool done = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (done) break;
      const unsigned long long inc = __ballot((w[q] >> 62) == 2);
      const uint32_t stop = inc ? (uint32_t)(__ffsll((long long)inc) - 1) : 64u;
      acc = sc_op<MAX>(acc, sc_wave_red<MAX>(lane <= stop ? (w[q] & ST_VAL) : 0ull));
      done = inc != 0;
    }
    if (done) return acc;
    hi -= 256;
  }
}
template <bool MAX>
__device__ __forceinline__ unsigned long long fu_chain(unsigned long long* st, uint32_t t, unsigned long long agg,
                                                       uint32_t lane, unsigned long long* s_in) {
  if (threadIdx.x < 64) {
    unsigned long long in = 0;
    if (t == 0) {
      if (lane == 0) st_st(&st[0], ST_INC | st_cap(agg));
    } else {
      if (lane == 0) st_st(&st[t], ST_AGG | st_cap(agg));
      in = sc_lookback4<MAX>(st, t, lane);
      if (lane == 0) st_st(&st[t], ST_INC | st_cap(sc_op<MAX>(in, agg)));
    }
    if (lane == 0) *s_in = in;
  }
  __syncthreads();
  return *s_in;
}

// One tile of the fused pass.  The tile's elements have global indices
// gbase + li, li in [0, mt); src.word(li) is element li's packed word and
// src.key_after(li) the key of the global element after it (KEY_EMPTY past
// the end).  t is the tile's look-back index (tiles in global order).
// Src::kCheck: the source is a caller's list that must be in key order;
// an element whose successor's key is not larger is reported through
// src.unordered() (the bad-input flag).
// scal: [0] cut (= n beforehand); st: 2 * ntiles zeroed words; part: FPART
// words per tile (written, not accumulated).
template <int FM, class Src>
__device__ __forceinline__ void fused_tile(const Src& src, uint32_t t, uint64_t gbase, uint32_t mt, const PkView& pv,
                                           uint64_t n, unsigned long long endkey, unsigned long long* st,
                                           uint64_t ntiles, unsigned long long* __restrict__ part,
                                           unsigned long long* scal) {
  typedef fkey_t<FM> KT;
  constexpr int NW = FB / 64;
  __shared__ unsigned long long s_w[NW], s_inm, s_inc, s_red[NW][FPART];
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t lbase = wid * (64 * FI);
  KT w[FI];
  unsigned long long tm = 0;
#pragma unroll
  for (int k = 0; k < FI; ++k) {
    const uint32_t li = lbase + (uint32_t)k * 64 + lane;
    w[k] = li < mt ? src.word(li) : (KT)0;
    const unsigned long long sk = li < mt ? pk_sink(w[k], pv) : 0ull;
    tm = sk > tm ? sk : tm;
  }
  // prefix max of sinks
  {
    const unsigned long long wagg = sc_wave_red<true>(st_cap(tm));
    if (lane == 0) s_w[wid] = wagg;
  }
  __syncthreads();
  unsigned long long pre = 0, agg = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    const unsigned long long v = s_w[x];
    if (x < (int)wid) pre = v > pre ? v : pre;
    agg = v > agg ? v : agg;
  }
  const unsigned long long m_in = fu_chain<true>(st, t, agg, lane, &s_inm);
  unsigned long long carry = st_uncap(m_in > pre ? m_in : pre);  // prefix max before the wave's first element
  unsigned long long pm[FI], fmask[FI], key[FI];
  uint32_t wcnt = 0;
#pragma unroll
  for (int k = 0; k < FI; ++k) {
    const uint32_t li = lbase + (uint32_t)k * 64 + lane;
    const uint64_t i = gbase + li;
    const bool valid = li < mt;
    const KT wk = w[k];
    unsigned long long inc = sc_wave_scan<true>(valid ? pk_sink(wk, pv) : 0ull, lane);
    inc = inc > carry ? inc : carry;
    const unsigned long long up = __shfl_up(inc, 1, 64);
    const unsigned long long before = lane ? up : carry;
    const unsigned long long kk = valid ? pk_key(wk, pv) : KEY_EMPTY;
    key[k] = kk;
    fmask[k] = __ballot(valid && (i == 0 || kk > before));
    wcnt += (uint32_t)__popcll(fmask[k]);
    pm[k] = inc;
    carry = __shfl(inc, 63, 64);
  }
  // start counts
  __syncthreads();  // s_w is reused
  if (lane == 0) s_w[wid] = wcnt;
  __syncthreads();
  unsigned long long cpre = 0, cagg = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) {
    const unsigned long long v = s_w[x];
    if (x < (int)wid) cpre += v;
    cagg += v;
  }
  const unsigned long long c_in = fu_chain<false>(st + ntiles, t, cagg, lane, &s_inc);
  // the tile's Q1 candidate: its first start j > 0 with j - starts_before_j >= n - j
  unsigned long long best = KEY_EMPTY;
  {
    uint64_t cb = c_in + cpre;
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < FI; ++k) {
      const unsigned long long F = fmask[k];
      if (best == KEY_EMPTY && F) {
        const uint64_t j = gbase + lbase + (uint64_t)k * 64 + lane;
        const uint64_t before_j = cb + (uint64_t)__popcll(F & below);
        const unsigned long long q = __ballot(((F >> lane) & 1ull) && j > 0 && j - before_j >= n - j);
        if (q) best = gbase + lbase + (uint64_t)k * 64 + (uint64_t)(__ffsll((long long)q) - 1);
      }
      cb += (uint64_t)__popcll(F);
    }
  }
  __syncthreads();  // s_w is reused
  if (lane == 0) s_w[wid] = best;
  __syncthreads();
  unsigned long long cut = n;
#pragma unroll
  for (int x = 0; x < NW; ++x) cut = s_w[x] < cut ? s_w[x] : cut;
  if (threadIdx.x == 0 && cut < n) atomicMin(&scal[0], cut);
  // record the tile's elements below its own cut
  unsigned long long cold = 0, trav = 0;
  uint32_t nc0 = 0, nc1 = 0, nc2 = 0;
  bool unordered = false;
#pragma unroll
  for (int k = 0; k < FI; ++k) {
    const uint32_t li = lbase + (uint32_t)k * 64 + lane;
    const uint64_t i = gbase + li;
    const KT wk = w[k];
    const unsigned long long kk = key[k];
    // the next element's key: the next lane, the next round's lane 0, or (the wave's last element) the source
    unsigned long long kn = __shfl_down(kk, 1, 64);
    if (k + 1 < FI) {
      const unsigned long long k0 = __shfl(key[k + 1], 0, 64);
      if (lane == 63) kn = k0;
    } else if (lane == 63) {
      kn = li < mt ? src.key_after(li) : KEY_EMPTY;
    }
    if (Src::kCheck && li < mt && i + 1 < n && !(kn > kk)) unordered = true;
    uint32_t c = 3;
    bool rec = false;
    if (li < mt && i < cut) {
      c = (uint32_t)(wk & 3u);
      if (pk_sink(wk, pv) == KEY_EMPTY) cold += ((pv.p2 ? (kk & (pv.T - 1)) : kk % pv.T) == 0) ? 1u : 0u;
      else rec = true;
      if ((fmask[k] >> lane) & 1ull) trav -= kk;  // this element starts a replay
      const unsigned long long gm = pm[k];
      if (i + 1 == cut || (i + 1 < n ? kn > gm : true)) trav += (gm == KEY_EMPTY) ? endkey : gm;  // ends one
    }
    nc0 += (uint32_t)__popcll(__ballot(rec && c == 0));
    nc1 += (uint32_t)__popcll(__ballot(rec && c == 1));
    nc2 += (uint32_t)__popcll(__ballot(rec && c == 2));
  }
  if (Src::kCheck && __ballot(unordered) && lane == 0) src.unordered();
  cold = sc_wave_red<false>(cold);
  trav = sc_wave_red<false>(trav);
  if (lane == 0) {
    s_red[wid][0] = cold;
    s_red[wid][1] = trav;
    s_red[wid][2] = nc0;
    s_red[wid][3] = nc1;
    s_red[wid][4] = nc2;
  }
  __syncthreads();
  if (threadIdx.x < FPART) {
    unsigned long long v = 0;
#pragma unroll
    for (int x = 0; x < NW; ++x) v += s_red[x][threadIdx.x];
    part[(uint64_t)t * FPART + threadIdx.x] = v;
  }
}

// Tiles of FCHUNK consecutive sorted words (the rocPRIM-sorted array).
template <int FM>
struct GlobalTile {
  static constexpr bool kCheck = false;
  const fkey_t<FM>* wd;
  uint64_t gbase, n;
  PkView pv;
  __device__ fkey_t<FM> word(uint32_t li) const { return wd[gbase + li]; }
  __device__ unsigned long long key_after(uint32_t li) const {
    const uint64_t i = gbase + li + 1;
    return i < n ? pk_key(wd[i], pv) : KEY_EMPTY;
  }
  __device__ void unordered() const {}
};

// Tiles of FCHUNK consecutive samples of a caller's list that is already in
// key order (pluss_dev_faithful_hist_sorted): each sample's packed word is
// made where it is read -- no keys pass, no sort -- and the order is checked.
template <int FM>
struct SampleTile {
  static constexpr bool kCheck = true;
  const uint64_t* smp;
  uint64_t gbase, n;
  const Model* m;
  uint32_t ref;
  PkView pv;
  GTable g;
  __device__ fkey_t<FM> word(uint32_t li) const { return pk_word_of<fkey_t<FM>>(*m, ref, smp[gbase + li], g); }
  __device__ unsigned long long key_after(uint32_t li) const {
    const uint64_t i = gbase + li + 1;
    return i < n ? pk_key(pk_word_of<fkey_t<FM>>(*m, ref, smp[i], g), pv) : KEY_EMPTY;
  }
  __device__ void unordered() const { atomicOr(&g.flags[1], 1u); }
};

// Tiles of a generated key-order list (pluss_dev_gen_faithful_refs): the
// samples never exist in memory.
template <int FM>
struct GenTile {
  static constexpr bool kCheck = false;
  const KeyGen* k;
  uint64_t gbase, n;
  const Model* m;
  PkView pv;
  GTable g;
  __device__ fkey_t<FM> word(uint32_t li) const {
    return pk_word_of<fkey_t<FM>>(*m, k->ref, keygen_sample(*k, gbase + li), g);
  }
  __device__ unsigned long long key_after(uint32_t li) const {
    const uint64_t i = gbase + li + 1;
    return i < n ? pk_key(pk_word_of<fkey_t<FM>>(*m, k->ref, keygen_sample(*k, i), g), pv) : KEY_EMPTY;
  }
  __device__ void unordered() const {}
};

// scal: [0] cut (= n beforehand), [4] tile counter; st: 2 * fu_tiles(n) zeroed words;
// part: FPART words per chunk (written, not accumulated)
template <int FM>
__global__ __launch_bounds__(FB) void k_faith_fused(const void* __restrict__ words, PkView pv, uint64_t n,
                                                    unsigned long long endkey, unsigned long long* st,
                                                    unsigned long long* __restrict__ part,
                                                    unsigned long long* scal) {
  __shared__ unsigned long long s_tile;
  if (threadIdx.x == 0) s_tile = atomicAdd(&scal[4], 1ull);
  __syncthreads();
  const uint32_t t = (uint32_t)s_tile;
  const uint64_t gbase = (uint64_t)t * FCHUNK;
  const uint32_t mt = (uint32_t)(n - gbase < FCHUNK ? n - gbase : FCHUNK);
  const GlobalTile<FM> src{static_cast<const fkey_t<FM>*>(words), gbase, n, pv};
  fused_tile<FM>(src, t, gbase, mt, pv, n, endkey, st, fu_tiles(n), part, scal);
}

// The same pass straight over a key-ordered sample list (GEN = false) or a
// generated key-order list (GEN = true, `smp` unused).
template <int FM, bool GEN>
__global__ __launch_bounds__(FB) void k_faith_fused_direct(Model m, uint32_t ref, const uint64_t* __restrict__ smp,
                                                           KeyGen kg, PkView pv, uint64_t n, unsigned long long endkey,
                                                           unsigned long long* st,
                                                           unsigned long long* __restrict__ part,
                                                           unsigned long long* scal, GTable g) {
  __shared__ unsigned long long s_tile;
  if (threadIdx.x == 0) s_tile = atomicAdd(&scal[4], 1ull);
  __syncthreads();
  const uint32_t t = (uint32_t)s_tile;
  const uint64_t gbase = (uint64_t)t * FCHUNK;
  const uint32_t mt = (uint32_t)(n - gbase < FCHUNK ? n - gbase : FCHUNK);
  if (GEN) {
    const GenTile<FM> src{&kg, gbase, n, &m, pv, g};
    fused_tile<FM>(src, t, gbase, mt, pv, n, endkey, st, fu_tiles(n), part, scal);
  } else {
    const SampleTile<FM> src{smp, gbase, n, &m, ref, pv, g};
    fused_tile<FM>(src, t, gbase, mt, pv, n, endkey, st, fu_tiles(n), part, scal);
  }
}

// Sum the partials of the tiles that start below the cut, then what
// k_faith_finish does (Q3, the -1 key, traversed) and the case counts.
__global__ __launch_bounds__(BLOCK) void k_faith_fused_finish(uint32_t ref, uint64_t n, PkView pv,
                                                             const unsigned long long* st, uint64_t ntiles,
                                                             const unsigned long long* part,
                                                             const unsigned long long* scal, GTable g) {
  __shared__ unsigned long long red[BLOCK / 64][FPART];
  const uint64_t cut = scal[0];
  unsigned long long v[FPART] = {0, 0, 0, 0, 0};
  for (uint64_t t = threadIdx.x; t < ntiles && t * FCHUNK < cut; t += BLOCK)
#pragma unroll
    for (int f = 0; f < FPART; ++f) v[f] += part[t * FPART + f];
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
#pragma unroll
  for (int f = 0; f < FPART; ++f) {
    v[f] = sc_wave_red<false>(v[f]);
    if (lane == 0) red[wid][f] = v[f];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot[FPART] = {0, 0, 0, 0, 0};
    for (int x = 0; x < BLOCK / 64; ++x)
      for (int f = 0; f < FPART; ++f) tot[f] += red[x][f];
    unsigned long long cold = tot[0];
    if (n > 0 && cut == n) {  // Q3: nothing dropped; the owner of the largest sink stays in LAT
      const unsigned long long gm = st_uncap(st[ntiles - 1] & ST_VAL);
      if (gm != KEY_EMPTY && (pv.p2 ? (gm & (pv.T - 1)) : gm % pv.T) == 0) cold += 1;
    }
    g_add(g, make_key(ref, 0, -1), cold);
    g.trav[ref] += tot[1];
    for (int c = 0; c < 3; ++c)
      if (tot[2 + c]) atomicAdd(&g.bins[ref * 3 + c], tot[2 + c]);
  }
}


// Record the shard's samples with global index < cut: RI bins, tid-0 cold
// samples, and the traversed contributions of the replays that start or end
// here (a replay ends at j when j + 1 == cut or j + 1 starts one; for the
// shard's last sample that is `next_start`, decided by the caller).
//
// Packed words (FM_PK*): a recorded sample's key is its reference's
// (ref, case) key, so the cases are counted by ballots and added to the
// direct bin row blockIdx % 64 (folded by k_export like clean-mode counts);
// (key, sink) pairs take the exact-key path.
template <bool FAST, int FM = FM_PAIRS>
__global__ __launch_bounds__(BLOCK) void k_faith_hist(Model m, uint32_t ref, FlagArgs fa,
                                                      const unsigned long long* __restrict__ sinks, uint64_t n,
                                                      int next_start, unsigned long long* scal, GTable g) {
  constexpr bool PKD = FM != FM_PAIRS;
  __shared__ unsigned long long tk[PKD ? 1 : TCAP];
  __shared__ unsigned int tc[PKD ? 1 : TCAP];
  __shared__ unsigned long long red[5];  // cold, traversed, case 0/1/2 counts
  const BlockTable bt{tk, tc};
  if (!PKD) bt_init(bt);
  WaveCache wc;
  wc_init(wc);
  if (threadIdx.x < 5) red[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t j_off = fa.j_off;
  const uint64_t cut = scal[0];
  const uint64_t lim = cut > j_off ? (cut - j_off < n ? cut - j_off : n) : 0;  // local samples recorded
  const uint64_t endkey = m.A * m.T;
  unsigned long long cold = 0, trav = 0;
  uint32_t nc0 = 0, nc1 = 0, nc2 = 0;  // wave totals of recorded samples per case (packed words)
  const uint64_t step = (uint64_t)gridDim.x * BLOCK;
  const uint32_t lane = __lane_id();
  for (uint64_t base = (uint64_t)blockIdx.x * BLOCK; base < lim; base += step) {
    const uint64_t i = base + threadIdx.x;
    const bool v = i < lim;
    uint64_t key = KEY_NONE;
    bool rec = false;
    uint32_t c = 3;
    // each lane decodes its own key once; the next element's key (for "does
    // a replay end here?") comes from the neighbouring lane
    const unsigned long long k = i < n ? key_at<FM>(fa.keys, i, fa.pv) : KEY_EMPTY;
    unsigned long long k_next = __shfl_down(k, 1, 64);
    if (lane == 63 && i + 1 < n) k_next = key_at<FM>(fa.keys, i + 1, fa.pv);
    if (v) {
      unsigned long long s;
      if (PKD) {
        const fkey_t<FM> word = static_cast<const fkey_t<FM>*>(fa.keys)[i];
        c = (uint32_t)(word & 3u);
        const int64_t ri = c == 0 ? fa.pv.ri[0] : (c == 1 ? fa.pv.ri[1] : fa.pv.ri[2]);
        s = (c == 3 || ri < 0 || k == KEY_EMPTY) ? KEY_EMPTY : k + (unsigned long long)ri * m.T;
      } else {
        s = sinks[i];
      }
      if (s == KEY_EMPTY) {
        cold += ((fa.pv.p2 ? (k & (fa.pv.T - 1)) : k % fa.pv.T) == 0) ? 1u : 0u;  // tid 0
      } else if (PKD) {
        rec = true;
      } else {
        const int64_t ri = (int64_t)((s - k) / m.T);
        key = make_key(ref, share_kind(m, ref, ri), ri);
        rec = true;
      }
      const unsigned long long before = i == 0 ? fa.pmax_in : gmax(fa.pmax, i - 1, fa.pmax_in);
      if (j_off + i == 0 || k > before) trav -= k;  // this element starts a replay
      const unsigned long long gm = gmax(fa.pmax, i, fa.pmax_in);
      const bool ends = j_off + i + 1 == cut || (i + 1 < n ? k_next > gm : next_start != 0);
      if (ends) trav += (gm == KEY_EMPTY) ? endkey : gm;
    }
    if (PKD) {
      nc0 += (uint32_t)__popcll(__ballot(rec && c == 0));
      nc1 += (uint32_t)__popcll(__ballot(rec && c == 1));
      nc2 += (uint32_t)__popcll(__ballot(rec && c == 2));
    } else {
      wave_count(wc, bt, g, key, rec);
    }
  }
  cold = sc_wave_red<false>(cold);
  trav = sc_wave_red<false>(trav);
  if (lane == 0) {
    atomicAdd(&red[0], cold);
    atomicAdd(&red[1], trav);
  }
  if (PKD && __lane_id() == 0) {
    if (nc0) atomicAdd(&red[2], (unsigned long long)nc0);
    if (nc1) atomicAdd(&red[3], (unsigned long long)nc1);
    if (nc2) atomicAdd(&red[4], (unsigned long long)nc2);
  }
  if (!PKD) bt_finish(wc, bt, g);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&scal[1], red[0]);
    atomicAdd(&scal[2], red[1]);
  }
  if (PKD && threadIdx.x < 3 && red[2 + threadIdx.x])
    atomicAdd(&g.bins[(blockIdx.x & (NBROW - 1)) * BSTRIDE + ref * 3 + threadIdx.x], red[2 + threadIdx.x]);
}

// Q3 (only on the shard holding the global last sample, with nothing
// dropped): the owner of the final largest sink stays in LAT; +1 cold if it
// is tid 0.  Every shard materialises key -1 (r10:671), possibly with 0.
__global__ void k_faith_finish(Model m, uint32_t ref, uint64_t n, uint64_t n_total, int is_last,
                               unsigned long long pmax_in, const unsigned long long* pmax,
                               const unsigned long long* scal, GTable g) {
  unsigned long long cold = scal[1];
  if (is_last && n > 0 && scal[0] == n_total) {
    const unsigned long long gm = gmax(pmax, n - 1, pmax_in);
    if (gm != KEY_EMPTY && gm % m.T == 0) cold += 1;
  }
  g_add(g, make_key(ref, 0, -1), cold);
  g.trav[ref] += scal[2];
}

template <typename T>
static int grow(T** p, uint64_t n) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess) {
    set_error("hipMalloc failed for faithful-mode buffers");
    return PLUSS_ERR_ALLOC;
  }
  return PLUSS_OK;
}

static int faith_check_shape(const pluss_ctx* ctx) {
  if ((uint64_t)ctx->cfg.n % ((uint64_t)ctx->cfg.chunk * (uint64_t)ctx->cfg.threads) != 0) {
    set_error("faithful mode needs N % (chunk*threads) == 0 (lockstep interleaving order)");
    return PLUSS_ERR_CONFIG;
  }
  return PLUSS_OK;
}

static unsigned key_bits(const Model& m) {  // keys < A*T: sort only the significant bits
  unsigned end_bit = 1;
  while (end_bit < 64 && (m.A * m.T) >> end_bit) ++end_bit;
  return end_bit;
}

static unsigned pk_bits(const Model& m) {  // packed words < N^3 << 2
  const uint64_t top = (uint64_t)m.N * m.N * m.N - 1;
  unsigned b = 1;
  while (b < 62 && (top >> b)) ++b;
  return b + 2;
}

static int faith_fm(const Model& m) {
  if (!m.fast) return FM_PAIRS;
  return pk_bits(m) <= 32 ? FM_PK32 : FM_PK64;
}

static int grid_of(uint64_t n) {
  const uint64_t b = (n + BLOCK * 4 - 1) / (BLOCK * 4);
  return b < 1 ? 1 : (b > (uint64_t)MAX_BLOCKS ? MAX_BLOCKS : (int)b);
}

// buffers for n samples (sort words or keys + sinks, sorted copies, prefix max, scan of the start flags)
static int faith_reserve(pluss_ctx* ctx, FaithfulBufs& b, uint64_t n, hipStream_t s) {
  if (!b.scal) {
    if (int rc = grow(&b.scal, 8)) return rc;
  }
  if (n > 0xFFFFFFFFull) {
    set_error("faithful mode: at most 2^32-1 samples per reference");
    return PLUSS_ERR_CONFIG;
  }
  if (n > b.cap) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    int rc = 0;
    if ((rc = grow(&b.keys, n)) || (rc = grow(&b.sinks, n)) || (rc = grow(&b.keys_s, n)) ||
        (rc = grow(&b.sinks_s, n)) || (rc = grow(&b.pmax, n + FPART)) || (rc = grow(&b.nstart, n)) ||
        (rc = grow(&b.st, 2 * sc_tiles(n))))
      return rc;
    b.cap = n;
  }
  return PLUSS_OK;
}

static int faith_tmp(pluss_ctx* ctx, FaithfulBufs& b, uint64_t n, hipStream_t s) {
  size_t t1 = 0, t2 = 0, t3 = 0;
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PK32) {  // packed words: keys-only sort, pmax over the recomputed sinks
    uint32_t *k = (uint32_t*)b.keys, *ks = (uint32_t*)b.keys_s;
    PLUSS_HIP_CHECK(rocprim::radix_sort_keys(nullptr, t1, k, ks, n, 0, pk_bits(ctx->m), s));
    auto it = rocprim::make_transform_iterator(ks, PkSinkOp<uint32_t>{make_pkview(ctx->m, 0)});
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(nullptr, t2, it, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
  } else if (fm == FM_PK64) {
    PLUSS_HIP_CHECK(rocprim::radix_sort_keys(nullptr, t1, b.keys, b.keys_s, n, 0, pk_bits(ctx->m), s));
    auto it = rocprim::make_transform_iterator(b.keys_s, PkSinkOp<unsigned long long>{make_pkview(ctx->m, 0)});
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(nullptr, t2, it, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
  } else {
    PLUSS_HIP_CHECK(
        rocprim::radix_sort_pairs(nullptr, t1, b.keys, b.keys_s, b.sinks, b.sinks_s, n, 0, key_bits(ctx->m), s));
    PLUSS_HIP_CHECK(
        rocprim::inclusive_scan(nullptr, t2, b.sinks_s, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
  }
  {
    const FlagArgs fa{b.keys_s, b.pmax, 0, 0, make_pkview(ctx->m, 0)};
    auto it = rocprim::make_transform_iterator(rocprim::counting_iterator<uint64_t>(0), FlagOp<FM_PAIRS>{fa});
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(nullptr, t3, it, b.nstart, n, rocprim::plus<unsigned int>(), s));
  }
  size_t need = t1 > t2 ? t1 : t2;
  need = need > t3 ? need : t3;
  if (need > b.tmp_bytes) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    if (b.tmp) (void)hipFree(b.tmp);
    b.tmp = nullptr;
    if (hipMalloc(&b.tmp, need) != hipSuccess) {
      set_error("hipMalloc failed for rocprim temporary storage");
      return PLUSS_ERR_ALLOC;
    }
    b.tmp_bytes = need;
  }
  return PLUSS_OK;
}

static int faith_keys(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, const uint64_t* d_samples, uint64_t n, uint64_t lo, uint64_t hi,
                      unsigned long long* cnt, hipStream_t s) {
  const Model& m = ctx->m;
  const int fm = faith_fm(m);
  if (fm == FM_PK32)
    hipLaunchKernelGGL((k_faith_keys<true, FM_PK32>), dim3(grid_of(n)), dim3(BLOCK), 0, s, m, (uint32_t)ref, d_samples,
                       n, lo, hi, (void*)b.keys, b.sinks, cnt, ctx->g);
  else if (fm == FM_PK64)
    hipLaunchKernelGGL((k_faith_keys<true, FM_PK64>), dim3(grid_of(n)), dim3(BLOCK), 0, s, m, (uint32_t)ref, d_samples,
                       n, lo, hi, (void*)b.keys, b.sinks, cnt, ctx->g);
  else
    hipLaunchKernelGGL(k_faith_keys<false>, dim3(grid_of(n)), dim3(BLOCK), 0, s, m, (uint32_t)ref, d_samples, n, lo,
                       hi, (void*)b.keys, b.sinks, cnt, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

// sort the shard's n (key, sink) pairs by key and take the prefix max of sinks
static int faith_sort(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, uint64_t n, hipStream_t s, bool with_pmax = true) {
  if (int rc = faith_tmp(ctx, b, n, s)) return rc;
  size_t sz = b.tmp_bytes;
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PK32) {
    uint32_t *k = (uint32_t*)b.keys, *ks = (uint32_t*)b.keys_s;
    PLUSS_HIP_CHECK(rocprim::radix_sort_keys(b.tmp, sz, k, ks, n, 0, pk_bits(ctx->m), s));
    if (!with_pmax) return PLUSS_OK;
    sz = b.tmp_bytes;
    auto it = rocprim::make_transform_iterator(ks, PkSinkOp<uint32_t>{make_pkview(ctx->m, (uint32_t)ref)});
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, it, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
    return PLUSS_OK;
  }
  if (fm == FM_PK64) {
    PLUSS_HIP_CHECK(rocprim::radix_sort_keys(b.tmp, sz, b.keys, b.keys_s, n, 0, pk_bits(ctx->m), s));
    if (!with_pmax) return PLUSS_OK;
    sz = b.tmp_bytes;
    auto it = rocprim::make_transform_iterator(b.keys_s,
                                               PkSinkOp<unsigned long long>{make_pkview(ctx->m, (uint32_t)ref)});
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, it, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
    return PLUSS_OK;
  }
  PLUSS_HIP_CHECK(
      rocprim::radix_sort_pairs(b.tmp, sz, b.keys, b.keys_s, b.sinks, b.sinks_s, n, 0, key_bits(ctx->m), s));
  if (!with_pmax) return PLUSS_OK;
  sz = b.tmp_bytes;
  PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, b.sinks_s, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
  return PLUSS_OK;
}

static int faith_starts(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, uint64_t n, uint64_t j_off, unsigned long long pmax_in,
                        hipStream_t s) {
  const FlagArgs fa{b.keys_s, b.pmax, j_off, pmax_in, make_pkview(ctx->m, (uint32_t)ref)};
  size_t sz = b.tmp_bytes;
  rocprim::counting_iterator<uint64_t> idx(0);
  const int fm = faith_fm(ctx->m);
  // nstart = inclusive scan of the start flags, evaluated inside the scan
  if (fm == FM_PK32)
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, rocprim::make_transform_iterator(idx, FlagOp<FM_PK32>{fa}),
                                            b.nstart, n, rocprim::plus<unsigned int>(), s));
  else if (fm == FM_PK64)
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, rocprim::make_transform_iterator(idx, FlagOp<FM_PK64>{fa}),
                                            b.nstart, n, rocprim::plus<unsigned int>(), s));
  else
    PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, rocprim::make_transform_iterator(idx, FlagOp<FM_PAIRS>{fa}),
                                            b.nstart, n, rocprim::plus<unsigned int>(), s));
  return PLUSS_OK;
}

// Q1 cut of this shard's elements into scal[0] (already holding the default)
static int faith_cut(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, uint64_t n, uint64_t j_off, unsigned long long pmax_in,
                     uint64_t s_off, uint64_t n_total, hipStream_t s) {
  const FlagArgs fa{b.keys_s, b.pmax, j_off, pmax_in, make_pkview(ctx->m, (uint32_t)ref)};
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PK32)
    hipLaunchKernelGGL(k_faith_cut<FM_PK32>, dim3(grid_of(n)), dim3(BLOCK), 0, s, fa, b.nstart, n, s_off, n_total,
                       b.scal);
  else if (fm == FM_PK64)
    hipLaunchKernelGGL(k_faith_cut<FM_PK64>, dim3(grid_of(n)), dim3(BLOCK), 0, s, fa, b.nstart, n, s_off, n_total,
                       b.scal);
  else
    hipLaunchKernelGGL(k_faith_cut<FM_PAIRS>, dim3(grid_of(n)), dim3(BLOCK), 0, s, fa, b.nstart, n, s_off, n_total,
                       b.scal);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

static int faith_record(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, uint64_t n, uint64_t j_off, unsigned long long pmax_in,
                        int next_start, uint64_t n_total, int is_last, hipStream_t s) {
  const Model& m = ctx->m;
  if (n) {
    const FlagArgs fa{b.keys_s, b.pmax, j_off, pmax_in, make_pkview(m, (uint32_t)ref)};
    const int fm = faith_fm(m);
    if (fm == FM_PK32)
      hipLaunchKernelGGL((k_faith_hist<true, FM_PK32>), dim3(grid_of(n)), dim3(BLOCK), 0, s, m, (uint32_t)ref, fa,
                         b.sinks_s, n, next_start, b.scal, ctx->g);
    else if (fm == FM_PK64)
      hipLaunchKernelGGL((k_faith_hist<true, FM_PK64>), dim3(grid_of(n)), dim3(BLOCK), 0, s, m, (uint32_t)ref, fa,
                         b.sinks_s, n, next_start, b.scal, ctx->g);
    else
      hipLaunchKernelGGL(k_faith_hist<false>, dim3(grid_of(n)), dim3(BLOCK), 0, s, m, (uint32_t)ref, fa, b.sinks_s, n,
                         next_start, b.scal, ctx->g);
  }
  hipLaunchKernelGGL(k_faith_finish, dim3(1), dim3(1), 0, s, m, (uint32_t)ref, n, n_total, is_last, pmax_in, b.pmax,
                     b.scal, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->tables_dirty = true;
  return PLUSS_OK;
}

// the radix-sort pipeline of one sampler_<REF> over its buffer set, on stream s
static int faith_pipeline_sorted(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, const uint64_t* d_samples, uint64_t n,
                                 hipStream_t s) {
  if (n == 0) return PLUSS_OK;
  if (int rc = faith_keys(ctx, b, ref, d_samples, n, 0, 0, nullptr, s)) return rc;
  if (int rc = faith_sort(ctx, b, ref, n, s, false)) return rc;
  const int fm = faith_fm(ctx->m);
  if (fm != FM_PAIRS) {
    const uint64_t nt = fu_tiles(n);
    hipLaunchKernelGGL(k_faith_scan_init, dim3((unsigned)std::min<uint64_t>((2 * nt + BLOCK - 1) / BLOCK + 1, 64)),
                       dim3(BLOCK), 0, s, b.scal, n, b.st, 2 * nt);
    const PkView pv = make_pkview(ctx->m, (uint32_t)ref);
    const unsigned long long endkey = ctx->m.A * ctx->m.T;
    unsigned long long* part = b.pmax;  // the prefix max is not stored: its buffer holds the partials
    if (fm == FM_PK32)
      hipLaunchKernelGGL(k_faith_fused<FM_PK32>, dim3((unsigned)nt), dim3(FB), 0, s, (const void*)b.keys_s, pv, n,
                         endkey, b.st, part, b.scal);
    else
      hipLaunchKernelGGL(k_faith_fused<FM_PK64>, dim3((unsigned)nt), dim3(FB), 0, s, (const void*)b.keys_s, pv, n,
                         endkey, b.st, part, b.scal);
    hipLaunchKernelGGL(k_faith_fused_finish, dim3(1), dim3(BLOCK), 0, s, (uint32_t)ref, n, pv, b.st, nt, part,
                       b.scal, ctx->g);
    PLUSS_HIP_CHECK(hipGetLastError());
    ctx->tables_dirty = true;
    return PLUSS_OK;
  }
  const uint64_t nw = 2 * sc_tiles(n);
  hipLaunchKernelGGL(k_faith_scan_init, dim3((unsigned)std::min<uint64_t>((nw + BLOCK - 1) / BLOCK + 1, 64)),
                     dim3(BLOCK), 0, s, b.scal, n, b.st, nw);
  const FlagArgs fa{b.keys_s, b.pmax, 0, 0, make_pkview(ctx->m, (uint32_t)ref)};
  const dim3 grid((unsigned)sc_tiles(n));
  if (fm == FM_PK32)
    hipLaunchKernelGGL(k_faith_scan<FM_PK32>, grid, dim3(BLOCK), 0, s, fa, b.sinks_s, b.pmax, n, b.st, b.scal);
  else if (fm == FM_PK64)
    hipLaunchKernelGGL(k_faith_scan<FM_PK64>, grid, dim3(BLOCK), 0, s, fa, b.sinks_s, b.pmax, n, b.st, b.scal);
  else
    hipLaunchKernelGGL(k_faith_scan<FM_PAIRS>, grid, dim3(BLOCK), 0, s, fa, b.sinks_s, b.pmax, n, b.st, b.scal);
  PLUSS_HIP_CHECK(hipGetLastError());
  return faith_record(ctx, b, ref, n, 0, 0, 0, n, 1, s);
}

// One sampler_<REF>: keys, radix sort, fused scan.
int launch_faithful(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, hipStream_t s) {
  if (int rc = faith_check_shape(ctx)) return rc;
  FaithfulBufs& b = ctx->fb;
  if (int rc = faith_reserve(ctx, b, n, s)) return rc;
  return faith_pipeline_sorted(ctx, b, ref, d_samples, n, s);
}

// ---- direct passes over key-ordered lists: no keys pass, no sort.  One
// launch of k_faith_fused_direct (FCHUNK-element tiles chained by decoupled
// look-back) and the finish kernel.
static int faith_direct_shape(const pluss_ctx* ctx, const char* api) {
  if (int rc = faith_check_shape(ctx)) return rc;
  if (!ctx->m.fast) {
    set_error(std::string(api) + ": needs N % (cls/ds) == 0 (packed words); use pluss_dev_faithful_hist");
    return PLUSS_ERR_CONFIG;
  }
  return PLUSS_OK;
}

static int faith_reserve_direct(FaithfulBufs& b, uint64_t n, hipStream_t s) {
  if (!b.scal) {
    if (int rc = grow(&b.scal, 8)) return rc;
  }
  if (n > 0xFFFFFFFFull) {
    set_error("faithful mode: at most 2^32-1 samples per reference");
    return PLUSS_ERR_CONFIG;
  }
  const uint64_t nt = fu_tiles(n);
  if (nt > b.dcap) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    int rc = 0;
    if ((rc = grow(&b.dst, 2 * nt)) || (rc = grow(&b.dpart, nt * FPART))) return rc;
    b.dcap = nt;
  }
  return PLUSS_OK;
}

// kg == nullptr: the samples are read from d_samples (checked to be in key order)
static int faith_pipeline_direct(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, const uint64_t* d_samples,
                                 const KeyGen* kg, uint64_t n, hipStream_t s) {
  if (n == 0) return PLUSS_OK;
  const Model& m = ctx->m;
  const uint64_t nt = fu_tiles(n);
  hipLaunchKernelGGL(k_faith_scan_init, dim3((unsigned)std::min<uint64_t>((2 * nt + BLOCK - 1) / BLOCK + 1, 64)),
                     dim3(BLOCK), 0, s, b.scal, n, b.dst, 2 * nt);
  const PkView pv = make_pkview(m, (uint32_t)ref);
  const unsigned long long endkey = m.A * m.T;
  const KeyGen k = kg ? *kg : KeyGen{};
  const bool pk32 = faith_fm(m) == FM_PK32;
#define PLUSS_DIRECT(FMV, GENV)                                                                                  \
  hipLaunchKernelGGL((k_faith_fused_direct<FMV, GENV>), dim3((unsigned)nt), dim3(FB), 0, s, m, (uint32_t)ref, \
                     d_samples, k, pv, n, endkey, b.dst, b.dpart, b.scal, ctx->g)
  if (kg) {
    if (pk32) PLUSS_DIRECT(FM_PK32, true);
    else PLUSS_DIRECT(FM_PK64, true);
  } else {
    if (pk32) PLUSS_DIRECT(FM_PK32, false);
    else PLUSS_DIRECT(FM_PK64, false);
  }
#undef PLUSS_DIRECT
  hipLaunchKernelGGL(k_faith_fused_finish, dim3(1), dim3(BLOCK), 0, s, (uint32_t)ref, n, pv, b.dst, nt, b.dpart,
                     b.scal, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->tables_dirty = true;
  return PLUSS_OK;
}

int launch_faithful_sorted(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, hipStream_t s) {
  if (int rc = faith_direct_shape(ctx, "pluss_dev_faithful_hist_sorted")) return rc;
  if (int rc = faith_reserve_direct(ctx->fb, n, s)) return rc;
  return faith_pipeline_direct(ctx, ctx->fb, ref, d_samples, nullptr, n, s);
}

// The six references' pipelines on streams of their own, forked from s and
// joined back into it, as r10's main runs one thread per reference
// (r10:3203-3257).  per_ref(r, buffers, stream) enqueues reference r.
template <class F>
static int fork_refs(pluss_ctx* ctx, const uint64_t* counts, hipStream_t s, F&& per_ref) {
  if (!ctx->fst[0]) {
    for (int r = 0; r < 6; ++r) PLUSS_HIP_CHECK(hipStreamCreateWithFlags(&ctx->fst[r], hipStreamNonBlocking));
    for (int e = 0; e < 7; ++e) PLUSS_HIP_CHECK(hipEventCreateWithFlags(&ctx->fev[e], hipEventDisableTiming));
  }
  PLUSS_HIP_CHECK(hipEventRecord(ctx->fev[6], s));
  for (int r = 0; r < 6; ++r) {
    if (!counts[r]) continue;
    PLUSS_HIP_CHECK(hipStreamWaitEvent(ctx->fst[r], ctx->fev[6], 0));
    if (int rc = per_ref(r, ctx->fbr[r], ctx->fst[r])) return rc;
    PLUSS_HIP_CHECK(hipEventRecord(ctx->fev[r], ctx->fst[r]));
    PLUSS_HIP_CHECK(hipStreamWaitEvent(s, ctx->fev[r], 0));
  }
  return PLUSS_OK;
}

// All six sampler_<REF> of one list at once (radix-sort pipeline).
int launch_faithful_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t* counts, hipStream_t s) {
  if (int rc = faith_check_shape(ctx)) return rc;
  uint64_t off[6], total = 0;
  for (int r = 0; r < 6; ++r) {
    off[r] = total;
    total += counts[r];
  }
  if (total && !d_samples) {
    set_error("pluss_dev_faithful_hist_refs: null sample list");
    return PLUSS_ERR_CONFIG;
  }
  for (int r = 0; r < 6; ++r) {  // every allocation before the fork
    if (!counts[r]) continue;
    if (int rc = faith_reserve(ctx, ctx->fbr[r], counts[r], s)) return rc;
    if (int rc = faith_tmp(ctx, ctx->fbr[r], counts[r], s)) return rc;
  }
  return fork_refs(ctx, counts, s, [&](int r, FaithfulBufs& b, hipStream_t rs) {
    return faith_pipeline_sorted(ctx, b, r, d_samples + off[r], counts[r], rs);
  });
}

// All six over a key-ordered list (each reference's block in key order).
int launch_faithful_sorted_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t* counts, hipStream_t s) {
  if (int rc = faith_direct_shape(ctx, "pluss_dev_faithful_hist_sorted_refs")) return rc;
  uint64_t off[6], total = 0;
  for (int r = 0; r < 6; ++r) {
    off[r] = total;
    total += counts[r];
  }
  if (total && !d_samples) {
    set_error("pluss_dev_faithful_hist_sorted_refs: null sample list");
    return PLUSS_ERR_CONFIG;
  }
  for (int r = 0; r < 6; ++r)
    if (counts[r])
      if (int rc = faith_reserve_direct(ctx->fbr[r], counts[r], s)) return rc;
  return fork_refs(ctx, counts, s, [&](int r, FaithfulBufs& b, hipStream_t rs) {
    return faith_pipeline_direct(ctx, b, r, d_samples + off[r], nullptr, counts[r], rs);
  });
}

// All six over generated key-order lists (pluss_expand_sorted's lists of
// totals[r] samples, never written to memory).
int launch_gen_faithful_refs(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, hipStream_t s) {
  if (int rc = faith_direct_shape(ctx, "pluss_dev_gen_faithful_refs")) return rc;
  KeyGen kg[6];
  for (int r = 0; r < 6; ++r) {
    if (!totals[r]) continue;
    if (int rc = keygen_check(ctx, r, totals[r], 0, totals[r], "pluss_dev_gen_faithful_refs")) return rc;
    kg[r] = keygen_of(ctx, seed, r, totals[r]);
    if (int rc = faith_reserve_direct(ctx->fbr[r], totals[r], s)) return rc;
  }
  return fork_refs(ctx, totals, s, [&](int r, FaithfulBufs& b, hipStream_t rs) {
    return faith_pipeline_direct(ctx, b, r, nullptr, &kg[r], totals[r], rs);
  });
}

// ---- key-range shards (multi-GPU faithful mode; the caller exchanges the
// ---- per-shard summaries between phases)
int faith_shard_keys(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, uint64_t lo, uint64_t hi,
                     pluss_faith_shard* out, hipStream_t s) {
  FaithfulBufs& b = ctx->fb;
  if (int rc = faith_check_shape(ctx)) return rc;
  if (int rc = faith_reserve(ctx, b, n, s)) return rc;
  FaithShard& f = ctx->fsh;
  f = FaithShard{};
  f.ref = ref;
  PLUSS_HIP_CHECK(hipMemsetAsync(b.scal + 3, 0, 8, s));
  if (n)
    if (int rc = faith_keys(ctx, b, ref, d_samples, n, lo, hi, b.scal + 3, s)) return rc;
  unsigned long long m = 0;
  PLUSS_HIP_CHECK(hipMemcpyAsync(&m, b.scal + 3, 8, hipMemcpyDeviceToHost, s));
  PLUSS_HIP_CHECK(hipStreamSynchronize(s));
  f.n = m;
  out->n = m;
  out->first_key = KEY_EMPTY;
  out->max_sink = 0;
  if (m) {
    if (int rc = faith_sort(ctx, b, ref, m, s)) return rc;
    const int fm = faith_fm(ctx->m);
    unsigned long long w64 = 0;
    uint32_t w32 = 0;
    if (fm == FM_PK32) PLUSS_HIP_CHECK(hipMemcpyAsync(&w32, b.keys_s, 4, hipMemcpyDeviceToHost, s));
    else PLUSS_HIP_CHECK(hipMemcpyAsync(&w64, b.keys_s, 8, hipMemcpyDeviceToHost, s));
    PLUSS_HIP_CHECK(hipMemcpyAsync(&out->max_sink, b.pmax + (m - 1), 8, hipMemcpyDeviceToHost, s));
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    const PkView pv = make_pkview(ctx->m, (uint32_t)ref);  // the smallest key of the shard
    out->first_key = fm == FM_PK32 ? pk_key(w32, pv) : (fm == FM_PK64 ? pk_key(w64, pv) : w64);
  }
  f.max_sink = out->max_sink;
  f.phase = 1;
  return PLUSS_OK;
}

int faith_shard_starts(pluss_ctx* ctx, uint64_t j_off, uint64_t pmax_in, pluss_faith_shard* out, hipStream_t s) {
  FaithfulBufs& b = ctx->fb;
  FaithShard& f = ctx->fsh;
  if (f.phase != 1) {
    set_error("pluss_dev_faithful_shard_starts: call pluss_dev_faithful_shard_keys first");
    return PLUSS_ERR_CONFIG;
  }
  f.j_off = j_off;
  f.pmax_in = pmax_in;
  out->n_starts = 0;
  if (f.n) {
    if (int rc = faith_starts(ctx, b, f.ref, f.n, j_off, pmax_in, s)) return rc;
    unsigned int c = 0;
    PLUSS_HIP_CHECK(hipMemcpyAsync(&c, b.nstart + (f.n - 1), 4, hipMemcpyDeviceToHost, s));
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    out->n_starts = c;
  }
  f.phase = 2;
  return PLUSS_OK;
}

int faith_shard_cut(pluss_ctx* ctx, uint64_t s_off, uint64_t n_total, pluss_faith_shard* out, hipStream_t s) {
  FaithfulBufs& b = ctx->fb;
  FaithShard& f = ctx->fsh;
  if (f.phase != 2) {
    set_error("pluss_dev_faithful_shard_cut: call pluss_dev_faithful_shard_starts first");
    return PLUSS_ERR_CONFIG;
  }
  if (f.j_off + f.n > n_total) {
    set_error("pluss_dev_faithful_shard_cut: n_total is smaller than this shard's end");
    return PLUSS_ERR_CONFIG;
  }
  f.n_total = n_total;
  out->cut = n_total;
  if (f.n) {
    hipLaunchKernelGGL(k_faith_init, dim3(1), dim3(1), 0, s, b.scal, n_total);
    if (int rc = faith_cut(ctx, b, f.ref, f.n, f.j_off, f.pmax_in, s_off, n_total, s)) return rc;
    PLUSS_HIP_CHECK(hipMemcpyAsync(&out->cut, b.scal, 8, hipMemcpyDeviceToHost, s));
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
  }
  f.phase = 3;
  return PLUSS_OK;
}

int faith_shard_hist(pluss_ctx* ctx, uint64_t cut, uint64_t next_first_key, int is_last, hipStream_t s) {
  FaithfulBufs& b = ctx->fb;
  FaithShard& f = ctx->fsh;
  if (f.phase != 3) {
    set_error("pluss_dev_faithful_shard_hist: call pluss_dev_faithful_shard_cut first");
    return PLUSS_ERR_CONFIG;
  }
  if (cut > f.n_total) {
    set_error("pluss_dev_faithful_shard_hist: cut > n_total");
    return PLUSS_ERR_CONFIG;
  }
  const unsigned long long last = f.max_sink > f.pmax_in ? f.max_sink : f.pmax_in;  // global pmax at the shard end
  const int next_start = next_first_key != KEY_EMPTY && next_first_key > last;
  hipLaunchKernelGGL(k_faith_init, dim3(1), dim3(1), 0, s, b.scal, cut);
  f.phase = 0;
  return faith_record(ctx, b, f.ref, f.n, f.j_off, f.pmax_in, next_start, f.n_total, is_last, s);
}

}  // namespace pluss
