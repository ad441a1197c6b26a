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

// ---- the one-GPU scan over key-ordered elements, the six references of a
// list in ONE pipeline of four launches (whatever the element source: sorted
// packed words after the radix sort, a caller's key-ordered samples, or
// samples generated in key order):
//   k_fa_max     per tile of TILE elements: the largest sink (a caller's list:
//                the key-order check; samples / generated lists: the packed
//                sort word of every element, written once for the scan);
//   k_fa_prefix  one workgroup per reference: exclusive prefix max of the
//                tile maxima = the running max of sinks entering each tile;
//   k_fa_scan    every tile independently (no chain across tiles): prefix
//                max inside the tile, start flags, the tile's start count,
//                its Q1 bound (hmax) and the records of all its elements;
//   k_fa_finish  one workgroup per reference: the exclusive sum of the start
//                counts locates the tile holding the Q1 cut (the condition
//                j - starts_before_j >= n - j is monotone in j), the tiles
//                before it are summed, that tile is scanned again below the
//                cut; Q3, the -1 key, traversed, the bins.
constexpr int TB = 256, TI = 16;            // threads per tile, elements per thread
constexpr uint32_t TILE = TB * TI;          // elements per tile
constexpr int FPART = 5;                    // per tile: cold (tid 0), traversed, case 0/1/2 counts
__host__ __device__ inline uint64_t fa_tiles(uint64_t n) { return (n + TILE - 1) / TILE; }

enum : int { SRC_W32 = 0, SRC_W64 = 1, SRC_SAMPLES = 2, SRC_GEN = 3 };

struct FaRefs {
  uint64_t n[6];
  uint64_t toff[7];    // first (global) tile of each reference; toff[6] = all tiles
  const void* src[6];  // SRC_W*: sorted packed words; SRC_SAMPLES: the key-ordered samples
  PkView pv[6];
  KeyGen kg[6];        // SRC_GEN
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

template <bool P2>
__device__ __forceinline__ Elem elem_of_sample(const Model& m, const PkView& v, uint32_t ref, uint64_t x, GTable g) {
  const Sample s = unpack(x);
  if (s.ref != ref || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N) {
    atomicOr(&g.flags[1], 1u);
    return Elem{KEY_EMPTY, KEY_EMPTY, 3u, 0u, ~0ull};
  }
  KeyDigits d;
  d.c1 = s.c1;
  d.c2 = (ref == C0 || ref == C1) ? 0u : s.c2;
  if (P2) {
    const uint32_t k = s.c0 >> m.csshift;
    d.t = k & (m.T - 1);
    d.q = ((k >> v.tsh) << m.csshift) | (s.c0 & m.csmask);
  } else {
    const uint32_t k = fdiv(s.c0, m.dCS), kt = fdiv(k, m.dT);
    d.t = k - kt * m.T;
    d.q = kt * m.CS + (s.c0 - k * m.CS);
  }
  return elem_of_digits<P2>(m, v, ref, d);
}

// a packed sort word (rank << 2 | case), rank = ((q*N + c1)*N + c2)*T + tid
template <bool P2, typename KT>
__device__ __forceinline__ Elem elem_of_word(const Model& m, const PkView& v, uint32_t ref, KT w) {
  if (w == (KT) ~(KT)0) return Elem{KEY_EMPTY, KEY_EMPTY, 3u, 0u, ~0ull};
  uint64_t r = (uint64_t)(w >> 2);
  KeyDigits d;
  if (P2) {
    d.t = (uint32_t)(r & (v.T - 1));
    r >>= v.tsh;
    d.c2 = (uint32_t)(r & (v.N - 1));
    r >>= v.nsh;
    d.c1 = (uint32_t)(r & (v.N - 1));
    d.q = (uint32_t)(r >> v.nsh);
  } else {
    d.t = (uint32_t)(r % v.T);
    r /= v.T;
    d.c2 = (uint32_t)(r % v.N);
    r /= v.N;
    d.c1 = (uint32_t)(r % v.N);
    d.q = (uint32_t)(r / v.N);
  }
  const uint32_t c = (uint32_t)(w & 3u);
  const uint64_t a = ((uint64_t)d.q * m.N + d.c1) * m.S + ref_off(ref, d.c2);
  const uint64_t key = P2 ? ((a << v.tsh) | d.t) : a * m.T + d.t;
  const int64_t ri = c == 0 ? v.ri[0] : (c == 1 ? v.ri[1] : v.ri[2]);
  const unsigned long long dt = P2 ? ((unsigned long long)ri << v.tsh) : (unsigned long long)ri * m.T;
  return Elem{key, (c == 3 || ri < 0) ? KEY_EMPTY : key + dt, c, d.t == 0 ? 1u : 0u, (unsigned long long)w};
}

template <int SRC>
using fa_raw_t = typename std::conditional<SRC == SRC_W32, uint32_t, unsigned long long>::type;

// element i of reference r read straight from the source (global memory)
template <int SRC, bool P2>
__device__ __forceinline__ Elem fa_elem(const Model& m, const FaRefs& a, uint32_t r, uint64_t i, GTable g) {
  if (SRC == SRC_GEN) return elem_of_digits<P2>(m, a.pv[r], r, keygen_digits_at(a.kg[r], i));
  const fa_raw_t<SRC> w = static_cast<const fa_raw_t<SRC>*>(a.src[r])[i];
  if (SRC == SRC_SAMPLES) return elem_of_sample<P2>(m, a.pv[r], r, (uint64_t)w, g);
  return elem_of_word<P2>(m, a.pv[r], r, w);
}

// A tile's elements as read from memory (raw words / samples), staged in LDS:
// loaded coalesced (thread x, round k: element k*TB + x), read back by each
// thread as its contiguous run (x*TI + k).  One padding slot per TI elements
// keeps the run reads at 2-way bank conflicts.
constexpr uint32_t FA_LDS = TILE + TILE / TI;
__device__ __forceinline__ uint32_t fa_slot(uint32_t e) { return e + e / TI; }

template <int SRC>
__device__ __forceinline__ void fa_stage(const FaRefs& a, uint32_t r, uint64_t base, uint32_t mt,
                                         fa_raw_t<SRC>* lds) {
  if (SRC == SRC_GEN) return;
  const fa_raw_t<SRC>* src = static_cast<const fa_raw_t<SRC>*>(a.src[r]) + base;
#pragma unroll
  for (int k = 0; k < TI; ++k) {
    const uint32_t e = (uint32_t)k * TB + threadIdx.x;
    if (e < mt) lds[fa_slot(e)] = src[e];
  }
  __syncthreads();
}

// A lane's run of consecutive elements: read from the staged tile, or
// generated in sequence (GEN: keyrunf_* when the whole tile lies in block A
// with small strata -- tile-uniform -- else one direct decode per sample).
template <int SRC, bool P2>
struct FaCursor {
  const Model& m;
  const FaRefs& a;
  uint32_t r;
  uint64_t base;
  uint32_t e;
  const fa_raw_t<SRC>* lds;
  GTable g;
  bool fast;
  KeyRunF run;
  __device__ FaCursor(const Model& m_, const FaRefs& a_, uint32_t r_, uint64_t base_, uint32_t e0,
                      const fa_raw_t<SRC>* lds_, GTable g_)
      : m(m_), a(a_), r(r_), base(base_), e(e0), lds(lds_), g(g_), fast(false) {
    if (SRC == SRC_GEN) {
      fast = keyrun_fast_ok(a.kg[r], base, TILE);
      if (fast) keyrunf_start(a.kg[r], run, base + e0);
    }
  }
  // the element at the cursor; then the cursor moves on
  __device__ Elem next() {
    Elem x;
    if (SRC == SRC_GEN) {
      if (fast) {
        x = elem_of_digits<P2>(m, a.pv[r], r, keyrunf_digits(a.kg[r], run));
        keyrunf_next(a.kg[r], run);
      } else {
        x = elem_of_digits<P2>(m, a.pv[r], r, keygen_digits_at(a.kg[r], base + e));
      }
    } else {
      const fa_raw_t<SRC> w = lds[fa_slot(e)];
      if (SRC == SRC_SAMPLES) x = elem_of_sample<P2>(m, a.pv[r], r, (uint64_t)w, g);
      else x = elem_of_word<P2>(m, a.pv[r], r, w);
    }
    ++e;
    return x;
  }
};

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

// the one reference a scanned tile belongs to (copied out of FaRefs by the
// kernel, so the body never indexes the kernel argument itself)
struct FaOne {
  FaTile T;
  uint64_t n;
  const void* src;
  PkView pv;
};
__device__ __forceinline__ FaOne fa_one(const FaRefs& a, uint64_t gt) {
  FaOne o;
  o.T = fa_tile(a, gt);
  o.n = a.n[o.T.r];
  o.src = a.src[o.T.r];
  o.pv = a.pv[o.T.r];
  return o;
}

// ---- pass 1 (k_fa_max*): per tile, the largest sink; for a caller's list
// the key-order check; for sample / generated sources also the packed sort
// word of every element (written once, read by the scan).
//
// Lists in memory (sorted words, a caller's samples): element-strided, thread
// x round k holds element k*TB + x, so every load and word store is coalesced
// and no LDS staging is needed (occupancy is not capped by LDS).  The body is
// instantiated per reference (tile-uniform switch), so the decode and the
// case rules fold to the reference's own few instructions.
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

template <int SRC, bool CHECK, bool P2, int WK, uint32_t REF>
__device__ __forceinline__ void fa_max_tile(const Model& m, const FaOne& o, unsigned long long* __restrict__ tmax,
                                            void* words, GTable g, unsigned long long* s_w,
                                            unsigned long long (*s_first)[TB / 64],
                                            unsigned long long (*s_last)[TB / 64]) {
  using wk_t = typename std::conditional<WK == 8, unsigned long long, uint32_t>::type;
  constexpr int NW = TB / 64;
  const FaTile& T = o.T;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const fa_raw_t<SRC>* src = static_cast<const fa_raw_t<SRC>*>(o.src) + T.base;
  wk_t* out = static_cast<wk_t*>(words) + blockIdx.x * (uint64_t)TILE;
  const bool full = T.mt == TILE;
  fa_raw_t<SRC> raw[TI];
#pragma unroll
  for (int k = 0; k < TI; ++k) {  // every load in flight before the first decode
    const uint32_t e = (uint32_t)k * TB + threadIdx.x;
    raw[k] = (full || e < T.mt) ? src[e] : (fa_raw_t<SRC>)0;
  }
  unsigned long long tm = 0;
  bool bad = false, unordered = false;
#pragma unroll
  for (int k = 0; k < TI; ++k) {
    const uint32_t e = (uint32_t)k * TB + threadIdx.x;
    const bool v = full || e < T.mt;
    Elem x{KEY_EMPTY, 0ull, 3u, 0u, ~0ull};
    if (v) {
      x = fa_decode_ref<SRC, P2, REF>(m, o.pv, raw[k], bad);
      tm = x.sink > tm ? x.sink : tm;
      if (WK) out[e] = (wk_t)x.w;
    }
    if (CHECK) {  // strictly increasing keys: against the previous lane here, across waves/rounds below
      const unsigned long long up = __shfl_up(x.key, 1, 64);
      unordered |= v && lane > 0 && !(x.key > up);
      if (lane == 0) s_first[k][wid] = x.key;
      if (lane == 63) s_last[k][wid] = x.key;
    }
  }
  if (CHECK) {
    __syncthreads();
    if (threadIdx.x < TI * NW) {  // the first element of (round k, wave w) against the element before it
      const uint32_t k = threadIdx.x / NW, w = threadIdx.x % NW;
      const uint32_t e = k * TB + w * 64;
      if (e < T.mt && (e > 0 || T.base > 0)) {
        bool b2 = false;
        const unsigned long long prev =
            e > 0 ? (w > 0 ? s_last[k][w - 1] : s_last[k - 1][NW - 1]) : fa_decode_ref<SRC, P2, REF>(m, o.pv, src[-1], b2).key;
        unordered |= !(s_first[k][w] > prev);
      }
    }
  }
  if (__ballot(bad || unordered) && lane == 0) atomicOr(&g.flags[1], 1u);
  tm = sc_wave_red<true>(tm);
  if (lane == 0) s_w[wid] = tm;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long x = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) x = s_w[w] > x ? s_w[w] : x;
    tmax[blockIdx.x] = x;
  }
}

// the reference's first tile also materialises its -1 (cold) key in the main
// table and keeps the slot, so the finish pass only adds the count
__device__ __forceinline__ void fa_cold_slot(const FaTile& T, GTable g, unsigned long long* slots) {
  if (T.lt == 0 && threadIdx.x == 0) slots[T.r] = g_slot(g, make_key(T.r, 0, -1));
}

template <int SRC, bool CHECK, bool P2, int WK>
__global__ __launch_bounds__(TB) void k_fa_max(Model m, FaRefs a, unsigned long long* __restrict__ tmax, void* words,
                                               unsigned long long* slots, GTable g) {
  static_assert(SRC != SRC_GEN, "generated lists: k_fa_max_gen");
  constexpr int NW = TB / 64;
  __shared__ unsigned long long s_w[NW];
  __shared__ unsigned long long s_first[CHECK ? TI : 1][NW], s_last[CHECK ? TI : 1][NW];
  const FaOne o = fa_one(a, blockIdx.x);
  fa_cold_slot(o.T, g, slots);
#define PLUSS_FA_MAX(R) fa_max_tile<SRC, CHECK, P2, WK, R>(m, o, tmax, words, g, s_w, s_first, s_last)
  switch (o.T.r) {
    case C0: PLUSS_FA_MAX(C0); break;
    case C1: PLUSS_FA_MAX(C1); break;
    case A0: PLUSS_FA_MAX(A0); break;
    case B0: PLUSS_FA_MAX(B0); break;
    case C2: PLUSS_FA_MAX(C2); break;
    default: PLUSS_FA_MAX(C3); break;
  }
#undef PLUSS_FA_MAX
}

// Generated lists: each lane generates its run of TI consecutive elements
// (incremental key-order digits: keyrunf_* when the whole tile lies in block A
// with small strata -- tile-uniform -- else one direct decode per sample), the
// words go out through LDS (coalesced).  Instantiated per reference.
template <bool P2, int WK, uint32_t REF>
__device__ __forceinline__ void fa_gen_tile(const Model& m, const KeyGen& kg, const PkView& pv, const FaTile& T,
                                            unsigned long long* __restrict__ tmax, void* words,
                                            unsigned long long* s_w, void* s_wd_) {
  using wk_t = typename std::conditional<WK == 8, unsigned long long, uint32_t>::type;
  wk_t* s_wd = static_cast<wk_t*>(s_wd_);
  constexpr int NW = TB / 64;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t e0 = threadIdx.x * TI;
  unsigned long long tm = 0;
  if (keyrun_fast_ok(kg, T.base, TILE)) {  // the whole tile: every lane's run is in range
    KeyRunF run;
    keyrunf_start(kg, run, T.base + e0);
#pragma unroll
    for (int k = 0; k < TI; ++k) {
      const Elem e = elem_of_digits<P2>(m, pv, REF, keyrunf_digits(kg, run));
      keyrunf_next(kg, run);
      tm = e.sink > tm ? e.sink : tm;
      s_wd[fa_slot(e0 + k)] = (wk_t)e.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < TI; ++k) {
      if (e0 + k < T.mt) {
        const Elem e = elem_of_digits<P2>(m, pv, REF, keygen_digits_at(kg, T.base + e0 + k));
        tm = e.sink > tm ? e.sink : tm;
        s_wd[fa_slot(e0 + k)] = (wk_t)e.w;
      }
    }
  }
  __syncthreads();
  wk_t* out = static_cast<wk_t*>(words) + blockIdx.x * (uint64_t)TILE;
#pragma unroll
  for (int k = 0; k < TI; ++k) {
    const uint32_t e = k * TB + threadIdx.x;
    if (e < T.mt) out[e] = s_wd[fa_slot(e)];
  }
  tm = sc_wave_red<true>(tm);
  if (lane == 0) s_w[wid] = tm;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long x = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) x = s_w[w] > x ? s_w[w] : x;
    tmax[blockIdx.x] = x;
  }
}

template <bool P2, int WK>
__global__ __launch_bounds__(TB) void k_fa_max_gen(Model m, FaRefs a, unsigned long long* __restrict__ tmax,
                                                   void* words, unsigned long long* slots, GTable g) {
  using wk_t = typename std::conditional<WK == 8, unsigned long long, uint32_t>::type;
  __shared__ unsigned long long s_w[TB / 64];
  __shared__ wk_t s_wd[FA_LDS];
  const FaTile T = fa_tile(a, blockIdx.x);
  fa_cold_slot(T, g, slots);
  // (the reference's generator and view copied out first: the kernel argument
  // itself is never passed down, which would put a copy of it in scratch)
#define PLUSS_FA_GEN(R)                                               \
  {                                                                   \
    const KeyGen kg = a.kg[R];                                        \
    const PkView pv = a.pv[R];                                        \
    fa_gen_tile<P2, WK, R>(m, kg, pv, T, tmax, words, s_w, s_wd);     \
  }
  switch (T.r) {
    case C0: PLUSS_FA_GEN(C0); break;
    case C1: PLUSS_FA_GEN(C1); break;
    case A0: PLUSS_FA_GEN(A0); break;
    case B0: PLUSS_FA_GEN(B0); break;
    case C2: PLUSS_FA_GEN(C2); break;
    default: PLUSS_FA_GEN(C3); break;
  }
#undef PLUSS_FA_GEN
}

// One workgroup per reference: pmin[t] = max of tmax over the reference's
// tiles before t (0 for its first).
constexpr int PB = 1024;
__global__ __launch_bounds__(PB) void k_fa_prefix(FaRefs a, const unsigned long long* __restrict__ tmax,
                                                  unsigned long long* __restrict__ pmin) {
  __shared__ unsigned long long s_w[PB / 64];
  const uint32_t r = blockIdx.x;
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

// ---- pass 2: the scan of one tile of packed words (TB threads; thread x
// owns the run [x*TI, (x+1)*TI), staged through LDS).  carry = the largest
// sink before the tile (pmin).  The start counts need no chain across tiles:
//   CUT = false (k_fa_scan, all tiles at once): the tile's start count, its
//     hmax = 2j - (starts of the tile before j) at its last start j > 0, and
//     the records of ALL its elements.  Q1's condition j - before_j >= n - j
//     is 2j - before_j >= n, increasing in j; with c_in starts before the
//     tile it holds at the tile's last start iff hmax >= n + c_in, so the cut
//     lies in the first tile where that holds, and every earlier tile is
//     recorded whole;
//   CUT = true (k_fa_finish, that one tile, c_in known): the cut and the
//     records below it.
// sh.out[0, FPART): cold, traversed, case 0/1/2 counts; sh.out[FPART]: the
// start count (CUT: the cut); sh.out[FPART + 1]: hmax.  (Results go through
// LDS: a store through a generic pointer here would keep the kernels' FaRefs
// argument copied to scratch.)
constexpr int FPW = FPART + 2;
template <int SRC, int NT = TB, int EPT = TI>
struct FaScanLds {
  unsigned long long w[NT / 64], c[NT / 64], red[NT / 64][FPW], out[FPW];
  unsigned long long rt[4];  // ri*T per case (KEY_EMPTY: cold; case 3: malformed)
  fa_raw_t<SRC> raw[TILE + TILE / EPT];
};
// LDS slot of tile element e for runs of EPT elements per thread (one pad per run)
template <int EPT>
__device__ __forceinline__ uint32_t fa_slot_n(uint32_t e) { return e + e / EPT; }


template <int SRC, bool P2, bool CUT, int NT, int EPT, bool FULLT>
__device__ __forceinline__ void fa_tile_scan_t(const Model& m, const FaOne& o, unsigned long long carry_in,
                                               uint64_t c_in, FaScanLds<SRC, NT, EPT>& sh) {
  static_assert(NT * EPT == (int)TILE && EPT <= 16, "a tile is NT threads x EPT elements");
  static_assert(SRC == SRC_W32 || SRC == SRC_W64, "the scan reads packed words");
  using raw_t = fa_raw_t<SRC>;
  constexpr int NW = NT / 64;
  const FaTile& T = o.T;
  constexpr bool full = FULLT;  // a whole tile: no per-element bounds in the loops below
  // ri*T per case (KEY_EMPTY: a cold case; case 3 = a malformed word, already flagged)
  unsigned long long rt[4];
#pragma unroll
  for (int c = 0; c < 3; ++c) rt[c] = o.pv.ri[c] < 0 ? KEY_EMPTY : (unsigned long long)o.pv.ri[c] * m.T;
  rt[3] = KEY_EMPTY;
  if (threadIdx.x < 4) sh.rt[threadIdx.x] = rt[threadIdx.x & 3];
  {
    const raw_t* src = static_cast<const raw_t*>(o.src) + T.base;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const uint32_t e = (uint32_t)k * NT + threadIdx.x;
      if (full || e < T.mt) sh.raw[fa_slot_n<EPT>(e)] = src[e];
    }
    __syncthreads();
  }
  const uint32_t r = T.r;
  const uint64_t n = o.n;
  const unsigned long long endkey = m.A * m.T;
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  const uint32_t e0 = threadIdx.x * EPT;                                      // this lane's run in the tile
  const uint32_t nv = e0 < T.mt ? (T.mt - e0 < EPT ? T.mt - e0 : EPT) : 0u;  // its valid elements
  const uint64_t i0 = T.base + e0;                                            // index of its first element
  // decode: keys in registers, cases (2 bits) and tid == 0 (at bit 2k) per
  // element; sinks are recomputed from key and case where needed (registers
  // for occupancy: this pass waits on its tile loads)
  unsigned long long key[EPT];
  auto sink_of = [&](unsigned long long kk, uint32_t c) -> unsigned long long {
    const unsigned long long d = sh.rt[c];  // an LDS table: no divergent selects
    const unsigned long long x = kk + d;    // d == KEY_EMPTY wraps below d: the max keeps KEY_EMPTY
    return x > d ? x : d;
  };
  uint32_t cases = 0, t0s = 0;
  unsigned long long lmax = 0;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    key[k] = KEY_EMPTY;
    if (full || (uint32_t)k < nv) {
      const raw_t w = sh.raw[fa_slot_n<EPT>(e0 + k)];
      uint32_t c, t;
      unsigned long long kk;
      if (P2) {  // rank = ((q*N + c1)*N + c2)*T + tid; q*N + c1 < 2^32 (fa_run)
        c = (uint32_t)w & 3u;
        const raw_t rk = w >> 2;
        t = (uint32_t)rk & (uint32_t)(o.pv.T - 1);
        const uint32_t c2 = (uint32_t)(rk >> o.pv.tsh) & (uint32_t)(o.pv.N - 1);
        const uint32_t qc = (uint32_t)(rk >> (o.pv.tsh + o.pv.nsh));
        const uint64_t a = (uint64_t)qc * (uint32_t)m.S + ref_off(r, c2);
        kk = (a << o.pv.tsh) | t;
      } else {
        const Elem e = elem_of_word<false>(m, o.pv, r, w);
        kk = e.key;
        c = e.c;
        t = e.t0 ? 0u : 1u;
      }
      const unsigned long long sk = sink_of(kk, c);
      key[k] = kk;
      lmax = sk > lmax ? sk : lmax;
      cases |= c << (2 * k);
      t0s |= (t == 0 ? 1u : 0u) << (2 * k);
    }
  }
  // running max of sinks entering this lane: the tile's incoming max, the
  // earlier waves' maxima, the earlier lanes' maxima
  const unsigned long long linc = sc_wave_scan<true>(lmax, lane);
  if (lane == 63) sh.w[wid] = linc;
  __syncthreads();
  unsigned long long carry = carry_in;
#pragma unroll
  for (int x = 0; x < NW; ++x)
    if (x < (int)wid) carry = sh.w[x] > carry ? sh.w[x] : carry;
  {
    const unsigned long long up = __shfl_up(linc, 1, 64);
    if (lane) carry = up > carry ? up : carry;
  }
  // Start flags (key > the running max before it; the reference's first
  // element) and, for the elements below lim, traversed: a replay starting
  // at p subtracts key_p; the replay ending at p - 1 adds the running max
  // there when p starts one, p == cut or p == n.  The end of a tile's last
  // element is counted by the next tile (its first element's boundary).
  uint32_t flags = 0;
  unsigned long long tpos = 0, tneg = 0;
  auto scan = [&](uint64_t lim, bool rec) {
    unsigned long long run = carry;
    flags = 0;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      if (full || (uint32_t)k < nv) {
        const uint64_t p = i0 + k;
        bool f = key[k] > run;
        if (k == 0) f = f || i0 == 0;
        flags |= (f ? 1u : 0u) << k;
        if (rec) {
          if (p < lim) {
            if (f) {
              tneg += key[k];
              if (p != 0) tpos += run;  // f implies run is a sink (not KEY_EMPTY)
            }
          } else if (CUT && p == lim) {
            tpos += run == KEY_EMPTY ? endkey : run;
          }
        }
        const unsigned long long sk = sink_of(key[k], (cases >> (2 * k)) & 3u);
        run = sk > run ? sk : run;
      }
    }
    if (rec && nv && i0 + nv == n && n <= lim) tpos += run == KEY_EMPTY ? endkey : run;  // the last element ends
  };
  if (!CUT) scan(n, true);
  else scan(n, false);
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
  uint64_t cut = n;
  unsigned long long hl = 0;
  if (CUT) {  // the first start j > 0 with j - before_j >= n - j; then the records below it
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
    if (rt[c] == KEY_EMPTY) packed += (unsigned long long)__popc(mc[c] & t0s);
    else packed += (unsigned long long)__popc(mc[c]) << (16 * (c + 1));
  }
  const unsigned long long v[3] = {sc_wave_red<false>(packed), sc_wave_red<false>(tpos - tneg),
                                   CUT ? 0ull : sc_wave_red<true>(hl)};
  if (lane == 0)
#pragma unroll
    for (int f = 0; f < 3; ++f) sh.red[wid][f] = v[f];
  __syncthreads();
  if (threadIdx.x < FPW) {
    unsigned long long x = 0;
    const uint32_t f = threadIdx.x;
    if (f == FPART) {
      x = CUT ? cut : cagg;
    } else if (f == FPART + 1) {
#pragma unroll
      for (int w = 0; w < NW; ++w) x = sh.red[w][2] > x ? sh.red[w][2] : x;
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

template <int SRC, bool P2, bool CUT, int NT = TB, int EPT = TI>
__device__ __forceinline__ void fa_tile_scan(const Model& m, const FaOne& o, unsigned long long carry_in,
                                             uint64_t c_in, FaScanLds<SRC, NT, EPT>& sh) {
  if (o.T.mt == TILE) fa_tile_scan_t<SRC, P2, CUT, NT, EPT, true>(m, o, carry_in, c_in, sh);
  else fa_tile_scan_t<SRC, P2, CUT, NT, EPT, false>(m, o, carry_in, c_in, sh);
}

template <int SRC, bool P2>
__global__ __launch_bounds__(TB) void k_fa_scan(Model m, FaRefs a, const unsigned long long* __restrict__ pmin,
                                                unsigned long long* __restrict__ part, GTable g) {
  __shared__ FaScanLds<SRC> sh;
  const FaOne o = fa_one(a, blockIdx.x);
  fa_tile_scan<SRC, P2, false>(m, o, pmin[blockIdx.x], 0, sh);
  if (threadIdx.x < FPW) part[blockIdx.x * (uint64_t)FPW + threadIdx.x] = sh.out[threadIdx.x];
}

// ---- pass 3, one workgroup of FT threads per reference with samples: the
// exclusive sum of its tiles' start counts locates the tile holding the Q1
// cut (the first with hmax >= n + starts before it); the tiles before it are
// summed whole, that tile is scanned again with its incoming start count
// (CUT; FT threads x TILE/FT elements); then Q3 (nothing dropped: the owner
// of the final largest sink stays in LAT, +1 cold if it is tid 0), the -1
// key (materialised even with 0, r10:196,671), traversed and the bins.
constexpr int FT = 1024;
template <int SRC, bool P2>
__global__ __launch_bounds__(FT) void k_fa_finish(Model m, FaRefs a, const unsigned long long* __restrict__ tmax,
                                                  const unsigned long long* __restrict__ pmin,
                                                  const unsigned long long* __restrict__ part,
                                                  const unsigned long long* __restrict__ slots, GTable g) {
  constexpr int NW = FT / 64;
  __shared__ FaScanLds<SRC, FT, TILE / FT> sh;
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
    const FaOne o = fa_one(a, t0 + ct);
    fa_tile_scan<SRC, P2, true, FT, TILE / FT>(m, o, pmin[t0 + ct], cin, sh);
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
    } else if (f == 1) {
      atomicAdd(&g.trav[r], x);
    } else if (x) {
      atomicAdd(&g.bins[r * 3 + (f - 2)], x);
    }
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

// ---- the scan pipeline (k_fa_*) over the references with a.n[r] > 0, on
// stream s.  Its buffers are the handle's (ctx->fb): tile maxima, prefixes
// and per-tile partials, sized by the tiles of all references.
static int fa_reserve(FaithfulBufs& b, uint64_t tiles, hipStream_t s) {
  if (!b.fslot) {
    if (int rc = grow(&b.fslot, 8)) return rc;
  }
  if (tiles > b.dcap) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    int rc = 0;
    if ((rc = grow(&b.dpart, tiles * FPW)) || (rc = grow(&b.tmax, tiles)) || (rc = grow(&b.pmin, tiles)))
      return rc;
    b.dcap = tiles;
  }
  return PLUSS_OK;
}

static int fa_run(pluss_ctx* ctx, FaRefs& a, int src, bool check, hipStream_t s) {
  const Model& m = ctx->m;
  uint64_t t = 0;
  for (int r = 0; r < 6; ++r) {
    if (a.n[r] > 0xFFFFFFFFull) {
      set_error("faithful mode: at most 2^32-1 samples per reference");
      return PLUSS_ERR_CONFIG;
    }
    a.toff[r] = t;
    t += fa_tiles(a.n[r]);
    a.pv[r] = make_pkview(m, (uint32_t)r);
  }
  a.toff[6] = t;
  if (t == 0) return PLUSS_OK;
  FaithfulBufs& b = ctx->fb;
  if (int rc = fa_reserve(b, t, s)) return rc;
  const GTable& g = ctx->g;
  // N, T, CS, CLS/DS powers of two: shift decoding (the scan's word decode
  // also keeps q*N + c1 < N*N/T in 32 bits)
  const bool p2 = m.p2 && a.pv[0].p2 && (uint64_t)m.N * m.N / m.T < (1ull << 32);
  // samples / generated lists: the first pass writes the packed sort words
  // (4 or 8 bytes, as the radix path sorts them) and the scan reads those
  const bool w32 = pk_bits(m) <= 32;
  FaRefs aw = a;
  if (src == SRC_SAMPLES || src == SRC_GEN) {
    const size_t need = t * (size_t)TILE * (w32 ? 4 : 8);
    if (need > b.words_bytes) {
      PLUSS_HIP_CHECK(hipStreamSynchronize(s));
      if (b.words) (void)hipFree(b.words);
      b.words = nullptr;
      b.words_bytes = 0;
      if (hipMalloc(&b.words, need) != hipSuccess) {
        set_error("hipMalloc failed for the faithful scan's word buffer");
        return PLUSS_ERR_ALLOC;
      }
      b.words_bytes = need;
    }
    for (int r = 0; r < 6; ++r)
      aw.src[r] = static_cast<char*>(b.words) + a.toff[r] * (uint64_t)TILE * (w32 ? 4 : 8);
  }
#define PLUSS_FA3(SRCV, CHK, P2V, WKV, SCANV)                                                                      \
  do {                                                                                                             \
    if constexpr (SRCV == SRC_GEN)                                                                                 \
      hipLaunchKernelGGL((k_fa_max_gen<P2V, WKV>), dim3((unsigned)t), dim3(TB), 0, s, m, a, b.tmax, b.words, b.fslot, g);   \
    else                                                                                                           \
      hipLaunchKernelGGL((k_fa_max<SRCV, CHK, P2V, WKV>), dim3((unsigned)t), dim3(TB), 0, s, m, a, b.tmax, b.words, \
                         b.fslot, g);                                                                                       \
    hipLaunchKernelGGL(k_fa_prefix, dim3(6), dim3(PB), 0, s, a, b.tmax, b.pmin);                                   \
    hipLaunchKernelGGL((k_fa_scan<SCANV, P2V>), dim3((unsigned)t), dim3(TB), 0, s, m, aw, b.pmin, b.dpart, g);    \
    hipLaunchKernelGGL((k_fa_finish<SCANV, P2V>), dim3(6), dim3(FT), 0, s, m, aw, b.tmax, b.pmin, b.dpart, b.fslot, \
                       g);    \
  } while (0)
#define PLUSS_FA2(SRCV, CHK, WKV, SCANV)            \
  do {                                              \
    if (p2) PLUSS_FA3(SRCV, CHK, true, WKV, SCANV); \
    else PLUSS_FA3(SRCV, CHK, false, WKV, SCANV);   \
  } while (0)
#define PLUSS_FA(SRCV, CHK)                    \
  do {                                         \
    if (w32) PLUSS_FA2(SRCV, CHK, 4, SRC_W32); \
    else PLUSS_FA2(SRCV, CHK, 8, SRC_W64);     \
  } while (0)
  switch (src) {
    case SRC_W32: PLUSS_FA2(SRC_W32, false, 0, SRC_W32); break;
    case SRC_W64: PLUSS_FA2(SRC_W64, false, 0, SRC_W64); break;
    case SRC_SAMPLES:
      if (check) PLUSS_FA(SRC_SAMPLES, true);
      else PLUSS_FA(SRC_SAMPLES, false);
      break;
    default: PLUSS_FA(SRC_GEN, false); break;
  }
#undef PLUSS_FA
#undef PLUSS_FA2
#undef PLUSS_FA3
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->tables_dirty = true;
  return PLUSS_OK;
}

static FaRefs fa_none() {
  FaRefs a;
  std::memset((void*)&a, 0, sizeof a);
  return a;
}

// the radix-sort pipeline's first half for one sampler_<REF>: packed words
// (or (key, sink) pairs) of its list, sorted into b.keys_s, on stream s
static int faith_keys_sorted(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, const uint64_t* d_samples, uint64_t n,
                             hipStream_t s) {
  if (int rc = faith_keys(ctx, b, ref, d_samples, n, 0, 0, nullptr, s)) return rc;
  return faith_sort(ctx, b, ref, n, s, faith_fm(ctx->m) == FM_PAIRS);
}

// (key, sink) pairs (shapes with N % W != 0): the rocPRIM scans and the record pass
static int faith_pairs_scan(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, uint64_t n, hipStream_t s) {
  const uint64_t nw = 2 * sc_tiles(n);
  hipLaunchKernelGGL(k_faith_scan_init, dim3((unsigned)std::min<uint64_t>((nw + BLOCK - 1) / BLOCK + 1, 64)),
                     dim3(BLOCK), 0, s, b.scal, n, b.st, nw);
  const FlagArgs fa{b.keys_s, b.pmax, 0, 0, make_pkview(ctx->m, (uint32_t)ref)};
  hipLaunchKernelGGL(k_faith_scan<FM_PAIRS>, dim3((unsigned)sc_tiles(n)), dim3(BLOCK), 0, s, fa, b.sinks_s, b.pmax, n,
                     b.st, b.scal);
  PLUSS_HIP_CHECK(hipGetLastError());
  return faith_record(ctx, b, ref, n, 0, 0, 0, n, 1, s);
}

// One sampler_<REF> over a list in any order: keys, radix sort, scan.
int launch_faithful(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, hipStream_t s) {
  if (int rc = faith_check_shape(ctx)) return rc;
  if (n == 0) return PLUSS_OK;
  FaithfulBufs& b = ctx->fb;
  if (int rc = faith_reserve(ctx, b, n, s)) return rc;
  if (int rc = faith_keys_sorted(ctx, b, ref, d_samples, n, s)) return rc;
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PAIRS) return faith_pairs_scan(ctx, b, ref, n, s);
  FaRefs a = fa_none();
  a.n[ref] = n;
  a.src[ref] = b.keys_s;
  return fa_run(ctx, a, fm == FM_PK32 ? SRC_W32 : SRC_W64, false, s);
}

static int faith_direct_shape(const pluss_ctx* ctx, const char* api) {
  if (int rc = faith_check_shape(ctx)) return rc;
  if (!ctx->m.fast) {
    set_error(std::string(api) + ": needs N % (cls/ds) == 0 (packed words); use pluss_dev_faithful_hist");
    return PLUSS_ERR_CONFIG;
  }
  return PLUSS_OK;
}

int launch_faithful_sorted(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, hipStream_t s) {
  if (int rc = faith_direct_shape(ctx, "pluss_dev_faithful_hist_sorted")) return rc;
  FaRefs a = fa_none();
  a.n[ref] = n;
  a.src[ref] = d_samples;
  return fa_run(ctx, a, SRC_SAMPLES, true, s);
}

// All six sampler_<REF> of one list in any order: each reference's keys and
// radix sort on a stream of its own, forked from s and joined back into it
// (r10's main runs one thread per reference, r10:3203-3257); then one scan
// pipeline for the six sorted arrays.
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
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PAIRS) {  // the pair path scans per reference on its stream
    return fork_refs(ctx, counts, s, [&](int r, FaithfulBufs& b, hipStream_t rs) {
      if (int rc = faith_keys_sorted(ctx, b, r, d_samples + off[r], counts[r], rs)) return rc;
      return faith_pairs_scan(ctx, b, r, counts[r], rs);
    });
  }
  uint64_t tiles = 0;
  for (int r = 0; r < 6; ++r) tiles += fa_tiles(counts[r]);
  if (int rc = fa_reserve(ctx->fb, tiles, s)) return rc;
  if (int rc = fork_refs(ctx, counts, s, [&](int r, FaithfulBufs& b, hipStream_t rs) {
        return faith_keys_sorted(ctx, b, r, d_samples + off[r], counts[r], rs);
      }))
    return rc;
  FaRefs a = fa_none();
  for (int r = 0; r < 6; ++r) {
    a.n[r] = counts[r];
    a.src[r] = ctx->fbr[r].keys_s;
  }
  return fa_run(ctx, a, fm == FM_PK32 ? SRC_W32 : SRC_W64, false, s);
}

// All six over a key-ordered list (each reference's block in key order).
int launch_faithful_sorted_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t* counts, hipStream_t s) {
  if (int rc = faith_direct_shape(ctx, "pluss_dev_faithful_hist_sorted_refs")) return rc;
  FaRefs a = fa_none();
  uint64_t off = 0;
  for (int r = 0; r < 6; ++r) {
    a.n[r] = counts[r];
    a.src[r] = d_samples ? d_samples + off : nullptr;
    off += counts[r];
  }
  if (off && !d_samples) {
    set_error("pluss_dev_faithful_hist_sorted_refs: null sample list");
    return PLUSS_ERR_CONFIG;
  }
  return fa_run(ctx, a, SRC_SAMPLES, true, s);
}

// All six over generated key-order lists (pluss_expand_sorted's lists of
// totals[r] samples, never written to memory).
int launch_gen_faithful_refs(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, hipStream_t s) {
  if (int rc = faith_direct_shape(ctx, "pluss_dev_gen_faithful_refs")) return rc;
  FaRefs a = fa_none();
  for (int r = 0; r < 6; ++r) {
    if (!totals[r]) continue;
    if (int rc = keygen_check(ctx, r, totals[r], 0, totals[r], "pluss_dev_gen_faithful_refs")) return rc;
    a.n[r] = totals[r];
    a.kg[r] = keygen_of(ctx, seed, r, totals[r]);
  }
  return fa_run(ctx, a, SRC_GEN, false, s);
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
