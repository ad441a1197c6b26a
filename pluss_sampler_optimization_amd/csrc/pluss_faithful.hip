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

#include <cstdio>

#include <algorithm>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "pluss_faithful.h"
#include "pluss_sort.h"

namespace pluss {
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

// scratch of the (key, sink) pair sort (shapes with N % (cls/ds) != 0; packed
// words are sorted by the bucket sort below): the (digit, block) histogram and
// its scan's block sums, in the sort scratch b.sbuf
static uint64_t pair_blocks(uint64_t n) { return (n + PTILE - 1) / PTILE; }
static size_t pair_hist_bytes(uint64_t n) { return ((size_t)256 * pair_blocks(n) * 4 + 255) & ~(size_t)255; }
static int srt_reserve(FaithfulBufs& b, uint64_t bytes, hipStream_t s);
static int faith_tmp(pluss_ctx* ctx, FaithfulBufs& b, uint64_t n, hipStream_t s) {
  (void)ctx;
  const uint64_t h = 256 * pair_blocks(n), nbs = (h + SBATCH - 1) / SBATCH;
  return srt_reserve(b, pair_hist_bytes(n) + 4 * nbs + 256, s);
}

// ---- the bucket sort of packed words (pluss_sort.h): the references' words,
// made from their samples (SMP: in[r] = the samples) or already made (in[r] =
// words), sorted into out (the references concatenated in order).  x1: 8 B x
// total scratch words; y: another 8 B x total when payloads are 8 bytes.
static int srt_reserve(FaithfulBufs& b, uint64_t bytes, hipStream_t s) {
  if (bytes > b.sbcap) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    if (int rc = grow(&b.sbuf, bytes)) return rc;
    b.sbcap = bytes;
  }
  return PLUSS_OK;
}

struct SrtPlan {
  SrtRefs a;
  uint64_t ntot, h1, g2max, h2max, nbs;
  bool p32;  // 4-byte payloads
  size_t o_h1, o_h2, o_bs, o_par, o_cmap, o_tot, o_deep, o_fast, bytes;
  bool fast1;     // level 1 without its count pass (k_srt_scatter1f; 4-byte payloads)
  uint64_t wmax;  // the words' range [0, wmax): 4 N^3
};

static SrtPlan srt_plan(const Model& m, const void* const in[6], const uint64_t cnt[6]) {
  SrtPlan P;
  std::memset((void*)&P, 0, sizeof P);
  const uint32_t wb = pk_bits(m);
  P.p32 = wb <= 32 + (uint32_t)SDIG;
  uint64_t e = 0, c = 0, h = 0, np = 0;
  for (int r = 0; r < 6; ++r) {
    uint32_t d1 = srt_d1(cnt[r], wb);
    if (cnt[r] && P.p32 && wb > 32 && d1 < wb - 32) d1 = wb - 32;  // every payload below 2^32
    const uint64_t nch = (cnt[r] + SC - 1) / SC;
    P.a.n[r] = cnt[r];
    P.a.eoff[r] = e;
    P.a.coff[r] = c;
    P.a.hoff[r] = h;
    P.a.d1[r] = d1;
    P.a.in[r] = in[r];
    e += cnt[r];
    c += nch;
    h += ((uint64_t)1 << d1) * nch;
    np += (uint64_t)1 << d1;
  }
  P.a.eoff[6] = e;
  P.a.coff[6] = c;
  P.a.hoff[6] = h;
  P.a.wb = wb;
  P.a.np = (uint32_t)np;
  P.a.tsh = 0;
  while ((1u << P.a.tsh) < m.T) ++P.a.tsh;
  P.ntot = e;
  P.h1 = h;
  P.g2max = e / SC + np + 1;
  P.h2max = P.g2max * SB;
  P.nbs = ((h > P.h2max ? h : P.h2max) + SBATCH - 1) / SBATCH;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  P.o_h1 = o;
  o = al(o + 4 * P.h1);
  P.o_h2 = o;
  o = al(o + 4 * P.h2max);
  P.o_bs = o;
  o = al(o + 4 * P.nbs);
  P.o_par = o;
  o = al(o + sizeof(SrtParent) * np);
  P.o_cmap = o;
  o = al(o + 4 * P.g2max);
  P.o_tot = o;  // [0] level-2 chunks, [1] hist2 entries, [2] deep items
  o = al(o + 16);
  P.o_deep = o;
  o = al(o + sizeof(SrtItem) * np * SB);
  P.o_fast = o;  // cap, off1, fill (np each), ovf, gate, glen, level 2's ovf, gate, glen, then its fills (np * 256)
  o = al(o + 4 * (3 * (size_t)np + 8 + (size_t)np * SB));
  P.bytes = o;
  // the count-free level 1: 4-byte payloads, and no reference whose top digit
  // decides every bit (its whole-bucket items would be read and written at
  // different places; such shapes are tiny)
  P.wmax = 4ull * (uint64_t)m.N * (uint64_t)m.N * (uint64_t)m.N;
  P.fast1 = P.p32;
  for (int r = 0; r < 6; ++r)
    if (cnt[r] && wb <= P.a.d1[r]) P.fast1 = false;
  // the count-free levels size X1 and Y as 2 payloads per sample and sum their
  // regions' capacities in 32 bits: past 2^31 samples the counted levels
  if (e > ((uint64_t)1 << 31)) P.fast1 = false;
  return P;
}

// exclusive scan of v[0, len) in place (dlen: the entries in use, on the device)
static void srt_scan(uint32_t* v, uint64_t len, const uint32_t* dlen, uint32_t* bsum, hipStream_t s) {
  const uint32_t nb = (uint32_t)((len + SBATCH - 1) / SBATCH);
  if (!nb) return;
  hipLaunchKernelGGL(k_scan_sums, dim3(nb), dim3(SB), 0, s, (const uint32_t*)v, len, dlen, bsum);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SB), 0, s, bsum, nb);
  hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(SB), 0, s, v, len, dlen, (const uint32_t*)bsum);
}

// OT: the output's type -- KT (the words) or, for 4-byte payloads of longer
// words, uint32_t (the payloads alone; SRC_W32P puts the digits back)
template <typename KT, typename PT, bool SMP, typename OT = KT>
static int srt_launch(pluss_ctx* ctx, FaithfulBufs& b, const SrtPlan& P, PT* X1, PT* Y, OT* out, hipStream_t s) {
  constexpr bool PFX = std::is_same<OT, KT>::value;
  const Model& m = ctx->m;
  unsigned char* B = b.sbuf;
  uint32_t* h1 = (uint32_t*)(B + P.o_h1);
  uint32_t* h2 = (uint32_t*)(B + P.o_h2);
  uint32_t* bs = (uint32_t*)(B + P.o_bs);
  SrtParent* par = (SrtParent*)(B + P.o_par);
  uint32_t* cmap = (uint32_t*)(B + P.o_cmap);
  uint32_t* tot = (uint32_t*)(B + P.o_tot);
  const SrtDeep dp{(SrtItem*)(B + P.o_deep), tot + 2, P.a.np * (uint32_t)SB, ctx->g.flags};
  uint32_t* cap = (uint32_t*)(B + P.o_fast);
  uint32_t* off1 = cap + P.a.np;
  uint32_t* fill = off1 + P.a.np;
  uint32_t* ovf = fill + P.a.np;
  uint32_t* gate = ovf + 1;
  uint32_t* glen = ovf + 2;
  SrtL2 l2{P.wmax, (uint32_t)std::min<uint64_t>(2 * P.ntot, 0xFFFFFFFFull), ovf + 8, ovf + 3, ovf + 4, ovf + 5};
  PLUSS_HIP_CHECK(hipMemsetAsync(tot, 0, 16, s));
  const unsigned g1 = (unsigned)P.a.coff[6];
  const bool p2 = m.p2 && (1u << P.a.tsh) == m.T;  // shift decodes of c0
  const bool fast = P.fast1 && std::is_same<PT, uint32_t>::value;
  if (fast) {
    // level 1 without a count: buckets over-allocated in X1 (the whole 8 B x
    // total scratch, 2 payloads per sample); then the counted level 1, gated
    // on an overflow (its scan over none of hist1 when the gate is shut)
    hipLaunchKernelGGL(k_srt_caps, dim3(1), dim3(SB), 0, s, P.a, P.wmax, (uint32_t)std::min<uint64_t>(2 * P.ntot,
                       0xFFFFFFFFull), cap, off1, fill, ovf);
    if (p2)
      hipLaunchKernelGGL((k_srt_scatter1f<KT, SMP, true>), dim3(g1 * SPL), dim3(SB1), 0, s, m, P.a,
                         (const uint32_t*)cap, (const uint32_t*)off1, fill, ovf, (uint32_t*)X1, ctx->g);
    else
      hipLaunchKernelGGL((k_srt_scatter1f<KT, SMP, false>), dim3(g1 * SPL), dim3(SB1), 0, s, m, P.a,
                         (const uint32_t*)cap, (const uint32_t*)off1, fill, ovf, (uint32_t*)X1, ctx->g);
    hipLaunchKernelGGL(k_srt_gate, dim3(1), dim3(1), 0, s, (const uint32_t*)ovf, (uint32_t)P.h1, gate, glen);
    PLUSS_STAGE(s, "sort: level 1, count-free");
  }
  const uint32_t* gt = fast ? gate : nullptr;
  if (p2)
    hipLaunchKernelGGL((k_srt_count1<KT, SMP, true>), dim3(g1), dim3(SB), 0, s, m, P.a, h1, ctx->g, gt);
  else
    hipLaunchKernelGGL((k_srt_count1<KT, SMP, false>), dim3(g1), dim3(SB), 0, s, m, P.a, h1, ctx->g, gt);
  srt_scan(h1, P.h1, fast ? glen : nullptr, bs, s);
  if (p2)
    hipLaunchKernelGGL((k_srt_scatter1<KT, PT, SMP, true>), dim3(g1), dim3(SB), 0, s, m, P.a, (const uint32_t*)h1, X1,
                       ctx->g, gt);
  else
    hipLaunchKernelGGL((k_srt_scatter1<KT, PT, SMP, false>), dim3(g1), dim3(SB), 0, s, m, P.a, (const uint32_t*)h1,
                       X1, ctx->g, gt);
  PLUSS_STAGE(s, "sort: level 1, counted");
  if (!fast) l2.fill = nullptr;  // (the counted level 2, ungated)
  hipLaunchKernelGGL(k_srt_plan, dim3(1), dim3(SB), 0, s, P.a, (const uint32_t*)h1, par, cmap, tot,
                     fast ? (const uint32_t*)fill : nullptr, (const uint32_t*)off1, (const uint32_t*)ovf, l2);
  PLUSS_STAGE(s, "sort: plan");
  if (fast) {  // level 2 without a count (unless level 1 overflowed), then the counted one gated on an overflow
    hipLaunchKernelGGL(k_srt_scatter2f<PT>, dim3((unsigned)P.g2max * SPL), dim3(SB1), 0, s, P.a,
                       (const SrtParent*)par, (const uint32_t*)cmap, (const uint32_t*)tot, (const PT*)X1, Y, l2);
    hipLaunchKernelGGL(k_srt_gate2, dim3(1), dim3(1), 0, s, (const uint32_t*)l2.ovf, (const uint32_t*)(tot + 1),
                       l2.gate, l2.glen);
  }
  PLUSS_STAGE(s, "sort: level 2, count-free");
  const uint32_t* gt2 = fast ? (const uint32_t*)l2.gate : nullptr;
  hipLaunchKernelGGL(k_srt_count2<PT>, dim3((unsigned)P.g2max), dim3(SB), 0, s, P.a, (const SrtParent*)par,
                     (const uint32_t*)cmap, (const uint32_t*)tot, (const PT*)X1, h2, gt2);
  srt_scan(h2, P.h2max, fast ? (const uint32_t*)l2.glen : tot + 1, bs, s);
  hipLaunchKernelGGL(k_srt_scatter2<PT>, dim3((unsigned)P.g2max), dim3(SB), 0, s, P.a, (const SrtParent*)par,
                     (const uint32_t*)cmap, (const uint32_t*)tot, (const uint32_t*)h2, (const PT*)X1, Y, gt2);
  PLUSS_STAGE(s, "sort: level 2, counted");
  hipLaunchKernelGGL((k_srt_final<PT, OT, PFX>), dim3(FG, P.a.np), dim3(SB), 0, s, P.a, (const SrtParent*)par,
                     (const uint32_t*)h2, (const PT*)X1, (const PT*)Y, out, dp, l2);
  PLUSS_STAGE(s, "sort: final");
  hipLaunchKernelGGL((k_srt_deep<PT, OT, PFX>), dim3(64), dim3(SB), 0, s, P.a, (const SrtParent*)par, X1, Y, out, dp);
  PLUSS_STAGE(s, "sort: deep");
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

// The sort of one or more references (cnt[r] = 0: none).  x1 (and y, for
// 8-byte payloads) hold 8 B x total each; neither may alias in[] or out.
// pay: when the payloads are 4 bytes and the words longer, out receives the
// payloads alone (uint32_t) and *pay_out the parents' table for SRC_W32P
// (false: out holds KT words).
struct SrtPay {
  bool on;
  const SrtParent* par;
  uint32_t pb[6], pn[6], hi[6];
  uint64_t eoff[6];
};
template <typename KT, bool SMP>
// narrow: the words are one key range's of the lists (a key-range shard's),
// so they fill a fraction of the word range: the count-free level 1 sizes its
// buckets for the whole range and would overflow, so the counted levels run
static int srt_sort(pluss_ctx* ctx, FaithfulBufs& b, const void* const in[6], const uint64_t cnt[6],
                    unsigned long long* x1, unsigned long long* y, KT* out, hipStream_t s, SrtPay* pay = nullptr,
                    bool narrow = false) {
  SrtPlan P = srt_plan(ctx->m, in, cnt);
  if (narrow) P.fast1 = false;
  if (!SMP && PLUSS_KNOB("WORDS_COUNTED")) P.fast1 = false;  // (diagnostic build only)
  if (pay) {  // (the parents' address once srt_reserve below has grown the scratch)
    pay->on = P.p32 && sizeof(KT) > 4;
    pay->par = nullptr;
    uint32_t pb = 0;
    const PkView v0 = make_pkview(ctx->m, 0);
    for (int r = 0; r < 6; ++r) {
      pay->pb[r] = pb;
      pay->pn[r] = 1u << P.a.d1[r];
      pay->hi[r] = P.a.wb - P.a.d1[r];
      pay->eoff[r] = P.a.eoff[r];
      pb += 1u << P.a.d1[r];
      // the lane-major decode puts the digit into the q*N + c1 field (fa_dec_w32p)
      if (cnt[r] && pay->hi[r] < 2 + v0.tsh + v0.nsh) pay->on = false;
    }
  }
  if (P.ntot == 0) return PLUSS_OK;
  if (P.ntot > 0xFFFFFFFFull) {
    set_error("faithful mode: the radix source sorts at most 2^32-1 samples per call");
    return PLUSS_ERR_CONFIG;
  }
  if (int rc = srt_reserve(b, P.bytes, s)) return rc;
  if (pay) pay->par = (const SrtParent*)(b.sbuf + P.o_par);
  if (P.p32) {
    uint32_t* X1 = reinterpret_cast<uint32_t*>(x1);
    // (the count-free level 1 spreads X1 over all of x1: Y then lives in y)
    uint32_t* Y = P.fast1 ? reinterpret_cast<uint32_t*>(y) : X1 + P.ntot;
    if (pay && pay->on) return srt_launch<KT, uint32_t, SMP, uint32_t>(ctx, b, P, X1, Y, (uint32_t*)(void*)out, s);
    return srt_launch<KT, uint32_t, SMP>(ctx, b, P, X1, Y, out, s);
  }
  return srt_launch<KT, unsigned long long, SMP>(ctx, b, P, x1, y, out, s);
}

// one reference's words, from its samples (SMP: d_in) or from the words in b.keys
template <typename KT, bool SMP>
static int srt_run(pluss_ctx* ctx, FaithfulBufs& b, int32_t ref, const void* d_in, uint64_t n, hipStream_t s) {
  const void* in[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  uint64_t cnt[6] = {0, 0, 0, 0, 0, 0};
  in[ref] = d_in;
  cnt[ref] = n;
  // scratch: the sample path writes b.keys / b.sinks; the word path reads b.keys, so its scratch is b.sinks_s / b.pmax
  return srt_sort<KT, SMP>(ctx, b, in, cnt, SMP ? b.keys : b.sinks_s, SMP ? b.sinks : b.pmax,
                           reinterpret_cast<KT*>(b.keys_s), s);
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

// sort n (key, sink) pairs by key: b.keys / b.sinks -> b.keys_s / b.sinks_s
// (k_faith_scan takes the prefix max of sinks); the LSD pair sort of
// pluss_sort.h over the keys' significant bits, ping-ponging between the two
// buffer pairs
static int faith_sort(pluss_ctx* ctx, FaithfulBufs& b, uint64_t n, hipStream_t s) {
  if (n == 0) return PLUSS_OK;
  if (int rc = faith_tmp(ctx, b, n, s)) return rc;
  const uint32_t nblk = (uint32_t)pair_blocks(n), passes = (key_bits(ctx->m) + 7) / 8;
  uint32_t* hist = (uint32_t*)b.sbuf;
  uint32_t* bsum = (uint32_t*)(b.sbuf + pair_hist_bytes(n));
  unsigned long long *ki = b.keys, *vi = b.sinks, *ko = b.keys_s, *vo = b.sinks_s;
  if (passes % 2 == 0) {  // (an even number of passes ends where it began: start from the other pair)
    PLUSS_HIP_CHECK(hipMemcpyAsync(b.keys_s, b.keys, n * 8, hipMemcpyDeviceToDevice, s));
    PLUSS_HIP_CHECK(hipMemcpyAsync(b.sinks_s, b.sinks, n * 8, hipMemcpyDeviceToDevice, s));
    std::swap(ki, ko);
    std::swap(vi, vo);
  }
  for (uint32_t p = 0; p < passes; ++p) {
    hipLaunchKernelGGL(k_pair_count, dim3(nblk), dim3(PB), 0, s, (const unsigned long long*)ki, n, 8 * p, hist, nblk);
    srt_scan(hist, (uint64_t)256 * nblk, nullptr, bsum, s);
    hipLaunchKernelGGL(k_pair_scatter, dim3(nblk), dim3(PB), 0, s, (const unsigned long long*)ki,
                       (const unsigned long long*)vi, n, 8 * p, (const uint32_t*)hist, nblk, ko, vo);
    std::swap(ki, ko);
    std::swap(vi, vo);
  }
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
static int fa_reserve(FaithfulBufs& b, uint64_t tiles, uint64_t chunks, hipStream_t s) {
  if (!b.fslot) {
    if (int rc = grow(&b.fslot, 8)) return rc;
  }
  if (tiles > b.dcap) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    int rc = 0;
    if ((rc = grow(&b.dpart, tiles * FPW)) || (rc = grow(&b.tmax, tiles)) || (rc = grow(&b.pmin, tiles)) ||
        (rc = grow(&b.klist, tiles * 2 * KL)) || (rc = grow(&b.slowq, tiles + 1)))
      return rc;
    PLUSS_HIP_CHECK(hipMemsetAsync(b.slowq, 0, 4, s));  // k_fa_chunk empties it after every pass
    b.dcap = tiles;
  }
  if (chunks > b.ccap) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    int rc = 0;
    if ((rc = grow(&b.cval, chunks)) || (rc = grow(&b.crec, chunks * CW)) || (rc = grow(&b.cflag, chunks))) return rc;
    PLUSS_HIP_CHECK(hipMemsetAsync(b.cflag, 0, chunks * sizeof(unsigned int), s));
    b.epoch = 0;
    b.ccap = chunks;
  }
  return PLUSS_OK;
}

// Tile and chunk offsets, buffers and the launch description of one pass
// over `a` (a.n set; one GPU: the whole lists, ntot = n; a key-range shard:
// joff, ntot set by the caller).  *L.t == 0: nothing to do.
static int fa_prepare(pluss_ctx* ctx, FaRefs& a, int src, bool check, bool shard, hipStream_t s, FaLaunch* out) {
  const Model& m = ctx->m;
  uint64_t t = 0;
  for (int r = 0; r < 6; ++r) {
    if (a.n[r] > 0xFFFFFFFFull) {
      set_error("faithful mode: at most 2^32-1 samples per reference");
      return PLUSS_ERR_CONFIG;
    }
    if (!shard) {
      a.ntot[r] = a.n[r];
      a.joff[r] = 0;
    }
    a.toff[r] = t;
    t += fa_tiles(a.n[r]);
    a.pv[r] = make_pkview(m, (uint32_t)r);
  }
  a.toff[6] = t;
  uint64_t c = 0;
  for (int r = 0; r < 6; ++r) {
    a.coff[r] = c;
    c += fa_chunks(a.toff[r + 1] - a.toff[r]);
  }
  a.coff[6] = c;
  if (src == SRC_SAMPLES && !check) {
    set_error("faithful mode: a caller's list is always order-checked");
    return PLUSS_ERR_CONFIG;
  }
  FaithfulBufs& b = ctx->fb;
  if (shard && !b.xin) {
    if (int rc = grow(&b.xin, XIN_W + 8)) return rc;
  }
  a.xin = shard ? b.xin : nullptr;
  // N, T, CS, CLS/DS powers of two: shift decoding (the word decode also
  // keeps q*N + c1 < N*N/T in 32 bits)
  const bool p2 = m.p2 && a.pv[0].p2 && (uint64_t)m.N * m.N / m.T < (1ull << 32);
  // the local pass's fast path: 24-bit multiplies (q*N + c1 < N*N/T and S
  // below 2^24) and the range check by bit masks (N a power of two)
  a.fast = (p2 && m.np2 && (uint64_t)m.N * m.N / m.T < (1ull << 24) && m.S < (1u << 24)) ? 1u : 0u;
  // the uniform source's staged elements carry whole keys (below 2^61) and a
  // leaf's keys as 32-bit increments (a row of a 2-D reference spans N*S*T keys)
  a.unidec = ((unsigned __int128)m.A * m.T < ((unsigned __int128)1 << 61) &&
              (uint64_t)m.N * m.S * m.T < (1ull << 32)) ? 1u : 0u;
  *out = FaLaunch{m, a, ctx->g, &b, p2, t, 0, FA_PH_ALL, s, nullptr};
  if (t == 0) return PLUSS_OK;
  // the uniform source's 2-D references, whose tiles span more than 2^32 keys
  // when the lists are sparse in them (C0 / C1 at every BASELINE shape): every
  // such tile left the lane-major pass for the queued one, which regenerated
  // it after the lane-major pass, ~0.1 ms at config 3 (r6r).  They run on a
  // second stream beside it instead (FaLaunch::side).
  if (src == SRC_UNI && a.fast && a.unidec && a.toff[2] > 0 && a.toff[2] < t) {
    bool sparse = false;
    for (int r = 0; r < 2; ++r)
      sparse |= a.n[r] > 0 && (unsigned __int128)m.A * m.T * TILE > ((unsigned __int128)a.ntot[r] << 32);
    if (sparse && !b.side && !b.capture) {  // (made on an eager pass: a capture only reuses them)
      if (hipStreamCreateWithFlags(&b.side, hipStreamNonBlocking) != hipSuccess) b.side = nullptr;
      for (hipEvent_t& e : b.sev)
        if (b.side && !e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    }
    // (eager passes only: with the side stream inside a group's captured
    // pass, the bench's config-3 group legs crashed on the host, r6ah-r6ak)
    if (sparse && b.side && b.sev[0] && b.sev[1] && (!b.capture || PLUSS_KNOB("SIDE_CAPTURE")))
      out->side = (uint32_t)a.toff[2];  // (the knob: diagnostic build only, the crash's reproduction)
  }
  if (int rc = fa_reserve(b, t, c, s)) return rc;
  if (!b.shrec) {
    if (int rc = grow(&b.shrec, 6 * SRW + 16)) return rc;
  }
  if (++b.epoch == 0) ++b.epoch;  // (0: never published)
  out->epoch = b.epoch;
  return PLUSS_OK;
}

static int fa_launch(pluss_ctx* ctx, const FaLaunch& L, int src, int phase) {
  FaLaunch l = L;
  l.phase = phase;
  switch (src) {
    case SRC_W32: fa_launch_w32(l); break;
    case SRC_W64: fa_launch_w64(l); break;
    case SRC_W32P: fa_launch_w32p(l); break;
    case SRC_SAMPLES: fa_launch_smp(l); break;
    case SRC_UNI: fa_launch_uni(l); break;
    default: fa_launch_gen(l); break;
  }
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->tables_dirty = true;
  return PLUSS_OK;
}

static int fa_run(pluss_ctx* ctx, FaRefs& a, int src, bool check, hipStream_t s) {
  FaLaunch L;
  if (int rc = fa_prepare(ctx, a, src, check, false, s, &L)) return rc;
  if (L.t == 0) return PLUSS_OK;
  return fa_launch(ctx, L, src, FA_PH_ALL);
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
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PK32) return srt_run<uint32_t, true>(ctx, b, ref, d_samples, n, s);
  if (fm == FM_PK64) return srt_run<unsigned long long, true>(ctx, b, ref, d_samples, n, s);
  if (int rc = faith_keys(ctx, b, ref, d_samples, n, 0, 0, nullptr, s)) return rc;
  return faith_sort(ctx, b, n, s);
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
  faith_shards_abandon(ctx);  // these share the handle's faithful buffers
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
  faith_shards_abandon(ctx);  // these share the handle's faithful buffers
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
  faith_shards_abandon(ctx);  // these share the handle's faithful buffers
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
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PAIRS) {  // (key, sink) pairs: per reference on a stream of its own
    for (int r = 0; r < 6; ++r) {  // every allocation before the fork
      if (!counts[r]) continue;
      if (int rc = faith_reserve(ctx, ctx->fbr[r], counts[r], s)) return rc;
      if (int rc = faith_tmp(ctx, ctx->fbr[r], counts[r], s)) return rc;
    }
    return fork_refs(ctx, counts, s, [&](int r, FaithfulBufs& b, hipStream_t rs) {
      if (int rc = faith_keys_sorted(ctx, b, r, d_samples + off[r], counts[r], rs)) return rc;
      return faith_pairs_scan(ctx, b, r, counts[r], rs);
    });
  }
  // packed words: one bucket sort of the six references (full-chip grids),
  // then one scan pipeline over the six sorted arrays
  FaithfulBufs& b = ctx->fb;
  if (int rc = faith_reserve(ctx, b, total, s)) return rc;
  const void* in[6];
  for (int r = 0; r < 6; ++r) in[r] = d_samples + off[r];
  FaRefs a = fa_none();
  if (fm == FM_PK32) {
    if (int rc = srt_sort<uint32_t, true>(ctx, b, in, counts, b.keys, b.sinks, (uint32_t*)b.keys_s, s)) return rc;
    for (int r = 0; r < 6; ++r) a.src[r] = (const uint32_t*)b.keys_s + off[r];
  } else {
    SrtPay pay{};
    if (int rc = srt_sort<unsigned long long, true>(ctx, b, in, counts, b.keys, b.sinks, b.keys_s, s, &pay)) return rc;
    if (pay.on) {  // 4-byte payloads read back with their parents' digits (SRC_W32P)
      for (int r = 0; r < 6; ++r) {
        a.src[r] = (const uint32_t*)b.keys_s + off[r];
        a.ppb[r] = pay.pb[r];
        a.ppn[r] = pay.pn[r];
        a.phi[r] = pay.hi[r];
        a.peoff[r] = pay.eoff[r];
      }
      a.ppar = pay.par;
      for (int r = 0; r < 6; ++r) a.n[r] = counts[r];
      return fa_run(ctx, a, SRC_W32P, false, s);
    }
    for (int r = 0; r < 6; ++r) a.src[r] = b.keys_s + off[r];
  }
  for (int r = 0; r < 6; ++r) a.n[r] = counts[r];
  return fa_run(ctx, a, fm == FM_PK32 ? SRC_W32 : SRC_W64, false, s);
}

// diagnostics: the bucket sort alone (include/pluss_diag.h)
int diag_sort_words(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, void* d_words,
                    int32_t* word_bytes, hipStream_t s) {
  faith_shards_abandon(ctx);  // these share the handle's faithful buffers
  if (int rc = faith_direct_shape(ctx, "pluss_diag_sort_words")) return rc;
  FaithfulBufs& b = ctx->fb;
  if (int rc = faith_reserve(ctx, b, n, s)) return rc;
  const int fm = faith_fm(ctx->m);
  *word_bytes = fm == FM_PK32 ? 4 : 8;
  if (n == 0) return PLUSS_OK;
  if (fm == FM_PK32) {
    if (int rc = srt_run<uint32_t, true>(ctx, b, ref, d_samples, n, s)) return rc;
  } else if (int rc = srt_run<unsigned long long, true>(ctx, b, ref, d_samples, n, s)) {
    return rc;
  }
  PLUSS_HIP_CHECK(hipMemcpyAsync(d_words, b.keys_s, n * (size_t)*word_bytes, hipMemcpyDeviceToDevice, s));
  return PLUSS_OK;
}

// All six over a key-ordered list (each reference's block in key order).
int launch_faithful_sorted_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t* counts, hipStream_t s) {
  faith_shards_abandon(ctx);  // these share the handle's faithful buffers
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
  faith_shards_abandon(ctx);  // these share the handle's faithful buffers
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

// ---- key-range shards of the single-read pipeline (multi-GPU faithful mode;
// dist.sharded_faithful_gen_hist): the caller exchanges the per-reference
// summaries between the four phases
// All six over r10's own distribution (uniform draws without replacement,
// r10:156-185) generated in key order inside the pass (pluss_uniform.h): the
// plan, then the pipeline staging each tile from it.
int launch_gen_uniform_faithful_refs(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, hipStream_t s) {
  faith_shards_abandon(ctx);  // these share the handle's faithful buffers
  if (int rc = faith_direct_shape(ctx, "pluss_dev_gen_uniform_faithful_refs")) return rc;
  FaRefs a = fa_none();
  uint64_t any = 0;
  for (int r = 0; r < 6; ++r) {
    a.n[r] = totals[r];
    any += totals[r];
  }
  if (!any) return PLUSS_OK;
  const UniSet* us = nullptr;
  if (int rc = uni_plan(ctx, seed, totals, s, &us)) return rc;
  a.us = us;
  return fa_run(ctx, a, SRC_UNI, false, s);
}

// ---- key-range shards of the single-read pipeline (multi-GPU faithful mode):
// every phase writes this shard's summary row in device memory and the next
// reads the rows of all shards, gathered by the caller (an RCCL all-gather in
// the group driver, pluss_group.hip, or dist.py); k_fa_xchg derives the
// shard's inputs on the device, so no phase waits for the host
__global__ void k_fa_sel_row(const unsigned long long* __restrict__ cnt, unsigned long long* __restrict__ row) {
  const uint32_t w = threadIdx.x;
  if (w < ROW_W) row[w] = w < 6 ? cnt[w] : 0ull;
}

static FaShards& shards_of(pluss_ctx* ctx) {
  if (!ctx->fsh2) ctx->fsh2 = new FaShards();
  return *ctx->fsh2;
}

static int shards_expect(pluss_ctx* ctx, int phase, const char* api, const uint64_t* d_rows, int32_t shard,
                         int32_t nshards) {
  if (!ctx->fsh2 || ctx->fsh2->phase != phase) {
    set_error(std::string(api) + ": out of order (the phases run local, carry, cut, hist on one handle, with no "
                                 "other faithful call in between)");
    return PLUSS_ERR_CONFIG;
  }
  if (!d_rows || nshards < 1 || shard < 0 || shard >= nshards) {
    set_error(std::string(api) + ": needs the gathered rows of all shards and 0 <= shard < nshards");
    return PLUSS_ERR_CONFIG;
  }
  return PLUSS_OK;
}

// phase 1's launches and summary row, whatever the source
static int shards_phase1(pluss_ctx* ctx, FaShards& f, uint64_t* d_row, hipStream_t s) {
  f.L.s = s;
  if (f.L.t)
    if (int rc = fa_launch(ctx, f.L, f.src, FA_PH_LOCAL)) return rc;
  FaithfulBufs& b = ctx->fb;
  hipLaunchKernelGGL(k_fa_shard_sums<0>, dim3(6), dim3(SS_NT), 0, s, f.L.a, b.tmax, b.crec, (unsigned long long*)d_row,
                     0);
  PLUSS_HIP_CHECK(hipGetLastError());
  PLUSS_STAGE(s, "shard phase 1 (local)");
  f.phase = SH_LOCAL;
  f.has_slice = true;
  return PLUSS_OK;
}

int faith_shards_local(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t seed, const uint64_t* totals,
                       const uint64_t* first, const uint64_t* n, uint64_t* d_row, hipStream_t s) {
  FaShards& f = shards_of(ctx);
  f = FaShards{};  // whatever an earlier pass left half finished
  if (int rc = faith_direct_shape(ctx, "pluss_dev_faithful_shards_local")) return rc;
  FaRefs a = fa_none();
  uint64_t off = 0;
  for (int r = 0; r < 6; ++r) {
    a.n[r] = n[r];
    a.ntot[r] = totals[r];
    a.joff[r] = first[r];
    if (first[r] > totals[r] || n[r] > totals[r] - first[r]) {
      set_error("pluss_dev_faithful_shards_local: [first, first + n) exceeds the list");
      return PLUSS_ERR_CONFIG;
    }
    if (d_samples) {
      a.src[r] = d_samples + off;
      off += n[r];
    } else if (n[r]) {
      if (int rc = keygen_check(ctx, r, totals[r], first[r], n[r], "pluss_dev_faithful_shards_local")) return rc;
      a.kg[r] = keygen_of(ctx, seed, r, totals[r]);
    }
  }
  f.src = d_samples ? SRC_SAMPLES : SRC_GEN;
  if (int rc = fa_prepare(ctx, a, f.src, true, true, s, &f.L)) return rc;
  return shards_phase1(ctx, f, d_row, s);
}

// arbitrary-order lists (what r10 hands over): every shard reads the whole
// lists and keeps its key range as packed sort words
int faith_shards_select(pluss_ctx* ctx, const uint64_t* d_lists, const uint64_t* totals, uint64_t key_lo,
                        uint64_t key_hi, uint64_t* d_row, hipStream_t s) {
  FaShards& f = shards_of(ctx);
  f = FaShards{};
  if (int rc = faith_direct_shape(ctx, "pluss_dev_faithful_shards_select")) return rc;
  uint64_t total = 0;
  for (int r = 0; r < 6; ++r) total += totals[r];
  if (total && !d_lists) {
    set_error("pluss_dev_faithful_shards_select: null sample lists");
    return PLUSS_ERR_CONFIG;
  }
  FaithfulBufs& b = ctx->fb;
  if (int rc = faith_reserve(ctx, b, total, s)) return rc;
  if (!b.xin)
    if (int rc = grow(&b.xin, XIN_W + 8)) return rc;
  unsigned long long* cnt = b.xin + XIN_W;
  PLUSS_HIP_CHECK(hipMemsetAsync(cnt, 0, 8 * sizeof(unsigned long long), s));
  const int fm = faith_fm(ctx->m);
  uint64_t off = 0;
  for (int r = 0; r < 6; ++r) {
    f.tot[r] = totals[r];
    if (totals[r]) {
      // reference r's words go to its own region of b.keys (room for its whole list)
      void* out = fm == FM_PK32 ? (void*)((uint32_t*)b.keys + off) : (void*)(b.keys + off);
      if (fm == FM_PK32)
        hipLaunchKernelGGL((k_faith_keys<true, FM_PK32>), dim3(grid_of(totals[r])), dim3(BLOCK), 0, s, ctx->m,
                           (uint32_t)r, d_lists + off, totals[r], key_lo, key_hi, out, (unsigned long long*)nullptr,
                           cnt + r, ctx->g);
      else
        hipLaunchKernelGGL((k_faith_keys<true, FM_PK64>), dim3(grid_of(totals[r])), dim3(BLOCK), 0, s, ctx->m,
                           (uint32_t)r, d_lists + off, totals[r], key_lo, key_hi, out, (unsigned long long*)nullptr,
                           cnt + r, ctx->g);
    }
    off += totals[r];
  }
  hipLaunchKernelGGL(k_fa_sel_row, dim3(1), dim3(ROW_W), 0, s, (const unsigned long long*)cnt,
                     (unsigned long long*)d_row);
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->tables_dirty = true;
  f.phase = SH_SELECTED;
  return PLUSS_OK;
}

// phase 1 of the selected words: the one host round trip of an arbitrary-order
// pass (the launch grids need this shard's counts), then the sort and the local pass
int faith_shards_local_selected(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                uint64_t* d_row, hipStream_t s) {
  if (int rc = shards_expect(ctx, SH_SELECTED, "pluss_dev_faithful_shards_local_selected", d_rows, shard, nshards))
    return rc;
  FaShards& f = *ctx->fsh2;
  std::vector<unsigned long long> rows((size_t)nshards * ROW_W);
  PLUSS_HIP_CHECK(hipMemcpyAsync(rows.data(), d_rows, rows.size() * 8, hipMemcpyDeviceToHost, s));
  PLUSS_HIP_CHECK(hipStreamSynchronize(s));
  FaRefs a = fa_none();
  const void* in[6];
  uint64_t cnt[6], woff = 0, soff = 0;
  const int fm = faith_fm(ctx->m);
  FaithfulBufs& b = ctx->fb;
  for (int r = 0; r < 6; ++r) {
    uint64_t before = 0, all = 0;
    for (int32_t x = 0; x < nshards; ++x) {
      const unsigned long long v = rows[(size_t)x * ROW_W + ROW_N + r];
      all += v;
      if (x < shard) before += v;
    }
    cnt[r] = rows[(size_t)shard * ROW_W + ROW_N + r];
    if (cnt[r] > f.tot[r] || all > f.tot[r]) {  // (a failed shard's row: the pass is reported at the fetch)
      cnt[r] = 0;
      all = before = 0;
    }
    a.n[r] = cnt[r];
    a.ntot[r] = all;
    a.joff[r] = before;
    in[r] = fm == FM_PK32 ? (const void*)((const uint32_t*)b.keys + woff) : (const void*)(b.keys + woff);
    a.src[r] = fm == FM_PK32 ? (const void*)((const uint32_t*)b.keys_s + soff) : (const void*)(b.keys_s + soff);
    woff += f.tot[r];
    soff += cnt[r];
  }
  bool narrow = false;  // (a key range of the lists: the counted sort levels, srt_sort)
  for (int r = 0; r < 6; ++r) narrow |= cnt[r] != f.tot[r];
  if (fm == FM_PK32) {
    if (int rc = srt_sort<uint32_t, false>(ctx, b, in, cnt, b.sinks_s, b.pmax, (uint32_t*)b.keys_s, s, nullptr,
                                           narrow))
      return rc;
  } else if (int rc = srt_sort<unsigned long long, false>(ctx, b, in, cnt, b.sinks_s, b.pmax, b.keys_s, s, nullptr,
                                                          narrow)) {
    return rc;
  }
  f.src = fm == FM_PK32 ? SRC_W32 : SRC_W64;
  if (int rc = fa_prepare(ctx, a, f.src, false, true, s, &f.L)) return rc;
  return shards_phase1(ctx, f, d_row, s);
}

// ---- arbitrary-order lists partitioned on the devices (pluss_group_sampled_hist)
// A device reads its slice of the caller's list once to count, once to place:
// each sample's reference r and key-range shard g (the largest g with
// bounds[g] <= key, a binary search over the S+1 bounds staged in LDS) make
// its bin g*6+r.  Workgroup b takes the contiguous block [n*b/B, n*(b+1)/B).
//   k_fa_part<true>   per block and bin the count -> hist[bin*B + b]
//   k_fa_part_scan    per bin: the total, and hist made the exclusive offsets
//   k_fa_part<false>  each sample's packed word to out[rstart[bin] + hist[bin*B+b]
//                     + its rank in the block] (ranks from wave-aggregated LDS
//                     atomics: the order inside a bin is arbitrary, it is sorted next)
// No global atomics; malformed samples raise the handle's bad-input flag.
constexpr int PT_NT = 256;

__host__ __device__ inline uint32_t part_bins(uint32_t S) { return 6 * S; }

template <bool COUNT, typename KT>
__global__ __launch_bounds__(PT_NT) void k_fa_part(Model m, const uint64_t* __restrict__ smp, uint64_t n,
                                                   const unsigned long long* __restrict__ bounds, uint32_t S,
                                                   uint32_t* __restrict__ hist, uint32_t B,
                                                   const unsigned long long* __restrict__ rstart, KT* __restrict__ out,
                                                   GTable g, uint32_t boff) {
  extern __shared__ unsigned long long pt_lds[];
  unsigned long long* lb = pt_lds;                       // S + 1 bounds
  uint32_t* lc = (uint32_t*)(pt_lds + S + 1);            // per bin: the block's count so far
  unsigned long long* lbase = pt_lds + S + 1 + (part_bins(S) + 1) / 2;  // scatter: per bin its base
  const uint32_t nb = part_bins(S), b = boff + blockIdx.x;
  for (uint32_t i = threadIdx.x; i <= S; i += PT_NT) lb[i] = bounds[i];
  for (uint32_t i = threadIdx.x; i < nb; i += PT_NT) {
    lc[i] = 0;
    if (!COUNT) lbase[i] = rstart[i] + hist[(size_t)i * B + b];
  }
  __syncthreads();
  const uint64_t lo = n * b / B, hi = n * (b + 1) / B;  // (n < 2^40, B <= 16384: no overflow)
  const uint32_t lane = __lane_id();
  for (uint64_t base = lo; base < hi; base += PT_NT) {
    const uint64_t i = base + threadIdx.x;
    uint32_t bin = ~0u;
    KT word = 0;
    if (i < hi) {
      const uint64_t x = smp[i];
      const Sample s = unpack(x);
      if (s.ref > 5 || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N) {
        atomicOr(&g.flags[1], 1u);
      } else {
        const uint32_t c2 = (s.ref == C0 || s.ref == C1) ? 0u : s.c2;
        uint64_t P;
        uint32_t t;
        position(m, s.ref, s.c0, s.c1, c2, &P, &t);
        const unsigned long long key = P * m.T + t;
        uint32_t a = 0, z = S;  // lb[a] <= key < lb[z]
        while (z - a > 1) {
          const uint32_t mid = (a + z) >> 1;
          if (lb[mid] <= key) a = mid;
          else z = mid;
        }
        bin = a * 6 + s.ref;
        if (!COUNT) word = pk_word_of<KT>(m, s.ref, x, g);
      }
    }
    // one LDS atomic per distinct bin of the wave
    unsigned long long pend = __ballot(bin != ~0u);
    while (pend) {
      const int lead = __ffsll((long long)pend) - 1;
      const uint32_t bb = __shfl(bin, lead, 64);
      const unsigned long long mk = __ballot(bin == bb);
      uint32_t at = 0;
      if ((int)lane == lead) at = atomicAdd(&lc[bb], (uint32_t)__popcll(mk));
      if (!COUNT) {
        at = __shfl(at, lead, 64);
        if (bin == bb) {
          const uint64_t o = lbase[bb] + at + __popcll(mk & ((1ull << lane) - 1));
          if (SRT_OK(o < n, 8, o, n)) out[o] = word;
        }
      }
      pend &= ~mk;
    }
  }
  if (COUNT) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += PT_NT) hist[(size_t)i * B + b] = lc[i];
  }
}

// one workgroup per bin: the exclusive scan of its B block counts, the total to tot[bin]
__global__ __launch_bounds__(PT_NT) void k_fa_part_scan(uint32_t* __restrict__ hist, uint32_t B,
                                                        unsigned long long* __restrict__ tot) {
  __shared__ unsigned long long ws[PT_NT / 64];
  uint32_t* h = hist + (size_t)blockIdx.x * B;
  const uint32_t per = (B + PT_NT - 1) / PT_NT, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t i0 = t * per, i1 = min(B, i0 + per);
  unsigned long long mine = 0;
  for (uint32_t i = i0; i < i1; ++i) mine += h[i];
  unsigned long long inc = mine;  // inclusive scan over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long v = __shfl_up(inc, d, 64);
    if ((int)lane >= d) inc += v;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  unsigned long long before = 0, all = 0;
  for (uint32_t x = 0; x < PT_NT / 64; ++x) {
    if (x < w) before += ws[x];
    all += ws[x];
  }
  unsigned long long run = before + inc - mine;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t v = h[i];
    h[i] = (uint32_t)run;
    run += v;
  }
  if (t == 0) tot[blockIdx.x] = all;
}

// copies of word segments {src offset, dst offset, count} (the exchange's
// receive blocks into per-(shard, reference) order): blockIdx.y = segment
template <typename KT>
__global__ __launch_bounds__(PT_NT) void k_fa_seg_copy(const unsigned long long* __restrict__ seg,
                                                       const KT* __restrict__ src, KT* __restrict__ dst) {
  const unsigned long long* q = seg + 3 * (size_t)blockIdx.y;
  const unsigned long long so = q[0], d = q[1], c = q[2];
  for (unsigned long long i = (unsigned long long)blockIdx.x * PT_NT + threadIdx.x; i < c;
       i += (unsigned long long)gridDim.x * PT_NT)
    dst[d + i] = src[so + i];
}

uint32_t faith_part_blocks(uint64_t n, uint32_t S) {
  uint64_t B = n / 16384;  // >= 16K samples per workgroup
  const uint64_t cap = std::max<uint64_t>(1, ((uint64_t)1 << 22) / part_bins(S));  // hist <= 16 MB
  // (up to 16K workgroups: the group counts its slice in 8 upload pieces, and
  // a piece of 2^25 samples over 512 workgroups of 64K ran at 0.8 TB/s, r6ab)
  B = std::min<uint64_t>(std::min<uint64_t>(B, 16384), cap);
  return (uint32_t)std::max<uint64_t>(B, 1);
}

#ifdef PLUSS_DEBUG_STAGES
}  // namespace pluss
extern "C" void pluss_debug_sort_dump(void) {
  unsigned long long h[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(pluss::g_srt_dbg), sizeof h);
  std::fprintf(stderr, "[sort checks] first failure code %llu index %llu bound %llu block %llx thread %llu; failures %llu;"
               " level-1 overflowing runs %llu, level-2 %llu; level-1 workgroups whose waves read different"
               " overflow flags %llu\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]);
}
namespace pluss {
#endif

int faith_word_bytes(const pluss_ctx* ctx) {
  const int fm = faith_fm(ctx->m);
  return fm == FM_PK32 ? 4 : fm == FM_PK64 ? 8 : 0;
}

static size_t part_lds(uint32_t S) { return 8 * ((size_t)S + 1 + (part_bins(S) + 1) / 2 + part_bins(S)); }

int faith_part_count(pluss_ctx* ctx, const uint64_t* d_smp, uint64_t n, const unsigned long long* d_bounds,
                     uint32_t S, uint32_t* d_hist, uint32_t B, unsigned long long* d_tot, hipStream_t s, uint32_t b0,
                     uint32_t b1, bool scan) {
  if (S < 1 || S > 1024 || part_lds(S) > 64 * 1024) {
    set_error("faithful partition: at most 1024 shards");
    return PLUSS_ERR_CONFIG;
  }
  if (b1 > B) b1 = B;
  if (b0 < b1) {
    if (faith_word_bytes(ctx) == 4)
      hipLaunchKernelGGL((k_fa_part<true, uint32_t>), dim3(b1 - b0), dim3(PT_NT), part_lds(S), s, ctx->m, d_smp, n,
                         d_bounds, S, d_hist, B, (const unsigned long long*)nullptr, (uint32_t*)nullptr, ctx->g, b0);
    else
      hipLaunchKernelGGL((k_fa_part<true, unsigned long long>), dim3(b1 - b0), dim3(PT_NT), part_lds(S), s, ctx->m,
                         d_smp, n, d_bounds, S, d_hist, B, (const unsigned long long*)nullptr,
                         (unsigned long long*)nullptr, ctx->g, b0);
  }
  if (scan) hipLaunchKernelGGL(k_fa_part_scan, dim3(part_bins(S)), dim3(PT_NT), 0, s, d_hist, B, d_tot);
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->tables_dirty = true;
  return PLUSS_OK;
}

int faith_part_scatter(pluss_ctx* ctx, const uint64_t* d_smp, uint64_t n, const unsigned long long* d_bounds,
                       uint32_t S, uint32_t* d_hist, uint32_t B, const unsigned long long* d_rstart, void* d_out,
                       hipStream_t s) {
  if (faith_word_bytes(ctx) == 4)
    hipLaunchKernelGGL((k_fa_part<false, uint32_t>), dim3(B), dim3(PT_NT), part_lds(S), s, ctx->m, d_smp, n, d_bounds,
                       S, d_hist, B, d_rstart, (uint32_t*)d_out, ctx->g, 0u);
  else
    hipLaunchKernelGGL((k_fa_part<false, unsigned long long>), dim3(B), dim3(PT_NT), part_lds(S), s, ctx->m, d_smp, n,
                       d_bounds, S, d_hist, B, d_rstart, (unsigned long long*)d_out, ctx->g, 0u);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int faith_seg_copy(const unsigned long long* d_seg, uint32_t nseg, uint64_t maxn, const void* src, void* dst,
                   int wbytes, hipStream_t s) {
  if (!nseg || !maxn) return PLUSS_OK;
  const uint32_t gx = (uint32_t)std::min<uint64_t>((maxn + PT_NT - 1) / PT_NT, 1024);
  if (wbytes == 4)
    hipLaunchKernelGGL(k_fa_seg_copy<uint32_t>, dim3(gx, nseg), dim3(PT_NT), 0, s, d_seg, (const uint32_t*)src,
                       (uint32_t*)dst);
  else
    hipLaunchKernelGGL(k_fa_seg_copy<unsigned long long>, dim3(gx, nseg), dim3(PT_NT), 0, s, d_seg,
                       (const unsigned long long*)src, (unsigned long long*)dst);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

// phase 1 over words already partitioned to this shard (in[r]: cnt[r] words of
// reference r, any order; all[r] and before[r]: the reference's words over all
// shards and over the shards before this one): the sort and the local pass
int faith_shards_local_words(pluss_ctx* ctx, const void* const in[6], const uint64_t* cnt, const uint64_t* all,
                             const uint64_t* before, uint64_t* d_row, hipStream_t s) {
  FaShards& f = shards_of(ctx);
  f = FaShards{};
  if (int rc = faith_direct_shape(ctx, "pluss_group_sampled_hist")) return rc;
  const int fm = faith_fm(ctx->m);
  if (fm == FM_PAIRS) {
    set_error("pluss_group_sampled_hist: packed words need N % (cls/ds) == 0");
    return PLUSS_ERR_CONFIG;
  }
  FaithfulBufs& b = ctx->fb;
  uint64_t tot = 0;
  for (int r = 0; r < 6; ++r) tot += cnt[r];
  if (int rc = faith_reserve(ctx, b, tot, s)) return rc;
  FaRefs a = fa_none();
  uint64_t soff = 0;
  for (int r = 0; r < 6; ++r) {
    f.tot[r] = all[r];
    a.n[r] = cnt[r];
    a.ntot[r] = all[r];
    a.joff[r] = before[r];
    a.src[r] = fm == FM_PK32 ? (const void*)((const uint32_t*)b.keys_s + soff) : (const void*)(b.keys_s + soff);
    soff += cnt[r];
  }
  // the same sort as one GPU's radix pass (4-byte payloads read back with
  // their parents' digits past N = 1024); the count-free levels only when the
  // shard holds whole lists (one shard), else the counted ones
  SrtPay pay{};
  bool narrow = false;
  for (int r = 0; r < 6; ++r) narrow |= cnt[r] != all[r];
  if (fm == FM_PK32) {
    if (int rc = srt_sort<uint32_t, false>(ctx, b, in, cnt, b.sinks_s, b.pmax, (uint32_t*)b.keys_s, s, nullptr,
                                           narrow))
      return rc;
  } else if (int rc = srt_sort<unsigned long long, false>(ctx, b, in, cnt, b.sinks_s, b.pmax, b.keys_s, s,
                                                          PLUSS_KNOB("WORDS_W64") ? nullptr : &pay, narrow)) {
    return rc;
  }
  ctx->tables_dirty = true;
  f.src = fm == FM_PK32 ? SRC_W32 : SRC_W64;
  if (pay.on) {
    f.src = SRC_W32P;
    soff = 0;
    for (int r = 0; r < 6; ++r) {
      a.src[r] = (const uint32_t*)b.keys_s + soff;
      soff += cnt[r];
      a.ppb[r] = pay.pb[r];
      a.ppn[r] = pay.pn[r];
      a.phi[r] = pay.hi[r];
      a.peoff[r] = pay.eoff[r];
    }
    a.ppar = pay.par;
  }
  if (int rc = fa_prepare(ctx, a, f.src, false, true, s, &f.L)) return rc;
  return shards_phase1(ctx, f, d_row, s);
}

// r10's own law (pluss_uniform.h) over key-range shards: shard g of G holds,
// per reference, the leaves [L*g/G, L*(g+1)/G) of the key-ordered space (L
// leaves), so its samples are a contiguous stretch of the list in key order.
// Phase 0 counts this shard's candidates (row[ROW_N + r]); after the gather
// every shard knows the candidates before it and in all (X0, T'), removes the
// ranks of its window, and so its slice of the list: [first, first + n) --
// read back once (the launch grids need n), then the local pass over the tiles
// of that slice, each generated from the shard's plan.
__global__ void k_ug_row(const UniSet* __restrict__ us, unsigned long long* __restrict__ row) {
  const uint32_t w = threadIdx.x;
  if (w >= ROW_W) return;
  unsigned long long v = 0;
  if (w >= ROW_N && w < ROW_N + 6) {
    const uint32_t r = w - ROW_N;
    v = us->pre[us->loff[r + 1]] - us->pre[us->loff[r]];
  }
  row[w] = v;
}

int faith_shards_uniform_count(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, int32_t shard, int32_t nshards,
                               uint64_t* d_row, hipStream_t s) {
  FaShards& f = shards_of(ctx);
  f = FaShards{};
  if (int rc = faith_direct_shape(ctx, "pluss_dev_faithful_shards_uniform_count")) return rc;
  if (nshards < 1 || shard < 0 || shard >= nshards) {
    set_error("pluss_dev_faithful_shards_uniform_count: needs 0 <= shard < nshards");
    return PLUSS_ERR_CONFIG;
  }
  for (int r = 0; r < 6; ++r) f.tot[r] = totals[r];
  if (int rc = uni_plan_count(ctx, seed, totals, (uint32_t)shard, (uint32_t)nshards, s)) return rc;
  hipLaunchKernelGGL(k_ug_row, dim3(1), dim3(ROW_W), 0, s, (const UniSet*)ctx->ub.set, (unsigned long long*)d_row);
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->tables_dirty = true;
  f.shard = shard;
  f.nshards = nshards;
  f.phase = SH_UCOUNT;
  return PLUSS_OK;
}

// the removal over this shard's candidate window, and this shard's slice copied
// to the host (asynchronously: a caller driving several shards issues every
// shard's window before waiting on any)
int faith_shards_uniform_window(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                hipStream_t s, bool to_host) {
  if (int rc = shards_expect(ctx, SH_UCOUNT, "pluss_dev_faithful_shards_uniform_local", d_rows, shard, nshards))
    return rc;
  FaShards& f = *ctx->fsh2;
  if (shard != f.shard || nshards != f.nshards) {
    set_error("pluss_dev_faithful_shards_uniform_local: shard / nshards differ from the count phase's");
    return PLUSS_ERR_CONFIG;
  }
  if (int rc = uni_plan_remove(ctx, (const unsigned long long*)d_rows, (uint32_t)shard, (uint32_t)nshards, s))
    return rc;
  if (to_host) PLUSS_HIP_CHECK(hipMemcpyAsync(ctx->ub.hinfo, ctx->ub.info, UI_W * 8, hipMemcpyDeviceToHost, s));
  f.phase = SH_UWINDOW;
  return PLUSS_OK;
}

// ... then the shard's slice, its tile map and the local pass (phase 1)
int faith_shards_uniform_finish(pluss_ctx* ctx, uint64_t* d_row, hipStream_t s, const uint64_t* known) {
  if (!ctx->fsh2 || ctx->fsh2->phase != SH_UWINDOW) {
    set_error("pluss_dev_faithful_shards_uniform_local: out of order");
    return PLUSS_ERR_CONFIG;
  }
  FaShards& f = *ctx->fsh2;
  const uint64_t* info = (const uint64_t*)ctx->ub.hinfo + 6;  // (first[6], n[6])
  if (known) {
    if (int rc = uni_slice_check(ctx, known, s)) return rc;
    info = known;
  } else {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
  }
  FaRefs a = fa_none();
  uint64_t n[6];
  for (int r = 0; r < 6; ++r) {
    const uint64_t first = info[r], m = info[6 + r];
    n[r] = f.tot[r] && first <= f.tot[r] && m <= f.tot[r] - first ? m : 0;  // (a flagged plan: reported at the fetch)
    a.n[r] = n[r];
    a.ntot[r] = f.tot[r];
    a.joff[r] = n[r] ? first : 0;
  }
  const UniSet* us = nullptr;
  if (int rc = uni_plan_tiles(ctx, n, s, &us)) return rc;
  a.us = us;
  f.src = SRC_UNI;
  if (int rc = fa_prepare(ctx, a, f.src, false, true, s, &f.L)) return rc;
  return shards_phase1(ctx, f, d_row, s);
}

int faith_shards_slice(pluss_ctx* ctx, uint64_t* first, uint64_t* n) {
  if (!ctx->fsh2 || !ctx->fsh2->has_slice) {
    set_error("pluss_dev_faithful_shards_slice: no key-range pass past its local phase on this handle");
    return PLUSS_ERR_CONFIG;
  }
  for (int r = 0; r < 6; ++r) {
    first[r] = ctx->fsh2->L.a.joff[r];
    n[r] = ctx->fsh2->L.a.n[r];
  }
  return PLUSS_OK;
}

int faith_shards_carry(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards, uint64_t* d_row,
                       hipStream_t s) {
  if (int rc = shards_expect(ctx, SH_LOCAL, "pluss_dev_faithful_shards_carry", d_rows, shard, nshards)) return rc;
  FaShards& f = *ctx->fsh2;
  FaithfulBufs& b = ctx->fb;
  f.L.s = s;
  hipLaunchKernelGGL(k_fa_xchg<0>, dim3(1), dim3(64), 0, s, (const unsigned long long*)d_rows, (uint32_t)nshards,
                     (uint32_t)shard, 2, b.xin, ctx->g);
  if (f.L.t)
    if (int rc = fa_launch(ctx, f.L, f.src, FA_PH_CHUNK)) return rc;
  hipLaunchKernelGGL(k_fa_shard_sums<0>, dim3(6), dim3(SS_NT), 0, s, f.L.a, b.tmax, b.crec, (unsigned long long*)d_row,
                     1);
  PLUSS_HIP_CHECK(hipGetLastError());
  PLUSS_STAGE(s, "shard phase 2 (carry)");
  f.phase = SH_CARRY;
  return PLUSS_OK;
}

int faith_shards_cut(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards, uint64_t* d_row,
                     hipStream_t s) {
  if (int rc = shards_expect(ctx, SH_CARRY, "pluss_dev_faithful_shards_cut", d_rows, shard, nshards)) return rc;
  FaShards& f = *ctx->fsh2;
  FaithfulBufs& b = ctx->fb;
  f.L.s = s;
  hipLaunchKernelGGL(k_fa_xchg<0>, dim3(1), dim3(64), 0, s, (const unsigned long long*)d_rows, (uint32_t)nshards,
                     (uint32_t)shard, 3, b.xin, ctx->g);
  hipLaunchKernelGGL(k_fa_shard_sums<0>, dim3(6), dim3(SS_NT), 0, s, f.L.a, b.tmax, b.crec, (unsigned long long*)d_row,
                     2);
  if (f.L.t) {
    f.L.row = (unsigned long long*)d_row;
    if (int rc = fa_launch(ctx, f.L, f.src, FA_PH_CUT)) return rc;
  }
  PLUSS_HIP_CHECK(hipGetLastError());
  PLUSS_STAGE(s, "shard phase 3 (cut)");
  f.phase = SH_CUT;
  return PLUSS_OK;
}

int faith_shards_hist(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards, hipStream_t s) {
  if (int rc = shards_expect(ctx, SH_CUT, "pluss_dev_faithful_shards_hist", d_rows, shard, nshards)) return rc;
  FaShards& f = *ctx->fsh2;
  FaithfulBufs& b = ctx->fb;
  f.phase = SH_NONE;
  hipLaunchKernelGGL(k_fa_xchg<0>, dim3(1), dim3(64), 0, s, (const unsigned long long*)d_rows, (uint32_t)nshards,
                     (uint32_t)shard, 4, b.xin, ctx->g);
  if (f.L.t)
    hipLaunchKernelGGL(k_fa_shard_apply<0>, dim3(1), dim3(64), 0, s, f.L.m, f.L.a, b.shrec,
                       (const unsigned long long*)b.xin, b.fslot, f.L.g);
  PLUSS_HIP_CHECK(hipGetLastError());
  PLUSS_STAGE(s, "shard phase 4 (hist)");
  ctx->tables_dirty = true;
  return PLUSS_OK;
}

void faith_shards_abandon(pluss_ctx* ctx) {
  if (ctx->fsh2) ctx->fsh2->phase = SH_NONE;
}

void faith_shards_free(pluss_ctx* ctx) {
  delete ctx->fsh2;
  ctx->fsh2 = nullptr;
}

}  // namespace pluss
