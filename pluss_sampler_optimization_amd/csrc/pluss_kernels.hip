// pluss_kernels.hip — gfx950 kernels of the PLUSS reuse-interval hot path.
//
//   k_count         (HOT, N % W == 0: every BASELINE shape) one pass over the
//                   packed sample list: each sample's (ref, case) is decided
//                   by 0-3 integer tests (pluss_model.h, case_fast) and counted
//                   by wave ballots / per-lane counters; one of three tails
//                   (accumulate, fused export, dense vector).  Replaces the
//                   replay loop of r10 sampler_<REF> (r10:275-654) and
//                   pluss_parallel_histogram_update (pluss_utils.h:726-729).
//   k_sampled_hist  the same for other shapes: exact RIs by line-element
//                   enumeration, keys through the wave cache (pluss_device.h).
//   k_fulltrace_count / k_fulltrace
//                   every access of the nest, indices generated in-kernel (no
//                   HBM input); replaces seq.cpp:37-333 / rayon.rs:186-378.
//   k_export        folds the replicas into a canonical sorted table.
//   k_ri_dump       per-sample (RI, sink key) parity dump.
//   k_expand        the sample-list bijection (pluss_model.h).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pluss_device.h"

namespace pluss {

// Exact key of an access on any shape (line-element enumeration).
__device__ __forceinline__ uint64_t key_generic(const Model& m, uint32_t ref, uint32_t c0, uint32_t c1, uint32_t c2) {
  const int64_t ri = ri_generic(m, ref, c0, c1, c2);
  return make_key(ref, share_kind(m, ref, ri), ri);
}

__device__ __forceinline__ uint64_t sample_key(const Model& m, uint64_t x, bool* bad) {
  const Sample s = unpack(x);
  const bool b = s.ref > 5 || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N;
  *bad = b;
  if (b) return KEY_NONE;  // the generic rules loop over line elements: skip bad input
  return key_generic(m, s.ref, s.c0, s.c1, s.c2);
}

// ------------------------------------------------------- GENERIC shapes --
// k_sampled_hist: shapes with N % W != 0, where a line can span two rows and
// a sample's RI is not one of a few closed forms.  One lane per sampled
// access: exact RI by line-element enumeration (ri_generic), keys counted
// through the wave-aggregated cache path (pluss_device.h).  Grid-stride over
// 16-byte sample pairs, UNROLL pairs per lane per step, the next step's loads
// issued before the current step's samples are counted.
constexpr int BIN_BAD = 18;  // dense vector slot of the malformed-sample count

__global__ __launch_bounds__(BLOCK) void k_sampled_hist(Model m, const uint64_t* __restrict__ smp, uint64_t n,
                                                        const uint64_t* __restrict__ head, int has_head, GTable g) {
  __shared__ unsigned long long tk[TCAP];
  __shared__ unsigned int tc[TCAP];
  const BlockTable bt{tk, tc};
  WaveCache wc;
  bt_init(bt);
  wc_init(wc);
  __syncthreads();

  const uint64_t npairs = n >> 1;
  const ulonglong2* __restrict__ v = reinterpret_cast<const ulonglong2*>(smp);
  const uint64_t step = (uint64_t)gridDim.x * BLOCK * UNROLL;
  bool anybad = false;
  uint64_t base = (uint64_t)blockIdx.x * BLOCK * UNROLL;
  const uint64_t last = npairs ? npairs - 1 : 0;  // loads are clamped, lanes past the end are masked
  ulonglong2 x[UNROLL];
  if (npairs) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t i = base + (uint64_t)u * BLOCK + threadIdx.x;
      x[u] = v[i < last ? i : last];
    }
  }
  for (; base < npairs; base += step) {
    ulonglong2 y[UNROLL];
    const uint64_t nb = base + step;
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {  // prefetch the next step
      const uint64_t i = nb + (uint64_t)u * BLOCK + threadIdx.x;
      y[u] = v[i < last ? i : last];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const bool ok = base + (uint64_t)u * BLOCK + threadIdx.x < npairs;
      bool b0, b1;
      const uint64_t k0 = sample_key(m, x[u].x, &b0);
      const uint64_t k1 = sample_key(m, x[u].y, &b1);
      anybad |= ok && (b0 || b1);
      wave_count(wc, bt, g, k0, ok && !b0);
      wave_count(wc, bt, g, k1, ok && !b1);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) x[u] = y[u];
  }
  if (((n & 1) || has_head) && blockIdx.x == 0 && threadIdx.x < 64) {
    // odd tail (lane 0) and, for an 8-byte-aligned list, its first sample (lane 1).
    // `head` always points at valid memory, so a speculated load cannot fault.
    const bool mine = (threadIdx.x == 0 && (n & 1)) || (threadIdx.x == 1 && has_head);
    const uint64_t* src = (threadIdx.x == 0 && n) ? smp + (n - 1) : head;
    const uint64_t xs = mine ? *src : 0;
    bool b = false;
    const uint64_t k = mine ? sample_key(m, xs, &b) : KEY_NONE;
    anybad |= mine && b;
    wave_count(wc, bt, g, k, mine && !b);
  }
  if (anybad) atomicOr(&g.flags[1], 1u);
  bt_finish(wc, bt, g);
}

// Accumulating tail: each bin with a count is added to its direct counter in
// row blockIdx % 64 (workgroups are dealt round-robin over the 8 XCDs, so a
// row is hit from one XCD, by 1/64 of the grid: 16 adds per address at 1024
// workgroups).  `tot` is in LDS, complete (after a barrier).
__device__ __forceinline__ void tail_accumulate(const unsigned long long* tot, GTable g) {
  if (threadIdx.x < 18 && tot[threadIdx.x])
    atomicAdd(&g.bins[(blockIdx.x & (NBROW - 1)) * BSTRIDE + threadIdx.x], tot[threadIdx.x]);
  if (threadIdx.x == BIN_BAD && tot[BIN_BAD]) atomicOr(&g.flags[1], 1u);
}

// Dense tail (pluss_dev_sampled_hist_dense): the 18 (ref, case) totals and
// the malformed-sample count of this launch go to out[0..18], and the state
// is left zeroed -- with no arrival counter, fence or extra load.  Every
// workgroup adds (1 << DARR_SHIFT | its count) to each of the DBINS words of
// its row (one wave instruction, 19 lanes, returning).  The add that returns
// arrivals == (workgroups in the row) - 1 is the row's last for that bin, so
// old + own is the row total: that lane zeroes the word and adds
// (1 << DARR_SHIFT | row total) to the bin's word in `dtot`; the add there
// that returns arrivals == rows - 1 holds the launch total, which the lane
// stores to out[b].  Critical path after the count: two returning atomics.
// `drows` (a power of two <= NBROW) rows: about sqrt(grid) balances the adds per word of the two levels.
__device__ __forceinline__ void tail_dense(const unsigned long long* tot, GTable g, unsigned long long* out,
                                           uint32_t drows) {
  if (threadIdx.x < DBINS) {
    const uint32_t b = threadIdx.x;
    const uint32_t row = blockIdx.x & (drows - 1);
    const uint32_t rows = gridDim.x < drows ? gridDim.x : drows;
    const uint32_t in_row = (gridDim.x - row + drows - 1) / drows;
    const unsigned long long v = (1ull << DARR_SHIFT) | tot[b];
    unsigned long long* w = &g.dbins[row * BSTRIDE + b];
    const unsigned long long old = __hip_atomic_fetch_add(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old >> DARR_SHIFT) == in_row - 1) {
      __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long v2 = (1ull << DARR_SHIFT) | ((old + v) & DCNT_MASK);
      unsigned long long* t = &g.dtot[b];
      const unsigned long long old2 = __hip_atomic_fetch_add(t, v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((old2 >> DARR_SHIFT) == rows - 1) {
        __hip_atomic_store(t, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out[b] = (old2 + v2) & DCNT_MASK;
      }
    }
    if (b == BIN_BAD && tot[BIN_BAD]) atomicOr(&g.flags[1], 1u);
  }
}

// Tail of a fused count+export launch, run by the last workgroup to finish:
// fold the direct bins of all replicas (equal keys merged), write the
// canonical table -- distinct keys ascending, then (~0, 0) up to `cap` --
// and leave the histogram empty (bins, traversed, the finish counter).
// Only used when the hash tables hold nothing (pluss_ctx::tables_dirty).
__device__ void bins_export_tail(const Model& m, GTable g, unsigned long long* ok, unsigned long long* oc,
                                 uint64_t cap, unsigned int* nout) {
  __shared__ unsigned long long ek[18], ec[18];
  __shared__ unsigned int en;
  const uint32_t t = threadIdx.x;
  if (t == 0) en = 0;
  if (t < 18) {
    ek[t] = m.keytab[t];
    ec[t] = 0;
  }
  if (t < 8) g.trav[t] = 0;
  __syncthreads();
  constexpr uint32_t PER = (NBROW * 18 + BLOCK - 1) / BLOCK;
  unsigned long long c[PER];
#pragma unroll
  for (uint32_t j = 0; j < PER; ++j) {  // every load in flight before the first is used
    const uint32_t i = t + j * BLOCK;
    c[j] = i < NBROW * 18
               ? __hip_atomic_load(&g.bins[(i / 18) * BSTRIDE + i % 18], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
               : 0ull;
  }
#pragma unroll
  for (uint32_t j = 0; j < PER; ++j) {
    const uint32_t i = t + j * BLOCK;
    if (c[j]) {
      atomicAdd(&ec[i % 18], c[j]);
      __hip_atomic_store(&g.bins[(i / 18) * BSTRIDE + i % 18], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  unsigned long long key = 0, tot = 0;
  uint32_t rank = 0;
  bool first = false;
  if (t < 18 && ec[t]) {
    key = ek[t];
    first = true;
    for (uint32_t j = 0; j < 18; ++j) {
      if (!ec[j]) continue;
      if (ek[j] == key) {
        tot += ec[j];
        first &= j >= t;
      }
    }
    if (first) {
      // rank = distinct nonzero keys below `key` (count each key at its first index)
      for (uint32_t j = 0; j < 18; ++j) {
        if (!ec[j] || ek[j] >= key) continue;
        bool jfirst = true;
        for (uint32_t i = 0; i < j; ++i) jfirst &= !(ec[i] && ek[i] == ek[j]);
        rank += jfirst;
      }
      atomicAdd(&en, 1u);
    }
  }
  __syncthreads();
  const uint32_t n = en;
  if (first && rank < cap) {
    ok[rank] = key;
    oc[rank] = tot;
  }
  uint64_t i0 = n < cap ? n : cap;
  if (((((uintptr_t)ok) | ((uintptr_t)oc)) & 15u) == 0) {  // 16-byte stores for the empty pairs
    if ((i0 & 1) && i0 < cap) {
      if (t == 0) {
        ok[i0] = KEY_EMPTY;
        oc[i0] = 0ull;
      }
      ++i0;
    }
    const uint64_t np = (cap - i0) / 2;
    ulonglong2* k2 = reinterpret_cast<ulonglong2*>(ok + i0);
    ulonglong2* c2 = reinterpret_cast<ulonglong2*>(oc + i0);
    for (uint64_t p = t; p < np; p += BLOCK) {
      k2[p] = ulonglong2{KEY_EMPTY, KEY_EMPTY};
      c2[p] = ulonglong2{0ull, 0ull};
    }
    i0 += 2 * np;
  }
  for (uint64_t i = i0 + t; i < cap; i += BLOCK) {
    ok[i] = KEY_EMPTY;
    oc[i] = 0ull;
  }
  if (t == 0) {
    *nout = n;
    if (n > cap) atomicOr(&g.flags[0], 2u);
    __hip_atomic_store(&g.flags[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// What a launch does after counting: TAIL_NONE accumulates into the
// handle's bins; TAIL_EXPORT (fused count + export) -- the last workgroup to
// finish writes the canonical table and empties the histogram; TAIL_DENSE
// writes this launch's dense counts to `dense` (tail_dense).
enum : int { TAIL_NONE = 0, TAIL_EXPORT = 1, TAIL_DENSE = 2 };
struct ExportArgs {
  unsigned long long* keys;
  unsigned long long* counts;
  uint64_t cap;
  unsigned int* nout;
  unsigned long long* dense;
  uint32_t drows;  // dense tail: rows of the first level (power of two <= NBROW)
};

// Fused export, after tail_accumulate: an arrival count without fences --
// every bin update is an agent-scope atomic RMW issued by wave 0 (threads
// 0..18), performed at the coherent point; once the wave's vmcnt drains they
// are visible to every XCD, and the last arriver reads them back with
// agent-scope atomic loads (bins_export_tail).  (A __threadfence here costs
// an L2 writeback + invalidate per workgroup, measured 4x the kernel's run
// time.)
__device__ __forceinline__ void tail_export(const Model& m, GTable g, const ExportArgs& ex) {
  __shared__ unsigned int amlast;
  if (threadIdx.x == 0) {
    // two-level arrival (one counter per bin row, then one per grid) so the
    // simultaneous finishes of ~1000 workgroups do not serialise on a single
    // address
    const uint32_t row = blockIdx.x & (NBROW - 1);
    const uint32_t rows = gridDim.x < NBROW ? gridDim.x : NBROW;
    const uint32_t in_row = (gridDim.x - row + NBROW - 1) / NBROW;
    unsigned long long* rc = &g.bins[row * BSTRIDE + BARRIVE];
    __builtin_amdgcn_s_waitcnt(0);
    bool last = false;
    if (__hip_atomic_fetch_add(rc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_row - 1) {
      __hip_atomic_store(rc, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(&g.flags[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == rows - 1;
    }
    amlast = last;
  }
  __syncthreads();
  if (amlast) bins_export_tail(m, g, ex.keys, ex.counts, ex.cap, ex.nout);
}

// --------------------------------------------------- HOT (FAST shapes) --
// k_count: the sampled pass for N % W == 0 shapes (every BASELINE shape).
// A "slot" is one sample per lane (64 per wave).  The wave finds the
// references present in the slot (almost always one: lists are per-reference
// blocks), and for each one evaluates only that reference's case conditions
// as lane predicates; their ballots, masked and popcounted, are added to
// per-wave counters held in scalar registers.  So a sample costs its field
// extraction and 0-3 compares (the rest is scalar work per 64 samples), and
// there are no per-sample LDS atomics.  Samples are read as 16-byte pairs by
// buffer loads with 32-bit offsets inside windows of up to 2^27 pairs; lanes
// past the end read zeros (range check) and are masked.
constexpr uint64_t CWIN = 1ull << 27;  // pairs per buffer window (2 GiB)

// bins: C0 0, C1 3, A0 6/7/8, B0 9/10/11, C2 12, C3 15/16/17, malformed 18 (= ref*3 + case).
// Counts live in one lane-indexed VGPR per wave: lane b holds bin b.
//
// Count the lanes `mr` of a slot whose reference is the wave-uniform `r`.
template <bool P2, bool NP2>
__device__ __forceinline__ void count_ref(const Model& m, uint32_t r, uint64_t mr, uint32_t lo, uint32_t hi,
                                          uint32_t& acc) {
  const uint32_t c2 = lo & 0xFFFFFu;
  const uint32_t c0 = (hi >> 8) & 0xFFFFFu;
  bool bad;
  if (NP2) {
    bad = ((lo & m.badlo) | (hi & m.badhi)) != 0u;
  } else {
    const uint32_t c1 = __builtin_amdgcn_alignbit(hi, lo, 20) & 0xFFFFFu;
    bad = (c0 > c1 ? (c0 > c2 ? c0 : c2) : (c1 > c2 ? c1 : c2)) >= m.N;
  }
  const uint64_t mb = r > 5 ? mr : (__ballot(bad) & mr);
  mr &= ~mb;
  const uint32_t nr = (uint32_t)__popcll(mr);
  const uint32_t Wm1 = m.W - 1;
  uint64_t a = mr, b = 0;  // lanes of case 0 and case 1 (case 2: the rest); C0, C1, C2 are always case 0
  if (r == C3) {  // case 0: c2+1 < N; case 1: c1 not the last element of its line
    const uint32_t c1 = __builtin_amdgcn_alignbit(hi, lo, 20) & 0xFFFFFu;
    const bool c1last = P2 ? (lo & (m.wmask << 20)) == (m.wmask << 20) : fmod_(c1, m.dW) == Wm1;
    a = __ballot(c2 + 1 < m.N) & mr;
    b = __ballot(!c1last) & mr & ~a;
  } else if (r == A0) {  // case 0: c2 not the last element of its line; case 1: c1+1 < N
    const uint32_t c1 = __builtin_amdgcn_alignbit(hi, lo, 20) & 0xFFFFFu;
    const bool c2last = P2 ? (lo & m.wmask) == m.wmask : fmod_(c2, m.dW) == Wm1;
    a = __ballot(!c2last) & mr;
    b = __ballot(c1 + 1 < m.N) & mr & ~a;
  } else if (r == B0) {  // case 0: c1 not the last element of its line; case 1: the thread owns a later row
    const uint32_t c1 = __builtin_amdgcn_alignbit(hi, lo, 20) & 0xFFFFFu;
    const bool c1last = P2 ? (lo & (m.wmask << 20)) == (m.wmask << 20) : fmod_(c1, m.dW) == Wm1;
    const uint32_t p = P2 ? (c0 & m.csmask) : fmod_(c0, m.dCS);
    const uint32_t nxt = c0 + 1 + (p + 1 == m.CS ? m.tcs : 0u);
    a = __ballot(!c1last) & mr;
    b = __ballot(nxt < m.N) & mr & ~a;
  }
  // lane-indexed add of a wave-uniform count: compare, select, add
  const uint32_t lane = __lane_id();
  auto bump = [&acc, lane](uint32_t bin, uint32_t v) { acc += lane == bin ? v : 0u; };
  if (r <= 5 && nr) {
    const uint32_t na = (uint32_t)__popcll(a);
    bump(r * 3, na);
    if (r == C3 || r == A0 || r == B0) {
      const uint32_t nb = (uint32_t)__popcll(b);
      bump(r * 3 + 1, nb);
      bump(r * 3 + 2, nr - na - nb);
    }
  }
  if (mb) bump(BIN_BAD, (uint32_t)__popcll(mb));
}

// One slot: the wave's first live lane names the reference; lanes with
// another reference (a slot that straddles two per-reference blocks, or a
// mixed list) are counted one reference at a time.
template <bool P2, bool NP2>
__device__ __forceinline__ void count_slot(const Model& m, uint64_t x, bool ok, uint32_t& acc) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t ref = hi >> 28;
  uint64_t live = __ballot(ok);
  if (live == 0) return;
  const uint32_t r0 = __builtin_amdgcn_readlane(ref, (int)__builtin_ctzll(live));
  const uint64_t m0 = __ballot(ref == r0) & live;
  count_ref<P2, NP2>(m, r0, m0, lo, hi, acc);
  live &= ~m0;
  while (live) {
    const uint32_t r = __builtin_amdgcn_readlane(ref, (int)__builtin_ctzll(live));
    const uint64_t mr = __ballot(ref == r) & live;
    live &= ~mr;
    count_ref<P2, NP2>(m, r, mr, lo, hi, acc);
  }
}

// All 2*UNR slots of a step (okm[k] = the live lanes of slot k; in k_count
// lane-pair u holds slots 2u and 2u+1).  A lane whose slot k is live has its
// slot 0 live too.  When every live sample of the step has the reference of the
// first live lane (almost always), that reference's conditions are evaluated
// for all slots in one straight-line block -- independent ballots the
// scheduler interleaves -- and the counts are summed in scalar registers
// before one lane-indexed add per bin.  Otherwise slot by slot.
template <bool P2, bool NP2, int UNR>
__device__ __forceinline__ void count_step(const Model& m, const uint32_t (&lo)[2 * UNR], const uint32_t (&hi)[2 * UNR],
                                           const uint64_t (&okm)[2 * UNR], uint32_t& acc) {
  constexpr int K = 2 * UNR;
  uint64_t any = 0;
#pragma unroll
  for (int k = 0; k < 2 * UNR; ++k) any |= okm[k];
  if (any == 0) return;
  const int l0 = (int)__builtin_ctzll(any);
  const uint32_t r0 = __builtin_amdgcn_readlane(hi[0] >> 28, l0);  // slot 0 is live wherever any slot is
  uint64_t mixed = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) mixed |= __ballot((hi[k] >> 28) != r0) & okm[k];
  if (r0 > 5 || mixed) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      count_slot<P2, NP2>(m, ((uint64_t)hi[k] << 32) | lo[k], (okm[k] >> __lane_id()) & 1, acc);
    return;
  }
  uint32_t nbad = 0, ng = 0, na = 0, nb = 0;
  uint64_t good[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    bool bad;
    if (NP2) {
      bad = ((lo[k] & m.badlo) | (hi[k] & m.badhi)) != 0u;
    } else {
      const uint32_t c2 = lo[k] & 0xFFFFFu, c0 = (hi[k] >> 8) & 0xFFFFFu;
      const uint32_t c1 = __builtin_amdgcn_alignbit(hi[k], lo[k], 20) & 0xFFFFFu;
      bad = (c0 > c1 ? (c0 > c2 ? c0 : c2) : (c1 > c2 ? c1 : c2)) >= m.N;
    }
    const uint64_t mb = __ballot(bad) & okm[k];
    good[k] = okm[k] & ~mb;
    nbad += (uint32_t)__popcll(mb);
    ng += (uint32_t)__popcll(good[k]);
  }
  const uint32_t Wm1 = m.W - 1;
  switch (r0) {
    case C3:
#pragma unroll
      for (int k = 0; k < K; ++k) {  // case 0: c2+1 < N; case 1: c1 not the last element of its line
        const uint32_t c2 = lo[k] & 0xFFFFFu;
        const uint32_t c1 = __builtin_amdgcn_alignbit(hi[k], lo[k], 20) & 0xFFFFFu;
        const bool c1last = P2 ? (lo[k] & (m.wmask << 20)) == (m.wmask << 20) : fmod_(c1, m.dW) == Wm1;
        const uint64_t a = __ballot(c2 + 1 < m.N) & good[k];
        na += (uint32_t)__popcll(a);
        nb += (uint32_t)__popcll(__ballot(!c1last) & good[k] & ~a);
      }
      break;
    case A0:
#pragma unroll
      for (int k = 0; k < K; ++k) {  // case 0: c2 not the last element of its line; case 1: c1+1 < N
        const uint32_t c2 = lo[k] & 0xFFFFFu;
        const uint32_t c1 = __builtin_amdgcn_alignbit(hi[k], lo[k], 20) & 0xFFFFFu;
        const bool c2last = P2 ? (lo[k] & m.wmask) == m.wmask : fmod_(c2, m.dW) == Wm1;
        const uint64_t a = __ballot(!c2last) & good[k];
        na += (uint32_t)__popcll(a);
        nb += (uint32_t)__popcll(__ballot(c1 + 1 < m.N) & good[k] & ~a);
      }
      break;
    case B0:
#pragma unroll
      for (int k = 0; k < K; ++k) {  // case 0: c1 not the last element of its line; case 1: a later owned row
        const uint32_t c0 = (hi[k] >> 8) & 0xFFFFFu;
        const uint32_t c1 = __builtin_amdgcn_alignbit(hi[k], lo[k], 20) & 0xFFFFFu;
        const bool c1last = P2 ? (lo[k] & (m.wmask << 20)) == (m.wmask << 20) : fmod_(c1, m.dW) == Wm1;
        const uint32_t p = P2 ? (c0 & m.csmask) : fmod_(c0, m.dCS);
        const uint32_t nxt = c0 + 1 + (p + 1 == m.CS ? m.tcs : 0u);
        const uint64_t a = __ballot(!c1last) & good[k];
        na += (uint32_t)__popcll(a);
        nb += (uint32_t)__popcll(__ballot(nxt < m.N) & good[k] & ~a);
      }
      break;
    default:  // C0, C1, C2: always case 0
      na = ng;
      break;
  }
  const uint32_t lane = __lane_id(), b0 = r0 * 3;
  acc += lane == b0 ? na : 0u;
  acc += lane == b0 + 1 ? nb : 0u;
  acc += lane == b0 + 2 ? ng - na - nb : 0u;
  acc += lane == BIN_BAD ? nbad : 0u;
}

// Per-lane counters of the vector fast path (count_step_lanes): for each
// reference the lanes count only the outcomes that need a per-sample test; the
// sample totals per reference are wave-uniform (every lane holds 2*UNR
// samples of the step) and live in scalar registers.
struct LaneCounts {
  uint32_t a_last, a_c1;    // A0: c2 last in its line; and c1+1 < N as well
  uint32_t c_lt, c_last;    // C3: c2+1 < N; c2 = N-1 with c1 last in its line
  uint32_t b_last, b_next;  // B0: c1 last in its line; and a later owned row as well
  // samples per reference per lane (wave-uniform); named, not an array, so no
  // switch is turned into an indexed (scratch) update
  uint32_t t_c0, t_c1, t_a0, t_b0, t_c2, t_c3;
};
__device__ __forceinline__ void lc_init(LaneCounts& c) {
  c.a_last = c.a_c1 = c.c_lt = c.c_last = c.b_last = c.b_next = 0;
  c.t_c0 = c.t_c1 = c.t_a0 = c.t_b0 = c.t_c2 = c.t_c3 = 0;
}

// 1 if x < y (both < 2^31), as an integer: no compare, no lane mask
__device__ __forceinline__ uint32_t lt01(uint32_t x, uint32_t y) { return (x - y) >> 31; }

// A full step whose samples all have the wave's reference r0 and are in
// range, for N, W and CS powers of two (every BASELINE shape).  Each test is
// integer arithmetic on the lane's own samples (VALU only); the scalar unit
// does one check and one branch per step.  Returns false (nothing counted)
// when the step needs count_step instead.
template <int UNR>
__device__ __forceinline__ bool count_step_lanes(const Model& m, const uint32_t (&lo)[2 * UNR],
                                                 const uint32_t (&hi)[2 * UNR], LaneCounts& c) {
  constexpr int K = 2 * UNR;
  const uint32_t r0 = __builtin_amdgcn_readfirstlane(hi[0] >> 28);
  if (r0 > 5) return false;
  uint32_t odd = 0;  // another reference, or an index >= N, somewhere in the lane's samples
#pragma unroll
  for (int k = 0; k < K; ++k) odd |= ((hi[k] ^ (r0 << 28)) & (0xF0000000u | m.badhi)) | (lo[k] & m.badlo);
  if (__ballot(odd != 0u) != 0) return false;
  const uint32_t wsh = m.wsh, wm = m.wmask;
  switch (r0) {
    case A0:
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t last = ((lo[k] & wm) + 1u) >> wsh;                                   // c2 % W == W-1
        const uint32_t c1n = lt01(__builtin_amdgcn_alignbit(hi[k], lo[k], 20) & 0xFFFFFu, m.N - 1);  // c1+1 < N
        c.a_last += last;
        c.a_c1 += last & c1n;
      }
      break;
    case B0:
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t last = (((lo[k] >> 20) & wm) + 1u) >> wsh;  // c1 % W == W-1
        const uint32_t c0 = (hi[k] >> 8) & 0xFFFFFu;
        const uint32_t pl = ((c0 & m.csmask) + 1u) >> m.csshift;   // c0 % CS == CS-1
        c.b_last += last;
        c.b_next += last & lt01(c0 + 1u + pl * m.tcs, m.N);        // the thread owns a later row
      }
      break;
    case C3:
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint32_t lt = lt01(lo[k] & 0xFFFFFu, m.N - 1);       // c2+1 < N
        const uint32_t last = (((lo[k] >> 20) & wm) + 1u) >> wsh;  // c1 % W == W-1
        c.c_lt += lt;
        c.c_last += (lt ^ 1u) & last;
      }
      break;
    default:  // C0, C1, C2: always case 0
      break;
  }
  // per-reference sample totals: branch-free scalar selects (wave-uniform)
  c.t_c0 += r0 == C0 ? (uint32_t)K : 0u;
  c.t_c1 += r0 == C1 ? (uint32_t)K : 0u;
  c.t_a0 += r0 == A0 ? (uint32_t)K : 0u;
  c.t_b0 += r0 == B0 ? (uint32_t)K : 0u;
  c.t_c2 += r0 == C2 ? (uint32_t)K : 0u;
  c.t_c3 += r0 == C3 ? (uint32_t)K : 0u;
  return true;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Fold the lane counters into the lane-indexed counts (lane b: bin b).
__device__ __forceinline__ void lc_flush(LaneCounts& c, uint32_t& acc) {
  const uint32_t al = wave_sum(c.a_last), ac = wave_sum(c.a_c1), cl = wave_sum(c.c_lt), cc = wave_sum(c.c_last);
  const uint32_t bl = wave_sum(c.b_last), bn = wave_sum(c.b_next);
  // per-lane sample counts are the same in every lane
  const uint32_t t0 = c.t_c0 * 64u, t1 = c.t_c1 * 64u, ta = c.t_a0 * 64u, tb = c.t_b0 * 64u, t4 = c.t_c2 * 64u,
                 t5 = c.t_c3 * 64u;
  const uint32_t bins[18] = {t0, 0, 0, t1, 0, 0, ta - al, ac, al - ac, tb - bl, bn, bl - bn,
                             t4, 0, 0, cl, t5 - cl - cc, cc};
  const uint32_t lane = __lane_id();
#pragma unroll
  for (uint32_t b = 0; b < 18; ++b) acc += lane == b ? bins[b] : 0u;
  lc_init(c);
}

// Add the wave's lane-indexed counts to the workgroup's LDS totals.
__device__ __forceinline__ void flush_counts(uint32_t& acc, unsigned long long* tot) {
  const uint32_t lane = __lane_id();
  if (lane < DBINS && acc) atomicAdd(&tot[lane], (unsigned long long)acc);
  acc = 0;
}

// ABL: 0 = the product kernel; diagnostics only (pluss_diag_dense, include/pluss_diag.h):
// 1 = the same loads, nothing counted; 2 = counted, no tail (nothing written).
// Sample loads are non-temporal (aux 2): the list is streamed once per pass.
template <bool P2, bool NP2, int TAIL, int ABL = 0>
__global__ __launch_bounds__(BLOCK) void k_count(Model m, const uint64_t* __restrict__ smp, uint64_t n,
                                                 const uint64_t* __restrict__ head, int has_head, GTable g,
                                                 ExportArgs ex) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int UNR = UNROLL, AUX = 2;
  __shared__ unsigned long long tot[DBINS];
  if (threadIdx.x < DBINS) tot[threadIdx.x] = 0;  // the barrier before the first flush orders this
  uint32_t acc = 0;  // lane b: count of bin b
  LaneCounts lc;     // the vector fast path's counters (count_step_lanes)
  lc_init(lc);
  const uint64_t npairs = n >> 1;
  const uint32_t step = gridDim.x * (uint32_t)(BLOCK * UNR);
  for (uint64_t w0 = 0; w0 < npairs; w0 += CWIN) {
    const uint32_t wn = (uint32_t)(npairs - w0 < CWIN ? npairs - w0 : CWIN);
    const uint64_t* wp = smp + 2 * w0;
    const uint32_t plo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)wp);
    const uint32_t phi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)wp >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uintptr_t)phi << 32) | plo), 0, (int)__builtin_amdgcn_readfirstlane(wn * 16u), 0x00020000);
    uint32_t base = blockIdx.x * (uint32_t)(BLOCK * UNR);
    u32x4 x[UNR];  // this step's pairs
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      x[u] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((base + u * BLOCK + threadIdx.x) * 16u), 0, AUX));
    for (; base < wn; base += step) {
      u32x4 y[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u)  // the next step's pairs (past the window: zeros)
        y[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rs, (int)((base + step + u * BLOCK + threadIdx.x) * 16u), 0, AUX));
      uint32_t lo[2 * UNR], hi[2 * UNR];
      uint64_t okm[2 * UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        lo[2 * u] = x[u].x;
        hi[2 * u] = x[u].y;
        lo[2 * u + 1] = x[u].z;
        hi[2 * u + 1] = x[u].w;
        okm[2 * u] = okm[2 * u + 1] = __ballot(base + u * BLOCK + threadIdx.x < wn);
      }
      if (ABL == 1) {  // diagnostics: the same loads, nothing counted
#pragma unroll
        for (int k = 0; k < 2 * UNR; ++k) acc ^= lo[k] ^ hi[k];
      } else if (!(P2 && NP2 && base + (uint32_t)(UNR * BLOCK) <= wn && count_step_lanes<UNR>(m, lo, hi, lc))) {
        count_step<P2, NP2, UNR>(m, lo, hi, okm, acc);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) x[u] = y[u];
    }
    if (ABL != 1) {  // per window: keeps the 32-bit lane counters from overflowing
      if (P2 && NP2) lc_flush(lc, acc);
      __syncthreads();
      flush_counts(acc, tot);
    }
  }
  if (((n & 1) || has_head) && blockIdx.x == 0 && threadIdx.x < 64) {
    // odd tail (lane 0) and, for an 8-byte-aligned list, its first sample (lane 1).
    // `head` always points at valid memory, so a speculated load cannot fault.
    const bool mine = (threadIdx.x == 0 && (n & 1)) || (threadIdx.x == 1 && has_head);
    const uint64_t* src = (threadIdx.x == 0 && n) ? smp + (n - 1) : head;
    const uint64_t xs = mine ? *src : 0;
    count_slot<P2, NP2>(m, xs, mine, acc);
    flush_counts(acc, tot);
  }
  if (ABL == 1 || ABL == 2) {
    if (acc == 0x5EED5EEDu || (ABL == 2 && tot[0] == 0x5EED5EEDu)) atomicOr(&g.flags[2], 1u);  // keeps the work alive
    return;
  }
  __syncthreads();
  if (TAIL == TAIL_DENSE) tail_dense(tot, g, ex.dense, ex.drows);
  else tail_accumulate(tot, g);
  if (TAIL == TAIL_EXPORT) tail_export(m, g, ex);
}

// ------------------------------------------------ generated and counted --
// k_gen_count: the key-order lists of the six references (pluss_model.h
// KeyGen) counted while they are generated -- the samples never touch
// memory; = pluss_dev_expand_sorted of every slice + one dense pass.  A wave
// step is 64 runs of GR consecutive samples of one reference (lane l: samples
// base + l*GR ... + GR-1, generated incrementally by keyrun_*); each
// reference's slice is padded to whole wave steps, so the reference, its
// generator and its case rules are wave-uniform.  A sample's outcome comes
// straight from its digits (case_of_digits); per-lane counters per
// (reference, case), folded at the end into k_count's dense tail.
constexpr uint32_t GR = 16;
struct GenArgs {
  KeyGen k[6];
  uint64_t first[6], n[6];
  uint64_t wbeg[7];  // first wave step of each reference; wbeg[6] = all steps
};

__global__ __launch_bounds__(BLOCK) void k_gen_count(Model m, GenArgs ga, GTable g, ExportArgs ex) {
  __shared__ unsigned long long tot[DBINS];
  if (threadIdx.x < DBINS) tot[threadIdx.x] = 0;
  uint32_t na[6], nb[6], nt[6];  // per reference: case 0, case 1, all (case 2 = the rest)
#pragma unroll
  for (int x = 0; x < 6; ++x) na[x] = nb[x] = nt[x] = 0;
  const uint32_t lane = __lane_id();
  const uint32_t Q = m.N / m.T;
  const uint64_t nw = (uint64_t)gridDim.x * (BLOCK / 64);
  const uint64_t w0 = (uint64_t)blockIdx.x * (BLOCK / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint64_t ws = w0; ws < ga.wbeg[6]; ws += nw) {
    uint32_t r = 0;
#pragma unroll
    for (int x = 1; x < 6; ++x) r += ws >= ga.wbeg[x] ? 1u : 0u;
    r = __builtin_amdgcn_readfirstlane(r);
    const KeyGen& kg = ga.k[r];
    const uint64_t j0 = (ws - ga.wbeg[r]) * (64 * GR) + lane * GR;  // this lane's run within the slice
    const uint64_t nr = ga.n[r];
    uint32_t a = 0, b = 0, v = 0;
    // straight-line 32-bit generation when the wave's whole range is in block A
    const uint64_t wfirst = ga.first[r] + (ws - ga.wbeg[r]) * (64 * GR);
    const bool fast = keyrun_fast_ok(kg, wfirst, 64 * GR);
    if (j0 < nr) {
      const uint32_t cnt = nr - j0 < GR ? (uint32_t)(nr - j0) : GR;
      auto tally = [&](const KeyDigits& d) {
        const uint32_t c = m.p2 ? case_of_digits<true>(m, r, d, Q) : case_of_digits<false>(m, r, d, Q);
        a += c == 0 ? 1u : 0u;
        b += c == 1 ? 1u : 0u;
      };
      if (fast) {
        KeyRunF run;
        keyrunf_start(kg, run, ga.first[r] + j0);
#pragma unroll
        for (uint32_t k = 0; k < GR; ++k) {
          if (k < cnt) tally(keyrunf_digits(kg, run));
          keyrunf_next(kg, run);
        }
      } else {
        for (uint32_t k = 0; k < cnt; ++k) tally(keygen_digits_at(kg, ga.first[r] + j0 + k));
      }
      v = cnt;
    }
#pragma unroll
    for (int x = 0; x < 6; ++x) {  // r is wave-uniform: one scalar branch
      if (r == (uint32_t)x) {
        na[x] += a;
        nb[x] += b;
        nt[x] += v;
      }
    }
  }
  uint32_t acc = 0;  // lane b: count of bin b
#pragma unroll
  for (int x = 0; x < 6; ++x) {
    const uint32_t A = wave_sum(na[x]), B = wave_sum(nb[x]), N = wave_sum(nt[x]);
    acc += lane == (uint32_t)(3 * x) ? A : 0u;
    acc += lane == (uint32_t)(3 * x + 1) ? B : 0u;
    acc += lane == (uint32_t)(3 * x + 2) ? N - A - B : 0u;
  }
  __syncthreads();
  flush_counts(acc, tot);
  __syncthreads();
  tail_dense(tot, g, ex.dense, ex.drows);
}

// ----------------------------------------------------------- full trace --
// GENERIC shapes (N % W != 0): one wave per (c0, c1) pair: C0, C1, then the
// c2 loop 64 iterations at a time, exact keys through the wave cache.
__global__ __launch_bounds__(BLOCK) void k_fulltrace(Model m, GTable g) {
  __shared__ unsigned long long tk[TCAP];
  __shared__ unsigned int tc[TCAP];
  const BlockTable bt{tk, tc};
  WaveCache wc;
  const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
  bt_init(bt);
  wc_init(wc);
  __syncthreads();
  const uint64_t nwaves = (uint64_t)gridDim.x * (BLOCK / 64);
  const uint64_t npairs = (uint64_t)m.N * m.N;
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g.trav[0], npairs * m.S);  // accesses traversed
  for (uint64_t pr = (uint64_t)blockIdx.x * (BLOCK / 64) + wave; pr < npairs; pr += nwaves) {
    const uint32_t c0 = (uint32_t)(pr / m.N), c1 = (uint32_t)(pr - (uint64_t)c0 * m.N);
    {
      const bool v = lane < 2;
      uint64_t key = KEY_NONE;
      if (v) key = key_generic(m, lane, c0, c1, 0);
      wave_count(wc, bt, g, key, v);
    }
    for (uint32_t c2b = 0; c2b < m.N; c2b += 64) {
      const uint32_t c2 = c2b + lane;
      const bool v = c2 < m.N;
#pragma unroll
      for (uint32_t ref = A0; ref <= C3; ++ref) {
        uint64_t key = KEY_NONE;
        if (v) key = key_generic(m, ref, c0, c1, c2);
        wave_count(wc, bt, g, key, v);
      }
    }
  }
  bt_finish(wc, bt, g);
}

// Full trace for N % W == 0 shapes, counted by ballots.  One wave per
// (c0, c1) pair; lanes over c2, 64 at a time.  Of the six accesses of an
// iteration only A0's and C3's outcome depends on c2 (the last element of a
// line, the last c2), so each lane evaluates those two predicates for its
// access and the wave popcounts their ballots; the outcomes of C0, C1, B0 and
// C2 are wave-uniform for the pair.  Counts go to a lane-indexed 64-bit
// register per wave (lane b: bin b), then the accumulate tail.
template <bool P2>
__global__ __launch_bounds__(BLOCK) void k_fulltrace_count(Model m, GTable g) {
  __shared__ unsigned long long tot[DBINS];
  if (threadIdx.x < DBINS) tot[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = __lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: pair indices in SGPRs
  unsigned long long acc = 0;
  auto bump = [&acc, lane](uint32_t bin, uint32_t v) { acc += lane == bin ? (unsigned long long)v : 0ull; };
  const uint32_t Wm1 = m.W - 1;
  const uint64_t nwaves = (uint64_t)gridDim.x * (BLOCK / 64);
  const uint64_t npairs = (uint64_t)m.N * m.N;
  const bool small = npairs < (1ull << 31);  // pair index fits the 32-bit fast division by N
  for (uint64_t pr = (uint64_t)blockIdx.x * (BLOCK / 64) + wave; pr < npairs; pr += nwaves) {
    const uint32_t c0 = small ? fdiv((uint32_t)pr, m.dN) : (uint32_t)(pr / m.N);
    const uint32_t c1 = (uint32_t)(pr - (uint64_t)c0 * m.N);
    uint32_t nlive = 0, nA0 = 0, nC3 = 0;  // accesses per reference; A0 case 0; C3 case 0
    for (uint32_t c2b = 0; c2b < m.N; c2b += 64) {
      const uint32_t c2 = c2b + lane;
      const uint64_t live = __ballot(c2 < m.N);
      const bool c2last = P2 ? (c2 & m.wmask) == m.wmask : fmod_(c2, m.dW) == Wm1;
      nlive += (uint32_t)__popcll(live);
      nA0 += (uint32_t)__popcll(__ballot(!c2last) & live);  // A0 -> A0(c2+1), same line
      nC3 += (uint32_t)__popcll(__ballot(c2 + 1 < m.N) & live);  // C3 -> C2(c2+1)
    }
    const bool c1last = (P2 ? (c1 & m.wmask) : fmod_(c1, m.dW)) == Wm1;
    const uint32_t p = P2 ? (c0 & m.csmask) : fmod_(c0, m.dCS);
    const bool row_next = c0 + 1 + (p + 1 == m.CS ? m.tcs : 0u) < m.N;
    bump(0, 1);                                           // C0 -> C1
    bump(3, 1);                                           // C1 -> C2(0)
    bump(6, nA0);                                         // A0, case 0
    bump(c1 + 1 < m.N ? 7 : 8, nlive - nA0);              // A0 at a line's last c2: next c1, or cold
    bump(!c1last ? 9 : (row_next ? 10 : 11), nlive);      // B0: next c1 / next owned row / cold
    bump(12, nlive);                                      // C2 -> C3
    bump(15, nC3);                                        // C3, case 0
    bump(!c1last ? 16 : 17, nlive - nC3);                 // C3 at c2 = N-1: next c1, or cold
  }
  if (lane < DBINS && acc) atomicAdd(&tot[lane], acc);
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g.trav[0], npairs * m.S);  // accesses traversed
  __syncthreads();
  tail_accumulate(tot, g);
}

// --------------------------------------------------------------- export --
// Fold main table + replicas, sort by key, write `cap` (key,count) pairs;
// unused pairs are (~0, 0) so tables compare and merge canonically.
constexpr int EXP_THREADS = 1024;
__global__ __launch_bounds__(EXP_THREADS) void k_export(Model m, GTable g, unsigned long long* ok,
                                                       unsigned long long* oc, uint64_t cap, unsigned int* nout,
                                                       int consume) {
  __shared__ unsigned long long sk[GCAP];
  __shared__ unsigned long long sc[GCAP];
  __shared__ unsigned long long ck[GCAP];
  __shared__ unsigned int cnt;
  __shared__ unsigned int full;
  for (uint32_t i = threadIdx.x; i < GCAP; i += EXP_THREADS) {
    sk[i] = KEY_NONE;
    sc[i] = 0;
  }
  if (threadIdx.x == 0) cnt = full = 0;
  __syncthreads();
  // Replicas always; the main table only if a spill reached it (flags[3]).
  // All of a thread's key and count loads are issued before any is used.
  constexpr uint32_t RSLOTS = NREP * RCAP, RPER = RSLOTS / EXP_THREADS, MPER = GCAP / EXP_THREADS;
  static_assert(RSLOTS % EXP_THREADS == 0 && GCAP % EXP_THREADS == 0, "slot counts must divide evenly");
  const bool main_used = __hip_atomic_load(&g.flags[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  {
    unsigned long long kk[RPER], cc[RPER];
#pragma unroll
    for (uint32_t j = 0; j < RPER; ++j) {
      kk[j] = g.rkeys[j * EXP_THREADS + threadIdx.x];
      cc[j] = g.rcounts[j * EXP_THREADS + threadIdx.x];
    }
#pragma unroll
    for (uint32_t j = 0; j < RPER; ++j)
      if (kk[j] != KEY_NONE && !lds_add<unsigned long long, GCAP>(sk, sc, kk[j], cc[j])) atomicOr(&full, 1u);
    if (consume) {  // export-and-reset: clear what this thread has read
#pragma unroll
      for (uint32_t j = 0; j < RPER; ++j) {
        g.rkeys[j * EXP_THREADS + threadIdx.x] = KEY_NONE;
        g.rcounts[j * EXP_THREADS + threadIdx.x] = 0;
      }
    }
  }
  if (main_used) {
    unsigned long long kk[MPER], cc[MPER];
#pragma unroll
    for (uint32_t j = 0; j < MPER; ++j) {
      kk[j] = g.keys[j * EXP_THREADS + threadIdx.x];
      cc[j] = g.counts[j * EXP_THREADS + threadIdx.x];
    }
#pragma unroll
    for (uint32_t j = 0; j < MPER; ++j)
      if (kk[j] != KEY_NONE && !lds_add<unsigned long long, GCAP>(sk, sc, kk[j], cc[j])) atomicOr(&full, 1u);
    if (consume) {
#pragma unroll
      for (uint32_t j = 0; j < MPER; ++j) {
        g.keys[j * EXP_THREADS + threadIdx.x] = KEY_NONE;
        g.counts[j * EXP_THREADS + threadIdx.x] = 0;
      }
    }
  }
  for (uint32_t i = threadIdx.x; i < NBROW * BSTRIDE; i += EXP_THREADS) {  // direct (ref, case) bins
    const uint32_t b = i % BSTRIDE;
    const unsigned long long c = b < 18 ? g.bins[i] : 0ull;
    if (c && !lds_add<unsigned long long, GCAP>(sk, sc, m.keytab[b], c)) atomicOr(&full, 1u);
    if (consume && c) g.bins[i] = 0;
  }
  if (consume && threadIdx.x < 8) g.trav[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < GCAP; i += EXP_THREADS) {
    if (sk[i] != KEY_NONE) {
      const unsigned int p = atomicAdd(&cnt, 1u);
      ck[p] = sk[i];
    }
  }
  __syncthreads();
  const uint32_t n = cnt;
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t i = n + threadIdx.x; i < P; i += EXP_THREADS) ck[i] = KEY_EMPTY;
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {  // bitonic sort of the distinct keys
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += EXP_THREADS) {
        const uint32_t ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const unsigned long long a = ck[i], b = ck[ixj];
          if ((a > b) == up) {
            ck[i] = b;
            ck[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint64_t i = threadIdx.x; i < cap; i += EXP_THREADS) {
    if (i < n) {  // counts follow their keys: look each sorted key up in the LDS table
      const unsigned long long key = ck[i];
      uint32_t s = slot_hash(key, GCAP);
      while (sk[s] != key) s = (s + 1) & (GCAP - 1);
      ok[i] = key;
      oc[i] = sc[s];
    } else {
      ok[i] = KEY_EMPTY;
      oc[i] = 0ull;
    }
  }
  if (threadIdx.x == 0) {
    *nout = n;
    if (n > cap || full) atomicOr(&g.flags[0], 2u);
    if (consume) g.flags[3] = 0;  // every thread read it before the first __syncthreads
  }
}

// ------------------------------------------------------------- RI dump --
template <bool FAST>
__global__ __launch_bounds__(BLOCK) void k_ri_dump(Model m, const uint64_t* __restrict__ smp, uint64_t n,
                                                   int64_t* __restrict__ ri_out, uint64_t* __restrict__ sink_out,
                                                   GTable g) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    const Sample s = unpack(smp[i]);
    if (s.ref > 5 || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N) {
      atomicOr(&g.flags[1], 1u);
      ri_out[i] = -2;
      if (sink_out) sink_out[i] = KEY_EMPTY;
      continue;
    }
    const int64_t ri = ri_of<FAST>(m, s.ref, s.c0, s.c1, s.c2);
    ri_out[i] = ri;
    if (sink_out) {
      uint64_t P;
      uint32_t t;
      position(m, s.ref, s.c0, s.c1, s.c2, &P, &t);
      sink_out[i] = ri < 0 ? KEY_EMPTY : ((P + (uint64_t)ri) * m.T + t);
    }
  }
}

// -------------------------------------------------------------- expand --
__global__ __launch_bounds__(BLOCK) void k_expand(Perm p, uint32_t ref, uint64_t first, uint64_t n,
                                                  uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    out[i] = perm_sample(p, ref, perm_apply(p, first + i));
  }
}

// ---------------------------------------------------- key-order lists --
// Samples [first, first + n) of a reference's key-order stratified list
// (pluss_model.h KeyGen).  Each thread generates a run of ER
// consecutive samples incrementally (keyrun_*) into LDS; the block then
// stores them coalesced.
constexpr uint32_t ER = 8;
__device__ __forceinline__ uint32_t er_slot(uint32_t e) { return e + e / ER; }
__global__ __launch_bounds__(BLOCK) void k_expand_sorted(KeyGen k, uint64_t first, uint64_t n,
                                                         uint64_t* __restrict__ out) {
  __shared__ unsigned long long buf[BLOCK * ER + BLOCK];
  for (uint64_t base = (uint64_t)blockIdx.x * BLOCK * ER; base < n; base += (uint64_t)gridDim.x * BLOCK * ER) {
    const uint64_t j0 = base + threadIdx.x * ER;
    if (j0 < n) {
      const uint32_t cnt = n - j0 < ER ? (uint32_t)(n - j0) : ER;
      if (keyrun_fast_ok(k, first + base, (uint64_t)BLOCK * ER)) {  // block-uniform
        KeyRunF run;
        keyrunf_start(k, run, first + j0);
#pragma unroll
        for (uint32_t x = 0; x < ER; ++x) {
          if (x < cnt) buf[er_slot(threadIdx.x * ER + x)] = keygen_pack(k, keyrunf_digits(k, run));
          keyrunf_next(k, run);
        }
      } else {
        for (uint32_t x = 0; x < cnt; ++x) buf[er_slot(threadIdx.x * ER + x)] = keygen_sample(k, first + j0 + x);
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t x = 0; x < ER; ++x) {
      const uint32_t e = x * BLOCK + threadIdx.x;
      if (base + e < n) out[base + e] = buf[er_slot(e)];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ launchers --
static int grid_for(uint64_t work, uint64_t per_block, int max_blocks = MAX_BLOCKS) {
  uint64_t b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > (uint64_t)max_blocks) b = max_blocks;
  return (int)b;
}

int launch_table_reset(pluss_ctx* ctx, hipStream_t s) {
  PLUSS_HIP_CHECK(hipMemsetAsync(ctx->d_table, 0, TABLE_BYTES, s));
  ctx->tables_dirty = false;
  return PLUSS_OK;
}

// Workgroups of a dense pass (k_count, TAIL_DENSE, the bench step).  Lists
// past the Infinity Cache stream from HBM, where fewer resident waves per CU
// queue fewer requests on the same channels.  Measured on MI355X with
// tools/grid_sweep.py (profiles/r05_grid_sweep.jsonl, N=1024 lists, median
// of 5): 1024 workgroups at 2^24 samples (20.73 us; 768: 20.78); 768 at 2^25
// (39.23 us; 1024: 39.54, 640: 39.48) and 2^26 (75.7 us; 1024: 77.1); 640 at
// 2^27 (149.2 us; 768: 150.0) and 2^28 (296.2 us; 768: 299.1).  The other
// tails keep MAX_BLOCKS (not swept).
static int dense_grid_cap(uint64_t n) {
  return n >= (1ull << 27) ? 640 : n >= (1ull << 25) ? 768 : MAX_BLOCKS;
}

// `fuse` != null: FAST shapes only, the launch also exports and resets (the
// caller checked pluss_ctx::tables_dirty) or writes the dense vector; n may
// then be 0.  The shape alone picks the kernel.  diag (pluss_diag_dense
// only): ABL variant and a workgroup cap instead of the product's.
static int hot_launch(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, hipStream_t s, const ExportArgs* fuse,
                      const char* api, int abl = 0, int grid_cap = 0) {
  if (n == 0 && !fuse) return PLUSS_OK;
  if (((uintptr_t)d_samples & 7u) != 0) {
    set_error(std::string(api) + ": sample buffer must be 8-byte aligned");
    return PLUSS_ERR_INPUT;
  }
  const uint64_t* head = d_samples;  // always dereferenceable; used only when has_head
  int has_head = 0;
  if (n && ((uintptr_t)d_samples & 15u) != 0) {  // peel one sample so the pairs are 16-byte aligned
    has_head = 1;
    ++d_samples;
    --n;
  }
  const Model& m = ctx->m;
  const ExportArgs none{nullptr, nullptr, 0, nullptr, nullptr, 0};
  const ExportArgs& ex = fuse ? *fuse : none;
  const int tail = fuse ? (fuse->dense ? TAIL_DENSE : TAIL_EXPORT) : TAIL_NONE;
  int cap = grid_cap > 0 ? grid_cap : (m.fast && tail == TAIL_DENSE ? dense_grid_cap(n) : MAX_BLOCKS);
  const int nb = grid_for((n >> 1) ? (n >> 1) : 1, (uint64_t)BLOCK * UNROLL, std::min(cap, 16384));
  const GTable& g = ctx->g;
  if (!m.fast) {
    ctx->tables_dirty = true;
    hipLaunchKernelGGL(k_sampled_hist, dim3(nb), dim3(BLOCK), 0, s, m, d_samples, n, head, has_head, g);
    PLUSS_HIP_CHECK(hipGetLastError());
    return PLUSS_OK;
  }
#define PLUSS_LAUNCH_COUNT(P2, NP2, TL, AB)                                                                        \
  hipLaunchKernelGGL((k_count<P2, NP2, TL, AB>), dim3(nb), dim3(BLOCK), 0, s, m, d_samples, n, head, has_head, g, ex)
#define PLUSS_LAUNCH_TAIL(P2, NP2)                                                        \
  do {                                                                                    \
    if (tail == TAIL_DENSE) PLUSS_LAUNCH_COUNT(P2, NP2, TAIL_DENSE, 0);                   \
    else if (tail == TAIL_EXPORT) PLUSS_LAUNCH_COUNT(P2, NP2, TAIL_EXPORT, 0);            \
    else PLUSS_LAUNCH_COUNT(P2, NP2, TAIL_NONE, 0);                                       \
  } while (0)
  if (abl) {  // diagnostics: every BASELINE shape is P2 && NP2
    if (!(m.p2 && m.np2)) {
      set_error(std::string(api) + ": the ablation variants need N, CLS/DS and chunk powers of two");
      return PLUSS_ERR_CONFIG;
    }
    if (abl == 1) PLUSS_LAUNCH_COUNT(true, true, TAIL_NONE, 1);
    else PLUSS_LAUNCH_COUNT(true, true, TAIL_NONE, 2);
  } else if (m.p2 && m.np2) {
    PLUSS_LAUNCH_TAIL(true, true);
  } else if (m.p2) {
    PLUSS_LAUNCH_TAIL(true, false);
  } else if (m.np2) {
    PLUSS_LAUNCH_TAIL(false, true);
  } else {
    PLUSS_LAUNCH_TAIL(false, false);
  }
#undef PLUSS_LAUNCH_TAIL
#undef PLUSS_LAUNCH_COUNT
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_sampled_hist(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, hipStream_t s) {
  return hot_launch(ctx, d_samples, n, s, nullptr, "pluss_dev_sampled_hist");
}

int launch_sampled_hist_export(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, unsigned long long* d_keys,
                               unsigned long long* d_counts, uint64_t cap, hipStream_t s) {
  if (ctx->m.fast && !ctx->tables_dirty) {
    const ExportArgs ex{d_keys, d_counts, cap, ctx->d_exp_n, nullptr, 0};
    return hot_launch(ctx, d_samples, n, s, &ex, "pluss_dev_sampled_hist_export");
  }
  if (int rc = hot_launch(ctx, d_samples, n, s, nullptr, "pluss_dev_sampled_hist_export")) return rc;
  return launch_export(ctx, d_keys, d_counts, cap, s, true);
}

static int dense_check(pluss_ctx* ctx, unsigned long long* d_counts, const char* api) {
  if (!ctx->m.fast) {
    set_error(std::string(api) + ": needs N % (cls/ds) == 0 (a dense (ref, case) histogram)");
    return PLUSS_ERR_CONFIG;
  }
  if (((uintptr_t)d_counts & 7u) != 0) {
    set_error(std::string(api) + ": counts buffer must be 8-byte aligned");
    return PLUSS_ERR_INPUT;
  }
  return PLUSS_OK;
}

int launch_sampled_hist_dense(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, unsigned long long* d_counts,
                              hipStream_t s) {
  if (int rc = dense_check(ctx, d_counts, "pluss_dev_sampled_hist_dense")) return rc;
  const ExportArgs ex{nullptr, nullptr, 0, nullptr, d_counts, DENSE_ROWS};
  return hot_launch(ctx, d_samples, n, s, &ex, "pluss_dev_sampled_hist_dense");
}

int launch_diag_dense(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, unsigned long long* d_counts,
                      int variant, int max_grid, hipStream_t s) {
  if (variant < 0 || variant > 2 || max_grid < 0) {
    set_error("pluss_diag_dense: variant must be 0, 1 or 2 and max_grid >= 0");
    return PLUSS_ERR_CONFIG;
  }
  if (int rc = dense_check(ctx, d_counts, "pluss_diag_dense")) return rc;
  const ExportArgs ex{nullptr, nullptr, 0, nullptr, d_counts, DENSE_ROWS};
  return hot_launch(ctx, d_samples, n, s, &ex, "pluss_diag_dense", variant, max_grid);
}

int launch_fulltrace(pluss_ctx* ctx, hipStream_t s) {
  const uint64_t npairs = (uint64_t)ctx->m.N * ctx->m.N;
  if (!ctx->m.fast) {
    ctx->tables_dirty = true;
    hipLaunchKernelGGL(k_fulltrace, dim3(grid_for(npairs, BLOCK / 64 * 8)), dim3(BLOCK), 0, s, ctx->m, ctx->g);
  } else {
    // the ballot kernel's waves are short dependency chains: 8 waves per SIMD (2048 workgroups) hide them
    const int nbc = grid_for(npairs, BLOCK / 64 * 8, 2048);
    if (ctx->m.p2)
      hipLaunchKernelGGL(k_fulltrace_count<true>, dim3(nbc), dim3(BLOCK), 0, s, ctx->m, ctx->g);
    else
      hipLaunchKernelGGL(k_fulltrace_count<false>, dim3(nbc), dim3(BLOCK), 0, s, ctx->m, ctx->g);
  }
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_ri_dump(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, int64_t* d_ri, uint64_t* d_sink,
                   hipStream_t s) {
  if (n == 0) return PLUSS_OK;
  const int nb = grid_for(n, BLOCK * 4);
  if (ctx->m.fast)
    hipLaunchKernelGGL(k_ri_dump<true>, dim3(nb), dim3(BLOCK), 0, s, ctx->m, d_samples, n, d_ri, d_sink, ctx->g);
  else
    hipLaunchKernelGGL(k_ri_dump<false>, dim3(nb), dim3(BLOCK), 0, s, ctx->m, d_samples, n, d_ri, d_sink, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_expand(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t first, uint64_t n, uint64_t* d_out,
                  hipStream_t s) {
  if (n == 0) return PLUSS_OK;
  const bool dim3_ = !(ref == C0 || ref == C1);
  const uint64_t span = ctx->cfg.range_full ? (uint64_t)ctx->cfg.n : (uint64_t)ctx->cfg.n - 1;
  if (span == 0) {
    set_error("pluss_expand_samples: empty index range (N=1 with range [0,N-2])");
    return PLUSS_ERR_CONFIG;
  }
  const Perm p = make_perm(seed, (uint32_t)ref, span, dim3_);
  if (first + n > p.D || first + n < first) {
    set_error("pluss_expand_samples: first+n exceeds the index domain of this reference");
    return PLUSS_ERR_CONFIG;
  }
  const int nb = grid_for(n, BLOCK * 4, 4096);
  hipLaunchKernelGGL(k_expand, dim3(nb), dim3(BLOCK), 0, s, p, (uint32_t)ref, first, n, d_out);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int keygen_check(const pluss_ctx* ctx, int32_t ref, uint64_t total, uint64_t first, uint64_t n, const char* api) {
  const pluss_cfg& c = ctx->cfg;
  if ((uint64_t)c.n % ((uint64_t)c.chunk * (uint64_t)c.threads) != 0) {
    set_error(std::string(api) + ": key-order lists need N % (chunk*threads) == 0");
    return PLUSS_ERR_CONFIG;
  }
  const uint64_t span = c.range_full ? (uint64_t)c.n : (uint64_t)c.n - 1;
  const uint64_t d = (ref == C0 || ref == C1) ? span * span : span * span * span;
  if (total < 1 || total > d || total >= (1ull << 32)) {
    set_error(std::string(api) + ": total must be in [1, min(span^d, 2^32 - 1)]");
    return PLUSS_ERR_CONFIG;
  }
  if (first > total || n > total - first) {
    set_error(std::string(api) + ": [first, first + n) exceeds the list");
    return PLUSS_ERR_CONFIG;
  }
  return PLUSS_OK;
}

KeyGen keygen_of(const pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total) {
  const pluss_cfg& c = ctx->cfg;
  return make_keygen((uint64_t)c.n, (uint64_t)c.threads, (uint64_t)c.chunk, c.range_full != 0, seed, (uint32_t)ref,
                     total);
}

int launch_expand_sorted(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first, uint64_t n,
                         uint64_t* d_out, hipStream_t s) {
  if (int rc = keygen_check(ctx, ref, total, first, n, "pluss_expand_sorted")) return rc;
  if (n == 0) return PLUSS_OK;
  const KeyGen k = keygen_of(ctx, seed, ref, total);
  hipLaunchKernelGGL(k_expand_sorted, dim3(grid_for(n, BLOCK * ER, 4096)), dim3(BLOCK), 0, s, k, first, n, d_out);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_gen_count_dense(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, const uint64_t* first,
                           const uint64_t* n, unsigned long long* d_counts, hipStream_t s) {
  if (int rc = dense_check(ctx, d_counts, "pluss_dev_gen_count_dense")) return rc;
  GenArgs ga;
  ga.wbeg[0] = 0;
  for (int r = 0; r < 6; ++r) {
    ga.first[r] = first[r];
    ga.n[r] = n[r];
    ga.k[r] = KeyGen{};
    if (n[r]) {
      if (int rc = keygen_check(ctx, r, totals[r], first[r], n[r], "pluss_dev_gen_count_dense")) return rc;
      ga.k[r] = keygen_of(ctx, seed, r, totals[r]);
    }
    ga.wbeg[r + 1] = ga.wbeg[r] + (n[r] + GR * 64 - 1) / (GR * 64);
  }
  const ExportArgs ex{nullptr, nullptr, 0, nullptr, d_counts, DENSE_ROWS};
  // ALU-bound: 8 waves per SIMD
  const int nb = grid_for(ga.wbeg[6] ? ga.wbeg[6] : 1, BLOCK / 64, 2048);
  hipLaunchKernelGGL(k_gen_count, dim3(nb), dim3(BLOCK), 0, s, ctx->m, ga, ctx->g, ex);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_export(pluss_ctx* ctx, unsigned long long* d_keys, unsigned long long* d_counts, uint64_t cap,
                  hipStream_t s, bool consume) {
  hipLaunchKernelGGL(k_export, dim3(1), dim3(EXP_THREADS), 0, s, ctx->m, ctx->g, d_keys, d_counts, cap,
                     ctx->d_exp_n, consume ? 1 : 0);
  PLUSS_HIP_CHECK(hipGetLastError());
  if (consume) ctx->tables_dirty = false;
  return PLUSS_OK;
}

}  // namespace pluss
