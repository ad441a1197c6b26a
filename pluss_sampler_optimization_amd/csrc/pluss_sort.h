// pluss_sort.h — the radix source's sort, hand-written for CDNA: the six
// references' samples in any order (r10 draws them with rand() into a
// priority_queue, r10:151-185) -> their packed sort words (rank << 2 | case,
// pluss_faithful.h) in ascending order per reference, i.e. r10's pop order,
// all references in one launch sequence (full-chip grids; no per-reference
// streams).  Replaces a library LSD radix sort (five 8-bit scatter passes over
// 8-byte keys at N = 4096) by a two-level MSD bucket sort:
//
//   k_srt_count1    per chunk of SC samples: each sample's word and a
//                   histogram of its top digit (d1 bits, <= 256 buckets) in
//                   LDS; one column per chunk: hist1[ref block][digit][chunk];
//   scan            exclusive scan of hist1 over all references = the
//                   absolute start of each (digit, chunk) run;
//   k_srt_scatter1  per chunk: batches of SBATCH words counting-sorted by digit
//                   in LDS, written as runs (coalesced) to X1 -- as PAYLOADS:
//                   the word without its top digit (4 bytes whenever that
//                   fits: N <= 2^11 + ...; 8 otherwise);
//   k_srt_plan      one workgroup: per top-level bucket (parent) its range and
//                   the split of parents past SCAP by d2 more bits into
//                   level-2 chunks (their count and histogram offsets);
//   k_srt_count2,   the same count / scan / batched scatter for the parents'
//   scan,           level-2 chunks, X1 -> Y (payloads stay within their
//   k_srt_scatter2  parent's range);
//   k_srt_final     one workgroup per item (a parent left whole, or a child of
//                   a split one): payloads to LDS, counting-sorted by their
//                   leading undecided bits, ties insertion-sorted, written as
//                   words (the parent's digit put back) to OUT;
//   k_srt_deep      items past SCAP (skewed or duplicated input only): split
//                   again 8 bits at a time, depth first, inside one workgroup.
//
// Every payload moves between HBM arrays three times (X1, Y, OUT), with 4-byte
// payloads when they fit.  A malformed sample raises the input flag (its word
// is 0; a flagged pass is never read).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "pluss_device.h"

namespace pluss {

// Diagnostic builds only (-DPLUSS_DEBUG_STAGES): bounds checks on the sort's
// global accesses; a failing one is recorded (code, index, bound, block) in
// g_srt_dbg -- the first one, plus a count -- and its access skipped.  In the
// product build SRT_OK(...) is `true` and compiles away.
#ifdef PLUSS_DEBUG_STAGES
__device__ unsigned long long g_srt_dbg[12];
__device__ __forceinline__ bool srt_ok(bool ok, uint32_t code, uint64_t idx, uint64_t bound) {
  if (!ok) {
    atomicAdd(&g_srt_dbg[5], 1ull);
    if (atomicCAS(&g_srt_dbg[0], 0ull, (unsigned long long)code) == 0ull) {
      g_srt_dbg[1] = idx;
      g_srt_dbg[2] = bound;
      g_srt_dbg[3] = blockIdx.x | ((unsigned long long)blockIdx.y << 32);
      g_srt_dbg[4] = threadIdx.x;
    }
  }
  return ok;
}
#define SRT_OK(cond, code, idx, bound) ::pluss::srt_ok((cond), (code), (uint64_t)(idx), (uint64_t)(bound))
#else
#define SRT_OK(cond, code, idx, bound) true
#endif

constexpr int SB = 256;                   // threads per sort workgroup
constexpr int SE = 16;                    // words per thread per batch
constexpr uint32_t SBATCH = SB * SE;      // words per LDS batch
constexpr uint32_t SC = 4 * SBATCH;       // words per count/scatter chunk (both levels)
constexpr uint32_t SCAP = 4096;           // largest item sorted in LDS (k_srt_final)
constexpr int SDIG = 8;                   // largest digit of a split (256 children)
constexpr int SDEPTH = 10;                // k_srt_deep's levels (64-bit words, 8-bit digits, + the item)
constexpr uint32_t SSPLIT = 3072;         // a split parent's children average at most this many words
static_assert(SCAP == SBATCH, "an item is one batch");

// the references of one sort (a kernel argument)
struct SrtRefs {
  uint64_t n[6];
  uint64_t eoff[7];   // first element of each reference in the concatenated arrays
  uint64_t coff[7];   // first level-1 chunk of each reference; coff[6] = all chunks
  uint64_t hoff[7];   // first hist1 entry of each reference; hoff[6] = all entries
  uint32_t d1[6];     // top digit bits per reference (0: one bucket)
  const void* in[6];  // samples (SMP) or words (!SMP) of each reference
  uint32_t wb;        // word bits
  uint32_t np;        // parents = sum of 2^d1
  uint32_t tsh;       // log2(T) (P2 decodes)
};

// (SrtParent, a top-level bucket, is in pluss_device.h: the scan pipeline reads it too)

// an item past SCAP for k_srt_deep: payloads [start, start + count) of X1
// (buf 0) or Y (buf 1) of parent p, equal on every bit >= hi
struct SrtItem {
  uint32_t start, count, hi, bufp;  // bufp = p << 1 | buf
};
struct SrtDeep {
  SrtItem* items;
  unsigned int* head;
  uint32_t cap;
  unsigned int* flags;  // the handle's flags: FLAG_SORT when an item finds the list full
};

__host__ __device__ inline uint32_t srt_log2_ceil(uint64_t x) {
  uint32_t b = 0;
  while (b < 63 && (1ull << b) < x) ++b;
  return b;
}
// top-level digit bits of a reference of n words (buckets of about 2K words, at most 256)
__host__ __device__ inline uint32_t srt_d1(uint64_t n, uint32_t wb) {
  const uint32_t l = srt_log2_ceil(n);
  uint32_t d = l > 11 ? l - 11 : 0;
  d = d > (uint32_t)SDIG ? (uint32_t)SDIG : d;
  return d > wb ? wb : d;
}
// children of a parent past SCAP: a digit of d2 bits, children of SSPLIT / 2 to
// SSPLIT words on average (uniform input: a few sd of ~50 around it, far below
// SCAP; k_srt_final's batches are mostly full and level 2 writes longer runs)
__host__ __device__ inline uint32_t srt_split_bits(uint32_t cnt, uint32_t hi) {
  uint32_t D = srt_log2_ceil((cnt + SSPLIT - 1) / SSPLIT);
  D = D < 1 ? 1 : (D > (uint32_t)SDIG ? (uint32_t)SDIG : D);
  return D > hi ? hi : D;
}
template <typename T>
__device__ __forceinline__ T srt_lowmask(uint32_t bits) {
  return bits >= 8 * sizeof(T) ? (T) ~(T)0 : (T)(((T)1 << bits) - 1);
}

// the reference a level-1 chunk belongs to (uniform)
__device__ __forceinline__ uint32_t srt_ref_of_chunk(const SrtRefs& a, uint64_t c) {
  uint32_t r = 0;
#pragma unroll
  for (int x = 1; x < 6; ++x) r += c >= a.coff[x] ? 1u : 0u;
  return __builtin_amdgcn_readfirstlane(r);
}
// per-reference fields copied out by selects on the (wave-uniform) reference:
// the kernel argument is never indexed dynamically -- a switch here was
// lowered to a private-memory copy of d1[] indexed by r, and no product
// kernel may request scratch
struct SrtOne {
  uint64_t n, eoff, c0, h0;
  uint32_t d1, nch;
  const void* in;
};
__device__ __forceinline__ SrtOne srt_one(const SrtRefs& a, uint32_t r) {
  SrtOne o{a.n[0], a.eoff[0], a.coff[0], a.hoff[0], a.d1[0], (uint32_t)(a.coff[1] - a.coff[0]), a.in[0]};
#pragma unroll
  for (uint32_t x = 1; x < 6; ++x) {
    const bool h = r == x;
    o.n = h ? a.n[x] : o.n;
    o.eoff = h ? a.eoff[x] : o.eoff;
    o.c0 = h ? a.coff[x] : o.c0;
    o.h0 = h ? a.hoff[x] : o.h0;
    o.d1 = h ? a.d1[x] : o.d1;
    o.nch = h ? (uint32_t)(a.coff[x + 1] - a.coff[x]) : o.nch;
    o.in = h ? a.in[x] : o.in;
  }
  return o;
}

// the raw input element: a caller's sample (SMP) or a word already made (!SMP)
template <typename KT, bool SMP>
using srt_raw_t = typename std::conditional<SMP, uint64_t, KT>::type;

// its word for reference REF (a malformed sample raises the input flag and
// becomes 0).  P2: CS, T and CLS/DS powers of two -- c0 -> (q, tid) by shifts.
template <typename KT, bool SMP, bool P2, uint32_t REF>
__device__ __forceinline__ KT srt_word(const Model& m, uint32_t tsh, srt_raw_t<KT, SMP> x, GTable g) {
  if constexpr (SMP) {
    const Sample s = unpack(x);
    if (s.ref != REF || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N) {
      atomicOr(&g.flags[1], 1u);
      return (KT)0;
    }
    const uint32_t c2 = (REF == C0 || REF == C1) ? 0u : s.c2;
    uint32_t t;
    uint64_t q;
    if constexpr (P2) {
      const uint32_t k = s.c0 >> m.csshift;
      t = k & (m.T - 1);
      q = ((uint64_t)(k >> tsh) << m.csshift) | (s.c0 & m.csmask);
    } else {
      const uint32_t k = fdiv(s.c0, m.dCS), p = s.c0 - k * m.CS;
      const uint32_t kt = fdiv(k, m.dT);
      t = k - kt * m.T;
      q = (uint64_t)kt * m.CS + p;
    }
    const uint64_t rank = ((q * m.N + s.c1) * m.N + c2) * m.T + t;
    return (KT)((rank << 2) | case_fast<P2>(m, REF, s.c0, s.c1, c2));
  } else {
    return x == (KT) ~(KT)0 ? (KT)0 : x;  // the key pass's malformed marker (already flagged)
  }
}
// one batch of SE words per thread: every load issued before the first word is made
template <typename KT, bool SMP, bool P2, uint32_t REF>
__device__ __forceinline__ void srt_load_words(const Model& m, uint32_t tsh, const void* in, uint64_t b, uint64_t e1,
                                               KT (&w)[SE], GTable g) {
  const srt_raw_t<KT, SMP>* src = static_cast<const srt_raw_t<KT, SMP>*>(in);
  srt_raw_t<KT, SMP> x[SE];
  const uint64_t last = e1 - 1;
#pragma unroll
  for (int k = 0; k < SE; ++k) {
    const uint64_t i = b + (uint64_t)k * SB + threadIdx.x;
    x[k] = __builtin_nontemporal_load(src + (i < last ? i : last));
  }
#pragma unroll
  for (int k = 0; k < SE; ++k) w[k] = srt_word<KT, SMP, P2, REF>(m, tsh, x[k], g);
}
#define PLUSS_SRT_REFS(BODY)       \
  switch (r) {                     \
    case C0: { BODY(C0); } break;  \
    case C1: { BODY(C1); } break;  \
    case A0: { BODY(A0); } break;  \
    case B0: { BODY(B0); } break;  \
    case C2: { BODY(C2); } break;  \
    default: { BODY(C3); } break;  \
  }

template <typename T>
__device__ __forceinline__ uint32_t srt_dig(T w, uint32_t lo, uint32_t mask) {
  return lo >= 8 * sizeof(T) ? 0u : (uint32_t)(w >> lo) & mask;
}

// exclusive scan of v[0, len) in LDS (len <= SB * 16), all SB threads; returns the total
__device__ __forceinline__ uint32_t srt_block_scan(uint32_t* v, uint32_t len, uint32_t* wsum) {
  const uint32_t per = (len + SB - 1) / SB;  // <= 16
  const uint32_t b = threadIdx.x * per;
  uint32_t loc[16], s = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    loc[k] = (k < per && b + k < len) ? v[b + k] : 0u;
    s += loc[k];
  }
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int x = 0; x < SB / 64; ++x) {
    pre += x < (int)wid ? wsum[x] : 0u;
    tot += wsum[x];
  }
  uint32_t run = pre + inc - s;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    if (k < per && b + k < len) v[b + k] = run;
    run += loc[k];
  }
  __syncthreads();
  return tot;
}

// ---- exclusive scan of a u32 array in place (three launches): block sums of
// SBATCH entries, their scan (one workgroup), the blocks rescanned with their
// prefix.  len: the host's bound; *dlen (if given): the entries in use.
__global__ __launch_bounds__(SB) void k_scan_sums(const uint32_t* __restrict__ v, uint64_t len,
                                                 const uint32_t* dlen, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t wsum[SB / 64];
  const uint64_t L = dlen ? (*dlen < len ? *dlen : len) : len;
  const uint64_t b = (uint64_t)blockIdx.x * SBATCH;
  uint32_t s = 0;
  if (b < L)
    for (uint32_t i = threadIdx.x; i < SBATCH && b + i < L; i += SB) s += v[b + i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (__lane_id() == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}
__global__ __launch_bounds__(SB) void k_scan_top(uint32_t* __restrict__ bsum, uint32_t nb) {
  __shared__ uint32_t v[SBATCH], wsum[SB / 64];
  uint32_t carry = 0;
  for (uint32_t b = 0; b < nb; b += SBATCH) {
    const uint32_t m = nb - b < SBATCH ? nb - b : SBATCH;
    for (uint32_t i = threadIdx.x; i < m; i += SB) v[i] = bsum[b + i];
    __syncthreads();
    const uint32_t tot = srt_block_scan(v, m, wsum);
    for (uint32_t i = threadIdx.x; i < m; i += SB) bsum[b + i] = v[i] + carry;
    carry += tot;
    __syncthreads();
  }
}
__global__ __launch_bounds__(SB) void k_scan_apply(uint32_t* __restrict__ v, uint64_t len, const uint32_t* dlen,
                                                  const uint32_t* __restrict__ bsum) {
  __shared__ uint32_t t[SBATCH], wsum[SB / 64];
  const uint64_t L = dlen ? (*dlen < len ? *dlen : len) : len;
  const uint64_t b = (uint64_t)blockIdx.x * SBATCH;
  if (b >= L) return;
  const uint32_t m = L - b < SBATCH ? (uint32_t)(L - b) : SBATCH;
  for (uint32_t i = threadIdx.x; i < m; i += SB) t[i] = v[b + i];
  __syncthreads();
  srt_block_scan(t, m, wsum);
  const uint32_t c = bsum[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < m; i += SB) v[b + i] = t[i] + c;
}

// One batch of up to SBATCH values (w[k] valid iff vmask bit k) counting-sorted
// by digit in LDS and written as runs: a value of digit d -> dst[cur[d] + its
// rank among the batch's values of digit d]; cur[d] advanced.  put(x): the
// value stored for x (the payload).
template <typename T, typename OT, class PUT>
__device__ __forceinline__ void srt_batch(const T (&w)[SE], uint32_t vmask, uint32_t lo, uint32_t mask, T* stage,
                                          uint32_t* bcnt, uint32_t* bst, uint32_t* cur, uint32_t* wsum,
                                          OT* __restrict__ dst, PUT&& put) {
  bcnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t r[SE];
#pragma unroll
  for (int k = 0; k < SE; ++k) r[k] = (vmask >> k) & 1u ? atomicAdd(&bcnt[srt_dig(w[k], lo, mask)], 1u) : 0u;
  __syncthreads();
  bst[threadIdx.x] = bcnt[threadIdx.x];
  __syncthreads();
  const uint32_t m = srt_block_scan(bst, SB, wsum);
#pragma unroll
  for (int k = 0; k < SE; ++k)
    if ((vmask >> k) & 1u) stage[bst[srt_dig(w[k], lo, mask)] + r[k]] = w[k];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += SB) {
    const T x = stage[i];
    const uint32_t d = srt_dig(x, lo, mask);
    dst[cur[d] + (i - bst[d])] = put(x);
  }
  __syncthreads();
  cur[threadIdx.x] += bcnt[threadIdx.x];
  __syncthreads();
}

// ---- level 1 ---------------------------------------------------------------
template <typename KT, bool SMP, bool P2>
__global__ __launch_bounds__(SB) void k_srt_count1(Model m, SrtRefs a, uint32_t* __restrict__ hist, GTable g,
                                                  const uint32_t* gate) {
  __shared__ uint32_t cnt[SB];
  if (gate && !*gate) return;  // (the count-free level 1 placed every payload)
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t r = srt_ref_of_chunk(a, blockIdx.x);
  const SrtOne o = srt_one(a, r);
  const uint64_t c = blockIdx.x - o.c0;
  const uint64_t e0 = c * SC, e1 = o.n - e0 < SC ? o.n : e0 + SC;
  const uint32_t lo = a.wb - o.d1, mask = (1u << o.d1) - 1;
#define PLUSS_SRT_COUNT1(R)                                                                  \
  for (uint64_t b = e0; b < e1; b += SBATCH) {                                               \
    KT w[SE];                                                                                \
    srt_load_words<KT, SMP, P2, R>(m, a.tsh, o.in, b, e1, w, g);                                        \
    _Pragma("unroll") for (int k = 0; k < SE; ++k) if (b + (uint64_t)k * SB + threadIdx.x < e1) \
        atomicAdd(&cnt[srt_dig(w[k], lo, mask)], 1u);                                        \
  }
  PLUSS_SRT_REFS(PLUSS_SRT_COUNT1)
#undef PLUSS_SRT_COUNT1
  __syncthreads();
  if (threadIdx.x <= mask) hist[o.h0 + (uint64_t)threadIdx.x * o.nch + c] = cnt[threadIdx.x];
}

template <typename KT, typename PT, bool SMP, bool P2>
__global__ __launch_bounds__(SB) void k_srt_scatter1(Model m, SrtRefs a, const uint32_t* __restrict__ hist,
                                                    PT* __restrict__ X1, GTable g, const uint32_t* gate) {
  __shared__ KT stage[SBATCH];
  __shared__ uint32_t bcnt[SB], bst[SB], cur[SB], wsum[SB / 64];
  if (gate && !*gate) return;
  const uint32_t r = srt_ref_of_chunk(a, blockIdx.x);
  const SrtOne o = srt_one(a, r);
  const uint64_t c = blockIdx.x - o.c0;
  const uint64_t e0 = c * SC, e1 = o.n - e0 < SC ? o.n : e0 + SC;
  const uint32_t lo = a.wb - o.d1, mask = (1u << o.d1) - 1;
  cur[threadIdx.x] = threadIdx.x <= mask ? hist[o.h0 + (uint64_t)threadIdx.x * o.nch + c] : 0u;
  const KT pm = srt_lowmask<KT>(lo);
  auto put = [&](KT x) { return (PT)(x & pm); };
#define PLUSS_SRT_SCATTER1(R)                                                \
  for (uint64_t b = e0; b < e1; b += SBATCH) {                               \
    KT w[SE];                                                                \
    uint32_t vm = 0;                                                         \
    srt_load_words<KT, SMP, P2, R>(m, a.tsh, o.in, b, e1, w, g);                        \
    _Pragma("unroll") for (int k = 0; k < SE; ++k)                           \
      vm |= (b + (uint64_t)k * SB + threadIdx.x < e1 ? 1u : 0u) << k;        \
    srt_batch<KT, PT>(w, vm, lo, mask, stage, bcnt, bst, cur, wsum, X1, put); \
  }
  PLUSS_SRT_REFS(PLUSS_SRT_SCATTER1)
#undef PLUSS_SRT_SCATTER1
}

// ---- level 1 without a count pass (uniform-like input; 4-byte payloads):
// each top-level bucket gets a region of X1 sized for its share of the word
// range plus a margin (k_srt_caps), and each chunk of SC1 = 16K samples
// reserves its runs there with one atomic per bucket (k_srt_scatter1f).  A
// run that does not fit raises *ovf and is not written; the counted kernels
// above then run after all (gated on *ovf) and redo level 1 exactly.
constexpr int SB1 = 512;                       // threads of k_srt_scatter1f (41 KB of LDS: 3 per CU)
constexpr uint32_t SC1 = SB1 * SE;             // samples per workgroup
constexpr uint32_t SPL = SC / SC1;             // workgroups per counted chunk (chunks never span references)
static_assert(SC % SC1 == 0, "the count-free scatter splits the counted path's chunks");

// capacity of bucket b of reference r: its share of the words [0, wmax) plus margin
__device__ __forceinline__ uint32_t srt_cap(const SrtRefs& a, uint32_t r, uint32_t b, uint64_t wmax) {
  const uint64_t n = a.n[r];
  if (a.d1[r] == 0) return (uint32_t)n;
  const uint32_t lo = a.wb - a.d1[r];
  const uint64_t b0 = (uint64_t)b << lo, b1 = (uint64_t)(b + 1) << lo;
  const uint64_t w = b0 >= wmax ? 0 : (b1 < wmax ? b1 : wmax) - b0;
  const double e = (double)n * ((double)w / (double)wmax);
  const double c = e * 1.125 + 8.0 * sqrt(e) + 256.0;
  return c >= (double)n ? (uint32_t)n : (uint32_t)c;
}

// one workgroup: every bucket's capacity and region start (off1), fills zeroed;
// a plan larger than X1 (x1cap payloads) raises *ovf at once
__global__ __launch_bounds__(SB) void k_srt_caps(SrtRefs a, uint64_t wmax, uint32_t x1cap, uint32_t* __restrict__ cap,
                                                uint32_t* __restrict__ off1, uint32_t* __restrict__ fill,
                                                uint32_t* __restrict__ ovf) {
  __shared__ uint32_t v[SBATCH], wsum[SB / 64];
  const uint32_t np = a.np;
  for (uint32_t p = threadIdx.x; p < np; p += SB) {
    uint32_t r = 0, base = 0;
    while (r < 5 && p >= base + (1u << a.d1[r])) {
      base += 1u << a.d1[r];
      ++r;
    }
    v[p] = srt_cap(a, r, p - base, wmax);
    cap[p] = v[p];
    fill[p] = 0;
  }
  __syncthreads();
  const uint32_t tot = srt_block_scan(v, np, wsum);
  for (uint32_t p = threadIdx.x; p < np; p += SB) off1[p] = v[p];
  if (threadIdx.x == 0) *ovf = tot > x1cap ? 1u : 0u;
}

// the gates of the counted level 1 (after the count-free one): gate = *ovf,
// glen = the hist1 entries its scan covers (none when the gate is shut)
__global__ void k_srt_gate(const uint32_t* __restrict__ ovf, uint32_t h1, uint32_t* __restrict__ gate,
                           uint32_t* __restrict__ glen) {
  const uint32_t o = *ovf ? 1u : 0u;
  gate[0] = o;
  glen[0] = o ? h1 : 0u;
}

// level 2's gates: gate = *ovf, glen = the hist2 entries in use (*h2used) or none
__global__ void k_srt_gate2(const uint32_t* __restrict__ ovf, const uint32_t* __restrict__ h2used,
                            uint32_t* __restrict__ gate, uint32_t* __restrict__ glen) {
  const uint32_t o = *ovf ? 1u : 0u;
  gate[0] = o;
  glen[0] = o ? *h2used : 0u;
}

template <typename KT, bool SMP, bool P2>
__global__ __launch_bounds__(SB1) void k_srt_scatter1f(Model m, SrtRefs a, const uint32_t* __restrict__ cap,
                                                      const uint32_t* __restrict__ off1, uint32_t* __restrict__ fill,
                                                      uint32_t* __restrict__ ovf, uint32_t* __restrict__ X1, GTable g) {
  __shared__ uint32_t stage[SC1];
  __shared__ uint8_t sdig[SC1];
  __shared__ uint32_t bcnt[SB], bst[SB], bbase[SB], wsum[SB / 64], s_of;
  // (the plan did not fit, or another workgroup's run did not: the counted
  // path runs.  Read once for the workgroup: *ovf may be raised while this
  // workgroup starts, and waves that saw different values -- some returning,
  // some going on without their bucket counters zeroed -- wrote runs at
  // garbage offsets)
  if (threadIdx.x == 0) s_of = *ovf;
#ifdef PLUSS_DEBUG_STAGES
  {  // (diagnostic: would the waves, each reading *ovf itself as before, have disagreed?)
    __shared__ uint32_t s_wv[SB1 / 64];
    const uint32_t v = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)ovf);
    if (__lane_id() == 0) s_wv[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t any = 0, all = 1;
      for (int x = 0; x < SB1 / 64; ++x) {
        any |= s_wv[x];
        all &= s_wv[x] ? 1u : 0u;
      }
      if (any && !all) atomicAdd(&g_srt_dbg[8], 1ull);  // waves of one workgroup saw different flags
    }
  }
#endif
  __syncthreads();
  if (s_of) return;
  const uint32_t r = srt_ref_of_chunk(a, blockIdx.x / SPL);
  const SrtOne o = srt_one(a, r);
  const uint64_t c = blockIdx.x - o.c0 * SPL;
  const uint64_t e0 = c * SC1;
  if (e0 >= o.n) return;  // (the last counted chunk's unused part)
  const uint64_t e1 = o.n - e0 < SC1 ? o.n : e0 + SC1;
  const uint32_t lo = a.wb - o.d1, mask = (1u << o.d1) - 1;
  uint32_t pbase = 0;  // the first parent of reference r
#pragma unroll
  for (int x = 0; x < 5; ++x) pbase += (uint32_t)x < r ? (1u << a.d1[x]) : 0u;
  if (threadIdx.x < SB) bcnt[threadIdx.x] = 0;
  __syncthreads();
  KT w[SE];
  uint32_t rk[SE];
#define PLUSS_SRT_LOAD1F(R)                                                                         \
  {                                                                                                 \
    const srt_raw_t<KT, SMP>* src = static_cast<const srt_raw_t<KT, SMP>*>(o.in);                   \
    srt_raw_t<KT, SMP> x[SE];                                                                       \
    _Pragma("unroll") for (int k = 0; k < SE; ++k) {                                                \
      const uint64_t i = e0 + (uint64_t)k * SB1 + threadIdx.x;                                      \
      x[k] = __builtin_nontemporal_load(src + (i < e1 ? i : e1 - 1));                               \
    }                                                                                               \
    _Pragma("unroll") for (int k = 0; k < SE; ++k) w[k] = srt_word<KT, SMP, P2, R>(m, a.tsh, x[k], g); \
  }
  PLUSS_SRT_REFS(PLUSS_SRT_LOAD1F)
#undef PLUSS_SRT_LOAD1F
#pragma unroll
  for (int k = 0; k < SE; ++k) {
    const uint64_t i = e0 + (uint64_t)k * SB1 + threadIdx.x;
    rk[k] = i < e1 ? atomicAdd(&bcnt[srt_dig(w[k], lo, mask)], 1u) : 0u;
  }
  __syncthreads();
  if (threadIdx.x < SB) {  // this chunk's run in each bucket's region
    const uint32_t d = threadIdx.x, n = bcnt[d];
    uint32_t at = 0;
    if (d <= mask && n) {
      const uint32_t p = pbase + d;
      at = atomicAdd(&fill[p], n);
      if (at + n > cap[p]) {
#ifdef PLUSS_DEBUG_STAGES
        atomicAdd(&g_srt_dbg[6], 1ull);  // (level-1 overflows, counted)
#endif
        atomicOr(ovf, 1u);
        at = 0xFFFFFFFFu;
      } else {
        at += off1[p];
      }
    }
    bbase[d] = at;
    bst[d] = n;
  }
  __syncthreads();
  {
    // a block scan of SB entries by the first SB threads (waves 0..3, 64 each)
    const uint32_t t = threadIdx.x, lane = __lane_id(), wid = t >> 6;
    uint32_t v = t < SB ? bst[t] : 0u, inc = v;
#pragma unroll
    for (int s2 = 1; s2 < 64; s2 <<= 1) {
      const uint32_t y = __shfl_up(inc, s2, 64);
      if (lane >= (uint32_t)s2) inc += y;
    }
    if (t < SB && lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int x = 0; x < SB / 64; ++x) pre += x < (int)wid ? wsum[x] : 0u;
    if (t < SB) bst[t] = pre + inc - v;
  }
  __syncthreads();
  const uint32_t pmask = lo >= 32 ? 0xFFFFFFFFu : (1u << lo) - 1u;
#pragma unroll
  for (int k = 0; k < SE; ++k) {
    const uint64_t i = e0 + (uint64_t)k * SB1 + threadIdx.x;
    if (i < e1) {
      const uint32_t d = srt_dig(w[k], lo, mask), q = bst[d] + rk[k];
      stage[q] = (uint32_t)w[k] & pmask;
      sdig[q] = (uint8_t)d;
    }
  }
  __syncthreads();
  const uint32_t mt = (uint32_t)(e1 - e0);
  for (uint32_t i = threadIdx.x; i < mt; i += SB1) {
    const uint32_t d = sdig[i], at = bbase[d];
    if (at != 0xFFFFFFFFu && SRT_OK(at + (i - bst[d]) < 2 * a.eoff[6], 1, at + (i - bst[d]), 2 * a.eoff[6]))
      X1[at + (i - bst[d])] = stage[i];
  }
}

// ---- level 2 without a count pass (after a count-free level 1): each split
// parent's children get regions of Y sized like the level-1 buckets (capped
// at SCAP, so no child goes deep), each level-2 chunk reserves its runs with
// one atomic per child (k_srt_scatter2f), and k_srt_final takes the children
// from their regions, their places in the output from the fills.  A run that
// does not fit raises *ovf; the counted level 2 then runs (gated) and the
// final pass reads its layout instead.
struct SrtL2 {
  uint64_t wmax;     // the words' range [0, wmax)
  uint32_t ycap;     // Y's payloads
  uint32_t* fill;    // per child (parent's cb2 + digit): payloads placed
  uint32_t* ovf;     // a child's run did not fit, or the regions do not fit Y
  uint32_t* gate;    // = *ovf, for the counted level 2 (k_srt_gate)
  uint32_t* glen;    // the hist2 entries its scan covers (none when the gate is shut)
};
// a bound on the capacities of nc children sharing count payloads (whatever the
// shares: sum sqrt(e_d) <= sqrt(nc * count)), so a parent's region is O(1) to size
__device__ __forceinline__ uint32_t srt_cap2_sum(uint32_t count, uint32_t nc) {
  const double b = (double)count * 1.125 + 8.0 * sqrt((double)count * (double)nc) + 65.0 * (double)nc;
  return (uint32_t)b + 1u;
}
// capacity of child d of split parent P: its share of the parent's word range
__device__ __forceinline__ uint32_t srt_cap2(const SrtRefs& a, const SrtParent& P, uint32_t d, uint64_t wmax) {
  const uint32_t lo1 = a.wb - a.d1[P.ref], lo2 = lo1 - P.d2;
  const uint64_t p0 = lo1 >= 64 ? 0 : (uint64_t)P.b1 << lo1;
  const uint64_t p1 = lo1 >= 64 ? wmax : p0 + ((uint64_t)1 << lo1);
  const uint64_t c0 = p0 + ((uint64_t)d << lo2), c1 = c0 + ((uint64_t)1 << lo2);
  const uint64_t pw = (p1 < wmax ? p1 : wmax) - p0;
  const uint64_t cw = c0 >= wmax ? 0 : (c1 < wmax ? c1 : wmax) - c0;
  const double e = (double)P.count * ((double)cw / (double)pw);
  const double c = e * 1.125 + 8.0 * sqrt(e) + 64.0;
  return c >= (double)SCAP ? SCAP : (uint32_t)c;
}

template <typename PT>
__global__ __launch_bounds__(SB1) void k_srt_scatter2f(const SrtRefs a, const SrtParent* __restrict__ par,
                                                      const uint32_t* __restrict__ cmap,
                                                      const uint32_t* __restrict__ tot, const PT* __restrict__ X1,
                                                      PT* __restrict__ Y, const SrtL2 l2) {
  // (no digit array beside the stage: a staged payload holds its own digit,
  // so the LDS is 38 KB and four workgroups share a CU)
  __shared__ PT stage[SC1];
  __shared__ uint32_t bcnt[SB], bst[SB], bbase[SB], ccap[SB], coff[SB], wsum[SB / 64], s_of;
  const uint32_t q2 = blockIdx.x / SPL, half = blockIdx.x - q2 * SPL;
  // (the three reads issued together; cmap has a slot for every workgroup's q2)
  const uint32_t t0 = tot[0], pi = cmap[q2];
  if (q2 >= t0) return;
  // a level 1 or region overflow: the counted level 2 runs (*l2.ovf read once
  // for the workgroup: it may be raised by another workgroup meanwhile, see
  // k_srt_scatter1f)
  if (threadIdx.x == 0) s_of = *l2.ovf;
  __syncthreads();
  if (s_of) return;
  const SrtParent P = par[pi];
  const uint32_t k = q2 - P.cbase;
  const uint32_t c0 = k * SC + half * SC1;  // this workgroup's part of the parent's k-th chunk
  if (c0 >= P.count) return;
  const uint32_t e0 = P.src + c0, e1 = P.count - c0 < SC1 ? P.src + P.count : e0 + SC1;
  const uint32_t lo = a.wb - a.d1[P.ref] - P.d2, mask = (1u << P.d2) - 1;
  PT w[SE];  // (loaded first: the capacities and their scan run while the loads are in flight)
  uint32_t rk[SE];
#pragma unroll
  for (int j = 0; j < SE; ++j) {
    const uint32_t i = e0 + (uint32_t)j * SB1 + threadIdx.x;
    const uint32_t ii = i < e1 ? i : e1 - 1;
    w[j] = SRT_OK(ii < 2 * a.eoff[6], 3, ii, 2 * a.eoff[6]) ? __builtin_nontemporal_load(X1 + ii) : (PT)0;
  }
  if (threadIdx.x < SB) bcnt[threadIdx.x] = 0;
  if (threadIdx.x < SB) {  // the children's capacities; their region offsets below
    ccap[threadIdx.x] = threadIdx.x <= mask ? srt_cap2(a, P, threadIdx.x, l2.wmax) : 0u;
    coff[threadIdx.x] = ccap[threadIdx.x];
  }
  __syncthreads();
  {
    const uint32_t t = threadIdx.x, lane = __lane_id(), wid = t >> 6;
    const uint32_t v = t < SB ? coff[t] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int s2 = 1; s2 < 64; s2 <<= 1) {
      const uint32_t y = __shfl_up(inc, s2, 64);
      if (lane >= (uint32_t)s2) inc += y;
    }
    if (t < SB && lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int x = 0; x < SB / 64; ++x) pre += x < (int)wid ? wsum[x] : 0u;
    if (t < SB) coff[t] = pre + inc - v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SE; ++j) {
    const uint32_t i = e0 + (uint32_t)j * SB1 + threadIdx.x;
    rk[j] = i < e1 ? atomicAdd(&bcnt[srt_dig(w[j], lo, mask)], 1u) : 0u;
  }
  __syncthreads();
  // this part's run in each child's region: reserved now, placed after the
  // scan and the staging (the atomic's round trip overlaps them)
  const uint32_t d = threadIdx.x;
  uint32_t n = 0, at = 0;
  if (d < SB) {
    n = bcnt[d];
    if (d <= mask && n) at = atomicAdd(&l2.fill[P.cb2 + d], n);
    bst[d] = n;
  }
  __syncthreads();
  {
    const uint32_t t = threadIdx.x, lane = __lane_id(), wid = t >> 6;
    const uint32_t v = t < SB ? bst[t] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int s2 = 1; s2 < 64; s2 <<= 1) {
      const uint32_t y = __shfl_up(inc, s2, 64);
      if (lane >= (uint32_t)s2) inc += y;
    }
    if (t < SB && lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int x = 0; x < SB / 64; ++x) pre += x < (int)wid ? wsum[x] : 0u;
    if (t < SB) bst[t] = pre + inc - v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SE; ++j) {
    const uint32_t i = e0 + (uint32_t)j * SB1 + threadIdx.x;
    if (i < e1) {
      const uint32_t dj = srt_dig(w[j], lo, mask);
      stage[bst[dj] + rk[j]] = w[j];
    }
  }
  if (d < SB) {
    if (d <= mask && n) {
      if (at + n > ccap[d]) {
#ifdef PLUSS_DEBUG_STAGES
        atomicAdd(&g_srt_dbg[7], 1ull);  // (level-2 overflows, counted)
#endif
        atomicOr(l2.ovf, 1u);
        at = 0xFFFFFFFFu;
      } else {
        at += P.ybase + coff[d];
      }
    }
    bbase[d] = at;
  }
  __syncthreads();
  const uint32_t mt = e1 - e0;
  for (uint32_t i = threadIdx.x; i < mt; i += SB1) {
    const PT x = stage[i];
    const uint32_t d = srt_dig(x, lo, mask), at = bbase[d];
    if (at != 0xFFFFFFFFu && SRT_OK(at + (i - bst[d]) < l2.ycap, 2, at + (i - bst[d]), l2.ycap))
      Y[at + (i - bst[d])] = x;
  }
}

// ---- the plan: parents, their splits and level-2 chunks (one workgroup).
// tot[0] = level-2 chunks, tot[1] = hist2 entries.
// fill (the count-free level 1, unless *ovf): every parent's count is its
// fill, its payloads at off1 in X1, its place in the sorted order the
// exclusive sum of the fills before it.
__global__ __launch_bounds__(SB) void k_srt_plan(SrtRefs a, const uint32_t* __restrict__ hist,
                                                SrtParent* __restrict__ par, uint32_t* __restrict__ cmap,
                                                uint32_t* __restrict__ tot, const uint32_t* __restrict__ fill,
                                                const uint32_t* __restrict__ off1, const uint32_t* __restrict__ ovf,
                                                const SrtL2 l2) {
  __shared__ uint32_t v1[SBATCH], v2[SBATCH], wsum[SB / 64];
  const uint32_t np = a.np;  // <= 6 * 256
  const bool filled = fill && !*ovf;
  if (filled) {  // the parents' starts: the fills' exclusive sum (references in order, eoff[0] = 0)
    for (uint32_t p = threadIdx.x; p < np; p += SB) v1[p] = fill[p];
    __syncthreads();
    srt_block_scan(v1, np, wsum);
  }
  // parent p -> (reference, digit): references in order, 2^d1 parents each
  auto locate = [&](uint32_t p, uint32_t& r, uint32_t& b1) {
    r = 0;
    uint32_t base = 0;
    while (r < 5 && p >= base + (1u << a.d1[r])) {
      base += 1u << a.d1[r];
      ++r;
    }
    b1 = p - base;
  };
  // start of bucket b of reference r (a reference without chunks: every bucket empty at its offset)
  auto bstart = [&](uint32_t r, uint32_t b) -> uint32_t {
    const uint32_t nch = (uint32_t)(a.coff[r + 1] - a.coff[r]);
    return nch ? hist[a.hoff[r] + (uint64_t)b * nch] : (uint32_t)a.eoff[r];
  };
  // (each thread's parents p = threadIdx.x + k * SB stay in registers and go
  // out once at the end: re-reading them from memory between the scans was
  // most of this kernel's time)
  constexpr int PPT = (6 * 256 + SB - 1) / SB;
  SrtParent pp[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const uint32_t p = threadIdx.x + (uint32_t)k * SB;
    if (p >= np) continue;
    uint32_t r, b1;
    locate(p, r, b1);
    uint32_t s, cnt, src;
    if (filled) {
      s = v1[p];
      cnt = fill[p];
      src = off1[p];
    } else {
      s = bstart(r, b1);
      const uint32_t e = b1 + 1 < (1u << a.d1[r]) ? bstart(r, b1 + 1) : (uint32_t)a.eoff[r + 1];
      cnt = e - s;
      src = s;
    }
    const uint32_t hi = a.wb - a.d1[r];
    const uint32_t d2 = (cnt > SCAP && hi > 0) ? srt_split_bits(cnt, hi) : 0u;
    const uint32_t nc2 = d2 ? (cnt + SC - 1) / SC : 0u;
    pp[k] = SrtParent{s, cnt, r, b1, d2, nc2, 0, 0, src, 0, 0};
  }
  __syncthreads();  // (v1 free again)
  if (filled && l2.fill) {  // the count-free level 2's regions: per parent a bound on its children's capacities
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const uint32_t p = threadIdx.x + (uint32_t)k * SB;
      if (p >= np) continue;
      v1[p] = pp[k].d2 ? srt_cap2_sum(pp[k].count, 1u << pp[k].d2) : 0u;
      v2[p] = pp[k].d2 ? 1u << pp[k].d2 : 0u;
    }
    __syncthreads();
    const uint32_t ysum = srt_block_scan(v1, np, wsum);
    const uint32_t nchild = srt_block_scan(v2, np, wsum);
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const uint32_t p = threadIdx.x + (uint32_t)k * SB;
      if (p >= np) continue;
      pp[k].ybase = v1[p];
      pp[k].cb2 = v2[p];
    }
    for (uint32_t i = threadIdx.x; i < nchild; i += SB) l2.fill[i] = 0;
    if (threadIdx.x == 0) *l2.ovf = ysum > l2.ycap ? 1u : 0u;
    __syncthreads();
  } else if (l2.fill && threadIdx.x == 0) {
    *l2.ovf = 1u;  // (level 1 took the counted path: so does level 2)
  }
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const uint32_t p = threadIdx.x + (uint32_t)k * SB;
    if (p >= np) continue;
    v1[p] = pp[k].nc2;
    v2[p] = pp[k].nc2 << pp[k].d2;
  }
  __syncthreads();
  const uint32_t g2 = srt_block_scan(v1, np, wsum);
  const uint32_t h2 = srt_block_scan(v2, np, wsum);
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const uint32_t p = threadIdx.x + (uint32_t)k * SB;
    if (p >= np) continue;
    pp[k].cbase = v1[p];
    pp[k].h2off = v2[p];
    par[p] = pp[k];
    for (uint32_t j = 0; j < pp[k].nc2; ++j) cmap[v1[p] + j] = p;
  }
  if (threadIdx.x == 0) {
    tot[0] = g2;
    tot[1] = h2;
  }
}

// ---- level 2 (grid: the host's bound on level-2 chunks; tot[0] in use)
template <typename PT>
__global__ __launch_bounds__(SB) void k_srt_count2(const SrtRefs a, const SrtParent* __restrict__ par,
                                                  const uint32_t* __restrict__ cmap, const uint32_t* __restrict__ tot,
                                                  const PT* __restrict__ X1, uint32_t* __restrict__ hist2,
                                                  const uint32_t* gate) {
  __shared__ uint32_t cnt[SB];
  if (blockIdx.x >= tot[0] || (gate && !*gate)) return;
  const SrtParent P = par[cmap[blockIdx.x]];
  const uint32_t k = blockIdx.x - P.cbase;
  const uint32_t e0 = P.src + k * SC, e1 = P.count - k * SC < SC ? P.src + P.count : e0 + SC;
  const uint32_t lo = a.wb - a.d1[P.ref] - P.d2, mask = (1u << P.d2) - 1;
  cnt[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t b = e0; b < e1; b += SBATCH) {
    PT w[SE];
    const uint32_t last = e1 - 1;
#pragma unroll
    for (int j = 0; j < SE; ++j) {
      const uint32_t i = b + (uint32_t)j * SB + threadIdx.x;
      w[j] = X1[i < last ? i : last];
    }
#pragma unroll
    for (int j = 0; j < SE; ++j)
      if (b + (uint32_t)j * SB + threadIdx.x < e1) atomicAdd(&cnt[srt_dig(w[j], lo, mask)], 1u);
  }
  __syncthreads();
  if (threadIdx.x <= mask) hist2[P.h2off + threadIdx.x * P.nc2 + k] = cnt[threadIdx.x];
}

template <typename PT>
__global__ __launch_bounds__(SB) void k_srt_scatter2(const SrtRefs a, const SrtParent* __restrict__ par,
                                                    const uint32_t* __restrict__ cmap,
                                                    const uint32_t* __restrict__ tot, const uint32_t* __restrict__ hist2,
                                                    const PT* __restrict__ X1, PT* __restrict__ Y, const uint32_t* gate) {
  __shared__ PT stage[SBATCH];
  __shared__ uint32_t bcnt[SB], bst[SB], cur[SB], wsum[SB / 64];
  if (blockIdx.x >= tot[0] || (gate && !*gate)) return;
  const SrtParent P = par[cmap[blockIdx.x]];
  const uint32_t k = blockIdx.x - P.cbase;
  const uint32_t e0 = P.src + k * SC, e1 = P.count - k * SC < SC ? P.src + P.count : e0 + SC;
  const uint32_t lo = a.wb - a.d1[P.ref] - P.d2, mask = (1u << P.d2) - 1;
  const uint32_t base = hist2[P.h2off];
  cur[threadIdx.x] = threadIdx.x <= mask ? P.start + hist2[P.h2off + threadIdx.x * P.nc2 + k] - base : 0u;
  auto put = [](PT x) { return x; };
  for (uint32_t b = e0; b < e1; b += SBATCH) {
    PT w[SE];
    uint32_t vm = 0;
    const uint32_t last = e1 - 1;
#pragma unroll
    for (int j = 0; j < SE; ++j) {
      const uint32_t i = b + (uint32_t)j * SB + threadIdx.x;
      w[j] = X1[i < last ? i : last];
      vm |= (i < e1 ? 1u : 0u) << j;
    }
    srt_batch<PT, PT>(w, vm, lo, mask, stage, bcnt, bst, cur, wsum, Y, put);
  }
}

// Sort one item (count <= SCAP payloads of src[s, s + count), equal on every bit
// >= hi) in LDS and write it as words to OUT: counting sort by the leading D
// undecided bits, then an insertion sort of each run of equal leading bits
// (runs average below one payload).  bb: SCAP payloads; c: SCAP + 1 words.
template <typename PT, typename KT>
__device__ __forceinline__ void srt_sort_item(const PT* __restrict__ src, uint32_t s, uint32_t cnt, uint32_t hi,
                                              KT prefix, KT* __restrict__ OUT, PT* bb, uint32_t* c,
                                              uint32_t* wsum) {
  PT w[SE];
  const uint32_t last = cnt - 1;
#pragma unroll
  for (int k = 0; k < SE; ++k) {  // nt: past L1 (the deep pass reads back what this workgroup wrote)
    const uint32_t i = (uint32_t)k * SB + threadIdx.x;
    w[k] = __builtin_nontemporal_load(src + s + (i < last ? i : last));
  }
  if (hi == 0) {  // every payload equal
#pragma unroll
    for (int k = 0; k < SE; ++k) {
      const uint32_t i = (uint32_t)k * SB + threadIdx.x;
      if (i < cnt) OUT[s + i] = prefix | (KT)w[k];
    }
    return;
  }
  uint32_t D = srt_log2_ceil(cnt);
  D = D < 1 ? 1 : D;
  D = D > hi ? hi : D;
  const uint32_t nb = 1u << D, lo = hi - D, mask = nb - 1;
  for (uint32_t i = threadIdx.x; i < nb; i += SB) c[i] = 0;
  __syncthreads();
  uint32_t r[SE];
#pragma unroll
  for (int k = 0; k < SE; ++k) {
    const uint32_t i = (uint32_t)k * SB + threadIdx.x;
    r[k] = i < cnt ? atomicAdd(&c[srt_dig(w[k], lo, mask)], 1u) : 0u;
  }
  __syncthreads();
  srt_block_scan(c, nb, wsum);
  if (threadIdx.x == 0) c[nb] = cnt;
#pragma unroll
  for (int k = 0; k < SE; ++k) {
    const uint32_t i = (uint32_t)k * SB + threadIdx.x;
    if (i < cnt) bb[c[srt_dig(w[k], lo, mask)] + r[k]] = w[k];
  }
  __syncthreads();
  if (lo > 0) {  // runs of equal leading bits: insertion sort (one thread per run)
    for (uint32_t d = threadIdx.x; d < nb; d += SB) {
      const uint32_t b0 = c[d], e = c[d + 1];
      for (uint32_t i = b0 + 1; i < e; ++i) {
        const PT x = bb[i];
        uint32_t j = i;
        while (j > b0 && bb[j - 1] > x) {
          bb[j] = bb[j - 1];
          --j;
        }
        bb[j] = x;
      }
    }
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < cnt; i += SB) OUT[s + i] = prefix | (KT)bb[i];
}

template <typename KT>
__device__ __forceinline__ KT srt_prefix(const SrtRefs& a, const SrtParent& P) {
  const uint32_t hi = a.wb - a.d1[P.ref];
  return hi >= 8 * sizeof(KT) ? (KT)0 : (KT)((KT)P.b1 << hi);
}

// The final pass's workgroup barrier.  (An LDS-only barrier -- s_waitcnt
// lgkmcnt(0); s_barrier in inline asm, which would keep the next item's
// prefetched loads in flight -- misplaced a few words per 10^5 on gfx950 in
// tests/test_gpu_sort.py, intermittently; the full barrier never did.)
__device__ __forceinline__ void srt_lds_sync() { __syncthreads(); }

// srt_block_scan with the final pass's barrier and 16-byte reads
__device__ __forceinline__ void srt_block_scan_lds(uint32_t* v, uint32_t len, uint32_t* wsum) {
  const uint32_t per = (len + SB - 1) / SB;  // <= 16
  const uint32_t b = threadIdx.x * per;
  uint32_t loc[16], sum = 0;
  if ((len & (4 * SB - 1)) == 0) {  // len a multiple of 1024: 16-byte LDS reads (no bank conflicts)
#pragma unroll
    for (uint32_t k = 0; k < 16; k += 4) {
      const uint4 q = k < per ? *reinterpret_cast<const uint4*>(v + b + k) : make_uint4(0, 0, 0, 0);
      loc[k] = q.x;
      loc[k + 1] = q.y;
      loc[k + 2] = q.z;
      loc[k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) loc[k] = (k < per && b + k < len) ? v[b + k] : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) sum += loc[k];
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[wid] = inc;
  srt_lds_sync();
  uint32_t pre = 0;
#pragma unroll
  for (int x = 0; x < SB / 64; ++x) pre += x < (int)wid ? wsum[x] : 0u;
  uint32_t run = pre + inc - sum;
  if ((len & (4 * SB - 1)) == 0) {  // 16-byte writes too
#pragma unroll
    for (uint32_t k = 0; k < 16; k += 4) {
      uint4 q;
      q.x = run;
      q.y = q.x + loc[k];
      q.z = q.y + loc[k + 1];
      q.w = q.z + loc[k + 2];
      run = q.w + loc[k + 3];
      if (k < per) *reinterpret_cast<uint4*>(v + b + k) = q;
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      if (k < per && b + k < len) v[b + k] = run;
      run += loc[k];
    }
  }
  srt_lds_sync();
}

template <typename PT, int NSE>
__device__ __forceinline__ void srt_item_load(const PT* __restrict__ src, uint32_t s, uint32_t cnt, PT (&w)[NSE]) {
  const uint32_t last = cnt - 1;
#pragma unroll
  for (int k = 0; k < NSE; ++k) {
    const uint32_t i = (uint32_t)k * SB + threadIdx.x;
    w[k] = __builtin_nontemporal_load(src + s + (i < last ? i : last));
  }
}

// srt_sort_item on payloads already in registers, LDS-only barriers: a
// counting sort by the leading D undecided bits groups the payloads in bb;
// each payload's final place is its group's start plus the number of the
// group's payloads below it (ties: below it in bb), written to ob; then ob
// goes out in order.  Groups average at most one payload (D = log2(cnt)), so
// the count is a short loop in every lane (no per-thread insertion sort, which
// diverged).  bb, ob: SCAP payloads; c: SCAP + 1 words; all free on return.
template <typename PT, typename KT, int NSE>
__device__ __forceinline__ void srt_item_sort(const PT (&w)[NSE], uint32_t s, uint32_t cnt, uint32_t hi, KT prefix,
                                              KT* __restrict__ OUT, PT* bb, PT* ob, uint32_t* c, uint32_t* wsum) {
  if (hi == 0) {  // every payload equal
#pragma unroll
    for (int k = 0; k < NSE; ++k) {
      const uint32_t i = (uint32_t)k * SB + threadIdx.x;
      if (i < cnt) OUT[s + i] = prefix | (KT)w[k];
    }
    return;
  }
  uint32_t D = srt_log2_ceil(cnt);
  D = D < 10 ? 10 : D;  // (nb a multiple of 1024: the scan's 16-byte reads)
  D = D > hi ? hi : D;
  const uint32_t nb = 1u << D, lo = hi - D, mask = nb - 1;
  for (uint32_t i = threadIdx.x; i < nb; i += SB) c[i] = 0;
  srt_lds_sync();
  uint32_t r[NSE];
#pragma unroll
  for (int k = 0; k < NSE; ++k) {
    const uint32_t i = (uint32_t)k * SB + threadIdx.x;
    r[k] = i < cnt ? atomicAdd(&c[srt_dig(w[k], lo, mask)], 1u) : 0u;
  }
  if (threadIdx.x == 0) c[nb] = cnt;  // (the group end of the last digit; visible after the scan's barrier)
  srt_lds_sync();
  srt_block_scan_lds(c, nb, wsum);
  uint32_t g0[NSE], g1[NSE];
#pragma unroll
  for (int k = 0; k < NSE; ++k) {
    const uint32_t i = (uint32_t)k * SB + threadIdx.x;
    const uint32_t d = srt_dig(w[k], lo, mask);
    g0[k] = c[d];
    g1[k] = c[d + 1];
    if (i < cnt) bb[g0[k] + r[k]] = w[k];
  }
  srt_lds_sync();
  if (lo == 0) {  // equal digits are equal payloads: bb is sorted
    for (uint32_t i = threadIdx.x; i < cnt; i += SB) OUT[s + i] = prefix | (KT)bb[i];
    srt_lds_sync();
    return;
  }
#pragma unroll
  for (int k = 0; k < NSE; ++k) {
    const uint32_t i = (uint32_t)k * SB + threadIdx.x;
    if (i < cnt) {
      // (a group averages below two payloads: four straight-line reads per
      // payload instead of this loop were 1.4x slower, LDS-bound)
      const uint32_t p = g0[k] + r[k];
      uint32_t at = g0[k];
      for (uint32_t j = g0[k]; j < g1[k]; ++j) {
        const PT y = bb[j];
        at += (y < w[k] || (y == w[k] && j < p)) ? 1u : 0u;
      }
      ob[at] = w[k];
    }
  }
  srt_lds_sync();
  for (uint32_t i = threadIdx.x; i < cnt; i += SB) OUT[s + i] = prefix | (KT)ob[i];
  srt_lds_sync();
}

// ---- k_srt_final: grid (FG, parents).  A parent left whole is one item
// (workgroup 0); a split parent's children d = x, x + FG, ... go to workgroup
// x, each child's payloads loaded while the previous one is sorted.  Items
// past SCAP go to the deep list.
constexpr uint32_t FG = 4;
// (4 waves per SIMD asked: the payload-only instantiation was otherwise given
// 150 VGPRs and scratch, 3 waves, and ran 1.4x slower)
template <typename PT, typename KT, bool PFX = true>  // !PFX: the payloads alone (SRC_W32P)
__global__ __launch_bounds__(SB) __attribute__((amdgpu_waves_per_eu(sizeof(PT) == 4 ? 4 : 1))) void k_srt_final(const SrtRefs a, const SrtParent* __restrict__ par,
                                                 const uint32_t* __restrict__ hist2, const PT* __restrict__ X1,
                                                 const PT* __restrict__ Y, KT* __restrict__ OUT, SrtDeep dp,
                                                 const SrtL2 l2) {
  // ob, the ranked payloads, reuses the counters once each payload holds its
  // group bounds in registers (4-byte payloads; 8-byte ones get their own)
  constexpr bool OB_IN_C = sizeof(PT) == sizeof(uint32_t);
  __shared__ PT bb[SCAP + 4], obx[OB_IN_C ? 1 : SCAP];  // (bb: srt_item_sort's reads past a group's end)
  __shared__ uint32_t c[SCAP + 1], bnd[SB + 1], ysrc[SB], wsum[SB / 64];
  PT* ob = OB_IN_C ? reinterpret_cast<PT*>(c) : obx;
  const uint32_t p = blockIdx.y;
  const SrtParent P = par[p];
  const uint32_t hi1 = a.wb - a.d1[P.ref];
  const KT prefix = PFX ? srt_prefix<KT>(a, P) : (KT)0;
  auto deep = [&](uint32_t s, uint32_t cnt, uint32_t hi, uint32_t buf) {
    if (threadIdx.x == 0) {
      const unsigned int q = atomicAdd(dp.head, 1u);
      if (q < dp.cap) dp.items[q] = SrtItem{s, cnt, hi, p << 1 | buf};
      else atomicOr(&dp.flags[0], FLAG_SORT);  // never written past the list: the pass reports it instead
    }
  };
  // an item of cnt <= SCAP payloads in NSE registers per thread, the fewest
  // that hold it (the slots past cnt are predicated off but still issued)
  // (payloads read from src[rs, rs + cnt), written as words to OUT[s, s + cnt))
  // (always inlined: the payload-only instantiation otherwise made it a call, with scratch)
  auto item = [&](const PT* __restrict__ src, uint32_t rs, uint32_t s, uint32_t cnt, uint32_t hi)
                  __attribute__((always_inline)) {
    if (cnt <= 8 * SB) {
      PT w[8];
      srt_item_load<PT, 8>(src, rs, cnt, w);
      srt_item_sort<PT, KT, 8>(w, s, cnt, hi, prefix, OUT, bb, ob, c, wsum);
    } else if (cnt <= 12 * SB) {
      PT w[12];
      srt_item_load<PT, 12>(src, rs, cnt, w);
      srt_item_sort<PT, KT, 12>(w, s, cnt, hi, prefix, OUT, bb, ob, c, wsum);
    } else {
      PT w[SE];
      srt_item_load<PT, SE>(src, rs, cnt, w);
      srt_item_sort<PT, KT, SE>(w, s, cnt, hi, prefix, OUT, bb, ob, c, wsum);
    }
  };
  if (P.d2 == 0) {
    if (blockIdx.x != 0 || P.count == 0) return;
    if (P.count > SCAP) {
      deep(P.start, P.count, hi1, 0);
      return;
    }
    if (!SRT_OK((uint64_t)P.src + P.count <= 2 * a.eoff[6], 4, (uint64_t)P.src + P.count, 2 * a.eoff[6]) ||
        !SRT_OK((uint64_t)P.start + P.count <= a.eoff[6], 5, (uint64_t)P.start + P.count, a.eoff[6]))
      return;
    item(X1, P.src, P.start, P.count, hi1);
    return;
  }
  const uint32_t nc = 1u << P.d2, hi = hi1 - P.d2;
  const bool f2 = l2.fill && !*l2.ovf;  // the count-free level 2's layout
  if (f2) {  // children in their Y regions (capacities scanned), output places from the fills
    const uint32_t d = threadIdx.x;
    ysrc[d] = d < nc ? srt_cap2(a, P, d, l2.wmax) : 0u;
    bnd[d] = d < nc ? l2.fill[P.cb2 + d] : 0u;
    __syncthreads();
    srt_block_scan(ysrc, SB, wsum);
    srt_block_scan(bnd, SB, wsum);
    if (d < nc) {
      ysrc[d] += P.ybase;
      bnd[d] += P.start;
    }
    if (d == 0) bnd[nc] = P.start + P.count;
  } else {
    const uint32_t base = hist2[P.h2off];
    for (uint32_t i = threadIdx.x; i <= nc; i += SB)
      bnd[i] = i < nc ? P.start + hist2[P.h2off + i * P.nc2] - base : P.start + P.count;
  }
  __syncthreads();
  for (uint32_t d = blockIdx.x; d < nc; d += FG) {  // this workgroup's children
    const uint32_t s = bnd[d], cnt = bnd[d + 1] - s;
    if (cnt == 0) continue;
    if (cnt > SCAP) {  // (the counted layout only: a region holds at most SCAP)
      deep(s, cnt, hi, 1);
      continue;
    }
    if (!SRT_OK((uint64_t)(f2 ? ysrc[d] : s) + cnt <= l2.ycap, 6, (uint64_t)(f2 ? ysrc[d] : s) + cnt, l2.ycap) ||
        !SRT_OK((uint64_t)s + cnt <= a.eoff[6] && bnd[d + 1] >= s, 7, (uint64_t)s + cnt, a.eoff[6]))
      continue;
    item(Y, f2 ? ysrc[d] : s, s, cnt, hi);
  }
}

// ---- k_srt_deep: items past SCAP (skewed or duplicated words), split by
// 8-bit digits depth first inside one workgroup; a level's children alternate
// between Y and X1 at the same offsets; every item ends in OUT as words.
template <typename PT, typename KT, bool PFX = true>
__global__ __launch_bounds__(SB) void k_srt_deep(const SrtRefs a, const SrtParent* __restrict__ par,
                                                PT* __restrict__ X1, PT* __restrict__ Y, KT* __restrict__ OUT,
                                                SrtDeep dp) {
  __shared__ PT stage[SBATCH];  // also the final sort's payload buffer (SBATCH == SCAP)
  __shared__ uint32_t off[SDEPTH][SB + 1], c[SCAP + 1], bcnt[SB], bst[SB], cur[SB], wsum[SB / 64];
  __shared__ SrtItem lv[SDEPTH];
  __shared__ uint32_t nxt[SDEPTH], nchild[SDEPTH];
  const uint32_t nd = *dp.head < dp.cap ? *dp.head : dp.cap;
  auto put = [](PT x) { return x; };
  for (uint32_t q = blockIdx.x; q < nd; q += gridDim.x) {
    int top = 0;
    const SrtItem root = dp.items[q];
    const KT prefix = PFX ? srt_prefix<KT>(a, par[root.bufp >> 1]) : (KT)0;
    if (threadIdx.x == 0) {
      lv[0] = root;
      nxt[0] = 0xFFFFFFFFu;  // not split yet
    }
    __syncthreads();
    while (top >= 0) {
      const SrtItem it = lv[top];
      const uint32_t buf = it.bufp & 1u;
      const uint32_t D = it.hi < (uint32_t)SDIG ? it.hi : (uint32_t)SDIG;
      if (nxt[top] == 0xFFFFFFFFu) {  // first visit
        if (it.count <= SCAP || it.hi == 0) {
          if (it.count <= SCAP) {
            srt_sort_item<PT, KT>(buf ? Y : X1, it.start, it.count, it.hi, prefix, OUT, stage, c, wsum);
          } else {  // all equal
            const PT* src = buf ? Y : X1;
            for (uint32_t i = threadIdx.x; i < it.count; i += SB)
              OUT[it.start + i] = prefix | (KT)__builtin_nontemporal_load(src + it.start + i);
          }
          __syncthreads();
          --top;
          continue;
        }
        const uint32_t lo = it.hi - D, mask = (1u << D) - 1;
        const PT* src = buf ? Y : X1;
        PT* dst = buf ? X1 : Y;
        bcnt[threadIdx.x] = 0;
        __syncthreads();
        for (uint32_t b = 0; b < it.count; b += SBATCH) {  // histogram
#pragma unroll
          for (int k = 0; k < SE; ++k) {
            const uint32_t i = b + (uint32_t)k * SB + threadIdx.x;
            if (i < it.count) atomicAdd(&bcnt[srt_dig(__builtin_nontemporal_load(src + it.start + i), lo, mask)], 1u);
          }
        }
        __syncthreads();
        off[top][threadIdx.x] = bcnt[threadIdx.x];
        __syncthreads();
        srt_block_scan(off[top], SB, wsum);
        if (threadIdx.x == 0) {
          off[top][SB] = it.count;
          nxt[top] = 0;
          nchild[top] = mask + 1;
        }
        cur[threadIdx.x] = it.start + off[top][threadIdx.x];
        __syncthreads();
        for (uint32_t b = 0; b < it.count; b += SBATCH) {
          PT w[SE];
          uint32_t vm = 0;
#pragma unroll
          for (int k = 0; k < SE; ++k) {
            const uint32_t i = b + (uint32_t)k * SB + threadIdx.x;
            w[k] = __builtin_nontemporal_load(src + it.start + (i < it.count ? i : it.count - 1));
            vm |= (i < it.count ? 1u : 0u) << k;
          }
          srt_batch<PT, PT>(w, vm, lo, mask, stage, bcnt, bst, cur, wsum, dst, put);
        }
      }
      uint32_t d = nxt[top];  // the next non-empty child, if any
      const uint32_t nc = nchild[top];
      while (d < nc && off[top][d + 1] == off[top][d]) ++d;
      __syncthreads();
      if (d >= nc) {
        --top;
        continue;
      }
      if (threadIdx.x == 0) {
        nxt[top] = d + 1;
        lv[top + 1] = SrtItem{it.start + off[top][d], off[top][d + 1] - off[top][d], it.hi - D, it.bufp ^ 1u};
        nxt[top + 1] = 0xFFFFFFFFu;
      }
      __syncthreads();
      ++top;
    }
  }
}

// ---- (key, value) pairs by key: shapes with N % (CLS/DS) != 0, whose sink is
// not a function of a 2-bit case (pluss_faithful.hip faith_sort).  An LSD
// radix sort by 8-bit digits, stable: per pass a per-block digit histogram
// (k_pair_count), its exclusive scan over (digit, block) -- the scan kernels
// above -- and k_pair_scatter: each block of PT pairs sorted by the digit in
// LDS by eight stable one-bit splits (a block scan each), then written at its
// digit's place.  The pairs ping-pong between two buffer pairs.  Only the
// generic shapes take it (tests, small lists): simple, stable, no scratch.
constexpr int PB = 256;                  // threads of the pair kernels
constexpr int PE = 8;                    // pairs per thread (32 KB of LDS per block)
constexpr uint32_t PTILE = PB * PE;      // pairs per block

__global__ __launch_bounds__(PB) void k_pair_count(const unsigned long long* __restrict__ keys, uint64_t n,
                                                   uint32_t sh, uint32_t* __restrict__ hist, uint32_t nblk) {
  __shared__ uint32_t c[256];
  c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * PTILE;
#pragma unroll
  for (int k = 0; k < PE; ++k) {
    const uint64_t i = base + (uint64_t)k * PB + threadIdx.x;
    if (i < n) atomicAdd(&c[(uint32_t)(keys[i] >> sh) & 255u], 1u);
  }
  __syncthreads();
  hist[(uint64_t)threadIdx.x * nblk + blockIdx.x] = c[threadIdx.x];
}

// exclusive scan of one value per thread over the block (PB threads)
__device__ __forceinline__ uint32_t pair_block_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
  const uint32_t lane = __lane_id(), wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  __syncthreads();  // (wsum reused)
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int x = 0; x < PB / 64; ++x) {
    pre += x < (int)wid ? wsum[x] : 0u;
    tot += wsum[x];
  }
  total = tot;
  return pre + inc - v;
}

__global__ __launch_bounds__(PB) void k_pair_scatter(const unsigned long long* __restrict__ kin,
                                                     const unsigned long long* __restrict__ vin, uint64_t n,
                                                     uint32_t sh, const uint32_t* __restrict__ hist, uint32_t nblk,
                                                     unsigned long long* __restrict__ kout,
                                                     unsigned long long* __restrict__ vout) {
  __shared__ unsigned long long kk[PTILE], vv[PTILE];
  __shared__ uint32_t c[256], gb[256], wsum[PB / 64];
  const uint64_t base = (uint64_t)blockIdx.x * PTILE;
  const uint32_t m = n - base < PTILE ? (uint32_t)(n - base) : PTILE;  // pairs in this block
  c[threadIdx.x] = 0;
  gb[threadIdx.x] = hist[(uint64_t)threadIdx.x * nblk + blockIdx.x];
  // coalesced loads; the pad past m sorts last (digit 255, after every real pair)
#pragma unroll
  for (int k = 0; k < PE; ++k) {
    const uint32_t e = (uint32_t)k * PB + threadIdx.x;
    kk[e] = e < m ? kin[base + e] : ~0ull;
    vv[e] = e < m ? vin[base + e] : 0ull;
  }
  __syncthreads();
  // thread t holds pairs [PE*t, PE*t + PE) in order; eight stable splits by the digit's bits
  unsigned long long k[PE], v[PE];
#pragma unroll
  for (int j = 0; j < PE; ++j) {
    k[j] = kk[PE * threadIdx.x + j];
    v[j] = vv[PE * threadIdx.x + j];
  }
  for (uint32_t b = 0; b < 8; ++b) {
    uint32_t ones = 0;
#pragma unroll
    for (int j = 0; j < PE; ++j) ones += (uint32_t)(k[j] >> (sh + b)) & 1u;
    uint32_t tot0;
    const uint32_t z0 = pair_block_scan((uint32_t)PE - ones, wsum, tot0);  // zeros before this thread's run
    uint32_t o0 = PE * threadIdx.x - z0;                                    // ones before it
    uint32_t z = z0;
    __syncthreads();  // (every thread's run read before any is overwritten)
#pragma unroll
    for (int j = 0; j < PE; ++j) {
      const bool one = (k[j] >> (sh + b)) & 1u;
      const uint32_t at = one ? tot0 + o0 : z;
      o0 += one ? 1u : 0u;
      z += one ? 0u : 1u;
      kk[at] = k[j];
      vv[at] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PE; ++j) {
      k[j] = kk[PE * threadIdx.x + j];
      v[j] = vv[PE * threadIdx.x + j];
    }
  }
  // the block's digit histogram and each digit's first place in the sorted block
#pragma unroll
  for (int j = 0; j < PE; ++j)
    if (PE * threadIdx.x + j < m) atomicAdd(&c[(uint32_t)(k[j] >> sh) & 255u], 1u);
  __syncthreads();
  uint32_t all;
  const uint32_t first = pair_block_scan(c[threadIdx.x], wsum, all);
  __syncthreads();
  c[threadIdx.x] = first;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PE; ++j) {
    const uint32_t e = PE * threadIdx.x + j;
    if (e < m) {
      const uint32_t d = (uint32_t)(k[j] >> sh) & 255u;
      const uint64_t at = (uint64_t)gb[d] + (e - c[d]);
      kout[at] = k[j];
      vout[at] = v[j];
    }
  }
}

}  // namespace pluss
