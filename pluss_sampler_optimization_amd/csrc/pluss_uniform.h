// pluss_uniform.h — r10's own sample distribution generated directly in r10's
// pop order.
//
// r10 draws each reference's samples with rand() % (N-1) per index and
// rejects duplicates (r10:156-185): a uniform S-subset of the reference's
// span^d iteration points (the Feistel lists' distribution).
// Its priority queue then pops them in key order a*T+tid (IterationComp,
// pluss_utils.h:175-267).  This generator produces that same distribution
// already in key order, without a sort:
//
//   1. candidates: every point is a candidate independently with probability
//      p = min(1, (S + 10 sqrt(S) + 32) / D) (D points).  The points are cut
//      into leaves of consecutive points in key order -- a leaf is one key
//      "row" (q, c1) of 3-D references, or q of 2-D ones, cut into blocks of K
//      w-values (w = c2, or c1) times the simulated threads -- so a leaf's
//      candidate count is Binomial(G_l, p), drawn per leaf by inversion from a
//      counter-based hash (about UG_MEAN per leaf); the candidates themselves
//      are a uniform subset of the leaf of that size (independent uniform
//      offsets, sorted, redrawn on a duplicate), i.e. Bernoulli(p) sampling
//      of the whole space;
//   2. conditioned on T' >= S candidates, removing a uniform (T'-S)-subset of
//      them (the first T'-S outputs of a keyed Feistel permutation of the
//      candidate ranks [0, T')) leaves a uniform S-subset of the points
//      (exchangeability: Bernoulli sampling conditioned on its size is
//      uniform over subsets of that size, and so is a uniform sub-subset).
//      T' < S (probability about Phi(-10) = 7.6e-24) is reported as an error.
//
// Sample i of the list is the i-th surviving candidate in key order.  The
// per-leaf counts, their prefix, the removal bitmap and its prefix form the
// plan (pluss_uniform.hip); any tile of TILE consecutive samples is then
// generated independently from it (k_fa_* SRC_UNI, k_ug_expand).  Every
// floating-point step is an IEEE add, multiply or divide in a fixed order
// (no FMA contraction, no library call), so the host oracle
// (oracle/pluss_oracle.c orc_expand_uniform) reproduces the lists bit for bit.
#pragma once
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "pluss_model.h"

#if defined(__HIPCC__)
#include "pluss_internal.h"
#endif

namespace pluss {

constexpr uint32_t UG_MEAN = 16;     // expected candidates per leaf (K0)
constexpr uint32_t UG_DIRECT = 64;   // leaves of at most this many points: one Bernoulli draw per point
constexpr uint32_t UG_LEAFMAX = 1024;  // more candidates in one leaf: PLUSS_ERR_CAPACITY (P < 1e-300)
constexpr uint32_t UG_CAP = 6144;      // candidates of one tile's leaves (LDS words)
constexpr uint32_t UG_TRIES = 4096;    // redraws of a leaf's offsets before FLAG_UNI (P(dup) <= 1/2 per draw)
constexpr uint32_t UG_TILE = 4096;     // samples per tile (== the faithful pipeline's TILE)

struct UniGen {
  uint32_t ref, dim3, T, span, Q, CS;
  uint32_t tsh, tp2, cssh, csp2;  // T = 2^tsh, CS = 2^cssh (shift decodes)
  uint64_t S, D;                  // samples, points
  uint64_t W, K, nb;              // w-values per row, w-values per leaf, leaves per row
  uint64_t RA, RB, LA, L;         // rows of block A / B, leaves of block A, all leaves
  double p, r;                    // candidate probability per point; p / (1 - p)
  double pm[4];                   // (1 - p)^G of the four leaf sizes: block A / B x full / last block of a row
  uint64_t base;                  // hash key of (seed, ref)
  Div64 dnb, dspan, dtA, dtB;     // division by nb, span, T, T-1
  FastDiv fA, fB;                 // 32-bit division by T, T-1 (a leaf's offset -> w, t)
};

// (1 - p)^G by square and multiply, a fixed sequence of IEEE multiplies (host
// and device agree bit for bit)
PM_HD double uni_pow1p(double b, uint64_t e) {
  double pm = 1.0;
  for (; e; e >>= 1) {
    if (e & 1) pm = pm * b;
    b = b * b;
  }
  return pm;
}

// Host: the generator of S samples of reference `ref` (validated by the
// caller: N % (CS*T) == 0, 1 <= S <= span^d, S + 10 sqrt(S) + 32 < 2^32).
inline UniGen make_unigen(uint64_t N, uint64_t T, uint64_t CS, bool range_full, uint64_t seed, uint32_t ref,
                          uint64_t S) {
  UniGen u;
  u.ref = ref;
  u.dim3 = (ref == C0 || ref == C1) ? 0u : 1u;
  u.T = (uint32_t)T;
  u.CS = (uint32_t)CS;
  u.span = (uint32_t)(range_full ? N : N - 1);
  u.Q = (uint32_t)(N / T);
  const uint64_t QA = range_full ? u.Q : u.Q - 1;
  u.W = u.span;
  u.RA = u.dim3 ? QA * u.span : QA;
  u.RB = range_full ? 0 : (u.dim3 ? u.span : 1);
  u.D = (u.RA * T + u.RB * (T - 1)) * u.W;
  u.S = S;
  const double E = (double)S + 10.0 * sqrt((double)S) + 32.0;
  u.p = E >= (double)u.D ? 1.0 : E / (double)u.D;
  u.r = u.p < 1.0 ? u.p / (1.0 - u.p) : 0.0;
  const double kk = (double)UG_MEAN / ((double)T * u.p);
  u.K = kk < 1.0 ? 1 : (kk >= (double)u.W ? u.W : (uint64_t)kk);
  // balanced leaves: a row cut into nb = round(W / K) blocks of ceil(W / nb)
  // w-values (not K, K, ..., and a sliver of a few points); about 11-24
  // candidates per leaf
  const uint64_t nb0 = (2 * u.W + u.K) / (2 * u.K) ? (2 * u.W + u.K) / (2 * u.K) : 1;
  u.K = (u.W + nb0 - 1) / nb0;
  if (u.K > 0xFFFFFFFFull / T) u.K = 0xFFFFFFFFull / T;  // a leaf's points fit 32 bits
  u.nb = (u.W + u.K - 1) / u.K;
  u.LA = u.RA * u.nb;
  u.L = u.LA + u.RB * u.nb;
  u.base = mix64(seed ^ ((uint64_t)(ref + 1) * 0x9E3779B97F4A7C15ull) ^ 0xC2B2AE3D27D4EB4Full);
  u.tsh = 0;
  while ((1ull << u.tsh) < T) ++u.tsh;
  u.tp2 = (1ull << u.tsh) == T ? 1u : 0u;
  u.cssh = 0;
  while ((1ull << u.cssh) < CS) ++u.cssh;
  u.csp2 = (1ull << u.cssh) == CS ? 1u : 0u;
  // a leaf has K w-values (the row's last block: W - (nb-1) K) times T threads (block B: T - 1)
  const uint64_t kl = u.W - (u.nb - 1) * u.K;
  u.pm[0] = uni_pow1p(1.0 - u.p, u.K * T);
  u.pm[1] = uni_pow1p(1.0 - u.p, kl * T);
  u.pm[2] = uni_pow1p(1.0 - u.p, u.K * (T > 1 ? T - 1 : 1));
  u.pm[3] = uni_pow1p(1.0 - u.p, kl * (T > 1 ? T - 1 : 1));
  u.dnb = make_div64(u.nb);
  u.dspan = make_div64(u.span ? u.span : 1);
  u.dtA = make_div64(T);
  u.dtB = make_div64(T > 1 ? T - 1 : 1);
  u.fA = make_fastdiv((uint32_t)T);
  u.fB = make_fastdiv((uint32_t)(T > 1 ? T - 1 : 1));
  return u;
}

// a leaf: its block (0: A, 1: B), row, w-block, w-values and points
struct UniLeaf {
  uint32_t blk;
  uint64_t row, wb, kw, tb, G;
};
PM_HD UniLeaf uni_leaf(const UniGen& u, uint64_t l) {
  UniLeaf f;
  f.blk = l >= u.LA ? 1u : 0u;
  const uint64_t lb = f.blk ? l - u.LA : l;
  f.row = div64(lb, u.dnb);
  f.wb = lb - f.row * u.nb;
  const uint64_t w0 = f.wb * u.K;
  f.kw = u.W - w0 < u.K ? u.W - w0 : u.K;
  f.tb = f.blk ? u.T - 1 : u.T;
  f.G = f.kw * f.tb;
  return f;
}

// the leaf's hash key for attempt a (a = ~0: per-point draws, ~1: the count)
PM_HD uint64_t uni_leafkey(const UniGen& u, uint64_t l, uint32_t a) {
  return mix64(u.base + l * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)a * 0xD1B54A32D192ED03ull);
}
PM_HD uint64_t uni_hash(uint64_t lk, uint64_t i) { return mix64(lk + i * 0x8CB92BA72F3D8DD7ull); }
PM_HD double uni_u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

// per-point Bernoulli draws (small or dense leaves: with p <= 1/64 and at most
// 4*UG_MEAN expected candidates, independent offsets collide rarely)
PM_HD bool uni_direct(const UniGen& u, const UniLeaf& f) {
  return f.G <= UG_DIRECT || (double)f.G * u.p > 64.0 || u.p > 0.015625;
}

// The leaf's candidate count: Binomial(G, p) by inversion of one uniform
// draw u against the CDF: the smallest x with u < cdf(x), at most G, where
// pmf(0) = (1-p)^G (square and multiply), pmf(x+1) = ((pmf(x) (G-x)) / (x+1))
// p/(1-p) and cdf(x) = cdf(x-1) + pmf(x), each an IEEE operation in this
// order.  (The device reads cdf from a table of the same values, k_ug_pmt, and
// binary-searches it.)
PM_HD uint64_t uni_count(const UniGen& u, uint64_t l) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  const UniLeaf f = uni_leaf(u, l);
  if (u.p >= 1.0) return f.G;
  if (uni_direct(u, f)) {
    const uint64_t lk = uni_leafkey(u, l, 0xFFFFFFFFu);
    uint64_t c = 0;
    for (uint64_t j = 0; j < f.G; ++j) c += uni_u01(uni_hash(lk, j)) < u.p ? 1u : 0u;
    return c;
  }
  // (1 - p)^G: one of the four leaf sizes' values, computed once (make_unigen)
  // (selects, not an index: an indexed copy of the generator went to scratch)
  double pm = f.blk ? (f.kw == u.K ? u.pm[2] : u.pm[3]) : (f.kw == u.K ? u.pm[0] : u.pm[1]);
  const double x_u = uni_u01(uni_hash(uni_leafkey(u, l, 0xFFFFFFFEu), 0));
  double cdf = pm;
  uint64_t x = 0;
  while (!(x_u < cdf) && x < f.G) {
    pm = pm * (double)(f.G - x);
    pm = pm / (double)(x + 1);
    pm = pm * u.r;
    ++x;
    cdf = cdf + pm;
  }
  return x;
}

// candidate offset i (attempt a) of a counted leaf: uniform in [0, G).  Leaves
// of at most UG_PAIRG points take two offsets from one 64-bit hash, 32 bits
// each (a relative bias below G / 2^32 <= 1.6e-5); larger ones one per hash.
constexpr uint64_t UG_PAIRG = 1ull << 16;
PM_HD uint64_t uni_offset(uint64_t lk, uint64_t i, uint64_t G) {
  if (G <= UG_PAIRG) {
    const uint64_t h = uni_hash(lk, i >> 1);
    const uint32_t half = (i & 1) ? (uint32_t)(h >> 32) : (uint32_t)h;
    return ((uint64_t)half * G) >> 32;
  }
  return mulhi64(uni_hash(lk, i), G);
}

// ---- the removal permutation: a keyed cycle-walking Feistel permutation of
// the candidate ranks [0, Tp); its first Tp - S outputs are removed
struct UniPerm {
  uint32_t key[4], h;
  uint64_t D, mask;
};
PM_HD UniPerm uni_perm_make(const UniGen& u, uint64_t Tp) {
  UniPerm p;
  p.D = Tp;
  p.h = 1;
  while ((1ull << (2 * p.h)) < Tp) ++p.h;
  p.mask = (1ull << p.h) - 1;
  for (int r = 0; r < 4; ++r)
    p.key[r] = (uint32_t)mix64(u.base ^ ((uint64_t)(r + 1) * 0xD1B54A32D192ED03ull) ^ 0x6A09E667F3BCC909ull);
  return p;
}
PM_HD uint64_t uni_perm(const UniPerm& p, uint64_t y) {
  const uint32_t mask = (uint32_t)p.mask;
  do {
    uint32_t L = (uint32_t)(y >> p.h), R = (uint32_t)y & mask;
    for (int r = 0; r < 4; ++r) {
      const uint32_t t = R;
      R = L ^ (lowbias32(R ^ p.key[r]) & mask);
      L = t;
    }
    y = ((uint64_t)L << p.h) | R;
  } while (y >= p.D);
  return y;
}

// digits of the point at offset o of leaf f (o < f.G: w = wb*K + o / tb, t = o % tb)
PM_HD KeyDigits uni_digits(const UniGen& u, const UniLeaf& f, uint64_t o) {
  KeyDigits d;
  uint64_t wq;
  if (!f.blk && u.tp2) {
    wq = o >> u.tsh;
    d.t = (uint32_t)(o & (u.T - 1));
  } else {
    const Div64& dt = f.blk ? u.dtB : u.dtA;
    wq = div64(o, dt);
    d.t = (uint32_t)(o - wq * f.tb);
  }
  const uint32_t w = (uint32_t)(f.wb * u.K + wq);
  if (f.blk) {
    d.q = u.Q - 1;
    d.c1 = u.dim3 ? (uint32_t)f.row : w;
  } else if (u.dim3) {
    const uint64_t q = div64(f.row, u.dspan);
    d.q = (uint32_t)q;
    d.c1 = (uint32_t)(f.row - q * u.span);
  } else {
    d.q = (uint32_t)f.row;
    d.c1 = w;
  }
  d.c2 = u.dim3 ? w : 0u;
  return d;
}

// packed sample ref|c0|c1|c2 of digits (c0 = ((q / CS) * T + t) * CS + q % CS)
PM_HD uint64_t uni_pack(const UniGen& u, const KeyDigits& d) {
  const uint32_t c0 = (u.csp2 && u.tp2) ? (((((d.q >> u.cssh) << u.tsh) | d.t) << u.cssh) | (d.q & (u.CS - 1)))
                                        : ((d.q / u.CS) * u.T + d.t) * u.CS + d.q % u.CS;
  return pack(u.ref, c0, d.c1, d.c2);
}

// ---- the plan of up to six references' lists (device memory) ----------------
struct UniSet {
  UniGen u[6];
  uint64_t loff[7];     // first leaf of each reference in cnt / pre; loff[6] = all leaves
  uint64_t lbase[6];    // the reference's leaf (in UniGen's numbering) held at loff[r]: 0 on one GPU; a
                        // key-range shard holds the leaves [lbase, lbase + loff[r+1] - loff[r]) and ranks
                        // its candidates from its own first one (the plan's coordinates are the shard's)
  uint64_t woff[7];     // first removal-bitmap word of each reference
  uint64_t tmoff[7];    // first tile-map entry of each reference (tiles of UG_TILE samples)
  const uint32_t* cnt;  // candidates per leaf
  const uint64_t* pre;  // exclusive prefix of cnt over all leaves (loff[6] + 1 words)
  const uint32_t* bits; // removed candidate ranks, per reference
  const uint64_t* rb;   // exclusive prefix of the bitmap words' popcounts (woff[6] + 1 words)
  const uint32_t* tmap; // per tile: the leaf holding its first sample
  unsigned int* flags;  // the handle's flags (FLAG_UNI)
  const double* pmt;    // per reference and leaf size class: uni_count's cdf(0..xm), +inf past it, [UG_PMT-1] = xm
};
constexpr int UI_W = 24;  // a plan's info words (UniBufs::info): [0,6) removed ranks below it, [6,12) first, [12,18) n
constexpr uint32_t UG_PMT = UG_LEAFMAX + 2;  // table entries per leaf size class (4 classes per reference)

#if defined(__HIPCC__)
// uni_count with the CDF read from the reference's table for the leaf's size
// class (the same doubles: the table is that recurrence and sum, run once per
// class by k_ug_pmt): a binary search of UG_CDF entries, no loop per lane.
// Entries past the class's reach xm (mean + 40 sd + 64) are +inf and
// cdf[UG_PMT - 1] holds xm: a draw past it (P < 1e-300) returns UG_LEAFMAX + 1
// (flagged by the caller) unless G lies within the reach.
constexpr uint32_t UG_CDF = 512;  // searched entries (xm < 448: the counted leaves expect at most 64 candidates)
__device__ __forceinline__ uint64_t uni_count_tab(const UniGen& u, uint64_t l, const double* __restrict__ pmt) {
  const UniLeaf f = uni_leaf(u, l);
  if (u.p >= 1.0 || uni_direct(u, f)) return uni_count(u, l);
  const double* t = pmt + ((f.blk ? 2 : 0) + (f.kw == u.K ? 0 : 1)) * UG_PMT;
  const double x_u = uni_u01(uni_hash(uni_leafkey(u, l, 0xFFFFFFFEu), 0));
  uint32_t lo = 0;  // entries below lo are <= x_u
#pragma unroll
  for (uint32_t step = UG_CDF / 2; step; step >>= 1)
    if (t[lo + step - 1] <= x_u) lo += step;
  const uint64_t xm = (uint64_t)t[UG_PMT - 1];
  if (lo > xm && f.G > xm) return UG_LEAFMAX + 1;
  return lo < f.G ? lo : f.G;
}
#endif

#if defined(__HIPCC__)
// candidates of reference r before leaf l / removed candidates of rank < x
__device__ __forceinline__ uint64_t uni_pre(const UniSet* __restrict__ us, uint32_t r, uint64_t l) {
  return us->pre[us->loff[r] + l] - us->pre[us->loff[r]];
}
__device__ __forceinline__ uint64_t uni_word(const UniSet* __restrict__ us, uint32_t r, uint64_t x) {
  const uint64_t w = us->woff[r] + (x >> 5), e = us->woff[r + 1] - 1;  // (clamped: a flagged plan stays in bounds)
  return w < e ? w : e;
}
__device__ __forceinline__ uint64_t uni_removed_before(const UniSet* __restrict__ us, uint32_t r, uint64_t x) {
  const uint64_t w = uni_word(us, r, x);
  const uint32_t below = us->bits[w] & ((1u << (x & 31)) - 1u);
  return us->rb[w] - us->rb[us->woff[r]] + (uint64_t)__popc(below);
}

// Generate samples [lt*UG_TILE, lt*UG_TILE + mt) of reference r's list into
// raw[slot(e)] (e = sample - lt*UG_TILE), all NT threads of the workgroup;
// cand: LDS scratch of UG_CAND words.  The leaves from the one holding the
// tile's first sample to the one holding the next tile's first are
// regenerated: the removal bitmap's words over their candidate ranks and the
// words' removed-before counts are staged in LDS first (a few hundred words,
// coalesced), then each thread draws one leaf's candidates in key order and
// packs every surviving one at its sample index:
//   per-point draws (small or dense leaves) come out in order;
//   up to UG_NET offsets are sorted in registers (an odd-even merge network);
//   larger leaves (rare) are insertion-sorted in a shared LDS scratch of
//   UG_SCR words, or, when the tile's large leaves overflow it, emitted by
//   repeated minimum search over their offsets (no scratch; O(c^2)).
// A window past UG_CAP candidates or a leaf past UG_LEAFMAX (neither happens
// with probability above 1e-20) sets FLAG_UNI.
constexpr uint32_t UG_WCAP = UG_CAP / 32 + 2;  // bitmap words over a window of UG_CAP ranks
constexpr uint32_t UG_SCR = 768;               // the large leaves' scratch (words; 4 workgroups of the scan per CU)
constexpr uint32_t UG_CAND = UG_SCR + 2 * UG_WCAP + 1;  // cand: scratch, the window's words and counts, an allocator

// a leaf's row decoded once, and its packed samples' fixed bits: the digits
// of offset o are then shifts (block A, T a power of two)
struct UniRowD {
  uint32_t q, c1, w0;
};
__device__ __forceinline__ UniRowD uni_row(const UniGen& u, const UniLeaf& f) {
  UniRowD d;
  d.w0 = (uint32_t)(f.wb * u.K);
  if (f.blk) {
    d.q = u.Q - 1;
    d.c1 = u.dim3 ? (uint32_t)f.row : 0u;
  } else if (u.dim3) {
    const uint64_t q = div64(f.row, u.dspan);
    d.q = (uint32_t)q;
    d.c1 = (uint32_t)(f.row - q * u.span);
  } else {
    d.q = (uint32_t)f.row;
    d.c1 = 0;
  }
  return d;
}
// = uni_pack(u, uni_digits(u, f, o))
__device__ __forceinline__ uint64_t uni_pack_row(const UniGen& u, const UniLeaf& f, const UniRowD& rd, uint32_t o) {
  uint32_t wq, t;
  if (!f.blk && u.tp2) {
    wq = o >> u.tsh;
    t = o & (u.T - 1);
  } else {
    wq = (uint32_t)div64(o, f.blk ? u.dtB : u.dtA);
    t = o - wq * (uint32_t)f.tb;
  }
  KeyDigits d;
  const uint32_t w = rd.w0 + wq;
  d.t = t;
  d.q = rd.q;
  d.c1 = u.dim3 ? rd.c1 : w;
  d.c2 = u.dim3 ? w : 0u;
  return uni_pack(u, d);
}

// uni_offset for G < 2^32, in 32-bit pieces (floor(h * G / 2^64) for the large leaves)
__device__ __forceinline__ uint32_t uni_offset32(uint64_t lk, uint32_t i, uint32_t G) {
  if (G <= UG_PAIRG) {
    const uint64_t h = uni_hash(lk, i >> 1);
    return __umulhi((i & 1) ? (uint32_t)(h >> 32) : (uint32_t)h, G);
  }
  const uint64_t h = uni_hash(lk, i);
  const uint64_t t = (uint64_t)(uint32_t)(h >> 32) * G + __umulhi((uint32_t)h, G);
  return (uint32_t)(t >> 32);
}
// ascending sort of NC (a power of two) values in registers: Batcher's
// odd-even merge sort (191 compare-exchanges for 32, a bitonic network 240)
template <int NC>
__device__ __forceinline__ void uni_sort_net(uint32_t (&v)[NC]) {
#pragma unroll
  for (int p = 1; p < NC; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j + k < NC; j += 2 * k)
#pragma unroll
        for (int i = 0; i < k && i + j + k < NC; ++i)
          if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const uint32_t a = v[i + j], b = v[i + j + k];
            v[i + j] = a < b ? a : b;
            v[i + j + k] = a < b ? b : a;
          }
}
// leaves of at most this many candidates: sorted in registers (30, not 32:
// the 32-wide network held the uniform scan at 128 VGPRs with 16 B of spills;
// P(c > 30) = 5e-4 at UG_MEAN 16, those leaves take the large-leaf path and
// draw the same offsets)
constexpr uint32_t UG_NET = 30;

// What the faithful scan needs of a shape to take staged elements decoded
// (uni_stage DEC): the key's low 32 bits and the case flags, per candidate,
// from its leaf's constants (k_fa_local_lm)
struct UniDec {
  uint32_t N, Wm1, Q, S, nsh, tsh;
};

// Generate samples [lt*UG_TILE, lt*UG_TILE + mt) of reference r's list into
// raw[slot(e)] (e = sample - lt*UG_TILE), all NT threads of the workgroup;
// cand: LDS scratch of UG_CAND words.  DEC: instead of the packed sample,
// raw[e] = its faithful key a*T + tid's low 32 bits | case 0 flag << 32 |
// case 1 flag << 33 | tid == 0 << 34 | the key's high bits << 35
// (fa_lane_tile's element, nothing left to decode; shapes whose keys stay
// below 2^61 and whose leaves span less than 2^32 keys, FaRefs::unidec).
// DEC emits in two phases (round 6): each leaf's thread writes, per kept
// candidate, only (its leaf's slot in `tab`, its offset) -- a few
// instructions per slot of the 32-slot emission -- and the leaf's fixed
// decode bits once into tab; then every thread decodes its share of the
// tile's elements from the table.  (Decoding inside each of a leaf's 32
// predicated slots held the row's constants live through the sorting
// network: 128 VGPRs and 80 B of register spills per lane.)  `tab`: tcap
// LDS words of 8 bytes; the leaves go in rounds of at most tcap leaves whose
// key bases lie within 2^32 of the round's first (one round for a dense tile).
template <int NT, bool DEC, class SLOT>
__device__ __forceinline__ void uni_stage(const UniSet* __restrict__ us, uint32_t r, uint64_t lt, uint32_t mt,
                                          unsigned long long* raw, uint32_t* cand, unsigned int* flags,
                                          SLOT&& slot, const UniDec dz = UniDec{}, unsigned long long* tab = nullptr,
                                          uint32_t tcap = 0) {
  // the generator and the plan's arrays copied out once: read through the
  // plan pointer after every LDS store (generic stores may alias it), they
  // were reloaded from memory per candidate
  const UniGen u = us->u[r];
  const uint32_t* __restrict__ cnt = us->cnt;
  const uint64_t* __restrict__ pre = us->pre;
  const uint64_t tm0 = us->tmoff[r], nt = us->tmoff[r + 1] - tm0, lg0 = us->loff[r];
  const uint64_t nl = us->loff[r + 1] - lg0, lbase = us->lbase[r];  // (leaves held; their first's number)
  const uint64_t la = us->tmap[tm0 + lt], lb = lt + 1 < nt ? us->tmap[tm0 + lt + 1] : nl - 1;
  const uint64_t pbase = pre[lg0];
  const bool leaves_ok = nl > 0 && la <= lb && lb < nl && (!DEC || tcap > 0);
  const uint64_t r0 = leaves_ok ? pre[lg0 + la] - pbase : 0, rend = leaves_ok ? pre[lg0 + lb + 1] - pbase : 0;
  if (!leaves_ok || rend - r0 > UG_CAP) {
    if (threadIdx.x == 0) atomicOr(flags, FLAG_UNI);
    __syncthreads();
    return;
  }
  // the window's bitmap words [wlo, wlo + nw] (reference-relative; one past
  // its last, so any leaf can read two words) and their removed-before counts
  const uint64_t wo = us->woff[r], wend = us->woff[r + 1] - wo;  // (a flagged plan's indices are clamped)
  const uint64_t wlo = r0 >> 5;
  const uint32_t nw = rend > r0 ? (uint32_t)(((rend - 1) >> 5) - wlo + 1) : 0u;
  uint32_t* scr = cand;
  uint32_t* bw = cand + UG_SCR;
  uint32_t* rbw = bw + UG_WCAP;
  uint32_t* alloc = rbw + UG_WCAP;
  const uint64_t wl = wlo < wend ? wlo : wend - 1;
  const uint64_t rem0 = us->rb[wo + wl] - us->rb[wo];
  for (uint32_t i = threadIdx.x; i <= nw; i += NT) {
    const uint64_t w = wlo + i < wend ? wlo + i : wend - 1;
    bw[i] = wlo + i < wend ? us->bits[wo + w] : 0u;
    rbw[i] = (uint32_t)(us->rb[wo + w] - us->rb[wo] - rem0);
  }
  if (threadIdx.x == 0) *alloc = 0;
  __syncthreads();
  const uint64_t f0 = lt * UG_TILE;
  // tile element of window rank (wlo << 5) if nothing before it were removed: a
  // window rank xr (kept, with remr removed below it in the window) lands at
  // ebase + xr - remr
  const int32_t ebase = (int32_t)((int64_t)(wlo << 5) - (int64_t)rem0 - (int64_t)f0);
  // (DEC) a leaf's key base: ((q << nsh) + (3-D ? c1 : w0)) * S + (C0, C1: ref; else ref + 4 w0), times T
  auto leaf_key = [&](const UniRowD& rd) -> uint64_t {
    const uint32_t qc0 = (rd.q << dz.nsh) + (u.dim3 ? rd.c1 : rd.w0);
    return ((uint64_t)qc0 * dz.S + (u.ref < 2 ? u.ref : u.ref + 4u * rd.w0)) << dz.tsh;
  };
  // leaf l's candidates (DEC: its table slot ts, the round's key base K0)
  auto leaf = [&](uint64_t l, uint32_t ts, uint64_t K0) {
    const uint32_t c = cnt[lg0 + l];
    if (!c) return;
    if (c > UG_LEAFMAX) {
      atomicOr(flags, FLAG_UNI);
      return;
    }
    // (32-bit, relative to the window: a window holds at most UG_CAP candidates)
    const uint32_t xr = (uint32_t)(pre[lg0 + l] - pbase - (wlo << 5));  // rank of the leaf's first, from bit 0 of bw[0]
    const UniLeaf f = uni_leaf(u, lbase + l);
    const UniRowD rd = uni_row(u, f);
    // candidate i of the leaf (in key order) has rank x0 + i; the removed ones are skipped
    // tile-relative index of the leaf's first candidate if nothing of it were
    // removed (computed where it is used: held through the sorting network it
    // pushed the uniform scan past 128 VGPRs)
    auto first_e = [&]() -> int32_t {
      const uint32_t remr = rbw[xr >> 5] + (uint32_t)__popc(bw[xr >> 5] & ((1u << (xr & 31u)) - 1u));
      return ebase + (int32_t)xr - (int32_t)remr;  // (remr: removed in the window before it)
    };
    // the packed sample's fixed bits for this leaf (block A, T and CS powers of
    // two: every BASELINE shape): offset o adds t = o % T to c0 and w = o / T
    // to c2 (3-D) or c1 (2-D); other leaves divide
    const bool fastp = !f.blk && u.tp2 && u.csp2;
    if constexpr (DEC) {
      // the leaf's entry: its key base relative to the round's, and its row's
      // decode bits (pluss_faithful.h fa_dec_digits: for 3-D references only
      // c2 = w moves, so case 0 is ((w & am) != av) && w < alim and case 1 a
      // leaf constant): w0 | case-1 flag << 20 | av << 21 | block B << 22
      uint32_t av = 1u, b1 = 1u;
      if (u.ref == C3) b1 = (rd.c1 & dz.Wm1) != dz.Wm1 ? 1u : 0u;
      else if (u.ref == A0) b1 = rd.c1 + 1 < dz.N ? 1u : 0u;
      else if (u.ref == B0) {
        av = (rd.c1 & dz.Wm1) != dz.Wm1 ? 1u : 0u;
        b1 = rd.q + 1 < dz.Q ? 1u : 0u;
      }
      const uint32_t meta = rd.w0 | (b1 << 20) | ((av & 1u) << 21) | (f.blk << 22);
      tab[ts] = (unsigned long long)(uint32_t)(leaf_key(rd) - K0) | ((unsigned long long)meta << 32);
    }
    const uint32_t c0b = ((rd.q >> u.cssh) << (u.tsh + u.cssh)) | (rd.q & (u.CS - 1));
    const uint64_t pkb = pack(u.ref, c0b, u.dim3 ? rd.c1 : 0u, u.dim3 ? rd.w0 : 0u);
    const FastDiv fd = f.blk ? u.fB : u.fA;
    const uint32_t tb = (uint32_t)f.tb;
    auto put = [&](uint32_t e, uint32_t o, auto fastc) {  // candidate at offset o, kept as tile element e < mt
      if constexpr (!DEC) {
        constexpr bool FP = decltype(fastc)::value;       // (block A, T and CS powers of two: shifts)
        const uint32_t wq = FP ? o >> u.tsh : (uint32_t)(((uint64_t)umulhi32(o, fd.m) + o) >> fd.s);
        const uint32_t t = FP ? o & (u.T - 1) : o - wq * tb;
        uint64_t pk;
        if (FP) {
          pk = pkb | ((uint64_t)t << (40 + u.cssh));
          pk = u.dim3 ? pk + wq : pk | ((uint64_t)(rd.w0 + wq) << 20);  // (c2 = w0 + wq < 2^20)
        } else {
          pk = uni_pack_row(u, f, rd, o);
        }
        raw[slot(e)] = pk;
      } else {
        reinterpret_cast<uint2*>(raw)[e] = make_uint2(o, ts);  // (slot << 32 | offset, decoded after the round)
      }
    };
    // one candidate at a time, the removed ones counted as they come (the rare paths)
    int32_t e = 0;
    auto emit = [&](uint32_t i, uint32_t o) {
      const uint32_t x = xr + i;
      if ((bw[x >> 5] >> (x & 31)) & 1u) return;
      if ((uint32_t)e < mt) put((uint32_t)e, o, std::false_type{});
      ++e;
    };
    const uint64_t gl = lbase + l;      // the leaf's number (its hash key's)
    const uint32_t G = (uint32_t)f.G;  // (K*T < 2^32)
    const bool direct = uni_direct(u, f);
    if (u.p >= 1.0) {
      e = first_e();
      for (uint32_t j = 0; j < c; ++j) emit(j, j);
    } else if (direct) {  // per-point draws: already in order
      const uint64_t lk = uni_leafkey(u, gl, 0xFFFFFFFFu);
      e = first_e();
      uint32_t k = 0;
      for (uint32_t j = 0; j < G && k < c; ++j)
        if (uni_u01(uni_hash(lk, j)) < u.p) emit(k++, j);
    } else if (c <= UG_NET) {
      // the common leaf: its offsets drawn and sorted in registers (an insertion
      // sort through LDS was a chain of dependent LDS round trips, divergent per lane)
      uint32_t v[UG_NET];
      const uint64_t lm = uni_leafkey(u, gl, 0);  // (draw a's key: lm ^ a * the draw constant, uni_leafkey)
      for (uint32_t a = 0;; ++a) {
        if (a == UG_TRIES) {
          atomicOr(flags, FLAG_UNI);
          break;
        }
        const uint64_t lk = lm ^ ((uint64_t)a * 0xD1B54A32D192ED03ull);
        if (G <= UG_PAIRG) {  // two offsets per hash; slots past every lane's count skipped
#pragma unroll
          for (uint32_t q = 0; q < UG_NET; q += 2) {
            v[q] = v[q + 1] = 0xFFFFFFFFu;
            if (__any(q < c)) {
              const uint64_t h = uni_hash(lk, q >> 1);
              if (q < c) v[q] = __umulhi((uint32_t)h, G);
              if (q + 1 < c) v[q + 1] = __umulhi((uint32_t)(h >> 32), G);
            }
          }
        } else {
#pragma unroll
          for (uint32_t q = 0; q < UG_NET; ++q) v[q] = q < c ? uni_offset32(lk, q, G) : 0xFFFFFFFFu;
        }
        uni_sort_net<UG_NET>(v);
        bool dup = false;  // (offsets < G <= 2^32 - 1: the padding sorts last and never matches)
#pragma unroll
        for (uint32_t q = 0; q + 1 < UG_NET; ++q) dup |= v[q] == v[q + 1] && q + 1 < c;
        if (!dup) break;
      }
      // the leaf's removed candidates from its two bitmap words at once (c <= 32
      // ranks from x0); candidate q is tile element be + q - (removed below q)
      const int32_t be = first_e();
      const uint32_t w0i = xr >> 5;
      const uint64_t W = (uint64_t)bw[w0i] | ((uint64_t)bw[w0i + 1] << 32);
      const uint32_t rm = (uint32_t)(W >> (xr & 31u)) & (c >= 32 ? 0xFFFFFFFFu : (1u << c) - 1u);
      auto slots = [&](auto fastc) {
#pragma unroll
        for (uint32_t q = 0; q < UG_NET; ++q) {
          const int32_t e = be + (int32_t)q - (int32_t)__popc(rm & ((1u << q) - 1u));
          if (q < c && !((rm >> q) & 1u) && (uint32_t)e < mt) put((uint32_t)e, v[q], fastc);
        }
      };
      if (DEC || !fastp) slots(std::false_type{});
      else slots(std::true_type{});
    } else {  // a large leaf (rare)
      const uint32_t off = atomicAdd(alloc, c);
      uint64_t lk = 0;
      for (uint32_t a = 0;; ++a) {  // independent uniform offsets, sorted; redrawn on a duplicate
        if (a == UG_TRIES) {
          atomicOr(flags, FLAG_UNI);
          break;
        }
        lk = uni_leafkey(u, gl, a);
        bool dup = false;
        if (off + c <= UG_SCR) {
          uint32_t* seg = scr + off;
          for (uint32_t i = 0; i < c; ++i) {
            const uint32_t x = uni_offset32(lk, i, G);
            uint32_t j = i, y = 0;
            while (j > 0 && (y = seg[j - 1]) > x) {
              seg[j] = y;
              --j;
            }
            dup |= j > 0 && y == x;
            seg[j] = x;
          }
        } else {
          for (uint32_t i = 1; i < c && !dup; ++i) {
            const uint32_t x = uni_offset32(lk, i, G);
            for (uint32_t j = 0; j < i; ++j) dup |= uni_offset32(lk, j, G) == x;
          }
        }
        if (!dup) break;
      }
      e = first_e();
      if (off + c <= UG_SCR) {
        for (uint32_t i = 0; i < c; ++i) emit(i, scr[off + i]);
      } else {  // no scratch left: the offsets in order by repeated minimum search
        int64_t last = -1;
        for (uint32_t i = 0; i < c; ++i) {
          uint32_t m = 0xFFFFFFFFu;
          for (uint32_t j = 0; j < c; ++j) {
            const uint32_t x = uni_offset32(lk, j, G);
            if ((int64_t)x > last && x < m) m = x;
          }
          emit(i, m);
          last = m;
        }
      }
    }
  };
  if constexpr (!DEC) {
    for (uint64_t l = la + threadIdx.x; l <= lb; l += NT) leaf(l, 0u, 0ull);
    __syncthreads();
    return;
  } else {
    // the tile element of leaf l's first kept candidate (l in [la, lb + 1])
    auto first_elem = [&](uint64_t l) -> int64_t {
      const uint32_t xr = (uint32_t)(pre[lg0 + l] - pbase - (wlo << 5));
      const uint32_t remr = rbw[xr >> 5] + (uint32_t)__popc(bw[xr >> 5] & ((1u << (xr & 31u)) - 1u));
      return (int64_t)ebase + (int64_t)xr - (int64_t)remr;
    };
    auto key_of_leaf = [&](uint64_t l) { return leaf_key(uni_row(u, uni_leaf(u, lbase + l))); };
    // the reference's decode constants (fa_dec_digits): case 0 = ((w & am) != av) && w < alim
    const uint32_t am = u.ref == A0 ? dz.Wm1 : 0u, alim = u.ref == C3 ? dz.N - 1 : 0xFFFFFFFFu;
    const uint32_t dk = (u.dim3 ? 4u : dz.S) << dz.tsh;
    const bool tp2 = u.tp2 != 0;
    for (uint64_t l0 = la; l0 <= lb;) {
      const uint64_t K0 = key_of_leaf(l0);
      uint64_t l1 = lb - l0 >= tcap ? l0 + tcap - 1 : lb;
      if (key_of_leaf(l1) - K0 > 0xFFFFFFFFull) {  // (keys grow with the leaf: the last within 2^32 of K0)
        uint64_t lo = l0, hi = l1;
        while (lo < hi) {
          const uint64_t mid = lo + (hi - lo + 1) / 2;
          if (key_of_leaf(mid) - K0 <= 0xFFFFFFFFull) lo = mid;
          else hi = mid - 1;
        }
        l1 = lo;
      }
      // (a 32-bit loop over the round's slots: the leaf is l0 + its slot)
      const uint32_t nr = (uint32_t)(l1 - l0);
      for (uint32_t i = threadIdx.x; i <= nr; i += NT) leaf(l0 + i, i, K0);
      __syncthreads();
      // this round's elements: (slot, offset) -> the decoded word
      const int64_t ea = first_elem(l0), eb = first_elem(l1 + 1);
      const uint32_t e0 = ea < 0 ? 0u : (ea > (int64_t)mt ? mt : (uint32_t)ea);
      const uint32_t e1 = eb < 0 ? 0u : (eb > (int64_t)mt ? mt : (uint32_t)eb);
      for (uint32_t e = e0 + threadIdx.x; e < e1; e += NT) {
        const unsigned long long pw = raw[e];
        const uint32_t o = (uint32_t)pw;
        const unsigned long long en = tab[(uint32_t)(pw >> 32)];
        const uint32_t meta = (uint32_t)(en >> 32), blk = (meta >> 22) & 1u;
        uint32_t wq, t;
        if (!blk && tp2) {
          wq = o >> u.tsh;
          t = o & (u.T - 1);
        } else {
          const FastDiv fd = blk ? u.fB : u.fA;
          wq = (uint32_t)(((uint64_t)umulhi32(o, fd.m) + o) >> fd.s);
          t = o - wq * (blk ? u.T - 1 : u.T);
        }
        const uint32_t w = (meta & 0xFFFFFu) + wq, av = (meta >> 21) & 1u;
        const uint32_t ca = ((w & am) != (u.ref == A0 ? dz.Wm1 : av) && w < alim) ? 1u : 0u;
        const unsigned long long key = K0 + (uint32_t)en + (uint32_t)(wq * dk + t);
        raw[e] = (unsigned long long)(uint32_t)key |
                 ((unsigned long long)(ca | (((meta >> 20) & 1u) << 1) | (t == 0 ? 4u : 0u) |
                                       ((uint32_t)(key >> 32) << 3)) << 32);
      }
      __syncthreads();
      l0 = l1 + 1;
    }
  }
}
#endif

}  // namespace pluss
