// pluss_uniform.hip — r10's uniform draw in key order (pluss_uniform.h): the
// plan kernels, the materialised lists (pluss_dev_expand_uniform_sorted) and
// the faithful pass over lists generated inside it
// (pluss_dev_gen_uniform_faithful_refs).
//
// Plan, all references at once (a few small launches, no host round trip):
//   k_ug_count   every leaf's candidate count (Binomial by inversion);
//   scan         their exclusive prefix over all leaves (candidate ranks);
//   k_ug_remove  per reference T' = its candidates, the ranks F(0..T'-S-1) of
//                the removal permutation set in its bitmap (T' < S: FLAG_UNI);
//   scan         the prefix of the bitmap words' popcounts;
//   k_ug_tiles   per leaf its surviving candidates' sample indices; the leaf
//                holding each tile's first sample.
// A tile of samples is then generated from the plan alone (uni_stage).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "pluss_faithful.h"
#include "pluss_uniform.h"

namespace pluss {

constexpr uint32_t UB = 256, UE = 16, UBATCH = UB * UE;  // scan: threads, values per thread, per block

template <int MODE>
__device__ __forceinline__ uint64_t ug_val(const uint32_t* in, uint64_t i) {
  return MODE ? (uint64_t)__popc(in[i]) : (uint64_t)in[i];
}

// per block of UBATCH values: their sum
template <int MODE>
__global__ __launch_bounds__(UB) void k_ug_bsum(const uint32_t* __restrict__ in, uint64_t n,
                                               uint64_t* __restrict__ bsum) {
  __shared__ uint64_t w[UB / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * UBATCH;
  uint64_t s = 0;
  for (uint32_t k = 0; k < UE; ++k) {
    const uint64_t i = b0 + (uint64_t)k * UB + threadIdx.x;
    if (i < n) s += ug_val<MODE>(in, i);
  }
  s = sc_wave_red<false>(s);
  if (__lane_id() == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// exclusive scan of the nb block sums in place (one workgroup); bsum[nb] = the total
__global__ __launch_bounds__(UB) void k_ug_btop(uint64_t* __restrict__ bsum, uint32_t nb) {
  __shared__ uint64_t w[UB / 64];
  uint64_t carry = 0;
  for (uint32_t b = 0; b < nb; b += UB) {
    const uint32_t i = b + threadIdx.x;
    const uint64_t v = i < nb ? bsum[i] : 0ull;
    const uint64_t inc = sc_wave_scan<false>(v, __lane_id());
    if (__lane_id() == 63) w[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (uint32_t x = 0; x < UB / 64; ++x) {
      if (x < (threadIdx.x >> 6)) pre += w[x];
      tot += w[x];
    }
    if (i < nb) bsum[i] = carry + pre + inc - v;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}

// out[i] = exclusive prefix of the values (out[n] = the total).  The block's
// values go through LDS both ways: read and written coalesced (a thread's own
// run of UE consecutive values read straight from memory was a 64-byte
// stride per lane, ~2 TB/s), scanned as runs of UE per thread.
__device__ __forceinline__ uint32_t ug_pad(uint32_t i) { return i + (i >> 4); }  // (runs of 16: conflict-free)
template <int MODE>
__global__ __launch_bounds__(UB) void k_ug_bapply(const uint32_t* __restrict__ in, uint64_t n,
                                                 const uint64_t* __restrict__ bsum, uint64_t* __restrict__ out) {
  __shared__ uint64_t w[UB / 64];
  __shared__ uint64_t sv[UBATCH + UBATCH / 16];
  const uint64_t b0 = (uint64_t)blockIdx.x * UBATCH;
#pragma unroll
  for (uint32_t k = 0; k < UE; ++k) {
    const uint32_t i = k * UB + threadIdx.x;
    sv[ug_pad(i)] = b0 + i < n ? ug_val<MODE>(in, b0 + i) : 0ull;
  }
  __syncthreads();
  const uint32_t j0 = threadIdx.x * UE;
  uint64_t v[UE], s = 0;
#pragma unroll
  for (uint32_t k = 0; k < UE; ++k) {
    v[k] = sv[ug_pad(j0 + k)];
    s += v[k];
  }
  const uint64_t inc = sc_wave_scan<false>(s, __lane_id());
  if (__lane_id() == 63) w[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint64_t pre = bsum[blockIdx.x];
  for (uint32_t x = 0; x < (threadIdx.x >> 6); ++x) pre += w[x];
  uint64_t run = pre + inc - s;
#pragma unroll
  for (uint32_t k = 0; k < UE; ++k) {
    sv[ug_pad(j0 + k)] = run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < UE; ++k) {
    const uint32_t i = k * UB + threadIdx.x;
    if (b0 + i < n) out[b0 + i] = sv[ug_pad(i)];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = bsum[gridDim.x];
}

static int ug_scan(const uint32_t* in, uint64_t n, uint64_t* bsum, uint64_t* out, int mode, hipStream_t s) {
  const uint32_t nb = (uint32_t)((n + UBATCH - 1) / UBATCH);
  if (nb == 0) {
    PLUSS_HIP_CHECK(hipMemsetAsync(out, 0, 8, s));
    return PLUSS_OK;
  }
  if (mode) hipLaunchKernelGGL(k_ug_bsum<1>, dim3(nb), dim3(UB), 0, s, in, n, bsum);
  else hipLaunchKernelGGL(k_ug_bsum<0>, dim3(nb), dim3(UB), 0, s, in, n, bsum);
  hipLaunchKernelGGL(k_ug_btop, dim3(1), dim3(UB), 0, s, bsum, nb);
  if (mode) hipLaunchKernelGGL(k_ug_bapply<1>, dim3(nb), dim3(UB), 0, s, in, n, (const uint64_t*)bsum, out);
  else hipLaunchKernelGGL(k_ug_bapply<0>, dim3(nb), dim3(UB), 0, s, in, n, (const uint64_t*)bsum, out);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

__device__ __forceinline__ uint32_t ug_ref_of(const uint64_t* off, uint64_t g) {
  uint32_t r = 0;
  for (int x = 1; x < 6; ++x) r += g >= off[x] ? 1u : 0u;
  return r;
}

// the CDF table of every reference's four leaf sizes: uni_count's recurrence
// and running sum, the same operations in the same order (no contraction).
// One wave per (reference, size class): lane 0 runs them (sequential, a
// division per step) only as far as the mean + 40 standard deviations + 64
// (xm, kept in the last entry); the entries past it are +inf, filled by the
// whole wave (a draw that reaches them, P < 1e-300, is flagged like any leaf
// past UG_LEAFMAX).
__global__ __launch_bounds__(64) void k_ug_pmt(const UniSet* __restrict__ us, double* __restrict__ pmt) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
  const uint32_t r = blockIdx.x >> 2, cls = blockIdx.x & 3u;
  if (us->loff[r + 1] == us->loff[r] && us->u[r].S == 0) return;
  const UniGen& u = us->u[r];
  if (u.p >= 1.0) return;
  const uint64_t kl = u.W - (u.nb - 1) * u.K, tb = cls >= 2 ? (u.T > 1 ? u.T - 1 : 1) : u.T;
  const uint64_t G = ((cls & 1u) ? kl : u.K) * tb;
  const double mean = (double)G * u.p;
  const double xmd = mean + 40.0 * sqrt(mean) + 64.0;
  const uint64_t xm = xmd < (double)(UG_CDF - 2) ? (uint64_t)xmd : UG_CDF - 2;
  double* t = pmt + (r * 4 + cls) * UG_PMT;
  for (uint64_t x = xm + 1 + threadIdx.x; x < UG_PMT - 1; x += 64) t[x] = __builtin_inf();
  if (threadIdx.x == 0) {
    double pm = cls == 0 ? u.pm[0] : cls == 1 ? u.pm[1] : cls == 2 ? u.pm[2] : u.pm[3];
    double cdf = pm;
    t[0] = cdf;
    for (uint64_t x = 0; x < xm; ++x) {
      if (x < G) {
        pm = pm * (double)(G - x);
        pm = pm / (double)(x + 1);
        pm = pm * u.r;
      } else {
        pm = 0.0;
      }
      cdf = cdf + pm;
      t[x + 1] = cdf;
    }
    t[UG_PMT - 1] = (double)xm;
  }
}

// (references outermost: the generator's fields are wave-uniform, scalar
// loads).  Leaf l of the plan is the generator's leaf lbase[r] + l.
__global__ __launch_bounds__(UB) void k_ug_count(const UniSet* __restrict__ us, uint32_t* __restrict__ cnt,
                                                unsigned int* flags) {
  const uint64_t stride = (uint64_t)gridDim.x * UB;
  for (uint32_t r = 0; r < 6; ++r) {
    const uint64_t g0 = us->loff[r], n = us->loff[r + 1] - g0, lb = us->lbase[r];
    if (!n) continue;
    const UniGen& u = us->u[r];  // (wave-uniform: scalar loads; a by-value copy went to scratch)
    const double* pmt = us->pmt + r * 4 * UG_PMT;
    for (uint64_t l = (uint64_t)blockIdx.x * UB + threadIdx.x; l < n; l += stride) {
      const uint64_t c = uni_count_tab(u, lb + l, pmt);
      if (c > UG_LEAFMAX) atomicOr(flags, FLAG_UNI);
      cnt[g0 + l] = c > UG_LEAFMAX ? UG_LEAFMAX + 1 : (uint32_t)c;
    }
  }
}

// The candidates of the earlier shards (X0) and of all shards (T') of
// reference r, from the gathered summary rows of a key-range pass (rows ==
// nullptr, one GPU: 0 and this plan's own candidates C).
__device__ __forceinline__ void ug_window(const unsigned long long* rows, uint32_t shard, uint32_t ns, uint32_t r,
                                          uint64_t C, uint64_t& X0, uint64_t& Tp) {
  if (!rows) {
    X0 = 0;
    Tp = C;
    return;
  }
  X0 = Tp = 0;
  for (uint32_t x = 0; x < ns; ++x) {
    const unsigned long long v = rows[(uint64_t)x * ROW_W + ROW_N + r];
    Tp += v;
    if (x < shard) X0 += v;
  }
}

// The removal bitmaps (zeroed) over this plan's candidate ranks: the ranks
// F(0 .. T'-S-1) of the removal permutation of all T' candidates that fall in
// [X0, X0 + C), at rank - X0; those below X0 are counted into rem0[r] (every
// shard evaluates the whole removed set, ~10 sqrt(S) ranks).  T' < S, a bitmap
// too small for C, or rows that disagree with this plan's C set FLAG_UNI.
__global__ __launch_bounds__(UB) void k_ug_remove(const UniSet* __restrict__ us, uint32_t* __restrict__ bits,
                                                 const unsigned long long* __restrict__ rows, uint32_t shard,
                                                 uint32_t ns, unsigned long long* __restrict__ rem0,
                                                 unsigned int* flags) {
  const uint64_t stride = (uint64_t)gridDim.x * UB;
  for (uint32_t r = 0; r < 6; ++r) {
    const UniGen& u = us->u[r];
    if (u.S == 0) continue;  // (a reference without samples)
    const uint64_t C = us->pre[us->loff[r + 1]] - us->pre[us->loff[r]];
    uint64_t X0, Tp;
    ug_window(rows, shard, ns, r, C, X0, Tp);
    const bool bad_rows = rows && rows[(uint64_t)shard * ROW_W + ROW_N + r] != C;
    if (Tp < u.S || (C >> 5) >= us->woff[r + 1] - us->woff[r] || bad_rows) {
      if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(flags, FLAG_UNI);
      continue;
    }
    const UniPerm P = uni_perm_make(u, Tp);
    const uint64_t m = Tp - u.S;
    uint32_t below = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * UB + threadIdx.x; i < m; i += stride) {
      const uint64_t y = uni_perm(P, i);
      if (y < X0) {
        ++below;
      } else if (y - X0 < C) {
        const uint64_t z = y - X0;
        atomicOr(&bits[us->woff[r] + (z >> 5)], 1u << (z & 31));
      }
    }
    if (rows) {
      const uint64_t b = sc_wave_red<false>((unsigned long long)below);
      if (__lane_id() == 0 && b) atomicAdd(&rem0[r], (unsigned long long)b);
    }
  }
}

// per reference: the list index of this plan's first survivor (X0 minus the
// removed ranks below X0; 0 on one GPU) and its survivors (C minus the ranks
// removed in its window) -> info[6 + r], info[12 + r]
__global__ void k_ug_info(const UniSet* __restrict__ us, const unsigned long long* __restrict__ rows, uint32_t shard,
                          uint32_t ns, unsigned long long* __restrict__ info) {
  const uint32_t r = threadIdx.x;
  if (r >= 6) return;
  const UniGen& u = us->u[r];
  unsigned long long first = 0, n = 0;
  if (u.S) {
    const uint64_t C = us->pre[us->loff[r + 1]] - us->pre[us->loff[r]];
    uint64_t X0, Tp;
    ug_window(rows, shard, ns, r, C, X0, Tp);
    const uint64_t removed = us->rb[us->woff[r + 1]] - us->rb[us->woff[r]];
    const uint64_t below = rows ? info[r] : 0ull;
    first = X0 >= below ? X0 - below : 0ull;
    n = C >= removed ? C - removed : 0ull;
    if (first > u.S) first = u.S;  // (a flagged plan: kept in range, reported at the fetch)
    if (n > u.S - first) n = u.S - first;
  }
  info[6 + r] = first;
  info[12 + r] = n;
}

// a replayed shard pass took its slice from an earlier identical pass: the
// device's own values must be the same (they are a function of the seed, the
// budget and the shard), else the pass reports a uniform-plan failure
struct UniSlice {
  unsigned long long w[12];  // first[6], n[6]
};
__global__ void k_ug_slice_check(const unsigned long long* __restrict__ info, UniSlice e, unsigned int* flags) {
  const uint32_t k = threadIdx.x;
  if (k < 12 && info[6 + k] != e.w[k]) {
    atomicOr(flags, FLAG_UNI);
#ifdef PLUSS_DEBUG_STAGES
    printf("uniform slice check: word %u device %llu known %llu\n", k, info[6 + k], e.w[k]);
#endif
  }
}

// per leaf: the sample index of its first surviving candidate and their
// number; the leaf holding each tile's first sample
__global__ __launch_bounds__(UB) void k_ug_tiles(const UniSet* __restrict__ us, uint32_t* __restrict__ tmap) {
  const uint64_t stride = (uint64_t)gridDim.x * UB;
  for (uint32_t r = 0; r < 6; ++r) {
    const uint64_t g0 = us->loff[r], n = us->loff[r + 1] - g0;
    const uint64_t tm0 = us->tmoff[r], nt = us->tmoff[r + 1] - tm0;
    for (uint64_t l = (uint64_t)blockIdx.x * UB + threadIdx.x; l < n; l += stride) {
      const uint32_t c = us->cnt[g0 + l];
      if (!c || c > UG_LEAFMAX) continue;
      const uint64_t x0 = uni_pre(us, r, l);
      const uint64_t b0 = uni_removed_before(us, r, x0), b1 = uni_removed_before(us, r, x0 + c);
      const uint64_t f = x0 - b0, kept = c - (b1 - b0);
      for (uint64_t t = (f + UG_TILE - 1) / UG_TILE; t * UG_TILE < f + kept && t < nt; ++t) tmap[tm0 + t] = (uint32_t)l;
    }
  }
}

// materialised list: samples [first, first + n) of reference r, one tile per workgroup
__global__ __launch_bounds__(UB) void k_ug_expand(const UniSet* __restrict__ us, uint32_t r, uint64_t first,
                                                 uint64_t n, uint64_t S, uint64_t* __restrict__ out,
                                                 unsigned int* flags) {
  __shared__ unsigned long long raw[UG_TILE];
  __shared__ uint32_t cand[UG_CAND];
  const uint64_t lt = first / UG_TILE + blockIdx.x;
  const uint64_t t0 = lt * UG_TILE;
  const uint32_t mt = (uint32_t)(S - t0 < UG_TILE ? S - t0 : UG_TILE);
  uni_stage<UB, false>(us, r, lt, mt, raw, cand, flags, [](uint32_t e) { return e; });
  for (uint32_t e = threadIdx.x; e < mt; e += UB) {
    const uint64_t i = t0 + e;
    if (i >= first && i < first + n) out[i - first] = raw[e];
  }
}

__global__ void k_ug_setup(const UniSet h, UniSet* d) { *d = h; }

// diagnostics (pluss_diag_uniform_parts): every full tile staged, nothing scanned
template <bool DEC>
__global__ __launch_bounds__(UB) __attribute__((amdgpu_waves_per_eu(4))) void k_ug_stage_only(
    const UniSet* __restrict__ us, UniDec dz, uint64_t* __restrict__ out) {
  __shared__ unsigned long long raw[UG_TILE], tab[DEC ? 294 : 1];  // (tab: the faithful scan's 2352 B)
  __shared__ uint32_t cand[UG_CAND];
  const uint64_t gt = blockIdx.x;
  uint32_t r = 0;
  for (uint32_t x = 1; x < 6; ++x) r += gt >= us->tmoff[x] ? 1u : 0u;
  r = __builtin_amdgcn_readfirstlane(r);
  const uint64_t lt = gt - us->tmoff[r], S = us->u[r].S;
  if ((lt + 1) * UG_TILE > S) return;  // (full tiles only)
  uni_stage<UB, DEC>(us, r, lt, UG_TILE, raw, cand, us->flags, [](uint32_t e) { return e; }, dz, tab, DEC ? 294u : 0u);
  if (threadIdx.x == 0) out[gt] = raw[0] ^ raw[UG_TILE - 1];
}

static int ug_grow(void** p, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return PLUSS_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, bytes) != hipSuccess) {
    set_error("hipMalloc failed for the uniform generator's plan");
    return PLUSS_ERR_ALLOC;
  }
  *cap = bytes;
  return PLUSS_OK;
}

int uni_check(const pluss_ctx* ctx, int32_t ref, uint64_t total, const char* api) {
  const pluss_cfg& c = ctx->cfg;
  if ((uint64_t)c.n % ((uint64_t)c.chunk * (uint64_t)c.threads) != 0) {
    set_error(std::string(api) + ": needs N % (chunk*threads) == 0 (key order)");
    return PLUSS_ERR_CONFIG;
  }
  const uint64_t span = c.range_full ? (uint64_t)c.n : (uint64_t)c.n - 1;
  const uint64_t D = (ref == PLUSS_C0 || ref == PLUSS_C1) ? span * span : span * span * span;
  const double E = (double)total + 10.0 * std::sqrt((double)total) + 32.0;
  if (total < 1 || total > D || E >= 4294967296.0) {
    set_error(std::string(api) + ": needs 1 <= total <= span^d and total + 10 sqrt(total) + 32 < 2^32");
    return PLUSS_ERR_CONFIG;
  }
  return PLUSS_OK;
}

// The plan, in three parts on stream s (ctx->ub; valid until the next plan on
// this handle):
//   uni_plan_count   the generators, this plan's leaves of each reference
//                    (one GPU: all of them; key-range shard `shard` of `ns`:
//                    the leaves [L*shard/ns, L*(shard+1)/ns)), their candidate
//                    counts and the counts' prefix;
//   uni_plan_remove  the removal bitmap over this plan's candidates (rows: the
//                    gathered summary rows of the shards' candidate counts,
//                    nullptr on one GPU), its prefix, and per reference the
//                    list index of the plan's first survivor and their number
//                    (ub.info[6 + r], [12 + r]);
//   uni_plan_tiles   the leaf holding each tile's first sample for n[r]
//                    samples per reference; *out = the device UniSet.
int uni_plan_count(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, uint32_t shard, uint32_t ns, hipStream_t s) {
  UniBufs& b = ctx->ub;
  if (!b.host) b.host = new UniSet();
  UniSet& h = *b.host;
  std::memset((void*)&h, 0, sizeof h);
  uint64_t L = 0, Wd = 0;
  for (int r = 0; r < 6; ++r) {
    h.loff[r] = L;
    h.woff[r] = Wd;
    if (!totals[r]) continue;
    if (int rc = uni_check(ctx, r, totals[r], "uniform key-order lists")) return rc;
    h.u[r] = make_unigen((uint64_t)ctx->cfg.n, (uint64_t)ctx->cfg.threads, (uint64_t)ctx->cfg.chunk,
                         ctx->cfg.range_full != 0, seed, (uint32_t)r, totals[r]);
    const uint64_t Lr = h.u[r].L;
    const uint64_t la = (uint64_t)((unsigned __int128)Lr * shard / ns), lb = (uint64_t)((unsigned __int128)Lr * (shard + 1) / ns);
    h.lbase[r] = la;
    L += lb - la;
    // room for this plan's candidates: their mean plus 20 standard deviations (or every point when p = 1)
    const double pts = std::min((double)h.u[r].D, (double)(lb - la) * (double)h.u[r].K * (double)h.u[r].T);
    const double E = h.u[r].p * pts;
    const uint64_t tmax = (uint64_t)(E + 20.0 * std::sqrt(E) + 1024.0);
    Wd += tmax / 32 + 2;
  }
  h.loff[6] = L;
  h.woff[6] = Wd;
  const uint64_t nbL = (L + UBATCH - 1) / UBATCH + 1, nbW = (Wd + UBATCH - 1) / UBATCH + 1;
  int rc = PLUSS_OK;
  if (!b.set) rc = ug_grow((void**)&b.set, &b.set_cap, sizeof(UniSet));
  if (!rc && !b.info) rc = ug_grow((void**)&b.info, &b.info_cap, UI_W * 8);
  if (!rc) rc = ug_grow((void**)&b.cnt, &b.cnt_cap, (L + 1) * 4);
  if (!rc) rc = ug_grow((void**)&b.pre, &b.pre_cap, (L + 1) * 8);
  if (!rc) rc = ug_grow((void**)&b.bits, &b.bits_cap, (Wd + 1) * 4);
  if (!rc) rc = ug_grow((void**)&b.rb, &b.rb_cap, (Wd + 1) * 8);
  if (!rc) {
    void* before = b.pmt;
    rc = ug_grow((void**)&b.pmt, &b.pmt_cap, 6 * 4 * UG_PMT * sizeof(double));
    if (b.pmt != before) b.pmt_valid = false;
  }
  if (!rc) rc = ug_grow((void**)&b.bsum, &b.bsum_cap, (nbL > nbW ? nbL : nbW) * 8 + 8);
  if (rc) return rc;
  if (!b.hinfo && hipHostMalloc((void**)&b.hinfo, UI_W * 8) != hipSuccess) {
    b.hinfo = nullptr;
    set_error("hipHostMalloc failed for the uniform generator's plan");
    return PLUSS_ERR_ALLOC;
  }
  h.cnt = b.cnt;
  h.pre = b.pre;
  h.bits = b.bits;
  h.rb = b.rb;
  h.tmap = b.tmap;
  h.pmt = b.pmt;
  h.flags = ctx->g.flags;
  // the plan's parameters travel as a kernel argument (ordered on the stream, no host buffer to keep)
  hipLaunchKernelGGL(k_ug_setup, dim3(1), dim3(1), 0, s, h, b.set);
  const int grid = (int)std::min<uint64_t>((L + UB - 1) / UB + 1, 4096);
  // the CDF tables depend on the shape and the sample counts only (p and the
  // four leaf sizes of each reference), not on the seed or the shard: kept
  // while they stay the same
  uint64_t key[6][10];
  std::memset(key, 0, sizeof key);
  for (int r = 0; r < 6; ++r) {
    const UniGen& g = h.u[r];
    if (!g.S) continue;
    std::memcpy(&key[r][0], &g.p, 8);
    std::memcpy(&key[r][1], &g.r, 8);
    key[r][2] = g.K;
    key[r][3] = g.W;
    key[r][4] = g.nb;
    key[r][5] = g.T;
    std::memcpy(&key[r][6], g.pm, 32);
  }
  if (!b.pmt_valid || std::memcmp(key, b.pmt_key, sizeof key) != 0) {
    hipLaunchKernelGGL(k_ug_pmt, dim3(24), dim3(64), 0, s, (const UniSet*)b.set, b.pmt);
    std::memcpy(b.pmt_key, key, sizeof key);
    b.pmt_valid = true;
  }
  hipLaunchKernelGGL(k_ug_count, dim3(grid), dim3(UB), 0, s, (const UniSet*)b.set, b.cnt, ctx->g.flags);
  if (int e = ug_scan(b.cnt, L, b.bsum, b.pre, 0, s)) return e;
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int uni_plan_remove(pluss_ctx* ctx, const unsigned long long* rows, uint32_t shard, uint32_t ns, hipStream_t s) {
  UniBufs& b = ctx->ub;
  const uint64_t Wd = b.host->woff[6];
  PLUSS_HIP_CHECK(hipMemsetAsync(b.bits, 0, (Wd + 1) * 4, s));
  PLUSS_HIP_CHECK(hipMemsetAsync(b.info, 0, UI_W * 8, s));
  hipLaunchKernelGGL(k_ug_remove, dim3(1024), dim3(UB), 0, s, (const UniSet*)b.set, b.bits, rows, shard, ns, b.info,
                     ctx->g.flags);
  if (int e = ug_scan(b.bits, Wd, b.bsum, b.rb, 1, s)) return e;
  hipLaunchKernelGGL(k_ug_info, dim3(1), dim3(64), 0, s, (const UniSet*)b.set, rows, shard, ns, b.info);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int uni_plan_tiles(pluss_ctx* ctx, const uint64_t* n, hipStream_t s, const UniSet** out) {
  UniBufs& b = ctx->ub;
  UniSet& h = *b.host;
  uint64_t Tt = 0;
  for (int r = 0; r < 6; ++r) {
    h.tmoff[r] = Tt;
    Tt += fa_tiles(n[r]);
  }
  h.tmoff[6] = Tt;
  if (int rc = ug_grow((void**)&b.tmap, &b.tmap_cap, (Tt + 1) * 4)) return rc;
  h.tmap = b.tmap;
  hipLaunchKernelGGL(k_ug_setup, dim3(1), dim3(1), 0, s, h, b.set);
  PLUSS_HIP_CHECK(hipMemsetAsync(b.tmap, 0, (Tt + 1) * 4, s));
  const uint64_t L = h.loff[6];
  const int grid = (int)std::min<uint64_t>((L + UB - 1) / UB + 1, 4096);
  hipLaunchKernelGGL(k_ug_tiles, dim3(grid), dim3(UB), 0, s, (const UniSet*)b.set, b.tmap);
  PLUSS_HIP_CHECK(hipGetLastError());
  *out = b.set;
  return PLUSS_OK;
}

int uni_slice_check(pluss_ctx* ctx, const uint64_t* known, hipStream_t s) {
  UniSlice e;
  for (int k = 0; k < 12; ++k) e.w[k] = known[k];
  hipLaunchKernelGGL(k_ug_slice_check, dim3(1), dim3(64), 0, s, (const unsigned long long*)ctx->ub.info, e,
                     ctx->g.flags);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

void uni_free(pluss_ctx* ctx) {
  UniBufs& b = ctx->ub;
  void* ub[] = {b.set, b.cnt, b.bits, b.tmap, b.pre, b.rb, b.bsum, b.pmt, b.info};
  for (void* p : ub)
    if (p) (void)hipFree(p);
  if (b.hinfo) (void)hipHostFree(b.hinfo);
  delete b.host;
  b = UniBufs();
}

// The whole plan of the lists on one GPU (every leaf; n = totals)
int uni_plan(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, hipStream_t s, const UniSet** out) {
  if (int rc = uni_plan_count(ctx, seed, totals, 0, 1, s)) return rc;
  if (int rc = uni_plan_remove(ctx, nullptr, 0, 1, s)) return rc;
  return uni_plan_tiles(ctx, totals, s, out);
}

int diag_uniform_parts(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, int32_t what, uint64_t* d_out,
                       hipStream_t s) {
  const UniSet* us = nullptr;
  if (int rc = uni_plan(ctx, seed, totals, s, &us)) return rc;
  if (what == 0) return PLUSS_OK;
  const Model& m = ctx->m;
  uint32_t nsh = 0, tsh = 0;
  while ((1ull << nsh) < m.N) ++nsh;
  while ((1ull << tsh) < m.T) ++tsh;
  const UniDec dz{(uint32_t)m.N, (uint32_t)m.W - 1u, (uint32_t)(m.N / m.T), (uint32_t)m.S, nsh, tsh};
  const unsigned tiles = (unsigned)ctx->ub.host->tmoff[6];
  if (!tiles) return PLUSS_OK;
  if (what == 1) hipLaunchKernelGGL(k_ug_stage_only<true>, dim3(tiles), dim3(UB), 0, s, us, dz, d_out);
  else hipLaunchKernelGGL(k_ug_stage_only<false>, dim3(tiles), dim3(UB), 0, s, us, dz, d_out);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_expand_uniform_sorted(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first,
                                 uint64_t n, uint64_t* d_out, hipStream_t s) {
  if (int rc = uni_check(ctx, ref, total, "pluss_dev_expand_uniform_sorted")) return rc;
  if (first > total || n > total - first) {
    set_error("pluss_dev_expand_uniform_sorted: [first, first + n) exceeds the list");
    return PLUSS_ERR_CONFIG;
  }
  if (!n) return PLUSS_OK;
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  t[ref] = total;
  const UniSet* us = nullptr;
  if (int rc = uni_plan(ctx, seed, t, s, &us)) return rc;
  const uint64_t tiles = (first + n - 1) / UG_TILE - first / UG_TILE + 1;
  hipLaunchKernelGGL(k_ug_expand, dim3((unsigned)tiles), dim3(UB), 0, s, us, (uint32_t)ref, first, n, total,
                     d_out, ctx->g.flags);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

}  // namespace pluss
