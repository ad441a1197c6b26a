// pluss_kernels.hip — gfx950 kernels of the PLUSS reuse-interval hot path.
//
//   k_sampled_hist  (HOT)  one lane per sampled access: decode the packed
//                   sample, jump to its next same-line touch on the simulated
//                   static schedule (pluss_model.h), and count the exact
//                   (ref, noshare/share, RI) key in an LDS-privatised
//                   open-addressing table.  Lanes with equal keys are merged
//                   by a wave ballot first, so one LDS atomic is issued per
//                   distinct key per wave.  Replaces the replay loop of
//                   r10 sampler_<REF> (r10:275-654) + pluss_parallel_histogram_update
//                   (pluss_utils.h:726-729).
//   k_fulltrace     every access of the nest, indices generated in-kernel (no
//                   HBM input); replaces seq.cpp:37-333 / rayon.rs:186-378.
//   k_slab_reduce   merges the per-workgroup tables into the handle's global table.
//   k_export        canonical (sorted) table for host fetch / cross-GPU merge.
//   k_ri_dump       per-sample (RI, sink key) parity dump.
//   k_expand        the sample-list bijection (pluss_model.h).
#include <hip/hip_runtime.h>

#include "pluss_device.h"

namespace pluss {

// ------------------------------------------------------------------ HOT --
template <bool FAST>
__global__ __launch_bounds__(BLOCK) void k_sampled_hist(Model m, const uint64_t* __restrict__ smp, uint64_t n,
                                                        const uint64_t* __restrict__ head, Slabs slabs, GTable g) {
  __shared__ unsigned long long tk[TCAP];
  __shared__ unsigned int tc[TCAP];
  __shared__ unsigned int nf;
  table_init(tk, tc);
  if (threadIdx.x == 0) nf = 0;
  __syncthreads();

  const uint64_t npairs = n >> 1;
  const ulonglong2* __restrict__ v = reinterpret_cast<const ulonglong2*>(smp);
  const uint64_t step = (uint64_t)gridDim.x * BLOCK * UNROLL;
  bool anybad = false;
  for (uint64_t base = (uint64_t)blockIdx.x * BLOCK * UNROLL; base < npairs; base += step) {
    ulonglong2 x[UNROLL];
    bool ok[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t i = base + (uint64_t)u * BLOCK + threadIdx.x;
      ok[u] = i < npairs;
      x[u] = ok[u] ? v[i] : ulonglong2{0, 0};
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      bool b0, b1;
      const uint64_t k0 = sample_key<FAST>(m, x[u].x, &b0);
      const uint64_t k1 = sample_key<FAST>(m, x[u].y, &b1);
      anybad |= ok[u] && (b0 || b1);
      wave_insert(tk, tc, g, k0, ok[u] && !b0);
      wave_insert(tk, tc, g, k1, ok[u] && !b1);
    }
  }
  if (((n & 1) || head) && blockIdx.x == 0 && threadIdx.x < 64) {
    // odd tail (lane 0) and, for an 8-byte-aligned list, its first sample (lane 1)
    bool b = false;
    const bool mine = (threadIdx.x == 0 && (n & 1)) || (threadIdx.x == 1 && head);
    const uint64_t k = mine ? sample_key<FAST>(m, threadIdx.x == 0 ? smp[n - 1] : *head, &b) : KEY_EMPTY;
    anybad |= mine && b;
    wave_insert(tk, tc, g, k, mine && !b);
  }
  if (anybad) atomicOr(&g.flags[1], 1u);
  __syncthreads();
  table_flush(tk, tc, &nf, slabs);
}

// ----------------------------------------------------------- full trace --
template <bool FAST>
__global__ __launch_bounds__(BLOCK) void k_fulltrace(Model m, Slabs slabs, GTable g) {
  __shared__ unsigned long long tk[TCAP];
  __shared__ unsigned int tc[TCAP];
  __shared__ unsigned int nf;
  table_init(tk, tc);
  if (threadIdx.x == 0) nf = 0;
  __syncthreads();
  const uint32_t lane = __lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * (BLOCK / 64);
  const uint64_t npairs = (uint64_t)m.N * m.N;
  for (uint64_t pr = (uint64_t)blockIdx.x * (BLOCK / 64) + threadIdx.x / 64; pr < npairs; pr += nwaves) {
    const uint32_t c0 = (uint32_t)(pr / m.N), c1 = (uint32_t)(pr - (uint64_t)c0 * m.N);
    {  // C0, C1 of this (c0, c1)
      const bool v = lane < 2;
      uint64_t key = KEY_EMPTY;
      if (v) {
        const int64_t ri = ri_of<FAST>(m, lane, c0, c1, 0);
        key = make_key(lane, 0, ri);
      }
      wave_insert(tk, tc, g, key, v);
    }
    for (uint32_t c2b = 0; c2b < m.N; c2b += 64) {
      const uint32_t c2 = c2b + lane;
      const bool v = c2 < m.N;
#pragma unroll
      for (uint32_t ref = A0; ref <= C3; ++ref) {
        uint64_t key = KEY_EMPTY;
        if (v) {
          const int64_t ri = ri_of<FAST>(m, ref, c0, c1, c2);
          key = make_key(ref, share_kind(m, ref, ri), ri);
        }
        wave_insert(tk, tc, g, key, v);
      }
    }
  }
  __syncthreads();
  table_flush(tk, tc, &nf, slabs);
}

// --------------------------------------------------------- slab reduce --
constexpr int RCAP = 1024;
__global__ __launch_bounds__(BLOCK) void k_slab_reduce(Slabs slabs, int nslabs, GTable g) {
  __shared__ unsigned long long tk[RCAP];
  __shared__ unsigned long long tc[RCAP];
  for (int i = threadIdx.x; i < RCAP; i += BLOCK) {
    tk[i] = KEY_EMPTY;
    tc[i] = 0;
  }
  __syncthreads();
  for (int b = blockIdx.x; b < nslabs; b += gridDim.x) {
    const unsigned int cnt = slabs.n[b];
    for (unsigned int i = threadIdx.x; i < cnt; i += BLOCK) {
      const uint64_t k = slabs.keys[(size_t)b * TCAP + i];
      const unsigned long long c = slabs.counts[(size_t)b * TCAP + i];
      if (!lds_add<unsigned long long, RCAP>(tk, tc, k, c)) g_add(g, k, c);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < RCAP; i += BLOCK)
    if (tk[i] != KEY_EMPTY) g_add(g, tk[i], tc[i]);
}

// --------------------------------------------------------------- export --
constexpr int EXP_THREADS = 1024;
__global__ __launch_bounds__(EXP_THREADS) void k_export(GTable g, unsigned long long* ok, unsigned long long* oc,
                                                       uint64_t cap, unsigned int* nout) {
  __shared__ unsigned long long sk[GCAP];
  __shared__ unsigned long long sc[GCAP];
  __shared__ unsigned int cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < GCAP; i += EXP_THREADS) {
    const unsigned long long k = g.keys[i];
    if (k != KEY_EMPTY) {
      const unsigned int p = atomicAdd(&cnt, 1u);
      sk[p] = k;
      sc[p] = g.counts[i];
    }
  }
  __syncthreads();
  const uint32_t n = cnt;
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t i = n + threadIdx.x; i < P; i += EXP_THREADS) {
    sk[i] = KEY_EMPTY;
    sc[i] = 0;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += EXP_THREADS) {
        const uint32_t ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const unsigned long long a = sk[i], b = sk[ixj];
          if ((a > b) == up) {
            sk[i] = b;
            sk[ixj] = a;
            const unsigned long long t = sc[i];
            sc[i] = sc[ixj];
            sc[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint64_t i = threadIdx.x; i < cap; i += EXP_THREADS) {
    ok[i] = i < n ? sk[i] : KEY_EMPTY;
    oc[i] = i < n ? sc[i] : 0ull;
  }
  if (threadIdx.x == 0) {
    *nout = n;
    if (n > cap) atomicOr(&g.flags[0], 2u);
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
    uint64_t y = perm_apply(p, first + i);
    uint64_t c2 = 0;
    if (p.dim3) {
      c2 = y % p.span;
      y /= p.span;
    }
    const uint64_t c1 = y % p.span, c0 = y / p.span;
    out[i] = pack(ref, (uint32_t)c0, (uint32_t)c1, (uint32_t)c2);
  }
}

// ------------------------------------------------------------ launchers --
static int grid_for(uint64_t work, uint64_t per_block) {
  uint64_t b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > (uint64_t)MAX_BLOCKS) b = MAX_BLOCKS;
  return (int)b;
}

int launch_table_reset(pluss_ctx* ctx, hipStream_t s) {
  ctx->slabs_pending = 0;  // pending partial tables belong to the histogram being discarded
  PLUSS_HIP_CHECK(hipMemsetAsync(ctx->g.keys, 0xFF, GCAP * sizeof(unsigned long long), s));
  PLUSS_HIP_CHECK(hipMemsetAsync(ctx->g.counts, 0, GCAP * sizeof(unsigned long long), s));
  PLUSS_HIP_CHECK(hipMemsetAsync(ctx->g.flags, 0, 4 * sizeof(unsigned int), s));
  PLUSS_HIP_CHECK(hipMemsetAsync(ctx->d_trav, 0, 8 * sizeof(unsigned long long), s));
  return PLUSS_OK;
}

// The per-workgroup tables of the last sampling launch are merged lazily, just
// before the slabs are reused or the table is read, so the sampling kernel can
// be timed on its own.
int flush_slabs(pluss_ctx* ctx, hipStream_t s) {
  const int nblocks = ctx->slabs_pending;
  if (!nblocks) return PLUSS_OK;
  ctx->slabs_pending = 0;
  const int rg = nblocks < 64 ? nblocks : 64;
  hipLaunchKernelGGL(k_slab_reduce, dim3(rg), dim3(BLOCK), 0, s, ctx->slabs, nblocks, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_sampled_hist(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, hipStream_t s) {
  if (n == 0) return PLUSS_OK;
  if (((uintptr_t)d_samples & 7u) != 0) {
    set_error("pluss_dev_sampled_hist: sample buffer must be 8-byte aligned");
    return PLUSS_ERR_INPUT;
  }
  if (int rc = flush_slabs(ctx, s)) return rc;
  const uint64_t* head = nullptr;
  if (((uintptr_t)d_samples & 15u) != 0) {  // peel one sample so the pairs are 16-byte aligned
    head = d_samples;
    ++d_samples;
    --n;
  }
  const int nb = grid_for((n >> 1) ? (n >> 1) : 1, (uint64_t)BLOCK * UNROLL);
  if (ctx->m.fast)
    hipLaunchKernelGGL(k_sampled_hist<true>, dim3(nb), dim3(BLOCK), 0, s, ctx->m, d_samples, n, head, ctx->slabs,
                       ctx->g);
  else
    hipLaunchKernelGGL(k_sampled_hist<false>, dim3(nb), dim3(BLOCK), 0, s, ctx->m, d_samples, n, head, ctx->slabs,
                       ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->slabs_pending = nb;
  return PLUSS_OK;
}

int launch_fulltrace(pluss_ctx* ctx, hipStream_t s) {
  if (int rc = flush_slabs(ctx, s)) return rc;
  const uint64_t npairs = (uint64_t)ctx->m.N * ctx->m.N;
  const int nb = grid_for(npairs, BLOCK / 64 * 8);
  if (ctx->m.fast)
    hipLaunchKernelGGL(k_fulltrace<true>, dim3(nb), dim3(BLOCK), 0, s, ctx->m, ctx->slabs, ctx->g);
  else
    hipLaunchKernelGGL(k_fulltrace<false>, dim3(nb), dim3(BLOCK), 0, s, ctx->m, ctx->slabs, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  ctx->slabs_pending = nb;
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
  const int nb = grid_for(n, BLOCK * 4);
  hipLaunchKernelGGL(k_expand, dim3(nb), dim3(BLOCK), 0, s, p, (uint32_t)ref, first, n, d_out);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

int launch_export(pluss_ctx* ctx, unsigned long long* d_keys, unsigned long long* d_counts, uint64_t cap,
                  hipStream_t s) {
  if (int rc = flush_slabs(ctx, s)) return rc;
  hipLaunchKernelGGL(k_export, dim3(1), dim3(EXP_THREADS), 0, s, ctx->g, d_keys, d_counts, cap, ctx->d_exp_n);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

}  // namespace pluss
