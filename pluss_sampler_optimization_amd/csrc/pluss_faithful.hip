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
//   start_j  <=>  j == 0 || key_j > pmax_{j-1}               (new START_SAMPLE)
//   Q1 (r10:356): first start j > 0 with (j - starts_before_j) >= S - j  -> drop [j, S)
//   Q2 (r10:669-674): cold samples count only when tid == 0
//   Q3 (r10:345): if nothing was dropped and no sample is cold, the sample owning
//                 the largest sink is left in LAT: +1 cold if its tid == 0
//   traversed (r10:694) = sum over replays of (end key - start key), end key =
//                 the replay's last sink, or A*T for a replay that runs to the end.
//
// Validated against the reference's own dumps (tests/golden/r10_*, 42/42).
#include <hip/hip_runtime.h>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "pluss_device.h"

namespace pluss {

template <bool FAST>
__global__ __launch_bounds__(BLOCK) void k_faith_keys(Model m, uint32_t ref, const uint64_t* __restrict__ smp,
                                                      uint64_t n, unsigned long long* __restrict__ keys,
                                                      unsigned long long* __restrict__ sinks, GTable g) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
    const Sample s = unpack(smp[i]);
    if (s.ref != ref || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N) {
      atomicOr(&g.flags[1], 1u);
      keys[i] = KEY_EMPTY;
      sinks[i] = KEY_EMPTY;
      continue;
    }
    const uint32_t c2 = (ref == C0 || ref == C1) ? 0u : s.c2;
    const int64_t ri = ri_of<FAST>(m, ref, s.c0, s.c1, c2);
    uint64_t P;
    uint32_t t;
    position(m, ref, s.c0, s.c1, c2, &P, &t);
    keys[i] = P * m.T + t;
    sinks[i] = ri < 0 ? KEY_EMPTY : (P + (uint64_t)ri) * m.T + t;
  }
}

__global__ void k_faith_init(unsigned long long* scal, uint64_t n) {
  scal[0] = n;  // cut
  scal[1] = 0;  // cold (tid 0)
  scal[2] = 0;  // traversed (mod 2^64)
}

__global__ __launch_bounds__(BLOCK) void k_faith_flags(const unsigned long long* __restrict__ keys,
                                                       const unsigned long long* __restrict__ pmax, uint64_t n,
                                                       unsigned int* __restrict__ flags) {
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (uint64_t)gridDim.x * BLOCK)
    flags[j] = (j == 0 || keys[j] > pmax[j - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(BLOCK) void k_faith_cut(const unsigned int* __restrict__ flags,
                                                     const unsigned int* __restrict__ nstart, uint64_t n,
                                                     unsigned long long* scal) {
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (uint64_t)gridDim.x * BLOCK) {
    if (j > 0 && flags[j]) {
      const uint64_t met = j - ((uint64_t)nstart[j] - 1);  // samples met before this START
      if (met >= n - j) atomicMin(&scal[0], (unsigned long long)j);
    }
  }
}

template <bool FAST>
__global__ __launch_bounds__(BLOCK) void k_faith_hist(Model m, uint32_t ref, const unsigned long long* __restrict__ keys,
                                                      const unsigned long long* __restrict__ sinks,
                                                      const unsigned long long* __restrict__ pmax,
                                                      const unsigned int* __restrict__ flags, uint64_t n,
                                                      unsigned long long* scal, GTable g) {
  __shared__ unsigned long long tk[TCAP];
  __shared__ unsigned int tc[TCAP];
  __shared__ unsigned long long red[2];
  const BlockTable bt{tk, tc};
  bt_init(bt);
  WaveCache wc;
  wc_init(wc);
  if (threadIdx.x == 0) red[0] = red[1] = 0;
  __syncthreads();
  const uint64_t cut = scal[0];
  const uint64_t endkey = m.A * m.T;
  unsigned long long cold = 0, trav = 0;
  const uint64_t step = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t base = (uint64_t)blockIdx.x * BLOCK; base < cut; base += step) {
    const uint64_t j = base + threadIdx.x;
    const bool v = j < cut;
    uint64_t key = KEY_NONE;
    bool rec = false;
    if (v) {
      const unsigned long long k = keys[j], s = sinks[j];
      if (s == KEY_EMPTY) {
        cold += (k % m.T == 0) ? 1u : 0u;
      } else {
        const int64_t ri = (int64_t)((s - k) / m.T);
        key = make_key(ref, share_kind(m, ref, ri), ri);
        rec = true;
      }
      if (flags[j]) trav -= k;
      if (j + 1 == cut || flags[j + 1]) trav += (pmax[j] == KEY_EMPTY) ? endkey : pmax[j];
    }
    wave_count(wc, bt, g, key, rec);
  }
  atomicAdd(&red[0], cold);
  atomicAdd(&red[1], trav);
  bt_finish(wc, bt, g);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&scal[1], red[0]);
    atomicAdd(&scal[2], red[1]);
  }
}

__global__ void k_faith_finish(Model m, uint32_t ref, uint64_t n, const unsigned long long* pmax,
                               const unsigned long long* scal, GTable g) {
  unsigned long long cold = scal[1];
  const uint64_t cut = scal[0];
  if (n > 0 && cut == n && pmax[n - 1] != KEY_EMPTY && (pmax[n - 1] % m.T) == 0) cold += 1;  // Q3
  g_add(g, make_key(ref, 0, -1), cold);  // the reference always materialises key -1 (r10:671)
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

int launch_faithful(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, hipStream_t s) {
  const Model& m = ctx->m;
  if ((uint64_t)ctx->cfg.n % ((uint64_t)ctx->cfg.chunk * (uint64_t)ctx->cfg.threads) != 0) {
    set_error("faithful mode needs N % (chunk*threads) == 0 (lockstep interleaving order)");
    return PLUSS_ERR_CONFIG;
  }
  FaithfulBufs& b = ctx->fb;
  if (!b.scal) {
    if (int rc = grow(&b.scal, 4)) return rc;
  }
  if (n == 0) return PLUSS_OK;
  ctx->tables_dirty = true;
  if (n > 0xFFFFFFFFull) {
    set_error("faithful mode: at most 2^32-1 samples per reference");
    return PLUSS_ERR_CONFIG;
  }
  if (n > b.cap) {
    PLUSS_HIP_CHECK(hipStreamSynchronize(s));
    int rc = 0;
    if ((rc = grow(&b.keys, n)) || (rc = grow(&b.sinks, n)) || (rc = grow(&b.keys_s, n)) ||
        (rc = grow(&b.sinks_s, n)) || (rc = grow(&b.pmax, n)) || (rc = grow(&b.flags, n)) || (rc = grow(&b.nstart, n)))
      return rc;
    b.cap = n;
  }
  // key range: keys < A*T, so sort only the significant bits
  unsigned end_bit = 1;
  while (end_bit < 64 && (m.A * m.T) >> end_bit) ++end_bit;
  size_t need = 0, t1 = 0, t2 = 0, t3 = 0;
  PLUSS_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, t1, b.keys, b.keys_s, b.sinks, b.sinks_s, n, 0, end_bit, s));
  PLUSS_HIP_CHECK(rocprim::inclusive_scan(nullptr, t2, b.sinks_s, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
  PLUSS_HIP_CHECK(rocprim::inclusive_scan(nullptr, t3, b.flags, b.nstart, n, rocprim::plus<unsigned int>(), s));
  need = t1 > t2 ? t1 : t2;
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
  const int nb = (int)((n + BLOCK * 4 - 1) / (BLOCK * 4) < (uint64_t)MAX_BLOCKS ? (n + BLOCK * 4 - 1) / (BLOCK * 4)
                                                                               : MAX_BLOCKS);
  const int grid = nb < 1 ? 1 : nb;
  if (m.fast)
    hipLaunchKernelGGL(k_faith_keys<true>, dim3(grid), dim3(BLOCK), 0, s, m, (uint32_t)ref, d_samples, n, b.keys,
                       b.sinks, ctx->g);
  else
    hipLaunchKernelGGL(k_faith_keys<false>, dim3(grid), dim3(BLOCK), 0, s, m, (uint32_t)ref, d_samples, n, b.keys,
                       b.sinks, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  size_t sz = b.tmp_bytes;
  PLUSS_HIP_CHECK(rocprim::radix_sort_pairs(b.tmp, sz, b.keys, b.keys_s, b.sinks, b.sinks_s, n, 0, end_bit, s));
  sz = b.tmp_bytes;
  PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, b.sinks_s, b.pmax, n, rocprim::maximum<unsigned long long>(), s));
  hipLaunchKernelGGL(k_faith_flags, dim3(grid), dim3(BLOCK), 0, s, b.keys_s, b.pmax, n, b.flags);
  PLUSS_HIP_CHECK(hipGetLastError());
  sz = b.tmp_bytes;
  PLUSS_HIP_CHECK(rocprim::inclusive_scan(b.tmp, sz, b.flags, b.nstart, n, rocprim::plus<unsigned int>(), s));
  hipLaunchKernelGGL(k_faith_init, dim3(1), dim3(1), 0, s, b.scal, n);
  hipLaunchKernelGGL(k_faith_cut, dim3(grid), dim3(BLOCK), 0, s, b.flags, b.nstart, n, b.scal);
  if (m.fast)
    hipLaunchKernelGGL(k_faith_hist<true>, dim3(grid), dim3(BLOCK), 0, s, m, (uint32_t)ref, b.keys_s, b.sinks_s, b.pmax,
                       b.flags, n, b.scal, ctx->g);
  else
    hipLaunchKernelGGL(k_faith_hist<false>, dim3(grid), dim3(BLOCK), 0, s, m, (uint32_t)ref, b.keys_s, b.sinks_s,
                       b.pmax, b.flags, n, b.scal, ctx->g);
  hipLaunchKernelGGL(k_faith_finish, dim3(1), dim3(1), 0, s, m, (uint32_t)ref, n, b.pmax, b.scal, ctx->g);
  PLUSS_HIP_CHECK(hipGetLastError());
  return PLUSS_OK;
}

}  // namespace pluss
