// pluss_device.h — device helpers shared by the kernel translation units:
// the exact-key histogram path (wave ballot -> per-wave scalar cache -> LDS
// table -> one of NREP global replica tables) and the handle's global table.
//
// Exact keys are required for bit-exact parity (SURVEY.md §7 hard part 2), but
// a GEMM sampler produces only a handful of distinct (ref, kind, RI) keys, and a
// wave's 64 samples usually share one or two of them.  So:
//   1. wave_count(): lanes with equal keys are counted by one ballot+popcount;
//   2. the (key, count) pair goes to a 4-entry cache held in SGPRs by the wave
//      (pure scalar compares and adds, no LDS latency on the hot path);
//   3. cache evictions and the end-of-block flush go to an LDS open-addressing
//      table, and each workgroup finally adds its few table entries into one of
//      NREP global replicas (blockIdx % NREP) so the end-of-kernel atomics are
//      spread over NREP addresses per key.  k_export folds the replicas.
#pragma once
#include <hip/hip_runtime.h>

#include "pluss_internal.h"

namespace pluss {

__device__ __forceinline__ uint32_t slot_hash(uint64_t k, uint32_t cap) {
  uint32_t h = (uint32_t)k * 0x9E3779B1u ^ (uint32_t)(k >> 32) * 0x85EBCA77u;
  h ^= h >> 15;
  return h & (cap - 1);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// Insert into a global open-addressing table of `cap` slots (any lane).
// Keys never change once published, so a stale read can only show KEY_NONE,
// which the CAS then corrects.  Returns false when the table is full.
__device__ __noinline__ bool g_add_cap(unsigned long long* keys, unsigned long long* counts, uint32_t cap,
                                       uint64_t key, uint64_t cnt) {
  uint32_t s = slot_hash(key, cap);
#pragma unroll 1
  for (uint32_t p = 0; p < cap; ++p) {
    unsigned long long k = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == KEY_NONE) {
      unsigned long long prev = atomicCAS(&keys[s], KEY_NONE, (unsigned long long)key);
      if (prev == KEY_NONE || prev == key) {
        atomicAdd(&counts[s], (unsigned long long)cnt);
        return true;
      }
    } else if (k == key) {
      atomicAdd(&counts[s], (unsigned long long)cnt);
      return true;
    }
    s = (s + 1) & (cap - 1);
  }
  return false;
}

// The main-table slot of `key`, inserted with count 0 when absent (so it is
// materialised even if nothing is added later); ~0 when the table is full
// (overflow flagged).
__device__ __noinline__ unsigned long long g_slot(GTable g, uint64_t key) {
  atomicOr(&g.flags[3], 1u);  // main table in use: k_export must scan it
  uint32_t s = slot_hash(key, GCAP);
#pragma unroll 1
  for (uint32_t p = 0; p < GCAP; ++p) {
    const unsigned long long k = __hip_atomic_load(&g.keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == KEY_NONE) {
      const unsigned long long prev = atomicCAS(&g.keys[s], KEY_NONE, (unsigned long long)key);
      if (prev == KEY_NONE || prev == key) return s;
    } else if (k == key) {
      return s;
    }
    s = (s + 1) & (GCAP - 1);
  }
  atomicOr(&g.flags[0], FLAG_OVERFLOW);
  return ~0ull;
}

__device__ __forceinline__ void g_add(GTable g, uint64_t key, uint64_t cnt) {
  atomicOr(&g.flags[3], 1u);  // main table in use: k_export must scan it
  if (!g_add_cap(g.keys, g.counts, GCAP, key, cnt)) atomicOr(&g.flags[0], FLAG_OVERFLOW);
}

__device__ __forceinline__ void g_add_rep(GTable g, uint32_t rep, uint64_t key, uint64_t cnt) {
  if (!g_add_cap(g.rkeys + (size_t)rep * RCAP, g.rcounts + (size_t)rep * RCAP, RCAP, key, cnt)) g_add(g, key, cnt);
}

// LDS table insert (one lane).  Returns false when the table is full.
template <typename CT, int CAP>
__device__ __noinline__ bool lds_add(unsigned long long* tk, CT* tc, uint64_t key, CT cnt) {
  uint32_t s = slot_hash(key, CAP);
#pragma unroll 1
  for (int p = 0; p < CAP; ++p) {
    unsigned long long k = __hip_atomic_load(&tk[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == KEY_NONE) {
      unsigned long long prev = atomicCAS(&tk[s], KEY_NONE, (unsigned long long)key);
      if (prev == KEY_NONE || prev == key) {
        atomicAdd(&tc[s], cnt);
        return true;
      }
    } else if (k == key) {
      atomicAdd(&tc[s], cnt);
      return true;
    }
    s = (s + 1) & (CAP - 1);
  }
  return false;
}

// Workgroup histogram: LDS table + per-wave scalar cache.
struct BlockTable {
  unsigned long long* tk;
  unsigned int* tc;
};

struct WaveCache {
  uint64_t k0, k1, k2, k3;
  uint32_t c0, c1, c2, c3;
  uint32_t victim;
};

__device__ __forceinline__ void wc_init(WaveCache& w) {
  w.k0 = w.k1 = w.k2 = w.k3 = KEY_NONE;
  w.c0 = w.c1 = w.c2 = w.c3 = 0;
  w.victim = 0;
}

__device__ __forceinline__ void bt_spill(BlockTable bt, GTable g, uint64_t key, uint32_t cnt) {
  if (key == KEY_NONE || cnt == 0) return;
  if (__lane_id() == 0) {
    if (!lds_add<unsigned int, TCAP>(bt.tk, bt.tc, key, cnt)) g_add(g, key, cnt);
  }
}

__device__ __forceinline__ uint32_t rfl32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) { return ((uint64_t)rfl32((uint32_t)(v >> 32)) << 32) | rfl32((uint32_t)v); }

// Count one uniform key `lk` `cnt` times in the wave's cache.  Every value is
// re-asserted wave-uniform (readfirstlane) so the cache lives in SGPRs and the
// compare chain is scalar.
__device__ __forceinline__ void wc_add(WaveCache& w, BlockTable bt, GTable g, uint64_t lk, uint32_t cnt) {
  if (w.k0 == lk) {
    w.c0 = rfl32(w.c0 + cnt);
  } else if (w.k1 == lk) {
    w.c1 = rfl32(w.c1 + cnt);
  } else if (w.k2 == lk) {
    w.c2 = rfl32(w.c2 + cnt);
  } else if (w.k3 == lk) {
    w.c3 = rfl32(w.c3 + cnt);
  } else {
    switch (w.victim) {  // evict round-robin into the LDS table
      case 0: bt_spill(bt, g, w.k0, w.c0); w.k0 = lk; w.c0 = cnt; break;
      case 1: bt_spill(bt, g, w.k1, w.c1); w.k1 = lk; w.c1 = cnt; break;
      case 2: bt_spill(bt, g, w.k2, w.c2); w.k2 = lk; w.c2 = cnt; break;
      default: bt_spill(bt, g, w.k3, w.c3); w.k3 = lk; w.c3 = cnt; break;
    }
    w.victim = rfl32((w.victim + 1) & 3);
  }
  w.k0 = rfl64(w.k0); w.k1 = rfl64(w.k1); w.k2 = rfl64(w.k2); w.k3 = rfl64(w.k3);
  w.c0 = rfl32(w.c0); w.c1 = rfl32(w.c1); w.c2 = rfl32(w.c2); w.c3 = rfl32(w.c3);
}

// Wave-aggregated count of per-lane keys.  All lanes of the wave must call it
// (converged); `valid` masks lanes without a sample.
__device__ __forceinline__ void wave_count(WaveCache& w, BlockTable bt, GTable g, uint64_t key, bool valid) {
  uint64_t pend = rfl64(__ballot(valid));
  while (pend) {
    const int leader = __builtin_ctzll(pend);
    const uint64_t lk = readlane64(key, leader);
    const uint64_t hit = rfl64(__ballot(key == lk) & pend);
    wc_add(w, bt, g, lk, (uint32_t)__popcll(hit));
    pend = rfl64(pend & ~hit);
  }
}

__device__ __forceinline__ void bt_init(BlockTable bt) {
  for (int i = threadIdx.x; i < TCAP; i += blockDim.x) {
    bt.tk[i] = KEY_NONE;
    bt.tc[i] = 0;
  }
}

// End of kernel: waves spill their caches, then the workgroup adds its table
// into replica blockIdx % NREP.
__device__ __forceinline__ void bt_finish(WaveCache& w, BlockTable bt, GTable g) {
  bt_spill(bt, g, w.k0, w.c0);
  bt_spill(bt, g, w.k1, w.c1);
  bt_spill(bt, g, w.k2, w.c2);
  bt_spill(bt, g, w.k3, w.c3);
  __syncthreads();
  const uint32_t rep = blockIdx.x & (NREP - 1);
  for (int i = threadIdx.x; i < TCAP; i += blockDim.x) {
    const unsigned long long k = bt.tk[i];
    if (k != KEY_NONE) g_add_rep(g, rep, k, bt.tc[i]);
  }
}

// the radix sort's top-level bucket (pluss_sort.h): range [start, start +
// count) of the concatenated arrays; split past SCAP into 2^d2 children through
// nc2 level-2 chunks.  (Here: the scan pipeline reads the parents' starts to put
// 4-byte payloads' digits back, pluss_faithful.h SRC_W32P.)
struct SrtParent {
  uint32_t start, count, ref, b1;
  uint32_t d2, nc2, cbase, h2off;
  uint32_t src;         // where its payloads are in X1 (the counted path: start)
  uint32_t ybase, cb2;  // count-free level 2: its children's region in Y, its first child's fill word
};

}  // namespace pluss
