// pluss_device.h — device helpers shared by the kernel translation units:
// the LDS-privatised exact-key histogram table, the wave-aggregated insert and
// the handle's global table.
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

// Global table insert (any lane).  Keys never change once published, so a
// stale read can only show KEY_EMPTY, which the CAS then corrects.
__device__ inline void g_add(GTable g, uint64_t key, uint64_t cnt) {
  uint32_t s = slot_hash(key, GCAP);
  for (uint32_t p = 0; p < GCAP; ++p) {
    unsigned long long k = __hip_atomic_load(&g.keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) {
      atomicAdd(&g.counts[s], (unsigned long long)cnt);
      return;
    }
    if (k == KEY_EMPTY) {
      unsigned long long prev = atomicCAS(&g.keys[s], KEY_EMPTY, (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) {
        atomicAdd(&g.counts[s], (unsigned long long)cnt);
        return;
      }
    }
    s = (s + 1) & (GCAP - 1);
  }
  atomicOr(&g.flags[0], 1u);
}

// LDS table insert (one lane).  Returns false when the table is full.
template <typename CT, int CAP>
__device__ __forceinline__ bool lds_add(unsigned long long* tk, CT* tc, uint64_t key, CT cnt) {
  uint32_t s = slot_hash(key, CAP);
  for (int p = 0; p < CAP; ++p) {
    unsigned long long k = __hip_atomic_load(&tk[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k == key) {
      atomicAdd(&tc[s], cnt);
      return true;
    }
    if (k == KEY_EMPTY) {
      unsigned long long prev = atomicCAS(&tk[s], KEY_EMPTY, (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) {
        atomicAdd(&tc[s], cnt);
        return true;
      }
    }
    s = (s + 1) & (CAP - 1);
  }
  return false;
}

// Wave-aggregated insert: the lanes holding the same key are counted with one
// ballot + popcount and inserted once by a leader lane.  All lanes of the wave
// must call it (converged); `valid` masks lanes without a sample.
__device__ __forceinline__ void wave_insert(unsigned long long* tk, unsigned int* tc, GTable g, uint64_t key,
                                            bool valid) {
  uint64_t pend = __ballot(valid);
  while (pend) {
    const int leader = __builtin_ctzll(pend);
    const uint64_t lk = readlane64(key, leader);
    const uint64_t hit = __ballot(valid && key == lk) & pend;
    if ((int)__lane_id() == leader) {
      const unsigned int c = (unsigned int)__popcll(hit);
      if (!lds_add<unsigned int, TCAP>(tk, tc, lk, c)) g_add(g, lk, c);
    }
    pend &= ~hit;
  }
}

template <bool FAST>
__device__ __forceinline__ uint64_t sample_key(const Model& m, uint64_t x, bool* bad) {
  const Sample s = unpack(x);
  const bool b = s.ref > 5 || s.c0 >= m.N || s.c1 >= m.N || s.c2 >= m.N;
  *bad = b;
  if (b) return KEY_EMPTY;
  const int64_t ri = ri_of<FAST>(m, s.ref, s.c0, s.c1, s.c2);
  return make_key(s.ref, share_kind(m, s.ref, ri), ri);
}

__device__ __forceinline__ void table_init(unsigned long long* tk, unsigned int* tc) {
  for (int i = threadIdx.x; i < TCAP; i += BLOCK) {
    tk[i] = KEY_EMPTY;
    tc[i] = 0;
  }
}

__device__ __forceinline__ void table_flush(unsigned long long* tk, unsigned int* tc, unsigned int* nf, Slabs slabs) {
  for (int i = threadIdx.x; i < TCAP; i += BLOCK) {
    const unsigned long long k = tk[i];
    if (k != KEY_EMPTY) {
      const unsigned int pos = atomicAdd(nf, 1u);
      slabs.keys[(size_t)blockIdx.x * TCAP + pos] = k;
      slabs.counts[(size_t)blockIdx.x * TCAP + pos] = tc[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) slabs.n[blockIdx.x] = *nf;
}

}  // namespace pluss
