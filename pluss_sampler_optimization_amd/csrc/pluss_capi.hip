// pluss_capi.hip — the extern "C" boundary (include/pluss_gpu.h).
//
// Host-side plumbing only: configuration checks, handle lifetime, device
// buffers, launches on the caller's stream and copies of the final histogram.
// All per-sample work runs in the kernels of pluss_kernels.hip /
// pluss_faithful.hip; there is no CPU fallback — without a usable HIP device
// every entry point returns PLUSS_ERR_HIP.
#include <hip/hip_runtime.h>


#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/pluss_diag.h"
#include "pluss_internal.h"

namespace pluss {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

int validate_cfg(const pluss_cfg* c, Model* m) {
  if (!c) {
    set_error("null pluss_cfg");
    return PLUSS_ERR_CONFIG;
  }
  if (c->n < 1 || c->n >= (1 << 20)) {
    set_error("cfg.n must be in [1, 2^20) (20-bit sample fields)");
    return PLUSS_ERR_CONFIG;
  }
  if (c->threads < 1 || c->threads > 65536 || c->chunk < 1 || c->chunk > 65536 ||
      c->threads * c->chunk > (1ll << 30)) {
    set_error("cfg.threads and cfg.chunk must be in [1, 65536] with threads*chunk < 2^30");
    return PLUSS_ERR_CONFIG;
  }
  if (c->ds < 1 || c->cls < c->ds || c->cls % c->ds != 0 || c->cls / c->ds > 4096) {
    set_error("cfg.cls must be a positive multiple of cfg.ds (<= 4096 elements per line)");
    return PLUSS_ERR_CONFIG;
  }
  if ((c->mode != PLUSS_MODE_CLEAN && c->mode != PLUSS_MODE_FAITHFUL) ||
      (c->thr_variant != PLUSS_THR_R10 && c->thr_variant != PLUSS_THR_V1) || (c->range_full != 0 && c->range_full != 1)) {
    set_error("cfg.mode / cfg.thr_variant / cfg.range_full out of range");
    return PLUSS_ERR_CONFIG;
  }
  if (m) *m = make_model((uint64_t)c->n, (uint64_t)c->threads, (uint64_t)c->chunk, (uint64_t)c->ds,
                         (uint64_t)c->cls, c->thr_variant == PLUSS_THR_V1);
  return PLUSS_OK;
}

// The error a pass's flags report: flags[1] (malformed input) and the bits of
// flags[0], each with its own message and code; shared by the one-GPU fetch
// and the group's merge (`who`: the shard prefix of the message, or "").
int flags_error(unsigned int f0, unsigned int bad, const std::string& who) {
  if (bad) {
    set_error(who + "malformed sample: ref > 5, an index >= N, or a reference other than the one requested");
    return PLUSS_ERR_INPUT;
  }
  if (f0 & FLAG_SHARD) {
    set_error(who + "a key-range shard of this faithful pass failed (its summary row carried an error word)");
    return PLUSS_ERR_PEER;
  }
  if (f0 & FLAG_SORT) {
    set_error(who + "the bucket sort's plan exceeded its capacity (faithful radix source)");
    return PLUSS_ERR_CAPACITY;
  }
  if (f0 & FLAG_UNI) {
    set_error(who + "uniform key-order generator: fewer candidates than samples, or a candidate window past its "
              "capacity (probability below 1e-20; another seed draws afresh)");
    return PLUSS_ERR_CAPACITY;
  }
  if (f0 & FLAG_LOOKBACK) {
    set_error(who + "faithful pass stalled: a chunk's predecessor never published its running max (another kernel "
              "holding the GPU?)");
    return PLUSS_ERR_HIP;
  }
  if (f0) {
    set_error(who + "histogram table overflow (more distinct (ref,kind,RI) keys than the table holds)");
    return PLUSS_ERR_CAPACITY;
  }
  return PLUSS_OK;
}

static int check_flags(pluss_ctx* ctx) {
  unsigned int f[4] = {0, 0, 0, 0};
  PLUSS_HIP_CHECK(hipMemcpy(f, ctx->g.flags, sizeof f, hipMemcpyDeviceToHost));
  return flags_error(f[0], f[1], "");
}

// stream == NULL is HIP's null stream (ordered with the caller's null-stream
// work, as every HIP API takes it); the handle's own stream is pluss_ctx_stream()
static hipStream_t pick(pluss_ctx* ctx, void* stream) {
  ctx->last = (hipStream_t)stream;
  ctx->has_last = true;
  return ctx->last;
}

static void decode_entry(uint64_t key, uint64_t cnt, pluss_hist_entry* e) {
  e->ref = (int32_t)key_ref(key);
  e->kind = (int32_t)key_kind(key);
  e->ri = key_ri(key);
  e->count = cnt;
}

}  // namespace pluss

using namespace pluss;

extern "C" {

const char* pluss_last_error(void) { return g_err.c_str(); }

int pluss_version(void) { return 1; }

int pluss_device_count(int* n) {
  if (!n) return PLUSS_ERR_CONFIG;
  PLUSS_HIP_CHECK(hipGetDeviceCount(n));
  return PLUSS_OK;
}

int pluss_default_counts(int64_t n, uint64_t total, uint64_t counts[6]) {
  // r10 uses 164 samples for the 2-D references and 2098 for the 3-D ones at
  // N=128 (r10:156,1688).  Generalised: 2-D refs get
  // ceil(1% of (N-1)^2); the rest is split evenly over the four 3-D refs with
  // the remainder going to B0.
  if (n < 2 || !counts) {
    set_error("pluss_default_counts: n must be >= 2");
    return PLUSS_ERR_CONFIG;
  }
  const uint64_t m = (uint64_t)(n - 1);
  const uint64_t c2d = (m * m + 99) / 100;
  if (2 * c2d > total) {
    set_error("pluss_default_counts: total too small for the 2-D references");
    return PLUSS_ERR_CONFIG;
  }
  const uint64_t rest = total - 2 * c2d, c3d = rest / 4;
  if (c3d + (rest - 4 * c3d) > m * m * m) {
    set_error("pluss_default_counts: more 3-D samples than distinct iteration points");
    return PLUSS_ERR_CONFIG;
  }
  counts[PLUSS_C0] = counts[PLUSS_C1] = c2d;
  counts[PLUSS_A0] = counts[PLUSS_C2] = counts[PLUSS_C3] = c3d;
  counts[PLUSS_B0] = c3d + (rest - 4 * c3d);
  return PLUSS_OK;
}

int pluss_ctx_create(const pluss_cfg* cfg, pluss_ctx** out) {
  if (!out) return PLUSS_ERR_CONFIG;
  *out = nullptr;
  Model m;
  if (int rc = validate_cfg(cfg, &m)) return rc;
  int ndev = 0;
  PLUSS_HIP_CHECK(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev) {
    set_error("cfg.device out of range (" + std::to_string(ndev) + " HIP devices)");
    return PLUSS_ERR_CONFIG;
  }
  PLUSS_HIP_CHECK(hipSetDevice(cfg->device));
  pluss_ctx* c = new pluss_ctx();
  std::memset((void*)c, 0, sizeof(pluss_ctx));
  c->fb = FaithfulBufs();
  for (auto& f : c->fbr) f = FaithfulBufs();
  c->cfg = *cfg;
  c->m = m;
  c->device = cfg->device;
  auto fail = [&](const char* what) {
    set_error(std::string("pluss_ctx_create: ") + what);
    pluss_ctx_destroy(c);
    return PLUSS_ERR_ALLOC;
  };
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream");
  if (hipMalloc(&c->d_table, TABLE_BYTES) != hipSuccess) return fail("table");
  {
    unsigned long long* base = (unsigned long long*)c->d_table;
    c->g.keys = base;
    c->g.rkeys = base + GCAP;
    c->g.counts = base + GCAP + NREP * RCAP;
    c->g.rcounts = base + 2 * GCAP + NREP * RCAP;
    c->g.bins = base + 2 * (GCAP + NREP * RCAP);
    c->g.flags = (unsigned int*)(c->g.bins + NBROW * BSTRIDE);
    c->g.trav = c->g.bins + NBROW * BSTRIDE + 4;
    c->g.dbins = base + DB_OFF;
    c->g.dtot = base + DB_OFF + NBROW * BSTRIDE;
  }
  if (hipMalloc((void**)&c->d_exp_keys, GCAP * 8) != hipSuccess) return fail("export");
  if (hipMalloc((void**)&c->d_exp_counts, GCAP * 8) != hipSuccess) return fail("export");
  if (hipMalloc((void**)&c->d_exp_n, 16) != hipSuccess) return fail("export");
  if (int rc = launch_table_reset(c, c->stream)) {
    pluss_ctx_destroy(c);
    return rc;
  }
  if (hipStreamSynchronize(c->stream) != hipSuccess) return fail("init sync");
  *out = c;
  return PLUSS_OK;
}

int pluss_ctx_destroy(pluss_ctx* c) {
  if (!c) return PLUSS_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->d_table,  c->d_exp_keys, c->d_exp_counts, c->d_exp_n, c->fb.keys,  c->fb.sinks,
                  c->fb.keys_s, c->fb.sinks_s, c->fb.pmax,      c->fb.nstart, c->fb.tmp,
                  c->fb.scal, c->fb.st, c->fb.dpart, c->fb.tmax, c->fb.pmin, c->fb.fslot,
                  c->fb.klist, c->fb.slowq, c->fb.cval, c->fb.crec, c->fb.cflag, c->fb.shrec,
                  c->fb.xin,   c->fb.sbuf};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  for (const auto& f : c->fbr) {
    void* fr[] = {f.keys,  f.sinks, f.keys_s, f.sinks_s, f.pmax,  f.nstart, f.tmp,   f.scal,  f.st,
                  f.dpart, f.tmax,  f.pmin,   f.fslot,   f.klist, f.slowq,  f.cval,  f.crec,  f.cflag,
                  f.shrec, f.xin,  f.sbuf};
    for (void* p : fr)
      if (p) (void)hipFree(p);
  }
  uni_free(c);
  if (c->fb.side) (void)hipStreamDestroy(c->fb.side);
  for (hipEvent_t e : c->fb.sev)
    if (e) (void)hipEventDestroy(e);
  for (int r = 0; r < 6; ++r)
    if (c->fst[r]) (void)hipStreamDestroy(c->fst[r]);
  for (int e = 0; e < 7; ++e)
    if (c->fev[e]) (void)hipEventDestroy(c->fev[e]);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  faith_shards_free(c);
  delete c;
  return PLUSS_OK;
}

void* pluss_ctx_stream(pluss_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int pluss_dev_hist_reset(pluss_ctx* ctx, void* stream) {
  if (!ctx) return PLUSS_ERR_CONFIG;
  return launch_table_reset(ctx, pick(ctx, stream));
}

int pluss_dev_sampled_hist(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, void* stream) {
  if (!ctx || (!d_samples && n)) return PLUSS_ERR_CONFIG;
  return launch_sampled_hist(ctx, d_samples, n, pick(ctx, stream));
}

int pluss_dev_faithful_hist(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, void* stream) {
  if (!ctx || (!d_samples && n) || ref < 0 || ref > 5) return PLUSS_ERR_CONFIG;
  return launch_faithful(ctx, ref, d_samples, n, pick(ctx, stream));
}

int pluss_dev_faithful_hist_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t counts[6], void* stream) {
  if (!ctx || !counts) return PLUSS_ERR_CONFIG;
  return launch_faithful_refs(ctx, d_samples, counts, pick(ctx, stream));
}

int pluss_dev_faithful_hist_sorted(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, void* stream) {
  if (!ctx || (!d_samples && n) || ref < 0 || ref > 5) return PLUSS_ERR_CONFIG;
  return launch_faithful_sorted(ctx, ref, d_samples, n, pick(ctx, stream));
}

int pluss_dev_faithful_hist_sorted_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t counts[6],
                                        void* stream) {
  if (!ctx || !counts) return PLUSS_ERR_CONFIG;
  return launch_faithful_sorted_refs(ctx, d_samples, counts, pick(ctx, stream));
}

int pluss_dev_gen_faithful_refs(pluss_ctx* ctx, uint64_t seed, const uint64_t totals[6], void* stream) {
  if (!ctx || !totals) return PLUSS_ERR_CONFIG;
  return launch_gen_faithful_refs(ctx, seed, totals, pick(ctx, stream));
}

int pluss_dev_gen_uniform_faithful_refs(pluss_ctx* ctx, uint64_t seed, const uint64_t totals[6], void* stream) {
  if (!ctx || !totals) return PLUSS_ERR_CONFIG;
  return launch_gen_uniform_faithful_refs(ctx, seed, totals, pick(ctx, stream));
}

int pluss_dev_expand_uniform_sorted(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first,
                                    uint64_t n, uint64_t* d_out, void* stream) {
  if (!ctx || ref < 0 || ref > 5 || (n && !d_out)) return PLUSS_ERR_CONFIG;
  return launch_expand_uniform_sorted(ctx, seed, ref, total, first, n, d_out, pick(ctx, stream));
}

int pluss_dev_fulltrace_hist(pluss_ctx* ctx, void* stream) {
  if (!ctx) return PLUSS_ERR_CONFIG;
  return launch_fulltrace(ctx, pick(ctx, stream));  // the kernel also adds N*N*(4N+2) to traversed[0]
}

int pluss_dev_sampled_ri(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, int64_t* d_ri, uint64_t* d_sink,
                         void* stream) {
  if (!ctx || (n && (!d_samples || !d_ri))) return PLUSS_ERR_CONFIG;
  return launch_ri_dump(ctx, d_samples, n, d_ri, d_sink, pick(ctx, stream));
}

int pluss_dev_expand(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t first, uint64_t n, uint64_t* d_out,
                     void* stream) {
  if (!ctx || ref < 0 || ref > 5 || (n && !d_out)) return PLUSS_ERR_CONFIG;
  return launch_expand(ctx, seed, ref, first, n, d_out, pick(ctx, stream));
}

int pluss_dev_expand_sorted(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first, uint64_t n,
                            uint64_t* d_out, void* stream) {
  if (!ctx || ref < 0 || ref > 5 || (n && !d_out)) return PLUSS_ERR_CONFIG;
  return launch_expand_sorted(ctx, seed, ref, total, first, n, d_out, pick(ctx, stream));
}

int pluss_dev_hist_export(pluss_ctx* ctx, uint64_t* d_keys, uint64_t* d_counts, uint64_t cap, void* stream) {
  if (!ctx || !d_keys || !d_counts) return PLUSS_ERR_CONFIG;
  return launch_export(ctx, (unsigned long long*)d_keys, (unsigned long long*)d_counts, cap, pick(ctx, stream));
}

int pluss_dev_hist_export_reset(pluss_ctx* ctx, uint64_t* d_keys, uint64_t* d_counts, uint64_t cap, void* stream) {
  if (!ctx || !d_keys || !d_counts) return PLUSS_ERR_CONFIG;
  return launch_export(ctx, (unsigned long long*)d_keys, (unsigned long long*)d_counts, cap, pick(ctx, stream), true);
}

int pluss_dev_sampled_hist_export(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, uint64_t* d_keys,
                                  uint64_t* d_counts, uint64_t cap, void* stream) {
  if (!ctx || (!d_samples && n) || !d_keys || !d_counts) return PLUSS_ERR_CONFIG;
  return launch_sampled_hist_export(ctx, d_samples, n, (unsigned long long*)d_keys, (unsigned long long*)d_counts,
                                    cap, pick(ctx, stream));
}

int pluss_dense_keys(const pluss_cfg* cfg, uint64_t keys[PLUSS_DENSE_BINS]) {
  Model m;
  if (!keys) return PLUSS_ERR_CONFIG;
  if (int rc = validate_cfg(cfg, &m)) return rc;
  if (!m.fast) {
    set_error("pluss_dense_keys: needs N % (cls/ds) == 0");
    return PLUSS_ERR_CONFIG;
  }
  for (int b = 0; b < PLUSS_DENSE_BINS; ++b) keys[b] = m.keytab[b];
  return PLUSS_OK;
}

int pluss_dev_sampled_hist_dense(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, uint64_t* d_counts,
                                 void* stream) {
  if (!ctx || (!d_samples && n) || !d_counts) return PLUSS_ERR_CONFIG;
  return launch_sampled_hist_dense(ctx, d_samples, n, (unsigned long long*)d_counts, pick(ctx, stream));
}

int pluss_dev_gen_count_dense(pluss_ctx* ctx, uint64_t seed, const uint64_t totals[6], const uint64_t first[6],
                              const uint64_t n[6], uint64_t* d_counts, void* stream) {
  if (!ctx || !totals || !first || !n || !d_counts) return PLUSS_ERR_CONFIG;
  return launch_gen_count_dense(ctx, seed, totals, first, n, (unsigned long long*)d_counts, pick(ctx, stream));
}

int pluss_diag_dense(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, uint64_t* d_counts, int32_t variant,
                     int32_t max_grid, void* stream) {
  if (!ctx || (!d_samples && n) || !d_counts) return PLUSS_ERR_CONFIG;
  return launch_diag_dense(ctx, d_samples, n, (unsigned long long*)d_counts, variant, max_grid, pick(ctx, stream));
}

int pluss_diag_sort_words(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, void* d_words,
                          int32_t* word_bytes, void* stream) {
  if (!ctx || (!d_samples && n) || (!d_words && n) || !word_bytes || ref < 0 || ref > 5) return PLUSS_ERR_CONFIG;
  return diag_sort_words(ctx, ref, d_samples, n, d_words, word_bytes, pick(ctx, stream));
}

int pluss_diag_uniform_parts(pluss_ctx* ctx, uint64_t seed, const uint64_t totals[6], int32_t what, uint64_t* d_out,
                             void* stream) {
  if (!ctx || !totals || what < 0 || what > 2 || (what && !d_out)) return PLUSS_ERR_CONFIG;
  return diag_uniform_parts(ctx, seed, totals, what, d_out, pick(ctx, stream));
}

int pluss_faithful_key_space(const pluss_cfg* cfg, uint64_t* key_end) {
  Model m;
  if (!key_end) return PLUSS_ERR_CONFIG;
  if (int rc = validate_cfg(cfg, &m)) return rc;
  if (m.A == 0) {
    set_error("faithful mode needs N % (chunk*threads) == 0 (lockstep interleaving order)");
    return PLUSS_ERR_CONFIG;
  }
  *key_end = m.A * m.T;
  return PLUSS_OK;
}

int pluss_dev_faithful_shards_local(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t seed, const uint64_t* totals,
                                    const uint64_t* first, const uint64_t* n, uint64_t* d_row, void* stream) {
  if (!ctx || !totals || !first || !n || !d_row) return PLUSS_ERR_CONFIG;
  return faith_shards_local(ctx, d_samples, seed, totals, first, n, d_row, pick(ctx, stream));
}

int pluss_dev_faithful_shards_select(pluss_ctx* ctx, const uint64_t* d_lists, const uint64_t* totals, uint64_t key_lo,
                                     uint64_t key_hi, uint64_t* d_row, void* stream) {
  if (!ctx || !totals || !d_row || key_lo > key_hi) return PLUSS_ERR_CONFIG;
  return faith_shards_select(ctx, d_lists, totals, key_lo, key_hi, d_row, pick(ctx, stream));
}

int pluss_dev_faithful_shards_local_selected(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                             uint64_t* d_row, void* stream) {
  if (!ctx || !d_row) return PLUSS_ERR_CONFIG;
  return faith_shards_local_selected(ctx, d_rows, shard, nshards, d_row, pick(ctx, stream));
}

int pluss_dev_faithful_shards_uniform_count(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, int32_t shard,
                                            int32_t nshards, uint64_t* d_row, void* stream) {
  if (!ctx || !totals || !d_row) return PLUSS_ERR_CONFIG;
  return faith_shards_uniform_count(ctx, seed, totals, shard, nshards, d_row, pick(ctx, stream));
}

int pluss_dev_faithful_shards_uniform_local(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                            uint64_t* d_row, void* stream) {
  if (!ctx || !d_row) return PLUSS_ERR_CONFIG;
  hipStream_t s = pick(ctx, stream);
  if (int rc = faith_shards_uniform_window(ctx, d_rows, shard, nshards, s)) return rc;
  return faith_shards_uniform_finish(ctx, d_row, s);
}

int pluss_dev_faithful_shards_slice(pluss_ctx* ctx, uint64_t first[6], uint64_t n[6]) {
  if (!ctx || !first || !n) return PLUSS_ERR_CONFIG;
  return faith_shards_slice(ctx, first, n);
}

int pluss_dev_faithful_shards_carry(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                    uint64_t* d_row, void* stream) {
  if (!ctx || !d_row) return PLUSS_ERR_CONFIG;
  return faith_shards_carry(ctx, d_rows, shard, nshards, d_row, pick(ctx, stream));
}

int pluss_dev_faithful_shards_cut(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                  uint64_t* d_row, void* stream) {
  if (!ctx || !d_row) return PLUSS_ERR_CONFIG;
  return faith_shards_cut(ctx, d_rows, shard, nshards, d_row, pick(ctx, stream));
}

int pluss_dev_faithful_shards_hist(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                   void* stream) {
  if (!ctx) return PLUSS_ERR_CONFIG;
  return faith_shards_hist(ctx, d_rows, shard, nshards, pick(ctx, stream));
}

int pluss_keyorder_index_range(const pluss_cfg* cfg, uint64_t seed, int32_t ref, uint64_t total, uint64_t key_lo,
                               uint64_t key_hi, uint64_t* i_lo, uint64_t* i_hi) {
  Model m;
  if (!i_lo || !i_hi || ref < 0 || ref > 5 || key_lo > key_hi) return PLUSS_ERR_CONFIG;
  if (int rc = validate_cfg(cfg, &m)) return rc;
  pluss_ctx probe;  // keygen_check / keygen_of read only the configuration
  probe.cfg = *cfg;
  probe.m = m;
  if (int rc = keygen_check(&probe, ref, total, 0, total, "pluss_keyorder_index_range")) return rc;
  const KeyGen k = keygen_of(&probe, seed, ref, total);
  // keys increase with the index (the list is in key order): two binary searches on the host
  auto first_at_least = [&](uint64_t key) {
    uint64_t lo = 0, hi = total;
    while (lo < hi) {
      const uint64_t mid = lo + (hi - lo) / 2;
      if (key_of_digits(m, (uint32_t)ref, keygen_digits_at(k, mid)) >= key) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  };
  *i_lo = first_at_least(key_lo);
  *i_hi = first_at_least(key_hi);
  return PLUSS_OK;
}

int pluss_hist_fetch(pluss_ctx* ctx, pluss_hist* out) {
  if (!ctx || !out) return PLUSS_ERR_CONFIG;
  hipStream_t s = ctx->has_last ? ctx->last : ctx->stream;
  if (int rc = launch_export(ctx, ctx->d_exp_keys, ctx->d_exp_counts, GCAP, s)) return rc;
  PLUSS_HIP_CHECK(hipStreamSynchronize(s));
  if (int rc = check_flags(ctx)) return rc;
  unsigned int n = 0;
  PLUSS_HIP_CHECK(hipMemcpy(&n, ctx->d_exp_n, 4, hipMemcpyDeviceToHost));
  std::vector<unsigned long long> k(n), c(n), tr(8);
  if (n) {
    PLUSS_HIP_CHECK(hipMemcpy(k.data(), ctx->d_exp_keys, n * 8ull, hipMemcpyDeviceToHost));
    PLUSS_HIP_CHECK(hipMemcpy(c.data(), ctx->d_exp_counts, n * 8ull, hipMemcpyDeviceToHost));
  }
  PLUSS_HIP_CHECK(hipMemcpy(tr.data(), ctx->g.trav, 64, hipMemcpyDeviceToHost));
  for (int r = 0; r < 6; ++r) out->traversed[r] = tr[r];
  out->n_entries = n;
  if (n > out->capacity) {
    set_error("pluss_hist_fetch: output capacity " + std::to_string(out->capacity) + " < " + std::to_string(n) +
              " bins");
    return PLUSS_ERR_CAPACITY;
  }
  for (unsigned int i = 0; i < n; ++i) decode_entry(k[i], c[i], &out->entries[i]);
  return PLUSS_OK;
}

int pluss_hist_from_tables(const uint64_t* keys, const uint64_t* counts, uint64_t n_pairs, pluss_hist* out) {
  if (!out || (n_pairs && (!keys || !counts))) return PLUSS_ERR_CONFIG;
  std::map<uint64_t, uint64_t> acc;
  for (uint64_t i = 0; i < n_pairs; ++i)
    if (keys[i] != KEY_EMPTY && keys[i] != KEY_NONE) acc[keys[i]] += counts[i];
  out->n_entries = acc.size();
  if (acc.size() > out->capacity) {
    set_error("pluss_hist_from_tables: output capacity too small");
    return PLUSS_ERR_CAPACITY;
  }
  uint64_t i = 0;
  for (auto& kv : acc) decode_entry(kv.first, kv.second, &out->entries[i++]);
  return PLUSS_OK;
}

// ---------------------------------------------------------- one-shot API --
struct Scoped {
  pluss_ctx* ctx = nullptr;
  std::vector<void*> bufs;
  ~Scoped() {
    for (void* p : bufs) (void)hipFree(p);
    if (ctx) pluss_ctx_destroy(ctx);
  }
};

static int upload(Scoped& sc, const uint64_t* h, uint64_t n, uint64_t** d) {
  *d = nullptr;
  if (!n) return PLUSS_OK;
  PLUSS_HIP_CHECK(hipMalloc((void**)d, n * 8));
  sc.bufs.push_back(*d);
  PLUSS_HIP_CHECK(hipMemcpy(*d, h, n * 8, hipMemcpyHostToDevice));
  return PLUSS_OK;
}

int pluss_gemm_sampled_hist(const pluss_cfg* cfg, const uint64_t* samples, uint64_t n, pluss_hist* out) {
  if (!out || (n && !samples)) return PLUSS_ERR_CONFIG;
  Scoped sc;
  if (int rc = pluss_ctx_create(cfg, &sc.ctx)) return rc;
  if (cfg->mode == PLUSS_MODE_CLEAN) {
    uint64_t* d = nullptr;
    if (int rc = upload(sc, samples, n, &d)) return rc;
    if (int rc = launch_sampled_hist(sc.ctx, d, n, sc.ctx->stream)) return rc;
  } else {
    // faithful: one sampler_<REF> per reference present in the list
    std::vector<uint64_t> per[6];
    for (uint64_t i = 0; i < n; ++i) {
      const uint32_t r = (uint32_t)(samples[i] >> 60);
      if (r > 5) {
        set_error("malformed sample: ref > 5");
        return PLUSS_ERR_INPUT;
      }
      per[r].push_back(samples[i]);
    }
    for (int r = 0; r < 6; ++r) {
      if (per[r].empty()) continue;
      uint64_t* d = nullptr;
      if (int rc = upload(sc, per[r].data(), per[r].size(), &d)) return rc;
      if (int rc = launch_faithful(sc.ctx, r, d, per[r].size(), sc.ctx->stream)) return rc;
    }
  }
  return pluss_hist_fetch(sc.ctx, out);
}

int pluss_gemm_fulltrace_hist(const pluss_cfg* cfg, pluss_hist* out) {
  if (!out) return PLUSS_ERR_CONFIG;
  Scoped sc;
  if (int rc = pluss_ctx_create(cfg, &sc.ctx)) return rc;
  if (int rc = pluss_dev_fulltrace_hist(sc.ctx, sc.ctx->stream)) return rc;
  return pluss_hist_fetch(sc.ctx, out);
}

int pluss_gemm_sampled_ri(const pluss_cfg* cfg, const uint64_t* samples, uint64_t n, int64_t* ri_out,
                          uint64_t* sink_key_out) {
  if (n && (!samples || !ri_out)) return PLUSS_ERR_CONFIG;
  Scoped sc;
  if (int rc = pluss_ctx_create(cfg, &sc.ctx)) return rc;
  if (!n) return PLUSS_OK;
  uint64_t *d = nullptr, *dri = nullptr, *dsk = nullptr;
  if (int rc = upload(sc, samples, n, &d)) return rc;
  PLUSS_HIP_CHECK(hipMalloc((void**)&dri, n * 8));
  sc.bufs.push_back(dri);
  if (sink_key_out) {
    PLUSS_HIP_CHECK(hipMalloc((void**)&dsk, n * 8));
    sc.bufs.push_back(dsk);
  }
  if (int rc = launch_ri_dump(sc.ctx, d, n, (int64_t*)dri, dsk, sc.ctx->stream)) return rc;
  PLUSS_HIP_CHECK(hipStreamSynchronize(sc.ctx->stream));
  if (int rc = check_flags(sc.ctx)) return rc;
  PLUSS_HIP_CHECK(hipMemcpy(ri_out, dri, n * 8, hipMemcpyDeviceToHost));
  if (sink_key_out) PLUSS_HIP_CHECK(hipMemcpy(sink_key_out, dsk, n * 8, hipMemcpyDeviceToHost));
  return PLUSS_OK;
}

int pluss_expand_samples(const pluss_cfg* cfg, uint64_t seed, int32_t ref, uint64_t first, uint64_t n,
                         uint64_t* out) {
  if ((n && !out) || ref < 0 || ref > 5) return PLUSS_ERR_CONFIG;
  Scoped sc;
  if (int rc = pluss_ctx_create(cfg, &sc.ctx)) return rc;
  if (!n) return PLUSS_OK;
  uint64_t* d = nullptr;
  PLUSS_HIP_CHECK(hipMalloc((void**)&d, n * 8));
  sc.bufs.push_back(d);
  if (int rc = launch_expand(sc.ctx, seed, ref, first, n, d, sc.ctx->stream)) return rc;
  PLUSS_HIP_CHECK(hipStreamSynchronize(sc.ctx->stream));
  PLUSS_HIP_CHECK(hipMemcpy(out, d, n * 8, hipMemcpyDeviceToHost));
  return PLUSS_OK;
}

int pluss_expand_sorted(const pluss_cfg* cfg, uint64_t seed, int32_t ref, uint64_t total, uint64_t first, uint64_t n,
                        uint64_t* out) {
  if ((n && !out) || ref < 0 || ref > 5) return PLUSS_ERR_CONFIG;
  Scoped sc;
  if (int rc = pluss_ctx_create(cfg, &sc.ctx)) return rc;
  if (int rc = keygen_check(sc.ctx, ref, total, first, n, "pluss_expand_sorted")) return rc;
  if (!n) return PLUSS_OK;
  uint64_t* d = nullptr;
  PLUSS_HIP_CHECK(hipMalloc((void**)&d, n * 8));
  sc.bufs.push_back(d);
  if (int rc = launch_expand_sorted(sc.ctx, seed, ref, total, first, n, d, sc.ctx->stream)) return rc;
  PLUSS_HIP_CHECK(hipStreamSynchronize(sc.ctx->stream));
  PLUSS_HIP_CHECK(hipMemcpy(out, d, n * 8, hipMemcpyDeviceToHost));
  return PLUSS_OK;
}

int pluss_expand_uniform_sorted(const pluss_cfg* cfg, uint64_t seed, int32_t ref, uint64_t total, uint64_t first,
                                uint64_t n, uint64_t* out) {
  if ((n && !out) || ref < 0 || ref > 5) return PLUSS_ERR_CONFIG;
  Scoped sc;
  if (int rc = pluss_ctx_create(cfg, &sc.ctx)) return rc;
  if (int rc = uni_check(sc.ctx, ref, total, "pluss_expand_uniform_sorted")) return rc;
  if (!n) return PLUSS_OK;
  uint64_t* d = nullptr;
  PLUSS_HIP_CHECK(hipMalloc((void**)&d, n * 8));
  sc.bufs.push_back(d);
  if (int rc = launch_expand_uniform_sorted(sc.ctx, seed, ref, total, first, n, d, sc.ctx->stream)) return rc;
  PLUSS_HIP_CHECK(hipStreamSynchronize(sc.ctx->stream));
  if (int rc = check_flags(sc.ctx)) return rc;
  PLUSS_HIP_CHECK(hipMemcpy(out, d, n * 8, hipMemcpyDeviceToHost));
  return PLUSS_OK;
}

}  // extern "C"
