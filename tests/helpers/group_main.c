/* The C-ABI multi-GPU group (include/pluss_gpu.h, pluss_group_*) driven from
 * plain C, the way the reference's own main()s would call it (r10's main runs
 * the six sampler_<REF> and merges, r10:3191-3278; the Rust main,
 * src/main.rs:17-44).  Every group result is compared with the same pass on
 * one device through the one-GPU entry points; prints one "ok <what>" line per
 * agreeing pass, "MISMATCH <what>" otherwise, and exits non-zero on any
 * failure.  Test-only (tests/test_group_capi.py).
 *
 * usage: group_main N THREADS TOTAL SHARDS_PER_DEVICE DEVICE...
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pluss_gpu.h"

#define CAP (1 << 14)
static int g_fail = 0;

static int same_hist(const pluss_hist* a, const pluss_hist* b) {
  if (a->n_entries != b->n_entries) return 0;
  for (uint64_t i = 0; i < a->n_entries; ++i) {
    const pluss_hist_entry *x = &a->entries[i], *y = &b->entries[i];
    if (x->ref != y->ref || x->kind != y->kind || x->ri != y->ri || x->count != y->count) return 0;
  }
  for (int r = 0; r < 6; ++r)
    if (a->traversed[r] != b->traversed[r]) return 0;
  return 1;
}

static void report(const char* what, int ok) {
  printf("%s %s\n", ok ? "ok" : "MISMATCH", what);
  if (!ok) g_fail = 1;
}

#define CHECK(call)                                                              \
  do {                                                                           \
    int rc_ = (call);                                                            \
    if (rc_) {                                                                   \
      fprintf(stderr, "%s: %d: %s\n", #call, rc_, pluss_last_error());           \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

static pluss_hist new_hist(void) {
  pluss_hist h;
  memset(&h, 0, sizeof h);
  h.entries = (pluss_hist_entry*)calloc(CAP, sizeof(pluss_hist_entry));
  h.capacity = CAP;
  return h;
}

/* a merged dense vector vs the whole list's histogram (bins of one key -- a
   reference's unused cases -- summed; no count outside the list's keys) */
static int dense_matches(const pluss_cfg* cfg, const uint64_t* gv, const pluss_hist* b) {
  uint64_t keys[PLUSS_DENSE_BINS];
  if (pluss_dense_keys(cfg, keys)) return 0;
  int ok = gv[PLUSS_DENSE_BINS] == 0;
  uint64_t total_dense = 0;
  for (int k = 0; k < PLUSS_DENSE_BINS; ++k) total_dense += gv[k];
  for (uint64_t i = 0; i < b->n_entries; ++i) {
    const pluss_hist_entry* e = &b->entries[i];
    const uint64_t key = ((uint64_t)e->ref << 60) | ((uint64_t)e->kind << 56) | (uint64_t)(e->ri + 2);
    uint64_t got = 0;
    for (int k = 0; k < PLUSS_DENSE_BINS; ++k)
      if (keys[k] == key) got += gv[k];
    ok &= got == e->count;
    total_dense -= got;
  }
  return ok && total_dense == 0;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s N THREADS TOTAL SHARDS_PER_DEVICE DEVICE...\n", argv[0]);
    return 2;
  }
  const int64_t N = atoll(argv[1]), T = atoll(argv[2]);
  const uint64_t total = strtoull(argv[3], NULL, 10);
  const int spd = atoi(argv[4]);
  const int ndev = argc - 5;
  int32_t devs[16];
  for (int i = 0; i < ndev && i < 16; ++i) devs[i] = atoi(argv[5 + i]);
  const uint64_t seed = 0x5EED0001;
  uint64_t counts[6];
  CHECK(pluss_default_counts(N, total, counts));

  /* the six references' Feistel lists on the host (what r10 draws, r10:156-185) */
  pluss_cfg clean = {N, T, 4, 8, 64, PLUSS_MODE_CLEAN, PLUSS_THR_R10, 0, devs[0]};
  pluss_cfg faith = clean;
  faith.mode = PLUSS_MODE_FAITHFUL;
  uint64_t* list = (uint64_t*)malloc(total * sizeof(uint64_t));
  uint64_t off = 0;
  for (int r = 0; r < 6; ++r) {
    CHECK(pluss_expand_samples(&clean, seed, r, 0, counts[r], list + off));
    off += counts[r];
  }
  int32_t local = 0, all = 0;

  /* clean mode over a host list */
  {
    pluss_group* g = NULL;
    CHECK(pluss_group_create(&clean, devs, ndev, spd, &g));
    CHECK(pluss_group_shards(g, &local, &all));
    printf("shards %d of %d\n", local, all);
    pluss_hist a = new_hist(), b = new_hist();
    CHECK(pluss_group_sampled_hist(g, list, total, &a));
    CHECK(pluss_gemm_sampled_hist(&clean, list, total, &b));
    report("clean sampled_hist", same_hist(&a, &b));

    /* resident lists, dense passes (the bench step), RCCL all-reduce: the
       merged vector of the last of 20 passes vs the whole list's histogram */
    uint64_t gv[PLUSS_DENSE_BINS + 1], ov[PLUSS_DENSE_BINS + 1];
    CHECK(pluss_group_expand(g, seed, counts));
    CHECK(pluss_group_dense(g, 20, gv));
    report("clean dense x20 (resident lists)", dense_matches(&clean, gv, &b));

    /* the lists changed under a captured pass: expand other counts, then 32
       passes (replayed from a graph of 16) must count the new lists */
    {
      uint64_t counts2[6], total2 = total / 2 + 7;
      CHECK(pluss_default_counts(N, total2, counts2));
      uint64_t* list2 = (uint64_t*)malloc(total2 * sizeof(uint64_t));
      uint64_t o2 = 0;
      for (int r = 0; r < 6; ++r) {
        CHECK(pluss_expand_samples(&clean, seed + 1, r, 0, counts2[r], list2 + o2));
        o2 += counts2[r];
      }
      pluss_hist b2 = new_hist();
      CHECK(pluss_gemm_sampled_hist(&clean, list2, total2, &b2));
      CHECK(pluss_group_dense(g, 32, gv));
      CHECK(pluss_group_expand(g, seed + 1, counts2));
      CHECK(pluss_group_dense(g, 32, gv));
      int ok2 = dense_matches(&clean, gv, &b2);
      CHECK(pluss_group_expand(g, seed, counts));
      CHECK(pluss_group_dense(g, 32, gv));
      ok2 &= dense_matches(&clean, gv, &b);
      report("clean dense x32 after re-expanding", ok2);
      free(b2.entries);
      free(list2);
    }

    /* generated key-order slices counted, vs one shard on one device */
    CHECK(pluss_group_gen_count_dense(g, seed, counts, gv));
    pluss_group_destroy(g);
    pluss_group* one = NULL;
    CHECK(pluss_group_create(&clean, devs, 1, 1, &one));
    CHECK(pluss_group_gen_count_dense(one, seed, counts, ov));
    pluss_group_destroy(one);
    report("clean gen_count_dense", memcmp(gv, ov, sizeof gv) == 0);
    free(a.entries);
    free(b.entries);
  }

  /* faithful mode: r10's six samplers over the list in any order (key-range shards) */
  {
    pluss_group* g = NULL;
    CHECK(pluss_group_create(&faith, devs, ndev, spd, &g));
    pluss_hist a = new_hist(), b = new_hist();
    CHECK(pluss_group_sampled_hist(g, list, total, &a));
    CHECK(pluss_gemm_sampled_hist(&faith, list, total, &b));
    report("faithful sampled_hist (any order)", same_hist(&a, &b));

    /* generated key-order lists: each shard generates only its key range */
    pluss_hist c1 = new_hist(), c2 = new_hist();
    CHECK(pluss_group_gen_faithful(g, seed, counts, &c1));
    pluss_ctx* c = NULL;
    CHECK(pluss_ctx_create(&faith, &c));
    CHECK(pluss_dev_hist_reset(c, NULL));
    CHECK(pluss_dev_gen_faithful_refs(c, seed, counts, NULL));
    CHECK(pluss_hist_fetch(c, &c2));
    report("faithful gen_faithful (key-order lists)", same_hist(&c1, &c2));

    /* r10's own law: each shard generates only its stretch of the uniform lists */
    pluss_hist u1 = new_hist(), u2 = new_hist();
    CHECK(pluss_group_gen_uniform_faithful(g, seed, counts, &u1));
    CHECK(pluss_dev_hist_reset(c, NULL));
    CHECK(pluss_dev_gen_uniform_faithful_refs(c, seed, counts, NULL));
    CHECK(pluss_hist_fetch(c, &u2));
    /* the same call again: captured, then replayed (one device), each equal */
    int same_u = same_hist(&u1, &u2);
    for (int k = 0; k < 3; ++k) {
      free(u1.entries);
      u1 = new_hist();
      CHECK(pluss_group_gen_uniform_faithful(g, seed, counts, &u1));
      same_u = same_u && same_hist(&u1, &u2);
    }
    report("faithful gen_uniform_faithful (r10's law)", same_u);
    free(u1.entries);
    free(u2.entries);
    pluss_ctx_destroy(c);
    pluss_group_destroy(g);
    free(a.entries);
    free(b.entries);
    free(c1.entries);
    free(c2.entries);
  }
  free(list);
  return g_fail;
}
