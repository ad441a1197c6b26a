/*
 * pluss_diag.h — diagnostics of libpluss_gpu.so.  NOT part of the drop-in
 * boundary (include/pluss_gpu.h): nothing in the product path calls these,
 * and no environment variable changes what a pluss_* entry point computes.
 * Used by tools/ablate.py (where the hot kernel's time goes),
 * tools/grid_sweep.py (workgroup count vs list size) and the sort tests.
 */
#ifndef PLUSS_DIAG_H
#define PLUSS_DIAG_H

#include <stdint.h>

#include "pluss_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
  PLUSS_DIAG_PRODUCT = 0,    /* the product dense pass (pluss_dev_sampled_hist_dense), d_counts written */
  PLUSS_DIAG_LOADS_ONLY = 1, /* the same sample loads, nothing counted, nothing written */
  PLUSS_DIAG_NO_TAIL = 2     /* counted, but no tail: nothing written */
};

/* One dense pass over a device sample list (N, CLS/DS and chunk powers of two
   for variants 1 and 2).  max_grid > 0 replaces the launcher's workgroup cap
   (product variant: the counts are still exact; tests use it to cover grids
   of 1..16384 workgroups).  Returns PLUSS_OK or PLUSS_ERR_*. */
int pluss_diag_dense(pluss_ctx *ctx, const uint64_t *d_samples, uint64_t n, uint64_t *d_counts, int32_t variant,
                     int32_t max_grid, void *stream);

/* The faithful radix source's sort alone (pluss_sort.h): the n samples of
   reference `ref` (any order) -> their packed sort words (rank << 2 | case) in
   ascending order, copied to d_words.  *word_bytes is set to 4 (N <= 1024) or
   8.  Needs N % (cls/ds) == 0.  Tests compare it with a host sort. */
int pluss_diag_sort_words(pluss_ctx *ctx, int32_t ref, const uint64_t *d_samples, uint64_t n, void *d_words,
                          int32_t *word_bytes, void *stream);

/* The uniform source's parts alone (r10's law, pluss_dev_gen_uniform_faithful_refs),
   to see where its pass time goes: what = 0 the plan (counts, prefix, removal,
   tile map); 1 the plan, then every full tile generated into LDS as the
   lane-major local pass stages it (nothing scanned; one word per tile written
   to d_out, which holds one u64 per tile of all references); 2 the same
   staging as the slow and rescan paths do it (packed samples). */
int pluss_diag_uniform_parts(pluss_ctx *ctx, uint64_t seed, const uint64_t totals[6], int32_t what, uint64_t *d_out,
                             void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PLUSS_DIAG_H */
