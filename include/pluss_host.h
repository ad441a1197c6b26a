/*
 * pluss_host.h — host half of the PLUSS pipeline (after the RI histograms):
 * CRI distribution, AET miss-ratio curve and the reference's text formats.
 * Runs on the CPU by design (north_star: "the AET-based miss-ratio-curve
 * conversion stays on the host"); it consumes the raw histograms produced by
 * libpluss_gpu.so (pluss_gpu.h) and never sees per-sample data.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   pluss_cri_r10        no_share_distribute + share_distribute, incl.
 *                        simulate_negative_binomial
 *                        c_lib/test/sampler/gemm-t4-pluss-pro-model-rs-ri-opt-r10.cpp:42-131,690-691
 *   pluss_cri_v1         pluss_cri_distribute(THREAD_NUM) = _pluss_cri_noshare_distribute
 *                        + _pluss_cri_racetrack, c_lib/test/runtime/pluss_utils.h:987-1131,1204-1208
 *   pluss_log2_merge     pluss_histogram_update into _RIHist (floor-log2), pluss_utils.h:665-689,722-725
 *   pluss_aet            pluss_AET, pluss_utils.h:758-804
 *   pluss_format_hist    _pluss_histogram_print, pluss_utils.h:690-702
 *   pluss_format_mrc     pluss_print_mrc, pluss_utils.h:851-883
 *   pluss_r10_host_pipeline  r10's main() after the sampler threads, r10:3259-3277
 *
 * The NBD pmf is GSL's gsl_ran_negative_binomial_pdf restated as
 * exp(lgamma(k+n) - lgamma(n) - lgamma(k+1) + n log p + k log1p(-p)); GSL is
 * not available in this environment, so agreement with a GSL build is not
 * pinned beyond the 6-digit printouts in tests/golden.
 */
#ifndef PLUSS_HOST_H
#define PLUSS_HOST_H

#include <stdint.h>

#include "pluss_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pluss_kv {
  int64_t key;  /* reuse interval (or cache size for an MRC point); -1 = cold */
  double value; /* count (or miss ratio) */
} pluss_kv;

/* r10 per-reference CRI: raw entries of ONE reference (kind 0/1) -> the
   sampler_<REF> output histogram (raw keys), sorted by key. */
int pluss_cri_r10(int64_t threads, const pluss_hist_entry *raw, uint64_t n, pluss_kv *out, uint64_t cap,
                  uint64_t *n_out);
/* full-trace (v1) CRI: raw noshare (binned floor-log2 first, as recorded by
   pluss_cri_noshare_histogram_update) and raw share entries of all references
   -> _RIHist (floor-log2 keys), sorted. */
int pluss_cri_v1(int64_t threads, const pluss_hist_entry *raw, uint64_t n, pluss_kv *out, uint64_t cap,
                 uint64_t *n_out);
/* merge histograms with floor-log2 binning of positive keys (pluss_histogram_update). */
int pluss_log2_merge(const pluss_kv *in, uint64_t n, pluss_kv *out, uint64_t cap, uint64_t *n_out);
/* AET: histogram -> MRC points (c, miss ratio) for c in [0, min(max RI, 327680)]. */
int pluss_aet(const pluss_kv *hist, uint64_t n, pluss_kv *mrc, uint64_t cap, uint64_t *n_out);
/* r10's whole host half after the samplers, one call (r10:3203-3277): the
   raw histograms of all six references (a pluss_hist as pluss_hist_fetch or
   pluss_group_* fill it) -> each reference's CRI output (pluss_cri_r10), run
   on `workers` host threads (0: one per reference present, as r10 runs each
   sampler_<REF> on a thread of its own, r10:3203-3257, with the CRI at its
   end, r10:690-691) -> merged with floor-log2 binning into the reuse
   histogram in r10's reference order C3 C2 A0 C0 B0 C1 (r10:3259-3276) ->
   pluss_aet -> pluss_print_mrc's text.  Each output is optional (NULL
   skips it; a NULL array with its count pointer set reports the size
   needed); PLUSS_ERR_CAPACITY when an array or the text buffer is too small
   (the counts are still set).  Replaces pluss_cri_r10 x 6 + pluss_log2_merge
   + pluss_aet + pluss_format_mrc chained by the caller. */
int pluss_r10_host_pipeline(int64_t threads, const pluss_hist *raw, int32_t workers, pluss_kv *reuse,
                            uint64_t reuse_cap, uint64_t *n_reuse, pluss_kv *mrc, uint64_t mrc_cap, uint64_t *n_mrc,
                            char *text, uint64_t text_cap, uint64_t *text_len);
/* text renderers (byte-compatible with std::cout defaults of the reference).
   Writes at most cap bytes incl. NUL; *len = bytes needed excluding NUL. */
int pluss_format_hist(const char *title, const pluss_kv *hist, uint64_t n, char *buf, uint64_t cap, uint64_t *len);
int pluss_format_mrc(const pluss_kv *mrc, uint64_t n, char *buf, uint64_t cap, uint64_t *len);

#ifdef __cplusplus
}
#endif
#endif /* PLUSS_HOST_H */
