/* The handle API's stream rule (include/pluss_gpu.h): stream == NULL is HIP's
 * null stream, ordered with the caller's own null-stream work.  A plain-C
 * caller mixes its null-stream copies and memsets with library passes on
 * NULL and checks every result without any explicit synchronisation (round
 * 4's g2 failure: NULL then meant the handle's own non-blocking stream, and a
 * caller's null-stream copy raced the pass).  Prints "ok <what>" per check,
 * "MISMATCH <what>" otherwise.  Test-only (tests/test_group_capi.py). */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "pluss_gpu.h"

static int g_fail = 0;
static void report(const char* what, int ok) {
  printf("%s %s\n", ok ? "ok" : "MISMATCH", what);
  if (!ok) g_fail = 1;
}

#define CHECK(call)                                                    \
  do {                                                                 \
    int rc_ = (int)(call);                                             \
    if (rc_) {                                                         \
      fprintf(stderr, "%s: %d: %s\n", #call, rc_, pluss_last_error()); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main(void) {
  const pluss_cfg cfg = {1024, 8, 4, 8, 64, PLUSS_MODE_CLEAN, PLUSS_THR_R10, 0, 0};
  const uint64_t n = 1ull << 26, seed = 0x5EED0001;
  pluss_ctx* c = NULL;
  CHECK(pluss_ctx_create(&cfg, &c));
  uint64_t *d = NULL, *out = NULL;
  CHECK(hipMalloc((void**)&d, n * 8));
  CHECK(hipMalloc((void**)&out, 64 * 8));
  uint64_t h[PLUSS_DENSE_BINS + 1];
  for (int rep = 0; rep < 3; ++rep) {
    /* the library fills the list (B0 samples) on the null stream, the caller
       overwrites it with zeros (C0 at (0,0): RI 1, bin 0) on the null
       stream, and the pass counts it on the null stream */
    CHECK(pluss_dev_expand(c, seed, PLUSS_B0, 0, n, d, NULL));
    CHECK(hipMemsetAsync(d, 0, n * 8, NULL));
    CHECK(pluss_dev_sampled_hist_dense(c, d, n, out, NULL));
    CHECK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
    int ok = h[0] == n;
    for (int b = 1; b <= PLUSS_DENSE_BINS; ++b) ok &= h[b] == 0;
    report("caller memset -> pass on NULL", ok);
  }
  /* a pass's list written by the library on NULL, read back by the caller's
     null-stream copy at once */
  uint64_t* hl = (uint64_t*)malloc(n * 8);
  uint64_t ref[4];
  CHECK(pluss_expand_samples(&cfg, seed, PLUSS_A0, 0, 2, ref));
  CHECK(pluss_expand_samples(&cfg, seed, PLUSS_A0, n - 2, 2, ref + 2));
  CHECK(hipMemsetAsync(d, 0xFF, n * 8, NULL));
  CHECK(pluss_dev_expand(c, seed, PLUSS_A0, 0, n, d, NULL));
  CHECK(hipMemcpyAsync(hl, d, n * 8, hipMemcpyDeviceToHost, NULL));
  CHECK(hipStreamSynchronize(NULL));
  report("library expand on NULL -> caller copy", hl[0] == ref[0] && hl[1] == ref[1] && hl[n - 2] == ref[2] &&
                                                      hl[n - 1] == ref[3]);
  /* the handle's own stream stays available explicitly */
  CHECK(pluss_dev_sampled_hist_dense(c, d, n, out, pluss_ctx_stream(c)));
  CHECK(hipStreamSynchronize((hipStream_t)pluss_ctx_stream(c)));
  CHECK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
  uint64_t tot = 0;
  for (int b = 0; b < PLUSS_DENSE_BINS; ++b) tot += h[b];
  report("pass on pluss_ctx_stream", tot == n && h[PLUSS_DENSE_BINS] == 0);
  free(hl);
  (void)hipFree(d);
  (void)hipFree(out);
  pluss_ctx_destroy(c);
  return g_fail;
}
