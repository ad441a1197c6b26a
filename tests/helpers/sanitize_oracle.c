/* Drives every oracle entry point on small inputs, for the ASan/UBSan and
   TSan builds of oracle/pluss_oracle.c (tests/test_sanitizers.py).  Test-only. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct { int64_t N, T, CS, DS, CLS; int32_t thr_variant, range_full; } orc_cfg;
typedef struct { int32_t ref, kind; int64_t ri; uint64_t count; } orc_entry;
int orc_fulltrace(const orc_cfg *c, orc_entry *out, int64_t cap, int64_t *n_out, int64_t *traversed);
int orc_fulltrace_mt(const orc_cfg *c, orc_entry *out, int64_t cap, int64_t *n_out, int64_t *traversed);
int orc_clean(const orc_cfg *c, const uint64_t *samples, int64_t n, int64_t *ri_out, int nthreads);
int orc_faithful(const orc_cfg *c, int REF, const uint64_t *samples, int64_t n, orc_entry *out, int64_t cap,
                 int64_t *n_out, int64_t *traversed);
int orc_expand(const orc_cfg *c, uint64_t seed, int ref, uint64_t first, uint64_t n, uint64_t *out);
int orc_expand_sorted(const orc_cfg *c, uint64_t seed, int ref, uint64_t S, uint64_t first, uint64_t n,
                      uint64_t *out);

int main(void) {
    orc_entry buf[4096];
    int64_t n = 0, trav = 0, n2 = 0, trav2 = 0;
    orc_cfg shapes[] = {{64, 4, 4, 8, 64, 1, 0}, {40, 3, 2, 8, 32, 0, 0}, {32, 8, 4, 8, 64, 0, 1}};
    for (int s = 0; s < 3; s++) {
        const orc_cfg *c = &shapes[s];
        if (orc_fulltrace(c, buf, 4096, &n, &trav)) return 1;
        if (orc_fulltrace_mt(c, buf, 4096, &n2, &trav2) || n2 != n || trav2 != trav) return 2;
        for (int ref = 0; ref < 6; ref++) {
            const uint64_t span = c->range_full ? (uint64_t)c->N : (uint64_t)c->N - 1;
            uint64_t cnt = ref < 2 ? span * span / 2 : 600;
            uint64_t *smp = malloc(cnt * 8);
            int64_t *ri = malloc(cnt * 8);
            if (orc_expand(c, 7, ref, 0, cnt, smp)) return 3;
            if (orc_clean(c, smp, (int64_t)cnt, ri, 4)) return 4;
            if (orc_faithful(c, ref, smp, (int64_t)cnt, buf, 4096, &n, &trav)) return 5;
            if (c->N % (c->CS * c->T) == 0) {
                if (orc_expand_sorted(c, 7, ref, cnt, 0, cnt, smp)) return 6;
                if (orc_faithful(c, ref, smp, (int64_t)cnt, buf, 4096, &n, &trav)) return 7;
            }
            free(smp);
            free(ri);
        }
    }
    printf("oracle sanitizer driver ok\n");
    return 0;
}
