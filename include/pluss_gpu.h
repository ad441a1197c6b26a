/*
 * pluss_gpu.h — C ABI of the MI355X-native PLUSS GEMM reuse-interval sampler.
 *
 * Drop-in boundary for the reference's sampler entry points (reference paths
 * relative to sauceeeeage/PLUSS_Sampler_Optimization):
 *
 *   pluss_gemm_sampled_hist   replaces  void sampler_<REF>(std::unordered_map<long,double>&)
 *                                        c_lib/test/sampler/gemm-t4-pluss-pro-model-rs-ri-opt-r10.cpp:135,698,1261,1667,2221,2638
 *                                        (the raw no_share/share histograms it builds before
 *                                        no_share_distribute, r10:690) — mode FAITHFUL;
 *                                        and the per-sample RI engine with every sample
 *                                        counted — mode CLEAN.
 *   pluss_gemm_fulltrace_hist replaces  fn sampler(pool) / rayon_sampler(...)
 *                                        src/gemm_sampler_rayon.rs:71,186 ;
 *                                        fn sampler() src/gemm_sampler.rs:56 ;
 *                                        void sampler() c_lib/test/sampler/gemm-t4-pluss-pro-model-ri-omp-seq.cpp:37
 *                                        (the per-tid _NoSharePRI/_SharePRI contents,
 *                                        runtime/pluss_utils.h:924-937, raw keys).
 *   pluss_gemm_sampled_ri     per-sample parity dump (no reference counterpart; the RI
 *                                        and sink the reference derives at r10:333/558).
 *   pluss_expand_samples      replaces  the rand()%(N-1) sample generation + dedup,
 *                                        r10:156-185 (deterministic, distinct by construction).
 *   pluss_default_counts      the per-reference sample counts of r10:156,719,1282,1688,2242,2659
 *                                        generalised to a total sample budget.
 *
 * Everything the reference hard-codes at compile time (THREAD_NUM, CHUNK_SIZE,
 * DS, CLS: c_lib/test/Makefile:14-15; N=128 literals; the two share thresholds
 * seq.cpp:203 vs r10:2482) is a field of pluss_cfg.  Outputs are caller-owned;
 * the library keeps no global state between calls except per-handle buffers.
 * No function throws across the ABI; all return 0 or a negative PLUSS_ERR_*.
 */
#ifndef PLUSS_GPU_H
#define PLUSS_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reference ids = access order inside one c1 iteration (seq.cpp:102-288) */
enum { PLUSS_C0 = 0, PLUSS_C1 = 1, PLUSS_A0 = 2, PLUSS_B0 = 3, PLUSS_C2 = 4, PLUSS_C3 = 5, PLUSS_NREFS = 6 };
enum { PLUSS_NOSHARE = 0, PLUSS_SHARE = 1 };
enum { PLUSS_MODE_CLEAN = 0, PLUSS_MODE_FAITHFUL = 1 };
enum { PLUSS_THR_R10 = 0, PLUSS_THR_V1 = 1 };

#define PLUSS_OK 0
#define PLUSS_ERR_CONFIG (-1)   /* invalid or unsupported pluss_cfg */
#define PLUSS_ERR_HIP (-2)      /* HIP runtime error (see pluss_last_error) */
#define PLUSS_ERR_ALLOC (-3)    /* device/host allocation failed */
#define PLUSS_ERR_CAPACITY (-4) /* output or histogram table too small */
#define PLUSS_ERR_INPUT (-5)    /* malformed sample (ref > 5 or index >= N, wrong ref) */
#define PLUSS_ERR_PEER (-6)     /* another shard or rank of a multi-GPU pass failed */

typedef struct pluss_cfg {
  int64_t n;           /* loop bound N of the GEMM nest (reference: literal 128) */
  int64_t threads;     /* simulated OpenMP threads (THREAD_NUM) */
  int64_t chunk;       /* static chunk size (CHUNK_SIZE) */
  int64_t ds;          /* element size in bytes (DS) */
  int64_t cls;         /* cache-line size in bytes (CLS); must be a multiple of ds */
  int32_t mode;        /* PLUSS_MODE_CLEAN | PLUSS_MODE_FAITHFUL */
  int32_t thr_variant; /* PLUSS_THR_R10: (4N+2)N (r10:2482) | PLUSS_THR_V1: (N+1)N+1 (seq.cpp:203) */
  int32_t range_full;  /* sample indices: 0 -> [0,N-2] like rand()%(N-1) (r10:159); 1 -> [0,N-1] */
  int32_t device;      /* HIP device ordinal */
} pluss_cfg;

/* one histogram bin: (reference, noshare/share, raw reuse interval) -> count.
   ri == -1 is the cold bin (the reference's key -1, seq.cpp:305-319, r10:196,671). */
typedef struct pluss_hist_entry {
  int32_t ref;
  int32_t kind;
  int64_t ri;
  uint64_t count;
} pluss_hist_entry;

typedef struct pluss_hist {
  pluss_hist_entry *entries; /* caller-owned array */
  uint64_t capacity;         /* entries available */
  uint64_t n_entries;        /* out: bins written, sorted by (ref, kind, ri) */
  uint64_t traversed[6];     /* out: faithful mode: per-ref accesses replayed (r10:694); full trace: total */
} pluss_hist;

typedef struct pluss_ctx pluss_ctx;

/* --- diagnostics ------------------------------------------------------- */
const char *pluss_last_error(void);
int pluss_device_count(int *n);
int pluss_version(void);

/* --- one-shot entry points (host buffers in, host histogram out) --------- */
int pluss_gemm_sampled_hist(const pluss_cfg *cfg, const uint64_t *samples, uint64_t n, pluss_hist *out);
int pluss_gemm_fulltrace_hist(const pluss_cfg *cfg, pluss_hist *out);
int pluss_gemm_sampled_ri(const pluss_cfg *cfg, const uint64_t *samples, uint64_t n, int64_t *ri_out,
                          uint64_t *sink_key_out);
int pluss_expand_samples(const pluss_cfg *cfg, uint64_t seed, int32_t ref, uint64_t first, uint64_t n,
                         uint64_t *out);
int pluss_default_counts(int64_t n, uint64_t total, uint64_t counts[6]);
/* Key-order stratified list: samples [first, first+n) of the
   `total` samples of reference `ref`, generated directly in the order r10's
   priority queue pops them (IterationComp, runtime/pluss_utils.h:175-267; key
   a*T+tid), one per stratum of the key-ordered iteration space at a keyed
   pseudo-random offset: distinct, strictly increasing in key, random access
   by index.  The list pluss_dev_faithful_hist_sorted consumes without a sort.
   Needs N % (chunk*threads) == 0 and 1 <= total <= min(span^d, 2^32-1). */
int pluss_expand_sorted(const pluss_cfg *cfg, uint64_t seed, int32_t ref, uint64_t total, uint64_t first, uint64_t n,
                        uint64_t *out);

/* r10's own draw in r10's pop order: samples [first, first+n)
   of the list of `total` distinct samples of reference `ref` drawn UNIFORMLY
   without replacement from its span^d iteration points -- the distribution of
   r10's rand() draw with duplicate rejection (r10:156-185) -- generated
   directly in key order (IterationComp, pluss_utils.h:175-267): Bernoulli
   candidates per leaf of the key-ordered space, then a uniform subset of
   them removed down to `total` (csrc/pluss_uniform.h).  Distinct, strictly
   increasing in key.  Needs N % (chunk*threads) == 0 and total + 10
   sqrt(total) + 32 < 2^32. */
int pluss_expand_uniform_sorted(const pluss_cfg *cfg, uint64_t seed, int32_t ref, uint64_t total, uint64_t first,
                                uint64_t n, uint64_t *out);

/* --- handle API: device-resident inputs, explicit streams ----------------
   `stream` is a hipStream_t, taken as every HIP API takes it: NULL is HIP's
   null stream, ordered with the caller's own null-stream work (copies,
   memsets, kernels).  The handle also owns a non-blocking stream,
   pluss_ctx_stream(), which a caller passes explicitly to run unordered with
   the null stream.  pluss_hist_fetch orders after the stream of the last
   call.  Device pointers are plain addresses of device memory on
   cfg->device.                                                             */
int pluss_ctx_create(const pluss_cfg *cfg, pluss_ctx **out);
int pluss_ctx_destroy(pluss_ctx *ctx);
void *pluss_ctx_stream(pluss_ctx *ctx);
int pluss_dev_expand(pluss_ctx *ctx, uint64_t seed, int32_t ref, uint64_t first, uint64_t n, uint64_t *d_out,
                     void *stream);
int pluss_dev_expand_sorted(pluss_ctx *ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first, uint64_t n,
                            uint64_t *d_out, void *stream);
int pluss_dev_hist_reset(pluss_ctx *ctx, void *stream);
/* clean mode: accumulate every sample of a mixed-reference list */
int pluss_dev_sampled_hist(pluss_ctx *ctx, const uint64_t *d_samples, uint64_t n, void *stream);
/* faithful mode: one sampler_<REF> over a list holding only reference `ref` */
int pluss_dev_faithful_hist(pluss_ctx *ctx, int32_t ref, const uint64_t *d_samples, uint64_t n, void *stream);
/* faithful mode, all six sampler_<REF> of one list at once (r10's main runs
   one thread per reference, r10:3203-3257): d_samples holds counts[0]
   samples of reference 0, then counts[1] of reference 1, ...; equal to six
   pluss_dev_faithful_hist calls.  The references run on streams of their
   own, joined back into `stream`. */
int pluss_dev_faithful_hist_refs(pluss_ctx *ctx, const uint64_t *d_samples, const uint64_t counts[6], void *stream);
/* faithful mode over a list ALREADY IN KEY ORDER (strictly increasing a*T+tid,
   e.g. pluss_dev_expand_sorted's): no sort, one pass reading 8 B per sample.
   Same result as pluss_dev_faithful_hist on any permutation of the list; a
   list that is not in key order is reported as PLUSS_ERR_INPUT at the next
   fetch.  N % (cls/ds) == 0 shapes (PLUSS_ERR_CONFIG otherwise). */
int pluss_dev_faithful_hist_sorted(pluss_ctx *ctx, int32_t ref, const uint64_t *d_samples, uint64_t n, void *stream);
int pluss_dev_faithful_hist_sorted_refs(pluss_ctx *ctx, const uint64_t *d_samples, const uint64_t counts[6],
                                        void *stream);
/* the six sampler_<REF> over generated key-order lists: equal to
   pluss_dev_expand_sorted(seed, r, totals[r], 0, totals[r]) for every r
   followed by pluss_dev_faithful_hist_sorted_refs, without the lists ever
   being written to memory (r10 generates its samples inside its timer,
   r10:156-185). */
int pluss_dev_gen_faithful_refs(pluss_ctx *ctx, uint64_t seed, const uint64_t totals[6], void *stream);
/* the same over r10's own distribution: pluss_dev_expand_uniform_sorted's
   lists, generated inside the pass (never written to memory) -- r10's whole
   sampler pass, its uniform draw included, without a sort */
int pluss_dev_gen_uniform_faithful_refs(pluss_ctx *ctx, uint64_t seed, const uint64_t totals[6], void *stream);
int pluss_dev_expand_uniform_sorted(pluss_ctx *ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first,
                                    uint64_t n, uint64_t *d_out, void *stream);
/* full trace: every access of the nest (sampling rate 1.0); accumulates like
   the other passes, and adds the N*N*(4N+2) accesses to traversed[0] */
int pluss_dev_fulltrace_hist(pluss_ctx *ctx, void *stream);
int pluss_dev_sampled_ri(pluss_ctx *ctx, const uint64_t *d_samples, uint64_t n, int64_t *d_ri, uint64_t *d_sink,
                         void *stream);
/* canonical table: `cap` (key,count) pairs sorted by key, unused = (~0,0);
   key = ref<<60 | kind<<56 | (ri+2).  Equal histograms give equal tables,
   so per-GPU tables can be exchanged by one collective and merged. */
int pluss_dev_hist_export(pluss_ctx *ctx, uint64_t *d_keys, uint64_t *d_counts, uint64_t cap, void *stream);
/* the same, and leave the handle's histogram empty for the next pass (bins and
   traversed counters; error flags are kept until pluss_dev_hist_reset) —
   one launch instead of export + reset between passes */
int pluss_dev_hist_export_reset(pluss_ctx *ctx, uint64_t *d_keys, uint64_t *d_counts, uint64_t cap, void *stream);
/* one pass: pluss_dev_sampled_hist, then pluss_dev_hist_export_reset — a
   single launch when N % (CLS/DS) == 0 and the handle holds only clean-mode
   counts (the last workgroup to finish writes the table) */
int pluss_dev_sampled_hist_export(pluss_ctx *ctx, const uint64_t *d_samples, uint64_t n, uint64_t *d_keys,
                                  uint64_t *d_counts, uint64_t cap, void *stream);
/* --- dense per-pass histogram (N % (cls/ds) == 0: every BASELINE shape) ----
   For these shapes a sample's (ref, kind, RI) key is one of PLUSS_DENSE_BINS
   fixed keys -- three outcomes per reference, bin = ref*3 + case (SURVEY.md
   A.3) -- so the histogram of a pass is a dense vector of counts.
   pluss_dense_keys:  the key of each bin (ref<<60 | kind<<56 | (ri+2), as in
                      the canonical table); PLUSS_ERR_CONFIG for other shapes.
   pluss_dev_sampled_hist_dense:  ONE launch counts every sample of the list
                      and OVERWRITES d_counts[0..PLUSS_DENSE_BINS] with this
                      pass's counts: [0..17] per bin, [18] malformed samples
                      (these also raise PLUSS_ERR_INPUT at the next fetch).
                      The handle's accumulating histogram is not touched.
                      Vectors of several GPUs merge by element-wise sum (one
                      all-reduce).  Replaces one r10 pass over all six
                      sampler_<REF> lists in clean mode (r10:135-3190). */
#define PLUSS_DENSE_BINS 18
int pluss_dense_keys(const pluss_cfg *cfg, uint64_t keys[PLUSS_DENSE_BINS]);
int pluss_dev_sampled_hist_dense(pluss_ctx *ctx, const uint64_t *d_samples, uint64_t n, uint64_t *d_counts,
                                 void *stream);
/* generation and counting in one launch: samples [first[r], first[r]+n[r])
   of every reference's key-order list of totals[r] samples (seed as in
   pluss_expand_sorted), counted into d_counts like the dense pass, without
   the list ever being written to memory -- the whole r10 pass, sample
   generation (r10:156-185) included.  Equal to pluss_dev_expand_sorted of
   each slice followed by pluss_dev_sampled_hist_dense. */
int pluss_dev_gen_count_dense(pluss_ctx *ctx, uint64_t seed, const uint64_t totals[6], const uint64_t first[6],
                              const uint64_t n[6], uint64_t *d_counts, void *stream);

/* --- faithful mode over key-range shards (multi-GPU) ----------------------
   r10's sampler_<REF> is one sequential pass over the whole key-ordered list
   (r10:187-695); the six references split over shards by contiguous ranges of
   the sort key a*T+tid (IterationComp order, pluss_utils.h:175-267), one shard
   per GPU (or several logical shards per GPU).  Each phase writes this shard's
   summary row (PLUSS_SHARD_ROW u64 words, device memory) and the next phase
   reads the rows of ALL shards, gathered by the caller in shard order (one
   all-gather between phases, e.g. ncclAllGather in place; the group API below
   does it itself).  No phase returns anything to the host, so with device
   all-gathers the pass runs without a host round trip (the selected source
   makes one, in local_selected).  The phases, on one handle per shard:

     1. pluss_dev_faithful_shards_local: this shard's slices -- n[r] samples of
        reference r from index first[r] of its key-ordered list of totals[r]
        samples: d_samples (the slices back to back) or, d_samples == NULL,
        generated (pluss_expand_sorted's lists, seed);
        or, for lists in ANY order, pluss_dev_faithful_shards_select (every
        shard passes the whole lists and keeps its key range [key_lo, key_hi)),
        then, after an all-gather, pluss_dev_faithful_shards_local_selected;
     2. pluss_dev_faithful_shards_carry   (the replay state entering the shard)
     3. pluss_dev_faithful_shards_cut     (r10's Q1 exit over all shards)
     4. pluss_dev_faithful_shards_hist    adds this shard's part of the
        histograms and traversed to the handle; the shards' tables are then
        summed (e.g. all-gather the exports) -- equal to one GPU's pass.
   A shard that fails a phase still takes part in every all-gather with
   row[PLUSS_SHARD_ROW_ERR] != 0; every shard then reports "a key-range shard
   failed" (PLUSS_ERR_PEER) at its next fetch instead of waiting forever.
   The row words (u64): [0,6) samples per reference, [6,12) largest sink,
   [12,18) replay starts, [18,24) first Q1 cut candidate, [31] error.
   Needs N % (chunk*threads) == 0 and N % (cls/ds) == 0. */
#define PLUSS_SHARD_ROW 32
#define PLUSS_SHARD_ROW_ERR 31

/* keys of this shape lie in [0, *key_end) (= accesses per thread * threads) */
int pluss_faithful_key_space(const pluss_cfg *cfg, uint64_t *key_end);

int pluss_dev_faithful_shards_local(pluss_ctx *ctx, const uint64_t *d_samples, uint64_t seed, const uint64_t *totals,
                                    const uint64_t *first, const uint64_t *n, uint64_t *d_row, void *stream);
int pluss_dev_faithful_shards_select(pluss_ctx *ctx, const uint64_t *d_lists, const uint64_t *totals, uint64_t key_lo,
                                     uint64_t key_hi, uint64_t *d_row, void *stream);
int pluss_dev_faithful_shards_local_selected(pluss_ctx *ctx, const uint64_t *d_rows, int32_t shard, int32_t nshards,
                                             uint64_t *d_row, void *stream);
int pluss_dev_faithful_shards_carry(pluss_ctx *ctx, const uint64_t *d_rows, int32_t shard, int32_t nshards,
                                    uint64_t *d_row, void *stream);
int pluss_dev_faithful_shards_cut(pluss_ctx *ctx, const uint64_t *d_rows, int32_t shard, int32_t nshards,
                                  uint64_t *d_row, void *stream);
int pluss_dev_faithful_shards_hist(pluss_ctx *ctx, const uint64_t *d_rows, int32_t shard, int32_t nshards,
                                   void *stream);

/* r10's own law over key-range shards: the lists of pluss_expand_uniform_sorted
   (uniform draws without replacement, r10:156-185, in key order), each shard
   generating only its stretch of every list.  Shard g of G holds, per
   reference, the leaves [L*g/G, L*(g+1)/G) of the key-ordered space (a leaf:
   one key row's block of points), so its samples are contiguous
   in key order.  Its first phase is split in two around one extra all-gather:
     0. pluss_dev_faithful_shards_uniform_count: this shard's candidates per
        reference (row[ROW_N + r], the words [0,6)); all-gather the rows;
     1. pluss_dev_faithful_shards_uniform_local: from the gathered rows, the
        candidates before this shard and in all, the removal of its window, so
        its slice [first, first + n) of each list (read back once: the launch
        grids need n), then the local pass over that slice, generated tile by
        tile (its row as phase 1 of the other sources);
   then carry, cut and hist as above.  The result equals
   pluss_dev_gen_uniform_faithful_refs on one device. */
int pluss_dev_faithful_shards_uniform_count(pluss_ctx *ctx, uint64_t seed, const uint64_t *totals, int32_t shard,
                                            int32_t nshards, uint64_t *d_row, void *stream);
int pluss_dev_faithful_shards_uniform_local(pluss_ctx *ctx, const uint64_t *d_rows, int32_t shard, int32_t nshards,
                                            uint64_t *d_row, void *stream);
/* the slice of each reference's list this handle's last key-range pass ran
   over (after its local phase): indices [first[r], first[r] + n[r]) */
int pluss_dev_faithful_shards_slice(pluss_ctx *ctx, uint64_t first[6], uint64_t n[6]);

/* Host only (no device): [*i_lo, *i_hi) = the indices of the samples of the
   key-order list of `total` samples of reference `ref` (pluss_expand_sorted's
   list) whose faithful keys lie in [key_lo, key_hi) -- the list is in key
   order, so two binary searches of the host generator.  A key-range shard of
   faithful mode generates exactly that slice. */
int pluss_keyorder_index_range(const pluss_cfg *cfg, uint64_t seed, int32_t ref, uint64_t total, uint64_t key_lo,
                               uint64_t key_hi, uint64_t *i_lo, uint64_t *i_hi);

/* --- multi-GPU groups ------------------------------------------------------
   The reference's callers run the six sampler_<REF> of r10 on host threads
   and merge (r10:3191-3278; Rust src/main.rs:17-44); a group runs one pass
   over every GPU of a node instead, and returns the merged histogram.  A
   group is a set of shards: shards_per_device >= 1 logical shards on each
   device (e.g. 8 on one device reproduce an 8-GPU job's partition and
   exchanges).  The exchanges are RCCL collectives over the
   devices (loaded on first use): one all-gather of the shards' summary rows
   between the phases of a faithful pass (no host round trip), and at the end
   of every pass one all-reduce of the shards' dense result vectors (bins,
   cold and traversed counts, one word per failure condition; shapes with
   N % (cls/ds) != 0: one all-gather of the shards' canonical tables).  A
   shard that fails on its host still takes part in every collective with its
   error word set, and every rank returns PLUSS_ERR_PEER (or its own error).  Clean mode shards every reference's sample index range
   (or a host list) into contiguous slices; faithful mode shards the sort key
   a*T+tid into contiguous ranges.  Results equal one device's and are the
   same on every rank.
     pluss_group_create       one process, `ndev` distinct devices (ranks 0..ndev-1)
     pluss_group_create_rank  one process of a multi-process job (one device,
                              cfg->device; rank `rank` of `nranks`): rank 0
                              makes the id with pluss_group_unique_id and the
                              caller hands it to every rank (MPI, a file, ...)
     pluss_group_sampled_hist a host list (every rank passes the same list):
                              clean: slices counted and merged; faithful: the
                              six samplers over the list's per-reference
                              samples (any order), key-range sharded
     pluss_group_gen_faithful the six samplers over generated key-order lists
                              (pluss_expand_sorted's), each shard generating
                              only its key range
     pluss_group_gen_uniform_faithful  the same over r10's own law
                              (pluss_expand_uniform_sorted's lists; equal to
                              pluss_dev_gen_uniform_faithful_refs on one device)
                              (both: one rank on one device captures a second
                              identical call -- same seed and totals, no other
                              group call between -- into a HIP graph without
                              collectives and replays it for later ones;
                              several ranks or devices: eager)
     pluss_group_expand       resident Feistel lists, each shard its slices of
                              counts[r] samples per reference (pluss_expand_samples)
     pluss_group_dense        `passes` dense passes over them (the bench step;
                              one rank on one device: replayed from HIP graphs
                              without collectives, which are identities there;
                              several ranks: eager); out: the last pass's
                              merged dense vector (as pluss_dev_sampled_hist_dense;
                              passes == 0: runs nothing, out all zero)
     pluss_group_gen_count_dense  generated key-order slices counted and merged */
typedef struct pluss_group pluss_group;
#define PLUSS_GROUP_ID_BYTES 128
int pluss_group_unique_id(uint8_t id[PLUSS_GROUP_ID_BYTES]);
int pluss_group_create(const pluss_cfg *cfg, const int32_t *devices, int32_t ndev, int32_t shards_per_device,
                       pluss_group **out);
int pluss_group_create_rank(const pluss_cfg *cfg, int32_t nranks, int32_t rank, const uint8_t id[PLUSS_GROUP_ID_BYTES],
                            int32_t shards_per_device, pluss_group **out);
int pluss_group_destroy(pluss_group *group);
int pluss_group_shards(const pluss_group *group, int32_t *local_shards, int32_t *total_shards);
int pluss_group_sampled_hist(pluss_group *group, const uint64_t *samples, uint64_t n, pluss_hist *out);
int pluss_group_gen_faithful(pluss_group *group, uint64_t seed, const uint64_t totals[6], pluss_hist *out);
int pluss_group_gen_uniform_faithful(pluss_group *group, uint64_t seed, const uint64_t totals[6], pluss_hist *out);
int pluss_group_expand(pluss_group *group, uint64_t seed, const uint64_t counts[6]);
int pluss_group_dense(pluss_group *group, uint32_t passes, uint64_t counts[PLUSS_DENSE_BINS + 1]);
int pluss_group_gen_count_dense(pluss_group *group, uint64_t seed, const uint64_t totals[6],
                                uint64_t counts[PLUSS_DENSE_BINS + 1]);

/* synchronise and copy the handle's histogram into a host pluss_hist */
int pluss_hist_fetch(pluss_ctx *ctx, pluss_hist *out);
/* merge canonical (key,count) tables on the host into a pluss_hist */
int pluss_hist_from_tables(const uint64_t *keys, const uint64_t *counts, uint64_t n_pairs, pluss_hist *out);

#ifdef __cplusplus
}
#endif
#endif /* PLUSS_GPU_H */
