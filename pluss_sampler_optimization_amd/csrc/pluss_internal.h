// pluss_internal.h — handle layout and kernel launchers shared by the
// translation units of libpluss_gpu.so.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/pluss_gpu.h"
#include "pluss_model.h"

namespace pluss {

constexpr int BLOCK = 256;             // 4 waves of 64
constexpr int TCAP = 256;              // LDS histogram slots per workgroup (power of two)
constexpr uint32_t GCAP = 4096;        // main global histogram slots (power of two)
constexpr uint32_t NREP = 8;           // global replica tables (one per XCD-sized group of workgroups)
constexpr uint32_t RCAP = 256;         // slots per replica (power of two)
constexpr int MAX_BLOCKS = 1024;       // 256 CUs x 4 workgroups
constexpr int UNROLL = 2;              // 16-byte sample pairs per lane per step (tools/ablate.py)
constexpr unsigned long long KEY_NONE = 0;  // free table slot (histogram keys are never 0)

constexpr uint32_t NBROW = 64;         // rows of direct (ref, case) counters (workgroup -> row blockIdx % 64)
constexpr uint32_t BSTRIDE = 32;       // u64 per row: 18 counters, [BARRIVE] arrival count; rows 256 B apart
constexpr uint32_t BARRIVE = 31;

// Dense per-pass histogram (pluss_dev_sampled_hist_dense): DBINS u64 counters
// per row (18 (ref, case) keys + the malformed-sample count), each word
// (arrivals << DARR_SHIFT | count) so the last adder of a word knows its total
// from the value its add returned.  dbins: NBROW rows, dtot: one row.
constexpr uint32_t DBINS = 19;
constexpr uint32_t DENSE_ROWS = 32;  // first-level rows of the dense tail (r02 sweep of 1..64 rows, tools/ablate.py)
constexpr int DARR_SHIFT = 44;
constexpr unsigned long long DCNT_MASK = (1ull << DARR_SHIFT) - 1;

// Global histogram state (one per handle), one contiguous allocation so a
// single memset resets it:
//   keys[GCAP] rkeys[NREP*RCAP] counts[GCAP] rcounts[NREP*RCAP] bins[NBROW*BSTRIDE] flags[8] trav[8]
//   (pad to 256 B) dbins[NBROW*BSTRIDE] dtot[BSTRIDE]
// FAST-mode kernels count into `bins` (18 fixed (ref, case) keys, Model::keytab);
// arbitrary exact keys (GENERIC shapes, faithful mode) go to the open-addressing
// replicas, spilling to the main table.
struct GTable {
  unsigned long long* keys;     // GCAP
  unsigned long long* rkeys;    // NREP * RCAP
  unsigned long long* counts;   // GCAP
  unsigned long long* rcounts;  // NREP * RCAP
  unsigned long long* bins;     // NBROW * BSTRIDE
  unsigned int* flags;          // [0] overflow, [1] bad input, [2] diagnostics, [3] main table used,
                                // [4] finished bin rows of a fused count+export launch
  unsigned long long* trav;     // [6] per-ref traversed (faithful) / [0] total (full trace)
  unsigned long long* dbins;    // NBROW * BSTRIDE: dense pass, per-row words (zero between passes)
  unsigned long long* dtot;     // BSTRIDE: dense pass, per-bin words over the rows (zero between passes)
};
// bits of flags[0] (each reported by its own message at the next fetch)
constexpr unsigned int FLAG_OVERFLOW = 1u;  // more distinct histogram keys than the tables hold
constexpr unsigned int FLAG_LOOKBACK = 2u;  // a faithful chunk's predecessor never published (stalled pass)
constexpr unsigned int FLAG_SHARD = 4u;     // a key-range shard of this pass failed (its row's error word)
constexpr unsigned int FLAG_SORT = 8u;      // the bucket sort's plan exceeded its capacity (input left unsorted)
constexpr unsigned int FLAG_UNI = 16u;      // the uniform key-order generator drew too few candidates (P ~ 1e-23)
constexpr size_t DB_OFF = (2 * (size_t)(GCAP + NREP * RCAP) + NBROW * BSTRIDE + 4 + 8 + BSTRIDE - 1) / BSTRIDE * BSTRIDE;
constexpr size_t TABLE_WORDS = DB_OFF + (size_t)(NBROW + 1) * BSTRIDE;
constexpr size_t TABLE_BYTES = TABLE_WORDS * 8;

struct FaithfulBufs {
  uint64_t cap = 0;
  unsigned long long *keys = nullptr, *sinks = nullptr, *keys_s = nullptr, *sinks_s = nullptr, *pmax = nullptr;
  unsigned int* nstart = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  unsigned long long* scal = nullptr;  // [0] cut, [1] cold, [2] traversed, [3] shard size, [4] scan tile counter
  unsigned long long* st = nullptr;    // look-back status words of the one-GPU scan (2 per tile)
  // the scan pipeline (pluss_faithful.hip k_fa_*): per tile the partials, the largest sink, the
  // running max entering it, its first local starts; the queue of tiles to scan again
  uint64_t dcap = 0;
  unsigned long long *dpart = nullptr, *tmax = nullptr, *pmin = nullptr, *klist = nullptr;
  unsigned int* slowq = nullptr;  // tiles the local fast path left: [0] count (zero between passes), then indices
  bool slowq_clean = false;       // slowq[0] is zero on the stream (k_fa_chunk emptied it): no reset launch needed
  bool capture = false;           // the pass is being captured into a graph: chunk flags reset inside it
  uint64_t ccap = 0;              // chunks (of k_fa_chunk's CH tiles) the buffers below hold
  unsigned long long *cval = nullptr, *crec = nullptr;  // per chunk: its largest sink; its summary for the finish
  unsigned int* cflag = nullptr;  // per chunk: the epoch of the pass that published cval (zeroed once)
  uint32_t epoch = 0;             // passes run on these buffers
  unsigned long long* shrec = nullptr;  // key-range shards: per reference the pass-3 record; staging words
  unsigned long long* xin = nullptr;    // key-range shards: this shard's exchange inputs (XIN_*), then 8 counters
  unsigned long long* fslot = nullptr;  // per reference: the main-table slot of its -1 (cold) key
  // the radix source's bucket sort (pluss_sort.h): its histograms, parents, chunk map, deep items
  uint64_t sbcap = 0;
  unsigned char* sbuf = nullptr;
  // the uniform source's sparse-reference tiles, run beside the lane-major pass
  // (fa_launch_t): a second stream and its fork / join events, made on first use
  hipStream_t side = nullptr;
  hipEvent_t sev[2] = {nullptr, nullptr};
};

struct UniSet;  // the uniform key-order generator's plan (pluss_uniform.h)
struct UniBufs {  // its device buffers (grown on demand, per handle)
  UniSet* set = nullptr;
  UniSet* host = nullptr;  // the host copy of *set (built by uni_plan_count, completed by uni_plan_tiles)
  uint32_t *cnt = nullptr, *bits = nullptr, *tmap = nullptr;
  uint64_t *pre = nullptr, *rb = nullptr, *bsum = nullptr;
  double* pmt = nullptr;  // the binomial pmf per leaf size (uni_count_tab)
  unsigned long long* info = nullptr;   // per reference: removed ranks below the plan, its first survivor, survivors
  uint64_t pmt_key[6][10] = {};         // what the CDF tables in pmt were built for (k_ug_pmt runs when it changes)
  bool pmt_valid = false;
  unsigned long long* hinfo = nullptr;  // pinned host copy of info (a key-range shard's one round trip)
  size_t set_cap = 0, cnt_cap = 0, bits_cap = 0, tmap_cap = 0, pre_cap = 0, rb_cap = 0, bsum_cap = 0, pmt_cap = 0,
         info_cap = 0;
};

struct FaShards;  // a key-range shard's state between the phases of pluss_dev_faithful_shards_* (pluss_faithful.h)

}  // namespace pluss

struct pluss_ctx {
  pluss_cfg cfg;
  pluss::Model m;
  int device;
  hipStream_t stream;
  pluss::GTable g;
  void* d_table;  // backing store of g (TABLE_BYTES)
  unsigned long long *d_exp_keys, *d_exp_counts;  // GCAP each, canonical export
  unsigned int* d_exp_n;
  pluss::FaithfulBufs fb;
  pluss::FaShards* fsh2;  // created on first use (faith_shards_local), freed by faith_shards_free
  pluss::FaithfulBufs fbr[6];  // per-reference buffers of pluss_dev_faithful_hist_refs
  pluss::UniBufs ub;           // the uniform key-order generator's plan
  hipStream_t fst[6];          // ... and its streams (created on first use)
  hipEvent_t fev[7];           // fork / join events
  hipStream_t last;   // stream of the most recent launch (fetch orders after it; NULL: HIP's null stream)
  bool has_last;      // a launch has set `last` (before the first: the handle's own stream)
  bool tables_dirty;  // hash tables may hold counts (GENERIC / faithful launches since the last reset)
};

namespace pluss {

// error plumbing
void set_error(const std::string& msg);
#define PLUSS_HIP_CHECK(expr)                                                                            \
  do {                                                                                                   \
    hipError_t e_ = (expr);                                                                              \
    if (e_ != hipSuccess) {                                                                              \
      ::pluss::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                             \
      return PLUSS_ERR_HIP;                                                                              \
    }                                                                                                    \
  } while (0)

// Diagnostic builds only (-DPLUSS_DEBUG_STAGES, build.py variant "stages", never
// the product library): after each named stage the stream is drained and the
// stage's outcome printed to stderr, so a device fault is pinned to the first
// stage that reports it.  Compiles to nothing in the product build.
#ifdef PLUSS_DEBUG_STAGES
void debug_stage(hipStream_t s, const char* what);
int debug_knob(const char* name);  // a diagnostic switch (environment PLUSS_KNOB_<name>; 0 when unset)
#define PLUSS_STAGE(s, what) ::pluss::debug_stage((s), (what))
#define PLUSS_KNOB(name) ::pluss::debug_knob(name)
#else
#define PLUSS_STAGE(s, what) ((void)0)
#define PLUSS_KNOB(name) 0
#endif

int validate_cfg(const pluss_cfg* cfg, Model* m);
// the error reported by a pass's flags (flags[0] bits, flags[1] malformed input), or PLUSS_OK
int flags_error(unsigned int f0, unsigned int bad, const std::string& who);

// launchers (return PLUSS_OK or PLUSS_ERR_*)
int launch_table_reset(pluss_ctx* ctx, hipStream_t s);
int launch_sampled_hist(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, hipStream_t s);
int launch_fulltrace(pluss_ctx* ctx, hipStream_t s);
int launch_ri_dump(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, int64_t* d_ri, uint64_t* d_sink,
                   hipStream_t s);
int launch_expand(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t first, uint64_t n, uint64_t* d_out,
                  hipStream_t s);
// key-order stratified lists (pluss_model.h KeyGen)
int keygen_check(const pluss_ctx* ctx, int32_t ref, uint64_t total, uint64_t first, uint64_t n, const char* api);
KeyGen keygen_of(const pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total);
int launch_expand_sorted(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first, uint64_t n,
                         uint64_t* d_out, hipStream_t s);
// generated key-order lists counted without materialising them (dense vector)
int launch_gen_count_dense(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, const uint64_t* first,
                           const uint64_t* n, unsigned long long* d_counts, hipStream_t s);
int launch_export(pluss_ctx* ctx, unsigned long long* d_keys, unsigned long long* d_counts, uint64_t cap,
                  hipStream_t s, bool consume = false);
// count a sample list and export-and-reset in one launch when only the direct
// bins can hold counts (FAST shapes); otherwise the two launches
int launch_sampled_hist_export(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, unsigned long long* d_keys,
                               unsigned long long* d_counts, uint64_t cap, hipStream_t s);
// count a sample list into a caller-owned dense vector of DBINS counts (FAST shapes), one launch
int launch_sampled_hist_dense(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, unsigned long long* d_counts,
                              hipStream_t s);
// diagnostics (include/pluss_diag.h): a dense pass with an ablation variant and/or a workgroup cap
int launch_diag_dense(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t n, unsigned long long* d_counts,
                      int variant, int max_grid, hipStream_t s);
int launch_faithful(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, hipStream_t s);
int launch_faithful_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t* counts, hipStream_t s);
int diag_sort_words(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, void* d_words,
                    int32_t* word_bytes, hipStream_t s);
// faithful mode over key-ordered lists (no sort) and generated key-order lists (no input)
int launch_faithful_sorted(pluss_ctx* ctx, int32_t ref, const uint64_t* d_samples, uint64_t n, hipStream_t s);
int launch_faithful_sorted_refs(pluss_ctx* ctx, const uint64_t* d_samples, const uint64_t* counts, hipStream_t s);
int launch_gen_faithful_refs(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, hipStream_t s);
// key-range shards of the single-read pipeline (all six references at once;
// summary rows in device memory, include/pluss_gpu.h PLUSS_SHARD_ROW)
int faith_shards_local(pluss_ctx* ctx, const uint64_t* d_samples, uint64_t seed, const uint64_t* totals,
                       const uint64_t* first, const uint64_t* n, uint64_t* d_row, hipStream_t s);
int faith_shards_select(pluss_ctx* ctx, const uint64_t* d_lists, const uint64_t* totals, uint64_t key_lo,
                        uint64_t key_hi, uint64_t* d_row, hipStream_t s);
int faith_shards_local_selected(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                uint64_t* d_row, hipStream_t s);
// arbitrary-order lists partitioned by (key-range shard, reference) on the
// device (the group's any-order faithful pass), and phase 1 over the words
uint32_t faith_part_blocks(uint64_t n, uint32_t S);
int faith_word_bytes(const pluss_ctx* ctx);
// (the count over workgroup blocks [b0, b1) of the B, and the bins' scan and
// totals when `scan`: the whole count is [0, B) with the scan; a caller that
// uploads the list in pieces counts each piece's blocks as it lands)
int faith_part_count(pluss_ctx* ctx, const uint64_t* d_smp, uint64_t n, const unsigned long long* d_bounds,
                     uint32_t S, uint32_t* d_hist, uint32_t B, unsigned long long* d_tot, hipStream_t s,
                     uint32_t b0 = 0, uint32_t b1 = ~0u, bool scan = true);
int faith_part_scatter(pluss_ctx* ctx, const uint64_t* d_smp, uint64_t n, const unsigned long long* d_bounds,
                       uint32_t S, uint32_t* d_hist, uint32_t B, const unsigned long long* d_rstart, void* d_out,
                       hipStream_t s);
int faith_seg_copy(const unsigned long long* d_seg, uint32_t nseg, uint64_t maxn, const void* src, void* dst,
                   int wbytes, hipStream_t s);
int faith_shards_local_words(pluss_ctx* ctx, const void* const in[6], const uint64_t* cnt, const uint64_t* all,
                             const uint64_t* before, uint64_t* d_row, hipStream_t s);
int faith_shards_carry(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards, uint64_t* d_row,
                       hipStream_t s);
int faith_shards_cut(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards, uint64_t* d_row,
                     hipStream_t s);
int faith_shards_hist(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards, hipStream_t s);
// r10's uniform law over key-range shards: candidates counted (phase 0), then
// the window (enqueued, slice read back asynchronously) and the local pass
int faith_shards_uniform_count(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, int32_t shard, int32_t nshards,
                               uint64_t* d_row, hipStream_t s);
// (known: the slice's 12 raw info words -- first[6], n[6] -- from an earlier
// identical pass: no read-back, nothing waits on the host, and the device's
// own values are checked against them (FLAG_UNI on a difference); the window
// then skips its copy to the host (to_host false).  A group's captured pass.)
int faith_shards_uniform_window(pluss_ctx* ctx, const uint64_t* d_rows, int32_t shard, int32_t nshards,
                                hipStream_t s, bool to_host = true);
int faith_shards_uniform_finish(pluss_ctx* ctx, uint64_t* d_row, hipStream_t s, const uint64_t* known = nullptr);
int faith_shards_slice(pluss_ctx* ctx, uint64_t* first, uint64_t* n);
void faith_shards_abandon(pluss_ctx* ctx);
// r10's uniform draw in key order (pluss_uniform.h / .hip)
int uni_check(const pluss_ctx* ctx, int32_t ref, uint64_t total, const char* api);
int uni_plan(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, hipStream_t s, const UniSet** out);
int uni_plan_count(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, uint32_t shard, uint32_t ns, hipStream_t s);
int uni_plan_remove(pluss_ctx* ctx, const unsigned long long* rows, uint32_t shard, uint32_t ns, hipStream_t s);
int uni_plan_tiles(pluss_ctx* ctx, const uint64_t* n, hipStream_t s, const UniSet** out);
// the plan's slice words (info[6, 18)) checked against known values (FLAG_UNI on a difference)
int uni_slice_check(pluss_ctx* ctx, const uint64_t* known, hipStream_t s);
void uni_free(pluss_ctx* ctx);
int diag_uniform_parts(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, int32_t what, uint64_t* d_out,
                       hipStream_t s);
int launch_expand_uniform_sorted(pluss_ctx* ctx, uint64_t seed, int32_t ref, uint64_t total, uint64_t first,
                                 uint64_t n, uint64_t* d_out, hipStream_t s);
int launch_gen_uniform_faithful_refs(pluss_ctx* ctx, uint64_t seed, const uint64_t* totals, hipStream_t s);  // a one-GPU faithful call ends any half-finished shard pass
void faith_shards_free(pluss_ctx* ctx);

}  // namespace pluss
