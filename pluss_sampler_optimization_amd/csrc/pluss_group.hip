// pluss_group.hip — multi-GPU behind the C ABI (include/pluss_gpu.h,
// pluss_group_*): one process drives a set of shards over one or more HIP
// devices (one pluss_ctx per shard, several logical shards per device if
// asked), or one rank of a multi-process job.  The exchanges run on the
// devices over RCCL (xGMI): one all-reduce of the 19-word dense vector per
// clean pass, one all-gather of the shards' summary rows between the phases
// of a faithful pass, one all-gather of the canonical tables at the end.
//
// Replaces what the reference's callers would otherwise have to write around
// the one-GPU entry points: r10's main (six sampler_<REF> threads, then the
// merge, r10:3191-3278) and the Rust main (src/main.rs:17-44) reach every GPU
// of a node through these calls.  RCCL is loaded on first use (dlopen of
// librccl.so.1: the copy a PyTorch process already mapped, else ROCm's), so
// one-GPU users of libpluss_gpu.so never load it.
//
// Shards are numbered device-major: global shard g = rank * spd + j lives on
// the device of RCCL rank `rank` (one per device; a process's local devices
// are ranks 0..ndev-1 of its own communicator, or its one device is rank
// `rank` of a multi-process communicator) as its j-th logical shard.
// Clean mode: shard g takes the slice [c*g/S, c*(g+1)/S) of every reference's
// index range (or of a host list).  Faithful mode: shard g takes the sort-key
// range [K*g/S, K*(g+1)/S) (K = pluss_faithful_key_space).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "pluss_faithful.h"

namespace pluss {

// ---- RCCL, loaded on first use ------------------------------------------------
struct Rccl {
  bool tried = false, ok = false;
  std::string why;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
static Rccl g_rccl;

static Rccl* rccl() {
  Rccl& R = g_rccl;
  if (R.tried) return R.ok ? &R : nullptr;
  R.tried = true;
  void* h = nullptr;
  for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
    if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
  if (!h) {
    R.why = std::string("cannot load librccl.so.1: ") + dlerror();
    return nullptr;
  }
  auto sym = [&](const char* s) {
    void* p = dlsym(h, s);
    if (!p && R.why.empty()) R.why = std::string("librccl.so.1 lacks ") + s;
    return p;
  };
  R.GetUniqueId = (decltype(R.GetUniqueId))sym("ncclGetUniqueId");
  R.CommInitRank = (decltype(R.CommInitRank))sym("ncclCommInitRank");
  R.CommInitAll = (decltype(R.CommInitAll))sym("ncclCommInitAll");
  R.CommDestroy = (decltype(R.CommDestroy))sym("ncclCommDestroy");
  R.AllReduce = (decltype(R.AllReduce))sym("ncclAllReduce");
  R.AllGather = (decltype(R.AllGather))sym("ncclAllGather");
  R.Send = (decltype(R.Send))sym("ncclSend");
  R.Recv = (decltype(R.Recv))sym("ncclRecv");
  R.GroupStart = (decltype(R.GroupStart))sym("ncclGroupStart");
  R.GroupEnd = (decltype(R.GroupEnd))sym("ncclGroupEnd");
  R.GetErrorString = (decltype(R.GetErrorString))sym("ncclGetErrorString");
  R.ok = R.why.empty();
  return R.ok ? &R : nullptr;
}

#define PLUSS_NCCL_CHECK(expr)                                                                       \
  do {                                                                                               \
    ncclResult_t r_ = (expr);                                                                        \
    if (r_ != ncclSuccess) {                                                                         \
      ::pluss::set_error(std::string(#expr) + ": " + g_rccl.GetErrorString(r_));                     \
      return PLUSS_ERR_HIP;                                                                          \
    }                                                                                                \
  } while (0)

// a HIP call's result as a PLUSS_* code (the error message set), without returning
static int hip_rc(hipError_t e, const char* what) {
  if (e == hipSuccess) return PLUSS_OK;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return PLUSS_ERR_HIP;
}

// per shard, the block all-gathered at the end of a one-shot pass over a shape
// with arbitrary keys (N % (cls/ds) != 0): its canonical table (GCAP keys, GCAP
// counts), traversed[8], flags[7] and a local-failure word
constexpr size_t GBLOCK = 2 * (size_t)GCAP + 16;
constexpr int GB_FAIL = 15;  // (tail word: nonzero when the shard failed on the host)

// The dense result vector of a shard (one slot of DVEC words; every shape with
// N % (cls/ds) == 0): a pass's whole histogram is then a fixed set of words,
// merged over the shards by a sum (one RCCL all-reduce) -- the 18 (ref, case)
// bins, the malformed count, per reference the -1 (cold) key's count and
// whether some shard materialised it (faithful mode, r10:196,671),
// traversed, and one word per failure condition (the number of shards that
// met it).  A shard that fails on the host still sends its slot, with the
// local-failure word set, so no rank waits in the all-reduce.
constexpr int DVEC = 48;
constexpr size_t MAX_RETIRED = 64;  // replaced graphs kept by a group (pluss_group::retired)
enum : int { GV_BAD = 18, GV_COLD = 19, GV_PRES = 25, GV_TRAV = 31, GV_COND = 37, GV_W = 45 };
enum : int { GC_LOCAL = 0, GC_BAD = 1, GC_OVERFLOW = 2, GC_LOOKBACK = 3, GC_SHARD = 4, GC_SORT = 5, GC_UNI = 6,
             GC_NONDENSE = 7 };

__global__ void k_group_sum(const unsigned long long* __restrict__ vecs, int n, unsigned long long* __restrict__ out) {
  const int i = threadIdx.x;
  if (i >= GV_W) return;
  unsigned long long s = 0;
  for (int j = 0; j < n; ++j) s += vecs[j * DVEC + i];
  out[i] = s;
}

// a shard's slot from its handle's histogram state: the direct bins folded over
// their rows, the tables' -1 keys (any other key: GC_NONDENSE, the merge falls
// back to the tables), traversed and the flags
__global__ __launch_bounds__(256) void k_group_vec(Model m, GTable g, unsigned long long* __restrict__ slot, int fail) {
  __shared__ unsigned long long v[GV_W];
  const uint32_t t = threadIdx.x;
  if (t < GV_W) v[t] = 0;
  __syncthreads();
  if (t < 18) {
    unsigned long long x = 0;
    for (uint32_t row = 0; row < NBROW; ++row) x += g.bins[row * BSTRIDE + t];
    v[t] = x;
  } else if (t >= 32 && t < 38) {
    v[GV_TRAV + (t - 32)] = g.trav[t - 32];
  } else if (t == 64) {
    const unsigned int f0 = g.flags[0];
    v[GV_COND + GC_LOCAL] = fail ? 1u : 0u;
    v[GV_COND + GC_BAD] = g.flags[1] ? 1u : 0u;
    v[GV_COND + GC_OVERFLOW] = (f0 & FLAG_OVERFLOW) ? 1u : 0u;
    v[GV_COND + GC_LOOKBACK] = (f0 & FLAG_LOOKBACK) ? 1u : 0u;
    v[GV_COND + GC_SHARD] = (f0 & FLAG_SHARD) ? 1u : 0u;
    v[GV_COND + GC_SORT] = (f0 & FLAG_SORT) ? 1u : 0u;
    v[GV_COND + GC_UNI] = (f0 & FLAG_UNI) ? 1u : 0u;
  }
  __syncthreads();
  for (uint32_t i = t; i < GCAP + NREP * RCAP; i += 256) {
    const unsigned long long k = i < GCAP ? g.keys[i] : g.rkeys[i - GCAP];
    if (k == KEY_NONE) continue;
    const unsigned long long c = i < GCAP ? g.counts[i] : g.rcounts[i - GCAP];
    const uint32_t r = key_ref(k);
    if (r < 6 && key_kind(k) == 0 && key_ri(k) == -1) {
      atomicAdd(&v[GV_COLD + r], c);
      v[GV_PRES + r] = 1;
      continue;
    }
    int b = -1;
#pragma unroll
    for (int x = 0; x < 18; ++x) b = m.keytab[x] == k ? x : b;
    if (b >= 0) atomicAdd(&v[b], c);
    else v[GV_COND + GC_NONDENSE] = 1;
  }
  __syncthreads();
  if (t < GV_W) slot[t] = v[t];
}

// a slot (or a gathered row / block) of a shard that failed on the host
__global__ void k_group_word(unsigned long long* w, unsigned long long v) { *w = v; }

// a shard's traversed and flags words into its gathered block
__global__ void k_group_block_tail(GTable g, unsigned long long* __restrict__ blk) {
  const int i = threadIdx.x;
  if (i < 8) blk[2 * GCAP + i] = g.trav[i];
  else if (i < 15) blk[2 * GCAP + i] = g.flags[i - 8];
}

// A faithful pass replayed from a HIP graph (one local device): the same call
// as the last one (source, seed, totals) captures the whole device side --
// table resets, the phases of every shard, the row gathers, the slots and the
// all-reduce -- once, and later identical calls replay it; the host then only
// fetches the merged vector.  Anything else runs eagerly and drops the graph.
// (~12 launches per shard and 5 collectives per pass: on 8 logical shards the
// host's launch rate, not the device, set the call's time.)
struct FaGraph {
  bool have = false, seen = false;
  int src = 0;  // 0 generated (gen_faithful), 1 uniform (gen_uniform_faithful)
  uint64_t seed = 0, totals[6] = {0, 0, 0, 0, 0, 0};
  std::vector<uint64_t> slice;  // (uniform) each local shard's slice from the last eager pass: first[6], n[6]
  hipGraphExec_t ex = nullptr;
};

// A device's buffers of the any-order faithful pass (grown on demand): its
// slice of the caller's list, the range bounds, the per-block bin counts, the
// all-gathered bin totals of every device, the bins' starts, the words placed
// by (shard, reference), and, over several devices, the received words, the
// words in per-shard order and the copy segments; host copies kept alive
// until the call's streams drain.
struct PartBufs {
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
  };
  Buf smp, bounds, hist, tot, rstart, words, recv, fin, seg;
  std::vector<unsigned long long> h_bounds, h_rstart, h_seg;
};

}  // namespace pluss

using namespace pluss;

struct pluss_group {
  pluss_cfg cfg;
  Model m;
  int ndev = 0, spd = 1;          // local devices, logical shards per device
  int nranks = 1, rank0 = 0;      // RCCL ranks; the rank of local device 0
  int nshards = 1;                // all shards of the job (nranks * spd)
  std::vector<int> dev;           // local device ordinals
  std::vector<pluss_ctx*> ctx;    // local shards, device-major
  std::vector<ncclComm_t> comm;   // per local device
  std::vector<hipStream_t> xs;    // per local device: the exchange stream
  std::vector<hipEvent_t> ev;     // per local shard / device: join events
  std::vector<unsigned long long*> rows;  // per device: nshards * ROW_W
  std::vector<unsigned long long*> vec;   // per device: spd dense vectors, then the merged one
  std::vector<unsigned long long*> blk;   // per device: nshards * GBLOCK
  std::vector<unsigned long long*> list;  // per local shard: resident samples (pluss_group_expand)
  std::vector<uint64_t> list_n;
  std::vector<unsigned long long*> hl;    // per local shard: its slice of a host list (clean sampled_hist)
  std::vector<uint64_t> hl_cap;
  std::vector<pluss::PartBufs> part;      // per device: the any-order faithful pass
  std::map<uint32_t, hipGraphExec_t> graphs;  // dense passes captured per batch size (one local device)
  pluss::FaGraph* fg = nullptr;               // the last faithful pass, captured (pluss_group_gen_faithful)
  // Replaced graphs, kept until the group is destroyed, never destroyed
  // before: on this ROCm (7.2), the first hipGraphLaunch of a graph
  // instantiated after another graph of the process was destroyed crashed
  // inside the HIP runtime on the host, intermittently (r5m; r6x: a
  // segmentation fault in hipGraphLaunch in round 1 of the replay probe;
  // with replaced graphs kept, 20 of 20 rounds clean, r6y).  At most
  // MAX_RETIRED: past that the group stops capturing and runs eagerly.
  std::vector<hipGraphExec_t> retired;
  // A pass being captured into a HIP graph.  The rule, one for every rank
  // count: a one-rank group makes no RCCL call at all (every collective is
  // the identity there: each shard writes its block of the one buffer), so
  // its captured passes hold none; groups of several ranks never capture and
  // run every pass eagerly.  (r5m: a host segfault while replaying a pass
  // whose capture held RCCL calls; r5p: a device fault in back-to-back
  // one-rank passes)
  bool capturing = false;
  std::vector<unsigned long long*> agr;       // per device: a failure word summed over the ranks (agree_failed)
};

namespace pluss {

static int gshard(const pluss_group* G, int d, int j) { return (G->rank0 + d) * G->spd + j; }
static pluss_ctx* shard(pluss_group* G, int d, int j) { return G->ctx[(size_t)d * G->spd + j]; }

static void group_free(pluss_group* G) {
  for (int d = 0; d < G->ndev; ++d) {
    (void)hipSetDevice(G->dev[d]);
    if (d < (int)G->xs.size() && G->xs[d]) (void)hipStreamSynchronize(G->xs[d]);
  }
  for (auto& kv : G->graphs) (void)hipGraphExecDestroy(kv.second);
  if (G->fg) {
    if (G->fg->ex) (void)hipGraphExecDestroy(G->fg->ex);
    delete G->fg;
  }
  for (hipGraphExec_t e : G->retired) (void)hipGraphExecDestroy(e);
  for (size_t i = 0; i < G->ctx.size(); ++i) {
    if (i < G->list.size() && G->list[i]) (void)hipFree(G->list[i]);
    if (i < G->hl.size() && G->hl[i]) (void)hipFree(G->hl[i]);
    if (G->ctx[i]) pluss_ctx_destroy(G->ctx[i]);
  }
  for (int d = 0; d < G->ndev; ++d) {
    (void)hipSetDevice(G->dev[d]);
    for (auto* v : {&G->rows, &G->vec, &G->blk, &G->agr})
      if (d < (int)v->size() && (*v)[d]) (void)hipFree((*v)[d]);
    if (d < (int)G->part.size()) {
      PartBufs& P = G->part[d];
      for (auto* b : {&P.smp, &P.bounds, &P.hist, &P.tot, &P.rstart, &P.words, &P.recv, &P.fin, &P.seg})
        if (b->p) (void)hipFree(b->p);
    }
    if (d < (int)G->comm.size() && G->comm[d] && g_rccl.ok) (void)g_rccl.CommDestroy(G->comm[d]);
    if (d < (int)G->xs.size() && G->xs[d]) (void)hipStreamDestroy(G->xs[d]);
  }
  for (auto e : G->ev)
    if (e) (void)hipEventDestroy(e);
  delete G;
}

// contexts, streams, events and exchange buffers once the ranks are known
static int group_setup(pluss_group* G) {
  const int S = G->spd;
  G->ctx.assign((size_t)G->ndev * S, nullptr);
  G->list.assign(G->ctx.size(), nullptr);
  G->list_n.assign(G->ctx.size(), 0);
  G->hl.assign(G->ctx.size(), nullptr);
  G->hl_cap.assign(G->ctx.size(), 0);
  G->xs.assign(G->ndev, nullptr);
  G->ev.assign(G->ctx.size() + G->ndev, nullptr);
  G->rows.assign(G->ndev, nullptr);
  G->vec.assign(G->ndev, nullptr);
  G->blk.assign(G->ndev, nullptr);
  G->agr.assign(G->ndev, nullptr);
  G->part.assign(G->ndev, PartBufs{});
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    for (int j = 0; j < S; ++j) {
      pluss_cfg c = G->cfg;
      c.device = G->dev[d];
      if (int rc = pluss_ctx_create(&c, &G->ctx[(size_t)d * S + j])) return rc;
    }
    PLUSS_HIP_CHECK(hipStreamCreateWithFlags(&G->xs[d], hipStreamNonBlocking));
    PLUSS_HIP_CHECK(hipMalloc((void**)&G->rows[d], (size_t)G->nshards * ROW_W * 8));
    PLUSS_HIP_CHECK(hipMemset(G->rows[d], 0, (size_t)G->nshards * ROW_W * 8));
    PLUSS_HIP_CHECK(hipMalloc((void**)&G->vec[d], (size_t)(S + 1) * DVEC * 8));
    PLUSS_HIP_CHECK(hipMemset(G->vec[d], 0, (size_t)(S + 1) * DVEC * 8));
    PLUSS_HIP_CHECK(hipMalloc((void**)&G->blk[d], (size_t)G->nshards * GBLOCK * 8));
    PLUSS_HIP_CHECK(hipMalloc((void**)&G->agr[d], 64));
    // the any-order pass's gathered bin totals (R x 6S words): allocated here,
    // so no rank can miss that all-gather for want of its buffer
    PartBufs::Buf& tb = G->part[d].tot;
    tb.cap = (size_t)G->nranks * 6 * G->nshards * 8;
    PLUSS_HIP_CHECK(hipMalloc(&tb.p, tb.cap));
  }
  for (auto& e : G->ev) PLUSS_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return PLUSS_OK;
}

static int group_check_cfg(const pluss_cfg* cfg, int32_t spd, Model* m) {
  if (int rc = validate_cfg(cfg, m)) return rc;
  if (spd < 1 || spd > 64) {
    set_error("pluss_group: shards_per_device must be in [1, 64]");
    return PLUSS_ERR_CONFIG;
  }
  return PLUSS_OK;
}

// every local shard's stream joins its device's exchange stream
static int join_shards(pluss_group* G) {
  for (int d = 0; d < G->ndev; ++d)
    for (int j = 0; j < G->spd; ++j) {
      const size_t i = (size_t)d * G->spd + j;
      PLUSS_HIP_CHECK(hipEventRecord(G->ev[i], G->ctx[i]->stream));
      PLUSS_HIP_CHECK(hipStreamWaitEvent(G->xs[d], G->ev[i], 0));
    }
  return PLUSS_OK;
}
// ... and forks back: every shard stream waits for its device's exchange
static int fork_shards(pluss_group* G) {
  for (int d = 0; d < G->ndev; ++d) {
    hipEvent_t e = G->ev[G->ctx.size() + d];
    PLUSS_HIP_CHECK(hipEventRecord(e, G->xs[d]));
    for (int j = 0; j < G->spd; ++j) PLUSS_HIP_CHECK(hipStreamWaitEvent(G->ctx[(size_t)d * G->spd + j]->stream, e, 0));
  }
  return PLUSS_OK;
}

// in-place all-gather of per-shard blocks of `w` u64 words over the ranks
// (each device holds every shard's slot; its own shards' slots are written)
static int gather_blocks(pluss_group* G, std::vector<unsigned long long*>& buf, size_t w) {
  if (int rc = join_shards(G)) return rc;
  // (one rank: every shard wrote its block of the one buffer, the all-gather
  // is the identity and is left out -- the rule at pluss_group::capturing)
  if (G->nranks == 1) return fork_shards(G);
  PLUSS_NCCL_CHECK(g_rccl.GroupStart());
  for (int d = 0; d < G->ndev; ++d) {
    unsigned long long* own = buf[d] + (size_t)(G->rank0 + d) * G->spd * w;
    PLUSS_NCCL_CHECK(g_rccl.AllGather(own, buf[d], (size_t)G->spd * w, ncclUint64, G->comm[d], G->xs[d]));
  }
  PLUSS_NCCL_CHECK(g_rccl.GroupEnd());
  PLUSS_STAGE(G->xs[0], "group: all-gather");
  return fork_shards(G);
}

static void shard_ranges(uint64_t c, int g, int S, uint64_t* first, uint64_t* n) {
  const uint64_t lo = (uint64_t)((unsigned __int128)c * g / S), hi = (uint64_t)((unsigned __int128)c * (g + 1) / S);
  *first = lo;
  *n = hi - lo;
}

// The first error of a group call on this rank (the local shards' own),
// kept while the call still runs every collective.
struct GErr {
  int rc = PLUSS_OK;
  std::string msg;
  void note(int r) {
    if (r && !rc) {
      rc = r;
      msg = pluss_last_error();
    }
  }
  void note(int r, const std::string& m) {
    if (r && !rc) {
      rc = r;
      msg = m;
    }
  }
};

// The end of a one-shot pass over a shape with arbitrary keys: every shard's
// canonical table, traversed, flags and failure word all-gathered, summed on
// the host (the same on every rank).  This rank's first error wins; a shard
// that failed anywhere fails the pass on every rank (PLUSS_ERR_PEER).
static int collect_tables(pluss_group* G, GErr& E, pluss_hist* out) {
  for (int d = 0; d < G->ndev; ++d) {
    E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
    for (int j = 0; j < G->spd; ++j) {
      pluss_ctx* c = shard(G, d, j);
      unsigned long long* b = G->blk[d] + (size_t)gshard(G, d, j) * GBLOCK;
      const int rc = pluss_dev_hist_export(c, (uint64_t*)b, (uint64_t*)(b + GCAP), GCAP, c->stream);
      E.note(rc);
      hipLaunchKernelGGL(k_group_block_tail, dim3(1), dim3(64), 0, c->stream, c->g, b);
      hipLaunchKernelGGL(k_group_word, dim3(1), dim3(1), 0, c->stream, b + 2 * GCAP + GB_FAIL, E.rc ? 1ull : 0ull);
      E.note(hip_rc(hipGetLastError(), "group block"));
    }
  }
  if (int rc = gather_blocks(G, G->blk, GBLOCK)) return rc;
  std::vector<unsigned long long> h((size_t)G->nshards * GBLOCK);
  PLUSS_HIP_CHECK(hipSetDevice(G->dev[0]));
  PLUSS_HIP_CHECK(hipMemcpyAsync(h.data(), G->blk[0], h.size() * 8, hipMemcpyDeviceToHost, G->xs[0]));
  for (int d = 0; d < G->ndev; ++d) PLUSS_HIP_CHECK(hipStreamSynchronize(G->xs[d]));
  if (E.rc) {
    set_error(E.msg);
    return E.rc;
  }
  std::vector<uint64_t> keys, cnts;
  keys.reserve((size_t)G->nshards * GCAP);
  cnts.reserve((size_t)G->nshards * GCAP);
  uint64_t trav[6] = {0, 0, 0, 0, 0, 0};
  for (int g = 0; g < G->nshards; ++g) {
    const unsigned long long* b = h.data() + (size_t)g * GBLOCK;
    if (b[2 * GCAP + GB_FAIL]) {
      set_error("shard " + std::to_string(g) + " of this group pass failed on its host");
      return PLUSS_ERR_PEER;
    }
  }
  for (int g = 0; g < G->nshards; ++g) {
    const unsigned long long* b = h.data() + (size_t)g * GBLOCK;
    const unsigned long long* fl = b + 2 * GCAP + 8;
    if (int rc = flags_error((unsigned int)fl[0], (unsigned int)fl[1], "shard " + std::to_string(g) + ": "))
      return rc;
    for (uint32_t i = 0; i < GCAP; ++i) {
      if (b[i] == KEY_EMPTY || b[i] == KEY_NONE) break;  // sorted, empties last
      keys.push_back(b[i]);
      cnts.push_back(b[GCAP + i]);
    }
    for (int r = 0; r < 6; ++r) trav[r] += b[2 * GCAP + r];
  }
  if (int rc = pluss_hist_from_tables(keys.data(), cnts.data(), keys.size(), out)) return rc;
  for (int r = 0; r < 6; ++r) out->traversed[r] = trav[r];
  return PLUSS_OK;
}

static int group_reset(pluss_group* G, GErr& E) {
  for (int d = 0; d < G->ndev; ++d) {
    E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
    for (int j = 0; j < G->spd; ++j) {
      pluss_ctx* c = shard(G, d, j);
      E.note(pluss_dev_hist_reset(c, c->stream));
    }
  }  // (the dense slots need no reset: k_group_vec and k_group_sum write every word)
  return E.rc;
}

// a shard's step: its error noted (first one wins) and its summary row marked
// failed, so every shard learns of it at the next gather
using ShardFn = std::function<int(pluss_ctx*, int d, int j, int g, uint64_t* row)>;

// One faithful key-range pass over the local shards, the rows exchanged
// between the phases: phase1 (each shard's first phase), then, after the
// first gather, the optional mid steps (mid1 on every shard, then mid2 on
// every shard: a source whose local phase needs the gathered rows, e.g. the
// uniform source's window, enqueued on all shards before any waits), then
// carry, cut and hist.  Returns only errors of the collectives themselves;
// shard failures are in E and in the rows.
static int group_faithful(pluss_group* G, const ShardFn& phase1, const ShardFn& mid1, const ShardFn& mid2,
                          GErr& E) {
  auto each = [&](const ShardFn& fn) {
    for (int d = 0; d < G->ndev; ++d) {
      (void)hipSetDevice(G->dev[d]);
      for (int j = 0; j < G->spd; ++j) {
        const int g = gshard(G, d, j);
        pluss_ctx* c = shard(G, d, j);
        unsigned long long* row = G->rows[d] + (size_t)g * ROW_W;
        if (const int rc = fn(c, d, j, g, (uint64_t*)row)) {
          E.note(rc);
          hipLaunchKernelGGL(k_group_word, dim3(1), dim3(1), 0, c->stream, row + ROW_ERR, 1ull);
        }
      }
    }
  };
  each(phase1);
  if (int rc = gather_blocks(G, G->rows, ROW_W)) return rc;
  if (mid1) {
    each(mid1);
    if (mid2) {
      // mid1 reads every shard's gathered row, and mid2's local phase writes
      // its own row into the same buffer: every local shard's mid1 first (the
      // uniform window reads the candidate counts that a local phase's sample
      // counts overwrite; without this join a captured 8-shard pass read them
      // half overwritten, r6v)
      if (int rc = join_shards(G)) return rc;
      if (int rc = fork_shards(G)) return rc;
      each(mid2);
    }
    if (int rc = gather_blocks(G, G->rows, ROW_W)) return rc;
  }
  each([&](pluss_ctx* c, int d, int, int g, uint64_t* row) {
    return pluss_dev_faithful_shards_carry(c, (const uint64_t*)G->rows[d], g, G->nshards, row, c->stream);
  });
  if (int rc = gather_blocks(G, G->rows, ROW_W)) return rc;
  each([&](pluss_ctx* c, int d, int, int g, uint64_t* row) {
    return pluss_dev_faithful_shards_cut(c, (const uint64_t*)G->rows[d], g, G->nshards, row, c->stream);
  });
  if (int rc = gather_blocks(G, G->rows, ROW_W)) return rc;
  each([&](pluss_ctx* c, int d, int, int g, uint64_t*) {
    return pluss_dev_faithful_shards_hist(c, (const uint64_t*)G->rows[d], g, G->nshards, c->stream);
  });
  return PLUSS_OK;
}

// the slots of the local shards summed per device, all-reduced over the ranks, on the exchange streams
static int dense_merge(pluss_group* G) {
  if (int rc = join_shards(G)) return rc;
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(64), 0, G->xs[d], (const unsigned long long*)G->vec[d], G->spd,
                       G->vec[d] + (size_t)G->spd * DVEC);
  }
  PLUSS_HIP_CHECK(hipGetLastError());
  if (G->nranks == 1) return fork_shards(G);  // (one rank: the all-reduce is the identity)
  PLUSS_NCCL_CHECK(g_rccl.GroupStart());
  for (int d = 0; d < G->ndev; ++d) {
    unsigned long long* v = G->vec[d] + (size_t)G->spd * DVEC;
    PLUSS_NCCL_CHECK(g_rccl.AllReduce(v, v, GV_W, ncclUint64, ncclSum, G->comm[d], G->xs[d]));
  }
  PLUSS_NCCL_CHECK(g_rccl.GroupEnd());
  PLUSS_STAGE(G->xs[0], "group: dense all-reduce");
  return fork_shards(G);
}

// one dense pass over the resident lists, everything on the exchange streams
// (capturable); a shard without a list sends a failed slot
static int dense_pass_on_xs(pluss_group* G, GErr& E) {
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    for (int j = 0; j < G->spd; ++j) {
      const size_t i = (size_t)d * G->spd + j;
      unsigned long long* slot = G->vec[d] + (size_t)j * DVEC;
      int rc = PLUSS_OK;
      if (!G->list[i]) {
        set_error("pluss_group_dense: no resident lists (pluss_group_expand first)");
        rc = PLUSS_ERR_CONFIG;
      } else {
        rc = pluss_dev_sampled_hist_dense(G->ctx[i], (const uint64_t*)G->list[i], G->list_n[i], (uint64_t*)slot,
                                          G->xs[d]);
      }
      if (rc) {
        E.note(rc);
        hipLaunchKernelGGL(k_group_word, dim3(1), dim3(1), 0, G->xs[d], slot + GV_COND + GC_LOCAL, 1ull);
      }
    }
    hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(64), 0, G->xs[d], (const unsigned long long*)G->vec[d], G->spd,
                       G->vec[d] + (size_t)G->spd * DVEC);
  }
  PLUSS_HIP_CHECK(hipGetLastError());
  if (G->nranks == 1) return PLUSS_OK;  // (one rank, one device: the all-reduce is the identity)
  PLUSS_NCCL_CHECK(g_rccl.GroupStart());
  for (int d = 0; d < G->ndev; ++d) {
    unsigned long long* v = G->vec[d] + (size_t)G->spd * DVEC;
    PLUSS_NCCL_CHECK(g_rccl.AllReduce(v, v, GV_W, ncclUint64, ncclSum, G->comm[d], G->xs[d]));
  }
  PLUSS_NCCL_CHECK(g_rccl.GroupEnd());
  return PLUSS_OK;
}

// Whether any rank of the job failed, the same answer on every rank: each
// device's failure word summed over the ranks (one 1-word all-reduce and a
// read-back).  A process that drives every rank itself (pluss_group_create)
// already knows: its GErr holds every device's error.  Used before a
// point-to-point exchange, where a rank that returned early would leave its
// peers waiting in ncclSend / ncclRecv.
static int agree_failed(pluss_group* G, bool mine, bool* any) {
  *any = mine;
  if (G->nranks == G->ndev) return PLUSS_OK;
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    hipLaunchKernelGGL(k_group_word, dim3(1), dim3(1), 0, G->xs[d], G->agr[d], mine ? 1ull : 0ull);
  }
  PLUSS_HIP_CHECK(hipGetLastError());
  PLUSS_NCCL_CHECK(g_rccl.GroupStart());
  for (int d = 0; d < G->ndev; ++d)
    PLUSS_NCCL_CHECK(g_rccl.AllReduce(G->agr[d], G->agr[d], 1, ncclUint64, ncclSum, G->comm[d], G->xs[d]));
  PLUSS_NCCL_CHECK(g_rccl.GroupEnd());
  unsigned long long v = 0;
  PLUSS_HIP_CHECK(hipSetDevice(G->dev[0]));
  PLUSS_HIP_CHECK(hipMemcpyAsync(&v, G->agr[0], 8, hipMemcpyDeviceToHost, G->xs[0]));
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    PLUSS_HIP_CHECK(hipStreamSynchronize(G->xs[d]));
  }
  *any = v != 0;
  return PLUSS_OK;
}

// the merged vector on the host once every exchange stream has drained; the
// first error: this rank's own, then a shard that failed anywhere, then the
// merged flags (each condition reported as one GPU's fetch reports it)
static int vec_fetch(pluss_group* G, const GErr& E, unsigned long long* v) {
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    PLUSS_HIP_CHECK(hipStreamSynchronize(G->xs[d]));
  }
  PLUSS_HIP_CHECK(hipSetDevice(G->dev[0]));
  PLUSS_HIP_CHECK(hipMemcpy(v, G->vec[0] + (size_t)G->spd * DVEC, GV_W * 8, hipMemcpyDeviceToHost));
  if (E.rc) {
    set_error(E.msg);
    return E.rc;
  }
  const unsigned long long* c = v + GV_COND;
  if (c[GC_LOCAL]) {
    set_error(std::to_string(c[GC_LOCAL]) + " shard(s) of this group pass failed on their host");
    return PLUSS_ERR_PEER;
  }
  const unsigned int f0 = (c[GC_OVERFLOW] ? FLAG_OVERFLOW : 0u) | (c[GC_LOOKBACK] ? FLAG_LOOKBACK : 0u) |
                          (c[GC_SHARD] ? FLAG_SHARD : 0u) | (c[GC_SORT] ? FLAG_SORT : 0u) | (c[GC_UNI] ? FLAG_UNI : 0u);
  return flags_error(f0, (v[GV_BAD] || c[GC_BAD]) ? 1u : 0u, "group pass: ");
}

// The end of a one-shot pass over a shape with N % (cls/ds) == 0: every
// shard's slot (k_group_vec), one all-reduce, the merged histogram built from
// the vector on the host.  A key outside the dense set (none expected) falls
// back to the tables, on every rank alike.
// the device half of the dense end of a pass: every shard's slot, the sum and the all-reduce
static int collect_enqueue(pluss_group* G, GErr& E) {
  for (int d = 0; d < G->ndev; ++d) {
    E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
    for (int j = 0; j < G->spd; ++j) {
      pluss_ctx* c = shard(G, d, j);
      hipLaunchKernelGGL(k_group_vec, dim3(1), dim3(256), 0, c->stream, G->m, c->g, G->vec[d] + (size_t)j * DVEC,
                         E.rc ? 1 : 0);
    }
    E.note(hip_rc(hipGetLastError(), "k_group_vec"));
  }
  PLUSS_STAGE(G->ctx[0]->stream, "collect: shard slots");
  return dense_merge(G);
}

// ... and the host half: the merged vector back, the histogram built from it
static int collect_finish(pluss_group* G, GErr& E, pluss_hist* out) {
  unsigned long long v[GV_W];
  const int rc = vec_fetch(G, E, v);
  if (rc) return rc;
  if (v[GV_COND + GC_NONDENSE]) return collect_tables(G, E, out);
  std::vector<uint64_t> keys, cnts;
  for (int b = 0; b < PLUSS_DENSE_BINS; ++b)
    if (v[b]) {
      keys.push_back(G->m.keytab[b]);
      cnts.push_back(v[b]);
    }
  for (int r = 0; r < 6; ++r)
    if (v[GV_PRES + r]) {  // the -1 key, materialised (r10:196,671), merged with a dense cold bin of the same key
      keys.push_back(make_key((uint32_t)r, 0, -1));
      cnts.push_back(v[GV_COLD + r]);
    }
  if (int rc2 = pluss_hist_from_tables(keys.data(), cnts.data(), keys.size(), out)) return rc2;
  for (int r = 0; r < 6; ++r) out->traversed[r] = v[GV_TRAV + r];
  return PLUSS_OK;
}

// The end of a one-shot pass over a shape with N % (cls/ds) == 0: every
// shard's slot (k_group_vec), one all-reduce, the merged histogram built from
// the vector on the host.  A key outside the dense set (none expected) falls
// back to the tables, on every rank alike.
static int collect(pluss_group* G, GErr& E, pluss_hist* out) {
  if (!G->m.fast) return collect_tables(G, E, out);
  if (int rc = collect_enqueue(G, E)) return rc;
  return collect_finish(G, E, out);
}

// any other pass on the shards' handles: the next gen_faithful starts eagerly
static void forget_faithful_graph(pluss_group* G) {
  if (G->fg) G->fg->seen = false;
}

// A faithful pass (source src: 0 generated, 1 uniform) run eagerly, captured
// or replayed (FaGraph).  body(E, captured) enqueues the pass from the table
// resets to its last phase; `extra`: whatever else a capture of this source
// needs from the eager pass before it is present.  The capture rule of
// pluss_group::capturing: one rank on one device only.
static int graph_pass(pluss_group* G, int src, uint64_t seed, const uint64_t totals[6], bool extra, pluss_hist* out,
                      const std::function<int(GErr&, bool)>& body) {
  if (!G->fg) G->fg = new FaGraph();
  FaGraph& F = *G->fg;
  const bool one = G->ndev == 1 && G->nranks == 1;
  const bool same =
      F.seen && F.src == src && F.seed == seed && std::memcmp(F.totals, totals, sizeof F.totals) == 0 && extra;
  if (one && same && F.have) {  // the captured pass, replayed
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[0]));
    PLUSS_HIP_CHECK(hipGraphLaunch(F.ex, G->xs[0]));
    GErr E;
    return collect_finish(G, E, out);
  }
  if (F.ex) G->retired.push_back(F.ex);  // (kept, not destroyed: pluss_group::retired)
  F.ex = nullptr;
  F.have = false;
  F.seen = true;
  F.src = src;
  F.seed = seed;
  std::memcpy(F.totals, totals, sizeof F.totals);
  // a second identical call is captured (the first ran eagerly and grew every
  // buffer); one-rank groups only, without their identity collectives
  const bool capture = one && same && G->m.fast && G->retired.size() < MAX_RETIRED;
  if (capture) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[0]));
    PLUSS_HIP_CHECK(hipStreamBeginCapture(G->xs[0], hipStreamCaptureModeThreadLocal));
    G->capturing = true;
    for (auto* c : G->ctx) c->fb.capture = true;
    if (int rc = fork_shards(G)) {  // (the shard streams join the capture)
      hipGraph_t gr = nullptr;
      (void)hipStreamEndCapture(G->xs[0], &gr);
      if (gr) (void)hipGraphDestroy(gr);
      G->capturing = false;
      for (auto* c : G->ctx) c->fb.capture = false;
      F.seen = false;
      return rc;
    }
  }
  GErr E;
  group_reset(G, E);
  int rc = body(E, capture);
  if (!capture) {
    if (rc || E.rc) F.seen = false;  // (a failed pass is not captured next)
    return rc ? rc : collect(G, E, out);
  }
  if (!rc) rc = collect_enqueue(G, E);
  if (!rc) rc = join_shards(G);  // (every forked stream rejoins before the capture ends)
  hipGraph_t gr = nullptr;
  const hipError_t ce = hipStreamEndCapture(G->xs[0], &gr);
  G->capturing = false;
  for (auto* c : G->ctx) c->fb.capture = false;
  if (!rc && !E.rc && ce == hipSuccess) {
    const hipError_t ie = hipGraphInstantiate(&F.ex, gr, nullptr, nullptr, 0);
    if (ie != hipSuccess) {
      F.ex = nullptr;
      set_error(std::string("faithful group pass: graph instantiate: ") + hipGetErrorString(ie));
      rc = PLUSS_ERR_HIP;
    }
  } else if (!rc && !E.rc) {
    set_error(std::string("faithful group pass: graph capture: ") + hipGetErrorString(ce));
    rc = PLUSS_ERR_HIP;
  }
  if (gr) (void)hipGraphDestroy(gr);
  F.seen = false;  // (a failed capture starts over; nothing of it ran)
  if (rc) return rc;
  if (E.rc) {
    set_error(E.msg);
    return E.rc;
  }
  F.seen = true;
  F.have = true;
  PLUSS_HIP_CHECK(hipGraphLaunch(F.ex, G->xs[0]));
  return collect_finish(G, E, out);
}

// a device buffer of at least `bytes` (the device's streams drained before it is replaced)
static int part_buf(pluss_group* G, int d, PartBufs::Buf& b, size_t bytes) {
  if (b.cap >= bytes && b.p) return PLUSS_OK;
  PLUSS_HIP_CHECK(hipStreamSynchronize(G->xs[d]));
  for (int j = 0; j < G->spd; ++j) PLUSS_HIP_CHECK(hipStreamSynchronize(shard(G, d, j)->stream));
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  if (hipMalloc(&b.p, bytes ? bytes : 8) != hipSuccess) {
    b.p = nullptr;
    set_error("pluss_group_sampled_hist: hipMalloc of " + std::to_string(bytes) + " bytes failed");
    return PLUSS_ERR_ALLOC;
  }
  b.cap = bytes ? bytes : 8;
  return PLUSS_OK;
}

// Faithful mode over an any-order host list (every rank passes the same list),
// shapes with N % (cls/ds) == 0, all of it on the devices:
//  1. device gd (of R) uploads only its slice [n*gd/R, n*(gd+1)/R), reads it
//     once to count its samples per bin (key-range shard g, reference r);
//  2. one all-gather of the bin totals (R x 6S words) and one host round trip
//     (the placements and the sorts' launch sizes need them);
//  3. the device reads its slice again and places each sample's packed word
//     in its bin's region (g-major: each destination's shards contiguous);
//  4. over several devices, one grouped RCCL send/receive per device pair
//     moves each destination's regions there, and a copy puts the received
//     words in (shard, reference) order; on one device the regions already are;
//  5. each shard sorts its words and runs the key-range phases (the rows
//     all-gathered between them), and the pass ends in the dense all-reduce.
// No sample goes through the host, no device holds more than its slice and
// its shards' words, and no shard reads another's samples.  A device that
// fails before the totals marks its block all ones: every rank sees it and
// fails the pass (PLUSS_ERR_PEER) after taking part in every collective.
static int group_any_order(pluss_group* G, const uint64_t* samples, uint64_t n, GErr& E, pluss_hist* out) {
  const int S = G->nshards, R = G->nranks, spd = G->spd;
  const uint32_t nb = 6u * (uint32_t)S;
  uint64_t key_end = 0;
  E.note(pluss_faithful_key_space(&G->cfg, &key_end));
  if (n >= ((uint64_t)1 << 40)) E.note(PLUSS_ERR_CONFIG, "pluss_group_sampled_hist: at most 2^40 samples");
  const int wb = faith_word_bytes(G->ctx[0]);
  std::vector<uint64_t> sl0(G->ndev), sln(G->ndev);
  std::vector<uint32_t> nblk(G->ndev);
  if (int rc = join_shards(G)) return rc;  // (the shards' table resets come first)
  PLUSS_STAGE(G->xs[0], "any-order: start (after the table resets)");
  for (int d = 0; d < G->ndev; ++d) {
    E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
    PartBufs& P = G->part[d];
    const int gd = G->rank0 + d;
    sl0[d] = (uint64_t)((unsigned __int128)n * gd / R);
    sln[d] = (uint64_t)((unsigned __int128)n * (gd + 1) / R) - sl0[d];
    nblk[d] = faith_part_blocks(sln[d], (uint32_t)S);
    int rc = E.rc;
    if (!rc) rc = part_buf(G, d, P.smp, sln[d] * 8);
    if (!rc) rc = part_buf(G, d, P.bounds, ((size_t)S + 1) * 8);
    if (!rc) rc = part_buf(G, d, P.hist, (size_t)nb * nblk[d] * 4);
    if (!rc) {
      P.h_bounds.resize((size_t)S + 1);
      for (int g = 0; g <= S; ++g) P.h_bounds[g] = (unsigned long long)((unsigned __int128)key_end * g / S);
      rc = hip_rc(hipMemcpyAsync(P.bounds.p, P.h_bounds.data(), P.h_bounds.size() * 8, hipMemcpyHostToDevice,
                                 G->xs[d]), "hipMemcpyAsync (bounds)");
    }
    // (P.tot is allocated with the group: every rank takes part in the gather below)
    unsigned long long* own = (unsigned long long*)P.tot.p + (size_t)gd * nb;
    if (!rc && sln[d])
      rc = hip_rc(hipMemcpyAsync(P.smp.p, samples + sl0[d], sln[d] * 8, hipMemcpyHostToDevice, G->xs[d]),
                  "hipMemcpyAsync (list slice)");
    // (uploading the slice in 8 pieces, each counted on a second stream as it
    // landed, saved at most 0.2 ms: 17-28 us between the pieces' copies, and
    // some calls stalled for several ms between pieces; r6ab/r6ac)
    if (!rc)
      rc = faith_part_count(shard(G, d, 0), (const uint64_t*)P.smp.p, sln[d], (const unsigned long long*)P.bounds.p,
                            (uint32_t)S, (uint32_t*)P.hist.p, nblk[d], own, G->xs[d]);
    if (rc) {
      E.note(rc);
      E.note(hip_rc(hipMemsetAsync(own, 0xFF, (size_t)nb * 8, G->xs[d]), "hipMemsetAsync"));
    }
  }
  PLUSS_STAGE(G->xs[0], "any-order: slice upload and partition count");
  std::vector<unsigned long long*> tots(G->ndev);
  for (int d = 0; d < G->ndev; ++d) tots[d] = (unsigned long long*)G->part[d].tot.p;
  if (int rc = gather_blocks(G, tots, (size_t)6 * R)) return rc;
  // the one host round trip: every device's bin totals
  std::vector<unsigned long long> T((size_t)R * nb);
  PLUSS_HIP_CHECK(hipSetDevice(G->dev[0]));
  PLUSS_HIP_CHECK(hipMemcpyAsync(T.data(), tots[0], T.size() * 8, hipMemcpyDeviceToHost, G->xs[0]));
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    PLUSS_HIP_CHECK(hipStreamSynchronize(G->xs[d]));
  }
  bool failed = false;
  for (int e = 0; e < R; ++e) failed |= T[(size_t)e * nb] == ~0ull;
  // per (shard, reference): its words over every device
  std::vector<uint64_t> bin_all(nb, 0);
  if (!failed)
    for (int e = 0; e < R; ++e)
      for (uint32_t x = 0; x < nb; ++x) bin_all[x] += T[(size_t)e * nb + x];
  for (uint32_t x = 0; x < nb && !failed; ++x)
    if (bin_all[x] > 0xFFFFFFFFull) {
      E.note(PLUSS_ERR_CONFIG, "faithful mode: at most 2^32-1 samples per reference and shard");
      failed = true;  // (the same on every rank)
    }
  if (failed) E.note(PLUSS_ERR_PEER, "a device's partition of the list failed");
  // each device's placement and, over several devices, the exchange
  std::vector<const unsigned char*> fin(G->ndev, nullptr);
  std::vector<std::vector<uint64_t>> foff(G->ndev);  // per local shard and reference: its words' start in fin
  for (int d = 0; d < G->ndev && !failed; ++d) {
    E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
    PartBufs& P = G->part[d];
    const int gd = G->rank0 + d;
    const unsigned long long* mine = T.data() + (size_t)gd * nb;
    P.h_rstart.assign(nb, 0);
    for (uint32_t x = 1; x < nb; ++x) P.h_rstart[x] = P.h_rstart[x - 1] + mine[x - 1];
    int rc = part_buf(G, d, P.rstart, (size_t)nb * 8);
    if (!rc) rc = part_buf(G, d, P.words, sln[d] * wb);
    if (!rc)
      rc = hip_rc(hipMemcpyAsync(P.rstart.p, P.h_rstart.data(), (size_t)nb * 8, hipMemcpyHostToDevice, G->xs[d]),
                  "hipMemcpyAsync (bin starts)");
    if (!rc)
      rc = faith_part_scatter(shard(G, d, 0), (const uint64_t*)P.smp.p, sln[d], (const unsigned long long*)P.bounds.p,
                              (uint32_t)S, (uint32_t*)P.hist.p, nblk[d], (const unsigned long long*)P.rstart.p,
                              P.words.p, G->xs[d]);
    E.note(rc);
    foff[d].assign((size_t)spd * 6, 0);
    if (R == 1) {  // the regions are already per (shard, reference)
      fin[d] = (const unsigned char*)P.words.p;
      for (int x = 0; x < spd * 6; ++x) foff[d][x] = P.h_rstart[x];
    }
  }
  if (R > 1 && !failed) {
    // what each device receives: from source e, e's words of this device's shards
    std::vector<uint64_t> rtot(G->ndev, 0);
    for (int d = 0; d < G->ndev; ++d) {
      const int gd = G->rank0 + d;
      for (int e = 0; e < R; ++e)
        for (int x = 0; x < spd * 6; ++x) rtot[d] += T[(size_t)e * nb + (size_t)gd * spd * 6 + x];
      PartBufs& P = G->part[d];
      E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
      E.note(part_buf(G, d, P.recv, rtot[d] * wb));
      E.note(part_buf(G, d, P.fin, rtot[d] * wb));
      E.note(part_buf(G, d, P.seg, (size_t)R * spd * 6 * 3 * 8));
    }
    // a failure since the totals' gather (a buffer, the placement) may be this
    // rank's alone: every rank learns of it before the send / receive, and all
    // of them skip the exchange together (the shards then fail their rows)
    bool any = false;
    if (int rc = agree_failed(G, E.rc != 0, &any)) return rc;
    if (any) {
      E.note(PLUSS_ERR_PEER, "a rank failed before the any-order exchange");
      failed = true;
    }
  }
  if (R > 1 && !failed) {
    PLUSS_NCCL_CHECK(g_rccl.GroupStart());
    for (int d = 0; d < G->ndev; ++d) {
      PartBufs& P = G->part[d];
      const int gd = G->rank0 + d;
      uint64_t roff = 0;
      for (int e = 0; e < R; ++e) {
        uint64_t sc = 0, rc = 0;
        for (int x = 0; x < spd * 6; ++x) {
          sc += T[(size_t)gd * nb + (size_t)e * spd * 6 + x];
          rc += T[(size_t)e * nb + (size_t)gd * spd * 6 + x];
        }
        const uint64_t soff = P.h_rstart[(size_t)e * spd * 6];
        if (sc)
          PLUSS_NCCL_CHECK(g_rccl.Send((const unsigned char*)P.words.p + soff * wb, sc * wb, ncclUint8, e, G->comm[d],
                                       G->xs[d]));
        if (rc)
          PLUSS_NCCL_CHECK(g_rccl.Recv((unsigned char*)P.recv.p + roff * wb, rc * wb, ncclUint8, e, G->comm[d],
                                       G->xs[d]));
        roff += rc;
      }
    }
    PLUSS_NCCL_CHECK(g_rccl.GroupEnd());
    // the received blocks [source][shard][reference] into [shard][reference][source]
    for (int d = 0; d < G->ndev; ++d) {
      PartBufs& P = G->part[d];
      const int gd = G->rank0 + d;
      E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
      uint64_t o = 0;
      for (int x = 0; x < spd * 6; ++x) {
        foff[d][x] = o;
        for (int e = 0; e < R; ++e) o += T[(size_t)e * nb + (size_t)gd * spd * 6 + x];
      }
      P.h_seg.clear();
      uint64_t roff = 0, maxn = 0;
      for (int e = 0; e < R; ++e) {
        uint64_t before_e = 0;
        for (int x = 0; x < spd * 6; ++x) {
          const uint64_t c = T[(size_t)e * nb + (size_t)gd * spd * 6 + x];
          uint64_t at = foff[d][x];
          for (int e2 = 0; e2 < e; ++e2) at += T[(size_t)e2 * nb + (size_t)gd * spd * 6 + x];
          if (c) {
            P.h_seg.push_back(roff + before_e);
            P.h_seg.push_back(at);
            P.h_seg.push_back(c);
            maxn = std::max(maxn, c);
          }
          before_e += c;
        }
        roff += before_e;
      }
      const uint32_t nseg = (uint32_t)(P.h_seg.size() / 3);
      // (a failure here stays local: fin[d] is left null, this device's shards
      // fail their rows and every rank still takes part in the phases' gathers)
      int rc = PLUSS_OK;
      if (nseg)
        rc = hip_rc(hipMemcpyAsync(P.seg.p, P.h_seg.data(), P.h_seg.size() * 8, hipMemcpyHostToDevice, G->xs[d]),
                    "hipMemcpyAsync (segments)");
      if (!rc) rc = faith_seg_copy((const unsigned long long*)P.seg.p, nseg, maxn, P.recv.p, P.fin.p, wb, G->xs[d]);
      E.note(rc);
      if (!rc) fin[d] = (const unsigned char*)P.fin.p;
    }
  }
  PLUSS_STAGE(G->xs[0], "any-order: placement and exchange");
  if (int rc = fork_shards(G)) return rc;  // (every shard's sort after its device's words)
  ShardFn loc = [&](pluss_ctx* c, int d, int j, int g, uint64_t* row) -> int {
    if (failed || !fin[d]) {
      set_error("a device's partition of the list failed");
      return PLUSS_ERR_PEER;
    }
    const void* in[6];
    uint64_t cnt[6], all[6], before[6];
    for (int r = 0; r < 6; ++r) {
      cnt[r] = bin_all[(size_t)g * 6 + r];
      all[r] = before[r] = 0;
      for (int g2 = 0; g2 < S; ++g2) {
        all[r] += bin_all[(size_t)g2 * 6 + r];
        if (g2 < g) before[r] += bin_all[(size_t)g2 * 6 + r];
      }
      in[r] = fin[d] + foff[d][(size_t)j * 6 + r] * wb;
    }
    return faith_shards_local_words(c, in, cnt, all, before, row, c->stream);
  };
  if (int rc = group_faithful(G, loc, nullptr, nullptr, E)) return rc;
  return collect(G, E, out);
}

}  // namespace pluss

extern "C" {

int pluss_group_unique_id(uint8_t id[PLUSS_GROUP_ID_BYTES]) {
  if (!id) return PLUSS_ERR_CONFIG;
  Rccl* R = rccl();
  if (!R) {
    set_error(g_rccl.why);
    return PLUSS_ERR_HIP;
  }
  ncclUniqueId u;
  PLUSS_NCCL_CHECK(R->GetUniqueId(&u));
  std::memcpy(id, u.internal, PLUSS_GROUP_ID_BYTES);
  return PLUSS_OK;
}

int pluss_group_create(const pluss_cfg* cfg, const int32_t* devices, int32_t ndev, int32_t shards_per_device,
                       pluss_group** out) {
  if (!out) return PLUSS_ERR_CONFIG;
  *out = nullptr;
  Model m;
  if (int rc = group_check_cfg(cfg, shards_per_device, &m)) return rc;
  int nd = 0;
  PLUSS_HIP_CHECK(hipGetDeviceCount(&nd));
  if (!devices || ndev < 1 || ndev > nd) {
    set_error("pluss_group_create: need 1 <= ndev <= " + std::to_string(nd) + " device ordinals");
    return PLUSS_ERR_CONFIG;
  }
  for (int i = 0; i < ndev; ++i)
    for (int k = 0; k < i; ++k)
      if (devices[i] < 0 || devices[i] >= nd || devices[i] == devices[k]) {
        set_error("pluss_group_create: device ordinals must be distinct and in range (several shards of one "
                  "device: shards_per_device)");
        return PLUSS_ERR_CONFIG;
      }
  if (devices[0] < 0 || devices[0] >= nd) {
    set_error("pluss_group_create: device ordinal out of range");
    return PLUSS_ERR_CONFIG;
  }
  Rccl* R = rccl();
  if (!R) {
    set_error(g_rccl.why);
    return PLUSS_ERR_HIP;
  }
  pluss_group* G = new pluss_group();
  G->cfg = *cfg;
  G->m = m;
  G->ndev = ndev;
  G->spd = shards_per_device;
  G->nranks = ndev;
  G->rank0 = 0;
  G->nshards = ndev * shards_per_device;
  G->dev.assign(devices, devices + ndev);
  G->comm.assign(ndev, nullptr);
  if (int rc = group_setup(G)) {
    const std::string e = pluss_last_error();
    group_free(G);
    set_error(e);
    return rc;
  }
  ncclResult_t r = R->CommInitAll(G->comm.data(), ndev, G->dev.data());
  if (r != ncclSuccess) {
    const std::string e = std::string("ncclCommInitAll: ") + R->GetErrorString(r);
    G->comm.assign(ndev, nullptr);
    group_free(G);
    set_error(e);
    return PLUSS_ERR_HIP;
  }
  *out = G;
  return PLUSS_OK;
}

int pluss_group_create_rank(const pluss_cfg* cfg, int32_t nranks, int32_t rank, const uint8_t id[PLUSS_GROUP_ID_BYTES],
                            int32_t shards_per_device, pluss_group** out) {
  if (!out || !id) return PLUSS_ERR_CONFIG;
  *out = nullptr;
  Model m;
  if (int rc = group_check_cfg(cfg, shards_per_device, &m)) return rc;
  if (nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("pluss_group_create_rank: need 0 <= rank < nranks");
    return PLUSS_ERR_CONFIG;
  }
  int nd = 0;
  PLUSS_HIP_CHECK(hipGetDeviceCount(&nd));
  if (cfg->device < 0 || cfg->device >= nd) {
    set_error("pluss_group_create_rank: cfg.device out of range");
    return PLUSS_ERR_CONFIG;
  }
  Rccl* R = rccl();
  if (!R) {
    set_error(g_rccl.why);
    return PLUSS_ERR_HIP;
  }
  pluss_group* G = new pluss_group();
  G->cfg = *cfg;
  G->m = m;
  G->ndev = 1;
  G->spd = shards_per_device;
  G->nranks = nranks;
  G->rank0 = rank;
  G->nshards = nranks * shards_per_device;
  G->dev.assign(1, cfg->device);
  G->comm.assign(1, nullptr);
  if (int rc = group_setup(G)) {
    const std::string e = pluss_last_error();
    group_free(G);
    set_error(e);
    return rc;
  }
  ncclUniqueId u;
  std::memcpy(u.internal, id, PLUSS_GROUP_ID_BYTES);
  (void)hipSetDevice(cfg->device);
  ncclResult_t r = R->CommInitRank(&G->comm[0], nranks, u, rank);
  if (r != ncclSuccess) {
    const std::string e = std::string("ncclCommInitRank: ") + R->GetErrorString(r);
    G->comm[0] = nullptr;
    group_free(G);
    set_error(e);
    return PLUSS_ERR_HIP;
  }
  *out = G;
  return PLUSS_OK;
}

int pluss_group_destroy(pluss_group* G) {
  if (G) group_free(G);
  return PLUSS_OK;
}

int pluss_group_shards(const pluss_group* G, int32_t* local, int32_t* total) {
  if (!G) return PLUSS_ERR_CONFIG;
  if (local) *local = G->ndev * G->spd;
  if (total) *total = G->nshards;
  return PLUSS_OK;
}

// the captured dense passes point at the resident lists and their sizes:
// dropped whenever the lists change (a replay would read freed lists)
static int drop_graphs(pluss_group* G) {
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    PLUSS_HIP_CHECK(hipStreamSynchronize(G->xs[d]));
  }
  for (auto& kv : G->graphs) G->retired.push_back(kv.second);  // (kept: pluss_group::retired)
  G->graphs.clear();
  return PLUSS_OK;
}

int pluss_group_expand(pluss_group* G, uint64_t seed, const uint64_t counts[6]) {
  if (!G || !counts) return PLUSS_ERR_CONFIG;
  forget_faithful_graph(G);
  if (int rc = drop_graphs(G)) return rc;
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    for (int j = 0; j < G->spd; ++j) {
      const size_t i = (size_t)d * G->spd + j;
      const int g = gshard(G, d, j);
      uint64_t f[6], n[6], tot = 0;
      for (int r = 0; r < 6; ++r) {
        shard_ranges(counts[r], g, G->nshards, &f[r], &n[r]);
        tot += n[r];
      }
      PLUSS_HIP_CHECK(hipStreamSynchronize(G->ctx[i]->stream));
      if (G->list[i]) (void)hipFree(G->list[i]);
      G->list[i] = nullptr;
      G->list_n[i] = 0;
      PLUSS_HIP_CHECK(hipMalloc((void**)&G->list[i], (tot ? tot : 1) * 8));
      uint64_t off = 0;
      for (int r = 0; r < 6; ++r) {
        if (int rc = pluss_dev_expand(G->ctx[i], seed, r, f[r], n[r], (uint64_t*)G->list[i] + off, G->ctx[i]->stream))
          return rc;
        off += n[r];
      }
      G->list_n[i] = tot;
    }
  }
  for (int d = 0; d < G->ndev; ++d)
    for (int j = 0; j < G->spd; ++j) PLUSS_HIP_CHECK(hipStreamSynchronize(shard(G, d, j)->stream));
  return PLUSS_OK;
}

int pluss_group_dense(pluss_group* G, uint32_t passes, uint64_t counts[PLUSS_DENSE_BINS + 1]) {
  if (!G) return PLUSS_ERR_CONFIG;
  forget_faithful_graph(G);
  if (!G->m.fast) {
    set_error("pluss_group_dense: needs N % (cls/ds) == 0");
    return PLUSS_ERR_CONFIG;
  }
  GErr E;
  bool lists = true;
  for (size_t i = 0; i < G->ctx.size(); ++i) lists &= G->list[i] != nullptr;
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    PLUSS_HIP_CHECK(hipMemsetAsync(G->vec[d], 0, (size_t)(G->spd + 1) * DVEC * 8, G->xs[d]));
  }
  if (passes == 0) {  // nothing to run: the zero vector
    if (counts)
      for (int b = 0; b <= PLUSS_DENSE_BINS; ++b) counts[b] = 0;
    return PLUSS_OK;
  }
  constexpr uint32_t BATCH = 16;  // passes per captured graph
  uint32_t left = passes;
  if (G->ndev == 1 && G->nranks == 1 && lists && left >= BATCH &&
      (G->graphs.count(BATCH) || G->retired.size() < MAX_RETIRED)) {
    // one rank, one local device: BATCH passes replayed from one HIP graph
    // (kernels and the shard sums; the all-reduce, the identity, left out)
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[0]));
    hipGraphExec_t ex = nullptr;
    auto it = G->graphs.find(BATCH);
    if (it != G->graphs.end()) {
      ex = it->second;
    } else {
      PLUSS_HIP_CHECK(hipStreamBeginCapture(G->xs[0], hipStreamCaptureModeThreadLocal));
      G->capturing = true;
      int rc = PLUSS_OK;
      for (uint32_t k = 0; k < BATCH && !rc; ++k) rc = dense_pass_on_xs(G, E);
      hipGraph_t gr = nullptr;
      const hipError_t e = hipStreamEndCapture(G->xs[0], &gr);
      G->capturing = false;
      if (rc || E.rc) {
        if (gr) (void)hipGraphDestroy(gr);
        return rc ? rc : E.rc;  // (host-side failures while capturing: nothing was launched)
      }
      if (e != hipSuccess) {
        set_error(std::string("pluss_group_dense: graph capture: ") + hipGetErrorString(e));
        return PLUSS_ERR_HIP;
      }
      const hipError_t e2 = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
      (void)hipGraphDestroy(gr);
      if (e2 != hipSuccess) {
        set_error(std::string("pluss_group_dense: graph instantiate: ") + hipGetErrorString(e2));
        return PLUSS_ERR_HIP;
      }
      G->graphs[BATCH] = ex;
    }
    for (; left >= BATCH; left -= BATCH) PLUSS_HIP_CHECK(hipGraphLaunch(ex, G->xs[0]));
  }
  for (; left; --left)
    if (int rc = dense_pass_on_xs(G, E)) return rc;
  unsigned long long v[GV_W];
  const int rc = vec_fetch(G, E, v);
  if (counts)
    for (int b = 0; b <= PLUSS_DENSE_BINS; ++b) counts[b] = v[b];  // (malformed samples: the count, and an error)
  return rc;
}

int pluss_group_gen_count_dense(pluss_group* G, uint64_t seed, const uint64_t totals[6],
                                uint64_t counts[PLUSS_DENSE_BINS + 1]) {
  if (!G || !totals) return PLUSS_ERR_CONFIG;
  forget_faithful_graph(G);
  GErr E;
  for (int d = 0; d < G->ndev; ++d) {
    PLUSS_HIP_CHECK(hipSetDevice(G->dev[d]));
    PLUSS_HIP_CHECK(hipMemsetAsync(G->vec[d], 0, (size_t)(G->spd + 1) * DVEC * 8, G->xs[d]));
  }
  if (int rc = fork_shards(G)) return rc;  // (the slots are cleared before the shards write them)
  for (int d = 0; d < G->ndev; ++d) {
    E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
    for (int j = 0; j < G->spd; ++j) {
      const int g = gshard(G, d, j);
      uint64_t f[6], n[6];
      for (int r = 0; r < 6; ++r) shard_ranges(totals[r], g, G->nshards, &f[r], &n[r]);
      pluss_ctx* c = shard(G, d, j);
      unsigned long long* slot = G->vec[d] + (size_t)j * DVEC;
      if (const int rc = pluss_dev_gen_count_dense(c, seed, totals, f, n, (uint64_t*)slot, c->stream)) {
        E.note(rc);
        hipLaunchKernelGGL(k_group_word, dim3(1), dim3(1), 0, c->stream, slot + GV_COND + GC_LOCAL, 1ull);
      }
    }
  }
  if (int rc = dense_merge(G)) return rc;
  unsigned long long v[GV_W];
  const int rc = vec_fetch(G, E, v);
  if (counts)
    for (int b = 0; b <= PLUSS_DENSE_BINS; ++b) counts[b] = v[b];
  return rc;
}

int pluss_group_sampled_hist(pluss_group* G, const uint64_t* samples, uint64_t n, pluss_hist* out) {
  if (!G || !out || (n && !samples)) return PLUSS_ERR_CONFIG;
  forget_faithful_graph(G);
  GErr E;
  group_reset(G, E);
  const int S = G->nshards;
  if (G->cfg.mode == PLUSS_MODE_CLEAN) {
    // shard g: the slice [n*g/S, n*(g+1)/S) of the list, any shape
    for (int d = 0; d < G->ndev; ++d) {
      E.note(hip_rc(hipSetDevice(G->dev[d]), "hipSetDevice"));
      for (int j = 0; j < G->spd; ++j) {
        const size_t i = (size_t)d * G->spd + j;
        uint64_t f, m;
        shard_ranges(n, gshard(G, d, j), S, &f, &m);
        if (G->hl_cap[i] < m || !G->hl[i]) {
          E.note(hip_rc(hipStreamSynchronize(G->ctx[i]->stream), "hipStreamSynchronize"));
          if (G->hl[i]) (void)hipFree(G->hl[i]);
          G->hl[i] = nullptr;
          G->hl_cap[i] = 0;
          if (const int rc = hip_rc(hipMalloc((void**)&G->hl[i], (m ? m : 1) * 8), "hipMalloc (group slice)")) {
            G->hl[i] = nullptr;
            E.note(rc);
            continue;  // (this shard sends a failed slot)
          }
          G->hl_cap[i] = m ? m : 1;
        }
        int rc = hip_rc(hipMemcpyAsync(G->hl[i], samples + f, m * 8, hipMemcpyHostToDevice, G->ctx[i]->stream),
                        "hipMemcpyAsync (group slice)");
        if (!rc) rc = pluss_dev_sampled_hist(G->ctx[i], (const uint64_t*)G->hl[i], m, G->ctx[i]->stream);
        E.note(rc);
      }
    }
    return collect(G, E, out);
  }
  if ((uint64_t)G->cfg.n % ((uint64_t)G->cfg.chunk * (uint64_t)G->cfg.threads) != 0) {
    set_error("faithful mode needs N % (chunk*threads) == 0 (lockstep interleaving order)");
    return PLUSS_ERR_CONFIG;  // (the same on every rank)
  }
  if (G->m.fast) return group_any_order(G, samples, n, E, out);
  // faithful, (key, sink) pairs (N % (cls/ds) != 0; not key-range sharded):
  // the job's first shard runs r10's six samplers, each over its reference's
  // samples in list order
  std::vector<uint64_t> per[6];
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t r = (uint32_t)(samples[i] >> 60);
    if (r > 5) {
      E.note(PLUSS_ERR_INPUT, "malformed sample: ref > 5");
      break;
    }
    per[r].push_back(samples[i]);
  }
  if (G->rank0 == 0 && !E.rc) {
    (void)hipSetDevice(G->dev[0]);
    pluss_ctx* c = G->ctx[0];
    for (int r = 0; r < 6 && !E.rc; ++r) {
      if (per[r].empty()) continue;
      uint64_t* dl = nullptr;
      int rc = hip_rc(hipMalloc((void**)&dl, per[r].size() * 8), "hipMalloc (group list)");
      if (!rc) rc = hip_rc(hipMemcpy(dl, per[r].data(), per[r].size() * 8, hipMemcpyHostToDevice), "hipMemcpy");
      if (!rc) rc = pluss_dev_faithful_hist(c, r, dl, per[r].size(), c->stream);
      if (!rc) rc = hip_rc(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
      if (dl) (void)hipFree(dl);
      E.note(rc);
    }
  }
  return collect_tables(G, E, out);
}

int pluss_group_gen_faithful(pluss_group* G, uint64_t seed, const uint64_t totals[6], pluss_hist* out) {
  if (!G || !totals || !out) return PLUSS_ERR_CONFIG;
  uint64_t key_end = 0;
  if (int rc = pluss_faithful_key_space(&G->cfg, &key_end)) return rc;  // (the same on every rank)
  const int S = G->nshards;
  return graph_pass(G, 0, seed, totals, true, out, [&](GErr& E, bool) {
    ShardFn gen = [&](pluss_ctx* c, int, int, int g, uint64_t* row) -> int {
      const uint64_t lo = (uint64_t)((unsigned __int128)key_end * g / S);
      const uint64_t hi = (uint64_t)((unsigned __int128)key_end * (g + 1) / S);
      uint64_t f[6] = {0, 0, 0, 0, 0, 0}, m[6] = {0, 0, 0, 0, 0, 0};
      for (int r = 0; r < 6; ++r) {
        if (!totals[r]) continue;
        uint64_t a = 0, b = 0;
        if (int rc = pluss_keyorder_index_range(&G->cfg, seed, r, totals[r], lo, hi, &a, &b)) return rc;
        f[r] = a;
        m[r] = b - a;
      }
      return pluss_dev_faithful_shards_local(c, nullptr, seed, totals, f, m, row, c->stream);
    };
    return group_faithful(G, gen, nullptr, nullptr, E);
  });
}

int pluss_group_gen_uniform_faithful(pluss_group* G, uint64_t seed, const uint64_t totals[6], pluss_hist* out) {
  if (!G || !totals || !out) return PLUSS_ERR_CONFIG;
  uint64_t key_end = 0;
  if (int rc = pluss_faithful_key_space(&G->cfg, &key_end)) return rc;  // (the same on every rank)
  const int S = G->nshards, local = G->ndev * G->spd;
  if (!G->fg) G->fg = new FaGraph();
  FaGraph& F = *G->fg;
  // a captured pass takes each shard's slice from the eager pass before it:
  // the one mid-pass read-back (the slice sizes the local pass's grids) is
  // what kept this pass from being captured
  const bool slices = F.slice.size() == (size_t)local * 12;
  return graph_pass(G, 1, seed, totals, slices, out, [&](GErr& E, bool captured) {
    // phase 0: each shard's candidates; then every shard's window (enqueued on
    // all shards before any waits for its slice), then each local pass
    ShardFn count = [&](pluss_ctx* c, int, int, int g, uint64_t* row) {
      return faith_shards_uniform_count(c, seed, totals, g, S, row, c->stream);
    };
    ShardFn window = [&](pluss_ctx* c, int d, int, int g, uint64_t*) {
      return faith_shards_uniform_window(c, (const uint64_t*)G->rows[d], g, S, c->stream, !captured);
    };
    ShardFn finish = [&](pluss_ctx* c, int d, int j, int, uint64_t* row) {
      return faith_shards_uniform_finish(c, row, c->stream,
                                         captured ? F.slice.data() + ((size_t)d * G->spd + j) * 12 : nullptr);
    };
    const int rc = group_faithful(G, count, window, finish, E);
    if (!captured && !rc) {  // (the eager pass waited for every slice: kept for the capture)
      F.slice.assign((size_t)local * 12, 0);
      for (int d = 0; d < G->ndev; ++d)
        for (int j = 0; j < G->spd; ++j) {
          const uint64_t* h = (const uint64_t*)shard(G, d, j)->ub.hinfo;
          if (h) std::memcpy(F.slice.data() + ((size_t)d * G->spd + j) * 12, h + 6, 12 * 8);
        }
    }
    return rc;
  });
}

}  // extern "C"
