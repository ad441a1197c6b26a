"""Python front end of the MI355X PLUSS sampler (thin layer over the C ABI).

Mirrors the reference's sampler entry points:

  sampled_hist(cfg, samples)  ~ r10 sampler_<REF>(histogram) raw histograms
                                (c_lib/test/sampler/gemm-t4-pluss-pro-model-rs-ri-opt-r10.cpp:135..3190)
  fulltrace_hist(cfg)         ~ seq sampler() / rayon sampler(pool)
                                (…-ri-omp-seq.cpp:37, src/gemm_sampler_rayon.rs:71)
  expand_samples(...)         ~ the rand()%(N-1) sample generation (r10:156-185)

Every computation runs in libpluss_gpu.so on a HIP device.
"""
import ctypes
from collections import defaultdict
from dataclasses import dataclass

import numpy as np

from ._lib import DENSE_BINS, GROUP_ID_BYTES, PlussCfg, PlussHist, PlussHistEntry, check, lib

REFS = ["C0", "C1", "A0", "B0", "C2", "C3"]
REF_ID = {r: i for i, r in enumerate(REFS)}
REF_ARRAY = {"C0": "C", "C1": "C", "A0": "A", "B0": "B", "C2": "C", "C3": "C"}
DIM = {"C0": 2, "C1": 2, "A0": 3, "B0": 3, "C2": 3, "C3": 3}
NOSHARE, SHARE = 0, 1
KEY_EMPTY = (1 << 64) - 1


@dataclass
class SamplerConfig:
    """Everything the reference fixes at compile time (Makefile:14-15, N=128 literals)."""
    n: int = 128           # GEMM loop bound N
    threads: int = 4       # THREAD_NUM
    chunk: int = 4         # CHUNK_SIZE
    ds: int = 8            # DS
    cls: int = 64          # CLS
    mode: str = "clean"    # "clean" (every sample) | "faithful" (r10 queue semantics)
    thr_variant: str = "r10"  # "r10": (4N+2)N (r10:2482) | "v1": (N+1)N+1 (seq.cpp:203)
    range_full: bool = False  # sample indices in [0,N-1] instead of rand()%(N-1)'s [0,N-2]
    device: int = 0

    def to_c(self):
        return PlussCfg(self.n, self.threads, self.chunk, self.ds, self.cls,
                        {"clean": 0, "faithful": 1}[self.mode], {"r10": 0, "v1": 1}[self.thr_variant],
                        1 if self.range_full else 0, self.device)


class Histogram:
    """Exact raw reuse-interval bins: {(ref, kind, ri): count}; ri = -1 is cold."""

    def __init__(self, bins=None, traversed=None):
        self.bins = dict(bins or {})
        self.traversed = list(traversed or [0] * 6)

    @classmethod
    def _from_c(cls, h):
        bins = {}
        for i in range(h.n_entries):
            e = h.entries[i]
            bins[(REFS[e.ref], int(e.kind), int(e.ri))] = int(e.count)
        return cls(bins, [int(x) for x in h.traversed])

    def _select(self, kind, ref):
        out = defaultdict(int)
        for (r, k, ri), c in self.bins.items():
            if k == kind and (ref is None or r == ref):
                out[ri] += c
        return dict(out)

    def noshare(self, ref=None):
        """{ri: count} of the noshare histogram (cold at key -1), like no_share_histogram (r10:146)."""
        return self._select(NOSHARE, ref)

    def share(self, ref=None):
        """{ri: count} of the share histogram (share_ratio THREAD_NUM-1, r10:2483)."""
        return self._select(SHARE, ref)

    def cold(self, ref=None):
        return self.noshare(ref).get(-1, 0)

    def total(self):
        return sum(self.bins.values())

    def __eq__(self, other):
        a = {k: v for k, v in self.bins.items() if v}
        b = {k: v for k, v in other.bins.items() if v}
        return a == b

    def __repr__(self):
        return f"Histogram({len(self.bins)} bins, total={self.total()})"


def _hist_buf(cap=1 << 14):
    entries = (PlussHistEntry * cap)()
    h = PlussHist()
    h.entries = entries
    h.capacity = cap
    return h, entries


def _u64(a):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return a, a.ctypes.data_as(ctypes.c_void_p)


def pack(ref, c0, c1, c2=0):
    """Packed sample ref(4)|c0(20)|c1(20)|c2(20)."""
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    return (rid << 60) | (int(c0) << 40) | (int(c1) << 20) | int(c2)


def pack_array(ref, idx):
    rid = np.uint64(REF_ID[ref] if isinstance(ref, str) else int(ref))
    idx = np.asarray(idx, dtype=np.uint64)
    c2 = idx[:, 2] if idx.shape[1] > 2 else np.zeros(len(idx), np.uint64)
    return (rid << np.uint64(60)) | (idx[:, 0] << np.uint64(40)) | (idx[:, 1] << np.uint64(20)) | c2


def unpack_array(s):
    s = np.asarray(s, dtype=np.uint64)
    m = np.uint64(0xFFFFF)
    return ((s >> np.uint64(60)).astype(np.int64), ((s >> np.uint64(40)) & m).astype(np.int64),
            ((s >> np.uint64(20)) & m).astype(np.int64), (s & m).astype(np.int64))


def sampled_hist(cfg, samples):
    """Histogram of a host sample list (clean: all samples; faithful: per-ref r10 semantics)."""
    s, p = _u64(samples)
    h, keep = _hist_buf()
    c = cfg.to_c()
    check(lib().pluss_gemm_sampled_hist(ctypes.byref(c), p, len(s), ctypes.byref(h)), "pluss_gemm_sampled_hist")
    return Histogram._from_c(h)


def fulltrace_hist(cfg):
    h, keep = _hist_buf()
    c = cfg.to_c()
    check(lib().pluss_gemm_fulltrace_hist(ctypes.byref(c), ctypes.byref(h)), "pluss_gemm_fulltrace_hist")
    return Histogram._from_c(h)


def sampled_ri(cfg, samples):
    """Per-sample (ri, sink_key) on the device; ri = -1 cold, sink = 2^64-1 for cold."""
    s, p = _u64(samples)
    ri = np.empty(len(s), dtype=np.int64)
    sink = np.empty(len(s), dtype=np.uint64)
    c = cfg.to_c()
    check(lib().pluss_gemm_sampled_ri(ctypes.byref(c), p, len(s), ri.ctypes.data_as(ctypes.c_void_p),
                                      sink.ctypes.data_as(ctypes.c_void_p)), "pluss_gemm_sampled_ri")
    return ri, sink


def expand_samples(cfg, seed, ref, first, n):
    out = np.empty(n, dtype=np.uint64)
    c = cfg.to_c()
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    check(lib().pluss_expand_samples(ctypes.byref(c), seed, rid, first, n, out.ctypes.data_as(ctypes.c_void_p)),
          "pluss_expand_samples")
    return out


def expand_sorted(cfg, seed, ref, total, first, n):
    """Samples [first, first+n) of reference `ref`'s key-order stratified list of
    `total` samples (generated in r10's pop order: no sort needed in faithful mode)."""
    out = np.empty(n, dtype=np.uint64)
    c = cfg.to_c()
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    check(lib().pluss_expand_sorted(ctypes.byref(c), seed, rid, total, first, n, out.ctypes.data_as(ctypes.c_void_p)),
          "pluss_expand_sorted")
    return out


def expand_uniform_sorted(cfg, seed, ref, total, first, n):
    """Samples [first, first+n) of reference `ref`'s list of `total` samples
    drawn uniformly without replacement (r10's rand() draw with duplicate
    rejection, r10:156-185), generated directly in r10's pop order."""
    out = np.empty(n, dtype=np.uint64)
    c = cfg.to_c()
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    check(lib().pluss_expand_uniform_sorted(ctypes.byref(c), seed, rid, total, first, n,
                                            out.ctypes.data_as(ctypes.c_void_p)), "pluss_expand_uniform_sorted")
    return out


def default_counts(n, total):
    counts = (ctypes.c_uint64 * 6)()
    check(lib().pluss_default_counts(n, total, counts), "pluss_default_counts")
    return [int(x) for x in counts]


def faithful_key_space(cfg):
    """Faithful-mode sort keys a*T+tid of this shape lie in [0, key_space)."""
    out = ctypes.c_uint64()
    check(lib().pluss_faithful_key_space(ctypes.byref(cfg.to_c()), ctypes.byref(out)), "pluss_faithful_key_space")
    return int(out.value)


def faithful_key(cfg, sample):
    """The faithful-mode sort key a*T + tid of one packed sample (r10's pop
    order, IterationComp, pluss_utils.h:175-267): a = q*R + c1*S + off is the
    sample's thread-local position (S = 4N+2, R = N*S, q its thread-local row,
    off C0:0 C1:1 A0:2+4c2 B0:3+4c2 C2:4+4c2 C3:5+4c2).  Needs N % (CS*T) == 0
    (the lockstep interleaving order faithful mode requires)."""
    x = int(sample)
    ref, c0, c1, c2 = x >> 60, (x >> 40) & 0xFFFFF, (x >> 20) & 0xFFFFF, x & 0xFFFFF
    N, T, CS = cfg.n, cfg.threads, cfg.chunk
    S = 4 * N + 2
    k = c0 // CS
    tid, q = k % T, (k // T) * CS + c0 % CS
    off = ref if ref < 2 else ref + 4 * c2
    return ((q * N + c1) * S + off) * T + tid


def keyorder_index_range(cfg, seed, ref, total, key_lo, key_hi, sample_at=None):
    """[i_lo, i_hi): the samples of the key-order list (expand_sorted, keys
    strictly increasing in the index) whose faithful keys lie in
    [key_lo, key_hi) -- two binary searches of the host generator
    (pluss_keyorder_index_range; no device).  sample_at(i) -> packed sample i
    replaces the generator (tests)."""
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    if sample_at is None:
        lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().pluss_keyorder_index_range(ctypes.byref(cfg.to_c()), seed, rid, total, key_lo, key_hi,
                                               ctypes.byref(lo), ctypes.byref(hi)), "pluss_keyorder_index_range")
        return int(lo.value), int(hi.value)

    def first_at_least(key):
        lo, hi = 0, total
        while lo < hi:
            mid = (lo + hi) // 2
            if faithful_key(cfg, sample_at(mid)) >= key:
                hi = mid
            else:
                lo = mid + 1
        return lo
    return first_at_least(key_lo), first_at_least(key_hi)


def dense_keys(cfg):
    """Keys of the PLUSS_DENSE_BINS dense bins (bin = ref*3 + case) of a shape with N % (cls/ds) == 0."""
    out = (ctypes.c_uint64 * DENSE_BINS)()
    check(lib().pluss_dense_keys(ctypes.byref(cfg.to_c()), out), "pluss_dense_keys")
    return [int(x) for x in out]


def hist_from_dense(cfg, counts):
    """Histogram of a dense count vector (DENSE_BINS counts, optionally followed by the malformed count).
    Bins with a zero count are not histogram keys (unlike faithful mode's cold
    bin, which r10 creates with += 0 at r10:196 and pluss_hist_from_tables keeps)."""
    c = np.asarray(counts).reshape(-1)[:DENSE_BINS].astype(np.int64).view(np.uint64)
    k = np.array(dense_keys(cfg), dtype=np.uint64)
    return hist_from_tables(k[c != 0], c[c != 0])


def hist_from_tables(keys, counts):
    k, kp = _u64(keys)
    c, cp = _u64(counts)
    h, keep = _hist_buf()
    check(lib().pluss_hist_from_tables(kp, cp, len(k), ctypes.byref(h)), "pluss_hist_from_tables")
    return Histogram._from_c(h)


class Context:
    """Handle API: device-resident samples, explicit HIP streams (raw pointers)."""

    def __init__(self, cfg):
        self.cfg = cfg
        self._c = cfg.to_c()
        self._h = ctypes.c_void_p()
        check(lib().pluss_ctx_create(ctypes.byref(self._c), ctypes.byref(self._h)), "pluss_ctx_create")

    @property
    def stream(self):
        return lib().pluss_ctx_stream(self._h)

    def _s(self, stream):
        """stream=None: the handle's own stream (the C ABI takes NULL as HIP's
        null stream, include/pluss_gpu.h)."""
        return self.stream if stream is None else stream

    def close(self):
        if self._h:
            lib().pluss_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, stream=None):
        check(lib().pluss_dev_hist_reset(self._h, self._s(stream)), "pluss_dev_hist_reset")

    def expand(self, seed, ref, first, n, d_out, stream=None):
        rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
        check(lib().pluss_dev_expand(self._h, seed, rid, first, n, d_out, self._s(stream)), "pluss_dev_expand")

    def expand_sorted(self, seed, ref, total, first, n, d_out, stream=None):
        rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
        check(lib().pluss_dev_expand_sorted(self._h, seed, rid, total, first, n, d_out, self._s(stream)),
              "pluss_dev_expand_sorted")

    def expand_uniform_sorted(self, seed, ref, total, first, n, d_out, stream=None):
        rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
        check(lib().pluss_dev_expand_uniform_sorted(self._h, seed, rid, total, first, n, d_out, self._s(stream)),
              "pluss_dev_expand_uniform_sorted")

    def gen_uniform_faithful_refs(self, seed, totals, stream=None):
        """The six samplers over r10's uniform draw generated in key order inside the pass."""
        c = (ctypes.c_uint64 * 6)(*[int(x) for x in totals])
        check(lib().pluss_dev_gen_uniform_faithful_refs(self._h, seed, c, self._s(stream)), "pluss_dev_gen_uniform_faithful_refs")

    def sampled_hist(self, d_samples, n, stream=None):
        check(lib().pluss_dev_sampled_hist(self._h, d_samples, n, self._s(stream)), "pluss_dev_sampled_hist")

    def faithful_hist(self, ref, d_samples, n, stream=None):
        rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
        check(lib().pluss_dev_faithful_hist(self._h, rid, d_samples, n, self._s(stream)), "pluss_dev_faithful_hist")

    def faithful_hist_refs(self, d_samples, counts, stream=None):
        """All six sampler_<REF> at once (r10's main: one thread per reference):
        d_samples holds counts[0] samples of reference 0, then counts[1] of
        reference 1, ...  Same result as six faithful_hist calls."""
        c = (ctypes.c_uint64 * 6)(*[int(x) for x in counts])
        check(lib().pluss_dev_faithful_hist_refs(self._h, d_samples, c, self._s(stream)), "pluss_dev_faithful_hist_refs")

    def faithful_hist_sorted(self, ref, d_samples, n, stream=None):
        """faithful_hist over a list already in key order (no sort; checked)."""
        rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
        check(lib().pluss_dev_faithful_hist_sorted(self._h, rid, d_samples, n, self._s(stream)), "pluss_dev_faithful_hist_sorted")

    def faithful_hist_sorted_refs(self, d_samples, counts, stream=None):
        c = (ctypes.c_uint64 * 6)(*[int(x) for x in counts])
        check(lib().pluss_dev_faithful_hist_sorted_refs(self._h, d_samples, c, self._s(stream)),
              "pluss_dev_faithful_hist_sorted_refs")

    def gen_faithful_refs(self, seed, totals, stream=None):
        """The six samplers over generated key-order lists (never materialised)."""
        c = (ctypes.c_uint64 * 6)(*[int(x) for x in totals])
        check(lib().pluss_dev_gen_faithful_refs(self._h, seed, c, self._s(stream)), "pluss_dev_gen_faithful_refs")

    def fulltrace(self, stream=None):
        check(lib().pluss_dev_fulltrace_hist(self._h, self._s(stream)), "pluss_dev_fulltrace_hist")

    def sampled_ri(self, d_samples, n, d_ri, d_sink, stream=None):
        check(lib().pluss_dev_sampled_ri(self._h, d_samples, n, d_ri, d_sink, self._s(stream)), "pluss_dev_sampled_ri")

    def export(self, d_keys, d_counts, cap, stream=None):
        check(lib().pluss_dev_hist_export(self._h, d_keys, d_counts, cap, self._s(stream)), "pluss_dev_hist_export")

    def export_reset(self, d_keys, d_counts, cap, stream=None):
        """export(), then leave the histogram empty for the next pass (one launch)."""
        check(lib().pluss_dev_hist_export_reset(self._h, d_keys, d_counts, cap, self._s(stream)), "pluss_dev_hist_export_reset")

    def sampled_hist_export(self, d_samples, n, d_keys, d_counts, cap, stream=None):
        """sampled_hist() then export_reset() -- one launch for N % (CLS/DS) == 0 shapes."""
        check(lib().pluss_dev_sampled_hist_export(self._h, d_samples, n, d_keys, d_counts, cap, self._s(stream)),
              "pluss_dev_sampled_hist_export")

    def sampled_hist_dense(self, d_samples, n, d_counts, stream=None):
        """One launch: this pass's dense counts (DENSE_BINS + 1 u64 at d_counts; see dense_keys)."""
        check(lib().pluss_dev_sampled_hist_dense(self._h, d_samples, n, d_counts, self._s(stream)),
              "pluss_dev_sampled_hist_dense")

    def gen_count_dense(self, seed, totals, first, n, d_counts, stream=None):
        """Generate slices [first[r], first[r]+n[r]) of the six key-order lists and
        count them (dense vector) in one launch; the lists never touch memory."""
        a = [(ctypes.c_uint64 * 6)(*[int(x) for x in v]) for v in (totals, first, n)]
        check(lib().pluss_dev_gen_count_dense(self._h, seed, a[0], a[1], a[2], d_counts, self._s(stream)),
              "pluss_dev_gen_count_dense")

    def diag_dense(self, d_samples, n, d_counts, variant=0, max_grid=0, stream=None):
        """Diagnostics (include/pluss_diag.h): a dense pass with an ablation variant
        (0 product, 1 loads only, 2 no tail) and/or a workgroup cap."""
        check(lib().pluss_diag_dense(self._h, d_samples, n, d_counts, variant, max_grid, self._s(stream)), "pluss_diag_dense")

    def diag_sort_words(self, ref, d_samples, n, d_words, stream=None):
        """Diagnostics (include/pluss_diag.h): the faithful radix source's bucket
        sort alone -- reference `ref`'s n samples (any order) -> its packed sort
        words, ascending, into d_words.  Returns the word size in bytes (4 or 8)."""
        rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
        wb = ctypes.c_int32(0)
        check(lib().pluss_diag_sort_words(self._h, rid, d_samples, n, d_words, ctypes.byref(wb), self._s(stream)),
              "pluss_diag_sort_words")
        return int(wb.value)

    def diag_uniform_parts(self, seed, totals, what, d_out, stream=None):
        """Diagnostics (include/pluss_diag.h): the uniform source's plan (0), or
        the plan and every full tile staged (1: as the lane-major pass, 2: packed)."""
        c = (ctypes.c_uint64 * 6)(*[int(x) for x in totals])
        check(lib().pluss_diag_uniform_parts(self._h, seed, c, what, d_out, self._s(stream)),
              "pluss_diag_uniform_parts")

    # faithful mode over key-range shards of the single-read pipeline, all six
    # references at once (pluss_dev_faithful_shards_*; dist.py): every phase
    # writes this shard's summary row (SHARD_ROW u64 at d_row, device memory)
    # and the next reads the rows of all shards gathered at d_rows
    def faithful_shards_local(self, d_samples, seed, totals, first, n, d_row, stream=None):
        """Phase 1 over key-ordered slices (d_samples None: generated slices)."""
        u6 = ctypes.c_uint64 * 6
        check(lib().pluss_dev_faithful_shards_local(self._h, d_samples, seed, u6(*map(int, totals)),
                                                    u6(*map(int, first)), u6(*map(int, n)), d_row, self._s(stream)),
              "pluss_dev_faithful_shards_local")

    def faithful_shards_select(self, d_lists, totals, key_lo, key_hi, d_row, stream=None):
        """Arbitrary-order lists (the six references' whole lists back to back):
        keep the samples whose keys lie in [key_lo, key_hi)."""
        u6 = ctypes.c_uint64 * 6
        check(lib().pluss_dev_faithful_shards_select(self._h, d_lists, u6(*map(int, totals)), key_lo, key_hi, d_row,
                                                     self._s(stream)), "pluss_dev_faithful_shards_select")

    def faithful_shards_local_selected(self, d_rows, shard, nshards, d_row, stream=None):
        """Phase 1 over the selected samples (reads the gathered rows on the host once)."""
        check(lib().pluss_dev_faithful_shards_local_selected(self._h, d_rows, shard, nshards, d_row, self._s(stream)),
              "pluss_dev_faithful_shards_local_selected")

    def faithful_shards_carry(self, d_rows, shard, nshards, d_row, stream=None):
        """Phase 2: the replay state entering this shard -> its replay-start counts."""
        check(lib().pluss_dev_faithful_shards_carry(self._h, d_rows, shard, nshards, d_row, self._s(stream)),
              "pluss_dev_faithful_shards_carry")

    def faithful_shards_cut(self, d_rows, shard, nshards, d_row, stream=None):
        """Phase 3: the starts before this shard -> its first Q1 cut candidates."""
        check(lib().pluss_dev_faithful_shards_cut(self._h, d_rows, shard, nshards, d_row, self._s(stream)),
              "pluss_dev_faithful_shards_cut")

    def faithful_shards_hist(self, d_rows, shard, nshards, stream=None):
        """Phase 4: add this shard's part of the histograms (the global cut from the rows)."""
        check(lib().pluss_dev_faithful_shards_hist(self._h, d_rows, shard, nshards, self._s(stream)),
              "pluss_dev_faithful_shards_hist")

    def faithful_shards_uniform_count(self, seed, totals, shard, nshards, d_row, stream=None):
        """r10's own law over key-range shards, phase 0: this shard's leaves'
        candidates per reference into its row (then all-gather the rows)."""
        u6 = ctypes.c_uint64 * 6
        check(lib().pluss_dev_faithful_shards_uniform_count(self._h, seed, u6(*map(int, totals)), shard, nshards,
                                                            d_row, self._s(stream)),
              "pluss_dev_faithful_shards_uniform_count")

    def faithful_shards_uniform_local(self, d_rows, shard, nshards, d_row, stream=None):
        """Phase 1 of the uniform source: this shard's slice from the gathered
        candidate counts (one host round trip), then its local pass."""
        check(lib().pluss_dev_faithful_shards_uniform_local(self._h, d_rows, shard, nshards, d_row,
                                                            self._s(stream)),
              "pluss_dev_faithful_shards_uniform_local")

    def faithful_shards_slice(self):
        """[(first, n)] per reference: the slices the last key-range pass ran over."""
        f, n = (ctypes.c_uint64 * 6)(), (ctypes.c_uint64 * 6)()
        check(lib().pluss_dev_faithful_shards_slice(self._h, f, n), "pluss_dev_faithful_shards_slice")
        return [(int(a), int(b)) for a, b in zip(f, n)]

    def fetch(self):
        h, keep = _hist_buf()
        check(lib().pluss_hist_fetch(self._h, ctypes.byref(h)), "pluss_hist_fetch")
        return Histogram._from_c(h)


def group_unique_id():
    """A fresh RCCL id (bytes) for Group.rank(): made on one rank, handed to all."""
    buf = (ctypes.c_uint8 * GROUP_ID_BYTES)()
    check(lib().pluss_group_unique_id(buf), "pluss_group_unique_id")
    return bytes(buf)


class Group:
    """pluss_group_*: one pass over several GPUs (or several logical shards of
    one GPU) behind the C ABI, merged over RCCL; results equal one GPU's."""

    def __init__(self, cfg, devices=(0,), shards_per_device=1, _h=None):
        self.cfg = cfg
        self._c = cfg.to_c()
        self._h = ctypes.c_void_p()
        if _h is not None:
            self._h = _h
            return
        devs = (ctypes.c_int32 * len(devices))(*devices)
        check(lib().pluss_group_create(ctypes.byref(self._c), devs, len(devices), shards_per_device,
                                       ctypes.byref(self._h)), "pluss_group_create")

    @classmethod
    def rank(cls, cfg, nranks, rank, uid, shards_per_device=1):
        """One process of a multi-process job (cfg.device: this rank's GPU)."""
        h = ctypes.c_void_p()
        c = cfg.to_c()
        buf = (ctypes.c_uint8 * GROUP_ID_BYTES).from_buffer_copy(uid)
        check(lib().pluss_group_create_rank(ctypes.byref(c), nranks, rank, buf, shards_per_device, ctypes.byref(h)),
              "pluss_group_create_rank")
        return cls(cfg, _h=h)

    def close(self):
        if self._h:
            lib().pluss_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def shards(self):
        a, b = ctypes.c_int32(), ctypes.c_int32()
        check(lib().pluss_group_shards(self._h, ctypes.byref(a), ctypes.byref(b)), "pluss_group_shards")
        return int(a.value), int(b.value)

    def sampled_hist(self, samples):
        s, p = _u64(samples)
        h, keep = _hist_buf()
        check(lib().pluss_group_sampled_hist(self._h, p, len(s), ctypes.byref(h)), "pluss_group_sampled_hist")
        return Histogram._from_c(h)

    def gen_faithful(self, seed, totals):
        h, keep = _hist_buf()
        check(lib().pluss_group_gen_faithful(self._h, seed, (ctypes.c_uint64 * 6)(*map(int, totals)), ctypes.byref(h)),
              "pluss_group_gen_faithful")
        return Histogram._from_c(h)

    def gen_uniform_faithful(self, seed, totals):
        """r10's own law (expand_uniform_sorted's lists) over the group's key-range shards."""
        h, keep = _hist_buf()
        check(lib().pluss_group_gen_uniform_faithful(self._h, seed, (ctypes.c_uint64 * 6)(*map(int, totals)),
                                                     ctypes.byref(h)), "pluss_group_gen_uniform_faithful")
        return Histogram._from_c(h)

    def expand(self, seed, counts):
        check(lib().pluss_group_expand(self._h, seed, (ctypes.c_uint64 * 6)(*map(int, counts))), "pluss_group_expand")

    def dense(self, passes=1):
        """`passes` dense passes over the resident lists; the last pass's merged vector."""
        out = (ctypes.c_uint64 * (DENSE_BINS + 1))()
        check(lib().pluss_group_dense(self._h, passes, out), "pluss_group_dense")
        return [int(x) for x in out]

    def gen_count_dense(self, seed, totals):
        out = (ctypes.c_uint64 * (DENSE_BINS + 1))()
        check(lib().pluss_group_gen_count_dense(self._h, seed, (ctypes.c_uint64 * 6)(*map(int, totals)), out),
              "pluss_group_gen_count_dense")
        return [int(x) for x in out]
