"""Multi-GPU sharding of the sampled path (one process per GPU).

Clean-mode reuse intervals are a pure function of (config, sample), so the
sample index range of every reference is split into contiguous per-rank
slices (each rank expands its own slices with the counter-based bijection: no
data-path communication).  The only exchange is the histogram merge: every
rank exports its canonical (key, count) table (pluss_dev_hist_export: sorted
keys, fixed capacity) and the tables are all-gathered over RCCL and summed by
key.  An all-gather of ~64 KB per rank replaces an all-reduce because the
exact-key tables are sparse (a dense all-reduce over exact RI values would
need one slot per possible RI).

For N % (cls/ds) == 0 shapes (every BASELINE configuration) the histogram
of a pass is a dense vector of PLUSS_DENSE_BINS (ref, case) counts
(pluss_dev_sampled_hist_dense), identical in layout on every rank, so the
merge is one element-wise all-reduce of DENSE_BINS + 1 int64 words
(sharded_clean_dense) -- the bench's multi-GPU step.

Faithful mode (one r10 sampler_<REF> with its cross-sample queue semantics)
needs one global key order, so it is sharded by contiguous ranges of the sort
key a*T+tid instead: every rank reads the whole per-reference
list, keeps and sorts its key range, and four small all-gathers of per-shard
summaries (count / first key / max sink, start count, cut candidate) carry
the scan state across shards (include/pluss_gpu.h, pluss_dev_faithful_shard_*).
"""
import numpy as np

from ._lib import DENSE_BINS, PlussError
from .api import (REFS, Context, Histogram, faithful_key_space, hist_from_dense, hist_from_tables,
                  keyorder_index_range)

TABLE_CAP = 4096
KEY_EMPTY = (1 << 64) - 1


def shard_ranges(counts, rank, world):
    """[(first, n)] per reference: contiguous slice `rank` of `world` of each index range."""
    out = []
    for c in counts:
        lo, hi = c * rank // world, c * (rank + 1) // world
        out.append((lo, hi - lo))
    return out


def merge_tables(keys, counts):
    """Sum gathered canonical tables by key -> Histogram (host-only)."""
    k = np.ascontiguousarray(np.asarray(keys).reshape(-1)).view(np.uint64)
    c = np.ascontiguousarray(np.asarray(counts).reshape(-1)).view(np.uint64)
    return hist_from_tables(k, c)


def allgather_tables(keys_t, counts_t, group=None):
    """All-gather per-rank (key, count) int64 tensors (device tensors with the
    nccl/RCCL backend, host tensors with gloo) and merge them."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    gk = torch.empty(world * keys_t.numel(), dtype=keys_t.dtype, device=keys_t.device)
    gc = torch.empty(world * counts_t.numel(), dtype=counts_t.dtype, device=counts_t.device)
    dist.all_gather_into_tensor(gk, keys_t, group=group)
    dist.all_gather_into_tensor(gc, counts_t, group=group)
    return merge_tables(gk.cpu().numpy(), gc.cpu().numpy())


def raise_together(err, group=None, device=None):
    """Every rank learns whether any rank failed (one all-reduce of an error
    word) and all raise together, so no rank is left waiting in a later
    collective.  `err` is this rank's exception or None."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if err is not None else 0], dtype=torch.int64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if err is not None:
        raise err
    if int(t.item()):
        raise PlussError("another rank's sampler pass failed (malformed samples or table overflow)")


def sharded_clean_hist(cfg, seed, counts, group=None, stream=None):
    """Every rank: expand its shard on its GPU, histogram it, merge across ranks.
    Returns the merged Histogram (identical on all ranks).  Malformed samples
    and table overflow on any rank raise PlussError on every rank before the
    tables are exchanged."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    parts = shard_ranges(counts, rank, world)
    n = sum(c for _, c in parts)
    dev = torch.device("cuda", cfg.device)
    samples = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    keys = torch.empty(TABLE_CAP, dtype=torch.int64, device=dev)
    cnts = torch.empty(TABLE_CAP, dtype=torch.int64, device=dev)
    sp = stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    err = None
    with Context(cfg) as ctx:
        try:  # any failure of the local pass is raised on every rank, before the exchange
            off = 0
            for ref, (first, c) in zip(range(len(REFS)), parts):
                ctx.expand(seed, ref, first, c, samples.data_ptr() + 8 * off, sp)
                off += c
            ctx.reset(sp)
            ctx.sampled_hist(samples.data_ptr(), n, sp)
            ctx.export(keys.data_ptr(), cnts.data_ptr(), TABLE_CAP, sp)
            torch.cuda.synchronize(dev)
            ctx.fetch()  # the handle's flags: malformed samples, table or export overflow
        except Exception as e:  # noqa: BLE001
            err = e
    gloo = dist.get_backend(group) == "gloo"  # e.g. several ranks sharing one GPU in tests
    raise_together(err, group, None if gloo else dev)
    if gloo:
        keys, cnts = keys.cpu(), cnts.cpu()
    return allgather_tables(keys, cnts, group)


def allreduce_dense(counts_t, group=None):
    """Element-wise sum of per-rank dense count vectors (int64 tensors: on the
    GPU with nccl/RCCL, on the CPU with gloo); in place, returns the tensor."""
    import torch.distributed as dist
    dist.all_reduce(counts_t, group=group)
    return counts_t


def sharded_clean_dense(cfg, seed, counts, group=None, stream=None):
    """Every rank: expand its shard on its GPU, one dense pass, all-reduce.
    Returns the merged Histogram (identical on all ranks)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    parts = shard_ranges(counts, rank, world)
    n = sum(c for _, c in parts)
    dev = torch.device("cuda", cfg.device)
    samples = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    dense = torch.zeros(DENSE_BINS + 1, dtype=torch.int64, device=dev)
    sp = stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    err = None
    with Context(cfg) as ctx:
        try:  # a failed local pass raises on every rank, before the all-reduce
            off = 0
            for ref, (first, c) in zip(range(len(REFS)), parts):
                ctx.expand(seed, ref, first, c, samples.data_ptr() + 8 * off, sp)
                off += c
            ctx.sampled_hist_dense(samples.data_ptr(), n, dense.data_ptr(), sp)
            torch.cuda.synchronize(dev)
        except Exception as e:  # noqa: BLE001
            err = e
    gloo = dist.get_backend(group) == "gloo"  # e.g. several ranks sharing one GPU in tests
    raise_together(err, group, None if gloo else dev)
    if gloo:
        dense = dense.cpu()
    v = allreduce_dense(dense, group).cpu().numpy()
    if v[DENSE_BINS]:
        raise ValueError(f"{int(v[DENSE_BINS])} malformed samples")
    return hist_from_dense(cfg, v)


def key_range(key_space, rank, world):
    """Contiguous slice `rank` of `world` of the faithful key space [0, key_space)."""
    return key_space * rank // world, key_space * (rank + 1) // world


def torch_allgather(group=None, device=None):
    """allgather(list of u64) -> one list per rank, over torch.distributed
    (int64 tensors on `device`: a GPU with nccl/RCCL, the CPU with gloo)."""
    import torch
    import torch.distributed as dist

    def allgather(vals):
        t = torch.tensor(np.array(vals, dtype=np.uint64).view(np.int64), device=device)
        out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(out, t, group=group)
        return [[int(v) for v in o.cpu().numpy().view(np.uint64)] for o in out]
    return allgather


def faithful_shard_protocol(shard, ref, d_samples, n, key_lo, key_hi, rank, allgather, stream=None, err=None):
    """The four phases of a key-range-sharded faithful sampler on `shard` (a
    Context, or any object with the same faithful_shard_* methods), exchanging
    the per-shard summaries with `allgather`.  Returns (n_total, cut).

    Every exchange carries an error word: a rank whose phase raised (or that
    enters with `err`, e.g. from generating its slice) still takes part in the
    exchange, and then every rank raises at that same exchange -- no rank is
    left waiting in a later collective."""
    def exchange(vals):
        nonlocal err
        g = allgather([1 if err is not None else 0] + list(vals))
        if err is not None:
            raise err
        if any(x[0] for x in g):
            raise PlussError("another rank's faithful shard pass failed")
        return [x[1:] for x in g]

    def phase(fn, *args, default):
        nonlocal err
        if err is not None:
            return default
        try:
            return fn(*args)
        except Exception as e:  # noqa: BLE001 -- re-raised at the next exchange, on every rank
            err = e
            return default
    m, first, mx = phase(shard.faithful_shard_keys, ref, d_samples, n, key_lo, key_hi, stream,
                         default=(0, KEY_EMPTY, 0))
    g = exchange([m, first, mx])
    j_off = sum(x[0] for x in g[:rank])
    n_total = sum(x[0] for x in g)
    pmax_in = max([x[2] for x in g[:rank] if x[0] > 0], default=0)
    later = [x for x in g[rank + 1:] if x[0] > 0]
    next_first = later[0][1] if later else KEY_EMPTY
    ns = phase(shard.faithful_shard_starts, j_off, pmax_in, stream, default=0)
    s_off = sum(x[0] for x in exchange([ns])[:rank])
    c = phase(shard.faithful_shard_cut, s_off, n_total, stream, default=n_total)
    cut = min(x[0] for x in exchange([c]))
    phase(shard.faithful_shard_hist, cut, next_first, not later, stream, default=None)
    exchange([])  # the last phase's error, before the caller's merge collectives
    return n_total, cut


def _export_fetch(ctx, keys, cnts, sp, dev):
    """Export the handle's canonical table and read its flags: (traversed, error or None)."""
    import torch
    try:
        ctx.export(keys.data_ptr(), cnts.data_ptr(), TABLE_CAP, sp)
        torch.cuda.synchronize(dev)
        return ctx.fetch().traversed, None
    except Exception as e:  # noqa: BLE001 -- raised on every rank by raise_together
        return [0] * 6, e


def sharded_faithful_hist(cfg, samples_by_ref, group=None, stream=None):
    """Faithful mode over key-range shards, one GPU per rank.

    samples_by_ref: {ref: device int64 tensor holding that reference's whole
    sample list} (identical on every rank).  Returns the merged Histogram,
    with `traversed` summed over ranks (identical on all ranks)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", cfg.device)
    ag = torch_allgather(group, dev if nccl else "cpu")
    lo, hi = key_range(faithful_key_space(cfg), rank, world)
    sp = stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    keys = torch.empty(TABLE_CAP, dtype=torch.int64, device=dev)
    cnts = torch.empty(TABLE_CAP, dtype=torch.int64, device=dev)
    with Context(cfg) as ctx:
        ctx.reset(sp)
        for ref, t in samples_by_ref.items():
            faithful_shard_protocol(ctx, ref, t.data_ptr(), t.numel(), lo, hi, rank, ag, sp)
        trav, err = _export_fetch(ctx, keys, cnts, sp, dev)
    raise_together(err, group, dev if nccl else None)
    tsum = [sum(col) % (1 << 64) for col in zip(*ag(trav))]
    if not nccl:
        keys, cnts = keys.cpu(), cnts.cpu()
    h = allgather_tables(keys, cnts, group)
    return Histogram(h.bins, tsum)


def faithful_shards_protocol(shard, d_samples, seed, totals, first, n, rank, allgather, stream=None, err=None):
    """Faithful mode over key-range shards of the single-read pipeline, all six
    references at once (pluss_dev_faithful_shards_*): `shard` (a Context, or
    any object with the same faithful_shards_* methods) holds this rank's
    slices [first[r], first[r] + n[r]) of the six key-ordered lists of
    totals[r] samples (d_samples; None: generated), and three exchanges of
    six-word summaries carry the scan across the ranks:
      1. (n, largest sink) -> the largest sink of the earlier ranks = the carry;
      2. the start counts -> the starts before this rank;
      3. the first Q1 cut candidates -> the global cut (their minimum).
    Every exchange carries an error word, as in faithful_shard_protocol.
    Returns the global cuts."""
    def exchange(vals):
        nonlocal err
        g = allgather([1 if err is not None else 0] + [int(v) for v in vals])
        if err is not None:
            raise err
        if any(x[0] for x in g):
            raise PlussError("another rank's faithful shard pass failed")
        return [x[1:] for x in g]

    def phase(fn, *args, default):
        nonlocal err
        if err is not None:
            return default
        try:
            return fn(*args)
        except Exception as e:  # noqa: BLE001 -- re-raised at the next exchange, on every rank
            err = e
            return default
    mx = phase(shard.faithful_shards_local, d_samples, seed, totals, first, n, stream, default=[0] * 6)
    g = exchange(list(n) + list(mx))
    carry = [max([x[6 + r] for x in g[:rank] if x[r] > 0], default=0) for r in range(6)]
    last = [not any(x[r] > 0 for x in g[rank + 1:]) for r in range(6)]
    st = phase(shard.faithful_shards_carry, carry, stream, default=[0] * 6)
    g = exchange(st)
    before = [sum(x[r] for x in g[:rank]) for r in range(6)]
    cand = phase(shard.faithful_shards_cut, before, stream, default=list(totals))
    g = exchange(cand)
    cut = [min(x[r] for x in g) for r in range(6)]
    phase(shard.faithful_shards_hist, cut, last, stream, default=None)
    exchange([])  # the last phase's error, before the caller's merge collectives
    return cut


def sharded_faithful_gen_hist(cfg, seed, totals, group=None, stream=None):
    """Faithful mode over key-range shards of the key-order lists
    (pluss_dev_expand_sorted's lists of totals[r] samples): each rank takes the
    samples whose keys fall in its range -- an index slice, found by the host
    search pluss_keyorder_index_range, since the lists are in key order and
    random access -- and generates them inside its single-read pass; no rank
    reads or holds a whole list.  Then the three-exchange protocol of
    faithful_shards_protocol.  Returns the merged Histogram (identical on
    every rank)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", cfg.device)
    ag = torch_allgather(group, dev if nccl else "cpu")
    lo, hi = key_range(faithful_key_space(cfg), rank, world)
    sp = stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    keys = torch.empty(TABLE_CAP, dtype=torch.int64, device=dev)
    cnts = torch.empty(TABLE_CAP, dtype=torch.int64, device=dev)
    err = None
    first, n = [0] * 6, [0] * 6
    try:
        for r, t in enumerate(totals):
            if t:
                a, b = keyorder_index_range(cfg, seed, r, int(t), lo, hi)
                first[r], n[r] = a, b - a
    except Exception as e:  # noqa: BLE001 -- raised on every rank by the protocol's first exchange
        err = e
    with Context(cfg) as ctx:
        ctx.reset(sp)
        faithful_shards_protocol(ctx, None, seed, [int(t) for t in totals], first, n, rank, ag, sp, err=err)
        trav, err = _export_fetch(ctx, keys, cnts, sp, dev)
    raise_together(err, group, dev if nccl else None)
    tsum = [sum(col) % (1 << 64) for col in zip(*ag(trav))]
    if not nccl:
        keys, cnts = keys.cpu(), cnts.cpu()
    h = allgather_tables(keys, cnts, group)
    return Histogram(h.bins, tsum)
