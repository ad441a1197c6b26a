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

Faithful mode (r10's six sampler_<REF> with their cross-sample queue
semantics) needs one global key order, so it is sharded by contiguous ranges
of the sort key a*T+tid instead.  Each phase of
pluss_dev_faithful_shards_* writes this rank's summary row in device memory;
the rows are all-gathered between phases (over RCCL the whole pass runs
without a host round trip) and the next phase derives its inputs from them on
the device.  The same protocol runs inside libpluss_gpu.so for one-process
multi-GPU callers (pluss_group_*, csrc/pluss_group.hip).
"""
import numpy as np

from ._lib import DENSE_BINS, SHARD_ROW, SHARD_ROW_ERR, PlussError
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


class DeviceRows:
    """The summary rows of a key-range-sharded faithful pass on this rank's
    GPU: `row` (this shard's SHARD_ROW words) and `rows` (all shards', in rank
    order) as device pointers for the pluss_dev_faithful_shards_* phases.
    exchange() all-gathers them: over RCCL on the device, ordered with the
    library's launches on the current stream (no host round trip); over gloo
    (several ranks sharing one GPU in tests) through host copies."""

    def __init__(self, world, dev, group=None):
        import torch
        import torch.distributed as dist
        self.group, self.world = group, world
        self.nccl = dist.get_backend(group) == "nccl"
        self._row = torch.zeros(SHARD_ROW, dtype=torch.int64, device=dev)
        self._rows = torch.zeros(world * SHARD_ROW, dtype=torch.int64, device=dev)
        self.row, self.rows = self._row.data_ptr(), self._rows.data_ptr()

    def fail(self):
        self._row[SHARD_ROW_ERR] = 1

    def exchange(self):
        import torch
        import torch.distributed as dist
        if self.nccl:
            dist.all_gather_into_tensor(self._rows, self._row, group=self.group)
            return
        torch.cuda.current_stream(self._row.device).synchronize()
        out = torch.empty(self.world * SHARD_ROW, dtype=torch.int64)
        dist.all_gather_into_tensor(out, self._row.cpu(), group=self.group)
        self._rows.copy_(out)


def faithful_shards_protocol(shard, phase1, rank, world, rx, stream=None, err=None, selected=False):
    """The phases of a key-range-sharded faithful pass on `shard` (a Context,
    or any object with the same faithful_shards_* methods), the rows exchanged
    by `rx` (DeviceRows, or a host stand-in with row / rows / fail / exchange)
    between phases:
      phase1(row)  this shard's first phase (faithful_shards_local over
                   key-ordered or generated slices, or faithful_shards_select
                   over arbitrary-order lists, then -- selected=True --
                   faithful_shards_local_selected after the first exchange);
      carry, cut, hist, with the gathered rows of all shards.
    A rank whose phase raises (or that enters with `err`) marks its row failed
    and still takes part in every exchange; the other ranks' device phases see
    the error word and their fetch raises (PLUSS_ERR_PEER), so no rank waits
    forever.  Returns this rank's error (None if it ran every phase)."""
    def run(fn, *args):
        nonlocal err
        if err is None:
            try:
                fn(*args)
            except Exception as e:  # noqa: BLE001 -- reported after the pass, on every rank
                err = e
        if err is not None:
            rx.fail()
    run(phase1, rx.row)
    rx.exchange()
    if selected:
        run(shard.faithful_shards_local_selected, rx.rows, rank, world, rx.row, stream)
        rx.exchange()
    run(shard.faithful_shards_carry, rx.rows, rank, world, rx.row, stream)
    rx.exchange()
    run(shard.faithful_shards_cut, rx.rows, rank, world, rx.row, stream)
    rx.exchange()
    run(shard.faithful_shards_hist, rx.rows, rank, world, stream)
    return err


def merge_results(ctx, err, dev, group=None):
    """The end of a sharded faithful pass: this rank's canonical table,
    traversed and error word, all-gathered in ONE collective and summed on
    the host (the same Histogram on every rank).  Raises on every rank if any
    rank failed."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    nccl = dist.get_backend(group) == "nccl"
    W = 2 * TABLE_CAP + 8
    blk = torch.zeros(W, dtype=torch.int64, device=dev)
    trav = [0] * 6
    if err is None:
        try:
            sp = torch.cuda.current_stream(dev).cuda_stream
            ctx.export(blk.data_ptr(), blk.data_ptr() + 8 * TABLE_CAP, TABLE_CAP, sp)
            trav = ctx.fetch().traversed  # the pass's one host wait; raises on this rank's flags
        except Exception as e:  # noqa: BLE001
            err = e
    tail = np.array(trav + [1 if err is not None else 0, 0], dtype=np.uint64).view(np.int64)
    blk[2 * TABLE_CAP:] = torch.from_numpy(tail).to(dev)
    if not nccl:
        blk = blk.cpu()
    out = torch.empty(world * W, dtype=torch.int64, device=blk.device)
    dist.all_gather_into_tensor(out, blk, group=group)
    g = out.cpu().numpy().view(np.uint64).reshape(world, W)
    if err is not None:
        raise err
    if g[:, 2 * TABLE_CAP + 6].any():
        raise PlussError("another rank's faithful shard pass failed")
    h = merge_tables(g[:, :TABLE_CAP], g[:, TABLE_CAP:2 * TABLE_CAP])
    tsum = [int(x) for x in g[:, 2 * TABLE_CAP:2 * TABLE_CAP + 6].sum(axis=0, dtype=np.uint64)]
    return Histogram(h.bins, tsum)


def _pass_stream(dev, stream):
    """The torch stream a sharded faithful pass runs on: the library's phases,
    the row exchanges (DeviceRows) and the merge all on it, so they are
    ordered.  A caller on the null stream gets a stream of its own for the
    pass (the library would take NULL as HIP's null stream, which is ordered
    too but serialises against every other stream of the device)."""
    import torch
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    return torch.cuda.Stream(dev) if st.cuda_stream == 0 else st


def _open(cfg, sp):
    """(Context, None), or (None, the error): a rank that cannot even open its
    handle (e.g. out of memory) still takes part in every exchange of the pass
    with its row marked failed, so the other ranks do not wait forever."""
    try:
        ctx = Context(cfg)
    except Exception as e:  # noqa: BLE001 -- reported after the pass, on every rank
        return None, e
    try:
        ctx.reset(sp)
    except Exception as e:  # noqa: BLE001
        ctx.close()
        return None, e
    return ctx, None


def sharded_faithful_hist(cfg, samples_by_ref, group=None, stream=None):
    """Faithful mode over key-range shards, one GPU per rank, over lists in
    any order (what r10 hands over).

    samples_by_ref: {ref: device int64 tensor holding that reference's whole
    sample list} (identical on every rank).  Every rank keeps its key range
    (faithful_shards_select), sorts it and runs the single-read pipeline's
    phases.  Returns the merged Histogram, with `traversed` summed over ranks
    (identical on all ranks)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", cfg.device)
    lo, hi = key_range(faithful_key_space(cfg), rank, world)
    st = _pass_stream(dev, stream)
    sp = st.cuda_stream
    totals = [0] * 6
    for r, t in samples_by_ref.items():
        totals[REFS.index(r) if isinstance(r, str) else int(r)] = t.numel()
    lists = torch.cat([samples_by_ref[r].reshape(-1) for r in sorted(samples_by_ref,
                       key=lambda x: REFS.index(x) if isinstance(x, str) else int(x))]) if samples_by_ref else \
        torch.zeros(1, dtype=torch.int64, device=dev)
    if st != torch.cuda.current_stream(dev):
        st.wait_stream(torch.cuda.current_stream(dev))  # (the caller's lists)
    with torch.cuda.stream(st):
        rx = DeviceRows(world, dev, group)
        ctx, err = _open(cfg, sp)
        try:
            err = faithful_shards_protocol(
                ctx, lambda row: ctx.faithful_shards_select(lists.data_ptr(), totals, lo, hi, row, sp), rank, world,
                rx, sp, err=err, selected=True)
            return merge_results(ctx, err, dev, group)
        finally:
            if ctx is not None:
                ctx.close()


def sharded_faithful_gen_hist(cfg, seed, totals, group=None, stream=None):
    """Faithful mode over key-range shards of the key-order lists
    (pluss_dev_expand_sorted's lists of totals[r] samples): each rank takes the
    samples whose keys fall in its range -- an index slice, found by the host
    search pluss_keyorder_index_range, since the lists are in key order and
    random access -- and generates them inside its single-read pass; no rank
    reads or holds a whole list.  Returns the merged Histogram (identical on
    every rank)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", cfg.device)
    lo, hi = key_range(faithful_key_space(cfg), rank, world)
    st = _pass_stream(dev, stream)
    sp = st.cuda_stream
    err = None
    first, n = [0] * 6, [0] * 6
    try:
        for r, t in enumerate(totals):
            if t:
                a, b = keyorder_index_range(cfg, seed, r, int(t), lo, hi)
                first[r], n[r] = a, b - a
    except Exception as e:  # noqa: BLE001 -- reported after the pass, on every rank
        err = e
    tot = [int(t) for t in totals]
    if st != torch.cuda.current_stream(dev):
        st.wait_stream(torch.cuda.current_stream(dev))  # (the caller's lists)
    with torch.cuda.stream(st):
        rx = DeviceRows(world, dev, group)
        ctx, err2 = _open(cfg, sp)
        try:
            err = faithful_shards_protocol(
                ctx, lambda row: ctx.faithful_shards_local(None, seed, tot, first, n, row, sp), rank, world, rx, sp,
                err=err or err2)
            return merge_results(ctx, err, dev, group)
        finally:
            if ctx is not None:
                ctx.close()
