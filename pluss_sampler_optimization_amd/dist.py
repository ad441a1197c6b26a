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
"""
import numpy as np

from .api import REFS, Context, hist_from_tables

TABLE_CAP = 4096


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


def sharded_clean_hist(cfg, seed, counts, group=None, stream=None):
    """Every rank: expand its shard on its GPU, histogram it, merge across ranks.
    Returns the merged Histogram (identical on all ranks)."""
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
    with Context(cfg) as ctx:
        off = 0
        for ref, (first, c) in zip(range(len(REFS)), parts):
            ctx.expand(seed, ref, first, c, samples.data_ptr() + 8 * off, sp)
            off += c
        ctx.reset(sp)
        ctx.sampled_hist(samples.data_ptr(), n, sp)
        ctx.export(keys.data_ptr(), cnts.data_ptr(), TABLE_CAP, sp)
        torch.cuda.synchronize(dev)
    if dist.get_backend(group) == "gloo":  # e.g. several ranks sharing one GPU in tests
        keys, cnts = keys.cpu(), cnts.cpu()
    return allgather_tables(keys, cnts, group)
