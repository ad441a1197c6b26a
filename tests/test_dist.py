"""Multi-process (world_size 2, gloo, CPU) checks of the sharded path: the
shard partition, the canonical-table exchange and the merge.  The per-rank
tables are built from the oracle's histogram of that rank's shard, encoded
exactly as pluss_dev_hist_export encodes them; the merged result must equal
the oracle histogram of the whole list.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _encode(hist_bins, cap=4096):
    """{(ref,kind,ri): count} -> canonical sorted (keys, counts) int64 arrays."""
    from pluss_sampler_optimization_amd import REF_ID
    keys = sorted(((REF_ID[r] << 60) | (k << 56) | (ri + 2), c) for (r, k, ri), c in hist_bins.items())
    K = np.full(cap, -1, dtype=np.int64)
    C = np.zeros(cap, dtype=np.int64)
    for i, (k, c) in enumerate(keys):
        K[i] = np.uint64(k).view(np.int64)
        C[i] = c
    return K, C


def _worker(rank, world, port, samples_per_ref, N, T, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle as orc
    from pluss_sampler_optimization_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = orc.cfg(N, T)
    counts = [min(samples_per_ref, (N - 1) ** (2 if r < 2 else 3)) for r in range(6)]
    parts = D.shard_ranges(counts, rank, world)
    mine = np.concatenate([orc.expand(c, 0x5EED0001, r, first, n) for r, (first, n) in enumerate(parts) if n])
    ri = orc.clean_ri(c, mine)
    refs = (mine >> np.uint64(60)).astype(np.int64)
    thr = (4 * N + 2) * N
    bins = {}
    for r, x in zip(refs, ri):
        k = 1 if (r == 3 and x > 0 and 2 * x > thr) else 0
        key = (orc.REFS[r], k, int(x))
        bins[key] = bins.get(key, 0) + 1
    K, C = _encode(bins)
    merged = D.allgather_tables(torch.from_numpy(K), torch.from_numpy(C))
    q.put((rank, merged.bins, len(mine)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_merge_equals_whole_list(orc, world):
    N, T, per = 64, 4, 700
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per, N, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = orc.cfg(N, T)
    counts = [min(per, (N - 1) ** (2 if r < 2 else 3)) for r in range(6)]
    whole = np.concatenate([orc.expand(c, 0x5EED0001, r, 0, n) for r, n in enumerate(counts)])
    ri = orc.clean_ri(c, whole)
    refs = (whole >> np.uint64(60)).astype(np.int64)
    want = {}
    for r, x in zip(refs, ri):
        k = 1 if (r == 3 and x > 0 and 2 * x > (4 * N + 2) * N) else 0
        key = (orc.REFS[r], k, int(x))
        want[key] = want.get(key, 0) + 1
    assert sum(n for _, _, n in res) == len(whole)
    for _, bins, _ in res:
        assert bins == want


def test_shard_ranges_partition():
    from pluss_sampler_optimization_amd.dist import shard_ranges
    counts = [10466, 10466, 4189071, 4189071, 4189071, 4189071]
    for world in (1, 2, 3, 8):
        seen = [0] * 6
        for rank in range(world):
            for r, (first, n) in enumerate(shard_ranges(counts, rank, world)):
                assert first == seen[r]
                seen[r] += n
        assert seen == counts


def _dense_worker(rank, world, port, samples_per_ref, N, T, q):
    """Per-rank dense vector (bin = ref*3 + case, located by pluss_dense_keys)
    from the oracle's RIs of this rank's shard, merged by dist.allreduce_dense."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle as orc
    import pluss_sampler_optimization_amd as P
    from pluss_sampler_optimization_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = orc.cfg(N, T)
    cfg = P.SamplerConfig(n=N, threads=T)
    keys = P.dense_keys(cfg)
    counts = [min(samples_per_ref, (N - 1) ** (2 if r < 2 else 3)) for r in range(6)]
    parts = D.shard_ranges(counts, rank, world)
    mine = np.concatenate([orc.expand(c, 0x5EED0001, r, first, n) for r, (first, n) in enumerate(parts) if n])
    ri = orc.clean_ri(c, mine)
    refs = (mine >> np.uint64(60)).astype(np.int64)
    v = np.zeros(P.DENSE_BINS + 1, np.int64)
    for r, x in zip(refs.tolist(), ri.tolist()):
        k = 1 if (r == 3 and x > 0 and 2 * x > (4 * N + 2) * N) else 0
        key = (r << 60) | (k << 56) | (x + 2)
        v[next(b for b in range(3 * r, 3 * r + 3) if keys[b] == key)] += 1
    merged = D.allreduce_dense(torch.from_numpy(v)).numpy()
    q.put((rank, P.hist_from_dense(cfg, merged).bins, len(mine)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dense_allreduce_equals_whole_list(orc, world):
    """The dense multi-GPU merge (bench step for N>1): per-rank (ref, case)
    vectors summed by one all-reduce == the oracle histogram of the whole list."""
    N, T, per = 64, 4, 600
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dense_worker, args=(r, world, port, per, N, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = orc.cfg(N, T)
    counts = [min(per, (N - 1) ** (2 if r < 2 else 3)) for r in range(6)]
    whole = np.concatenate([orc.expand(c, 0x5EED0001, r, 0, n) for r, n in enumerate(counts)])
    ri = orc.clean_ri(c, whole)
    refs = (whole >> np.uint64(60)).astype(np.int64)
    want = {}
    for r, x in zip(refs, ri):
        k = 1 if (r == 3 and x > 0 and 2 * x > (4 * N + 2) * N) else 0
        key = (orc.REFS[r], k, int(x))
        want[key] = want.get(key, 0) + 1
    assert sum(n for _, _, n in res) == len(whole)
    for _, bins, _ in res:
        assert bins == want


def _raise_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from pluss_sampler_optimization_amd import PlussError
    from pluss_sampler_optimization_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    for bad_rank in (None, 1):
        err = PlussError("malformed sample") if rank == bad_rank else None
        try:
            D.raise_together(err)
            out.append("ok")
        except PlussError as e:
            out.append("raised:" + ("other" if "another rank" in str(e) else "own"))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


def test_flag_errors_raise_on_every_rank():
    """A rank whose pass flagged malformed samples / overflow raises, and so do
    the others (one all-reduce of an error word), before any table exchange."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_raise_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res[0] == ["ok", "raised:other"]
    assert res[1] == ["ok", "raised:own"]


def _dense8_worker(rank, world, port, q):
    """Config 3's shape at the node's size: rank `rank` of 8 takes its slice of
    every reference's config-3 index range (default_counts(4096, 2^28)), a
    strided subset of which is counted into the dense (ref, case) vector by the
    closed forms; the vectors are merged by dist.allreduce_dense."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    import oracle as orc
    import pluss_sampler_optimization_amd as P
    from conftest import closed_form_ri
    from pluss_sampler_optimization_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, T = 4096, 8
    c = orc.cfg(N, T)
    cfg = P.SamplerConfig(n=N, threads=T)
    keys = np.array(P.dense_keys(cfg), dtype=np.uint64)
    counts = P.default_counts(N, 1 << 28)
    v = np.zeros(P.DENSE_BINS + 1, np.int64)
    mine = []
    for r, (first, n) in enumerate(D.shard_ranges(counts, rank, world)):
        idx = np.arange(first, first + n, 4096, dtype=np.uint64)
        s = np.concatenate([orc.expand(c, 0x5EED0001, r, int(i), 1) for i in idx[:64]] +
                           [orc.expand(c, 0x5EED0001, r, int(first), min(n, 2000))])
        mine.append(s)
    mine = np.unique(np.concatenate(mine))
    refs, c0, c1, c2 = P.unpack_array(mine)
    ri = closed_form_ri(N, T, 4, 8, refs, c0, c1, c2)
    kind = ((refs == 3) & (ri > 0) & (2 * ri > (4 * N + 2) * N)).astype(np.int64)
    key = (refs.astype(np.uint64) << np.uint64(60)) | (kind.astype(np.uint64) << np.uint64(56)) | (ri + 2).astype(np.uint64)
    for b in range(P.DENSE_BINS):  # C0/C1/C2 have one key for all three cases: its first bin
        if keys[b] not in keys[:b]:
            v[b] = int((key == keys[b]).sum())
    assert v.sum() == len(mine)
    merged = D.allreduce_dense(torch.from_numpy(v)).numpy()
    q.put((rank, merged.tolist(), mine.tolist()))
    dist.destroy_process_group()


def test_dense_allreduce_config3_world8(orc):
    """World size 8 (config 3's node) with config-3 vectors (N=4096, T=8, each
    rank's slice of the 2^28 budget): the all-reduced vector == the closed-form
    histogram of the union of the ranks' samples, identical on every rank."""
    import pluss_sampler_optimization_amd as P
    from conftest import closed_form_counts
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dense8_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allmine = np.concatenate([np.array(m, np.uint64) for _, _, m in res])
    assert len(np.unique(allmine)) == len(allmine)  # the slices are disjoint
    want = closed_form_counts(4096, 8, 4, allmine)
    cfg = P.SamplerConfig(n=4096, threads=8)
    for _, merged, _ in res:
        assert merged == res[0][1]
        assert P.hist_from_dense(cfg, np.array(merged, np.int64)).bins == want
