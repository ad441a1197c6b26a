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


@pytest.mark.parametrize("world", [2, 4])
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
