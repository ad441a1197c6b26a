"""FAITHFUL mode with 64-bit packed sort words (N^3 > 2^30, i.e. N > 1024:
configs 3 and 4) against the stepping r10 oracle (orc_faithful, which replays
r10's sampler_<REF> access by access: queue order, lockstep, Q1/Q3 exits,
LAT[0]-only cold; r10:135-696, Q1 r10:356, cold r10:669-674).

Every list goes through the three element sources of the scan pipeline:
  sorted     a caller's list already in pop order (no sort; order checked),
  radix      the same list shuffled (device radix sort first),
  generated  the key-order list generated inside the pipeline (KeyGen lists).
The oracle replays cost one step per lockstep access, so the lists are
either sparse key-order lists (short replays) or dense windows of a few rows
(long chains across scan tiles, Q1 cuts, cold samples in a thread's last
row) whose key span bounds the replay (tests/conftest.window_list).

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import numpy as np
import pytest

from conftest import all_tids_list, gpu_lockstep, window_list

pytestmark = pytest.mark.gpu

P = pytest.importorskip("pluss_sampler_optimization_amd")
torch = pytest.importorskip("torch")
SEED = 0x5EED0003


def stream():
    return torch.cuda.current_stream().cuda_stream


def three_sources(c, lists, seed=None, totals=None):
    """{source: Histogram} of the six samplers over `lists` (one per reference,
    key order): sorted, radix over a shuffled copy, and -- when `seed` is given
    (lists = expand_sorted(seed, totals)) -- the generated source."""
    counts = [len(x) for x in lists]
    s = np.concatenate(lists).astype(np.uint64)
    rng = np.random.default_rng(11)
    shuf = np.concatenate([x[rng.permutation(len(x))] for x in lists]).astype(np.uint64)
    t = torch.from_numpy(s.view(np.int64)).cuda()
    ts = torch.from_numpy(shuf.view(np.int64)).cuda()
    out = {}
    with P.Context(c) as ctx:
        runs = [("sorted", lambda: ctx.faithful_hist_sorted_refs(t.data_ptr(), counts, stream())),
                ("radix", lambda: ctx.faithful_hist_refs(ts.data_ptr(), counts, stream()))]
        if seed is not None:
            runs.append(("generated", lambda: ctx.gen_faithful_refs(seed, totals, stream())))
        for name, run in runs:
            ctx.reset(stream())
            run()
            out[name] = ctx.fetch()
    return out


def check_vs_oracle(orc, c, hs, lists, refs=None):
    oc = orc.cfg(c.n, c.threads, c.chunk)
    for r, ref in enumerate(P.REFS):
        if not len(lists[r]) or (refs and ref not in refs):
            continue
        want, trav = orc.faithful(oc, ref, lists[r])
        for name, h in hs.items():
            assert {k: v for k, v in h.bins.items() if k[0] == ref} == want, (c.n, ref, name)
            assert h.traversed[r] == trav, (c.n, ref, name)


def test_words64_generated_lists_n1056(orc):
    """N=1056 (T=8, CS=4) is the smallest N % 32 == 0 shape with 64-bit words.
    Key-order lists of several tiles (4096 samples per tile) per reference."""
    N, T = 1056, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = [20000, 20000, 12000, 250, 20000, 20000]
    lists = [P.expand_sorted(c, SEED, r, k, 0, k) for r, k in enumerate(totals)]
    hs = three_sources(c, lists, SEED, totals)
    check_vs_oracle(orc, c, hs, lists)


@pytest.mark.parametrize("N,T,qs", [(1056, 8, "first+last"), (1056, 8, "last"), (2048, 64, "first+last"),
                                    (4096, 8, "first+last"), (4096, 8, "last")])
def test_words64_dense_windows(orc, N, T, qs):
    """Dense windows (the first and/or the last thread-local row, c1 < 16):
    replays chain across tiles, Q1 cuts the list, B0 share reuses cross rows
    and B0 samples of a thread's last row are cold.  B0 at N=2048/T=64 is left
    to the N=1056 and 4096 cases (its first-row share replay is 1.1e9 lockstep
    steps in the oracle)."""
    Q = N // T
    rows = {"first+last": [0, Q - 1], "last": [Q - 1]}[qs]
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    lists = [window_list(N, T, 4, ref, 10000, rows, 16, 7 + r) for r, ref in enumerate(P.REFS)]
    hs = three_sources(c, lists)
    refs = [r for r in P.REFS if not (N == 2048 and r == "B0")]
    check_vs_oracle(orc, c, hs, lists, refs)
    if qs == "last":
        assert hs["sorted"].cold("B0") > 0


@pytest.mark.parametrize("kind", ["generated", "all_tids"])
def test_words64_over_1024_tiles(orc, kind):
    """A reference list of more than 1024 tiles (> 4.2 M samples) at N=4096:
    k_fa_finish's per-thread runs of tiles.  `all_tids`: every point sampled by
    all 8 threads, so Q1 cuts the list about half way, inside a tile far from
    either end."""
    N, T = 4096, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    n = 4_500_000
    lists = [np.zeros(0, np.uint64)] * 6
    if kind == "generated":
        totals = [0, 0, 0, 0, n, 0]
        lists[4] = P.expand_sorted(c, SEED, "C2", n, 0, n)
        hs = three_sources(c, lists, SEED, totals)
    else:
        lists[5] = all_tids_list(N, T, 4, "C3", n // T, [0, 1, 2], 5)
        hs = three_sources(c, lists)
    check_vs_oracle(orc, c, hs, lists)
    h = hs["sorted"]
    ref = "C2" if kind == "generated" else "C3"
    rec = sum(v for k, v in h.bins.items() if k[0] == ref and k[2] != -1)
    if kind == "all_tids":
        assert 0.3 * n < rec < 0.7 * n  # the Q1 cut lies inside the list
    else:
        assert rec >= n - 8  # sparse: at most Q1's exit at the very end drops a sample


def shards_by_hand(c, splits, totals, lists=None, seed=None):
    """The phases of pluss_dev_faithful_shards_* on one GPU, one handle per
    shard, the summary rows gathered by device copies (conftest.gpu_lockstep):
    splits[r] = the index boundaries of reference r's list over the shards
    (uneven, empty shards allowed).  lists: key-ordered sample lists (each
    shard gets its slices); None: the generated key-order lists of `seed`.
    Returns the merged Histogram."""
    S = len(splits[0]) - 1
    first = [[splits[r][k] for r in range(6)] for k in range(S)]
    n = [[splits[r][k + 1] - splits[r][k] for r in range(6)] for k in range(S)]
    ctxs = [P.Context(c) for _ in range(S)]
    bufs = []
    for k, ctx in enumerate(ctxs):
        ctx.reset(stream())
        if lists is not None:
            sl = np.concatenate([lists[r][first[k][r]:first[k][r] + n[k][r]] for r in range(6)]).astype(np.uint64)
            bufs.append(torch.from_numpy(sl.view(np.int64)).cuda() if len(sl) else None)
        else:
            bufs.append(None)
    ptr = [b.data_ptr() if b is not None else None for b in bufs]
    gpu_lockstep(ctxs, [lambda ctx, row, k=k: ctx.faithful_shards_local(ptr[k], seed or 0, totals, first[k], n[k], row,
                                                                         stream()) for k in range(S)], stream())
    bins, trav = {}, [0] * 6
    for ctx in ctxs:
        h = ctx.fetch()
        for key, v in h.bins.items():
            bins[key] = bins.get(key, 0) + v
        trav = [(a + b) % (1 << 64) for a, b in zip(trav, h.traversed)]
        ctx.close()
    return P.Histogram(bins, trav)


@pytest.mark.parametrize("kind", ["generated", "windows"])
def test_key_range_shards_equal_one_gpu(orc, kind):
    """The key-range-sharded single-read pipeline (multi-GPU faithful mode) run
    by hand as 5 uneven shards (one empty) at N=4096: equal to one GPU.
    `windows`: dense first/last-row lists whose replays chain across the shard
    boundaries and whose Q1 cuts fall inside a middle shard; also equal to the
    stepping oracle."""
    N, T = 4096, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    if kind == "generated":
        totals = P.default_counts(N, 1 << 22)
        lists = None
        with P.Context(c) as ctx:
            ctx.gen_faithful_refs(SEED, totals, stream())
            want = ctx.fetch()
    else:
        lists = [window_list(N, T, 4, ref, 10000, [0, N // T - 1], 16, 7 + r) for r, ref in enumerate(P.REFS)]
        totals = [len(x) for x in lists]
        want = three_sources(c, lists)["sorted"]
    fr = [0.0, 0.13, 0.13, 0.5, 0.61, 1.0]  # shard 1 is empty
    splits = [[int(round(f * t)) for f in fr] for t in totals]
    got = shards_by_hand(c, splits, totals, lists=lists, seed=SEED if lists is None else None)
    assert got.bins == want.bins and list(got.traversed) == list(want.traversed)
    if kind == "windows":
        check_vs_oracle(orc, c, {"shards": got}, lists, [r for r in P.REFS if r != "B0"])


def test_selected_key_range_shards_equal_one_gpu(orc):
    """Arbitrary-order lists (what r10 hands over) through the shard protocol's
    select + local_selected phases: every shard reads the whole shuffled lists,
    keeps its key range (5 uneven ranges, one empty), sorts it with the bucket
    sort and runs the single-read pipeline; merged == one GPU's radix source ==
    the stepping oracle."""
    N, T = 4096, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    lists = [window_list(N, T, 4, ref, 10000, [0, N // T - 1], 16, 17 + r) for r, ref in enumerate(P.REFS)]
    totals = [len(x) for x in lists]
    want = three_sources(c, lists)["radix"]
    rng = np.random.default_rng(5)
    shuf = np.concatenate([x[rng.permutation(len(x))] for x in lists]).astype(np.uint64)
    t = torch.from_numpy(shuf.view(np.int64)).cuda()
    ks = P.faithful_key_space(c)
    b = [0, ks // 9, ks // 9, ks // 2, (3 * ks) // 4, ks]  # shard 1 is empty
    ctxs = [P.Context(c) for _ in range(5)]
    for ctx in ctxs:
        ctx.reset(stream())
    gpu_lockstep(ctxs, [lambda ctx, row, k=k: ctx.faithful_shards_select(t.data_ptr(), totals, b[k], b[k + 1], row,
                                                                          stream()) for k in range(5)],
                 stream(), selected=True)
    bins, trav = {}, [0] * 6
    for ctx in ctxs:
        h = ctx.fetch()
        for key, v in h.bins.items():
            bins[key] = bins.get(key, 0) + v
        trav = [(x + y) % (1 << 64) for x, y in zip(trav, h.traversed)]
        ctx.close()
    assert bins == want.bins and trav == list(want.traversed)
    check_vs_oracle(orc, c, {"selected": P.Histogram(bins, trav)}, lists, [r for r in P.REFS if r != "B0"])
