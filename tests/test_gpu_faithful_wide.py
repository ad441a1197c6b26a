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

from conftest import all_tids_list, window_list

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
