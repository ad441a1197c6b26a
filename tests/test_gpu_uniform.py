"""r10's uniform draw generated in key order on the device (csrc/pluss_uniform.h
plan + tile staging) against the C oracle's restatement (orc_expand_uniform),
bit for bit, and faithful mode over it: the lists generated inside the pass
(pluss_dev_gen_uniform_faithful_refs) equal the same lists materialised and
read by the sorted source, and the stepping r10 oracle (orc_faithful).

Run on an MI355X:  python -m pytest tests/test_gpu_uniform.py -m gpu -x -q
"""
import numpy as np
import pytest

from conftest import gpu_lockstep

pytestmark = pytest.mark.gpu

P = pytest.importorskip("pluss_sampler_optimization_amd")
torch = pytest.importorskip("torch")
SEED = 0x5EED0001


def stream():
    return torch.cuda.current_stream().cuda_stream


CASES = [(64, 4, "A0", 1000, 0), (128, 4, "B0", 2098, 0), (128, 8, "C0", 164, 0), (64, 2, "C3", 30000, 0),
         (128, 4, "C2", 120_000, 0), (256, 8, "C1", 65025, 0), (512, 4, "B0", 3, 0), (64, 4, "C0", 3969, 0),
         (64, 4, "A0", 5000, 1), (4096, 8, "A0", 5000, 0), (2048, 64, "B0", 300_000, 0),
         (1024, 8, "C2", 4189071, 0), (1024, 8, "C1", 10466, 0),
         # leaves of ~23 expected candidates (one block per row): ~5 % of them past the
         # 32 sorted in registers, through the shared LDS scratch
         (256, 8, "C2", 184000, 0), (1024, 8, "C0", 2500, 0)]


@pytest.mark.parametrize("N,T,ref,S,full", CASES)
def test_device_lists_equal_oracle(orc, N, T, ref, S, full):
    c = P.SamplerConfig(n=N, threads=T, range_full=bool(full))
    oc = orc.cfg(N, T, range_full=full)
    want = orc.expand_uniform(oc, SEED, ref, S, 0, S)
    got = P.expand_uniform_sorted(c, SEED, ref, S, 0, S)
    np.testing.assert_array_equal(got, want)
    a, b = S // 5, S // 5 + max(1, S // 3)
    np.testing.assert_array_equal(P.expand_uniform_sorted(c, SEED, ref, S, a, b - a), want[a:b])


@pytest.mark.parametrize("N,T,total", [(64, 4, 12_000), (128, 4, 8720 * 4), (128, 8, 60_000), (256, 4, 200_000)])
def test_faithful_over_uniform_lists(orc, N, T, total):
    """The six samplers over r10's draw: generated inside the pass == the
    materialised lists through the sorted source == the stepping r10 oracle
    on the same lists."""
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, total)
    lists = [P.expand_uniform_sorted(c, SEED, r, n, 0, n) for r, n in enumerate(totals)]
    t = torch.from_numpy(np.concatenate(lists).view(np.int64)).cuda()
    with P.Context(c) as ctx:
        ctx.reset(stream())
        ctx.gen_uniform_faithful_refs(SEED, totals, stream())
        gen = ctx.fetch()
        ctx.reset(stream())
        ctx.faithful_hist_sorted_refs(t.data_ptr(), totals, stream())
        srt = ctx.fetch()
    assert gen.bins == srt.bins and gen.traversed == srt.traversed
    oc = orc.cfg(N, T)
    for r, ref in enumerate(P.REFS):
        want, wtrav = orc.faithful(oc, ref, lists[r])
        assert {k: v for k, v in gen.bins.items() if k[0] == ref} == want, ref
        assert gen.traversed[r] == wtrav, ref


def test_config3_uniform_pass(orc):
    """BASELINE config 3 on one GPU (N=4096, T=8, 2^28 samples): the lists
    generated inside the pass == materialised and read; a stretch of the C2
    list at its start, middle and end == the C oracle's."""
    N, T = 4096, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, 1 << 28)
    buf = torch.empty(sum(totals), dtype=torch.int64, device="cuda")
    with P.Context(c) as ctx:
        off = 0
        for r, n in enumerate(totals):
            ctx.expand_uniform_sorted(SEED, r, n, 0, n, buf.data_ptr() + 8 * off, stream())
            off += n
        ctx.reset(stream())
        ctx.faithful_hist_sorted_refs(buf.data_ptr(), totals, stream())
        srt = ctx.fetch()
        ctx.reset(stream())
        ctx.gen_uniform_faithful_refs(SEED, totals, stream())
        gen = ctx.fetch()
    assert gen.bins == srt.bins and gen.traversed == srt.traversed
    assert sum(gen.bins.values()) > 0.5 * sum(totals)
    n2 = totals[4]
    c2 = buf[sum(totals[:4]):sum(totals[:5])].cpu().numpy().view(np.uint64)
    oc = orc.cfg(N, T)
    for a in (0, n2 // 2, n2 - 50_000):
        np.testing.assert_array_equal(c2[a:a + 50_000], orc.expand_uniform(oc, SEED, "C2", n2, a, 50_000))


@pytest.mark.parametrize("spd", [1, 3, 8])
@pytest.mark.parametrize("N,T,total", [(64, 4, 12_000), (128, 4, 8720 * 4), (256, 4, 200_000)])
def test_group_over_uniform_lists(orc, N, T, total, spd):
    """test_faithful_over_uniform_lists through the C-ABI group (key-range
    shards, each generating only its stretch of the uniform lists): the
    stepping r10 oracle on the same lists."""
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, total)
    with P.Group(c, [0], spd) as g:
        h = g.gen_uniform_faithful(SEED, totals)
    oc = orc.cfg(N, T)
    for r, ref in enumerate(P.REFS):
        want, wtrav = orc.faithful(oc, ref, orc.expand_uniform(oc, SEED, ref, totals[r], 0, totals[r]))
        assert {k: v for k, v in h.bins.items() if k[0] == ref} == want, (ref, spd)
        assert h.traversed[r] == wtrav, (ref, spd)


# Uniform lists dense enough for Q1 to cut the 2-D references about half way
# (57 % recorded), the 3-D ones sparse (replays chained across tiles); B0 only
# where the oracle's share replays stay affordable (each is (N-7)(4N+2)
# lockstep accesses per thread)
DENSE = {1024: [500_000, 500_000, 20_000, 40, 300_000, 300_000],
         4096: [8_000_000, 8_000_000, 3_000, 0, 1_000_000, 1_000_000]}


@pytest.mark.parametrize("N", [1024, 4096])
def test_uniform_source_vs_oracle_at_baseline_n(orc, N):
    """The faithful pass over r10's law generated inside the pipeline, at the
    BASELINE configs' N (2 and 3): equal to the stepping r10 oracle
    (orc_faithful) replaying the oracle's own uniform lists, through one GPU
    and through a group of 5 logical shards; Q1 cuts C0/C1 inside the list."""
    T = 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = DENSE[N]
    with P.Context(c) as ctx:
        ctx.reset(stream())
        ctx.gen_uniform_faithful_refs(SEED, totals, stream())
        one = ctx.fetch()
    with P.Group(c, [0], 5) as g:
        grp = g.gen_uniform_faithful(SEED, totals)
    assert grp.bins == one.bins and grp.traversed == one.traversed
    oc = orc.cfg(N, T)
    for r, ref in enumerate(P.REFS):
        if not totals[r]:
            continue
        want, wtrav = orc.faithful(oc, ref, orc.expand_uniform(oc, SEED, ref, totals[r], 0, totals[r]))
        assert {k: v for k, v in one.bins.items() if k[0] == ref} == want, (N, ref)
        assert one.traversed[r] == wtrav, (N, ref)
    for ref in ("C0", "C1"):  # Q1 cut inside the list
        rec = sum(v for k, v in one.bins.items() if k[0] == ref and k[2] != -1)
        assert 0.3 * totals[P.REF_ID[ref]] < rec < 0.8 * totals[P.REF_ID[ref]]


def _oracle_all(orc, oc, seed, totals):
    """orc_faithful over the oracle's own uniform lists of every reference,
    the six replays on host threads at once (ctypes drops the GIL): {ref:
    (histogram, traversed)}."""
    from concurrent.futures import ThreadPoolExecutor

    def one(ref, n):
        return ref, orc.faithful(oc, ref, orc.expand_uniform(oc, seed, ref, n, 0, n))
    with ThreadPoolExecutor(6) as ex:
        futs = [ex.submit(one, ref, totals[r]) for r, ref in enumerate(P.REFS) if totals[r]]
        return dict(f.result() for f in futs)


def _b0_edges(N, T, s):
    """(cross-row reuses c1 % 8 == 7, cold: those in a thread's last row,
    first-row samples, last-row samples) of packed B0 samples."""
    m = np.uint64(0xFFFFF)
    c0 = ((s >> np.uint64(40)) & m).astype(np.int64)
    c1 = ((s >> np.uint64(20)) & m).astype(np.int64)
    q = (c0 // (4 * T)) * 4 + c0 % 4
    cross = c1 % 8 == 7
    last = q == N // T - 1
    return int(cross.sum()), int((cross & last).sum()), int((q == 0).sum()), int(last.sum())


# r10's law with B0 in the pass at the BASELINE shapes' N: seeds picked (on the
# CPU, over the oracle's own lists) so B0's few samples hold cross-row share
# reuses (c1 % 8 == 7, RI R - 7S), one cold sample in a thread's last row, and
# samples of the first and last thread-local rows; each cross-row or cold B0
# sample is one replay of (N - 7)(4N + 2) lockstep steps per thread in the
# oracle, so B0 stays small while C0 / C1 are dense enough for Q1 to cut them
# inside the list.  (N, T, seed, totals, B0 edges expected)
B0_LAW = [(4096, 8, 2066, [8_000_000, 8_000_000, 3_000, 48, 1_000_000, 1_000_000], (5, 1, 1, 1)),
          (2048, 64, 10, [2_000_000, 2_000_000, 5_000, 24, 1_000_000, 1_000_000], (2, 1, 2, 2))]


@pytest.mark.parametrize("N,T,seed,totals,edges", B0_LAW)
def test_uniform_b0_share_and_cold_at_baseline_n(orc, N, T, seed, totals, edges):
    """Config 3's N (4096, T=8) and config 4's shape (2048, T=64): the faithful
    pass over r10's law generated inside the pipeline, B0 included (the share
    split r10:2482-2486, cross-row reuses, cold samples of a thread's last
    row: r10:2221-2636), through one GPU and through a group of 5 logical
    key-range shards: equal to the stepping r10 oracle replaying the oracle's
    own lists; Q1 cuts C0 / C1 inside the list."""
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    oc = orc.cfg(N, T)
    assert _b0_edges(N, T, orc.expand_uniform(oc, seed, "B0", totals[3], 0, totals[3])) == edges
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(1) as ex:
        fut = ex.submit(_oracle_all, orc, oc, seed, totals)  # (the replays run while the GPU works)
        with P.Context(c) as ctx:
            ctx.reset(stream())
            ctx.gen_uniform_faithful_refs(seed, totals, stream())
            one = ctx.fetch()
        with P.Group(c, [0], 5) as g:
            grp = g.gen_uniform_faithful(seed, totals)
        want = fut.result()
    assert grp.bins == one.bins and grp.traversed == one.traversed
    for r, ref in enumerate(P.REFS):
        wbins, wtrav = want[ref]
        assert {k: v for k, v in one.bins.items() if k[0] == ref} == wbins, (N, ref)
        assert one.traversed[r] == wtrav, (N, ref)
    assert any(k[0] == "B0" and k[1] == 1 for k in one.bins)  # the share split (cross-row reuses)
    for ref in ("C0", "C1"):  # Q1 cut inside the list
        rec = sum(v for k, v in one.bins.items() if k[0] == ref and k[2] != -1)
        assert 0.3 * totals[P.REF_ID[ref]] < rec < 0.8 * totals[P.REF_ID[ref]]


def test_uniform_key_range_shards_by_hand(orc):
    """The uniform source's shard phases (uniform_count, gather,
    uniform_local, carry, cut, hist) run by hand over 6 handles on one GPU at
    config 2's shape: the shards' slices tile every list in order, and the
    merged histogram equals one GPU's pass."""
    N, T = 1024, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, 1 << 22)
    with P.Context(c) as ctx:
        ctx.reset(stream())
        ctx.gen_uniform_faithful_refs(SEED, totals, stream())
        want = ctx.fetch()
    ns = 6
    ctxs = [P.Context(c) for _ in range(ns)]
    for ctx in ctxs:
        ctx.reset(stream())
    gpu_lockstep(ctxs, [lambda ctx, row, k=k: ctx.faithful_shards_uniform_count(SEED, totals, k, ns, row, stream())
                        for k in range(ns)], stream(),
                 mid=lambda ctx, i, n_, grows, row: ctx.faithful_shards_uniform_local(grows, i, n_, row, stream()))
    bins, trav, nxt = {}, [0] * 6, [0] * 6
    for ctx in ctxs:
        for r, (first, n) in enumerate(ctx.faithful_shards_slice()):
            assert first == nxt[r] or n == 0, (r, first, nxt[r])
            nxt[r] = first + n if n else nxt[r]
        h = ctx.fetch()
        for key, v in h.bins.items():
            bins[key] = bins.get(key, 0) + v
        trav = [(a + b) % (1 << 64) for a, b in zip(trav, h.traversed)]
        ctx.close()
    assert nxt == totals
    assert bins == want.bins and trav == list(want.traversed)
