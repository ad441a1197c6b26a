"""Key-order stratified lists on the device, and the passes
that use their order: faithful mode without a sort (read from a key-ordered
list, or over lists generated on the fly), and generation fused with the
dense count.  Each is checked against the CPU oracle (orc_expand_sorted,
orc_faithful, the stepping clean RIs via closed forms) and against the
arbitrary-order pipelines (radix sort + scan, expand + dense pass) on the
same lists.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import numpy as np
import pytest

from conftest import closed_form_counts, expected_raw, golden_configs

pytestmark = pytest.mark.gpu

P = pytest.importorskip("pluss_sampler_optimization_amd")
torch = pytest.importorskip("torch")
GOLD = golden_configs()
SEED = 0x5EED0001


def stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("N,T,CS,rf,S", [(128, 4, 4, 0, 2098), (1024, 8, 4, 0, 4189071), (4096, 8, 4, 0, 67025020),
                                         (2048, 64, 4, 0, 4173354), (16, 1, 4, 0, 100), (4096, 8, 4, 0, 3),
                                         (256, 4, 4, 1, 255 ** 3), (64, 2, 1, 0, 5000)])
def test_expand_sorted_equals_oracle(orc, N, T, CS, rf, S):
    c = P.SamplerConfig(n=N, threads=T, chunk=CS, range_full=bool(rf))
    oc = orc.cfg(N, T, CS, range_full=rf)
    for ref in range(6):
        span = N if rf else N - 1
        tot = min(S, span ** (3 if ref >= 2 else 2))
        for first in {0, max(0, tot // 2 - 3000), max(0, tot - 6000)}:
            n = min(6000, tot - first)
            got = P.expand_sorted(c, SEED, ref, tot, first, n)
            np.testing.assert_array_equal(got, orc.expand_sorted(oc, SEED, ref, tot, first, n))


def test_expand_sorted_config2_lists_are_in_key_order(orc):
    """The whole config-2 lists (N=1024, T=8, 2^24 samples) on the device: per
    reference distinct and strictly increasing in the faithful sort key."""
    N, T = 1024, 8
    c = P.SamplerConfig(n=N, threads=T)
    counts = P.default_counts(N, 1 << 24)
    buf = torch.empty(1 << 24, dtype=torch.int64, device="cuda")
    with P.Context(c) as ctx:
        off = 0
        for r, k in enumerate(counts):
            ctx.expand_sorted(SEED, r, k, 0, k, buf.data_ptr() + 8 * off, stream())
            off += k
    host = buf.cpu().numpy().view(np.uint64)
    off = 0
    for r, k in enumerate(counts):
        key = orc.sort_key(N, T, 4, host[off:off + k])
        assert (key[1:] > key[:-1]).all(), r
        off += k
    np.testing.assert_array_equal(host[-5000:], orc.expand_sorted(orc.cfg(N, T), SEED, 5, counts[5],
                                                                   counts[5] - 5000, 5000))


@pytest.mark.parametrize("name,d,smp", GOLD, ids=[g[0] for g in GOLD])
def test_faithful_sorted_on_reference_samples(orc, name, d, smp):
    """The reference's own sample lists, put in key order on the host, through
    the no-sort path: r10's raw histograms and traversed counts."""
    N, T = d["N"], d["T"]
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    parts = []
    for ref in orc.REFS:
        s = orc.pack_array(ref, smp[ref])
        parts.append(s[np.argsort(orc.sort_key(N, T, 4, s), kind="stable")])
    t = torch.from_numpy(np.concatenate(parts).view(np.int64)).cuda()
    with P.Context(c) as ctx:
        ctx.faithful_hist_sorted_refs(t.data_ptr(), [len(p) for p in parts], stream())
        h = ctx.fetch()
        ctx.reset(stream())
        off = 0
        for r, p in enumerate(parts):
            ctx.faithful_hist_sorted(r, t.data_ptr() + 8 * off, len(p), stream())
            off += len(p)
        h1 = ctx.fetch()
    for ref in orc.REFS:
        exp, etrav = expected_raw(d, ref)
        assert {k: v for k, v in h.bins.items() if k[0] == ref} == exp, (name, ref)
        assert h.traversed[P.REF_ID[ref]] == etrav, (name, ref)
    assert h.bins == h1.bins and list(h.traversed) == list(h1.traversed)


@pytest.mark.parametrize("N,T,per", [(128, 4, 2098), (256, 4, 6000), (512, 4, 3000), (128, 8, 9000),
                                     (96, 4, 3000), (120, 3, 3000)])  # the last two: non-power-of-two decode
def test_faithful_sorted_and_generated_equal_oracle(orc, N, T, per):
    """Key-order lists: the no-sort path, the generated path and the radix-sort
    path (on a shuffled copy) all equal the stepping r10 oracle."""
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = [min(per, (N - 1) ** 2) if r < 2 else per for r in range(6)]
    lists = [P.expand_sorted(c, SEED + N, r, k, 0, k) for r, k in enumerate(totals)]
    s = np.concatenate(lists)
    t = torch.from_numpy(s.view(np.int64)).cuda()
    rng = np.random.default_rng(N)
    shuf = np.concatenate([x[rng.permutation(len(x))] for x in lists])
    ts = torch.from_numpy(shuf.view(np.int64)).cuda()
    with P.Context(c) as ctx:
        ctx.faithful_hist_sorted_refs(t.data_ptr(), totals, stream())
        h_sorted = ctx.fetch()
        ctx.reset(stream())
        ctx.gen_faithful_refs(SEED + N, totals, stream())
        h_gen = ctx.fetch()
        ctx.reset(stream())
        ctx.faithful_hist_refs(ts.data_ptr(), totals, stream())
        h_radix = ctx.fetch()
    oc = orc.cfg(N, T)
    for r, ref in enumerate(P.REFS):
        want, trav = orc.faithful(oc, ref, lists[r])
        assert {k: v for k, v in h_sorted.bins.items() if k[0] == ref} == want, (N, ref)
        assert h_sorted.traversed[r] == trav, (N, ref)
    for h in (h_gen, h_radix):
        assert h.bins == h_sorted.bins and list(h.traversed) == list(h_sorted.traversed)


@pytest.mark.parametrize("N,T,total", [(1024, 8, 1 << 24), (4096, 8, 1 << 22), (2048, 64, 1 << 22),
                                       (4096, 8, 1 << 28)])  # the last: config 3's whole budget on one GPU
def test_faithful_sorted_and_generated_at_baseline_shapes(N, T, total):
    """At BASELINE shapes (32-bit words at N=1024, 64-bit at 2048/4096) the
    three pipelines agree: no-sort over the materialised key-order list,
    generated lists, and the radix-sort path over the same list."""
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, total)
    buf = torch.empty(total, dtype=torch.int64, device="cuda")
    with P.Context(c) as ctx:
        off = 0
        for r, k in enumerate(totals):
            ctx.expand_sorted(SEED, r, k, 0, k, buf.data_ptr() + 8 * off, stream())
            off += k
        hs = []
        for run in (lambda: ctx.faithful_hist_sorted_refs(buf.data_ptr(), totals, stream()),
                    lambda: ctx.gen_faithful_refs(SEED, totals, stream()),
                    lambda: ctx.faithful_hist_refs(buf.data_ptr(), totals, stream())):
            ctx.reset(stream())
            run()
            hs.append(ctx.fetch())
    for h in hs[1:]:
        assert h.bins == hs[0].bins and list(h.traversed) == list(hs[0].traversed)
    assert 0 < hs[0].total() <= total + 6


def test_faithful_sorted_rejects_unordered_and_bad_lists():
    N, T = 128, 4
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    s = P.expand_sorted(c, SEED, "A0", 2098, 0, 2098)
    for bad in (s[::-1].copy(), np.concatenate([s[:1000], s[999:]]),  # reversed; a duplicate
                np.concatenate([s[:10], np.array([P.pack("B0", 1, 2, 3)], np.uint64), s[11:]])):  # wrong ref
        t = torch.from_numpy(bad.view(np.int64)).cuda()
        with P.Context(c) as ctx:
            ctx.faithful_hist_sorted("A0", t.data_ptr(), len(bad), stream())
            with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
                ctx.fetch()
    with P.Context(P.SamplerConfig(n=100, threads=5, chunk=4, mode="faithful")) as ctx:  # N % 8 != 0
        with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
            ctx.gen_faithful_refs(SEED, [0, 0, 10, 0, 0, 0], stream())


@pytest.mark.parametrize("N,T,total", [(4096, 8, 1 << 28), (1024, 8, 1 << 24), (2048, 64, 1 << 24), (96, 4, 40000),
                                       (128, 4, 6)])
def test_gen_count_equals_expand_and_count(N, T, total):
    """Generation fused with counting == the materialised key-order list through
    the dense pass == its closed-form histogram; rank slices of 8 sum to the
    whole (the sharded path)."""
    c = P.SamplerConfig(n=N, threads=T, chunk=3 if N == 96 else 4)
    totals = P.default_counts(N, total) if total > 6 else [1] * 6
    d = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device="cuda")
    d2 = torch.zeros_like(d)
    with P.Context(c) as ctx:
        ctx.gen_count_dense(SEED, totals, [0] * 6, totals, d.data_ptr(), stream())
        acc = torch.zeros_like(d)
        for rank in range(8):
            first = [k * rank // 8 for k in totals]
            n = [k * (rank + 1) // 8 - k * rank // 8 for k in totals]
            ctx.gen_count_dense(SEED, totals, first, n, d2.data_ptr(), stream())
            acc += d2
        if total <= 1 << 24:
            buf = torch.empty(sum(totals), dtype=torch.int64, device="cuda")
            off = 0
            for r, k in enumerate(totals):
                ctx.expand_sorted(SEED, r, k, 0, k, buf.data_ptr() + 8 * off, stream())
                off += k
            ctx.sampled_hist_dense(buf.data_ptr(), sum(totals), d2.data_ptr(), stream())
        torch.cuda.synchronize()
    v = d.cpu().numpy()
    assert v[P.DENSE_BINS] == 0 and v[:P.DENSE_BINS].sum() == sum(totals)
    assert (acc.cpu().numpy() == v).all()
    if total <= 1 << 24:
        assert (d2.cpu().numpy() == v).all()
        if N % 8 == 0:
            host = buf.cpu().numpy().view(np.uint64)
            assert P.hist_from_dense(c, v).bins == closed_form_counts(N, T, c.chunk, host)
