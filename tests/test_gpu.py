"""GPU parity tests: the HIP kernels (through the C ABI) against the CPU oracle
and the reference's own r10 dumps.  Integer results must be bit-exact.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import os

import numpy as np
import pytest

from conftest import closed_form_ri, expected_raw, golden_configs

pytestmark = pytest.mark.gpu

P = pytest.importorskip("pluss_sampler_optimization_amd")
GOLD = golden_configs()

IRREGULAR = [(16, 2, 4, 8, 64), (24, 3, 2, 8, 64), (12, 5, 1, 8, 64), (10, 1, 3, 8, 64), (5, 2, 1, 8, 64),
             (20, 2, 3, 4, 64), (18, 3, 2, 8, 32), (7, 2, 2, 8, 8), (100, 3, 5, 8, 64), (9, 4, 2, 16, 64),
             (1, 1, 1, 8, 64), (2, 3, 1, 8, 64)]


def cfg(N, T, CS=4, DS=8, CLS=64, **kw):
    return P.SamplerConfig(n=N, threads=T, chunk=CS, ds=DS, cls=CLS, **kw)


def oracle_clean_hist(orc, c, samples, thr_variant=0):
    """Histogram of every sample's stepping-replay RI (clean mode), as {(ref,kind,ri): count}."""
    ri = orc.clean_ri(c, samples, nthreads=8)
    refs = (samples >> np.uint64(60)).astype(np.int64)
    N = c.N
    thr = (N + 1) * N + 1 if thr_variant else (4 * N + 2) * N
    kind = ((refs == 3) & (ri > 0) & (2 * ri > thr)).astype(np.int64)
    out = {}
    for r, k, x in zip(refs, kind, ri):
        key = (P.REFS[r], int(k), int(x))
        out[key] = out.get(key, 0) + 1
    return out


def closed_form_hist(N, T, CS, samples):
    """{(ref, kind, ri): count} of a list from the closed forms (N % 8 == 0 shapes)."""
    refs, c0, c1, c2 = P.unpack_array(samples)
    ri = closed_form_ri(N, T, CS, 8, refs, c0, c1, c2)
    kind = ((refs == 3) & (ri > 0) & (2 * ri > (4 * N + 2) * N)).astype(np.int64)
    keys = (refs * 4 + kind) * (1 << 40) + (ri + 2)
    u, cnt = np.unique(keys, return_counts=True)
    return {(P.REFS[int(k >> 42)], int((k >> 40) & 3), int(k & ((1 << 40) - 1)) - 2): int(n) for k, n in zip(u, cnt)}


def all_samples(orc, smp):
    return np.concatenate([orc.pack_array(ref, smp[ref]) for ref in orc.REFS])


@pytest.mark.parametrize("name,d,smp", GOLD, ids=[g[0] for g in GOLD])
def test_faithful_gpu_equals_reference_r10_dumps(orc, name, d, smp):
    """FAITHFUL mode reproduces r10's raw per-reference histograms and traversed counts."""
    h = P.sampled_hist(cfg(d["N"], d["T"], mode="faithful"), all_samples(orc, smp))
    for ref in orc.REFS:
        exp, etrav = expected_raw(d, ref)
        got = {k: v for k, v in h.bins.items() if k[0] == ref}
        assert got == exp, (name, ref)
        assert h.traversed[P.REF_ID[ref]] == etrav, (name, ref)


@pytest.mark.parametrize("name,d,smp", GOLD, ids=[g[0] for g in GOLD])
def test_clean_gpu_equals_oracle_on_reference_samples(orc, name, d, smp):
    s = all_samples(orc, smp)
    h = P.sampled_hist(cfg(d["N"], d["T"]), s)
    assert h.bins == oracle_clean_hist(orc, orc.cfg(d["N"], d["T"]), s)


@pytest.mark.parametrize("shape", IRREGULAR, ids=[str(s) for s in IRREGULAR])
def test_ri_dump_generic_path_equals_oracle(orc, model_host, shape):
    N, T, CS, DS, CLS = shape
    from test_host_model import edge_samples
    s = edge_samples(orc, N, 256, seed=N + 7 * T)
    ri, sink = P.sampled_ri(cfg(N, T, CS, DS, CLS), s)
    np.testing.assert_array_equal(ri, orc.clean_ri(orc.cfg(N, T, CS, DS, CLS), s))
    _, _, hsink = model_host.ri(N, T, CS, DS, CLS, s, 0)
    np.testing.assert_array_equal(sink, hsink)
    h = P.sampled_hist(cfg(N, T, CS, DS, CLS), s)
    assert h.bins == oracle_clean_hist(orc, orc.cfg(N, T, CS, DS, CLS), s)


@pytest.mark.parametrize("N,T,CS,DS,CLS,thr", [(128, 4, 4, 8, 64, 1), (64, 8, 4, 8, 64, 0), (100, 3, 5, 8, 64, 1),
                                              (20, 2, 3, 4, 64, 1), (33, 4, 2, 8, 64, 0), (256, 4, 4, 8, 64, 1),
                                              (96, 3, 3, 8, 64, 1), (72, 5, 2, 8, 64, 0), (40, 2, 4, 8, 32, 1)])
def test_fulltrace_gpu_equals_oracle(orc, N, T, CS, DS, CLS, thr):
    """Full trace (sampling rate 1.0) == seq.cpp sampler() restated (per-source-ref raw bins):
    the ballot kernel (N % W == 0) and the exact-key kernel (other shapes)."""
    c = cfg(N, T, CS, DS, CLS, thr_variant="v1" if thr else "r10")
    h = P.fulltrace_hist(c)
    want, trav = orc.fulltrace(N, T, CS, DS, CLS, thr_variant=thr)
    assert h.bins == want
    assert h.traversed[0] == trav


def test_fulltrace_kat_n128(orc):
    """SURVEY.md §4 KAT against the reference seq binary."""
    h = P.fulltrace_hist(cfg(128, 4, thr_variant="v1"))
    assert h.noshare() == {-1: 12288, 1: 2127872, 3: 2097152, 4: 1835008, 486: 260096, 514: 1835008}
    assert h.share() == {62194: 253952}
    assert h.traversed[0] == 8421376


@pytest.mark.parametrize("N,rf", [(20, 0), (128, 0), (1024, 0), (31, 1)])
def test_expand_gpu_equals_oracle(orc, N, rf):
    c = cfg(N, 4, range_full=bool(rf))
    span = N if rf else N - 1
    for ref in range(6):
        n = min(20000, span ** (2 if ref < 2 else 3) - 5)
        a = P.expand_samples(c, 0x5EED0001, ref, 5, n)
        np.testing.assert_array_equal(a, orc.expand(orc.cfg(N, 4, range_full=rf), 0x5EED0001, ref, 5, n))
        assert len(np.unique(a)) == n


def test_faithful_gpu_equals_oracle_expanded_lists(orc):
    """Faithful mode on longer bijection lists (more Q1 drops and cold samples)."""
    for N, T, per in [(64, 4, 6000), (128, 8, 9000), (256, 4, 3000)]:
        c = cfg(N, T, mode="faithful")
        s = np.concatenate([P.expand_samples(c, 0x5EED0000 + N, r, 0, per if r >= 2 else min(per, (N - 1) ** 2))
                            for r in range(6)])
        h = P.sampled_hist(c, s)
        oc = orc.cfg(N, T)
        for ref in orc.REFS:
            part = s[(s >> np.uint64(60)) == np.uint64(P.REF_ID[ref])]
            want, trav = orc.faithful(oc, ref, part)
            got = {k: v for k, v in h.bins.items() if k[0] == ref}
            assert got == want, (N, T, ref)
            assert h.traversed[P.REF_ID[ref]] == trav, (N, T, ref)


def test_config2_full_size_clean_histogram():
    """BASELINE config 2 at full size (N=1024, T=8, 2^24 samples): the device
    histogram equals the closed-form histogram of the same list (an independent
    restatement) and accounts for every sample."""
    N, T = 1024, 8
    c = cfg(N, T)
    counts = P.default_counts(N, 1 << 24)
    s = np.concatenate([P.expand_samples(c, 0x5EED0001, r, 0, counts[r]) for r in range(6)])
    h = P.sampled_hist(c, s)
    assert h.total() == 1 << 24
    refs, c0, c1, c2 = P.unpack_array(s)
    ri = closed_form_ri(N, T, 4, 8, refs, c0, c1, c2)
    kind = (refs == 3) & (ri > 0) & (2 * ri > (4 * N + 2) * N)
    keys = (refs * 4 + kind.astype(np.int64)) * (1 << 40) + (ri + 2)
    u, cnt = np.unique(keys, return_counts=True)
    want = {(P.REFS[int(k >> 42)], int((k >> 40) & 3), int(k & ((1 << 40) - 1)) - 2): int(n) for k, n in zip(u, cnt)}
    assert h.bins == want


def test_invalid_samples_raise():
    c = cfg(32, 4)
    bad = np.array([P.pack("C3", 1, 2, 3), P.pack("A0", 40, 0, 0)], np.uint64)
    with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
        P.sampled_hist(c, bad)
    with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
        P.sampled_hist(c, np.array([7 << 60], np.uint64))
    with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
        P.sampled_hist(c, np.array([P.pack("C3", 1, 2, 3), P.pack("B0", 3, 2, 1), 7 << 60], np.uint64))
    with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
        P.sampled_hist(cfg(32, 4, mode="faithful"), bad)
    # the device is still healthy afterwards
    assert P.sampled_hist(c, bad[:1]).total() == 1


def test_empty_and_odd_lengths(orc):
    c = cfg(32, 4)
    assert P.sampled_hist(c, np.zeros(0, np.uint64)).bins == {}
    s = P.expand_samples(c, 1, "B0", 0, 777)
    for n in (1, 2, 3, 777):
        assert P.sampled_hist(c, s[:n]).bins == oracle_clean_hist(orc, orc.cfg(32, 4), s[:n])


def test_device_handle_path_and_canonical_export(orc):
    """Handle API with device-resident samples (torch memory), unaligned views,
    and the canonical table used for the cross-GPU merge."""
    torch = pytest.importorskip("torch")
    N, T = 256, 4
    c = cfg(N, T)
    counts = P.default_counts(N, 200000)
    total = sum(counts)
    buf = torch.empty(total + 1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with P.Context(c) as ctx:
        off = 1  # 8-byte aligned, not 16-byte aligned
        for r in range(6):
            ctx.expand(0x5EED0001, r, 0, counts[r], buf.data_ptr() + 8 * off, stream)
            off += counts[r]
        ctx.reset(stream)
        ctx.sampled_hist(buf.data_ptr() + 8, total, stream)
        keys = torch.empty(4096, dtype=torch.int64, device="cuda")
        cnts = torch.empty(4096, dtype=torch.int64, device="cuda")
        ctx.export(keys.data_ptr(), cnts.data_ptr(), 4096, stream)
        torch.cuda.synchronize()
        h = ctx.fetch()
        # export-and-reset: two passes give identical tables and leave the table empty
        k1 = torch.empty(4096, dtype=torch.int64, device="cuda")
        n1 = torch.empty(4096, dtype=torch.int64, device="cuda")
        ctx.reset(stream)  # fetch() does not clear; start the passes from an empty table
        for _ in range(2):
            ctx.sampled_hist(buf.data_ptr() + 8, total, stream)
            ctx.export_reset(k1.data_ptr(), n1.data_ptr(), 4096, stream)
            torch.cuda.synchronize()
            assert torch.equal(k1, keys) and torch.equal(n1, cnts)
        assert ctx.fetch().bins == {}
    host = buf[1:].cpu().numpy().view(np.uint64)
    assert h == P.sampled_hist(c, host)
    k = keys.cpu().numpy().view(np.uint64)
    n = cnts.cpu().numpy().view(np.uint64)
    used = k[k != np.uint64(2 ** 64 - 1)]
    assert (used[1:] > used[:-1]).all()
    assert P.hist_from_tables(k, n) == h
    assert h.total() == total


@pytest.mark.parametrize("N,T,CS", [(256, 4, 4), (96, 3, 3), (100, 3, 5)], ids=["fast_p2", "fast", "generic"])
def test_fused_count_and_export(orc, N, T, CS):
    """pluss_dev_sampled_hist_export (one launch on FAST shapes: the last
    workgroup writes the table) == sampled_hist + export_reset == the oracle;
    repeated passes, empty lists, unaligned lists, a too-small table, and a
    handle already holding faithful-mode counts (two-launch fallback)."""
    torch = pytest.importorskip("torch")
    c = cfg(N, T, CS)
    counts = P.default_counts(N, 60000)
    total = sum(counts)
    host = np.concatenate([P.expand_samples(c, 0x5EED0002, r, 0, counts[r]) for r in range(6)])
    buf = torch.from_numpy(np.concatenate([host[:1], host]).view(np.int64)).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    want = oracle_clean_hist(orc, orc.cfg(N, T, CS), host)

    def tables():
        return (torch.full((4096,), 7, dtype=torch.int64, device="cuda"),
                torch.full((4096,), 7, dtype=torch.int64, device="cuda"))

    def as_hist(k, n):
        return P.hist_from_tables(k.cpu().numpy().view(np.uint64), n.cpu().numpy().view(np.uint64))

    with P.Context(c) as ctx, P.Context(c) as ref_ctx:
        rk, rn = tables()
        ref_ctx.sampled_hist(buf.data_ptr() + 8, total, stream)
        ref_ctx.export_reset(rk.data_ptr(), rn.data_ptr(), 4096, stream)
        for off in (1, 0):  # 16-byte aligned list, then 8-byte aligned (peeled head)
            for _ in range(2):
                k, n = tables()
                cnt = total if off else total + 1
                ctx.sampled_hist_export(buf.data_ptr() + 8 * off, cnt, k.data_ptr(), n.data_ptr(), 4096, stream)
                torch.cuda.synchronize()
                if off:
                    assert torch.equal(k, rk) and torch.equal(n, rn)
                    assert as_hist(k, n).bins == want
                else:
                    assert as_hist(k, n).total() == total + 1
        assert ctx.fetch().bins == {}
        k, n = tables()  # an output table that is only 8-byte aligned
        ctx.sampled_hist_export(buf.data_ptr() + 8, total, k.data_ptr() + 8, n.data_ptr() + 8, 4095, stream)
        torch.cuda.synchronize()
        assert torch.equal(k[1:], rk[:4095]) and torch.equal(n[1:], rn[:4095]) and int(k[0]) == 7
        k, n = tables()
        ctx.sampled_hist_export(buf.data_ptr(), 0, k.data_ptr(), n.data_ptr(), 4096, stream)
        torch.cuda.synchronize()
        assert (k.cpu().numpy().view(np.uint64) == np.uint64(2 ** 64 - 1)).all() and (n.cpu() == 0).all()
        # a table smaller than the histogram: flagged, the next fetch reports it
        k, n = tables()
        ctx.sampled_hist_export(buf.data_ptr() + 8, total, k.data_ptr(), n.data_ptr(), 2, stream)
        with pytest.raises(P.PlussError):
            ctx.fetch()
        assert (k[2:].cpu() == 7).all()  # nothing written past `cap`
        ctx.reset(stream)
        if N % (CS * T):
            return  # faithful mode needs N % (chunk*threads) == 0
        # faithful counts already in the handle: the two-launch path folds them in
        fa = P.expand_samples(c, 0x5EED0003, "B0", 0, 5000)
        fbuf = torch.from_numpy(fa.view(np.int64)).cuda()
        for x in (ctx, ref_ctx):
            x.reset(stream)
            x.faithful_hist("B0", fbuf.data_ptr(), len(fa), stream)
        ref_ctx.sampled_hist(buf.data_ptr() + 8, total, stream)
        ref_ctx.export_reset(rk.data_ptr(), rn.data_ptr(), 4096, stream)
        k, n = tables()
        ctx.sampled_hist_export(buf.data_ptr() + 8, total, k.data_ptr(), n.data_ptr(), 4096, stream)
        torch.cuda.synchronize()
        assert torch.equal(k, rk) and torch.equal(n, rn)
        assert as_hist(k, n).total() == total + sum(P.sampled_hist(cfg(N, T, CS, mode="faithful"), fa).bins.values())
        # and afterwards the one-launch path is used again
        ctx.sampled_hist_export(buf.data_ptr() + 8, total, k.data_ptr(), n.data_ptr(), 4096, stream)
        torch.cuda.synchronize()
        assert as_hist(k, n).bins == want


@pytest.mark.parametrize("N,T,CS", [(256, 4, 4), (96, 3, 3), (96, 4, 4), (128, 3, 3)],
                         ids=["p2_np2", "fast", "p2", "np2"])
def test_dense_pass(orc, N, T, CS):
    """pluss_dev_sampled_hist_dense (one launch, dense (ref, case) counts) ==
    the oracle, pass after pass (the in-kernel state is left zeroed), over
    grids of 1..1024 workgroups (pluss_diag_dense's cap: 1..64 bin rows,
    uneven rows), unaligned and odd-length lists, an empty list, malformed
    samples; and it leaves the handle's accumulating histogram alone."""
    torch = pytest.importorskip("torch")
    c = cfg(N, T, CS)
    counts = P.default_counts(N, 400000)  # 391 workgroups by default: 64 rows of 6-7
    host = np.concatenate([P.expand_samples(c, 0x5EED0004, r, 0, counts[r]) for r in range(6)])
    total = len(host)
    buf = torch.from_numpy(np.concatenate([host[:1], host]).view(np.int64)).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    want = closed_form_hist(N, T, CS, host)
    sub = host[::97]  # the closed forms against the stepping oracle on a subsample
    assert closed_form_hist(N, T, CS, sub) == oracle_clean_hist(orc, orc.cfg(N, T, CS), sub)

    def out():
        return torch.full((P.DENSE_BINS + 2,), 7, dtype=torch.int64, device="cuda")

    def run(ctx, ptr, n, grid=None):
        d = out()
        if grid is None:
            ctx.sampled_hist_dense(ptr, n, d.data_ptr(), stream)
        else:
            ctx.diag_dense(ptr, n, d.data_ptr(), 0, grid, stream)
        torch.cuda.synchronize()
        v = d.cpu().numpy()
        assert v[P.DENSE_BINS + 1] == 7  # nothing written past the vector
        return v

    with P.Context(c) as ctx:
        ctx.reset(stream)
        ctx.sampled_hist(buf.data_ptr() + 8, 1000, stream)  # accumulating histogram: untouched by dense passes
        first = None
        for grid in (None, 1, 3, 64, 65, 200, 391):
            for _ in range(2):
                v = run(ctx, buf.data_ptr() + 8, total, grid)
                assert v[P.DENSE_BINS] == 0
                assert P.hist_from_dense(c, v).bins == want, grid
                first = v if first is None else first
                assert (v == first).all()
        v = run(ctx, buf.data_ptr(), total + 1)  # 8-byte aligned (peeled head), odd length
        assert P.hist_from_dense(c, v).total() == total + 1
        for n in (0, 1, 2, 3):
            v = run(ctx, buf.data_ptr() + 8, n)
            assert P.hist_from_dense(c, v).bins == oracle_clean_hist(orc, orc.cfg(N, T, CS), host[:n])
        assert (run(ctx, buf.data_ptr() + 8, 0)[:P.DENSE_BINS + 1] == 0).all()
        assert ctx.fetch().bins == oracle_clean_hist(orc, orc.cfg(N, T, CS), host[:1000])
        bad = torch.from_numpy(np.array([P.pack("C3", 1, 2, 3), P.pack("A0", N, 0, 0), 7 << 60, 0], np.uint64)
                               .view(np.int64)).cuda()
        v = run(ctx, bad.data_ptr(), 4)
        assert v[P.DENSE_BINS] == 2 and v[:P.DENSE_BINS].sum() == 2
        with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
            ctx.fetch()
        ctx.reset(stream)
        assert (run(ctx, buf.data_ptr() + 8, total) == first).all()  # healthy after the error
    with P.Context(cfg(100, 3, 5)) as g:
        with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
            g.sampled_hist_dense(buf.data_ptr(), 10, out().data_ptr(), stream)


@pytest.mark.parametrize("N,T,CS", [(128, 4, 4), (96, 3, 3)], ids=["p2_np2", "fast"])
def test_shuffled_mixed_reference_lists(orc, N, T, CS):
    """Lists whose waves hold every reference at once (the per-reference loop of
    k_count's slot counting) and malformed samples among them: accumulate,
    fused export and dense passes all equal the oracle."""
    torch = pytest.importorskip("torch")
    c = cfg(N, T, CS)
    counts = P.default_counts(N, 30000)
    host = np.concatenate([P.expand_samples(c, 0x5EED0005, r, 0, counts[r]) for r in range(6)])
    rng = np.random.default_rng(7)
    host = host[rng.permutation(len(host))]
    want = oracle_clean_hist(orc, orc.cfg(N, T, CS), host)
    stream = torch.cuda.current_stream().cuda_stream
    buf = torch.from_numpy(host.view(np.int64)).cuda()
    d = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device="cuda")
    with P.Context(c) as ctx:
        ctx.sampled_hist(buf.data_ptr(), len(host), stream)
        assert ctx.fetch().bins == want
        ctx.sampled_hist_dense(buf.data_ptr(), len(host), d.data_ptr(), stream)
        torch.cuda.synchronize()
        assert P.hist_from_dense(c, d.cpu().numpy()).bins == want
        # malformed samples scattered through the list: counted apart, flagged
        bad = np.array([7 << 60, 6 << 60 | 1, P.pack("B0", N, 0, 0), P.pack("C3", 0, N + 3, 0), P.pack("A0", 0, 0, N)],
                       np.uint64)
        mixed = np.insert(host, rng.integers(0, len(host), len(bad)), bad)
        mb = torch.from_numpy(mixed.view(np.int64)).cuda()
        ctx.reset(stream)
        ctx.sampled_hist_dense(mb.data_ptr(), len(mixed), d.data_ptr(), stream)
        torch.cuda.synchronize()
        v = d.cpu().numpy()
        assert v[P.DENSE_BINS] == len(bad)
        assert P.hist_from_dense(c, v).bins == want
        ctx.sampled_hist(mb.data_ptr(), len(mixed), stream)
        with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
            ctx.fetch()


def test_dense_pass_config2_full_size():
    """BASELINE config 2 (N=1024, T=8, 2^24 samples): the bench's step output
    equals the closed-form histogram of the list."""
    torch = pytest.importorskip("torch")
    N, T = 1024, 8
    c = cfg(N, T)
    counts = P.default_counts(N, 1 << 24)
    buf = torch.empty(1 << 24, dtype=torch.int64, device="cuda")
    d = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with P.Context(c) as ctx:
        off = 0
        for r in range(6):
            ctx.expand(0x5EED0001, r, 0, counts[r], buf.data_ptr() + 8 * off, stream)
            off += counts[r]
        for _ in range(3):
            ctx.sampled_hist_dense(buf.data_ptr(), 1 << 24, d.data_ptr(), stream)
        torch.cuda.synchronize()
    v = d.cpu().numpy()
    assert v[P.DENSE_BINS] == 0
    assert P.hist_from_dense(c, v).bins == closed_form_hist(N, T, 4, buf.cpu().numpy().view(np.uint64))


def test_long_windows_config4_t64(orc):
    """BASELINE config 4 shape (N=2048, T=64): long B reuse windows, share split and
    cold B samples in a thread's last row, checked against the closed forms."""
    N, T = 2048, 64
    c = cfg(N, T)
    s = P.expand_samples(c, 0x5EED0001, "B0", 0, 400000)
    # add cold candidates: c1 % 8 == 7 in each thread's last row
    last_rows = np.array([N - 1 - k for k in range(0, N, 4)][:32])
    extra = np.array([P.pack("B0", r, 8 * j + 7, j) for j, r in enumerate(last_rows)], np.uint64)
    s = np.unique(np.concatenate([s, extra]))
    h = P.sampled_hist(c, s)
    refs, c0, c1, c2 = P.unpack_array(s)
    ri = closed_form_ri(N, T, 4, 8, refs, c0, c1, c2)
    assert h.cold("B0") == int((ri == -1).sum()) > 0
    assert set(h.share("B0")) == {(N - 7) * (4 * N + 2)}
    assert h.share("B0")[(N - 7) * (4 * N + 2)] == int((ri == (N - 7) * (4 * N + 2)).sum())
    assert h.noshare("B0")[4 * N + 2] == int((ri == 4 * N + 2).sum())


def _dist_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    import pluss_sampler_optimization_amd as P2
    from pluss_sampler_optimization_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = P2.SamplerConfig(n=512, threads=4)
    counts = P2.default_counts(512, 1 << 20)
    h = D.sharded_clean_hist(cfg, 0x5EED0001, counts)
    hd = D.sharded_clean_dense(cfg, 0x5EED0001, counts)
    q.put((rank, h.bins, hd.bins))
    dist.destroy_process_group()


def test_sharded_two_ranks_on_one_gpu_equals_single_rank():
    """The sharded path (2 processes, each expanding and histogramming its slice
    on cuda:0; canonical tables all-gathered, or dense vectors all-reduced,
    over gloo) equals one process over the whole list."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = cfg_ = P.SamplerConfig(n=512, threads=4)
    counts = P.default_counts(512, 1 << 20)
    whole = np.concatenate([P.expand_samples(cfg_, 0x5EED0001, r, 0, c) for r, c in enumerate(counts)])
    want = P.sampled_hist(cfg, whole).bins
    for _, bins, dbins in res:
        assert bins == want
        assert dbins == want


KEY_EMPTY = (1 << 64) - 1


def _select_shards(ctxs, bounds, t, totals, stream):
    """The pluss_dev_faithful_shards_* phases over several handles in one
    process, each keeping its key range [bounds[i], bounds[i+1]) of the whole
    arbitrary-order lists (the six references back to back in t); the rows are
    gathered by device copies (conftest.gpu_lockstep)."""
    from conftest import gpu_lockstep
    return gpu_lockstep(ctxs, [lambda ctx, row, i=i: ctx.faithful_shards_select(t.data_ptr(), totals, bounds[i],
                                                                                 bounds[i + 1], row, stream)
                               for i in range(len(ctxs))], stream, selected=True)


def _merged(ctxs):
    bins, trav = {}, [0] * 6
    for ctx in ctxs:
        h = ctx.fetch()
        for k, v in h.bins.items():
            bins[k] = bins.get(k, 0) + v
        trav = [(a + b) % (1 << 64) for a, b in zip(trav, h.traversed)]
    return bins, trav


@pytest.mark.parametrize("name,d,smp", GOLD[:4], ids=[g[0] for g in GOLD[:4]])
def test_faithful_key_range_shards_equal_reference_dumps(orc, name, d, smp):
    """Faithful mode split over 3 key-range shards (3 handles on one GPU, one of
    them covering no key) reproduces the reference's r10 dumps."""
    torch = pytest.importorskip("torch")
    N, T = d["N"], d["T"]
    c = cfg(N, T, mode="faithful")
    ks = P.faithful_key_space(c)
    bounds = [0, ks // 3, ks // 3, ks]  # shard 1 is empty
    stream = torch.cuda.current_stream().cuda_stream
    lists = [orc.pack_array(ref, smp[ref]) for ref in orc.REFS]
    totals = [len(x) for x in lists]
    t = torch.from_numpy(np.concatenate(lists).astype(np.uint64).view(np.int64)).cuda()
    ctxs = [P.Context(c) for _ in range(3)]
    try:
        for x in ctxs:
            x.reset(stream)
        rows = _select_shards(ctxs, bounds, t, totals, stream).cpu().numpy()
        assert not rows[1, :6].any()  # the empty shard kept nothing
        bins, trav = _merged(ctxs)
    finally:
        for x in ctxs:
            x.close()
    for ref in orc.REFS:
        exp, etrav = expected_raw(d, ref)
        assert {k: v for k, v in bins.items() if k[0] == ref} == exp, (name, ref)
        assert trav[P.REF_ID[ref]] == etrav, (name, ref)


@pytest.mark.parametrize("N,T,per,nshards", [(128, 8, 20000, 2), (256, 4, 60000, 5), (64, 2, 30000, 8),
                                             (1024, 8, 5000000, 2)])
def test_faithful_key_range_shards_equal_one_gpu(N, T, per, nshards):
    """Longer lists (many replays, Q1 drops, cold samples): the sharded phases
    over arbitrary-order lists equal one-handle faithful mode exactly,
    traversed included.  The last case gives the 3-D references 1221 tiles
    each (the finish kernel's many-tile path)."""
    torch = pytest.importorskip("torch")
    c = cfg(N, T, mode="faithful")
    ks = P.faithful_key_space(c)
    bounds = [ks * i // nshards for i in range(nshards + 1)]
    stream = torch.cuda.current_stream().cuda_stream
    lists = [P.expand_samples(c, 0x5EED0000 + N, r, 0, per if r >= 2 else min(per, (N - 1) ** 2)) for r in range(6)]
    totals = [len(x) for x in lists]
    t = torch.from_numpy(np.concatenate(lists).view(np.int64)).cuda()
    ctxs = [P.Context(c) for _ in range(nshards)]
    one = P.Context(c)
    try:
        for x in ctxs + [one]:
            x.reset(stream)
        _select_shards(ctxs, bounds, t, totals, stream)
        one.faithful_hist_refs(t.data_ptr(), totals, stream)
        bins, trav = _merged(ctxs)
        h = one.fetch()
    finally:
        for x in ctxs + [one]:
            x.close()
    assert bins == h.bins
    assert trav == h.traversed


def test_faithful_shard_phase_order_is_enforced():
    """Phases out of order, a one-GPU faithful call between phases, or rows
    that do not cover the shard are configuration errors (a
    half-finished shard pass can never leak into a later pass)."""
    torch = pytest.importorskip("torch")
    c = cfg(64, 4, mode="faithful")
    stream = torch.cuda.current_stream().cuda_stream
    rows = torch.zeros(2 * P.SHARD_ROW, dtype=torch.int64, device="cuda")
    row = rows.data_ptr()
    with P.Context(c) as ctx:
        with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
            ctx.faithful_shards_carry(row, 0, 2, row, stream)
        with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
            ctx.faithful_shards_hist(row, 0, 2, stream)
        totals = [0, 0, 0, 0, 100, 0]
        ctx.faithful_shards_local(None, 1, totals, [0] * 6, totals, row, stream)
        with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
            ctx.faithful_shards_carry(row, 2, 2, row, stream)  # shard out of range
        ctx.gen_faithful_refs(1, totals, stream)  # a one-GPU pass ends the shard pass
        with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
            ctx.faithful_shards_carry(row, 0, 2, row, stream)
        # a re-issued local phase restarts cleanly: twice, then the whole pass == one GPU
        ctx.reset(stream)
        for _ in range(2):
            ctx.faithful_shards_local(None, 1, totals, [0] * 6, totals, rows[0:P.SHARD_ROW].data_ptr(), stream)
        rows[P.SHARD_ROW:] = 0
        rows[P.SHARD_ROW + 18:P.SHARD_ROW + 24] = torch.tensor(totals, dtype=torch.int64, device="cuda")
        for name in ("carry", "cut"):
            getattr(ctx, "faithful_shards_" + name)(rows.data_ptr(), 0, 2, rows.data_ptr(), stream)
        ctx.faithful_shards_hist(rows.data_ptr(), 0, 2, stream)
        got = ctx.fetch()
        ctx.reset(stream)
        ctx.gen_faithful_refs(1, totals, stream)
        assert got.bins == ctx.fetch().bins
    with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
        P.faithful_key_space(cfg(60, 4, mode="faithful"))


def test_failed_shard_row_fails_every_shard():
    """A row carrying the error word makes the other shards' passes record
    nothing and fail at their fetch with PLUSS_ERR_PEER (no shard waits)."""
    torch = pytest.importorskip("torch")
    c = cfg(64, 4, mode="faithful")
    stream = torch.cuda.current_stream().cuda_stream
    totals = [50, 50, 300, 300, 300, 300]
    rows = torch.zeros(2 * P.SHARD_ROW, dtype=torch.int64, device="cuda")
    with P.Context(c) as ctx:
        ctx.reset(stream)
        ctx.faithful_shards_local(None, 3, totals, [0] * 6, totals, rows.data_ptr(), stream)
        rows[P.SHARD_ROW + P.SHARD_ROW_ERR] = 1  # shard 1 failed
        for name in ("carry", "cut"):
            getattr(ctx, "faithful_shards_" + name)(rows.data_ptr(), 0, 2, rows.data_ptr(), stream)
        ctx.faithful_shards_hist(rows.data_ptr(), 0, 2, stream)
        with pytest.raises(P.PlussError, match="PLUSS_ERR_PEER"):
            ctx.fetch()


def _faith_dist_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    import pluss_sampler_optimization_amd as P2
    from pluss_sampler_optimization_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = P2.SamplerConfig(n=256, threads=8, mode="faithful")
    counts = P2.default_counts(256, 1 << 18)
    lists = {r: torch.from_numpy(P2.expand_samples(c, 0x5EED0001, r, 0, n).view("int64")).cuda()
             for r, n in enumerate(counts)}
    h = D.sharded_faithful_hist(c, lists)
    q.put((rank, h.bins, h.traversed))
    dist.destroy_process_group()


def test_sharded_faithful_two_ranks_on_one_gpu():
    """dist.sharded_faithful_hist end to end: 2 processes on cuda:0, summaries and
    tables exchanged over gloo, equals one process over the same lists."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_faith_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = P.SamplerConfig(n=256, threads=8, mode="faithful")
    counts = P.default_counts(256, 1 << 18)
    whole = np.concatenate([P.expand_samples(c, 0x5EED0001, r, 0, n) for r, n in enumerate(counts)])
    want = P.sampled_hist(c, whole)
    for _, bins, trav in res:
        assert bins == want.bins
        assert trav == want.traversed


CLI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pluss_sampler_optimization_amd",
                   "lib", "pluss_cli")


def test_cli_acc_matches_reference_seq_printout():
    """`pluss_cli acc` (full trace on the GPU + host CRI/AET) prints what the
    reference seq binary printed in `acc` mode, line for line after the timer."""
    import subprocess
    from conftest import GOLDEN
    out = subprocess.run([CLI, "acc", "--n", "128", "--threads", "4"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    want = open(os.path.join(GOLDEN, "seq_N128_T4_acc.txt")).read().splitlines()[1:]
    assert out.stdout.splitlines()[1:] == want


@pytest.mark.parametrize("name,d,smp", GOLD[:3], ids=[g[0] for g in GOLD[:3]])
def test_cli_replay_matches_reference_r10_printout(tmp_path, orc, name, d, smp):
    """`pluss_cli replay` on the reference's own sample list reproduces its printed
    per-reference CRI histograms, reuse histogram, MRC and max traversed."""
    import subprocess
    f = tmp_path / "samples.txt"
    with open(f, "w") as fh:
        for ref in orc.REFS:
            for row in smp[ref]:
                fh.write(f"SAMPLE {ref} {row[0]} {row[1]} {row[2]}\n")
    out = subprocess.run([CLI, "replay", str(f), "--n", str(d["N"]), "--threads", str(d["T"])],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()[1:]
    sections, cur = {}, None
    for line in lines:
        if line in ("C3", "C2", "A0", "C0", "B0", "C1", "Start to dump reuse time", "miss ratio",
                    "max iteration traversed"):
            cur = sections.setdefault(line, [])
        elif cur is not None:
            cur.append(line)
    rows = lambda ls: [[float(x) for x in l.split(",")] for l in ls]  # noqa: E731
    for ref in ("C3", "C2", "A0", "C0", "B0", "C1"):
        assert rows(sections[ref]) == d["printed"]["per_ref"][ref], ref
    assert rows(sections["Start to dump reuse time"]) == d["printed"]["reuse"]
    assert rows(sections["miss ratio"]) == d["printed"]["mrc"]
    assert int(sections["max iteration traversed"][0]) == d["printed"]["max_traversed"]


def _faithful_refs_vs_calls(c, s, counts, stream):
    """(concurrent six-reference call, six single-reference calls) on the same handle."""
    torch = pytest.importorskip("torch")
    t = torch.from_numpy(np.ascontiguousarray(s).view(np.int64)).cuda()
    with P.Context(c) as ctx:
        ctx.reset(stream)
        ctx.faithful_hist_refs(t.data_ptr(), counts, stream)
        h_refs = ctx.fetch()
        ctx.reset(stream)
        off = 0
        for r, n in enumerate(counts):
            if n:
                ctx.faithful_hist(r, t.data_ptr() + 8 * off, n, stream)
            off += n
        h_one = ctx.fetch()
        ctx.reset(stream)
        ctx.faithful_hist_refs(t.data_ptr(), counts, stream)  # again: buffers and streams are reused
        h_again = ctx.fetch()
    return h_refs, h_one, h_again


@pytest.mark.parametrize("name,d,smp", GOLD, ids=[g[0] for g in GOLD])
def test_faithful_refs_concurrent_equals_reference_dumps(orc, name, d, smp):
    """pluss_dev_faithful_hist_refs (the six samplers on their own streams) reproduces r10's dumps."""
    torch = pytest.importorskip("torch")
    s = all_samples(orc, smp)
    counts = [len(smp[ref]) for ref in orc.REFS]
    assert [P.REF_ID[r] for r in orc.REFS] == list(range(6))
    h, h_one, h_again = _faithful_refs_vs_calls(cfg(d["N"], d["T"], mode="faithful"), s, counts,
                                                torch.cuda.current_stream().cuda_stream)
    for ref in orc.REFS:
        exp, etrav = expected_raw(d, ref)
        assert {k: v for k, v in h.bins.items() if k[0] == ref} == exp, (name, ref)
        assert h.traversed[P.REF_ID[ref]] == etrav, (name, ref)
    assert h.bins == h_one.bins == h_again.bins
    assert list(h.traversed) == list(h_one.traversed) == list(h_again.traversed)


@pytest.mark.parametrize("N,T,CS,per", [(128, 4, 4, 6000), (100, 5, 4, 3000), (256, 8, 4, 40000), (64, 2, 4, 0)])
def test_faithful_refs_concurrent_equals_per_reference_calls(N, T, CS, per):
    """Packed-word (N % 8 == 0) and (key, sink) pair (N=100) shapes, longer lists, an empty
    list: the concurrent call equals one faithful_hist call per reference."""
    torch = pytest.importorskip("torch")
    c = cfg(N, T, CS, mode="faithful")
    counts = [min(per, (N - 1) ** 2) if r < 2 else per for r in range(6)]
    if per:
        counts[4] = per // 3  # unequal lengths
    parts = [P.expand_samples(c, 0x5EED0100 + N, r, 0, n) if n else np.zeros(0, np.uint64)
             for r, n in enumerate(counts)]
    s = np.concatenate(parts).astype(np.uint64)
    h, h_one, h_again = _faithful_refs_vs_calls(c, s, counts, torch.cuda.current_stream().cuda_stream)
    assert h.bins == h_one.bins == h_again.bins
    assert list(h.traversed) == list(h_one.traversed) == list(h_again.traversed)
    assert h.total() == h_one.total()


@pytest.mark.parametrize("rank", [0, 7])
def test_dense_pass_config3_shard(rank):
    """BASELINE config 3 (N=4096, T=8, 2^28 samples over 8 GPUs): one rank's slice
    (2^25 samples; rank 7 holds B0's +2 remainder) through the bench's step equals
    the closed-form histogram of that slice, and the eight slices tile the counts."""
    torch = pytest.importorskip("torch")
    N, T, world = 4096, 8, 8
    c = cfg(N, T)
    counts = P.default_counts(N, 1 << 28)
    assert sum(counts) == 1 << 28
    parts = [(cnt * rank // world, cnt * (rank + 1) // world - cnt * rank // world) for cnt in counts]
    assert sum(sum(cnt * (r + 1) // world - cnt * r // world for r in range(world)) for cnt in counts) == 1 << 28
    n = sum(k for _, k in parts)
    buf = torch.empty(n, dtype=torch.int64, device="cuda")
    d = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with P.Context(c) as ctx:
        off = 0
        for r, (lo, k) in enumerate(parts):
            ctx.expand(0x5EED0001, r, lo, k, buf.data_ptr() + 8 * off, stream)
            off += k
        for _ in range(2):
            ctx.sampled_hist_dense(buf.data_ptr(), n, d.data_ptr(), stream)
        torch.cuda.synchronize()
    v = d.cpu().numpy()
    assert v[P.DENSE_BINS] == 0
    h = P.hist_from_dense(c, v)
    assert h.total() == n
    assert h.bins == closed_form_hist(N, T, 4, buf.cpu().numpy().view(np.uint64))


def test_faithful_n4096_concurrent_equals_serial():
    """Faithful mode at the config-3 shape (N=4096: 64-bit packed words), 2^20 samples
    per 3-D reference: the six-stream call equals six calls."""
    torch = pytest.importorskip("torch")
    N, T = 4096, 8
    c = cfg(N, T, mode="faithful")
    counts = [20000, 20000, 1 << 20, 1 << 20, 1 << 20, 1 << 20]
    s = np.concatenate([P.expand_samples(c, 0x5EED0001, r, 0, k) for r, k in enumerate(counts)]).astype(np.uint64)
    h, h_one, h_again = _faithful_refs_vs_calls(c, s, counts, torch.cuda.current_stream().cuda_stream)
    assert h.bins == h_one.bins == h_again.bins
    assert list(h.traversed) == list(h_one.traversed) == list(h_again.traversed)
    assert 0 < h.total() - sum(h.cold(r) for r in P.REFS) <= sum(counts)


_ENV_PROBE = r'''
import json, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import pluss_sampler_optimization_amd as P
c = P.SamplerConfig(n=256, threads=4)
counts = P.default_counts(256, 300000)
s = np.concatenate([P.expand_samples(c, 0x5EED0006, r, 0, counts[r]) for r in range(6)])
t = torch.from_numpy(s.view(np.int64)).cuda()
d = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device="cuda")
with P.Context(c) as ctx:
    ctx.sampled_hist_dense(t.data_ptr(), len(s), d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
out = {"dense": d.cpu().tolist(),
       "hist": sorted([list(k) + [v] for k, v in P.sampled_hist(c, s).bins.items()]),
       "faithful": sorted([list(k) + [v] for k, v in
                           P.sampled_hist(P.SamplerConfig(n=256, threads=4, mode="faithful"), s).bins.items()]),
       "full": sorted([list(k) + [v] for k, v in P.fulltrace_hist(c).bins.items()])}
print(json.dumps(out))
'''


def test_environment_cannot_change_results(tmp_path):
    """The product entry points read no environment variable: the round-1
    diagnostic knobs (ablation, grid, legacy kernels, bucket path ...) set in
    the environment change nothing that pluss_dev_* / pluss_gemm_* return."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = tmp_path / "probe.py"
    probe.write_text(_ENV_PROBE)
    knobs = {"PLUSS_ABLATE": "3", "PLUSS_GRID": "1", "PLUSS_LEGACY": "1", "PLUSS_LANES": "0", "PLUSS_DROWS": "1",
             "PLUSS_BS": "1024", "PLUSS_FAITH_BUCKET": "1", "PLUSS_AUX": "3", "PLUSS_PREF": "2", "PLUSS_NT": "0",
             "PLUSS_UNROLL": "4", "PLUSS_PCS": "4", "PLUSS_FB_ABL": "1"}
    runs = []
    for extra in ({}, knobs):
        env = {k: v for k, v in os.environ.items() if not k.startswith("PLUSS_")}
        env.update(extra)
        r = subprocess.run([sys.executable, str(probe), root], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert runs[0] == runs[1]
    assert sum(runs[0]["dense"][:P.DENSE_BINS]) == 300000


@pytest.mark.parametrize("name,d,smp", GOLD[:2], ids=[g[0] for g in GOLD[:2]])
def test_cli_trace_and_json(tmp_path, orc, name, d, smp):
    """`pluss_cli replay --trace F --json J`: the trace has one line per sample
    whose RI equals the stepping oracle's per-sample replay; the JSON holds the
    same per-reference histograms, reuse histogram and MRC as the printout
    (itself checked against the reference above) and the traversed counts."""
    import json
    import subprocess
    f = tmp_path / "samples.txt"
    rows = []
    with open(f, "w") as fh:
        for ref in orc.REFS:
            for row in smp[ref]:
                fh.write(f"SAMPLE {ref} {row[0]} {row[1]} {row[2]}\n")
                rows.append((ref, int(row[0]), int(row[1]), int(row[2])))
    tr, js = tmp_path / "trace.txt", tmp_path / "out.json"
    out = subprocess.run([CLI, "replay", str(f), "--n", str(d["N"]), "--threads", str(d["T"]), "--trace", str(tr),
                          "--json", str(js)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    j = json.load(open(js))
    assert j["mode"] == "replay" and j["n"] == d["N"] and j["threads"] == d["T"]
    def same(got, printed):  # printed rows: key, value (6 significant digits), fraction
        assert [k for k, _ in got] == [r[0] for r in printed]
        assert np.allclose([v for _, v in got], [r[1] for r in printed], rtol=5e-6, atol=0)

    for ref in ("C3", "C2", "A0", "C0", "B0", "C1"):
        same(j["histograms"][ref], d["printed"]["per_ref"][ref])
    same(j["histograms"]["reuse"], d["printed"]["reuse"])
    mrc = dict((k, v) for k, v in j["mrc"])  # every printed (plateau-compressed) MRC row is in the JSON curve
    for c, mr in d["printed"]["mrc"]:
        assert c in mrc and abs(mrc[c] - mr) <= 5e-6 * max(abs(mr), 1e-6), (c, mr)
    assert max(j["traversed"]) == d["printed"]["max_traversed"]
    assert j["sampler"].startswith("faithful")
    text = open(tr).read().splitlines()
    assert text[0].startswith("# ref c0 c1 c2 ri sink_key")  # faithful run: the header says what the RIs are
    lines = [l.split() for l in text if not l.startswith("#")]
    assert [(l[0], int(l[1]), int(l[2]), int(l[3])) for l in lines] == rows
    packed = np.array([P.pack(r, a, b, c) for r, a, b, c in rows], dtype=np.uint64)
    want = orc.clean_ri(orc.cfg(d["N"], d["T"]), packed)
    assert [int(l[4]) for l in lines] == want.tolist()


def _faith_gen_dist_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    import pluss_sampler_optimization_amd as P2
    from pluss_sampler_optimization_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = P2.SamplerConfig(n=512, threads=8, mode="faithful")
    h = D.sharded_faithful_gen_hist(c, 0x5EED0001, P2.default_counts(512, 1 << 20))
    q.put((rank, h.bins, h.traversed))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_faithful_generated_lists_on_one_gpu(world):
    """dist.sharded_faithful_gen_hist: each rank generates only the slice of the
    key-order lists inside its key range (no rank holds a whole list), the
    four-phase shard protocol over gloo; equals one GPU's gen_faithful_refs."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_faith_gen_dist_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = P.SamplerConfig(n=512, threads=8, mode="faithful")
    with P.Context(c) as one:
        one.gen_faithful_refs(0x5EED0001, P.default_counts(512, 1 << 20))
        want = one.fetch()
    for _, bins, trav in res:
        assert bins == want.bins
        assert list(trav) == list(want.traversed)


def _random_shapes(seed, k):
    """k random GEMM shapes (fixed seed): N, T, CS, DS, CLS with CLS a multiple
    of DS; faithful ones also with N % (CS*T) == 0."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < k:
        T = int(rng.choice([1, 2, 3, 4, 5, 8, 16]))
        CS = int(rng.choice([1, 2, 3, 4, 8]))
        DS = int(rng.choice([4, 8]))
        CLS = DS * int(rng.choice([1, 2, 4, 8, 16]))
        N = int(rng.integers(8, 200))
        if len(out) % 2:  # every other shape in r10's lockstep order (faithful mode too)
            N = CS * T * max(1, N // (CS * T))
        if N // (CS * T) < 1 or N < 8:
            continue
        out.append((N, T, CS, DS, CLS))
    return out


RANDOM_SHAPES = _random_shapes(20261017, 24)


@pytest.mark.parametrize("shape", RANDOM_SHAPES, ids=[str(s) for s in RANDOM_SHAPES])
def test_random_shapes_clean_and_faithful_equal_oracle(orc, shape):
    """A fixed-seed sweep of random shapes (any N, T, CS, DS, CLS; lines that
    span rows; N % (CS*T) != 0): clean mode == the stepping oracle's per-sample
    replay histogram; where N % (CS*T) == 0 (r10's lockstep order), faithful
    mode == the oracle's r10 sampler on the same lists, with traversed."""
    N, T, CS, DS, CLS = shape
    c = cfg(N, T, CS, DS, CLS)
    span = N - 1
    per = [min(800, span ** (2 if r < 2 else 3)) for r in range(6)]
    s = np.concatenate([P.expand_samples(c, 0x5EED0100 + N, r, 0, n) for r, n in enumerate(per) if n > 0])
    oc = orc.cfg(N, T, CS, DS, CLS)
    assert P.sampled_hist(c, s).bins == oracle_clean_hist(orc, oc, s)
    if N % (CS * T) == 0:
        cf = cfg(N, T, CS, DS, CLS, mode="faithful")
        h = P.sampled_hist(cf, s)
        for ref in orc.REFS:
            part = s[(s >> np.uint64(60)) == np.uint64(P.REF_ID[ref])]
            want, trav = orc.faithful(oc, ref, part)
            assert {k: v for k, v in h.bins.items() if k[0] == ref} == want, (shape, ref)
            assert h.traversed[P.REF_ID[ref]] == trav, (shape, ref)


@pytest.mark.parametrize("N,T", [(104, 2), (264, 2)])
def test_pair_sort_shapes_vs_oracle(orc, N, T):
    """Shapes with N % (CLS/DS) != 0 (DS=4: lines of 16 elements) take the
    (key, sink) pair path, sorted by the hand-written LSD pair sort (no
    library sort left): tens of thousands of samples per reference in any
    order (several blocks per pass; 3 passes at N=104, 4 at N=264, so both
    buffer parities end in place), through the six-reference and the
    one-reference entry points == the stepping r10 oracle."""
    c = cfg(N, T, 4, 4, 64, mode="faithful")
    span = N - 1
    per = [min(6000, span * span), min(6000, span * span), 40000, 3000, 40000, 40000]
    lists = [P.expand_samples(c, 0x5EED0200 + N, r, 0, n) for r, n in enumerate(per)]
    s = np.concatenate(lists)
    h = P.sampled_hist(c, s)
    oc = orc.cfg(N, T, 4, 4, 64)
    for r, ref in enumerate(P.REFS):
        want, trav = orc.faithful(oc, ref, lists[r])
        assert {k: v for k, v in h.bins.items() if k[0] == ref} == want, (N, ref)
        assert h.traversed[r] == trav, (N, ref)
    one = P.sampled_hist(c, lists[4])  # (one reference)
    assert {k: v for k, v in one.bins.items() if k[0] == "C2"} == {k: v for k, v in h.bins.items() if k[0] == "C2"}
