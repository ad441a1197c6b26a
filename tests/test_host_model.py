"""CPU checks of the product's integer model and host logic (no GPU).

The device kernels evaluate pluss_model.h; here the same header is compiled
for the host (tests/helpers/model_host.cpp) and compared with the stepping
oracle, so the reuse rules are exercised on irregular shapes before any GPU
run.  Also: the faithful-mode sort/scan formulation on the reference dumps,
the C-ABI exports, and the sample-count rule.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, closed_form_ri, expected_raw, golden_configs

SHAPES = [(16, 2, 4, 8, 64), (24, 3, 2, 8, 64), (12, 5, 1, 8, 64), (10, 1, 3, 8, 64), (5, 2, 1, 8, 64),
          (3, 1, 1, 8, 64), (32, 4, 4, 8, 64), (20, 2, 3, 4, 64), (18, 3, 2, 8, 32), (7, 2, 2, 8, 8),
          (64, 4, 4, 8, 64), (100, 3, 5, 8, 64), (9, 4, 2, 16, 64), (1, 1, 1, 8, 64), (2, 3, 1, 8, 64)]


def edge_samples(orc, N, cnt, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for r in range(6):
        c0 = rng.integers(0, N, cnt); c1 = rng.integers(0, N, cnt)
        c2 = rng.integers(0, N, cnt) if r >= 2 else np.zeros(cnt, np.int64)
        c1[: cnt // 8] = N - 1
        if r >= 2:
            c2[cnt // 8: cnt // 4] = N - 1
        c0[cnt // 4: cnt // 3] = N - 1
        out.append(orc.pack_array(r, np.stack([c0, c1, c2], 1)))
    return np.concatenate(out)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_model_rules_match_stepping_oracle(orc, model_host, shape):
    N, T, CS, DS, CLS = shape
    s = edge_samples(orc, N, 64, seed=N * 31 + T)
    want = orc.clean_ri(orc.cfg(N, T, CS, DS, CLS), s)
    gen, _, _ = model_host.ri(N, T, CS, DS, CLS, s, 0)
    np.testing.assert_array_equal(gen, want)
    if N % (CLS // DS) == 0:
        fast, _, _ = model_host.ri(N, T, CS, DS, CLS, s, 1)
        np.testing.assert_array_equal(fast, want)


def test_fast_rules_equal_closed_forms_large(orc, model_host):
    N, T, CS = 1024, 8, 4
    s = edge_samples(orc, N, 5000, seed=7)
    refs = (s >> np.uint64(60)).astype(np.int64)
    c0 = ((s >> np.uint64(40)) & np.uint64(0xFFFFF)).astype(np.int64)
    c1 = ((s >> np.uint64(20)) & np.uint64(0xFFFFF)).astype(np.int64)
    c2 = (s & np.uint64(0xFFFFF)).astype(np.int64)
    fast, kind, _ = model_host.ri(N, T, CS, 8, 64, s, 1)
    np.testing.assert_array_equal(fast, closed_form_ri(N, T, CS, 8, refs, c0, c1, c2))
    share = (refs == 3) & (fast > 0) & (2 * fast > (4 * N + 2) * N)
    np.testing.assert_array_equal(kind.astype(bool), share)


def test_fastdiv_exact(model_host):
    rng = np.random.default_rng(3)
    ds = list(range(1, 70)) + [127, 128, 129, 1000, 4095, 65535, 65536, 1 << 20, (1 << 30) + 7]
    ns = np.concatenate([np.arange(0, 5000), rng.integers(0, (1 << 31) - 1, 3000), [(1 << 31) - 1]])
    for d in ds:
        for n in ns[:: max(1, len(ns) // 800)]:
            assert model_host.lib.mh_fdiv(int(n), d) == int(n) // d, (n, d)


@pytest.mark.parametrize("N,rf", [(20, 0), (21, 1), (128, 0), (1024, 0)])
def test_product_bijection_equals_oracle_spec(orc, model_host, N, rf):
    """The device's sample bijection (pluss_model.h, host build) and the oracle's
    independent implementation produce identical lists."""
    c = orc.cfg(N, 4, range_full=rf)
    span = N if rf else N - 1
    for ref in range(6):
        n = min(3000, span ** (2 if ref < 2 else 3) - 11)
        a = model_host.expand(N, rf, 0x5EED0001, ref, 11, n)
        b = orc.expand(c, 0x5EED0001, ref, 11, n)
        np.testing.assert_array_equal(a, b)
        assert len(np.unique(a)) == n


def _faithful_scan_model(N, T, CS, ref, s, ri):
    """The sort/scan form used by pluss_faithful.hip, in numpy."""
    refi = (s >> np.uint64(60)).astype(np.int64)
    c0 = ((s >> np.uint64(40)) & np.uint64(0xFFFFF)).astype(np.int64)
    c1 = ((s >> np.uint64(20)) & np.uint64(0xFFFFF)).astype(np.int64)
    c2 = (s & np.uint64(0xFFFFF)).astype(np.int64)
    S_, R = 4 * N + 2, N * (4 * N + 2)
    k = c0 // CS; t = k % T; q = (k // T) * CS + c0 % CS
    P = q * R + c1 * S_ + np.where(refi < 2, refi, refi + 4 * c2)
    INF = np.uint64(2 ** 64 - 1)
    key = (P * T + t).astype(np.uint64)
    sink = np.where(ri < 0, INF, ((P + np.maximum(ri, 0)) * T + t).astype(np.uint64))
    o = np.argsort(key, kind="stable")
    key, sink, rio, to = key[o], sink[o], ri[o], t[o]
    n = len(key)
    pmax = np.maximum.accumulate(sink)
    start = np.ones(n, bool)
    start[1:] = key[1:] > pmax[:-1]
    nst = np.cumsum(start)
    j = np.arange(n)
    cand = start & (j > 0) & ((j - (nst - 1)) >= n - j)
    cut = int(j[cand].min()) if cand.any() else n
    thr = (4 * N + 2) * N
    hist = {}
    for x in range(cut):
        r = int(rio[x])
        if r >= 0:
            kk = 1 if (ref == "B0" and 2 * r > thr) else 0
            hist[(ref, kk, r)] = hist.get((ref, kk, r), 0) + 1
    cold = int(((rio[:cut] < 0) & (to[:cut] == 0)).sum())
    if cut == n and pmax[n - 1] != INF and int(pmax[n - 1]) % T == 0:
        cold += 1
    hist[(ref, 0, -1)] = cold
    A = (N // T) * R
    trav = 0
    for x in range(cut):
        if start[x]:
            trav -= int(key[x])
        if x == cut - 1 or start[x + 1]:
            trav += A * T if pmax[x] == INF else int(pmax[x])
    return hist, trav


GOLD = golden_configs()


@pytest.mark.parametrize("name,d,smp", GOLD, ids=[g[0] for g in GOLD])
def test_faithful_scan_formulation_matches_reference(orc, model_host, name, d, smp):
    N, T = d["N"], d["T"]
    for ref in orc.REFS:
        s = orc.pack_array(ref, smp[ref])
        ri, _, _ = model_host.ri(N, T, 4, 8, 64, s, 1)
        h, trav = _faithful_scan_model(N, T, 4, ref, s, ri)
        exp, etrav = expected_raw(d, ref)
        assert h == exp, (name, ref)
        assert trav == etrav, (name, ref)


def test_capi_library_exports_every_header_symbol():
    """libpluss_gpu.so loads without a GPU and exports what include/pluss_gpu.h declares."""
    from pluss_sampler_optimization_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "pluss_gpu.h")).read()
    declared = set(re.findall(r"\b(pluss_[a-z_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS)
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(L, name), name
    _lib.lib()  # argtypes binding succeeds


def test_default_counts_match_survey_configs():
    """SURVEY.md §8d / BASELINE.md §3 sample budgets (host-only function)."""
    from pluss_sampler_optimization_amd import default_counts
    assert default_counts(1024, 1 << 24) == [10466, 10466, 4189071, 4189071, 4189071, 4189071]
    assert default_counts(4096, 1 << 28) == [167691, 167691, 67025018, 67025020, 67025018, 67025018]
    assert default_counts(2048, 1 << 24) == [41903, 41903, 4173352, 4173354, 4173352, 4173352]
    c = default_counts(1024, 1 << 24)
    assert sum(c) == 1 << 24


def test_config_errors_are_reported_without_gpu():
    from pluss_sampler_optimization_amd import PlussError, SamplerConfig, default_counts
    with pytest.raises(PlussError):
        default_counts(1, 100)
    with pytest.raises(KeyError):
        SamplerConfig(mode="bogus").to_c()


def test_dense_keys_follow_closed_forms_without_gpu():
    """pluss_dense_keys (host-only): bin ref*3+case holds the closed-form RI of
    that case, B0's long reuse classed share by the r10 threshold."""
    from pluss_sampler_optimization_amd import PlussError, REFS, SamplerConfig, dense_keys
    for N, T in ((1024, 8), (128, 4), (2048, 64)):
        S, W = 4 * N + 2, 8
        want = {("C0", 0): 1, ("C1", 0): 3, ("C2", 0): 1, ("C3", 0): 3, ("C3", 1): 1, ("C3", 2): -1,
                ("A0", 0): 4, ("A0", 1): S - 4 * (W - 1), ("A0", 2): -1,
                ("B0", 0): S, ("B0", 1): N * S - (W - 1) * S, ("B0", 2): -1}
        keys = dense_keys(SamplerConfig(n=N, threads=T))
        assert len(keys) == 18
        for b, k in enumerate(keys):
            ref, case = REFS[b // 3], b % 3
            ri = want.get((ref, case), want.get((ref, 0)))
            kind = 1 if ref == "B0" and ri > 0 and 2 * ri > (4 * N + 2) * N else 0
            assert k == (b // 3) << 60 | kind << 56 | (ri + 2), (N, ref, case)
    with pytest.raises(PlussError, match="PLUSS_ERR_CONFIG"):
        dense_keys(SamplerConfig(n=100, threads=3, chunk=5))  # N % (cls/ds) != 0


KEYGEN_SHAPES = [(128, 4, 4, 0, 2098), (128, 4, 4, 1, 2098), (1024, 8, 4, 0, 4189071), (4096, 8, 4, 0, 67025020),
                 (2048, 64, 4, 0, 4173354), (64, 2, 1, 0, 5000), (16, 1, 4, 0, 100), (32, 4, 2, 0, 1),
                 (4096, 8, 4, 0, 3), (256, 4, 4, 1, 255 ** 3), (256, 4, 4, 0, 255 ** 3)]


@pytest.mark.parametrize("N,T,CS,rf,S", KEYGEN_SHAPES, ids=[str(s) for s in KEYGEN_SHAPES])
def test_key_order_lists_host_model_equals_oracle(orc, model_host, N, T, CS, rf, S):
    """The key-order stratified generator (pluss_model.h keygen_sample, what the
    kernels run) == its independent restatement in the oracle, on slices at the
    start, the block A/B seam and the end; the list is distinct, in range and
    strictly increasing in the faithful sort key (r10's pop order)."""
    import ctypes
    L = model_host.lib
    L.mh_expand_sorted.argtypes = [ctypes.c_int64] * 3 + [ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                          ctypes.POINTER(ctypes.c_uint64)]
    c = orc.cfg(N, T, CS, range_full=rf)
    for ref in range(6):
        span = N if rf else N - 1
        tot = min(S, span ** (3 if ref >= 2 else 2))
        for first, n in {(0, min(tot, 5000)), (max(0, tot - 5000), min(tot, 5000)),
                         (max(0, tot // 2 - 2500), min(tot, 5000))}:
            want = orc.expand_sorted(c, 0x5EED0007, ref, tot, first, n)
            got = np.empty(n, np.uint64)
            assert L.mh_expand_sorted(N, T, CS, rf, 0x5EED0007, ref, tot, first, n,
                                      got.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
            np.testing.assert_array_equal(got, want)
            key = orc.sort_key(N, T, CS, want)
            assert (key[1:] > key[:-1]).all()
            m = np.uint64(0xFFFFF)
            for sh in (40, 20, 0):
                assert (((want >> np.uint64(sh)) & m) < span).all()
            assert ((want >> np.uint64(60)) == ref).all()
    if S <= 300000:  # the whole list: every sample distinct, spread over the whole key range
        tot = min(S, (N if rf else N - 1) ** 3)
        full = orc.expand_sorted(c, 1, "B0", tot, 0, tot)
        assert len(np.unique(full)) == tot


@pytest.mark.parametrize("N,T,CS,rf,S", KEYGEN_SHAPES, ids=[str(s) for s in KEYGEN_SHAPES])
def test_key_order_runs_equal_direct(model_host, N, T, CS, rf, S):
    """The incremental run path (keyrun_*: digits carried along consecutive
    samples, what the fused kernels use) == the direct per-sample decode, for
    runs of 1, 16 and 1000 starting anywhere (block A, the A/B seam, block B)."""
    import ctypes
    L = model_host.lib
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.mh_expand_sorted.argtypes = [ctypes.c_int64] * 3 + [ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p]
    L.mh_expand_sorted_runs.argtypes = L.mh_expand_sorted.argtypes[:-1] + [ctypes.c_uint64, u64p]
    L.mh_expand_sorted_fast.argtypes = L.mh_expand_sorted_runs.argtypes
    fast_seen = set()
    for ref in range(6):
        span = N if rf else N - 1
        tot = min(S, span ** (3 if ref >= 2 else 2))
        for first in sorted({0, max(0, tot // 2 - 3000), max(0, tot - 6000), max(0, tot - tot // (N // T) - 3000)}):
            n = min(6000, tot - first)
            want = np.empty(n, np.uint64)
            L.mh_expand_sorted(N, T, CS, rf, 9, ref, tot, first, n, want.ctypes.data_as(u64p))
            for run in (1, 16, 1000):
                got = np.empty(n, np.uint64)
                fast_seen.add(L.mh_expand_sorted_runs(N, T, CS, rf, 9, ref, tot, first, n, run,
                                                       got.ctypes.data_as(u64p)))
                np.testing.assert_array_equal(got, want)
                got[:] = 0
                L.mh_expand_sorted_fast(N, T, CS, rf, 9, ref, tot, first, n, run, got.ctypes.data_as(u64p))
                np.testing.assert_array_equal(got, want)
    if (N, T, S) in ((1024, 8, 4189071), (4096, 8, 67025020), (2048, 64, 4173354)):
        assert 1 in fast_seen  # the BASELINE lists take the fast path


def test_div64_round_up_divider(model_host):
    import ctypes
    L = model_host.lib
    L.mh_div64.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    L.mh_div64.restype = ctypes.c_uint64
    rng = np.random.default_rng(3)
    ds = [1, 2, 3, 7, 8, 1023, 4095, 4096, 65535, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, (1 << 63) - 25, 1 << 63,
          (1 << 64) - 1] + [int(x) for x in rng.integers(1, 1 << 62, 40)]
    ns = [0, 1, (1 << 64) - 1, (1 << 63), (1 << 32) - 1] + [int(x) for x in rng.integers(0, 1 << 63, 60)]
    for d in ds:
        for n in ns + [d - 1, d, d + 1, 2 * d - 1]:
            n &= (1 << 64) - 1
            assert L.mh_div64(n, d) == n // d, (n, d)


@pytest.mark.parametrize("N,T,CS", [(64, 4, 4), (96, 3, 4), (1024, 8, 4), (4096, 8, 4), (2048, 64, 4)])
def test_keyorder_index_range_selects_a_key_range(orc, N, T, CS):
    """faithful_key (the host key of dist.sharded_faithful_gen_hist) equals the
    oracle's sort key; keyorder_index_range's binary searches over a key-order
    list give exactly the indices whose keys fall in the range (what a rank of
    the generated-list faithful shards generates)."""
    import pluss_sampler_optimization_amd as P
    c = orc.cfg(N, T, CS)
    pc = P.SamplerConfig(n=N, threads=T, chunk=CS, mode="faithful")
    for ref in range(6):
        tot = min(3000, (N - 1) ** (3 if ref >= 2 else 2))
        s = orc.expand_sorted(c, 0x5EED0003, ref, tot, 0, tot)
        key = orc.sort_key(N, T, CS, s)
        assert [P.faithful_key(pc, x) for x in s] == [int(k) for k in key]
        at = lambda i: s[i]  # noqa: E731
        hi_key = int(key[-1]) + 1
        for lo, hi in ((0, hi_key), (hi_key // 3, 2 * hi_key // 3), (int(key[7]), int(key[7]) + 1),
                       (int(key[7]) + 1, int(key[8])), (hi_key, 2 * hi_key)):
            a, b = P.keyorder_index_range(pc, 0, ref, tot, lo, hi, sample_at=at)
            # the library's host-only search (pluss_keyorder_index_range: no device) over its own generator
            assert P.keyorder_index_range(pc, 0x5EED0003, ref, tot, lo, hi) == (a, b)
            inside = np.nonzero((key >= lo) & (key < hi))[0]
            if len(inside):
                assert (a, b) == (inside[0], inside[-1] + 1)
            else:
                assert a == b
