"""r10's sample draw in key order (csrc/pluss_uniform.h, restated
in C by oracle/pluss_oracle.c orc_expand_uniform) on the CPU.

r10 draws each reference's samples with rand() % (N-1) per index and rejects
duplicates (r10:156-185): a uniform S-subset of the span^d points.  The key-
order generator must give that distribution: every list is distinct and
strictly increasing in r10's pop order (IterationComp, pluss_utils.h:175-267),
slices are random access, and the counts over partitions of the points --
per thread-local row q, per simulated thread, per c1 / c2 residue -- follow
the multivariate hypergeometric law of a uniform draw (chi-square at BASELINE
config 2's budget).  The stratified key-order lists (orc_expand_sorted) are
run through the same partition tests as a contrast where a stratum pattern
would show.  The device lists are compared with these in tests/test_gpu_uniform.py.
"""
import numpy as np
import pytest
from scipy import stats

SEED = 0x5EED0001


def keys(orc, c, s):
    return orc.sort_key(c.N, c.T, c.CS, s).astype(np.uint64)


@pytest.mark.parametrize("N,T,ref,S", [(64, 4, "A0", 1000), (128, 4, "B0", 2098), (128, 8, "C0", 164),
                                       (64, 2, "C3", 30000), (128, 4, "C2", 120_000), (256, 8, "C1", 65025),
                                       (512, 4, "B0", 3), (64, 4, "C0", 3969)])
def test_lists_are_distinct_sorted_and_random_access(orc, N, T, ref, S):
    c = orc.cfg(N, T)
    s = orc.expand_uniform(c, SEED, ref, S, 0, S)
    k = keys(orc, c, s)
    assert len(s) == S and (k[1:] > k[:-1]).all()
    m = np.uint64(0xFFFFF)
    c0, c1, c2 = (s >> np.uint64(40)) & m, (s >> np.uint64(20)) & m, s & m
    assert (c0 < N - 1).all() and (c1 < N - 1).all()  # rand() % (N-1) (Q4)
    if ref in ("C0", "C1"):
        assert (c2 == 0).all()
    else:
        assert (c2 < N - 1).all()
    a, b = S // 3, S // 3 + max(1, S // 4)
    assert (orc.expand_uniform(c, SEED, ref, S, a, b - a) == s[a:b]).all()
    if S == (N - 1) ** (2 if ref in ("C0", "C1") else 3):  # every point: the whole space in key order
        assert len(np.unique(s)) == S


def test_range_full_and_seeds(orc):
    c = orc.cfg(64, 4, range_full=1)
    s = orc.expand_uniform(c, SEED, "A0", 5000, 0, 5000)
    assert ((s >> np.uint64(40)) & np.uint64(0xFFFFF)).max() == 63  # c0 = N-1 is drawn with range_full
    k = keys(orc, c, s)
    assert (k[1:] > k[:-1]).all()
    t = orc.expand_uniform(orc.cfg(64, 4), SEED + 1, "A0", 5000, 0, 5000)
    assert not np.array_equal(orc.expand_uniform(orc.cfg(64, 4), SEED, "A0", 5000, 0, 5000), t)


def _chi2_p(counts, expected):
    counts = np.asarray(counts, np.float64)
    expected = np.asarray(expected, np.float64)
    chi = ((counts - expected) ** 2 / expected).sum()
    return stats.chi2.sf(chi, len(counts) - 1)


def _parts(N, T, CS, s):
    m = np.uint64(0xFFFFF)
    c0 = ((s >> np.uint64(40)) & m).astype(np.int64)
    c1 = ((s >> np.uint64(20)) & m).astype(np.int64)
    c2 = (s & m).astype(np.int64)
    k = c0 // CS
    return {"q": (k // T) * CS + c0 % CS, "tid": k % T, "c1%64": c1 % 64, "c2%64": c2 % 64, "c1": c1,
            "c2": c2, "c0": c0}


@pytest.mark.parametrize("ref", ["C2", "B0", "C0"])
def test_uniform_inclusion_config2(orc, ref):
    """BASELINE config 2 (N=1024, T=8, 2^24 samples: 4,189,071 per 3-D
    reference, 10,466 per 2-D one): the counts per thread-local row q, per
    thread, per c1 and per c2 residue agree with a uniform draw over the
    (N-1)^d points (chi-square p > 1e-4 for every partition); rows sampled by
    a uniform draw hold S/(N-1) samples per c0 value (binomial bounds)."""
    N, T, CS = 1024, 8, 4
    c = orc.cfg(N, T)
    S = 10466 if ref == "C0" else 4189071
    s = orc.expand_uniform(c, SEED, ref, S, 0, S)
    span = N - 1
    parts = _parts(N, T, CS, s)
    # c0 is uniform over [0, N-2]: q/tid cells hold an equal share of the c0 values
    n0 = np.bincount(parts["c0"], minlength=span)[:span]
    assert _chi2_p(n0, np.full(span, S / span)) > 1e-4
    sd = np.sqrt(S / span * (1 - 1 / span))
    assert np.abs(n0 - S / span).max() < 6 * sd
    for name in ("c1%64", "c1") + (("c2%64", "c2") if ref != "C0" else ()):
        v = parts[name]
        if name.endswith("%64"):
            exp = np.array([len(range(r, span, 64)) for r in range(64)], np.float64) * S / span
            got = np.bincount(v, minlength=64)
        else:
            exp = np.full(span, S / span)
            got = np.bincount(v, minlength=span)[:span]
        assert _chi2_p(got, exp) > 1e-4, name
    # thread x row cells (c0 = ((q/CS)*T + tid)*CS + q%CS): equal point counts except the missing c0 = N-1
    cell = parts["q"] * T + parts["tid"]
    got = np.bincount(cell, minlength=N)
    pts = np.ones(N)
    pts[N - 1] = 0  # (q, tid) of c0 = N-1
    exp = pts / pts.sum() * S
    keep = exp > 0
    assert got[~keep].sum() == 0
    assert _chi2_p(got[keep], exp[keep]) > 1e-4


def test_pairwise_spacing_matches_uniform(orc):
    """Gaps between consecutive samples of a uniform draw in key order are
    (about) geometric; a stratified list has none below its stratum spacing
    pattern.  The mean and variance of the point-index gaps fit a uniform
    draw's."""
    N, T = 128, 4
    c = orc.cfg(N, T)
    S = 20000
    s = orc.expand_uniform(c, SEED, "C3", S, 0, S)
    span = N - 1
    p = _parts(N, T, 4, s)
    # point index in key order: ((q*span + c1)*span + c2)*T + tid  (block A: q < Q-1)
    qa = p["q"] < N // T - 1
    idx = (((p["q"] * span + p["c1"]) * span + p["c2"]) * T + p["tid"])[qa]
    D = (N // T - 1) * span * span * T
    gaps = np.diff(np.sort(idx)).astype(np.float64)
    mean_gap = D / (qa.sum() + 1)
    assert abs(gaps.mean() / mean_gap - 1) < 0.03
    assert abs(gaps.std() / gaps.mean() - 1) < 0.05  # exponential-like: std ~ mean (a stratified list: << mean)
    st = orc.expand_sorted(c, SEED, "C3", S, 0, S)
    ps = _parts(N, T, 4, st)
    qs = ps["q"] < N // T - 1
    idx_s = (((ps["q"] * span + ps["c1"]) * span + ps["c2"]) * T + ps["tid"])[qs]
    gs = np.diff(np.sort(idx_s)).astype(np.float64)
    assert gs.std() / gs.mean() < 0.7  # the stratified list's gaps are far more regular
