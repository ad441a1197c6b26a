"""CPU check of the bucket sort's index arithmetic (csrc/pluss_sort.h and
srt_plan in csrc/pluss_faithful.hip): the level-1 / level-2 histograms,
parents, level-2 chunks and items are restated here over the words of real
sample lists (host-computed), and every index the kernels form is checked to
stay inside the buffers srt_plan sizes -- the hist1 / hist2 columns, the chunk
map, the deep-item list -- and the items to tile each reference's range.
Shapes: one reference with the other five empty (the single-reference entry
points), all six, tiny and skewed lists."""
import numpy as np
import pytest

from test_gpu_sort import host_words

SB, SE = 256, 16
SBATCH = SB * SE
SC = 4 * SBATCH
SCAP = 4096
SSPLIT = 3072
SDIG = 8


def log2_ceil(x):
    b = 0
    while b < 63 and (1 << b) < x:
        b += 1
    return b


def d1_of(n, wb):
    l = log2_ceil(n)
    d = l - 11 if l > 11 else 0
    return min(d, SDIG, wb)


def split_bits(cnt, hi):
    D = log2_ceil((cnt + SSPLIT - 1) // SSPLIT)
    D = max(1, min(D, SDIG))
    return min(D, hi)


def pk_bits(N):
    top, b = N ** 3 - 1, 1
    while b < 62 and (top >> b):
        b += 1
    return b + 2


def plan_and_check(N, words):
    """words: six uint64 arrays (a reference's words, any order)."""
    wb = pk_bits(N)
    p32 = wb <= 32 + SDIG
    cnt = [len(w) for w in words]
    d1 = []
    for n in cnt:
        d = d1_of(n, wb)
        if n and p32 and wb > 32 and d < wb - 32:
            d = wb - 32
        d1.append(d)
    nch = [(n + SC - 1) // SC for n in cnt]
    eoff = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    hoff = np.concatenate([[0], np.cumsum([(1 << d) * c for d, c in zip(d1, nch)])]).astype(np.int64)
    npar = sum(1 << d for d in d1)
    ntot = int(eoff[6])
    g2max = ntot // SC + npar + 1
    h2max = g2max * SB
    # level 1: hist1[ref block][digit][chunk], exclusive scan over everything
    h1 = np.zeros(int(hoff[6]), np.int64)
    for r in range(6):
        lo = wb - d1[r]
        for c in range(nch[r]):
            w = words[r][c * SC:(c + 1) * SC]
            dig = (w >> np.uint64(lo)).astype(np.int64) if lo < 64 else np.zeros(len(w), np.int64)
            dig &= (1 << d1[r]) - 1
            for d, k in zip(*np.unique(dig, return_counts=True)):
                idx = hoff[r] + d * nch[r] + c
                assert hoff[r] <= idx < hoff[r + 1]
                h1[idx] = k
    s1 = np.concatenate([[0], np.cumsum(h1)[:-1]]) if len(h1) else h1
    # parents (k_srt_plan)
    par = []
    for r in range(6):
        for b in range((1 << d1[r])):
            bstart = (lambda bb: int(s1[hoff[r] + bb * nch[r]]) if nch[r] else int(eoff[r]))
            s = bstart(b)
            e = bstart(b + 1) if b + 1 < (1 << d1[r]) else int(eoff[r + 1])
            c = e - s
            hi = wb - d1[r]
            d2 = split_bits(c, hi) if (c > SCAP and hi > 0) else 0
            nc2 = (c + SC - 1) // SC if d2 else 0
            assert eoff[r] <= s <= e <= eoff[r + 1]
            par.append((s, c, r, b, d2, nc2))
    assert len(par) == npar <= 6 * 256
    g2 = sum(p[5] for p in par)
    h2 = sum(p[5] << p[4] for p in par)
    assert g2 < g2max and h2 <= h2max
    # items: parents left whole and children (the children's sizes need the level-2 digits)
    ndeep, covered = 0, 0
    for (s, c, r, b, d2, nc2) in par:
        if c == 0:
            continue
        if d2 == 0:
            ndeep += c > SCAP
            covered += c
            continue
        # the parent's payloads: the words of reference r whose top digit is b
        w = words[r]
        lo1 = wb - d1[r]
        top = (w >> np.uint64(lo1)).astype(np.int64) if lo1 < 64 else np.zeros(len(w), np.int64)
        mine = w[top == b]
        assert len(mine) == c
        dig = ((mine >> np.uint64(lo1 - d2)).astype(np.int64)) & ((1 << d2) - 1)
        sizes = np.bincount(dig, minlength=1 << d2)
        assert sizes.sum() == c
        ndeep += int((sizes > SCAP).sum())
        covered += c
    assert covered == ntot
    assert ndeep <= npar * SB
    return npar, g2, h2, ndeep


REFS = ["C0", "C1", "A0", "B0", "C2", "C3"]


def feistel_words(mh, N, T, ref, n):
    """Words of the Feistel list (host build of pluss_model.h's generator)."""
    import ctypes
    s = np.empty(n, np.uint64)
    assert mh.lib.mh_expand(N, 0, 0x5EED0007, REFS.index(ref), 0, n, s.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
    return host_words(N, T, 4, 8, ref, s)


@pytest.mark.parametrize("N,T", [(4096, 8), (1024, 8), ((1 << 20) - 32, 8)])
def test_one_reference_others_empty(model_host, N, T):
    for ref, n in (("C0", 200_000), ("C2", 70_001), ("C3", 1), ("B0", 2049)):
        words = [np.zeros(0, np.uint64)] * 6
        words[REFS.index(ref)] = feistel_words(model_host, N, T, ref, n)
        plan_and_check(N, words)


def srt_cap(n, d1, wb, b, wmax):
    """k_srt_caps's capacity of bucket b (pluss_sort.h srt_cap)."""
    if d1 == 0:
        return n
    lo = wb - d1
    b0, b1 = b << lo, (b + 1) << lo
    w = 0 if b0 >= wmax else min(b1, wmax) - b0
    e = float(n) * (float(w) / float(wmax))
    c = e * 1.125 + 8.0 * np.sqrt(e) + 256.0
    return n if c >= n else int(c)


@pytest.mark.parametrize("N,T,n", [(4096, 8, 3_000_000), (1024, 8, 700_000), (1056, 8, 400_000), (2048, 64, 500_000),
                                   (4096, 8, 2049), (4096, 8, 40_000)])
def test_count_free_level1_capacities(model_host, N, T, n):
    """The count-free level 1 (k_srt_scatter1f): every bucket of a uniform
    (Feistel) list fits its capacity, so the counted fallback does not run,
    and the regions fit X1 (2 payloads per sample)."""
    wb = pk_bits(N)
    wmax = 4 * N ** 3
    for ref in ("C3", "A0", "C0"):
        w = feistel_words(model_host, N, T, ref, n)
        d = d1_of(n, wb)
        if wb <= 32 + SDIG and wb > 32 and d < wb - 32:
            d = wb - 32
        caps = [srt_cap(n, d, wb, b, wmax) for b in range(1 << d)]
        if sum(caps) > 2 * n:  # k_srt_caps raises the overflow at once: the counted level 1 runs
            assert n < 40_000
            continue
        top = (w >> np.uint64(wb - d)).astype(np.int64) if d else np.zeros(n, np.int64)
        counts = np.bincount(top, minlength=1 << d)
        assert (counts <= np.array(caps)).all(), (ref, int((counts - np.array(caps)).max()))


def srt_cap2(wb, d1, b1, d2, count, d, wmax):
    """k_srt_scatter2f's capacity of child d of a split parent (pluss_sort.h srt_cap2)."""
    lo1 = wb - d1
    lo2 = lo1 - d2
    p0 = b1 << lo1
    p1 = p0 + (1 << lo1)
    c0 = p0 + (d << lo2)
    c1 = c0 + (1 << lo2)
    pw = min(p1, wmax) - p0
    cw = 0 if c0 >= wmax else min(c1, wmax) - c0
    e = float(count) * (float(cw) / float(pw))
    c = e * 1.125 + 8.0 * np.sqrt(e) + 64.0
    return SCAP if c >= SCAP else int(c)


@pytest.mark.parametrize("N,T,n", [(4096, 8, 3_000_000), (1024, 8, 900_000), (2048, 64, 1_500_000)])
def test_count_free_level2_capacities(model_host, N, T, n):
    """The count-free level 2 (k_srt_scatter2f): every child of a uniform
    list's split parents fits its region (at most SCAP), so neither the
    counted level 2 nor the deep pass runs."""
    wb = pk_bits(N)
    wmax = 4 * N ** 3
    for ref in ("C3", "C0"):
        w = feistel_words(model_host, N, T, ref, n)
        d1 = d1_of(n, wb)
        if wb <= 32 + SDIG and wb > 32 and d1 < wb - 32:
            d1 = wb - 32
        lo1 = wb - d1
        top = (w >> np.uint64(lo1)).astype(np.int64)
        nsplit = 0
        for b1 in range(1 << d1):
            mine = w[top == b1]
            c = len(mine)
            if c <= SCAP:
                continue
            d2 = split_bits(c, lo1)
            nsplit += 1
            dig = ((mine >> np.uint64(lo1 - d2)).astype(np.int64)) & ((1 << d2) - 1)
            sizes = np.bincount(dig, minlength=1 << d2)
            caps = np.array([srt_cap2(wb, d1, b1, d2, c, d, wmax) for d in range(1 << d2)])
            assert (caps <= SCAP).all() and (sizes <= caps).all(), (ref, b1, int((sizes - caps).max()))
        assert nsplit > 0 or n <= 256 * SCAP


def test_six_references_and_skew(model_host):
    words = [feistel_words(model_host, 4096, 8, r, n) if n else np.zeros(0, np.uint64) for r, n in
             (("C0", 30_000), ("C1", 0), ("A0", 300_000), ("B0", 5), ("C2", 4096), ("C3", 70_000))]
    plan_and_check(4096, words)
    # skew: every word in one top-level bucket (items past SCAP -> deep)
    w = np.sort(feistel_words(model_host, 4096, 8, "A0", 200_000))[:50_000]
    npar, g2, h2, ndeep = plan_and_check(4096, [np.zeros(0, np.uint64)] * 2 + [w] + [np.zeros(0, np.uint64)] * 3)
    assert ndeep >= 0
