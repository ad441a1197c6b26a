"""The faithful radix source's bucket sort (csrc/pluss_sort.h, through
pluss_diag_sort_words) against a host sort of the same packed words.

A reference's arbitrary-order list (r10 draws rand() samples into a
priority_queue, r10:151-185) becomes its packed sort words rank << 2 | case in
ascending order: rank = ((q*N + c1)*N + c2)*T + tid is the key order of
IterationComp (pluss_utils.h:175-267), the case bits follow the closed RI
rules.  The words are restated here in numpy, independently of
the device code, and the device's sorted array must equal np.sort of them --
for uniform lists (two-level buckets), skewed and duplicated lists (the deep
splits), tiny lists, and the widest words (N = 2^20 - 32, 62 bits).

Run on an MI355X:  python -m pytest tests/test_gpu_sort.py -m gpu -x -q
"""
import numpy as np
import pytest

from conftest import all_tids_list, window_list

pytestmark = pytest.mark.gpu

P = pytest.importorskip("pluss_sampler_optimization_amd")
torch = pytest.importorskip("torch")
SEED = 0x5EED0007


def host_words(N, T, CS, W, ref, samples):
    """rank << 2 | case of each sample (uint64), restated in numpy."""
    rid = P.REF_ID[ref]
    s = np.asarray(samples, np.uint64)
    c2 = (s & np.uint64(0xFFFFF)).astype(np.int64)
    c1 = ((s >> np.uint64(20)) & np.uint64(0xFFFFF)).astype(np.int64)
    c0 = ((s >> np.uint64(40)) & np.uint64(0xFFFFF)).astype(np.int64)
    if rid < 2:
        c2 = np.zeros_like(c2)
    k, p = c0 // CS, c0 % CS
    kt, t = k // T, k % T
    q = kt * CS + p
    rank = (((q * N + c1) * N + c2) * T + t).astype(np.uint64)
    a = np.ones(len(s), bool)
    b = np.ones(len(s), bool)
    if ref == "C3":
        a, b = c2 + 1 < N, (c1 & (W - 1)) != W - 1
    elif ref == "A0":
        a, b = (c2 & (W - 1)) != W - 1, c1 + 1 < N
    elif ref == "B0":
        a, b = (c1 & (W - 1)) != W - 1, q + 1 < N // T
    case = np.where(a, 0, np.where(b, 1, 2)).astype(np.uint64)
    return (rank << np.uint64(2)) | case


def device_sort(c, ref, samples):
    s = np.ascontiguousarray(samples, np.uint64)
    t = torch.from_numpy(s.view(np.int64)).cuda()
    out = torch.empty(max(len(s), 1), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    with P.Context(c) as ctx:
        wb = ctx.diag_sort_words(ref, t.data_ptr(), len(s), out.data_ptr(), st)
        torch.cuda.synchronize()
    raw = out.cpu().numpy().view(np.uint8)
    return (raw[:4 * len(s)].view(np.uint32).astype(np.uint64) if wb == 4 else raw[:8 * len(s)].view(np.uint64)), wb


def check(N, T, ref, samples, wb_want):
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    got, wb = device_sort(c, ref, samples)
    assert wb == wb_want
    want = np.sort(host_words(N, T, 4, 8, ref, samples))
    np.testing.assert_array_equal(got, want)


def feistel(N, T, ref, n):
    c = P.SamplerConfig(n=N, threads=T)
    return P.expand_samples(c, SEED, P.REF_ID[ref], 0, n)


@pytest.mark.parametrize("N,T,wb", [(4096, 8, 8), (1024, 8, 4)])
@pytest.mark.parametrize("ref", ["C0", "A0", "B0", "C3"])
def test_uniform_lists(N, T, wb, ref):
    """Feistel lists (any order): 2^20 samples -- 256 top-level buckets, each
    split into items -- and the 2-D references' sparse ranks (c2 = 0)."""
    n = 1 << 20 if ref not in ("C0", "C1") else 200_000
    check(N, T, ref, feistel(N, T, ref, n), wb)


@pytest.mark.parametrize("n", [1, 2, 100, 2048, 2049, 4096, 4097, 9000, 70_001])
def test_small_and_boundary_sizes(n):
    """One top-level bucket (n <= 2048), the first split (n > 2048), one
    item at SCAP, an item past it, and a partial last chunk."""
    check(4096, 8, "C2", feistel(4096, 8, "C2", n), 8)


def test_duplicates_and_all_equal():
    """Repeated samples (equal words: the deep splits run out of digits) and a
    list of one sample repeated."""
    base = feistel(4096, 8, "A0", 50_000)
    rng = np.random.default_rng(1)
    dup = np.concatenate([base, base[:20_000], base[:5_000]])
    check(4096, 8, "A0", dup[rng.permutation(len(dup))], 8)
    check(4096, 8, "B0", np.full(30_000, P.pack("B0", 17, 5, 9), np.uint64), 8)


def test_skewed_dense_rows():
    """Every sample in the first three thread-local rows, sampled by all 8
    threads (4.5 M words over 3/512 of the key space): top-level buckets far
    past SCAP, items split again depth first."""
    s = all_tids_list(4096, 8, 4, "C3", 500_000, [0, 1, 2], 5)
    rng = np.random.default_rng(2)
    check(4096, 8, "C3", s[rng.permutation(len(s))], 8)
    w = window_list(4096, 8, 4, "B0", 200_000, [0, 511], 16, 3)
    check(4096, 8, "B0", w[rng.permutation(len(w))], 8)


def test_widest_words():
    """N = 2^20 - 32 (T=8): ranks up to N^3, 62-bit words."""
    N = (1 << 20) - 32
    check(N, 8, "C3", feistel(N, 8, "C3", 300_000), 8)


@pytest.mark.parametrize("ref", ["C0", "C1"])
def test_skewed_sparse_ranks(ref):
    """The 2-D references' sparse ranks (c2 = 0: the low rank bits always
    zero) concentrated in two thread-local rows of every thread (60,000 of the
    65,520 points): a few top-level buckets far past SCAP, split and split
    again on digits whose low part never varies -- the shape of round 3's
    C0 failures (tests above at N=4096), skewed."""
    w = window_list(4096, 8, 4, ref, 60_000, [0, 1], 0, 9)
    rng = np.random.default_rng(4)
    check(4096, 8, ref, w[rng.permutation(len(w))], 8)
