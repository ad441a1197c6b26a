"""r10's uniform draw generated in key order on the device (csrc/pluss_uniform.h
plan + tile staging) against the C oracle's restatement (orc_expand_uniform),
bit for bit, and faithful mode over it: the lists generated inside the pass
(pluss_dev_gen_uniform_faithful_refs) equal the same lists materialised and
read by the sorted source, and the stepping r10 oracle (orc_faithful).

Run on an MI355X:  python -m pytest tests/test_gpu_uniform.py -m gpu -x -q
"""
import numpy as np
import pytest

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
