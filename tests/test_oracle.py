"""Pin the CPU oracle to the reference: r10 dumps, full-trace KATs, closed forms.

CPU only (no GPU): this is what makes the oracle trustworthy before it is used
as the checker of the HIP kernels.
"""
import numpy as np
import pytest

from conftest import closed_form_ri, expected_raw, golden_configs

GOLD = golden_configs()


@pytest.mark.parametrize("name,d,smp", GOLD, ids=[g[0] for g in GOLD])
def test_faithful_oracle_matches_reference_r10_dumps(orc, name, d, smp):
    """The C restatement of sampler_<REF> reproduces the reference's raw
    histograms and `traversed` counts for all six references (r10:690,694)."""
    c = orc.cfg(d["N"], d["T"])
    for ref in orc.REFS:
        got, trav = orc.faithful(c, ref, orc.pack_array(ref, smp[ref]))
        exp, etrav = expected_raw(d, ref)
        assert got == exp, (name, ref)
        assert trav == etrav, (name, ref)


def _merge(h, kind):
    out = {}
    for (r, k, ri), c in h.items():
        if k == kind:
            out[ri] = out.get(ri, 0) + c
    return out


def test_fulltrace_oracle_kat_n128_t4(orc):
    """SURVEY.md §4 KAT: raw per-tid RI multiset of seq.cpp at N=128, T=4 (verified
    against the compiled reference), 8,421,376 accesses traversed (seq.cpp:332)."""
    h, trav = orc.fulltrace(128, 4, thr_variant=1)
    assert trav == 8421376
    assert _merge(h, 0) == {-1: 12288, 1: 2127872, 3: 2097152, 4: 1835008, 486: 260096, 514: 1835008}
    assert _merge(h, 1) == {62194: 253952}


def test_fulltrace_oracle_log2_views(orc):
    """The reference prints the noshare histogram floor-log2 binned (pluss_utils.h:665-689)."""
    from pluss_sampler_optimization_amd.host import log2_floor_bins
    h, _ = orc.fulltrace(128, 4, thr_variant=1)
    assert log2_floor_bins(_merge(h, 0)) == {-1: 12288, 1: 2127872, 2: 2097152, 4: 1835008, 256: 260096,
                                             512: 1835008}


@pytest.mark.parametrize("N,T", [(64, 4), (256, 4), (128, 8), (128, 2), (32, 1)])
def test_fulltrace_oracle_closed_form_totals(orc, N, T):
    """Appendix A.3 totals for N % (CS*T) == 0."""
    h, trav = orc.fulltrace(N, T, thr_variant=1)
    ns, sh = _merge(h, 0), _merge(h, 1)
    exp_ns = {1: N * N + 7 * N * N // 8 + N ** 3, 3: N ** 3, 4: 7 * N ** 3 // 8, 4 * N - 26: N * N * (N - 1) // 8,
              4 * N + 2: 7 * N ** 3 // 8, -1: (2 + T) * N * N // 8}
    exp_sh = {(N - 7) * (4 * N + 2): (N // T - 1) * T * N * N // 8} if N // T > 1 else {}
    assert ns == exp_ns
    assert sh == exp_sh
    assert trav == N * N * (4 * N + 2)


@pytest.mark.parametrize("N,T,CS", [(128, 4, 4), (64, 8, 2), (96, 3, 4)])
def test_clean_oracle_matches_closed_forms(orc, N, T, CS):
    rng = np.random.default_rng(N + T)
    refs = np.repeat(np.arange(6), 200)
    c0 = rng.integers(0, N, len(refs)); c1 = rng.integers(0, N, len(refs)); c2 = rng.integers(0, N, len(refs))
    c2[refs < 2] = 0
    c1[::7] = N - 1
    c2[(refs >= 2) & (np.arange(len(refs)) % 5 == 0)] = N - 1
    s = np.array([orc.pack(int(r), a, b, c) for r, a, b, c in zip(refs, c0, c1, c2)], np.uint64)
    got = orc.clean_ri(orc.cfg(N, T, CS), s, nthreads=4)
    np.testing.assert_array_equal(got, closed_form_ri(N, T, CS, 8, refs, c0, c1, c2))


def test_oracle_expand_is_a_bijection(orc):
    c = orc.cfg(20, 4)
    for ref in ("C0", "A0"):
        D = 19 ** (2 if ref == "C0" else 3)
        s = orc.expand(c, 0x5EED0001, ref, 0, D)
        assert len(np.unique(s)) == D
        r = (s >> np.uint64(60)).astype(int)
        assert (r == orc.REF_ID[ref]).all()
        for sh in (40, 20, 0):
            v = ((s >> np.uint64(sh)) & np.uint64(0xFFFFF)).astype(int)
            assert v.max() <= 18
