"""Host-side views of raw reuse-interval histograms.

The device histograms are exact-key (raw RI).  The reference bins some of its
histograms on the host side of the hot path; these helpers derive those views
from the exact bins so they can be compared with the reference's printouts.
"""


def floor_pow2(x):
    """_polybench_to_highest_power_of_two (pluss_utils.h:665-679; utils.rs:121-134): highest set bit."""
    return 1 << (int(x).bit_length() - 1)


def ceil_pow2(x):
    """Rust unsafe_utils.rs:228-230 uses u64::next_power_of_two (ceil)."""
    x = int(x)
    return 1 << (x - 1).bit_length() if x > 1 else 1


def log2_floor_bins(hist):
    """{ri: count} -> {floor_pow2(ri): count}; keys <= 0 (cold -1) unbinned (pluss_utils.h:682-683)."""
    out = {}
    for ri, c in hist.items():
        k = floor_pow2(ri) if ri > 0 else ri
        out[k] = out.get(k, 0) + c
    return out


def log2_ceil_bins(hist):
    out = {}
    for ri, c in hist.items():
        k = ceil_pow2(ri) if ri > 0 else ri
        out[k] = out.get(k, 0) + c
    return out
