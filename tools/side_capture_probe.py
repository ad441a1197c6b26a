"""The uniform source's side stream inside a group's captured pass (diagnostic
build, knob SIDE_CAPTURE): repeated identical group calls at N=4096 with the
BASELINE 2-D budgets, a native backtrace on a host fault.
usage: PLUSS_PROBE_LIB=stages PLUSS_KNOB_SIDE_CAPTURE=1 python tools/side_capture_probe.py"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
if os.environ.get("PLUSS_PROBE_LIB") == "stages":
    import pluss_sampler_optimization_amd._lib as L  # noqa: E402
    L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "stages", "libpluss_gpu.so")
import pluss_sampler_optimization_amd as P  # noqa: E402
import torch  # noqa: E402

bt = ctypes.CDLL(os.path.join(HERE, "native", "libsegv_bt.so"))
N, T = 4096, 8
c = P.SamplerConfig(n=N, threads=T, mode="faithful")
c2 = P.default_counts(N, 1 << 28)[0]
totals = [c2, c2, 200_000, 200_000, 200_000, 200_000]
st = torch.cuda.Stream()
with P.Context(c) as ctx:
    ctx.reset(st.cuda_stream)
    ctx.gen_uniform_faithful_refs(31, totals, st.cuda_stream)
    st.synchronize()
    one = ctx.fetch()
assert bt.segv_bt_install() == 0  # (after the first GPU work: the runtime's own handlers are in by then)
for spd in (1, 8):
    with P.Group(c, [0], spd) as g:
        for k in range(4):
            print(f"spd {spd} call {k}", file=sys.stderr, flush=True)
            h = g.gen_uniform_faithful(31, totals)
            print(spd, k, "equal" if h.bins == one.bins and h.traversed == one.traversed else "DIFFERENT", flush=True)
