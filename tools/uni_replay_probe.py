"""Repeated identical uniform group passes (eager, captured, replayed) at the
C group test's small shape, against one device; the stage build prints any
slice-check difference.  usage: PLUSS_PROBE_LIB=stages python tools/uni_replay_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
if os.environ.get("PLUSS_PROBE_LIB") == "stages":
    import pluss_sampler_optimization_amd._lib as L  # noqa: E402
    L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "stages", "libpluss_gpu.so")
import pluss_sampler_optimization_amd as P  # noqa: E402
import torch  # noqa: E402

for (N, T, total) in ((128, 4, 200000), (1024, 8, 1 << 22)):
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, total)
    st = torch.cuda.Stream()
    with P.Context(c) as ctx:
        ctx.reset(st.cuda_stream)
        ctx.gen_uniform_faithful_refs(7, totals, st.cuda_stream)
        st.synchronize()
        one = ctx.fetch()
    for spd in (1, 2, 8):
        with P.Group(c, [0], spd) as g:
            for k in range(4):
                try:
                    h = g.gen_uniform_faithful(7, totals)
                    print(N, spd, k, "equal" if (h.bins == one.bins and h.traversed == one.traversed) else "DIFFERENT",
                          flush=True)
                except Exception as e:  # noqa: BLE001
                    print(N, spd, k, "ERROR", e, flush=True)
