"""Faithful group passes at config 3 (pluss_group_gen_faithful / _uniform /
pluss_group_sampled_hist over an any-order host list) on one device with 1, 2
and 8 logical shards: host clock per call (median), for a kernel trace of
where the fixed cost goes.
usage: python tools/group_time.py [generated|uniform|any_order] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
if os.environ.get("PLUSS_PROBE_LIB") == "stages":  # the stage-checked diagnostic build (tools/r5p_probe.py)
    import pluss_sampler_optimization_amd._lib as L  # noqa: E402
    L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "stages", "libpluss_gpu.so")
import pluss_sampler_optimization_amd as P  # noqa: E402

src = sys.argv[1] if len(sys.argv) > 1 else "generated"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
c = P.SamplerConfig(n=4096, threads=8, mode="faithful")
totals = P.default_counts(4096, 1 << 28)
SEED = 0x5EED0001
lst = None
one = None
if src == "any_order":
    import torch
    total = sum(totals)
    host = torch.empty(total, dtype=torch.int64, pin_memory=True)
    d = torch.empty(total, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    with P.Context(c) as ctx:
        off = 0
        for r, n in enumerate(totals):
            ctx.expand(SEED, r, 0, n, d.data_ptr() + 8 * off, st.cuda_stream)
            off += n
        ctx.reset(st.cuda_stream)
        ctx.faithful_hist_refs(d.data_ptr(), totals, st.cuda_stream)
        st.synchronize()
        one = ctx.fetch()
    host.copy_(d)
    del d
    lst = host.numpy().view("uint64")
out = {}
for spd in (1, 2, 8):
    with P.Group(c, [0], spd) as g:
        if src == "generated":
            call = lambda: g.gen_faithful(SEED, totals)  # noqa: E731
        elif src == "uniform":
            call = lambda: g.gen_uniform_faithful(SEED, totals)  # noqa: E731
        else:
            call = lambda: g.sampled_hist(lst)  # noqa: E731
        if os.environ.get("PLUSS_PROBE_LIB") == "stages" and src == "any_order":
            L.lib().pluss_debug_sort_dump()  # (the stage build's sort checks so far: after the last group)
        print(f"shards {spd}: call 0", file=sys.stderr, flush=True)  # (progress: which call a failure hit)
        h = call()
        print(f"shards {spd}: call 1", file=sys.stderr, flush=True)
        call()  # (the second identical call is captured into a graph)
        ts = []
        for k in range(reps):
            print(f"shards {spd}: call {2 + k}", file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            call()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        out[f"shards_{spd}"] = ts[len(ts) // 2]
        if one is not None:
            out[f"equal_{spd}"] = h.bins == one.bins and list(h.traversed) == list(one.traversed)
print(json.dumps({"source": src, **out}))
