"""Faithful group passes at config 3 (pluss_group_gen_faithful / _uniform) on
one device with 1, 2 and 8 logical shards: host clock per call (median), for
a kernel trace of where the fixed cost goes.
usage: python tools/group_time.py [generated|uniform] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import pluss_sampler_optimization_amd as P  # noqa: E402

src = sys.argv[1] if len(sys.argv) > 1 else "generated"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
c = P.SamplerConfig(n=4096, threads=8, mode="faithful")
totals = P.default_counts(4096, 1 << 28)
out = {}
for spd in (1, 2, 8):
    with P.Group(c, [0], spd) as g:
        call = (lambda: g.gen_faithful(0x5EED0001, totals)) if src == "generated" else \
            (lambda: g.gen_uniform_faithful(0x5EED0001, totals))
        call()
        call()  # (the second identical call is captured into a graph)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            call()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        out[f"shards_{spd}"] = ts[len(ts) // 2]
print(json.dumps({"source": src, **out}))
