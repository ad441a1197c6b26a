"""Driver for rocprofv3 kernel traces of the side paths at BASELINE sizes:
faithful mode over the config-2 list (2^24 samples, one r10 sampler per
reference) and the config-5 full trace (N=512, T=4).  Twice each (warm, then
profiled); prints the wall times."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402

N, T, total = 1024, 8, 1 << 24
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
counts = P.default_counts(N, total)
buf = torch.empty(total, dtype=torch.int64, device=dev)
with P.Context(P.SamplerConfig(n=N, threads=T)) as ctx:
    off = 0
    for r, c in enumerate(counts):
        ctx.expand(0x5EED0001, r, 0, c, buf.data_ptr() + 8 * off, s.cuda_stream)
        off += c
torch.cuda.synchronize()
mode = os.environ.get("PROF_FAITH", "serial")  # serial: one faithful_hist per reference; concurrent: faithful_hist_refs
with P.Context(P.SamplerConfig(n=N, threads=T, mode="faithful")) as ctx:
    for rep in range(3):
        ctx.reset(s.cuda_stream)
        torch.cuda.synchronize()
        t = time.perf_counter()
        if mode == "concurrent":
            ctx.faithful_hist_refs(buf.data_ptr(), counts, s.cuda_stream)
        else:
            off = 0
            for r, c in enumerate(counts):
                ctx.faithful_hist(r, buf.data_ptr() + 8 * off, c, s.cuda_stream)
                off += c
        torch.cuda.synchronize()
        print(f"faithful 2^24 ({mode}): {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
with P.Context(P.SamplerConfig(n=512, threads=4, thr_variant="v1")) as ctx:
    for rep in range(2):
        t = time.perf_counter()
        ctx.fulltrace(s.cuda_stream)
        torch.cuda.synchronize()
        print(f"full trace N=512: {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
