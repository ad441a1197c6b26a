"""Minimal driver for rocprofv3 passes over the faithful radix source (the
bucket sort, csrc/pluss_sort.h, then the scan pipeline) at config 3's shape:
N=4096, T=8, 2^28 samples of the six Feistel lists (arbitrary order).
PROF_REPS passes; PROF_LOG2 to change the size."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402

SEED = 0x5EED0001
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
sp = s.cuda_stream
N, total = 4096, 1 << int(os.environ.get("PROF_LOG2", 28))
counts = P.default_counts(N, total)
buf = torch.empty(total, dtype=torch.int64, device=dev)
ctx = P.Context(P.SamplerConfig(n=N, threads=8, mode="faithful"))
off = 0
for r, c in enumerate(counts):
    ctx.expand(SEED, r, 0, c, buf.data_ptr() + 8 * off, sp)
    off += c
for _ in range(int(os.environ.get("PROF_REPS", 3))):
    ctx.reset(sp)
    ctx.faithful_hist_refs(buf.data_ptr(), counts, sp)
torch.cuda.synchronize()
h = ctx.fetch()
assert h.total() > 0
print("ok radix", h.total())
