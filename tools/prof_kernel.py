"""Minimal driver for rocprofv3 counter passes: expand the config-2 sample list
once, then launch the hot kernel a few times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402

N, T, total = 1024, 8, 1 << 24
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
cfg = P.SamplerConfig(n=N, threads=T)
counts = P.default_counts(N, total)
buf = torch.empty(total, dtype=torch.int64, device=dev)
ctx = P.Context(cfg)
off = 0
for r, c in enumerate(counts):
    ctx.expand(0x5EED0001, r, 0, c, buf.data_ptr() + 8 * off, s.cuda_stream)
    off += c
keys = torch.empty(4096, dtype=torch.int64, device=dev)
cnts = torch.empty(4096, dtype=torch.int64, device=dev)
ctx.reset(s.cuda_stream)
for _ in range(int(os.environ.get("PROF_REPS", 5))):  # the bench step: one fused count+export launch
    ctx.sampled_hist_export(buf.data_ptr(), total, keys.data_ptr(), cnts.data_ptr(), 4096, s.cuda_stream)
torch.cuda.synchronize()
h = P.hist_from_tables(keys.cpu().numpy().view("uint64"), cnts.cpu().numpy().view("uint64"))
assert h.total() == total
print("ok")
