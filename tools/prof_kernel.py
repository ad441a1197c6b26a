"""Minimal driver for rocprofv3 counter passes: expand the bench's sample list
(config 3: N=4096, T=8, 2^28 samples on one GPU; PROF_N / PROF_T / PROF_LOG2
override) once, then launch the hot kernel a few times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402

N, T = int(os.environ.get("PROF_N", 4096)), int(os.environ.get("PROF_T", 8))
total = 1 << int(os.environ.get("PROF_LOG2", 28))
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
dense = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev)
for _ in range(int(os.environ.get("PROF_REPS", 5))):  # the bench step: one dense-pass launch
    ctx.sampled_hist_dense(buf.data_ptr(), total, dense.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
assert P.hist_from_dense(cfg, dense.cpu().numpy()).total() == total
print("ok")
