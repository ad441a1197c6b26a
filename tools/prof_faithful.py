"""Minimal driver for rocprofv3 passes over the faithful (r10 queue semantics)
pipeline: config 2's budget (N=1024, T=8, 2^24 samples, six references in one
pass).  PROF_FAITH=sorted (key-order list in HBM, read once), generated (the
same lists generated inside the pass), radix (Feistel lists in any order,
sorted inside the pass) or uniform (r10's draw generated in key order inside
the pass); PROF_REPS passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402

SEED = 0x5EED0001
mode = os.environ.get("PROF_FAITH", "sorted")
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
sp = s.cuda_stream
# PROF_SHAPE=config3: N=4096, T=8, 2^28 samples (the headline shape on one GPU)
N, total = (4096, 1 << 28) if os.environ.get("PROF_SHAPE") == "config3" else (1024, 1 << 24)
cfg = P.SamplerConfig(n=N, threads=8, mode="faithful")
counts = P.default_counts(N, total)
buf = torch.empty(total, dtype=torch.int64, device=dev)
scratch = torch.empty(total // 4096 + 16, dtype=torch.int64, device=dev)
ctx = P.Context(cfg)
off = 0
for r, c in enumerate(counts):
    if mode == "radix":  # the Feistel lists (any order), sorted inside the pass
        ctx.expand(SEED, r, 0, c, buf.data_ptr() + 8 * off, sp)
    else:
        ctx.expand_sorted(SEED, r, c, 0, c, buf.data_ptr() + 8 * off, sp)
    off += c
for _ in range(int(os.environ.get("PROF_REPS", 5))):
    ctx.reset(sp)
    if mode == "sorted":
        ctx.faithful_hist_sorted_refs(buf.data_ptr(), counts, sp)
    elif mode == "radix":
        ctx.faithful_hist_refs(buf.data_ptr(), counts, sp)
    elif mode == "uniform":
        ctx.gen_uniform_faithful_refs(SEED, counts, sp)
    elif mode == "uni_stage":  # diagnostics: the plan and every full tile staged, nothing scanned
        ctx.diag_uniform_parts(SEED, counts, 1, scratch.data_ptr(), sp)
    else:
        ctx.gen_faithful_refs(SEED, counts, sp)
torch.cuda.synchronize()
h = ctx.fetch()
assert h.total() > 0 or mode == "uni_stage"
print("ok", mode, h.total())
