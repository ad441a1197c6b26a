"""Step-by-step probe of the six-reference radix pass (pluss_dev_faithful_hist_refs)
on one device: uniform Feistel lists and skewed / malformed lists, each call
synchronised and reported before the next, so a failing call names itself.
usage: python tools/radix_probe.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import pluss_sampler_optimization_amd as P  # noqa: E402
import torch  # noqa: E402

st = torch.cuda.Stream()


def run(N, name, counts, lst):
    c = P.SamplerConfig(n=N, threads=8, mode="faithful")
    d = torch.from_numpy(np.ascontiguousarray(lst).view(np.int64)).to("cuda")
    torch.cuda.synchronize()
    print("start", N, name, flush=True)
    with P.Context(c) as ctx:
        ctx.reset(st.cuda_stream)
        ctx.faithful_hist_refs(d.data_ptr(), counts, st.cuda_stream)
        st.synchronize()
        try:
            h = ctx.fetch()
            print("ok", N, name, h.total(), flush=True)
        except P.PlussError as e:
            print("error", N, name, str(e)[:120], flush=True)


for N in (1024, 2048):
    c = P.SamplerConfig(n=N, threads=8, mode="faithful")
    for tot in (1 << 20, (1 << 20) // 3):
        counts = P.default_counts(N, tot)
        lst = np.concatenate([P.expand_samples(c, 5, r, 0, n) for r, n in enumerate(counts)])
        run(N, f"feistel {tot}", counts, lst)
    counts = P.default_counts(N, 1 << 20)
    lst = np.concatenate([P.expand_samples(c, 5, r, 0, n) for r, n in enumerate(counts)])
    off = np.concatenate([[0], np.cumsum(counts)])
    srt = lst.copy()
    for r in range(6):
        srt[off[r]:off[r + 1]] = np.sort(srt[off[r]:off[r + 1]])
    run(N, "each reference sorted", counts, srt)
    rep = lst.copy()
    for r in range(6):
        rep[off[r]:off[r + 1]] = rep[off[r]]
    run(N, "each reference one sample repeated", counts, rep)
    bad = np.zeros_like(lst)
    run(N, "all zero words", counts, bad)
print("done", flush=True)
