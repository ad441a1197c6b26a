"""Faithful-mode pass time of the four sources (key-ordered list, generated
lists, radix sort of a Feistel list, r10's uniform draw generated in key order) on the bench's faithful workload
(N=1024, T=8, 2^24 samples) or other shapes.
usage: python tools/fa_time.py [N T log2(samples)]..."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import pluss_sampler_optimization_amd as P  # noqa: E402

SEED = 0x5EED0001
args = sys.argv[1:]
only = None  # --only radix,uniform: time those sources alone (e.g. under a kernel trace)
if "--only" in args:
    i = args.index("--only")
    only = set(args[i + 1].split(","))
    del args[i:i + 2]
shapes = [tuple(int(x) for x in args[i:i + 3]) for i in range(0, len(args), 3)] or [(1024, 8, 24)]
st = torch.cuda.Stream()
sp = st.cuda_stream


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for N, T, lg in shapes:
    total = 1 << lg
    counts = P.default_counts(N, total)
    buf = torch.empty(total, dtype=torch.int64, device="cuda")
    scratch = torch.empty(total // 4096 + 16, dtype=torch.int64, device="cuda")
    fe = torch.empty(total, dtype=torch.int64, device="cuda")
    with P.Context(P.SamplerConfig(n=N, threads=T, mode="faithful")) as ctx:
        off = 0
        for r, c in enumerate(counts):
            ctx.expand_sorted(SEED, r, c, 0, c, buf.data_ptr() + 8 * off, sp)
            ctx.expand(SEED, r, 0, c, fe.data_ptr() + 8 * off, sp)
            off += c
        runs = {"sorted": lambda: ctx.faithful_hist_sorted_refs(buf.data_ptr(), counts, sp),
                "generated": lambda: ctx.gen_faithful_refs(SEED, counts, sp),
                "radix": lambda: ctx.faithful_hist_refs(fe.data_ptr(), counts, sp),
                "uniform": lambda: ctx.gen_uniform_faithful_refs(SEED, counts, sp),
                # (diagnostics: the uniform source's plan alone, and plan + staging of every full tile)
                "uni_plan": lambda: ctx.diag_uniform_parts(SEED, counts, 0, scratch.data_ptr(), sp),
                "uni_stage_dec": lambda: ctx.diag_uniform_parts(SEED, counts, 1, scratch.data_ptr(), sp),
                "uni_stage_packed": lambda: ctx.diag_uniform_parts(SEED, counts, 2, scratch.data_ptr(), sp)}
        res = {"N": N, "T": T, "samples": total}
        hs = {}
        runs = {k: v for k, v in runs.items() if only is None or k in only or k == "sorted"}
        for name, run in runs.items():
            ctx.reset(sp)
            run()
            torch.cuda.synchronize()
            if not name.startswith("uni_"):
                hs[name] = ctx.fetch()
            res[name + "_ms"] = timed(run)
        if "generated" in hs:
            assert hs["sorted"].bins == hs["generated"].bins
        res["recorded"] = hs["sorted"].total()
        print(json.dumps(res), flush=True)
