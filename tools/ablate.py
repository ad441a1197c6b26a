"""Where the hot kernel's time goes (diagnostics, include/pluss_diag.h):
the product dense pass (k_count, TAIL_DENSE), the same sample loads with
nothing counted (variant 1), counting without the tail (variant 2), and a
torch copy of the same buffer for a bandwidth reference.  Config-3
shape (N=4096, T=8) at 2^24 / 2^26 / 2^28 samples.  One JSON line per
variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402


def timeit(fn, stream, reps=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    N, T = int(os.environ.get("ABL_N", 4096)), int(os.environ.get("ABL_T", 8))
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    cfg = P.SamplerConfig(n=N, threads=T)
    for lg in [int(x) for x in os.environ.get("ABL_SIZES", "24,26,28").split(",")]:
        total = 1 << lg
        counts = P.default_counts(N, total)
        buf = torch.empty(total, dtype=torch.int64, device=dev)
        ctx = P.Context(cfg)
        off = 0
        for r, c in enumerate(counts):
            ctx.expand(0x5EED0001, r, 0, c, buf.data_ptr() + 8 * off, s.cuda_stream)
            off += c
        dense = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev)
        for name, variant in (("product", 0), ("loads_only", 1), ("no_tail", 2)):
            ms = timeit(lambda: ctx.diag_dense(buf.data_ptr(), total, dense.data_ptr(), variant, 0, s.cuda_stream), s)
            print(json.dumps({"samples": total, "variant": name, "ms": ms, "GBps": 8 * total / ms / 1e6}), flush=True)
        ctx.sampled_hist_dense(buf.data_ptr(), total, dense.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        assert int(dense[:P.DENSE_BINS].sum()) == total and int(dense[P.DENSE_BINS]) == 0
        dst = torch.empty_like(buf)
        ms = timeit(lambda: dst.copy_(buf), s)
        print(json.dumps({"samples": total, "variant": "torch_copy", "ms": ms, "GBps_rd+wr": 16 * total / ms / 1e6}),
              flush=True)
        del dst
        ctx.close()
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
