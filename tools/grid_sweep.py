"""Diagnostics: k_count (dense tail) time vs workgroup count (PLUSS_GRID), interleaved
repeats so clock drift does not favour one setting.  One JSON line per (size, grid)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402
from ablate import timeit  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    cfg = P.SamplerConfig(n=1024, threads=8)
    grids = [int(g) for g in os.environ.get("SWEEP", "0,768,896,1024,1152,1280,1536,2048").split(",")]
    for total in [1 << int(b) for b in os.environ.get("SIZES", "24,26").split(",")]:
        counts = P.default_counts(1024, total)
        buf = torch.empty(total, dtype=torch.int64, device=dev)
        ctx = P.Context(cfg)
        off = 0
        for r, c in enumerate(counts):
            ctx.expand(0x5EED0001, r, 0, c, buf.data_ptr() + 8 * off, s.cuda_stream)
            off += c
        dense = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev)
        res = {g: [] for g in grids}
        for _ in range(5):
            for g in grids:
                if g:
                    os.environ["PLUSS_GRID"] = str(g)
                else:
                    os.environ.pop("PLUSS_GRID", None)
                res[g].append(timeit(lambda: ctx.sampled_hist_dense(buf.data_ptr(), total, dense.data_ptr(),
                                                                    s.cuda_stream), s, reps=100))
        os.environ.pop("PLUSS_GRID", None)
        for g in grids:
            ms = min(res[g])
            print(json.dumps({"samples": total, "grid": g or "default", "min_ms": ms,
                              "median_ms": sorted(res[g])[2], "GBps": 8 * total / ms / 1e6}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
