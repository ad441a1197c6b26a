"""Diagnostics: k_count (dense tail) time vs workgroup cap (pluss_diag_dense's
max_grid; 0 = the launcher's default), interleaved repeats so clock drift
does not favour one setting.  One JSON line per (size, grid)."""
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
    N = int(os.environ.get("SWEEP_N", 4096))
    cfg = P.SamplerConfig(n=N, threads=8)
    grids = [int(g) for g in os.environ.get("SWEEP", "0,512,640,768,1024").split(",")]
    for total in [1 << int(b) for b in os.environ.get("SIZES", "24,26,28").split(",")]:
        counts = P.default_counts(N, total)
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
                res[g].append(timeit(lambda: ctx.diag_dense(buf.data_ptr(), total, dense.data_ptr(), 0, g,
                                                             s.cuda_stream), s, reps=20))
        for g in grids:
            v = sorted(res[g])
            print(json.dumps({"samples": total, "grid": g or "default", "min_ms": v[0], "median_ms": v[2],
                              "GBps": 8 * total / v[2] / 1e6}), flush=True)
        ctx.close()
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
