"""Debug: fused generate+count vs expand_sorted + dense pass, per rank slice."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402

N, T, total = int(sys.argv[1]), int(sys.argv[2]), 1 << int(sys.argv[3])
c = P.SamplerConfig(n=N, threads=T)
totals = P.default_counts(N, total)
sp = torch.cuda.current_stream().cuda_stream
d = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device="cuda")
d2 = torch.zeros_like(d)
with P.Context(c) as ctx:
    for rank in range(-1, 8):
        if rank < 0:
            first, n = [0] * 6, totals
        else:
            first = [k * rank // 8 for k in totals]
            n = [k * (rank + 1) // 8 - k * rank // 8 for k in totals]
        ctx.gen_count_dense(0x5EED0001, totals, first, n, d.data_ptr(), sp)
        buf = torch.empty(sum(n), dtype=torch.int64, device="cuda")
        off = 0
        for r in range(6):
            ctx.expand_sorted(0x5EED0001, r, totals[r], first[r], n[r], buf.data_ptr() + 8 * off, sp)
            off += n[r]
        ctx.sampled_hist_dense(buf.data_ptr(), sum(n), d2.data_ptr(), sp)
        torch.cuda.synchronize()
        a, b = d.cpu().numpy(), d2.cpu().numpy()
        print(rank, "fused", a.tolist(), flush=True)
        print(rank, "exp+count", b.tolist(), "equal", (a == b).all(), flush=True)
        del buf
