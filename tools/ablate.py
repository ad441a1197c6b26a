"""Split the hot kernel's time (diagnostics; defaults: UNROLL=2, NT=1, grid 1024): PLUSS_ABLATE=3 loads only
(k_count's buffer loads), =4 count without the tail, =2 loads only and =1 loads + key computation (both on the lane-counter kernel,
PLUSS_LEGACY=1), default = product kernel (k_count, ballot counting).  Also a torch copy for a
bandwidth reference.  Prints one JSON line per variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402


def timeit(fn, stream, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    N, T = int(os.environ.get("ABL_N", 1024)), int(os.environ.get("ABL_T", 8))
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    cfg = P.SamplerConfig(n=N, threads=T)
    for total in (1 << 24, 1 << 26):
        counts = P.default_counts(N, total)
        buf = torch.empty(total, dtype=torch.int64, device=dev)
        ctx = P.Context(cfg)
        off = 0
        for r, c in enumerate(counts):
            ctx.expand(0x5EED0001, r, 0, c, buf.data_ptr() + 8 * off, s.cuda_stream)
            off += c
        torch.cuda.synchronize()
        variants = [dict(PLUSS_ABLATE=m) for m in ("3", "4", "2", "1")] + [{}, dict(PLUSS_LEGACY="1")]
        variants += [dict(PLUSS_NT="0"), dict(PLUSS_PCS="4")]
        variants += [dict(PLUSS_ABLATE="2", PLUSS_GRID=g) for g in ("2048", "4096")]
        for v in variants:
            for k in ("PLUSS_ABLATE", "PLUSS_UNROLL", "PLUSS_GRID", "PLUSS_NT", "PLUSS_PCS", "PLUSS_LEGACY"):
                os.environ.pop(k, None)
            os.environ.update(v)
            ms = timeit(lambda: ctx.sampled_hist(buf.data_ptr(), total, s.cuda_stream), s)
            print(json.dumps({"samples": total, **v, "ms": ms, "GBps": 8 * total / ms / 1e6}), flush=True)
        for k in ("PLUSS_ABLATE", "PLUSS_UNROLL", "PLUSS_GRID", "PLUSS_NT", "PLUSS_PCS", "PLUSS_LEGACY"):
            os.environ.pop(k, None)
        keys = torch.empty(4096, dtype=torch.int64, device=dev)
        cnts = torch.empty(4096, dtype=torch.int64, device=dev)
        fused = [{}, dict(PLUSS_LEGACY="1")]
        for v in fused:
            for k in ("PLUSS_UNROLL", "PLUSS_GRID", "PLUSS_NT", "PLUSS_LEGACY"):
                os.environ.pop(k, None)
            os.environ.update(v)
            ms = timeit(lambda: ctx.sampled_hist_export(buf.data_ptr(), total, keys.data_ptr(), cnts.data_ptr(), 4096,
                                                        s.cuda_stream), s)
            print(json.dumps({"samples": total, "fused": v, "fused_count_export_ms": ms, "GBps": 8 * total / ms / 1e6}),
                  flush=True)
        for k in ("PLUSS_UNROLL", "PLUSS_GRID", "PLUSS_NT"):
            os.environ.pop(k, None)

        dense = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev)
        for v in [{}, dict(PLUSS_LANES="0"), dict(PLUSS_LEGACY="1"), dict(PLUSS_GRID="768"), dict(PLUSS_GRID="512"), dict(PLUSS_GRID="2048"),
                  dict(PLUSS_PREF="2"), dict(PLUSS_PREF="2", PLUSS_GRID="512"), dict(PLUSS_PREF="3"),
                  dict(PLUSS_UNROLL="1"), dict(PLUSS_DROWS="8"), dict(PLUSS_DROWS="16"),
                  dict(PLUSS_DROWS="64"), dict(PLUSS_BS="1024"), dict(PLUSS_BS="1024", PLUSS_GRID="512"),
                  dict(PLUSS_NT="0"), dict(PLUSS_UNROLL="4")] + [dict(PLUSS_AUX=a) for a in
                                                                  ("0", "1", "2", "3", "16", "17", "18", "19")]:
            for k in ("PLUSS_UNROLL", "PLUSS_GRID", "PLUSS_NT", "PLUSS_LEGACY", "PLUSS_DROWS", "PLUSS_BS", "PLUSS_AUX",
                      "PLUSS_LANES", "PLUSS_PREF"):
                os.environ.pop(k, None)
            os.environ.update(v)
            ms = timeit(lambda: ctx.sampled_hist_dense(buf.data_ptr(), total, dense.data_ptr(), s.cuda_stream), s)
            print(json.dumps({"samples": total, "dense": v, "dense_ms": ms, "GBps": 8 * total / ms / 1e6}),
                  flush=True)
        for k in ("PLUSS_UNROLL", "PLUSS_GRID", "PLUSS_NT", "PLUSS_LEGACY", "PLUSS_DROWS", "PLUSS_BS", "PLUSS_AUX",
                      "PLUSS_LANES", "PLUSS_PREF"):
            os.environ.pop(k, None)
        torch.cuda.synchronize()
        assert int(dense[:P.DENSE_BINS].sum()) == total and int(dense[P.DENSE_BINS]) == 0

        def two():
            ctx.sampled_hist(buf.data_ptr(), total, s.cuda_stream)
            ctx.export_reset(keys.data_ptr(), cnts.data_ptr(), 4096, s.cuda_stream)
        ms = timeit(two, s)
        print(json.dumps({"samples": total, "count_then_export_reset_ms": ms, "GBps": 8 * total / ms / 1e6}),
              flush=True)
        dst = torch.empty_like(buf)
        ms = timeit(lambda: dst.copy_(buf), s)
        print(json.dumps({"samples": total, "torch_copy_ms": ms, "GBps_rd+wr": 16 * total / ms / 1e6}), flush=True)
        ctx.reset(s.cuda_stream)
        ctx.sampled_hist(buf.data_ptr(), total, s.cuda_stream)
        h = ctx.fetch()
        assert h.total() == total
        ctx.close()


if __name__ == "__main__":
    main()
