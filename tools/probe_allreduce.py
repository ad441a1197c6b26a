"""Host-overhead probe for the N>1 bench step on one GPU (world size 1 over RCCL).

Times three shapes of the multi-GPU step with the same dense-histogram launch:
  eager   : launch + dist.all_reduce(async) per step (what bench.py does)
  graph   : G steps (launch + all_reduce) captured into one HIP graph, replayed
  launch  : the launch alone
Run: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/probe_allreduce.py
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pluss_sampler_optimization_amd as P  # noqa: E402


def main():
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    cfg = P.SamplerConfig(n=1024, threads=8, chunk=4, ds=8, cls=64, mode="clean", device=0)
    total = 1 << 24
    counts = P.default_counts(cfg.n, total)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    samples = torch.empty(total, dtype=torch.int64, device=dev)
    ctx = P.Context(cfg)
    off = 0
    for ref, cnt in enumerate(counts):
        ctx.expand(0x5EED0001, ref, 0, cnt, samples.data_ptr() + 8 * off, sp)
        off += cnt
    dense = [torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev) for _ in range(2)]
    ctx.reset(sp)
    torch.cuda.synchronize()
    K = 400

    def run(body, k):
        for _ in range(20):
            body()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            body()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    out = {}
    out["launch_us"] = run(lambda: ctx.sampled_hist_dense(samples.data_ptr(), total, dense[0].data_ptr(), sp), K)
    st = [0]

    def eager():
        i = st[0] % 2
        st[0] += 1
        ctx.sampled_hist_dense(samples.data_ptr(), total, dense[i].data_ptr(), sp)
        dist.all_reduce(dense[i], async_op=True).wait()

    out["eager_us"] = run(eager, K)

    def host_only():
        dist.all_reduce(dense[0], async_op=True).wait()

    out["allreduce_only_us"] = run(host_only, K)
    G = 10
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for j in range(G):
                ctx.sampled_hist_dense(samples.data_ptr(), total, dense[j % 2].data_ptr(), sp)
                dist.all_reduce(dense[j % 2])
        out["graph_us_per_step"] = run(g.replay, K // G) / G
    except Exception as e:  # report, do not hide
        out["graph_error"] = repr(e)[:300]
    torch.cuda.synchronize()
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
