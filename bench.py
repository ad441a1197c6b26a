#!/usr/bin/env python
"""bench.py — throughput of the PLUSS sampled reuse-interval hot path on MI355X.

Workload (BASELINE.json configs[1]): GEMM N=1024,
8 simulated threads, chunk 4, DS=8, CLS=64, clean mode, 2^24 sampled
accesses per GPU (default per-reference split, keyed Feistel sample lists).
One step = one launch of the sampling kernel over the resident sample list
that leaves this pass's complete histogram -- the dense vector of
(ref, case) counts, pluss_dev_sampled_hist_dense -- in HBM and its own
state zeroed for the next pass; with N>1 GPUs the step also all-reduces the
per-GPU vectors over RCCL (the only exchange of the path).  Samples are
sharded across ranks with no other communication, so per-GPU work is fixed
(weak scaling).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import pluss_sampler_optimization_amd as P  # noqa: E402

METRIC = "sampled accesses/sec (node) at 1/2/4/8 MI355X; HBM roofline %; MRC abs err"
SEED = 0x5EED0001
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_PER_SAMPLE = 8   # one packed u64 sample descriptor read once

CONFIGS = {
    "config2": dict(n=1024, threads=8, per_gpu=1 << 24,
                    workload="GEMM N=1024, 8 simulated threads, chunk 4, 2^24 sampled accesses per GPU (clean)"),
    "config4": dict(n=2048, threads=64, per_gpu=1 << 24,
                    workload="GEMM N=2048, 64 simulated threads, chunk 4, 2^24 sampled accesses per GPU (clean)"),
    # north_star's target: 2^28 samples in total, split over the ranks (strong scaling)
    "config3": dict(n=4096, threads=8, total=1 << 28,
                    workload="GEMM N=4096, 8 simulated threads, chunk 4, 2^28 sampled accesses in total (clean)"),
}


def shard(counts, rank, world):
    """Contiguous slice of each reference's sample-index range for this rank."""
    out = []
    for c in counts:
        lo, hi = c * rank // world, c * (rank + 1) // world
        out.append((lo, hi - lo))
    return out


def cpu_baseline(cfg, host_samples, target_s):
    """The reference's per-sample replay (stepping oracle, one host thread per
    core) on a bounded, evenly strided sub-sample of the same list."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    orc.build()
    threads = max(1, min(16, os.cpu_count() or 1))
    oc = orc.cfg(cfg.n, cfg.threads, cfg.chunk, cfg.ds, cfg.cls)
    rng = np.random.default_rng(1)
    pilot = host_samples[rng.choice(len(host_samples), 512, replace=False)]
    t = time.perf_counter()
    orc.clean_ri(oc, pilot, nthreads=threads)
    per = (time.perf_counter() - t) / len(pilot)
    n = int(min(len(host_samples), max(2048, target_s / max(per, 1e-9))))
    stride = max(1, len(host_samples) // n)
    sub = host_samples[::stride][:n]
    t = time.perf_counter()
    orc.clean_ri(oc, sub, nthreads=threads)
    dt = time.perf_counter() - t
    return {"value": len(sub) / dt, "unit": "sampled accesses/s", "cores": threads, "kind": "port",
            "sample": f"every {stride}th sample of the rank-0 list ({len(sub)} samples, all six references), "
                      f"stepping replay of each sample's simulated thread (oracle/pluss_oracle.c orc_clean), "
                      f"{dt:.1f} s wall on {threads} host threads"}


def closed_form_hist(cfg, host):
    """Independent restatement of the per-sample rules (numpy) for the MRC check."""
    s = host.astype(np.uint64)
    m = np.uint64(0xFFFFF)
    refs = (s >> np.uint64(60)).astype(np.int64)
    c0 = ((s >> np.uint64(40)) & m).astype(np.int64)
    c1 = ((s >> np.uint64(20)) & m).astype(np.int64)
    c2 = (s & m).astype(np.int64)
    N, T, CS, W = cfg.n, cfg.threads, cfg.chunk, cfg.cls // cfg.ds
    S = 4 * N + 2
    p = c0 % CS
    nxt = np.where(p != CS - 1, c0 + 1, c0 + 1 + (T - 1) * CS)
    ri = np.select([refs == 0, refs == 1, refs == 4,
                    (refs == 5) & (c2 < N - 1), (refs == 5) & (c1 % W != W - 1), refs == 5,
                    (refs == 2) & (c2 % W != W - 1), (refs == 2) & (c1 + 1 < N), refs == 2,
                    (refs == 3) & (c1 % W != W - 1), (refs == 3) & (nxt < N), refs == 3],
                   [1, 3, 1, 3, 1, -1, 4, S - 4 * (W - 1), -1, S, N * S - (W - 1) * S, -1])
    kind = ((refs == 3) & (ri > 0) & (2 * ri > (4 * N + 2) * N)).astype(np.int64)
    keys = (refs * 4 + kind) * (1 << 40) + (ri + 2)
    u, cnt = np.unique(keys, return_counts=True)
    return P.Histogram({(P.REFS[int(k >> 42)], int((k >> 40) & 3), int(k & ((1 << 40) - 1)) - 2): int(n)
                        for k, n in zip(u, cnt)})


def mrc_check(cfg, h, samples):
    """MRC abs err: r10 host pipeline (CRI -> log2 merge -> AET) on the device
    histogram vs on an independent closed-form histogram of the same samples
    (with N>1 GPUs: rank 0's shard)."""
    from pluss_sampler_optimization_amd import host as H
    ref = closed_form_hist(cfg, samples.cpu().numpy().view(np.uint64))
    assert h.total() == ref.total(), (h.total(), ref.total())
    _, _, m_gpu = H.mrc_from_r10(cfg.threads, h)
    _, _, m_ref = H.mrc_from_r10(cfg.threads, ref)
    keys = set(m_gpu) | set(m_ref)
    return max(abs(m_gpu.get(k, 0.0) - m_ref.get(k, 0.0)) for k in keys)


def fulltrace_bench(device, stream):
    """BASELINE config 5: full trace (sampling rate 1.0) GEMM N=512, T=4: back-to-back
    launches accumulating into one histogram, timed by HIP events on their stream."""
    cfg = P.SamplerConfig(n=512, threads=4, thr_variant="v1", device=device)
    reps = 20
    with P.Context(cfg) as ctx:
        ctx.fulltrace(stream.cuda_stream)
        ctx.reset(stream.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            ctx.fulltrace(stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        dt = e0.elapsed_time(e1) * 1e-3 / reps
        h = ctx.fetch()
    acc = 512 * 512 * (4 * 512 + 2)
    assert h.total() == acc * reps and h.traversed[0] == acc * reps
    return {"workload": "GEMM N=512, T=4, full trace (every access evaluated)", "accesses": acc,
            "ms": dt * 1e3, "accesses_per_s": acc / dt,
            "kernel": "pluss::k_fulltrace_count<true> (ballot counting; HIP events over 20 launches)"}


def faithful_bench(cfg, samples, stream):
    """FAITHFUL mode (r10 queue semantics: sort + scans) over the same 2^24 list: the six
    sampler_<REF> at once (pluss_dev_faithful_hist_refs, one stream per reference, as r10
    runs one thread per reference), and one after another for comparison."""
    fcfg = P.SamplerConfig(n=cfg.n, threads=cfg.threads, chunk=cfg.chunk, mode="faithful", device=cfg.device)
    counts = P.default_counts(cfg.n, len(samples))
    out = {"samples": len(samples)}
    with P.Context(fcfg) as ctx:
        def concurrent():
            ctx.reset(stream.cuda_stream)
            ctx.faithful_hist_refs(samples.data_ptr(), counts, stream.cuda_stream)

        def serial():
            ctx.reset(stream.cuda_stream)
            off = 0
            for r, c in enumerate(counts):
                ctx.faithful_hist(r, samples.data_ptr() + 8 * off, c, stream.cuda_stream)
                off += c
        hs = {}
        for name, run in (("concurrent", concurrent), ("serial", serial)):
            run()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / 3
            hs[name] = ctx.fetch()
            out[name + "_ms"] = dt * 1e3
    h = hs["concurrent"]
    assert h.bins == hs["serial"].bins and list(h.traversed) == list(hs["serial"].traversed)
    out.update({"ms": out["concurrent_ms"], "samples_per_s": len(samples) / (out["concurrent_ms"] * 1e-3),
                "recorded": h.total() - sum(h.cold(r) for r in P.REFS), "max_traversed": max(h.traversed)})
    return out


def pmc_traffic(samples_per_launch):
    """Per-launch HBM bytes of the hot kernel from the committed rocprofv3 --pmc
    summary, if it was taken at this launch size (tools/prof_round.sh)."""
    path = os.path.join(ROOT, "profiles", "pmc_sampled_hist.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    return d.get("hbm_bytes_per_launch") if d.get("samples_per_launch") == samples_per_launch else None


def allreduce_cpu(t):
    out = t.cpu()
    dist.all_reduce(out)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="config2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=20,
                    help="steps per captured HIP graph for the timed region (0: eager launches)")
    ap.add_argument("--allreduce", action="store_true",
                    help="rehearsal: run the merge all-reduce even at world size 1 (with or without torch.distributed.run)")
    ap.add_argument("--no-extras", action="store_true", help="skip the full-trace / faithful side measurements")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend (nccl = RCCL over xGMI; gloo only to rehearse N>1 on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    local = local % max(1, torch.cuda.device_count())  # rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local)
    if world > 1 or args.allreduce:
        if world == 1:  # --allreduce without a launcher: a one-rank group on the loopback address
            for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29531")):
                os.environ.setdefault(k, v)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    spec = CONFIGS[args.config]
    cfg = P.SamplerConfig(n=spec["n"], threads=spec["threads"], chunk=4, ds=8, cls=64, mode="clean", device=local)
    total = spec["total"] if "total" in spec else spec["per_gpu"] * world
    counts = P.default_counts(cfg.n, total)
    parts = shard(counts, rank, world)
    n_local = sum(c for _, c in parts)

    dev = torch.device("cuda", local)
    # a dedicated stream: the HIP events below and the library's launches must
    # share it (the null stream would make the library use its own stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    samples = torch.empty(n_local, dtype=torch.int64, device=dev)
    # two output vectors: step k writes dense[k % 2] while the all-reduce of
    # step k-1 (N>1) may still be running on RCCL's stream
    dense = [torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev) for _ in range(2)]
    pending = [None, None]
    nsteps = [0]
    ctx = P.Context(cfg)
    off = 0
    for ref, (lo, cnt) in enumerate(parts):
        ctx.expand(SEED, ref, lo, cnt, samples.data_ptr() + 8 * off, sp)
        off += cnt
    torch.cuda.synchronize()

    def enqueue(k):
        """Enqueue k steps.  Step s (global count) writes dense[s % 2]: one
        launch counts every sample; the last adder of each bin writes this
        pass's total to the vector and zeroes the kernel's state for the next
        pass.  N>1: the vector is then summed over the ranks."""
        for _ in range(k):
            i = nsteps[0] % 2
            nsteps[0] += 1
            if pending[i] is not None:  # the all-reduce that last read dense[i] (stream-ordered wait)
                pending[i].wait()
                pending[i] = None
            ctx.sampled_hist_dense(samples.data_ptr(), n_local, dense[i].data_ptr(), sp)
            if world > 1 or args.allreduce:  # element-wise sum of the per-GPU vectors (counts < 2^63)
                if args.backend == "nccl":
                    # asynchronous: RCCL's stream waits for this launch, and the
                    # next step's launch overlaps the collective
                    pending[i] = dist.all_reduce(dense[i], async_op=True)
                else:
                    dense[i].copy_(allreduce_cpu(dense[i]))
        for j in range(2):  # join: every all-reduce of these steps is complete (stream-ordered)
            if pending[j] is not None:
                pending[j].wait()
                pending[j] = None
        return (nsteps[0] - 1) % 2  # the vector of the last step

    ctx.reset(sp)
    enqueue(args.warmup)
    # The timed steps are replayed from HIP graphs of G steps (kernel launches
    # and, N>1, the all-reduces with their double-buffer dependencies): one
    # graph launch per G steps instead of a Python launch + a c10d call per
    # step, whose host cost alone (~25 us per all-reduce) exceeds a 21 us step.
    # Each graph is replayed once, untimed, before timing (its upload).
    graphs = []  # (graph, steps, vector of its last step)
    launch_mode = "eager"
    if args.graph and args.backend == "nccl":
        G = min(args.steps, args.graph)
        try:
            for size in ([G] if args.steps % G == 0 else [G, args.steps % G]):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
                    last = enqueue(size)
                g.replay()
                graphs.append((g, size, last))
            launch_mode = f"hipGraph replay, {G} steps per graph"
        except Exception as e:  # capture refused: time the same steps eagerly, and say so
            print(f"bench: graph capture failed ({e!r}); timing eager launches", file=sys.stderr)
            torch.cuda.synchronize()
            graphs = []
            launch_mode = "eager (graph capture failed)"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on the library's stream bracket the timed region: with one
    # launch per step (N=1) their span / K is the kernel's average duration
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    if graphs:
        g, size, last = graphs[0]
        for _ in range(args.steps // size):
            g.replay()
        if len(graphs) > 1:
            g, size, last = graphs[1]
            g.replay()
    else:
        last = enqueue(args.steps)  # every step's all-reduce is inside the timed region
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kern_ms = e0.elapsed_time(e1) / args.steps
    # correctness of the (merged) histogram: every sample of every rank is counted once
    dv = dense[last].cpu().numpy()  # the last step's (merged) histogram
    assert dv[P.DENSE_BINS] == 0, "malformed samples"
    h = P.hist_from_dense(cfg, dv)
    assert h.total() == total, (h.total(), total)

    achieved = BYTES_PER_SAMPLE * n_local / (kern_ms * 1e-3) / 1e9
    result = {
        "metric": METRIC,
        "value": total * args.steps / elapsed,
        "unit": "sampled accesses/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if "total" in spec else "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: keyed cycle-walking Feistel sample lists (seed 0x5EED0001), indices in [0,N-2]",
        "config": {"workload": spec["workload"], "N": cfg.n, "threads": cfg.threads, "chunk": 4, "ds": 8,
                   "cls": 64, "mode": "clean", "samples_per_gpu": n_local, "global_samples": total,
                   "parallelism": f"sample-shard x{world}" + (
                       f" + {'RCCL' if args.backend == 'nccl' else 'gloo'} all_reduce of the dense histogram"
                       if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(n_local)},
        "kernel": {"name": "pluss::k_count<true,true,true,TAIL_DENSE,2> (per-lane integer case tests on full "
                           "uniform steps, ballots otherwise; nt buffer loads; dense tail)",
                   "avg_ms": kern_ms, "timing": "HIP events on the launch stream around the K timed steps / K"
                   + (" (includes the overlapped all-reduces)" if world > 1 else ""),
                   "bytes_per_launch": BYTES_PER_SAMPLE * n_local},
        "launch": launch_mode,
        "histogram_bins": len(h.bins),
    }
    if rank == 0:
        if world > 1:  # the MRC check needs this rank's own histogram: one more (untimed) local pass
            local_dense = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev)
            ctx.sampled_hist_dense(samples.data_ptr(), n_local, local_dense.data_ptr(), sp)
            h = P.hist_from_dense(cfg, local_dense.cpu().numpy())
        result["mrc_abs_err"] = mrc_check(cfg, h, samples)
    if rank == 0 and world == 1 and not args.no_extras:
        result["fulltrace"] = fulltrace_bench(local, stream)
        result["faithful"] = faithful_bench(cfg, samples, stream)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = samples.cpu().numpy().view(np.uint64)
        result["cpu_baseline"] = cpu_baseline(cfg, host, args.cpu_seconds)
    else:
        result["cpu_baseline"] = None
    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
