#!/usr/bin/env python
"""bench.py — throughput of the PLUSS sampled reuse-interval hot path on MI355X.

Workload (BASELINE.json configs[2], the metric's headline; SURVEY.md §8d
config 3): GEMM N=4096, 8 simulated threads, chunk 4, DS=8, CLS=64, clean
mode, 2^28 sampled accesses IN TOTAL, split over the ranks (strong scaling:
--gpus 1 puts all 2^28 on one GPU).  Per-reference keyed Feistel sample lists
are expanded on the device and resident in HBM before timing.

One step = one launch of the sampling kernel over the rank's resident list
that leaves this pass's complete histogram -- the dense vector of (ref, case)
counts, pluss_dev_sampled_hist_dense -- in HBM and its own state zeroed for
the next pass; with N>1 GPUs the step also all-reduces the 19-word vectors
over RCCL (the only exchange of the path).  In the reference the whole
sampler pass is the timed unit (r10:3199-3278).

    python bench.py [--gpus N --steps K --warmup W]      (N>1: spawns N ranks)
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

METRIC = "sampled accesses/sec (node) at 1/2/4/8 MI355X; HBM roofline %; MRC abs err"
SEED = 0x5EED0001
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_PER_SAMPLE = 8   # one packed u64 sample descriptor read once

CONFIGS = {
    # north_star's target and the metric's headline: 2^28 samples in total, split over the ranks
    "config3": dict(n=4096, threads=8, total=1 << 28,
                    workload="GEMM N=4096, 8 simulated threads, chunk 4, 2^28 sampled accesses in total (clean)"),
    "config2": dict(n=1024, threads=8, per_gpu=1 << 24,
                    workload="GEMM N=1024, 8 simulated threads, chunk 4, 2^24 sampled accesses per GPU (clean)"),
    "config4": dict(n=2048, threads=64, per_gpu=1 << 24,
                    workload="GEMM N=2048, 64 simulated threads, chunk 4, 2^24 sampled accesses per GPU (clean)"),
}


_KEPT_GRAPHS = []  # HIP graphs kept alive until the process exits (r5m)

def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="config3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=20,
                    help="steps per captured HIP graph for the timed region (0: eager launches)")
    ap.add_argument("--allreduce", action="store_true",
                    help="rehearsal: run the merge all-reduce even at world size 1")
    ap.add_argument("--no-extras", action="store_true", help="skip the side measurements (full trace, faithful, MRC)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend (nccl = RCCL over xGMI; gloo only to rehearse N>1 on one GPU)")
    return ap.parse_args()


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """--gpus N>1 without a launcher: start N rank processes (one per GPU) and
    wait for them.  Runs before this process touches the GPU (nothing here has
    imported the library or called into HIP), so no GPU-initialised process
    is ever replaced; the children do the work and rank 0 prints the line."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # a rank that fails would leave the others waiting in a collective: stop them
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


def shard(counts, rank, world):
    """Contiguous slice of each reference's sample-index range for this rank."""
    out = []
    for c in counts:
        lo, hi = c * rank // world, c * (rank + 1) // world
        out.append((lo, hi - lo))
    return out


def host_cores():
    """Host cores this job may use: the affinity set, capped by the cgroup CPU
    quota and by OMP_NUM_THREADS when set.  (The GPU box runs a one-GPU job on
    a share of a larger machine -- 16 cores, exported as OMP_NUM_THREADS -- while
    nproc reports the whole machine.)"""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 256))


def median_time(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2], ts


def cpu_baseline(cfg, host, ri_gpu_fn, budget_s):
    """The reference's per-sample replay (oracle/pluss_oracle.c orc_clean: each
    sample's simulated thread stepped access by access, as r10's replay does)
    on every host core, over a bounded, evenly strided sub-sample of the same
    list; median of repeated runs.  Its RIs are checked against the device's
    per-sample RI dump of the same sub-sample."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    orc.build()
    import pluss_sampler_optimization_amd as P
    threads = host_cores()
    oc = orc.cfg(cfg.n, cfg.threads, cfg.chunk, cfg.ds, cfg.cls)
    # a pilot on a strided sub-sample sizes the timed one (~budget/10 per run,
    # 10 runs, median: SURVEY §8d); the size is a power of two, so the timed
    # sub-sample is always one of a few fixed strided sets of the list
    pilot = host[:: max(1, len(host) // 512)][:512]
    t = time.perf_counter()
    orc.clean_ri(oc, pilot, nthreads=threads)
    per = (time.perf_counter() - t) / len(pilot)
    n = 1 << max(8, int(np.log2(max(2.0, budget_s / 10 / max(per, 1e-9)))))
    n = min(n, 1 << 20, len(host))
    stride = max(1, len(host) // n)
    sub = np.ascontiguousarray(host[::stride][:n])
    out = {}
    med, ts = median_time(lambda: out.__setitem__("ri", orc.clean_ri(oc, sub, nthreads=threads)), 10)
    ri_gpu = ri_gpu_fn(sub)
    assert np.array_equal(out["ri"], ri_gpu), "CPU oracle RIs differ from the device RI dump"
    return {"value": len(sub) / med, "unit": "sampled accesses/s", "cores": threads, "kind": "port",
            "sample": f"every {stride}th sample of the rank-0 list ({len(sub)} samples, all six references); "
                      f"stepping replay of each sample's simulated thread (orc_clean, the r10 per-sample "
                      f"replay restated in C), {threads} host threads, median of {len(ts)} runs "
                      f"({min(ts):.2f}-{max(ts):.2f} s); RIs equal the device dump of the same samples",
            "parity_checked_samples": len(sub)}


def cpu_fulltrace_baseline(reps=10):
    """BASELINE configs[0] (run.sh speed, N=128, T=4 full trace): the full-trace
    oracle with one host thread per simulated tid (as rayon_sampler runs one task
    per tid, src/gemm_sampler_rayon.rs:107-126), median of `reps` runs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    orc.build()
    res = {}
    med, ts = median_time(lambda: res.__setitem__("h", orc.fulltrace_mt(128, 4, thr_variant=1)), reps)
    h, trav = res["h"]
    assert trav == 128 * 128 * (4 * 128 + 2)
    return {"workload": "GEMM N=128, T=4, full trace (run.sh speed analogue)", "accesses": trav,
            "value": trav / med, "unit": "accesses/s", "cores": 4, "kind": "port",
            "sample": f"orc_fulltrace_mt, one host thread per simulated tid, median of {reps} runs "
                      f"({min(ts) * 1e3:.1f}-{max(ts) * 1e3:.1f} ms)"}


def mrc_vs_reference(device):
    """MRC abs err against the reference's own printouts: every committed r10 dump
    (tests/golden, N=64..256) replayed through FAITHFUL mode on the device and the
    host r10 pipeline (CRI -> log2 merge -> AET); max |MRC - printed MRC| over all
    printed rows.  The printouts hold 6 significant digits."""
    import glob
    import numpy as np
    import pluss_sampler_optimization_amd as P
    from pluss_sampler_optimization_amd import host as H
    order = ["C3", "C2", "A0", "C0", "B0", "C1"]
    worst, rows = 0.0, 0
    for js in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "r10_*.json"))):
        d = json.load(open(js))
        z = np.load(js[:-5] + ".npz")
        s = np.concatenate([P.pack_array(r, z[r]) for r in P.REFS])
        h = P.sampled_hist(P.SamplerConfig(n=d["N"], threads=d["T"], mode="faithful", device=device), s)
        per = {r: H.r10_sampler_output(d["T"], {k: v for k, v in h.bins.items() if k[0] == r}) for r in order}
        mrc = H.aet(H.log2_merge(*[per[r] for r in order]))
        got = [[float(x) for x in line.split(",")] for line in H.format_mrc(mrc).splitlines()[1:]]
        want = d["printed"]["mrc"]
        assert len(got) == len(want) and all(g[0] == w[0] for g, w in zip(got, want)), js
        full = dict(mrc)
        worst = max([worst] + [abs(full.get(int(w[0]), g[1]) - w[1]) for g, w in zip(got, want)])
        rows += len(want)
    return {"max_abs_err_vs_reference_printout": worst, "rows": rows,
            "fixtures": "tests/golden/r10_*.json (7 reference r10 runs, N=64/128/256, T=2/4/8)",
            "note": "printout precision is 6 significant digits; agreement with real GSL to 1e-9 is unpinned "
                    "(GSL absent); at BASELINE sizes the MRC is computed by the same host code from histograms "
                    "that are bit-exact (parity tests)"}


def fulltrace_bench(P, torch, device, stream):
    """BASELINE config 5: full trace (sampling rate 1.0) GEMM N=512, T=4 (and
    config 1's N=128 for the CPU comparison): back-to-back launches accumulating
    into one histogram, timed by HIP events on their stream."""
    out = {}
    for N, reps in ((512, 20), (128, 50)):
        cfg = P.SamplerConfig(n=N, threads=4, thr_variant="v1", device=device)
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
        acc = N * N * (4 * N + 2)
        assert h.total() == acc * reps and h.traversed[0] == acc * reps
        out[f"N{N}"] = {"workload": f"GEMM N={N}, T=4, full trace (every access evaluated)", "accesses": acc,
                        "ms": dt * 1e3, "accesses_per_s": acc / dt}
    out["kernel"] = "pluss::k_fulltrace_count<true> (ballot counting; HIP events over back-to-back launches)"
    return out


def faithful_bench(P, torch, device, stream):
    """FAITHFUL mode (r10 queue semantics) at config 2 (N=1024, T=8, 2^24
    samples), the six sampler_<REF> at once (one stream per reference, as r10
    runs one thread per reference):
      radix:     the Feistel list (arbitrary order): the hand-written bucket sort
                 of the six references (csrc/pluss_sort.h) -> the single-read
                 scan pipeline (pluss_dev_faithful_hist_refs);
      sorted:    the key-order list (pluss_dev_expand_sorted) read once, no sort
                 (pluss_dev_faithful_hist_sorted_refs): 8 B per sample;
      generated: the same key-order lists generated inside the pass, no input
                 (pluss_dev_gen_faithful_refs)."""
    fcfg = P.SamplerConfig(n=1024, threads=8, mode="faithful", device=device)
    total = 1 << 24
    counts = P.default_counts(1024, total)
    dev = torch.device("cuda", device)
    feistel = torch.empty(total, dtype=torch.int64, device=dev)
    keyord = torch.empty(total, dtype=torch.int64, device=dev)
    sp = stream.cuda_stream
    out = {"workload": "GEMM N=1024, T=8, 2^24 samples (config 2 budget), faithful, six references concurrently",
           "samples": total}
    with P.Context(fcfg) as ctx:
        off = 0
        for r, c in enumerate(counts):
            ctx.expand(SEED, r, 0, c, feistel.data_ptr() + 8 * off, sp)
            ctx.expand_sorted(SEED, r, c, 0, c, keyord.data_ptr() + 8 * off, sp)
            off += c
        runs = {"radix": lambda: ctx.faithful_hist_refs(feistel.data_ptr(), counts, sp),
                "sorted": lambda: ctx.faithful_hist_sorted_refs(keyord.data_ptr(), counts, sp),
                "generated": lambda: ctx.gen_faithful_refs(SEED, counts, sp)}
        hs = {}
        for name, run in runs.items():
            ctx.reset(sp)
            run()
            torch.cuda.synchronize()
            hs[name] = ctx.fetch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                run()
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            out[name] = {"ms": ms, "samples_per_s": total / (ms * 1e-3)}
    # the key-order list through both of its paths gives one histogram
    assert hs["sorted"].bins == hs["generated"].bins and list(hs["sorted"].traversed) == list(hs["generated"].traversed)
    out["sorted"]["hbm_GBps"] = 8 * total / (out["sorted"]["ms"] * 1e-3) / 1e9
    # the sorted pass reads its 8 B per sample once (algorithmic bytes); HBM
    # traffic per pass from the committed PMC summary (tools/pmc_faithful_summary.py)
    traffic = None
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_faithful.json")))
        if d.get("samples_per_pass") == total:
            traffic = d.get("hbm_bytes_per_pass")
    except (OSError, ValueError):
        pass
    ach = out["sorted"]["hbm_GBps"]
    out["sorted"]["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                                 "note": "achieved = 8 B x samples / pass time (the whole pipeline, six references); "
                                         "traffic = HBM bytes of one pass (PMC)"}
    out["sorted"]["recorded"] = hs["sorted"].total() - sum(hs["sorted"].cold(r) for r in P.REFS)
    out["radix"]["recorded"] = hs["radix"].total() - sum(hs["radix"].cold(r) for r in P.REFS)
    out["note"] = ("radix = arbitrary-order input (sort inside the pass); sorted = input already in r10's pop "
                   "order, checked in-kernel; generated = the key-order list made inside the pass")
    return out


def faithful_config3_bench(P, torch, device, stream, reps=20):
    """FAITHFUL mode (r10's queue semantics, bit-exact with the reference's
    sampler_<REF> on the same sample list) at the headline shape: N=4096,
    T=8, 2^28 samples on one GPU, six references concurrently.  sorted = the
    key-order list resident in HBM, read once per pass (8 B per sample);
    generated = the same lists generated inside the pass; radix = r10's real
    input, a list in arbitrary order (the keyed Feistel lists, as rand() draws
    them, r10:156-185), sorted inside the pass; uniform = r10's distribution
    generated in key order inside the pass (pluss_dev_gen_uniform_faithful_refs)."""
    N, T, total = 4096, 8, 1 << 28
    counts = P.default_counts(N, total)
    fcfg = P.SamplerConfig(n=N, threads=T, mode="faithful", device=device)
    dev = torch.device("cuda", device)
    buf = torch.empty(total, dtype=torch.int64, device=dev)
    fe = torch.empty(total, dtype=torch.int64, device=dev)
    sp = stream.cuda_stream
    out = {"workload": "GEMM N=4096, T=8, 2^28 samples (config 3 on one GPU), faithful, six references",
           "samples": total}
    with P.Context(fcfg) as ctx:
        off = 0
        for r, c in enumerate(counts):
            ctx.expand_sorted(SEED, r, c, 0, c, buf.data_ptr() + 8 * off, sp)
            ctx.expand(SEED, r, 0, c, fe.data_ptr() + 8 * off, sp)
            off += c
        runs = {"sorted": (lambda: ctx.faithful_hist_sorted_refs(buf.data_ptr(), counts, sp), reps),
                "generated": (lambda: ctx.gen_faithful_refs(SEED, counts, sp), reps),
                "radix": (lambda: ctx.faithful_hist_refs(fe.data_ptr(), counts, sp), reps),
                "uniform": (lambda: ctx.gen_uniform_faithful_refs(SEED, counts, sp), reps)}
        hs = {}
        for name, (run, k) in runs.items():
            ctx.reset(sp)
            run()
            torch.cuda.synchronize()
            hs[name] = ctx.fetch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(k):
                run()
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / k
            out[name] = {"ms": ms, "samples_per_s": total / (ms * 1e-3)}
    out["radix"]["recorded"] = hs["radix"].total() - sum(hs["radix"].cold(r) for r in P.REFS)
    out["radix"]["over_sorted"] = out["radix"]["ms"] / out["sorted"]["ms"]
    out["uniform"]["recorded"] = hs["uniform"].total() - sum(hs["uniform"].cold(r) for r in P.REFS)
    out["uniform"]["note"] = ("r10's own distribution (uniform draw without replacement, r10:156-185) generated in "
                              "key order inside the pass: plan + tile staging, no list in memory, no sort")
    del buf, fe
    assert hs["sorted"].bins == hs["generated"].bins and list(hs["sorted"].traversed) == list(hs["generated"].traversed)
    ach = 8 * total / (out["sorted"]["ms"] * 1e-3) / 1e9
    traffic = None  # HBM bytes per pass from the committed PMC summary (tools/gpu_pmc_faithful.sh, PROF_SHAPE=config3)
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_faithful_config3.json")))
        if d.get("samples_per_pass") == total:
            traffic = d.get("hbm_bytes_per_pass")
    except (OSError, ValueError):
        pass
    out["sorted"]["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                                 "note": "achieved = 8 B x samples / pass time (the whole pipeline, six references); "
                                         "traffic = HBM bytes of one pass: the samples read once plus the per-tile "
                                         "summaries and local-start lists"}
    out["recorded"] = hs["sorted"].total() - sum(hs["sorted"].cold(r) for r in P.REFS)
    out["traversed"] = list(hs["sorted"].traversed)
    return out


def faithful_pipeline_bench(P, torch, device, stream, reps=3):
    """r10's whole timed unit (r10:3199-3278) at BASELINE shapes, end to end:
    the six references' sample lists generated, the six sampler_<REF>
    (faithful mode, r10's queue semantics), the raw histograms fetched, then on
    the host r10's per-reference CRI (no_share_distribute + share_distribute,
    pluss_cri_r10), the floor-log2 merge into the reuse histogram, pluss_AET
    and the MRC printout.  Sources of the lists:
      feistel_radix: uniform lists in arbitrary order (r10's rand() draw,
                     r10:156-185), generated on the device and sorted inside the
                     pass (the radix source);
      uniform:       r10's distribution generated in key order inside the pass
                     (pluss_dev_gen_uniform_faithful_refs: no list, no sort);
      generated:     key-order stratified lists generated inside the pass.
    Host clock around everything, median of `reps`; `host_share` = the CRI ->
    MRC text part's fraction."""
    from pluss_sampler_optimization_amd import host as H
    out = {}
    sp = stream.cuda_stream
    dev = torch.device("cuda", device)
    for name, N, total in (("config2", 1024, 1 << 24), ("config3", 4096, 1 << 28)):
        counts = P.default_counts(N, total)
        fcfg = P.SamplerConfig(n=N, threads=8, mode="faithful", device=device)
        buf = torch.empty(total, dtype=torch.int64, device=dev)
        res = {"workload": f"GEMM N={N}, T=8, {total} samples (BASELINE {name} budget on one GPU), faithful"}
        with P.Context(fcfg) as ctx:
            def feistel_radix():
                off = 0
                for r, c in enumerate(counts):
                    ctx.expand(SEED, r, 0, c, buf.data_ptr() + 8 * off, sp)
                    off += c
                ctx.faithful_hist_refs(buf.data_ptr(), counts, sp)

            def generated():
                ctx.gen_faithful_refs(SEED, counts, sp)

            def uniform():
                ctx.gen_uniform_faithful_refs(SEED, counts, sp)
            for src, dev_part in (("feistel_radix", feistel_radix), ("uniform", uniform), ("generated", generated)):
                runs = []
                for k in range(reps + 1):  # the first run warms (code load, buffers)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    ctx.reset(sp)
                    dev_part()
                    h = ctx.fetch()  # waits for the device; the raw histograms on the host
                    t1 = time.perf_counter()
                    _, text = H.mrc_text_from_r10(8, h)
                    t2 = time.perf_counter()
                    if k:
                        runs.append((t2 - t0, t2 - t1))
                runs.sort()
                tot_s, host_s = runs[len(runs) // 2]
                res[src] = {"ms": tot_s * 1e3, "host_ms": host_s * 1e3, "host_share": host_s / tot_s,
                            "samples_per_s": total / tot_s, "mrc_rows": len(text.splitlines()) - 1,
                            "recorded": h.total() - sum(h.cold(r) for r in P.REFS)}
        del buf
        out[name] = res
    out["note"] = ("one pass of r10's timer: lists -> six faithful samplers -> fetch -> pluss_cri_r10 per reference "
                   "-> log2 merge -> pluss_aet (the reference's walk, 327,681 cache sizes) -> MRC text "
                   "(host.mrc_text_from_r10); host clock, median of %d" % reps)
    return out


def end_to_end_bench(P, torch, cfg, counts, parts, stream, steps=20):
    """Sample generation inside the timed unit, as in r10 (r10:156-185 within the
    timer r10:3199): this rank's slices of the six key-order lists generated and
    counted in one launch (pluss_dev_gen_count_dense; the samples never touch
    memory), and, for comparison, generated into HBM and then counted."""
    dev = torch.device("cuda", cfg.device)
    sp = stream.cuda_stream
    first = [lo for lo, _ in parts]
    n = [k for _, k in parts]
    n_local = sum(n)
    d = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev)
    d2 = torch.zeros_like(d)
    buf = torch.empty(n_local, dtype=torch.int64, device=dev)
    out = {}
    with P.Context(cfg) as ctx:
        def fused():
            ctx.gen_count_dense(SEED, counts, first, n, d.data_ptr(), sp)

        def expand():
            off = 0
            for r in range(6):
                ctx.expand_sorted(SEED, r, counts[r], first[r], n[r], buf.data_ptr() + 8 * off, sp)
                off += n[r]

        def count():
            ctx.sampled_hist_dense(buf.data_ptr(), n_local, d2.data_ptr(), sp)
        for name, fn in (("gen_count_fused", fused), ("expand_sorted", expand), ("count", count)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(steps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            out[name + "_ms"] = e0.elapsed_time(e1) / steps
    assert (d.cpu() == d2.cpu()).all(), "fused generate+count differs from expand + count"
    assert int(d[:P.DENSE_BINS].sum()) == n_local
    out["samples_per_gpu"] = n_local
    out["fused_samples_per_s"] = n_local / (out["gen_count_fused_ms"] * 1e-3)
    out["expand_then_count_samples_per_s"] = n_local / ((out["expand_sorted_ms"] + out["count_ms"]) * 1e-3)
    out["fused_over_count"] = out["gen_count_fused_ms"] / out["count_ms"]
    out["note"] = ("key-order stratified lists (pluss_expand_sorted, same per-reference budget and seed); "
                   "fused = one launch, generation + counting; count = the headline kernel over the materialised list")
    return out


def collective_costs(args, torch, dist, ctx, samples, n_local, dense, stream, reps=20):
    """N>1: the step's parts measured apart -- the kernel alone (K launches,
    no collective, HIP events on the launch stream) and one all-reduce of the
    dense vector issued eagerly and waited for (median of `reps`, host clock,
    every rank in step by a barrier first)."""
    sp = stream.cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(args.steps):
        ctx.sampled_hist_dense(samples.data_ptr(), n_local, dense[0].data_ptr(), sp)
    e1.record(stream)
    torch.cuda.synchronize()
    kernel_ms = e0.elapsed_time(e1) / args.steps
    t = dense[1] if args.backend == "nccl" else dense[1].cpu()
    ts = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.all_reduce(t)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return {"kernel_only_ms": kernel_ms, "allreduce_eager_us": ts[len(ts) // 2] * 1e6,
            "allreduce_words": int(t.numel()), "backend": args.backend,
            "note": "kernel_only_ms: the K timed launches without their all-reduces (HIP events); "
                    "allreduce_eager_us: one eager all-reduce of the dense vector and its wait, median; in the timed "
                    "steps each step's all-reduce is issued eagerly and asynchronously (no collective inside a HIP "
                    "graph), overlapped with the next launch"}


def faithful_sharded_bench(P, torch, dist, device, stream, world, reps=3):
    """N>1: FAITHFUL mode at config 3 (N=4096, T=8, 2^28 samples in total)
    over key-range shards, one per rank (dist.sharded_faithful_gen_hist): each
    rank generates the samples of its key range inside its single-read pass,
    three six-word all-gathers carry the scan across the ranks, the tables are
    merged.  Time per pass: max over ranks."""
    from pluss_sampler_optimization_amd import dist as D
    N, T, total = 4096, 8, 1 << 28
    counts = P.default_counts(N, total)
    fcfg = P.SamplerConfig(n=N, threads=T, mode="faithful", device=device)
    h = D.sharded_faithful_gen_hist(fcfg, SEED, counts, stream=stream)  # warm-up
    ts = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h = D.sharded_faithful_gen_hist(fcfg, SEED, counts, stream=stream)
        torch.cuda.synchronize()
        nccl = dist.get_backend() == "nccl"
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device=torch.device("cuda", device) if nccl else "cpu")
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        ts.append(float(dt.item()))
    ms = sorted(ts)[len(ts) // 2] * 1e3
    return {"workload": "GEMM N=4096, T=8, 2^28 samples in total (config 3), faithful, key-range shards, "
                        "lists generated inside the pass", "ranks": world, "ms": ms,
            "samples_per_s": total / (ms * 1e-3), "recorded": h.total() - sum(h.cold(r) for r in P.REFS),
            "note": "host clock around the whole sharded pass (4 phases, 3 all-gathers, table merge); median of "
                    f"{reps}, max over ranks"}


def capi_group_bench(P, torch, dist, cfg, counts, total, world, rank, backend, steps, warmup):
    """The same dense step through the C ABI's multi-GPU group (pluss_group_*,
    csrc/pluss_group.hip): the library holds the shards' resident lists, runs
    the count and the RCCL all-reduce of the 19-word vector itself (one rank
    on one device: replayed from HIP graphs of 16 steps without the identity
    all-reduce; several ranks: eager) -- what a C++ or Rust caller
    of the reference gets without torch.  N>1: one rank per process, the RCCL
    id made by rank 0 and handed over by torch.distributed.  N=1 also runs 8
    logical shards on the one GPU (SURVEY §4.4's exchange rehearsal: not a
    scaling point)."""
    def run(g, label):
        g.expand(SEED, counts)
        g.dense(warmup)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        v = g.dense(steps)
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=torch.device("cuda", cfg.device))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        ok = sum(v[:P.DENSE_BINS]) == total and v[P.DENSE_BINS] == 0
        return {"shards": g.shards()[1], "ms_per_step": el / steps * 1e3, "value": total * steps / el,
                "unit": "sampled accesses/s", "merged_vector_accounts_for_every_sample": bool(ok), "label": label}
    if world > 1:
        if backend != "nccl":
            return {"skipped": "the group's RCCL communicator needs one GPU per rank (gloo rehearsal)"}
        obj = [P.group_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        with P.Group.rank(cfg, world, rank, obj[0]) as g:
            out = run(g, f"{world} ranks x 1 shard")
    else:
        with P.Group(cfg, [cfg.device], 1) as g:
            out = run(g, "1 device x 1 shard")
        with P.Group(cfg, [cfg.device], 8) as g:
            out["logical_shards_8"] = run(g, "1 device x 8 logical shards (rehearsal)")
        out["faithful"], out["faithful_uniform"], out["faithful_any_order"] = capi_group_faithful(P, cfg)
    out["note"] = ("host clock around pluss_group_dense(K) (K passes, each a count launch per shard, the per-device "
                   "sum and one RCCL all-reduce, until the merged vector is back on the host)")
    return out


def capi_group_faithful(P, cfg, reps=3):
    """Faithful mode at config 3 (2^28 samples) through the C-ABI group on one
    device with 1, 2 and 8 logical key-range shards: generated key-order lists
    (pluss_group_gen_faithful), r10's own law (pluss_group_gen_uniform_faithful)
    and an any-order host list (pluss_group_sampled_hist, 1 and 8 shards).
    Rows exchanged between phases on the device (RCCL over several ranks; with
    one rank the exchanges are identities and a replayed pass leaves them
    out), the pass ending in the dense vector.  Host clock around the whole call,
    median of `reps` after two warm calls (the second identical gen_faithful call
    is captured into a HIP graph and replayed after); every shard count's
    histogram equals the one-shard one."""
    fcfg = P.SamplerConfig(n=4096, threads=cfg.threads, chunk=cfg.chunk, mode="faithful", device=cfg.device)
    totals = P.default_counts(4096, 1 << 28)

    def leg(call, spds=(1, 2, 8)):
        out, ref = {}, None
        for spd in spds:
            with P.Group(fcfg, [cfg.device], spd) as g:
                h = call(g)  # (the first call grows the buffers, a second identical one is captured)
                h = call(g)
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    h = call(g)
                    ts.append(time.perf_counter() - t0)
            ts.sort()
            ref = ref or h
            out[f"shards_{spd}"] = {"ms": ts[len(ts) // 2] * 1e3, "equals_one_shard": h == ref and
                                    h.traversed == ref.traversed}
        return out
    out = leg(lambda g: g.gen_faithful(SEED, totals))
    out["workload"] = "GEMM N=4096, T=8, 2^28 samples (config 3), faithful, generated key-order lists, one device"
    uni = leg(lambda g: g.gen_uniform_faithful(SEED, totals))
    uni["workload"] = ("the same over r10's own law (pluss_group_gen_uniform_faithful: uniform draws without "
                       "replacement in key order, each shard generating only its stretch of every list)")
    # r10's any-order input handed over in host memory (pinned): the keyed
    # Feistel lists, as rand() draws them (r10:156-185)
    import torch
    dev = torch.device("cuda", cfg.device)
    total = sum(totals)
    host = torch.empty(total, dtype=torch.int64, pin_memory=True)
    with P.Context(fcfg) as ctx:
        d = torch.empty(total, dtype=torch.int64, device=dev)
        st = torch.cuda.Stream(device=dev)
        off = 0
        for r, c in enumerate(totals):
            ctx.expand(SEED, r, 0, c, d.data_ptr() + 8 * off, st.cuda_stream)
            off += c
        st.synchronize()
        host.copy_(d)
        ts = []
        for _ in range(reps):  # the upload alone, for scale (the group's copy is the same bytes)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d.copy_(host, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        del d
    ts.sort()
    lst = host.numpy().view("uint64")
    anyo = leg(lambda g: g.sampled_hist(lst), spds=(1, 8))
    anyo["h2d_ms"] = ts[len(ts) // 2] * 1e3
    anyo["workload"] = ("the same shape over r10's any-order input (pluss_group_sampled_hist: a host list, the "
                        "Feistel lists in pinned memory): each device uploads its slice, partitions it by key-range "
                        "shard and reference on the device, (several devices: one grouped send/receive), each shard "
                        "sorts its words; h2d_ms = the same bytes' upload alone")
    del lst, host
    return out, uni, anyo


def pmc_traffic(samples_per_launch):
    """Per-launch HBM bytes of the hot kernel from the committed rocprofv3 --pmc
    summary, if it was taken at this launch size (tools/prof_round.sh)."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_sampled_hist.json")))
    except (OSError, ValueError):
        return None
    return d.get("hbm_bytes_per_launch") if d.get("samples_per_launch") == samples_per_launch else None


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import pluss_sampler_optimization_amd as P

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    local = local % max(1, torch.cuda.device_count())  # rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local)
    if world > 1 or args.allreduce:
        if world == 1:  # --allreduce without a launcher: a one-rank group on the loopback address
            for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"),
                         ("MASTER_PORT", str(free_port()))):
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

    def expand():  # this rank's slices of the six Feistel lists into HBM (the headline input)
        off = 0
        for ref, (lo, cnt) in enumerate(parts):
            ctx.expand(SEED, ref, lo, cnt, samples.data_ptr() + 8 * off, sp)
            off += cnt
    expand()  # the list the timed steps read (and the first, cold call: code loading, first touch)
    e_x0, e_x1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e_x0.record(stream)
    for _ in range(3):  # warm: the same list generated again (bit-identical, r10:156-185's work)
        expand()
    e_x1.record(stream)
    torch.cuda.synchronize()
    expand_ms = e_x0.elapsed_time(e_x1) / 3
    collective = world > 1 or args.allreduce

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
            if collective:  # element-wise sum of the per-GPU vectors (counts < 2^63)
                if args.backend == "nccl":
                    # asynchronous: RCCL's stream waits for this launch, and the
                    # next step's launch overlaps the collective
                    pending[i] = dist.all_reduce(dense[i], async_op=True)
                else:
                    t = dense[i].cpu()
                    dist.all_reduce(t)
                    dense[i].copy_(t)
        for j in range(2):  # join: every all-reduce of these steps is complete (stream-ordered)
            if pending[j] is not None:
                pending[j].wait()
                pending[j] = None
        return (nsteps[0] - 1) % 2  # the vector of the last step

    ctx.reset(sp)
    enqueue(args.warmup)
    # The timed steps are replayed from HIP graphs of G steps (one graph launch
    # per G steps instead of a Python launch per step) when a step holds no
    # collective.  With N>1 every step's all-reduce is issued eagerly: no RCCL
    # call is ever captured into a graph (the library's capture rule, DESIGN.md
    # section 8).  The graphs are kept alive to the end of the run: on this
    # ROCm a graph launched after another graph was destroyed crashed inside
    # the HIP runtime (r5m).
    graphs = []  # (graph, steps, vector of its last step)
    launch_mode = "eager (one c10d all_reduce per step, asynchronous)" if collective else "eager"
    if args.graph and not collective:
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

    _KEPT_GRAPHS.extend(graphs)  # (never destroyed before exit: see above)
    kern_ms = e0.elapsed_time(e1) / args.steps
    # correctness of the (merged) histogram: every sample of every rank is counted once
    dv = dense[last].cpu().numpy()  # the last step's (merged) histogram
    assert dv[P.DENSE_BINS] == 0, "malformed samples"
    h = P.hist_from_dense(cfg, dv)
    assert h.total() == total, (h.total(), total)

    # stream-read peak of this access pattern on this GPU: the same launch with
    # the same sample loads and nothing counted (pluss_diag_dense, loads only)
    scratch = torch.zeros(P.DENSE_BINS + 1, dtype=torch.int64, device=dev)
    for _ in range(3):
        ctx.diag_dense(samples.data_ptr(), n_local, scratch.data_ptr(), 1, 0, sp)
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e2.record(stream)
    for _ in range(20):
        ctx.diag_dense(samples.data_ptr(), n_local, scratch.data_ptr(), 1, 0, sp)
    e3.record(stream)
    torch.cuda.synchronize()
    loads_ms = e2.elapsed_time(e3) / 20

    collective_info = None
    if collective:
        collective_info = collective_costs(args, torch, dist, ctx, samples, n_local, dense, stream)
    capi_group = None
    if not args.no_extras:
        try:  # a side line: its failure must not cost the headline line
            capi_group = capi_group_bench(P, torch, dist, cfg, counts, total, world, rank, args.backend,
                                          args.steps, args.warmup)
        except Exception as e:  # noqa: BLE001
            capi_group = {"error": repr(e)}
    faithful_shards = None
    if world > 1 and not args.no_extras:
        try:  # a side line: its failure must not cost the headline line
            faithful_shards = faithful_sharded_bench(P, torch, dist, local, stream, world)
        except Exception as e:  # noqa: BLE001
            faithful_shards = {"error": repr(e)}

    achieved = BYTES_PER_SAMPLE * n_local / (kern_ms * 1e-3) / 1e9
    stream_peak = BYTES_PER_SAMPLE * n_local / (loads_ms * 1e-3) / 1e9
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
                       if collective else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(n_local),
                     "measured_stream_read_peak": stream_peak,
                     "frac_of_measured_peak": achieved / stream_peak},
        "kernel": {"name": "pluss::k_count<true,true,TAIL_DENSE> (per-lane integer case tests on full uniform "
                           "steps, ballots otherwise; nt buffer loads; dense tail)",
                   "avg_ms": kern_ms, "timing": "HIP events on the launch stream around the K timed steps / K"
                   + (" (includes the overlapped all-reduces)" if collective else ""),
                   "bytes_per_launch": BYTES_PER_SAMPLE * n_local,
                   "loads_only_ms": loads_ms},
        "feistel_expand_ms": expand_ms,
        "feistel_expand_then_count": {
            "ms": expand_ms + kern_ms, "samples_per_s": n_local / ((expand_ms + kern_ms) * 1e-3),
            "expand_over_step": expand_ms / kern_ms,
            "note": "the headline's own list generated on the device (k_expand, warm, mean of 3) and then counted "
                    "once: r10 draws its samples inside its timer (r10:156-185 within r10:3199)"},
        "launch": launch_mode,
        "histogram_bins": len(h.bins),
    }
    if collective_info is not None:
        result["collective"] = collective_info
    if faithful_shards is not None:
        result["faithful_sharded"] = faithful_shards
    if capi_group is not None:
        result["capi_group"] = capi_group
    if not args.no_extras:
        result["end_to_end"] = end_to_end_bench(P, torch, cfg, counts, parts, stream)
    if rank == 0 and not args.no_extras:
        result["mrc"] = mrc_vs_reference(local)
    if rank == 0 and world == 1 and not args.no_extras:
        result["fulltrace"] = fulltrace_bench(P, torch, local, stream)
        result["faithful"] = faithful_bench(P, torch, local, stream)
        try:  # a side line: its failure must not cost the headline line
            result["faithful_config3"] = faithful_config3_bench(P, torch, local, stream)
        except Exception as e:  # noqa: BLE001
            result["faithful_config3"] = {"error": repr(e)}
        try:
            result["faithful_pipeline"] = faithful_pipeline_bench(P, torch, local, stream)
        except Exception as e:  # noqa: BLE001
            result["faithful_pipeline"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = samples.cpu().numpy().view(np.uint64)

        def ri_gpu(sub):
            ri, _ = P.sampled_ri(cfg, sub)
            return ri
        result["cpu_baseline"] = cpu_baseline(cfg, host, ri_gpu, args.cpu_seconds)
        result["cpu_fulltrace_config1"] = cpu_fulltrace_baseline()
    else:
        result["cpu_baseline"] = None
    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
