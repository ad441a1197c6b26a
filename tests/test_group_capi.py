"""Multi-GPU behind the C ABI (include/pluss_gpu.h, pluss_group_*;
csrc/pluss_group.hip): a plain-C caller (tests/helpers/group_main.c, the
shape of the reference's own main()s, r10:3191-3278 / src/main.rs:17-44)
drives a group of shards over RCCL and checks every merged result against
the same pass on one device.  On the one-GPU box: one device with one shard
(a one-rank RCCL communicator) and one device with 8 logical shards (SURVEY
§4.4: an 8-GPU job's partition and exchanges on one card).  The Python Group
wrapper is also checked against the reference's own r10 dumps."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import expected_raw, golden_configs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "pluss_sampler_optimization_amd", "lib")
SRC = os.path.join(ROOT, "tests", "helpers", "group_main.c")


def build(out_dir):
    if not os.path.exists(os.path.join(LIBDIR, "libpluss_gpu.so")):
        pytest.skip("libraries not built")
    exe = os.path.join(out_dir, "group_main")
    cc = shutil.which("gcc") or pytest.skip("no gcc")
    r = subprocess.run([cc, "-O2", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-o", exe,
                        SRC, "-L", LIBDIR, "-lpluss_gpu", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_c_caller_compiles_and_links(tmp_path):
    exe = build(str(tmp_path))
    out = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "libpluss_gpu.so" in out


@pytest.mark.gpu
@pytest.mark.parametrize("N,T,total,spd", [(128, 4, 200000, 1), (128, 4, 200000, 8), (256, 8, 1 << 20, 8),
                                           (1024, 8, 1 << 22, 3)])
def test_c_group_equals_one_device(tmp_path, N, T, total, spd):
    exe = build(str(tmp_path))
    r = subprocess.run([exe, str(N), str(T), str(total), str(spd), "0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    lines = [x for x in r.stdout.strip().splitlines() if x.split(" ")[0] in ("shards", "ok", "MISMATCH")]  # (RCCL's banner)
    assert lines[0] == f"shards {spd} of {spd}"
    assert lines[1:] == ["ok clean sampled_hist", "ok clean dense x20 (resident lists)",
                         "ok clean dense x32 after re-expanding", "ok clean gen_count_dense",
                         "ok faithful sampled_hist (any order)", "ok faithful gen_faithful (key-order lists)",
                         "ok faithful gen_uniform_faithful (r10's law)"]


STREAM_SRC = os.path.join(ROOT, "tests", "helpers", "stream_main.c")


def build_stream(out_dir):
    if not os.path.exists(os.path.join(LIBDIR, "libpluss_gpu.so")):
        pytest.skip("libraries not built")
    exe = os.path.join(out_dir, "stream_main")
    cc = shutil.which("gcc") or pytest.skip("no gcc")
    r = subprocess.run([cc, "-O2", "-std=c11", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I",
                        os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", "-o", exe, STREAM_SRC, "-L", LIBDIR,
                        "-lpluss_gpu", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIBDIR}",
                        "-Wl,-rpath,/opt/rocm/lib"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_stream_caller_compiles_and_links(tmp_path):
    exe = build_stream(str(tmp_path))
    assert "libpluss_gpu.so" in subprocess.run(["ldd", exe], capture_output=True, text=True).stdout


@pytest.mark.gpu
def test_null_stream_orders_with_callers_work(tmp_path):
    """stream == NULL is HIP's null stream (include/pluss_gpu.h): a C caller's
    null-stream memsets and copies interleaved with library calls on NULL
    need no synchronisation of their own (round 4's g2 race)."""
    exe = build_stream(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    lines = [x for x in r.stdout.strip().splitlines() if x.split(" ")[0] in ("ok", "MISMATCH")]
    assert lines == ["ok caller memset -> pass on NULL"] * 3 + ["ok library expand on NULL -> caller copy",
                                                                "ok pass on pluss_ctx_stream"]


P = None


def _P():
    global P
    if P is None:
        P = pytest.importorskip("pluss_sampler_optimization_amd")
    return P


@pytest.mark.gpu
@pytest.mark.parametrize("spd", [1, 8])
@pytest.mark.parametrize("name,d,smp", golden_configs()[:4], ids=[g[0] for g in golden_configs()[:4]])
def test_group_reproduces_reference_dumps(orc, name, d, smp, spd):
    """The reference's r10 sample lists through a group (key-range shards,
    rows all-gathered over RCCL, tables merged): its raw histograms."""
    P = _P()
    N, T = d["N"], d["T"]
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    lst = np.concatenate([orc.pack_array(ref, smp[ref]) for ref in orc.REFS])
    with P.Group(c, [0], spd) as g:
        h = g.sampled_hist(np.random.default_rng(3).permutation(lst))
    for r, ref in enumerate(orc.REFS):
        exp, etrav = expected_raw(d, ref)
        assert {k: v for k, v in h.bins.items() if k[0] == ref} == exp, (name, ref)
        assert h.traversed[r] == etrav, (name, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("spd", [1, 8])
@pytest.mark.parametrize("N,T,total", [(128, 4, 50000), (256, 8, 400000), (1024, 8, 1 << 20)])
def test_group_uniform_faithful_equals_one_device(N, T, total, spd):
    """r10's own law over key-range shards (each shard generating only its
    stretch of the uniform lists): the one-device pass over the same lists,
    and, at N=128, the stepping r10 oracle over the materialised lists."""
    P = _P()
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    counts = P.default_counts(N, total)
    with P.Group(c, [0], spd) as g:
        h = g.gen_uniform_faithful(77, counts)
    import torch
    st = torch.cuda.Stream()
    with P.Context(c) as ctx:
        ctx.reset(st.cuda_stream)
        ctx.gen_uniform_faithful_refs(77, counts, st.cuda_stream)
        st.synchronize()
        one = ctx.fetch()
    assert h.bins == one.bins and h.traversed == one.traversed


@pytest.mark.gpu
@pytest.mark.parametrize("spd", [1, 8])
def test_group_faithful_replays_equal_one_device(spd):
    """Repeated identical pluss_group_gen_faithful calls (the second captured
    into a HIP graph, later ones replayed) give the one-device pass every
    time; a different seed in between runs eagerly and drops the graph; the
    group's other passes in between invalidate it too."""
    P = _P()
    import torch
    N, T = 1024, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, 1 << 22)
    st = torch.cuda.Stream()

    def one(seed):
        with P.Context(c) as ctx:
            ctx.reset(st.cuda_stream)
            ctx.gen_faithful_refs(seed, totals, st.cuda_stream)
            st.synchronize()
            return ctx.fetch()
    a, b = one(11), one(12)
    with P.Group(c, [0], spd) as g:
        for seed in (11, 11, 11, 11, 12, 11, 11, 11):
            h = g.gen_faithful(seed, totals)
            w = a if seed == 11 else b
            assert h.bins == w.bins and h.traversed == w.traversed, seed
        g.gen_uniform_faithful(11, totals)  # another pass on the same handles
        for _ in range(3):
            h = g.gen_faithful(11, totals)
            assert h.bins == a.bins and h.traversed == a.traversed


@pytest.mark.gpu
@pytest.mark.parametrize("spd", [1, 3, 8])
def test_group_uniform_replays_equal_one_device(spd):
    """Repeated identical pluss_group_gen_uniform_faithful calls: the first
    eager (it reads every shard's slice back), the second captured with those
    slices (no read-back, the device's own slice checked against them), later
    ones replayed; each equals the one-device uniform pass.  A different seed
    in between runs eagerly; a generated pass in between drops the graph."""
    P = _P()
    import torch
    N, T = 1024, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, 1 << 22)
    st = torch.cuda.Stream()

    def one(seed):
        with P.Context(c) as ctx:
            ctx.reset(st.cuda_stream)
            ctx.gen_uniform_faithful_refs(seed, totals, st.cuda_stream)
            st.synchronize()
            return ctx.fetch()
    a, b = one(21), one(22)
    with P.Group(c, [0], spd) as g:
        for seed in (21, 21, 21, 21, 22, 21, 21, 21):
            h = g.gen_uniform_faithful(seed, totals)
            w = a if seed == 21 else b
            assert h.bins == w.bins and h.traversed == w.traversed, seed
        g.gen_faithful(21, totals)  # another pass on the same handles
        for _ in range(3):
            h = g.gen_uniform_faithful(21, totals)
            assert h.bins == a.bins and h.traversed == a.traversed


@pytest.mark.gpu
def test_group_graph_replacement_rounds():
    """r5m's sequence: groups created and destroyed in
    turn, each replacing its captured graph twice (a new seed, then a new
    uniform pass) and capturing again.  A group that destroyed a replaced
    graph crashed the host in hipGraphLaunch within two rounds (r6x); kept
    graphs ran 20 rounds clean (r6y, r6z).  Here 4 rounds, every result
    equal to one device."""
    P = _P()
    import torch
    N, T = 1024, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, 1 << 21)
    st = torch.cuda.Stream()
    want = {}
    for seed in (41, 42):
        with P.Context(c) as ctx:
            ctx.reset(st.cuda_stream)
            ctx.gen_faithful_refs(seed, totals, st.cuda_stream)
            st.synchronize()
            want[seed] = ctx.fetch()
    for _ in range(4):
        for spd in (8, 1):
            with P.Group(c, [0], spd) as g:
                for seed in (41, 41, 41, 42, 42, 41, 41, 41):
                    h = g.gen_faithful(seed, totals)
                    assert h.bins == want[seed].bins and h.traversed == want[seed].traversed
                g.gen_uniform_faithful(41, totals)
                for _ in range(3):
                    h = g.gen_faithful(41, totals)
                    assert h.bins == want[41].bins


@pytest.mark.gpu
@pytest.mark.parametrize("spd", [1, 8])
def test_group_uniform_replays_sparse_2d_references(spd):
    """N=4096 with the BASELINE budget of the 2-D references (1% of (N-1)^2):
    their tiles span more than 2^32 keys, so eager passes run them on the
    handle's side stream and captured passes queue them (the side stream
    inside a captured pass crashed the bench on the host, r6ah); repeated
    group calls -- eager, captured, replayed -- equal the one-device pass."""
    P = _P()
    import torch
    N, T = 4096, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    c2 = P.default_counts(N, 1 << 28)[0]
    totals = [c2, c2, 200_000, 200_000, 200_000, 200_000]
    st = torch.cuda.Stream()
    with P.Context(c) as ctx:
        ctx.reset(st.cuda_stream)
        ctx.gen_uniform_faithful_refs(31, totals, st.cuda_stream)
        st.synchronize()
        one = ctx.fetch()
    with P.Group(c, [0], spd) as g:
        for _ in range(4):
            h = g.gen_uniform_faithful(31, totals)
            assert h.bins == one.bins and h.traversed == one.traversed


@pytest.mark.gpu
@pytest.mark.parametrize("spd", [1, 3, 8])
@pytest.mark.parametrize("N,total", [(1024, 1 << 20), (2048, 1 << 20)])
def test_group_any_order_equals_one_device(N, total, spd):
    """r10's any-order input through the group, partitioned on the device by
    (key-range shard, reference) (4-byte words at N=1024, 8-byte at 2048):
    the one-device radix pass over the same lists; then a shorter shuffled
    list on the same group (buffers reused), and a malformed sample
    (PLUSS_ERR_INPUT)."""
    P = _P()
    import torch
    c = P.SamplerConfig(n=N, threads=8, mode="faithful")
    st = torch.cuda.Stream()

    def lists(seed, tot):
        counts = P.default_counts(N, tot)
        lst = np.concatenate([P.expand_samples(c, seed, r, 0, n) for r, n in enumerate(counts)])
        return counts, lst

    def one(counts, lst):
        d = torch.from_numpy(lst.view(np.int64)).to("cuda")
        with P.Context(c) as ctx:
            ctx.reset(st.cuda_stream)
            ctx.faithful_hist_refs(d.data_ptr(), counts, st.cuda_stream)
            st.synchronize()
            return ctx.fetch()
    counts, lst = lists(5, total)
    counts2, lst2 = lists(6, total // 3)
    w1, w2 = one(counts, lst), one(counts2, lst2)
    with P.Group(c, [0], spd) as g:
        h = g.sampled_hist(lst)
        assert h.bins == w1.bins and list(h.traversed) == list(w1.traversed)
        h = g.sampled_hist(np.random.default_rng(1).permutation(lst2))
        assert h.bins == w2.bins and list(h.traversed) == list(w2.traversed)
        h = g.sampled_hist(lst)  # (again, after the smaller one)
        assert h.bins == w1.bins and list(h.traversed) == list(w1.traversed)
        bad = lst2.copy()
        bad[len(bad) // 2] = (3 << 60) | (np.uint64(N + 5) << np.uint64(40))
        with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
            g.sampled_hist(bad)
        h = g.sampled_hist(lst2)  # (a failed pass leaves the group usable)
        assert h.bins == w2.bins


@pytest.mark.gpu
def test_group_any_order_config3_equals_one_device():
    """BASELINE config 3's any-order list (N=4096, T=8, 2^28 Feistel samples)
    through the group at 1, 2 and 8 logical shards, two calls each on one
    group (the second on grown buffers: the sequence that faulted in r5p):
    every call equals the one-device radix pass.  The group's word sorts take
    the same count-free levels and 4-byte payloads as that pass (at one shard
    their level-1 buckets fit; at 2 and 8 a shard's words fill a fraction of
    the word range and the counted level-1 fallback runs)."""
    P = _P()
    import torch
    N, T = 4096, 8
    c = P.SamplerConfig(n=N, threads=T, mode="faithful")
    totals = P.default_counts(N, 1 << 28)
    st = torch.cuda.Stream()
    host = torch.empty(sum(totals), dtype=torch.int64, pin_memory=True)
    d = torch.empty(sum(totals), dtype=torch.int64, device="cuda")
    with P.Context(c) as ctx:
        off = 0
        for r, n in enumerate(totals):
            ctx.expand(0x5EED0001, r, 0, n, d.data_ptr() + 8 * off, st.cuda_stream)
            off += n
        ctx.reset(st.cuda_stream)
        ctx.faithful_hist_refs(d.data_ptr(), totals, st.cuda_stream)
        st.synchronize()
        one = ctx.fetch()
    host.copy_(d)
    del d
    lst = host.numpy().view(np.uint64)
    assert sum(one.bins.values()) > 0.5 * sum(totals)
    for spd in (1, 2, 8):
        with P.Group(c, [0], spd) as g:
            for call in range(2):
                h = g.sampled_hist(lst)
                assert h.bins == one.bins and list(h.traversed) == list(one.traversed), (spd, call)


@pytest.mark.gpu
def test_group_pairs_shape_and_errors(orc):
    """A shape with N % (cls/ds) != 0 ((key, sink) pairs, not key-range
    sharded: the job's first shard runs the samplers) equals one device; a
    malformed sample fails the group pass."""
    P = _P()
    c = P.SamplerConfig(n=100, threads=1, mode="faithful")
    lst = np.concatenate([P.expand_samples(c, 9, r, 0, n) for r, n in enumerate(P.default_counts(100, 20000))])
    with P.Group(c, [0], 4) as g:
        assert g.sampled_hist(lst) == P.sampled_hist(c, lst)
        bad = lst.copy()
        bad[7] = (7 << 60) | 1
        with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
            g.sampled_hist(bad)
    cc = P.SamplerConfig(n=128, threads=4)
    with P.Group(cc, [0], 2) as g:
        bad = np.concatenate([P.expand_samples(cc, 9, r, 0, 1000) for r in range(6)])
        bad[5] = (2 << 60) | (200 << 40)  # index >= N
        with pytest.raises(P.PlussError, match="PLUSS_ERR_INPUT"):
            g.sampled_hist(bad)
        with pytest.raises(P.PlussError, match="PLUSS_ERR_CONFIG"):
            g.dense(1)  # no resident lists yet
