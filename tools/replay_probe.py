"""The gen_faithful replay sequence of test_group_faithful_replays_equal_one_device
at 8 logical shards, repeated in one process with a native backtrace on a
host fault (tools/native/segv_bt.c).  usage: python tools/replay_probe.py [rounds]"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
if os.environ.get("PLUSS_PROBE_LIB") == "stages":
    import pluss_sampler_optimization_amd._lib as L  # noqa: E402
    L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "stages", "libpluss_gpu.so")
bt = ctypes.CDLL(os.path.join(HERE, "native", "libsegv_bt.so"))
import pluss_sampler_optimization_amd as P  # noqa: E402
import torch  # noqa: E402

assert bt.segv_bt_install() == 0
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
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
for k in range(rounds):
    for spd in (8, 1):
        with P.Group(c, [0], spd) as g:
            for i, seed in enumerate((11, 11, 11, 11, 12, 11, 11, 11)):
                print(f"round {k} spd {spd} call {i} seed {seed}", file=sys.stderr, flush=True)
                h = g.gen_faithful(seed, totals)
                w = a if seed == 11 else b
                assert h.bins == w.bins and h.traversed == w.traversed, (k, spd, i)
            g.gen_uniform_faithful(11, totals)
            for i in range(3):
                print(f"round {k} spd {spd} after uniform {i}", file=sys.stderr, flush=True)
                h = g.gen_faithful(11, totals)
                assert h.bins == a.bins and h.traversed == a.traversed
    print(f"round {k} ok", flush=True)
