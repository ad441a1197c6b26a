"""Key-range-sharded faithful mode (multi-GPU path) on the CPU.

The row exchange of pluss_sampler_optimization_amd.dist.faithful_shards_protocol
runs over gloo with world sizes 1-8.  Each rank's shard is a host emulation
of the device phases of pluss_dev_faithful_shards_* (pluss_faithful.hip:
the select / local / carry / cut / hist launches and k_fa_xchg's derivation
of a shard's inputs from the gathered summary rows) on host arrays; keys and
sinks come from the oracle's per-sample RI.  Merged over ranks, the histogram
and the summed `traversed` must equal the oracle's sequential restatement of
r10's sampler_<REF> (oracle/pluss_oracle.c orc_faithful), which is pinned to
the reference's dumps.  The device phases themselves are checked against
one-GPU faithful mode in tests/test_gpu.py and tests/test_gpu_faithful_wide.py.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, expected_raw, golden_configs

GOLD = golden_configs()

KEY_EMPTY = (1 << 64) - 1
OFF = {"C0": 0, "C1": 1, "A0": 2, "B0": 3, "C2": 4, "C3": 5}
REFS = ["C0", "C1", "A0", "B0", "C2", "C3"]
ROW, ERR = 32, 31  # PLUSS_SHARD_ROW, PLUSS_SHARD_ROW_ERR
N_, MAX_, STARTS_, CUT_ = 0, 6, 12, 18  # row word offsets (pluss_faithful.h ROW_*)


def keys_and_sinks(orc, c, N, T, CS, ref, samples):
    """Sort key a*T+tid and sink key (a+RI)*T+tid of every sample."""
    ri = orc.clean_ri(c, samples)
    _, c0, c1, c2 = [x.astype(np.int64) for x in _unpack(samples)]
    if ref in ("C0", "C1"):
        c2 = np.zeros_like(c2)
    S = 4 * N + 2
    R = N * S
    t = (c0 // CS) % T
    q = (c0 // (CS * T)) * CS + c0 % CS
    off = OFF[ref] + (4 * c2 if ref not in ("C0", "C1") else 0)
    P = q * R + c1 * S + off
    keys = (P * T + t).astype(np.uint64)
    sinks = np.where(ri < 0, np.uint64(KEY_EMPTY), ((P + np.maximum(ri, 0)) * T + t).astype(np.uint64))
    return keys, sinks, ri


def _unpack(s):
    s = np.asarray(s, np.uint64)
    m = np.uint64(0xFFFFF)
    return (s >> np.uint64(60), (s >> np.uint64(40)) & m, (s >> np.uint64(20)) & m, s & m)


class PeerFailed(RuntimeError):
    pass


class HostShards:
    """Host emulation of the pluss_dev_faithful_shards_* phases, all six
    references at once.  ks[r] = (keys, sinks) of reference r's whole list:
    key-ordered (faithful_shards_local's slices) or in any order
    (faithful_shards_select keeps a key range).  Rows are numpy u64 arrays."""

    def __init__(self, N, T, ks):
        self.N, self.T, self.ks = N, T, ks
        self.bins, self.trav = {}, [0] * 6
        self.peer_failed = False

    # -- phase 1
    def _row1(self, row):
        row[:] = 0
        for r in range(6):
            row[N_ + r] = self.n[r]
            row[MAX_ + r] = max((int(x) for x in self.s[r]), default=0)
            row[CUT_ + r] = self.tot[r]

    def faithful_shards_local(self, d, seed, totals, first, n, row, stream=None):
        self.tot, self.first, self.n = list(totals), list(first), list(n)
        self.k = [self.ks[r][0][first[r]:first[r] + n[r]] for r in range(6)]
        self.s = [self.ks[r][1][first[r]:first[r] + n[r]] for r in range(6)]
        self._row1(row)

    def faithful_shards_select(self, d, totals, lo, hi, row, stream=None):
        self.sel = []
        row[:] = 0
        for r in range(6):
            k, s = self.ks[r]
            m = (k >= np.uint64(lo)) & (k < np.uint64(hi))
            self.sel.append((k[m], s[m]))
            row[N_ + r] = int(m.sum())

    def faithful_shards_local_selected(self, rows, shard, ns, row, stream=None):
        R = rows.reshape(ns, ROW)
        self._check(R)
        self.tot = [int(R[:, N_ + r].sum()) for r in range(6)]
        self.first = [int(R[:shard, N_ + r].sum()) for r in range(6)]
        self.n = [int(R[shard, N_ + r]) for r in range(6)]
        order = [np.argsort(k, kind="stable") for k, _ in self.sel]
        self.k = [k[o] for (k, _), o in zip(self.sel, order)]
        self.s = [s[o] for (_, s), o in zip(self.sel, order)]
        self._row1(row)

    # -- k_fa_xchg: a failed shard anywhere makes the pass record nothing
    def _check(self, R):
        if R[:, ERR].any():
            self.peer_failed = True

    def _walk(self, r):  # (flag, run before) of each element of the slice
        run, out = self.carry[r], []
        for i in range(self.n[r]):
            f = self.first[r] + i == 0 or int(self.k[r][i]) > run
            out.append((f, run))
            run = max(run, int(self.s[r][i]))
        return out, run

    def faithful_shards_carry(self, rows, shard, ns, row, stream=None):
        R = rows.reshape(ns, ROW)
        self._check(R)
        self.carry = [max([int(R[x, MAX_ + r]) for x in range(shard) if R[x, N_ + r]], default=0) for r in range(6)]
        for r in range(6):
            row[STARTS_ + r] = sum(f for f, _ in self._walk(r)[0])

    def faithful_shards_cut(self, rows, shard, ns, row, stream=None):
        R = rows.reshape(ns, ROW)
        self._check(R)
        for r in range(6):
            c, nb = self.tot[r], int(R[:shard, STARTS_ + r].sum())
            for i, (f, _) in enumerate(self._walk(r)[0]):
                j = self.first[r] + i
                if f and j > 0 and j - nb >= self.tot[r] - j:
                    c = j
                    break
                nb += f
            row[CUT_ + r] = c

    def faithful_shards_hist(self, rows, shard, ns, stream=None):
        R = rows.reshape(ns, ROW)
        self._check(R)
        if self.peer_failed:
            return
        N, T = self.N, self.T
        thr = (4 * N + 2) * N
        endkey = (N // T) * N * (4 * N + 2) * T
        for r, ref in enumerate(REFS):
            cut = int(R[:, CUT_ + r].min())
            last = not R[shard + 1:, N_ + r].any()
            if self.n[r] == 0 or cut < self.first[r]:
                continue
            walk, final = self._walk(r)
            cold, trav = 0, 0
            for i, (f, run) in enumerate(walk):
                j = self.first[r] + i
                if j == cut:
                    trav += endkey if run == KEY_EMPTY else run  # the replay ends at the cut
                    break
                kk, ss = int(self.k[r][i]), int(self.s[r][i])
                if ss == KEY_EMPTY:
                    cold += kk % T == 0
                else:
                    ri = (ss - kk) // T
                    kind = 1 if (ref == "B0" and ri > 0 and 2 * ri > thr) else 0
                    self.bins[(ref, kind, ri)] = self.bins.get((ref, kind, ri), 0) + 1
                if f:
                    trav += run - kk
            if cut == self.tot[r] and last:
                if final != KEY_EMPTY and final % T == 0:
                    cold += 1
                trav += endkey if final == KEY_EMPTY else final
            key = (ref, 0, -1)
            self.bins[key] = self.bins.get(key, 0) + cold
            self.trav[r] = (self.trav[r] + trav) % (1 << 64)

    def fetch(self):  # the device's FLAG_SHARD -> PLUSS_ERR_PEER
        if self.peer_failed:
            raise PeerFailed("a key-range shard of this faithful pass failed")


class HostRows:
    """The gloo host stand-in of dist.DeviceRows."""

    def __init__(self, world):
        self.world = world
        self.row = np.zeros(ROW, np.uint64)
        self.rows = np.zeros(world * ROW, np.uint64)

    def fail(self):
        self.row[ERR] = 1

    def exchange(self):
        import torch
        import torch.distributed as dist
        out = torch.empty(self.world * ROW, dtype=torch.int64)
        dist.all_gather_into_tensor(out, torch.from_numpy(self.row.view(np.int64).copy()))
        self.rows[:] = out.numpy().view(np.uint64)


def lockstep(shards, phase1s, selected=False):
    """The protocol over several emulated shards in one process, rows exchanged by hand."""
    ns = len(shards)
    rows = [np.zeros(ROW, np.uint64) for _ in shards]
    for sh, p1, row in zip(shards, phase1s, rows):
        p1(sh, row)
    steps = (["local_selected"] if selected else []) + ["carry", "cut"]
    for name in steps:
        g = np.concatenate(rows)
        for i, sh in enumerate(shards):
            getattr(sh, "faithful_shards_" + name)(g, i, ns, rows[i])
    g = np.concatenate(rows)
    for i, sh in enumerate(shards):
        sh.faithful_shards_hist(g, i, ns)


def merged(shards):
    got, trav = {}, [0] * 6
    for sh in shards:
        for k, v in sh.bins.items():
            got[k] = got.get(k, 0) + v
        trav = [(a + b) % (1 << 64) for a, b in zip(trav, sh.trav)]
    return got, trav


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lists(orc, c, N, T, per, seed, sorted_):
    ks, totals = [], []
    for r, ref in enumerate(orc.REFS):
        cnt = min(per, (N - 1) ** (2 if r < 2 else 3))
        s = orc.expand_sorted(c, seed, r, cnt, 0, cnt) if sorted_ else orc.expand(c, seed, r, 0, cnt)
        keys, sinks, _ = keys_and_sinks(orc, c, N, T, 4, ref, s)
        ks.append((keys, sinks))
        totals.append(cnt)
    return ks, totals


def _worker(rank, world, port, N, T, per, mode, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import oracle as orc
    from pluss_sampler_optimization_amd import dist as D
    from test_dist_faithful import HostRows, HostShards, _lists
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = orc.cfg(N, T)
    key_space = (N // T) * N * (4 * N + 2) * T
    lo, hi = D.key_range(key_space, rank, world)
    ks, totals = _lists(orc, c, N, T, per, 0x5EED0000 + N, mode == "sorted")
    sh = HostShards(N, T, ks)
    if mode == "sorted":
        first, n = [], []
        for keys, _ in ks:
            inside = np.nonzero((keys >= np.uint64(lo)) & (keys < np.uint64(hi)))[0]
            first.append(int(inside[0]) if len(inside) else 0)
            n.append(len(inside))
        p1 = lambda row: sh.faithful_shards_local(None, 0, totals, first, n, row)  # noqa: E731
    else:
        p1 = lambda row: sh.faithful_shards_select(None, totals, lo, hi, row)  # noqa: E731
    err = D.faithful_shards_protocol(sh, p1, rank, world, HostRows(world), selected=mode == "select")
    assert err is None
    q.put((rank, sh.bins, sh.trav))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,N,T,per,mode", [(1, 64, 4, 3000, "select"), (2, 64, 4, 3000, "select"),
                                                (3, 128, 8, 4000, "select"), (4, 64, 2, 2500, "select"),
                                                (8, 128, 8, 4000, "select"), (1, 64, 4, 3000, "sorted"),
                                                (2, 64, 4, 3000, "sorted"), (3, 128, 8, 4000, "sorted"),
                                                (8, 128, 8, 4000, "sorted")])
def test_key_range_shards_equal_sequential_sampler(orc, world, N, T, per, mode):
    """dist.faithful_shards_protocol over gloo: arbitrary-order lists through
    select + local_selected (four row exchanges), key-order lists through local
    (three); merged over ranks == the oracle's sequential r10 sampler of each
    reference's whole list."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, T, per, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = orc.cfg(N, T)
    for r, ref in enumerate(orc.REFS):
        cnt = min(per, (N - 1) ** (2 if r < 2 else 3))
        s = (orc.expand_sorted(c, 0x5EED0000 + N, r, cnt, 0, cnt) if mode == "sorted"
             else orc.expand(c, 0x5EED0000 + N, r, 0, cnt))
        want, wtrav = orc.faithful(c, ref, s)
        got, trav = {}, 0
        for _, bins, tr in res:
            for k, v in bins.items():
                if k[0] == ref:
                    got[k] = got.get(k, 0) + v
            trav = (trav + tr[r]) % (1 << 64)
        assert got == want, (world, ref)
        assert trav == wtrav, (world, ref)


@pytest.mark.parametrize("name,d,smp", GOLD, ids=[g[0] for g in GOLD])
def test_key_range_shards_on_reference_dumps(orc, name, d, smp):
    """Single process, 3 emulated shards with an uneven split (the middle one
    covering no key of some references), on the reference's r10 dumps."""
    N, T = d["N"], d["T"]
    c = orc.cfg(N, T)
    key_space = (N // T) * N * (4 * N + 2) * T
    bounds = [0, key_space // 7, key_space // 2, key_space]
    ks, totals = [], []
    for ref in orc.REFS:
        s = orc.pack_array(ref, smp[ref])
        keys, sinks, _ = keys_and_sinks(orc, c, N, T, 4, ref, s)
        ks.append((keys, sinks))
        totals.append(len(s))
    shards = [HostShards(N, T, ks) for _ in range(3)]
    lockstep(shards, [lambda sh, row, i=i: sh.faithful_shards_select(None, totals, bounds[i], bounds[i + 1], row)
                      for i in range(3)], selected=True)
    got, trav = merged(shards)
    for r, ref in enumerate(orc.REFS):
        exp, etrav = expected_raw(d, ref)
        assert {k: v for k, v in got.items() if k[0] == ref} == exp, (name, ref)
        assert trav[r] == etrav, (name, ref)


class FailingShards(HostShards):
    """A shard whose phase `phase` raises (as a device phase does on a HIP
    error or a bad argument)."""

    def __init__(self, *a, phase):
        super().__init__(*a)
        self.phase = phase

    def _maybe(self, name):
        if self.phase == name:
            raise RuntimeError("injected failure in " + name)

    def faithful_shards_select(self, *a, **k):
        self._maybe("select")
        return super().faithful_shards_select(*a, **k)

    def faithful_shards_carry(self, *a, **k):
        self._maybe("carry")
        return super().faithful_shards_carry(*a, **k)

    def faithful_shards_cut(self, *a, **k):
        self._maybe("cut")
        return super().faithful_shards_cut(*a, **k)

    def faithful_shards_hist(self, *a, **k):
        self._maybe("hist")
        return super().faithful_shards_hist(*a, **k)


def _fail_worker(rank, world, port, bad, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import oracle as orc
    from pluss_sampler_optimization_amd import dist as D
    from test_dist_faithful import FailingShards, HostRows, PeerFailed, _lists
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, T = 64, 4
    c = orc.cfg(N, T)
    lo, hi = D.key_range((N // T) * N * (4 * N + 2) * T, rank, world)
    ks, totals = _lists(orc, c, N, T, 1500, 0x5EED0040, False)
    out = []
    for phase in ("select", "carry", "cut", "entry", None):
        sh = FailingShards(N, T, ks, phase=phase if rank == bad else None)
        pre = RuntimeError("injected failure before the pass") if (phase == "entry" and rank == bad) else None
        err = D.faithful_shards_protocol(sh, lambda row: sh.faithful_shards_select(None, totals, lo, hi, row),
                                         rank, world, HostRows(world), err=pre, selected=True)
        try:
            if err is not None:
                raise err
            sh.fetch()
            out.append("ok")
        except PeerFailed:
            out.append("other")
        except RuntimeError as e:
            out.append("own" if "injected" in str(e) else "?")
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


def test_failing_rank_raises_on_every_rank():
    """A rank whose phase raises (or that enters the pass with an error) marks
    its row and still takes part in every exchange: it reports its own error,
    every other rank's pass sees the error word and reports the peer failure
    at its fetch -- nobody waits forever; the next pass on the same process
    group works.  (A failure in the last phase, after the last exchange, is
    caught by merge_results' single all-gather.)"""
    world, bad = 4, 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fail_worker, args=(r, world, port, bad, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        want = "own" if r == bad else "other"
        assert res[r] == [want, want, want, want, "ok"], (r, res[r])


def test_protocol_exchange_count():
    """The sorted/generated pass exchanges rows three times, the selected pass
    four times; the phase order is fixed."""
    from pluss_sampler_optimization_amd import dist as D
    calls = []

    class Rx:
        row, rows = "row", "rows"

        def fail(self):
            calls.append("fail")

        def exchange(self):
            calls.append("x")

    class Sh:
        def __getattr__(self, name):
            return lambda *a: calls.append(name.replace("faithful_shards_", ""))
    for selected, want in ((False, ["p1", "x", "carry", "x", "cut", "x", "hist"]),
                           (True, ["p1", "x", "local_selected", "x", "carry", "x", "cut", "x", "hist"])):
        calls.clear()
        assert D.faithful_shards_protocol(Sh(), lambda row: calls.append("p1"), 0, 1, Rx(), selected=selected) is None
        assert calls == want
