"""ctypes wrapper for the CPU oracle (oracle/pluss_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product library never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

REFS = ["C0", "C1", "A0", "B0", "C2", "C3"]
REF_ID = {r: i for i, r in enumerate(REFS)}


class OrcCfg(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int64), ("T", ctypes.c_int64), ("CS", ctypes.c_int64),
                ("DS", ctypes.c_int64), ("CLS", ctypes.c_int64),
                ("thr_variant", ctypes.c_int32), ("range_full", ctypes.c_int32)]


class OrcEntry(ctypes.Structure):
    _fields_ = [("ref", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("ri", ctypes.c_int64), ("count", ctypes.c_uint64)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        L.orc_fulltrace.argtypes = [P(OrcCfg), P(OrcEntry), ctypes.c_int64, P(ctypes.c_int64), P(ctypes.c_int64)]
        L.orc_fulltrace_mt.argtypes = L.orc_fulltrace.argtypes
        L.orc_clean.argtypes = [P(OrcCfg), P(ctypes.c_uint64), ctypes.c_int64, P(ctypes.c_int64), ctypes.c_int]
        L.orc_faithful.argtypes = [P(OrcCfg), ctypes.c_int, P(ctypes.c_uint64), ctypes.c_int64,
                                   P(OrcEntry), ctypes.c_int64, P(ctypes.c_int64), P(ctypes.c_int64)]
        L.orc_expand.argtypes = [P(OrcCfg), ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                 P(ctypes.c_uint64)]
        L.orc_expand_sorted.argtypes = [P(OrcCfg), ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint64, P(ctypes.c_uint64)]
        L.orc_expand_sorted.restype = ctypes.c_int
        L.orc_expand_uniform.argtypes = L.orc_expand_sorted.argtypes
        L.orc_expand_uniform.restype = ctypes.c_int
        for f in (L.orc_fulltrace, L.orc_fulltrace_mt, L.orc_clean, L.orc_faithful, L.orc_expand):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def cfg(N, T, CS=4, DS=8, CLS=64, thr_variant=0, range_full=0):
    return OrcCfg(N, T, CS, DS, CLS, thr_variant, range_full)


def _entries_to_dict(buf, n):
    """{(ref_name, kind, ri): count}; kind 0 = noshare, 1 = share, ri -1 = cold."""
    out = {}
    for i in range(n):
        e = buf[i]
        out[(REFS[e.ref], e.kind, e.ri)] = e.count
    return out


def fulltrace(N, T, CS=4, DS=8, CLS=64, thr_variant=1):
    """Full-trace raw histogram keyed by SOURCE reference (seq.cpp sampler()).

    thr_variant=1 is the v1/seq share threshold (N+1)N+1 (seq.cpp:203)."""
    c = cfg(N, T, CS, DS, CLS, thr_variant)
    cap = 4096
    buf = (OrcEntry * cap)()
    n = ctypes.c_int64()
    trav = ctypes.c_int64()
    rc = lib().orc_fulltrace(ctypes.byref(c), buf, cap, ctypes.byref(n), ctypes.byref(trav))
    if rc:
        raise RuntimeError(f"orc_fulltrace rc={rc}")
    return _entries_to_dict(buf, n.value), trav.value


def fulltrace_mt(N, T, CS=4, DS=8, CLS=64, thr_variant=1):
    """orc_fulltrace with one host thread per simulated tid (same result)."""
    c = cfg(N, T, CS, DS, CLS, thr_variant)
    cap = 4096
    buf = (OrcEntry * cap)()
    n = ctypes.c_int64()
    trav = ctypes.c_int64()
    rc = lib().orc_fulltrace_mt(ctypes.byref(c), buf, cap, ctypes.byref(n), ctypes.byref(trav))
    if rc:
        raise RuntimeError(f"orc_fulltrace_mt rc={rc}")
    return _entries_to_dict(buf, n.value), trav.value


def clean_ri(c, samples, nthreads=1):
    """Per-sample forward RI by stepping (-1 = cold)."""
    s = np.ascontiguousarray(samples, dtype=np.uint64)
    ri = np.empty(len(s), dtype=np.int64)
    rc = lib().orc_clean(ctypes.byref(c), s.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(s),
                         ri.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), nthreads)
    if rc:
        raise RuntimeError(f"orc_clean rc={rc}")
    return ri


def faithful(c, ref, samples):
    """Raw r10 histogram of one sampler_<REF> on the given sample list.

    Returns ({(ref, kind, ri): count}, traversed)."""
    s = np.ascontiguousarray(samples, dtype=np.uint64)
    cap = 1 << 16
    buf = (OrcEntry * cap)()
    n = ctypes.c_int64()
    trav = ctypes.c_int64()
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    rc = lib().orc_faithful(ctypes.byref(c), rid, s.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(s),
                            buf, cap, ctypes.byref(n), ctypes.byref(trav))
    if rc:
        raise RuntimeError(f"orc_faithful rc={rc}")
    return _entries_to_dict(buf, n.value), trav.value


def expand(c, seed, ref, first, n):
    out = np.empty(n, dtype=np.uint64)
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    rc = lib().orc_expand(ctypes.byref(c), seed, rid, first, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc:
        raise RuntimeError(f"orc_expand rc={rc}")
    return out


def expand_sorted(c, seed, ref, total, first, n):
    """Samples [first, first+n) of the key-order stratified list of `total`
    samples of reference `ref`."""
    out = np.empty(n, dtype=np.uint64)
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    rc = lib().orc_expand_sorted(ctypes.byref(c), seed, rid, total, first, n,
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc:
        raise RuntimeError(f"orc_expand_sorted rc={rc}")
    return out


def expand_uniform(c, seed, ref, total, first, n):
    """Samples [first, first+n) of the list of `total` samples of reference
    `ref` drawn uniformly without replacement, in key order (DESIGN.md §4,
    orc_expand_uniform)."""
    out = np.empty(n, dtype=np.uint64)
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    rc = lib().orc_expand_uniform(ctypes.byref(c), seed, rid, total, first, n,
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc:
        raise RuntimeError(f"orc_expand_uniform rc={rc}")
    return out


def sort_key(N, T, CS, samples):
    """Faithful sort key a*T + tid of packed samples, numpy."""
    s = np.asarray(samples, dtype=np.uint64)
    m = np.uint64(0xFFFFF)
    ref = (s >> np.uint64(60)).astype(np.int64)
    c0 = ((s >> np.uint64(40)) & m).astype(np.int64)
    c1 = ((s >> np.uint64(20)) & m).astype(np.int64)
    c2 = (s & m).astype(np.int64)
    k = c0 // CS
    t, q = k % T, (k // T) * CS + c0 % CS
    off = np.where(ref < 2, ref, ref + 4 * c2)
    S = 4 * N + 2
    return ((q * N * S + c1 * S + off) * T + t).astype(np.uint64)


def pack(ref, c0, c1, c2=0):
    rid = REF_ID[ref] if isinstance(ref, str) else int(ref)
    return (rid << 60) | (int(c0) << 40) | (int(c1) << 20) | int(c2)


def pack_array(ref, idx):
    """idx: (n, 3) or (n, 2) int array -> packed uint64 samples."""
    rid = np.uint64(REF_ID[ref] if isinstance(ref, str) else int(ref))
    idx = np.asarray(idx, dtype=np.uint64)
    c2 = idx[:, 2] if idx.shape[1] > 2 else np.zeros(len(idx), np.uint64)
    return (rid << np.uint64(60)) | (idx[:, 0] << np.uint64(40)) | (idx[:, 1] << np.uint64(20)) | c2
