"""ctypes binding of libpluss_gpu.so (include/pluss_gpu.h).

The library is loaded from this package's lib/ directory (built in-tree by
build.py).  There is deliberately no fallback: if the library is missing or a
call fails, an exception is raised.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libpluss_gpu.so")

PLUSS_OK = 0
DENSE_BINS = 18  # PLUSS_DENSE_BINS; a dense count vector holds DENSE_BINS + 1 words (the last: malformed samples)
ERRORS = {-1: "PLUSS_ERR_CONFIG", -2: "PLUSS_ERR_HIP", -3: "PLUSS_ERR_ALLOC", -4: "PLUSS_ERR_CAPACITY",
          -5: "PLUSS_ERR_INPUT", -6: "PLUSS_ERR_PEER"}
SHARD_ROW = 32      # PLUSS_SHARD_ROW: u64 words of a key-range shard's summary row
SHARD_ROW_ERR = 31  # PLUSS_SHARD_ROW_ERR
GROUP_ID_BYTES = 128

# every symbol declared in include/pluss_gpu.h
EXPORTS = [
    "pluss_last_error", "pluss_device_count", "pluss_version",
    "pluss_gemm_sampled_hist", "pluss_gemm_fulltrace_hist", "pluss_gemm_sampled_ri", "pluss_expand_samples",
    "pluss_default_counts", "pluss_expand_sorted", "pluss_dev_expand_sorted", "pluss_expand_uniform_sorted",
    "pluss_dev_expand_uniform_sorted", "pluss_dev_gen_uniform_faithful_refs",
    "pluss_ctx_create", "pluss_ctx_destroy", "pluss_ctx_stream", "pluss_dev_expand", "pluss_dev_hist_reset",
    "pluss_dev_sampled_hist", "pluss_dev_faithful_hist", "pluss_dev_faithful_hist_refs",
    "pluss_dev_faithful_hist_sorted", "pluss_dev_faithful_hist_sorted_refs", "pluss_dev_gen_faithful_refs",
    "pluss_dev_fulltrace_hist", "pluss_dev_sampled_ri",
    "pluss_dev_hist_export", "pluss_dev_hist_export_reset", "pluss_dev_sampled_hist_export", "pluss_hist_fetch",
    "pluss_hist_from_tables", "pluss_faithful_key_space", "pluss_keyorder_index_range",
    "pluss_dense_keys", "pluss_dev_sampled_hist_dense", "pluss_dev_gen_count_dense",
    "pluss_dev_faithful_shards_local", "pluss_dev_faithful_shards_select", "pluss_dev_faithful_shards_local_selected",
    "pluss_dev_faithful_shards_carry", "pluss_dev_faithful_shards_cut", "pluss_dev_faithful_shards_hist",
    "pluss_dev_faithful_shards_uniform_count", "pluss_dev_faithful_shards_uniform_local",
    "pluss_dev_faithful_shards_slice",
    "pluss_group_unique_id", "pluss_group_create", "pluss_group_create_rank", "pluss_group_destroy",
    "pluss_group_shards", "pluss_group_sampled_hist", "pluss_group_gen_faithful",
    "pluss_group_gen_uniform_faithful", "pluss_group_expand",
    "pluss_group_dense", "pluss_group_gen_count_dense",
]
# include/pluss_diag.h (diagnostics, not the drop-in boundary)
DIAG_EXPORTS = ["pluss_diag_dense", "pluss_diag_sort_words", "pluss_diag_uniform_parts"]


class PlussCfg(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("threads", ctypes.c_int64), ("chunk", ctypes.c_int64),
                ("ds", ctypes.c_int64), ("cls", ctypes.c_int64), ("mode", ctypes.c_int32),
                ("thr_variant", ctypes.c_int32), ("range_full", ctypes.c_int32), ("device", ctypes.c_int32)]


class PlussHistEntry(ctypes.Structure):
    _fields_ = [("ref", ctypes.c_int32), ("kind", ctypes.c_int32), ("ri", ctypes.c_int64),
                ("count", ctypes.c_uint64)]


class PlussHist(ctypes.Structure):
    _fields_ = [("entries", ctypes.POINTER(PlussHistEntry)), ("capacity", ctypes.c_uint64),
                ("n_entries", ctypes.c_uint64), ("traversed", ctypes.c_uint64 * 6)]


class PlussError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libpluss_gpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # PyTorch-ROCm wheels bundle their own libamdhip64 (same SONAME as ROCm's).
    # If our library were loaded first, a later `import torch` would map a
    # second HIP runtime into the process and torch would find no GPU.  Loading
    # torch first makes both share one runtime (the dynamic linker resolves our
    # NEEDED libamdhip64.so.7 to the copy torch already mapped).
    if os.environ.get("PLUSS_NO_TORCH_PRELOAD") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise PlussError(f"{LIB_PATH} is missing: build it with `python -m pluss_sampler_optimization_amd.build` "
                         "(hipcc, gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    u64, i64, i32, vp = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
    cfgp, histp = P(PlussCfg), P(PlussHist)
    sig = {
        "pluss_last_error": (ctypes.c_char_p, []),
        "pluss_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
        "pluss_version": (ctypes.c_int, []),
        "pluss_gemm_sampled_hist": (ctypes.c_int, [cfgp, vp, u64, histp]),
        "pluss_gemm_fulltrace_hist": (ctypes.c_int, [cfgp, histp]),
        "pluss_gemm_sampled_ri": (ctypes.c_int, [cfgp, vp, u64, vp, vp]),
        "pluss_expand_samples": (ctypes.c_int, [cfgp, u64, i32, u64, u64, vp]),
        "pluss_default_counts": (ctypes.c_int, [i64, u64, P(u64)]),
        "pluss_expand_sorted": (ctypes.c_int, [cfgp, u64, i32, u64, u64, u64, vp]),
        "pluss_dev_expand_sorted": (ctypes.c_int, [vp, u64, i32, u64, u64, u64, vp, vp]),
        "pluss_expand_uniform_sorted": (ctypes.c_int, [cfgp, u64, i32, u64, u64, u64, vp]),
        "pluss_dev_expand_uniform_sorted": (ctypes.c_int, [vp, u64, i32, u64, u64, u64, vp, vp]),
        "pluss_dev_gen_uniform_faithful_refs": (ctypes.c_int, [vp, u64, P(u64), vp]),
        "pluss_ctx_create": (ctypes.c_int, [cfgp, P(vp)]),
        "pluss_ctx_destroy": (ctypes.c_int, [vp]),
        "pluss_ctx_stream": (vp, [vp]),
        "pluss_dev_expand": (ctypes.c_int, [vp, u64, i32, u64, u64, vp, vp]),
        "pluss_dev_hist_reset": (ctypes.c_int, [vp, vp]),
        "pluss_dev_sampled_hist": (ctypes.c_int, [vp, vp, u64, vp]),
        "pluss_dev_faithful_hist": (ctypes.c_int, [vp, i32, vp, u64, vp]),
        "pluss_dev_faithful_hist_refs": (ctypes.c_int, [vp, vp, ctypes.POINTER(ctypes.c_uint64), vp]),
        "pluss_dev_faithful_hist_sorted": (ctypes.c_int, [vp, i32, vp, u64, vp]),
        "pluss_dev_faithful_hist_sorted_refs": (ctypes.c_int, [vp, vp, ctypes.POINTER(ctypes.c_uint64), vp]),
        "pluss_dev_gen_faithful_refs": (ctypes.c_int, [vp, u64, ctypes.POINTER(ctypes.c_uint64), vp]),
        "pluss_dev_fulltrace_hist": (ctypes.c_int, [vp, vp]),
        "pluss_dev_sampled_ri": (ctypes.c_int, [vp, vp, u64, vp, vp, vp]),
        "pluss_dev_hist_export": (ctypes.c_int, [vp, vp, vp, u64, vp]),
        "pluss_dev_hist_export_reset": (ctypes.c_int, [vp, vp, vp, u64, vp]),
        "pluss_dev_sampled_hist_export": (ctypes.c_int, [vp, vp, u64, vp, vp, u64, vp]),
        "pluss_hist_fetch": (ctypes.c_int, [vp, histp]),
        "pluss_hist_from_tables": (ctypes.c_int, [vp, vp, u64, histp]),
        "pluss_faithful_key_space": (ctypes.c_int, [cfgp, P(u64)]),
        "pluss_keyorder_index_range": (ctypes.c_int, [cfgp, u64, i32, u64, u64, u64, P(u64), P(u64)]),
        "pluss_dense_keys": (ctypes.c_int, [cfgp, P(u64)]),
        "pluss_dev_sampled_hist_dense": (ctypes.c_int, [vp, vp, u64, vp, vp]),
        "pluss_dev_gen_count_dense": (ctypes.c_int, [vp, u64, P(u64), P(u64), P(u64), vp, vp]),
        "pluss_diag_dense": (ctypes.c_int, [vp, vp, u64, vp, i32, i32, vp]),
        "pluss_diag_sort_words": (ctypes.c_int, [vp, i32, vp, u64, vp, ctypes.POINTER(i32), vp]),
        "pluss_diag_uniform_parts": (ctypes.c_int, [vp, u64, P(u64), i32, vp, vp]),
        "pluss_dev_faithful_shards_local": (ctypes.c_int, [vp, vp, u64, P(u64), P(u64), P(u64), vp, vp]),
        "pluss_dev_faithful_shards_select": (ctypes.c_int, [vp, vp, P(u64), u64, u64, vp, vp]),
        "pluss_dev_faithful_shards_local_selected": (ctypes.c_int, [vp, vp, i32, i32, vp, vp]),
        "pluss_dev_faithful_shards_carry": (ctypes.c_int, [vp, vp, i32, i32, vp, vp]),
        "pluss_dev_faithful_shards_cut": (ctypes.c_int, [vp, vp, i32, i32, vp, vp]),
        "pluss_dev_faithful_shards_hist": (ctypes.c_int, [vp, vp, i32, i32, vp]),
        "pluss_dev_faithful_shards_uniform_count": (ctypes.c_int, [vp, u64, P(u64), i32, i32, vp, vp]),
        "pluss_dev_faithful_shards_uniform_local": (ctypes.c_int, [vp, vp, i32, i32, vp, vp]),
        "pluss_dev_faithful_shards_slice": (ctypes.c_int, [vp, P(u64), P(u64)]),
        "pluss_group_unique_id": (ctypes.c_int, [vp]),
        "pluss_group_create": (ctypes.c_int, [cfgp, P(i32), i32, i32, P(vp)]),
        "pluss_group_create_rank": (ctypes.c_int, [cfgp, i32, i32, vp, i32, P(vp)]),
        "pluss_group_destroy": (ctypes.c_int, [vp]),
        "pluss_group_shards": (ctypes.c_int, [vp, P(i32), P(i32)]),
        "pluss_group_sampled_hist": (ctypes.c_int, [vp, vp, u64, histp]),
        "pluss_group_gen_faithful": (ctypes.c_int, [vp, u64, P(u64), histp]),
        "pluss_group_gen_uniform_faithful": (ctypes.c_int, [vp, u64, P(u64), histp]),
        "pluss_group_expand": (ctypes.c_int, [vp, u64, P(u64)]),
        "pluss_group_dense": (ctypes.c_int, [vp, ctypes.c_uint32, P(u64)]),
        "pluss_group_gen_count_dense": (ctypes.c_int, [vp, u64, P(u64), P(u64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc, what=""):
    if rc != PLUSS_OK:
        msg = lib().pluss_last_error().decode(errors="replace")
        raise PlussError(f"{what}: {ERRORS.get(rc, rc)}: {msg}")
    return rc
