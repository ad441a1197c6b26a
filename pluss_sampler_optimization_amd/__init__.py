"""MI355X-native PLUSS GEMM reuse-interval sampler.

The compute path is libpluss_gpu.so (HIP kernels for gfx950 behind the C ABI
in include/pluss_gpu.h); this package is its Python front end plus the host
pipeline that turns raw reuse-interval histograms into a miss-ratio curve.
"""
from ._lib import DENSE_BINS, LIB_PATH, SHARD_ROW, SHARD_ROW_ERR, PlussError, lib  # noqa: F401
from .api import (DIM, REF_ARRAY, REF_ID, REFS, Context, Group, Histogram, SamplerConfig,  # noqa: F401
                  default_counts, dense_keys, expand_samples, expand_sorted, expand_uniform_sorted, faithful_key, faithful_key_space,
                  fulltrace_hist, group_unique_id, hist_from_dense, hist_from_tables, keyorder_index_range, pack,
                  pack_array, sampled_hist, sampled_ri, unpack_array)

__all__ = ["SamplerConfig", "Histogram", "Context", "Group", "group_unique_id", "sampled_hist", "fulltrace_hist",
           "sampled_ri", "expand_samples", "expand_sorted", "expand_uniform_sorted", "default_counts", "faithful_key", "faithful_key_space",
           "keyorder_index_range", "hist_from_tables", "dense_keys", "hist_from_dense", "DENSE_BINS", "SHARD_ROW",
           "SHARD_ROW_ERR", "pack", "pack_array", "unpack_array", "REFS", "REF_ID", "REF_ARRAY", "DIM", "lib",
           "LIB_PATH", "PlussError"]
