"""Diagnostics: one faithful pass (N=128, T=4, reference sample list) through
the C ABI, path chosen by PLUSS_FAITH_BUCKET; prints each step."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: F401,E402
import pluss_sampler_optimization_amd as P  # noqa: E402
import oracle as orc  # noqa: E402

stem = os.path.join(ROOT, "tests", "golden", "r10_N128_T4_s1")
d = json.load(open(stem + ".json"))
z = np.load(stem + ".npz")
print("path", os.environ.get("PLUSS_FAITH_BUCKET", "bucket"), flush=True)
for ref in orc.REFS:
    s = orc.pack_array(ref, z[ref])
    print("ref", ref, len(s), flush=True)
    h = P.sampled_hist(P.SamplerConfig(n=128, threads=4, mode="faithful", device=0), s)
    exp = {(ref, 0, int(k)): v for k, v in d["raw"][ref]["noshare"].items()}
    exp.update({(ref, 1, int(k)): v for k, v in d["raw"][ref]["share"].items()})
    print("  match", h.bins == exp, h.traversed[P.REF_ID[ref]] == d["raw"][ref]["traversed"], flush=True)
