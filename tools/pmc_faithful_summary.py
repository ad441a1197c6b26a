"""Summarise rocprofv3 --pmc passes over tools/prof_faithful.py into
profiles/pmc_faithful.json: HBM bytes per faithful pass (sum over the pass's
kernels, mean over passes), FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM.

usage: python tools/pmc_faithful_summary.py gpurun_out/<run> <passes>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

run, passes = sys.argv[1], int(sys.argv[2])
per = defaultdict(lambda: defaultdict(float))  # counter -> kernel -> total
for f in glob.glob(os.path.join(run, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(x in k for x in ("k_fa_", "k_gen", "k_srt_", "k_ug_", "k_scan")):
            continue
        short = k.split("(")[0].replace("void ", "").replace("pluss::", "")
        per[r["Counter_Name"]][short] += float(r["Counter_Value"])
kern = {}
for c, d in per.items():
    for k, v in d.items():
        kern.setdefault(k, {})[c] = v / passes
fetch = sum(v.get("FETCH_SIZE", 0.0) for v in kern.values())
write = sum(v.get("WRITE_SIZE", 0.0) for v in kern.values())
c3 = os.environ.get("PROF_SHAPE") == "config3"
out = {
    "pipeline": "faithful pass, six references (k_fa_local_lm or k_fa_local_fast, k_fa_local, k_fa_chunk, k_fa_finish)",
    "workload": ("GEMM N=4096, T=8, 2^28 samples (config 3 on one GPU)" if c3 else
                 "GEMM N=1024, T=8, 2^24 samples (config 2 budget)"),
    "samples_per_pass": 1 << 28 if c3 else 1 << 24,
    "per_kernel_per_pass_KB": kern,
    "hbm_bytes_per_pass": (2 * fetch + write) * 1024 if per else None,
    "hbm_bytes_per_sample": (2 * fetch + write) * 1024 / ((1 << 28) if c3 else (1 << 24)) if per else None,
    "elements": os.environ.get("PROF_FAITH", "sorted"),
    "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 wide-read correction); WRITE_SIZE as is",
    "source": os.path.relpath(os.path.normpath(run), "gpurun_out"),
}
name = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_faithful.json"
json.dump(out, open(name, "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1))
