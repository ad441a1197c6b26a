"""Summarise rocprofv3 --pmc passes of the hot kernel (k_count, driven by tools/prof_kernel.py) into
profiles/pmc_sampled_hist.json.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half
the bytes of a wide coalesced streaming read on gfx950, so it is doubled;
WRITE_SIZE (KB) is taken as is.  Values are per launch (mean over dispatches).

usage: python tools/pmc_summary.py gpurun_out/<run> [samples_per_launch]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

run = sys.argv[1]
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
acc = defaultdict(list)
for f in glob.glob(os.path.join(run, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_count" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in acc.items()}
fetch = mean.get("FETCH_SIZE")
write = mean.get("WRITE_SIZE", 0.0)
out = {
    "kernel": "pluss::k_count<P2,NP2,NT,TAIL_DENSE> (the bench step)",
    "samples_per_launch": samples,
    "algorithmic_bytes_per_launch": 8 * samples,
    "counters_mean_per_launch": mean,
    "hbm_bytes_per_launch": None if fetch is None else (2 * fetch + write) * 1024,
    "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 wide-read correction); WRITE_SIZE as is",
    "source": os.path.relpath(os.path.normpath(run), "gpurun_out"),
}
os.makedirs("profiles", exist_ok=True)
json.dump(out, open("profiles/pmc_sampled_hist.json", "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1))
