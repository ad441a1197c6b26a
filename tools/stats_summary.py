"""Print a rocprofv3 run_kernel_stats.csv compactly: short kernel name, calls,
average and total microseconds, sorted by total time.

    python tools/stats_summary.py gpurun_out/<dir>/prof/run_kernel_stats.csv
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    name = r["Name"]
    if "rocprim" in name:
        m = re.search(r"(onesweep_iteration|global_offsets|histogram|scan|lookback|sort)\w*", name)
        short = "rocprim " + (m.group(0) if m else "?")
    else:
        short = re.sub(r"\(.*", "", name).replace("void ", "").replace("pluss::", "")
    out.append((float(r["TotalDurationNs"]), short, int(r["Calls"]), float(r["AverageNs"])))
for tot, short, calls, avg in sorted(out, reverse=True):
    print(f"{tot / 1e3:12.1f} us  {calls:6d} x {avg / 1e3:9.2f} us  {short}")
