"""Average duration of each (kernel, grid size) in a rocprofv3 kernel trace:
the launches of one kernel at different list sizes kept apart (the stats
summary averages them together).

    python tools/trace_by_grid.py gpurun_out/<dir>/prof/run_kernel_trace.csv [name-filter ...]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2:]
g = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pluss::", "")
    if flt and not any(f in n for f in flt):
        continue
    g[(n, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, wg), v in sorted(g.items(), key=lambda x: -sum(x[1])):
    print(f"{sum(v):12.1f} us  {len(v):5d} x {sum(v) / len(v):9.2f} us  {wg:8d} workgroups  {n}")
