"""Print the kernel timeline around the Nth dispatch of a kernel in a
rocprofv3 kernel trace: start offset, duration, name, grid.
usage: python tools/trace_seq.py <run_kernel_trace.csv> <name substring> [occurrence] [before] [after]"""
import csv
import sys

path, pat = sys.argv[1], sys.argv[2]
occ, before, after = (int(x) for x in (sys.argv[3:] + ["5", "3", "8"])[:3])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if pat in r["Kernel_Name"]]
i = idx[min(occ, len(idx) - 1)]
t0 = int(rows[max(0, i - before)]["Start_Timestamp"])
for r in rows[max(0, i - before):i + after]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  {r['Kernel_Name'][:70]}  grid={r['Grid_Size_X']}")
