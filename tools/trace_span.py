"""Where the time of repeated calls goes, from a rocprofv3 kernel trace: the
trace's kernels (and memory fills) split into calls at gaps longer than
`gap` us; per call its span (first start to last end), the kernels' busy time
(the union of their intervals), the number of launches, and the top kernels.

    python tools/trace_span.py gpurun_out/<dir>/prof/run_kernel_trace.csv [gap_us]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 2000.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pluss::", "")) for r in rows)
calls, cur = [], []
for e in ev:
    if cur and e[0] - max(x[1] for x in cur) > gap * 1e3:
        calls.append(cur)
        cur = []
    cur.append(e)
if cur:
    calls.append(cur)
for i, c in enumerate(calls):
    span = (max(x[1] for x in c) - c[0][0]) / 1e3
    busy, end = 0, 0
    for s, e, _ in c:
        s = max(s, end)
        if e > s:
            busy += e - s
            end = e
    top = collections.Counter()
    for s, e, n in c:
        top[n] += (e - s) / 1e3
    print(f"call {i}: span {span:9.1f} us  busy {busy / 1e3:9.1f} us  launches {len(c):4d}  "
          + ", ".join(f"{n} {t:.0f}" for n, t in top.most_common(5)))
