"""Summarise a rocprofv3 kernel trace (run_kernel_trace.csv): the last faithful
pass of tools/prof_side.py, kernel by kernel (short names), with its span
and the busy time of the union of kernel intervals.

    python tools/trace_summary.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    if "rocprim" in name:
        for tag in ("onesweep_iteration", "global_offsets", "block_sort", "merge", "FlagOp", "PkSink",
                    "init_lookback", "scan"):
            if tag in name:
                return "rocprim " + tag
        return "rocprim ?"
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
    ks.sort()
    # the faithful passes start at k_faith_keys launches; take the last pass (up to the full trace)
    starts = [i for i, k in enumerate(ks) if "k_faith_keys" in k[2]]
    if not starts:
        print("no faithful kernels")
        return
    # a pass = 6 k_faith_keys (one per reference) and what follows them
    first = starts[-6] if len(starts) >= 6 else starts[0]
    end = next((i for i in range(first, len(ks)) if "fulltrace" in ks[i][2]), len(ks))
    sel = ks[first:end]
    t0 = min(k[0] for k in sel)
    t1 = max(k[1] for k in sel)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        agg[n][0] += 1
        agg[n][1] += e - s
    print(f"kernels {len(sel)}  span {(t1 - t0) / 1e3:.1f} us  busy(union) {busy / 1e3:.1f} us")
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {n:60s} calls {c:3d}  sum {d / 1e3:8.1f} us  avg {d / c / 1e3:7.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
