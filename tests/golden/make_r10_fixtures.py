"""Convert dumps of the reference r10 sampler into committed golden fixtures.

PROVENANCE.  The inputs are the text dumps written during the survey phase of
this project by the reference sampler
c_lib/test/sampler/gemm-t4-pluss-pro-model-rs-ri-opt-r10.cpp, compiled from
/root/reference with its only two changes being (a) rand() replaced by a
seeded generator and (b) one print of each pushed sample (r10:182) and of the
raw no_share/share histograms just before no_share_distribute (r10:690).  The
GSL shim used in that build only feeds the CRI step *after* the dump, so the
raw RI histograms here do not depend on it.  This script does not build or run
anything from the reference: it only parses those dump files.

    err_<N>_<T>_<seed>.txt : "SAMPLE <REF> c0 c1 [c2]" lines, one per pushed sample
    out_<N>_<T>_<seed>.txt : "RAW_NOSHARE sampler_<REF> traversed=<k>" /
                              "RAW_SHARE sampler_<REF> n=<share_ratio>" headers
                              followed by "ri,count" lines

Output per configuration: r10_N<N>_T<T>_s<seed>.npz with one uint16 (n, 3)
array per reference (2-D references have c2 = 0) and r10_N<N>_T<T>_s<seed>.json
with the expected raw histograms: {ref: {"noshare": {ri: count},
"share": {ri: count}, "share_ratio": n, "traversed": k}}.

usage: python tests/golden/make_r10_fixtures.py [dump_dir]
"""
import glob
import json
import os
import re
import sys

import numpy as np

REFS = ["C0", "C1", "A0", "B0", "C2", "C3"]
HERE = os.path.dirname(os.path.abspath(__file__))


def convert(dump_dir, N, T, seed):
    samples = {r: [] for r in REFS}
    with open(os.path.join(dump_dir, f"err_{N}_{T}_{seed}.txt")) as f:
        for line in f:
            if line.startswith("SAMPLE"):
                p = line.split()
                iv = [int(x) for x in p[2:]] + [0]
                samples[p[1]].append(iv[:3])
    raw = {r: {"noshare": {}, "share": {}, "share_ratio": None, "traversed": None} for r in REFS}
    cur = kind = None
    with open(os.path.join(dump_dir, f"out_{N}_{T}_{seed}.txt")) as f:
        for line in f:
            line = line.strip()
            m = re.match(r"RAW_(NOSHARE|SHARE) sampler_(\w+)(?: traversed=(\d+))?(?: n=(\d+))?", line)
            if m:
                kind, cur = m.group(1).lower(), m.group(2)
                if m.group(3) is not None:
                    raw[cur]["traversed"] = int(m.group(3))
                if m.group(4) is not None:
                    raw[cur]["share_ratio"] = int(m.group(4))
                continue
            if cur and re.match(r"^-?\d+,[-\d.e+]+$", line):
                k, v = line.split(",")
                raw[cur][kind][int(k)] = int(round(float(v)))
            else:
                cur = None
    printed = parse_printed(os.path.join(dump_dir, f"out_{N}_{T}_{seed}.txt"))
    stem = os.path.join(HERE, f"r10_N{N}_T{T}_s{seed}")
    np.savez_compressed(stem + ".npz", **{r: np.array(samples[r], dtype=np.uint16).reshape(-1, 3) for r in REFS})
    with open(stem + ".json", "w") as f:
        json.dump({"N": N, "T": T, "CS": 4, "DS": 8, "CLS": 64, "seed": seed,
                   "source": "reference r10 sampler dump (see make_r10_fixtures.py)",
                   "raw": raw, "printed": printed}, f, indent=1, sort_keys=True)
    return stem


def parse_printed(path):
    """The reference's own printout after the raw dump (r10 main, r10:3280-3293):
    per-reference CRI-distributed histograms (_pluss_histogram_print: "ri,count,fraction",
    6 significant digits), the merged log2 reuse histogram, the MRC ("c, miss ratio")
    and "max iteration traversed"."""
    out = {"per_ref": {}, "reuse": [], "mrc": [], "max_traversed": None}
    cur = None
    lines = open(path).read().splitlines()
    i = 0
    while i < len(lines):
        line = lines[i].strip()
        if line in REFS:
            cur = out["per_ref"].setdefault(line, [])
        elif line == "Start to dump reuse time":
            cur = out["reuse"]
        elif line == "miss ratio":
            cur = out["mrc"]
        elif line == "max iteration traversed":
            out["max_traversed"] = int(lines[i + 1])
            cur = None
            i += 1
        elif line.startswith("RAW_"):
            cur = None
        elif cur is not None and re.match(r"^-?\d+,", line):
            cur.append([float(x) for x in line.split(",")])
        i += 1
    return out


def main():
    dump_dir = sys.argv[1] if len(sys.argv) > 1 else "/tmp/oracle"
    # the unmodified full-trace seq binary's `acc` printout at N=128, T=4
    # (seq.cpp:336-350): noshare (floor-log2), share, CRI reuse histogram, MRC
    seq = os.path.join(dump_dir, "seq_acc.txt")
    if os.path.exists(seq):
        with open(seq) as f, open(os.path.join(HERE, "seq_N128_T4_acc.txt"), "w") as g:
            g.write(f.read())
    for path in sorted(glob.glob(os.path.join(dump_dir, "out_*_*_*.txt"))):
        N, T, seed = (int(x) for x in os.path.basename(path)[4:-4].split("_"))
        print(convert(dump_dir, N, T, seed))


if __name__ == "__main__":
    main()
