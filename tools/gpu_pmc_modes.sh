#!/bin/bash
# rocprofv3 SQ counter passes (instruction mix, wave cycles, waits, LDS) over
# faithful passes at config 3 (tools/prof_faithful.py), each pass in its own run.
# usage: tools/gpu_pmc_modes.sh OUT "radix sorted ..." [kernel-name regex]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcm}
MODES=${2:-radix}
PAT=${3:-.}
mkdir -p "$OUT"
for mode in $MODES; do
  for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    tag=$(echo $c | cut -d' ' -f1)
    PROF_SHAPE=config3 PROF_FAITH=$mode PROF_REPS=3 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv \
      -d "$OUT/pmc_${mode}_$tag" -o run -- python tools/prof_faithful.py > "$OUT/pmc_${mode}_$tag.log" 2>&1 \
      || { echo "pass $mode $tag failed"; tail -5 "$OUT/pmc_${mode}_$tag.log"; exit 1; }
  done
done
python - "$OUT" "$MODES" "$PAT" <<'PY'
import csv, glob, os, re, sys, collections
run, modes, pat = sys.argv[1], sys.argv[2].split(), re.compile(sys.argv[3])
for mode in modes:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(run, f"pmc_{mode}_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pluss::", "")
            if pat.search(k):
                per[k][r["Counter_Name"]] += float(r["Counter_Value"]) / 3
    for k, d in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(mode, k, {c: "%.4g" % v for c, v in sorted(d.items())})
PY
