#!/bin/bash
# rocprofv3 counter passes over the uniform source at config 3 (tools/prof_faithful.py):
# the whole pass and the staging alone (diagnostics), SQ instruction/cycle counters and
# LDS counters, each pass in its own run.  usage: tools/gpu_pmc_uni.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcu}
mkdir -p "$OUT"
for mode in uniform uni_stage; do
  for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"; do
    tag=$(echo $c | cut -d' ' -f1)
    PROF_SHAPE=config3 PROF_FAITH=$mode PROF_REPS=3 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv \
      -d "$OUT/pmc_${mode}_$tag" -o run -- python tools/prof_faithful.py > "$OUT/pmc_${mode}_$tag.log" 2>&1 \
      || { echo "pass $mode $tag failed"; tail -5 "$OUT/pmc_${mode}_$tag.log"; exit 1; }
  done
done
python - "$OUT" <<'PY'
import csv, glob, os, sys, collections
run = sys.argv[1]
for mode in ("uniform", "uni_stage"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(run, f"pmc_{mode}_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pluss::", "")
            if "k_fa_local_lm" in k or "k_ug_stage_only" in k or "k_ug_count" in k:
                per[k][r["Counter_Name"]] += float(r["Counter_Value"]) / 3
    for k, d in per.items():
        print(mode, k, {c: "%.4g" % v for c, v in sorted(d.items())})
PY
