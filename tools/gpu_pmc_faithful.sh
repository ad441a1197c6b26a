#!/bin/bash
# rocprofv3 counter passes over the faithful pipeline (tools/prof_faithful.py):
# SQ cycle/instruction counters, FETCH_SIZE, WRITE_SIZE, each in its own run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcf}
MODE=${2:-sorted}
REPS=${PROF_REPS:-5}
mkdir -p "$OUT"
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
         FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $c | cut -d' ' -f1)
  PROF_FAITH=$MODE PROF_REPS=$REPS timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$tag" -o run -- python tools/prof_faithful.py > "$OUT/pmc_$tag.log" 2>&1 || { echo "pass $tag failed"; tail -5 "$OUT/pmc_$tag.log"; exit 1; }
done
python tools/pmc_faithful_summary.py "$OUT" $REPS "$OUT/pmc_faithful.json"   # PROF_SHAPE passes through
