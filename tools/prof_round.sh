#!/bin/bash
# Ablation timings + rocprofv3 PMC passes of the hot kernel (separate --pmc runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p "$OUT"
if [ "$2" != "noablate" ]; then
  echo "== ablate" && timeout -k 10 300 python tools/ablate.py > "$OUT/ablate.jsonl" 2> "$OUT/ablate.err" && cat "$OUT/ablate.jsonl" || exit 1
fi
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  echo "== pmc pass $i: $ctrs"
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/pmc$i" -o run -- python tools/prof_kernel.py > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc$i.log"; exit 1; }
  f=$(find "$OUT/pmc$i" -name "*counter_collection.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if "k_count" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"  {k}: mean {sum(v)/len(v):.4g} over {len(v)} dispatches")
PY
done
