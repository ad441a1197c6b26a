#!/bin/bash
# tools/gpu_r5g.sh (faithful/sort/group GPU tests, faithful times, radix trace),
# then the group call times (generated, uniform, any order).  usage: tools/gpu_r5p.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5p}
bash tools/gpu_r5g.sh "${1:-r5p}" || exit $?
for src in generated uniform any_order; do
  timeout -k 10 300 python tools/group_time.py $src 5 > "$OUT/group_$src.json" 2>&1 || { tail -5 "$OUT/group_$src.json"; exit 1; }
  tail -1 "$OUT/group_$src.json"
done
