#!/bin/bash
# Round 6 closing session: smoke, every GPU test, the bench line with its kernel
# trace, the config 2 / config 4 lines (tools/gpu_full_round.sh), then the group
# times (uniform, generated).  usage: tools/gpu_final_r6.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-r6final}
bash tools/gpu_full_round.sh "$OUT" || exit 1
for src in uniform generated; do
  timeout -k 10 300 python tools/group_time.py $src 7 > "gpurun_out/$OUT/group_$src.json" 2> "gpurun_out/$OUT/group_$src.err" \
    || { tail -3 "gpurun_out/$OUT/group_$src.err"; exit 1; }
  tail -1 "gpurun_out/$OUT/group_$src.json"
done
