#!/bin/bash
# Round-5 counter passes at config 3: the faithful sorted, radix and uniform
# passes (tools/gpu_pmc_faithful.sh: SQ counters, FETCH_SIZE, WRITE_SIZE, each
# pass in its own run).  usage: tools/gpu_pmc_r5.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-pmc5}
for mode in sorted radix uniform; do
  PROF_SHAPE=config3 PROF_REPS=3 bash tools/gpu_pmc_faithful.sh "$OUT/$mode" $mode || exit $?
  echo "$mode done"
done
