#!/bin/bash
# Round 6: a kernel + memory-copy trace of the any-order group pass (where the
# upload, the partition and the sort sit in time).  usage: tools/gpu_r6ab.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ab}
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/prof" -o run -- \
  python tools/group_time.py any_order 2 > "$OUT/run.log" 2>&1; rc=$?; tail -1 "$OUT/run.log"; exit $rc
