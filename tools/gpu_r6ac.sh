#!/bin/bash
# Round 6: the any-order group pass (upload pieces counted as they land, up to
# 16K partition blocks): group + sort tests, its times, and a kernel/copy trace.
# usage: tools/gpu_r6ac.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ac}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_group_capi.py \
  tests/test_gpu_sort.py > "$OUT/pytest.log" 2>&1; rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/group_time.py any_order 5 > "$OUT/group_any_order.json" 2> "$OUT/group_any_order.err" \
  || { tail -3 "$OUT/group_any_order.err"; exit 1; }
tail -1 "$OUT/group_any_order.json"
true
