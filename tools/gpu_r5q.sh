#!/bin/bash
# The group's any-order pass at config 3 (tools/group_time.py any_order), then the group tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5q}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/group_time.py any_order 3 > "$OUT/group_any_order.json" 2>&1; rc=$?; tail -3 "$OUT/group_any_order.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_group_capi.py \
  > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; exit $rc
