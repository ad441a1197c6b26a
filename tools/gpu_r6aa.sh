#!/bin/bash
# Round 6: the any-order group pass with the upload in pieces (each counted as
# it lands) and the partition's 4-deep loads; group + sort tests, the times,
# then the counter passes (tools/gpu_pmc_r6.sh).  usage: tools/gpu_r6aa.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6aa}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_group_capi.py \
  tests/test_gpu_sort.py > "$OUT/pytest.log" 2>&1; rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/group_time.py any_order 5 > "$OUT/group_any_order.json" 2> "$OUT/group_any_order.err" \
  || { tail -3 "$OUT/group_any_order.err"; exit 1; }
tail -1 "$OUT/group_any_order.json"
bash tools/gpu_pmc_r6.sh "${1:-r6aa}/pmc"
