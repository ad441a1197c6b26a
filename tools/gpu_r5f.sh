#!/bin/bash
# Round-5 check of the group's any-order faithful pass (device partition):
# the group tests, then its call times at config 3.  usage: tools/gpu_r5f.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5f}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_group_capi.py \
  > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/group_time.py any_order 3 > "$OUT/group_any.json" 2>&1 && tail -1 "$OUT/group_any.json" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python tools/group_time.py any_order 2 \
  > "$OUT/prof.log" 2>&1 && python tools/trace_span.py "$OUT/prof/run_kernel_trace.csv" > "$OUT/span.txt" 2>&1; tail -25 "$OUT/span.txt"
