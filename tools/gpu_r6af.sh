#!/bin/bash
# Round 6: the final sort with one more counting bit: sort + faithful wide
# tests, then the faithful config-3 times and a radix kernel trace.
# usage: tools/gpu_r6af.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6af}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sort.py \
  tests/test_gpu_faithful_wide.py > "$OUT/pytest.log" 2>&1; rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fa_time.py 4096 8 28 > "$OUT/fa_time.json" 2>&1 && tail -1 "$OUT/fa_time.json" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python tools/fa_time.py 4096 8 28 --only radix > "$OUT/radix.log" 2>&1 \
&& python tools/stats_summary.py "$OUT/prof/run_kernel_stats.csv" > "$OUT/stats.txt" && head -6 "$OUT/stats.txt"
