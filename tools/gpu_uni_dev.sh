#!/bin/bash
# Uniform-source development session: its GPU tests, the pass times at configs 2 and 3
# (tools/fa_time.py) and a kernel trace of the config-3 uniform pass.  usage: tools/gpu_uni_dev.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-unidev}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_uniform.py \
  tests/test_group_capi.py > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fa_time.py 1024 8 24 4096 8 28 --only uniform,uni_plan,uni_stage_dec,uni_stage_packed > "$OUT/fa_time.json" 2>&1 && cat "$OUT/fa_time.json" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python tools/fa_time.py 4096 8 28 --only uniform \
  > "$OUT/prof.log" 2>&1 && python tools/stats_summary.py "$OUT/prof/run_kernel_stats.csv" > "$OUT/stats.txt" && head -16 "$OUT/stats.txt"
